// Direct k^3 convolution (forward and backward-data) for SMALL grids with MANY channels: the
// codebook-level convs of the published model (128 -> 128 channels on 8x8x2 / 16x16x4 grids,
// vqvae/layers.py:377, :490, the stride-2 down blocks feeding them).  One output voxel tile
// holds only 128 voxels there, so a per-voxel engine leaves the GPU idle; this one splits the
// reduction channels over workgroups instead.
//
// Grid: x = 32-voxel tiles, y = 64-output-channel tiles, z = chunks of CC reduction channels
// (forward: input channels, backward-data: output channels).  A workgroup stages W for its
// (all taps) x (CC channels) x (64 outputs) block in LDS -- read with coalesced runs of the
// reference [Cout][Cin][k^3] layout -- and each thread accumulates 8 outputs of one voxel over
// every tap of its channel chunk.  Partials [z][voxel][out] (fp32 workspace) are summed in a
// fixed order by a second kernel that applies the fused forward / backward-data epilogue
// (deterministic; no atomics on the outputs).
#include "conv_epi.h"

#include <algorithm>

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int VT = 32;  // voxels per tile
constexpr int OT = 64;  // output channels per tile
constexpr int CPT = 8;  // output channels per thread: OT / (256 / VT)
constexpr size_t kSmallLds = 64 * 1024;

struct SArgs {
    ConvArgs c;
    int nvox;    // voxels of this pass's output grid
    int Rt, Ot;  // reduction / output channels
    int K3, nsplit;
    int vec;     // reduction rows readable as 4-channel vectors
};

template <typename T>
__device__ __forceinline__ void load4(const T *p, bool vec, int n, float (&o)[4]) {
    if constexpr (sizeof(T) == 2) {
        if (vec) {
            const uint2 u = *reinterpret_cast<const uint2 *>(p);
            o[0] = h2f_lo(u.x);
            o[1] = h2f_hi(u.x);
            o[2] = h2f_lo(u.y);
            o[3] = h2f_hi(u.y);
            return;
        }
    } else {
        if (vec) {
            const float4 f = *reinterpret_cast<const float4 *>(p);
            o[0] = f.x;
            o[1] = f.y;
            o[2] = f.z;
            o[3] = f.w;
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = j < n ? ld(p + j) : 0.f;
}

template <typename T, bool DG, int CC>
__global__ __launch_bounds__(256) void k_small(SArgs s, const T *__restrict__ in, const T *__restrict__ in2,
                                              const float *__restrict__ w, float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];  // [tap][CC][OT]
    const ConvArgs &a = s.c;
    const int tid = threadIdx.x;
    const int o_base = blockIdx.y * OT, r0 = blockIdx.z * CC;
    const int Ct = a.Cin + a.Cin2;  // the weight's second dimension
    const int K3 = s.K3;
    // weights: forward W(o, r, t) = w[(o * Ct + r) * K3 + t]; backward-data W(o = ci, r = co, t) =
    // w[(r * Ct + o) * K3 + t].  Index order chosen so consecutive threads read consecutive floats.
    for (int e = tid; e < K3 * CC * OT; e += 256) {
        const int t = e % K3, q = e / K3;
        int ol, rr;
        if (DG) {
            ol = q % OT;
            rr = q / OT;
        } else {
            rr = q % CC;
            ol = q / CC;
        }
        const int o = o_base + ol, r = r0 + rr;
        float val = 0.f;
        if (o < s.Ot && r < s.Rt) val = DG ? w[(int64_t(r) * Ct + o) * K3 + t] : w[(int64_t(o) * Ct + r) * K3 + t];
        wsh[(t * CC + rr) * OT + ol] = val;
    }
    __syncthreads();
    const int v = blockIdx.x * VT + tid % VT;
    const int cg = tid / VT;
    if (v >= s.nvox) return;
    // this pass's output-grid coordinates
    int gd, gw, gh, b;
    {
        const int nD = DG ? a.iD : a.oD, nW = DG ? a.iW : a.oW, nH = DG ? a.iH : a.oH;
        int t = v;
        gd = t % nD;
        t /= nD;
        gw = t % nW;
        t /= nW;
        gh = t % nH;
        b = t / nH;
    }
    const Prologue pro = make_prologue(DG ? VQ3D_PRO_NONE : a.pro_kind, a.pro_a, a.pro_b);
    float acc[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) acc[j] = 0.f;
    const int nr = min(CC, s.Rt - r0);
    // forward rows: x (channels [0, Cin)) then x2; backward-data rows: g
    const T *src = in;
    int ldr = DG ? a.Cout : a.Cin, roff = r0;
    if (!DG && r0 >= a.Cin) {
        src = in2;
        ldr = a.Cin2;
        roff = r0 - a.Cin;
    }
    const bool split_rows = !DG && a.Cin2 && r0 < a.Cin && r0 + nr > a.Cin;  // chunk straddles x | x2
    const int sH = DG ? a.oH : a.iH, sW = DG ? a.oW : a.iW, sD = DG ? a.oD : a.iD;
    int tap = 0;
    for (int kh = 0; kh < a.k; ++kh) {
        const int ih = DG ? bwd_index(gh, kh, a.s, a.p, a.iH, a.oH, a.circ) : fwd_index(gh, kh, a.s, a.p, a.iH, a.circ);
        for (int kw = 0; kw < a.k; ++kw) {
            const int iw =
                DG ? bwd_index(gw, kw, a.s, a.p, a.iW, a.oW, a.circ) : fwd_index(gw, kw, a.s, a.p, a.iW, a.circ);
            for (int kd = 0; kd < a.k; ++kd, ++tap) {
                const int id =
                    DG ? bwd_index(gd, kd, a.s, a.p, a.iD, a.oD, a.circ) : fwd_index(gd, kd, a.s, a.p, a.iD, a.circ);
                if ((ih | iw | id) < 0) continue;
                const int64_t pos = ((int64_t(b) * sH + ih) * sW + iw) * sD + id;
                float xv[CC];
                if (!split_rows) {
                    const T *row = src + pos * ldr + roff;
#pragma unroll
                    for (int q = 0; q < CC / 4; ++q) {
                        float f[4];
                        load4(row + 4 * q, s.vec != 0, nr - 4 * q, f);
#pragma unroll
                        for (int j = 0; j < 4; ++j) xv[4 * q + j] = f[j];
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < CC; ++j) {
                        const int r = r0 + j;
                        xv[j] = j < nr ? (r < a.Cin ? ld(in + pos * a.Cin + r) : ld(in2 + pos * a.Cin2 + r - a.Cin))
                                       : 0.f;
                    }
                }
                if (!DG && pro.kind != VQ3D_PRO_NONE) {
#pragma unroll
                    for (int j = 0; j < CC; ++j) xv[j] = j < nr ? pro.apply(xv[j]) : 0.f;
                }
                const float *wt = wsh + tap * CC * OT + cg * CPT;
#pragma unroll
                for (int j = 0; j < CC; ++j) {
                    const float4 w0 = *reinterpret_cast<const float4 *>(wt + j * OT);
                    const float4 w1 = *reinterpret_cast<const float4 *>(wt + j * OT + 4);
                    acc[0] = fmaf(xv[j], w0.x, acc[0]);
                    acc[1] = fmaf(xv[j], w0.y, acc[1]);
                    acc[2] = fmaf(xv[j], w0.z, acc[2]);
                    acc[3] = fmaf(xv[j], w0.w, acc[3]);
                    acc[4] = fmaf(xv[j], w1.x, acc[4]);
                    acc[5] = fmaf(xv[j], w1.y, acc[5]);
                    acc[6] = fmaf(xv[j], w1.z, acc[6]);
                    acc[7] = fmaf(xv[j], w1.w, acc[7]);
                }
            }
        }
    }
    float *pp = part + (int64_t(blockIdx.z) * s.nvox + v) * s.Ot;
    const int o0 = o_base + cg * CPT;
#pragma unroll
    for (int j = 0; j < CPT; ++j)
        if (o0 + j < s.Ot) pp[o0 + j] = acc[j];
}


// Matrix-core form (16-bit builds; reduction channels in chunks of 32, outputs in tiles of 16,
// 16-byte rows): the same partials [z][voxel][out] as k_small, z = (32-channel chunk, group of TG
// taps) -- the taps are split too, so a 128-voxel grid still spreads over ~100 workgroups.  A
// workgroup owns 32 voxels x 64 outputs; its (TG taps x 32 channels x 64 outputs) weight block is
// packed into MFMA A fragments in LDS (rows = outputs), each lane loads its voxel's 32-channel
// row of every tap as B fragments (16 bytes per tap, all in flight together), and each wave
// computes 16 voxels x 32 outputs: every lane ends with 4 consecutive outputs of one voxel, one
// 16-byte partial store per output tile.
template <bool DG, int TG>
__global__ __launch_bounds__(256) void k_small_mma(SArgs s, const h16_t *__restrict__ in, const h16_t *__restrict__ in2,
                                                  const float *__restrict__ w, float *__restrict__ part, int ntg) {
    extern __shared__ __attribute__((aligned(16))) uint4 wfr[];  // [TG][4 o-tiles][64 lanes]
    const ConvArgs &a = s.c;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kb = lane >> 4, row = lane & 15;
    const int o_base = int(blockIdx.y) * OT;
    const int zc = int(blockIdx.z) / ntg, t0 = int(blockIdx.z) % ntg * TG;
    const int r0 = zc * 32;
    const int Ct = a.Cin + a.Cin2, K3 = s.K3;
    const int ntap = min(TG, K3 - t0);
    // pack: thread per (output, channel) reads the group's TG consecutive taps of W(o, r, .)
    // (a thread per element with coalesced runs measured slower: 23.8 -> 46.7 us, r04g)
    h16_t *wh = reinterpret_cast<h16_t *>(wfr);
    for (int pr = tid; pr < OT * 32; pr += 256) {
        const int rl = pr & 31, ol = pr >> 5, o = o_base + ol, r = r0 + rl;
        const bool ok = o < s.Ot && r < s.Rt;
        const float *src = w + (ok ? (DG ? (int64_t(r) * Ct + o) * K3 : (int64_t(o) * Ct + r) * K3) + t0 : 0);
        const int e0 = ((ol >> 4) * 64 + (ol & 15) + 16 * (rl >> 3)) * 8 + (rl & 7);
#pragma unroll
        for (int ti = 0; ti < TG; ++ti) wh[ti * 4 * 64 * 8 + e0] = f2h(ok && ti < ntap ? src[ti] : 0.f);
    }
    // this lane's voxel (B column) in the pass's output grid
    const int v = int(blockIdx.x) * VT + (wave & 1) * 16 + row;
    const bool live = v < s.nvox;
    int gd, gw, gh, b;
    {
        const int nD = DG ? a.iD : a.oD, nW = DG ? a.iW : a.oW, nH = DG ? a.iH : a.oH;
        int t = live ? v : 0;
        gd = t % nD;
        t /= nD;
        gw = t % nW;
        t /= nW;
        gh = t % nH;
        b = t / nH;
    }
    const h16_t *src = in;
    int ldr = DG ? a.Cout : a.Cin, roff = r0;
    if (!DG && r0 >= a.Cin) {
        src = in2;
        ldr = a.Cin2;
        roff = r0 - a.Cin;
    }
    const int sH = DG ? a.oH : a.iH, sW = DG ? a.oW : a.iW, sD = DG ? a.oD : a.iD;
    uint4 bv[TG];
#pragma unroll
    for (int ti = 0; ti < TG; ++ti) {
        bv[ti] = uint4{0u, 0u, 0u, 0u};
        const int t = t0 + ti;
        if (!live || ti >= ntap) continue;
        const int kh = t / (a.k * a.k), kw = (t / a.k) % a.k, kd = t % a.k;
        const int ih = DG ? bwd_index(gh, kh, a.s, a.p, a.iH, a.oH, a.circ) : fwd_index(gh, kh, a.s, a.p, a.iH, a.circ);
        const int iw = DG ? bwd_index(gw, kw, a.s, a.p, a.iW, a.oW, a.circ) : fwd_index(gw, kw, a.s, a.p, a.iW, a.circ);
        const int id = DG ? bwd_index(gd, kd, a.s, a.p, a.iD, a.oD, a.circ) : fwd_index(gd, kd, a.s, a.p, a.iD, a.circ);
        if ((ih | iw | id) < 0) continue;
        const int64_t pos = ((int64_t(b) * sH + ih) * sW + iw) * sD + id;
        bv[ti] = *reinterpret_cast<const uint4 *>(src + pos * ldr + roff + 8 * kb);
    }
    if (!DG) {
        const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
        if (pro.kind != VQ3D_PRO_NONE) {
#pragma unroll
            for (int ti = 0; ti < TG; ++ti) {
                const int t = t0 + ti;
                if (!live || ti >= ntap) continue;
                const int kh = t / (a.k * a.k), kw = (t / a.k) % a.k, kd = t % a.k;
                // padded taps stay zero (k_small skips them); live rows get the prologue
                if ((fwd_index(gh, kh, a.s, a.p, a.iH, a.circ) | fwd_index(gw, kw, a.s, a.p, a.iW, a.circ) |
                     fwd_index(gd, kd, a.s, a.p, a.iD, a.circ)) < 0)
                    continue;
                uint32_t q[4] = {bv[ti].x, bv[ti].y, bv[ti].z, bv[ti].w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    q[j] = uint32_t(f2h(pro.apply(h2f_lo(q[j])))) | (uint32_t(f2h(pro.apply(h2f_hi(q[j])))) << 16);
                bv[ti] = uint4{q[0], q[1], q[2], q[3]};
            }
        }
    }
    __syncthreads();
    const int ot0 = 2 * (wave >> 1);  // the wave's two 16-output tiles
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ti = 0; ti < TG; ++ti) {
        const hx8 bf = __builtin_bit_cast(hx8, bv[ti]);
        acc0 = VQ3D_MFMA_16X16X32(__builtin_bit_cast(hx8, wfr[(ti * 4 + ot0) * 64 + lane]), bf, acc0, 0, 0, 0);
        acc1 = VQ3D_MFMA_16X16X32(__builtin_bit_cast(hx8, wfr[(ti * 4 + ot0 + 1) * 64 + lane]), bf, acc1, 0, 0, 0);
    }
    if (!live) return;
    float *pp = part + (int64_t(blockIdx.z) * s.nvox + v) * s.Ot;
    const int o0 = o_base + 16 * ot0 + 4 * kb, o1 = o0 + 16;
    if (o0 < s.Ot) *reinterpret_cast<float4 *>(pp + o0) = float4{acc0[0], acc0[1], acc0[2], acc0[3]};
    if (o1 < s.Ot) *reinterpret_cast<float4 *>(pp + o1) = float4{acc1[0], acc1[1], acc1[2], acc1[3]};
}

template <typename T, bool DG>
__global__ __launch_bounds__(256) void k_small_epi(SArgs s, const float *__restrict__ part, FwdEpi<T> fe,
                                                  BwdEpi<T> be, const float *__restrict__ gscale, T *__restrict__ out,
                                                  T *__restrict__ out2, float *dpre, float *dpost, GridSum gsum) {
    __shared__ float red[8];
    const ConvArgs &a = s.c;
    const ActDeriv dv = make_deriv(be);
    const float gs = gscale ? *gscale : 1.f;
    float pre = 0.f, post = 0.f;
    const int64_t n = int64_t(s.nvox) * s.Ot;
    const int64_t stride = int64_t(s.nvox) * s.Ot;
    for (int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x; e < n; e += int64_t(gridDim.x) * 256) {
        const int v = int(e / s.Ot), o = int(e - int64_t(v) * s.Ot);
        float acc[1] = {0.f};
        for (int z = 0; z < s.nsplit; ++z) acc[0] += part[z * stride + e];
        if (!DG)
            fwd_epilogue<T, 1>(a, fe, acc, v, o, out + int64_t(v) * a.Cout);
        else
            bwd_epilogue<T, 1>(a, be, dv, gs, gscale != nullptr, acc, v, o, out + int64_t(v) * a.Cin,
                               out2 ? out2 + int64_t(v) * a.Cin2 : nullptr, pre, post);
    }
    if (DG && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        grid_sum2<256>(gsum, pre, post, dpre, dpost, red);
    }
}

struct SPlan {
    SArgs s;
    int cc, nvt, nct;
    int mma, tg, ntg;  // matrix-core form: taps per group, tap groups
};

// reduction chunk of the VALU kernel k_small: the largest of 16 / 8 channels that still gives
// >= 256 workgroups and fits the LDS weight block, else 4
void valu_chunking(SPlan &p) {
    p.cc = 4;
    for (int cc : {16, 8}) {
        const int64_t wgs = int64_t(p.nvt) * p.nct * ((p.s.Rt + cc - 1) / cc);
        if (wgs >= 256 && size_t(p.s.K3) * cc * OT * 4 <= kSmallLds) {
            p.cc = cc;
            break;
        }
    }
    p.s.nsplit = (p.s.Rt + p.cc - 1) / p.cc;
}

SPlan plan_small(const vq3d_conv_desc *d, bool dgrad, const float *pa, const float *pb) {
    SPlan p;
    p.s.c = make_args(d, pa, pb);
    const int64_t nv = dgrad ? int64_t(d->batch) * d->in_h * d->in_w * d->in_d
                             : int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    p.s.nvox = int(nv);
    p.s.Rt = dgrad ? d->cout : d->cin + d->cin2;
    p.s.Ot = dgrad ? d->cin + d->cin2 : d->cout;
    p.s.K3 = d->kernel * d->kernel * d->kernel;
    p.nvt = int((nv + VT - 1) / VT);
    p.nct = (p.s.Ot + OT - 1) / OT;
    valu_chunking(p);
    // matrix cores: 16-bit data, 32-channel reduction chunks that never straddle x | x2, 16-output
    // tiles (the codebook levels' 64- / 128-channel convs)
    p.mma = d->dtype == VQ3D_HALF && p.s.Rt % 32 == 0 && p.s.Ot % 16 == 0 &&
            (dgrad ? d->cout % 32 == 0 : d->cin % 32 == 0 && d->cin2 % 32 == 0);
    p.tg = d->kernel == 3 ? 9 : 8;
    p.ntg = (p.s.K3 + p.tg - 1) / p.tg;
    if (p.mma) {
        p.cc = 32;
        p.s.nsplit = p.s.Rt / 32 * p.ntg;
    }
    return p;
}

}  // namespace

bool small_applicable(const vq3d_conv_desc *d, bool dgrad) {
    if (d->kernel <= 1 || d->kernel > 4) return false;
    if (dgrad && d->stride != 1 && d->stride != 2) return false;
    const int64_t nv = dgrad ? int64_t(d->batch) * d->in_h * d->in_w * d->in_d
                             : int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    const int rt = dgrad ? d->cout : d->cin + d->cin2;
    const int ot = dgrad ? d->cin + d->cin2 : d->cout;
    if (nv > 4096 || rt < 32 || ot < 16) return false;
    return size_t(d->kernel) * d->kernel * d->kernel * 4 * OT * 4 <= kSmallLds;
}

bool small_mma_form(const vq3d_conv_desc *d, bool dgrad) {
    return small_applicable(d, dgrad) && plan_small(d, dgrad, nullptr, nullptr).mma;
}

// partial rows of either form: a matrix-core plan falls back to k_small (its own, possibly
// larger, split) when an operand is not 16-byte aligned, so the workspace covers both
static size_t small_partials_bytes(const SPlan &p) {
    size_t n = size_t(p.s.nsplit) * p.s.nvox * p.s.Ot * 4;
    if (p.mma) {
        SPlan q = p;
        valu_chunking(q);
        n = std::max(n, size_t(q.s.nsplit) * q.s.nvox * q.s.Ot * 4);
    }
    return n;
}

size_t small_workspace(const vq3d_conv_desc *d, bool dgrad) {
    if (!small_applicable(d, dgrad)) return 0;
    return small_partials_bytes(plan_small(d, dgrad, nullptr, nullptr));
}

template <typename T>
int launch_small(const vq3d_conv_desc *d, bool dgrad, const void *in, const void *in2, const float *w,
                 const float *pa, const float *pb, const FwdEpi<T> &fe, const BwdEpi<T> &be, const float *gscale,
                 void *out, void *out2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t st) {
    SPlan p = plan_small(d, dgrad, pa, pb);
    if (!ws || ws_bytes < small_partials_bytes(p)) return fail("conv3d(small grid): workspace too small");
    auto al = [](const void *q, int ch, int esz) {
        return q == nullptr || ((reinterpret_cast<uintptr_t>(q) & 15) == 0 && (ch * esz) % 8 == 0);
    };
    const int esz = int(sizeof(T));
    p.s.vec = dgrad ? al(in, d->cout, esz) && d->cout % 4 == 0
                    : al(in, d->cin, esz) && al(in2, d->cin2, esz) && d->cin % 4 == 0 && d->cin2 % 4 == 0;
    const dim3 grid{unsigned(p.nvt), unsigned(p.nct), unsigned(p.s.nsplit)};
    float *part = static_cast<float *>(ws);
    if constexpr (std::is_same<T, h16_t>::value) {
        auto al16 = [](const void *q) { return q == nullptr || (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
        if (p.mma && al16(in) && al16(in2)) {
            const size_t lds = size_t(p.tg) * 4 * 64 * 16;
            if (p.tg == 9) {
                if (dgrad) k_small_mma<true, 9><<<grid, 256, lds, st>>>(p.s, (const h16_t *)in, nullptr, w, part, p.ntg);
                else k_small_mma<false, 9><<<grid, 256, lds, st>>>(p.s, (const h16_t *)in, (const h16_t *)in2, w, part, p.ntg);
            } else {
                if (dgrad) k_small_mma<true, 8><<<grid, 256, lds, st>>>(p.s, (const h16_t *)in, nullptr, w, part, p.ntg);
                else k_small_mma<false, 8><<<grid, 256, lds, st>>>(p.s, (const h16_t *)in, (const h16_t *)in2, w, part, p.ntg);
            }
            const int64_t n = int64_t(p.s.nvox) * p.s.Ot;
            const unsigned eb = unsigned(std::min<int64_t>((n + 255) / 256, 1024));
            if (dgrad)
                k_small_epi<T, true><<<eb, 256, 0, st>>>(p.s, part, fe, be, gscale, (T *)out, (T *)out2, dpre, dpost,
                                                      grid_sum_for(st, eb, dpre || dpost));
            else
                k_small_epi<T, false><<<eb, 256, 0, st>>>(p.s, part, fe, be, gscale, (T *)out, nullptr, nullptr, nullptr, GridSum{});
            return check_launch(dgrad ? "conv3d_bwd_data(small grid mma)" : "conv3d_fwd(small grid mma)");
        }
    }
    if (p.mma) valu_chunking(p);  // the VALU kernel's own split (small_partials_bytes covers it)
    const dim3 grid2{unsigned(p.nvt), unsigned(p.nct), unsigned(p.s.nsplit)};
    const size_t lds = size_t(p.s.K3) * p.cc * OT * 4;
#define KS(CC)                                                                                                  \
    case CC:                                                                                                    \
        if (dgrad)                                                                                              \
            k_small<T, true, CC><<<grid2, 256, lds, st>>>(p.s, (const T *)in, nullptr, w, part);                \
        else                                                                                                    \
            k_small<T, false, CC><<<grid2, 256, lds, st>>>(p.s, (const T *)in, (const T *)in2, w, part);        \
        break;
    switch (p.cc) {
        KS(4)
        KS(8)
        KS(16)
    default: return fail("conv3d(small grid): bad chunk");
    }
#undef KS
    const int64_t n = int64_t(p.s.nvox) * p.s.Ot;
    const unsigned eb = unsigned(std::min<int64_t>((n + 255) / 256, 1024));
    if (dgrad)
        k_small_epi<T, true><<<eb, 256, 0, st>>>(p.s, part, fe, be, gscale, (T *)out, (T *)out2, dpre, dpost,
                                                      grid_sum_for(st, eb, dpre || dpost));
    else
        k_small_epi<T, false><<<eb, 256, 0, st>>>(p.s, part, fe, be, gscale, (T *)out, nullptr, nullptr, nullptr, GridSum{});
    return check_launch(dgrad ? "conv3d_bwd_data(small grid)" : "conv3d_fwd(small grid)");
}

template int launch_small<float>(const vq3d_conv_desc *, bool, const void *, const void *, const float *,
                                 const float *, const float *, const FwdEpi<float> &, const BwdEpi<float> &,
                                 const float *, void *, void *, float *, float *, void *, size_t, hipStream_t);
template int launch_small<h16_t>(const vq3d_conv_desc *, bool, const void *, const void *, const float *,
                                  const float *, const float *, const FwdEpi<h16_t> &, const BwdEpi<h16_t> &,
                                  const float *, void *, void *, float *, float *, void *, size_t, hipStream_t);

}  // namespace vq3d
