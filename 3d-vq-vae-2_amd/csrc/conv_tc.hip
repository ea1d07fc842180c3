// 3x3x3 stride-1 convolutions with 1, 2 or 4 channels in and out, at most 4 channel pairs (the
// full-resolution levels of the published model: 2 -> 2 channels at 512x512x128, 1 -> 1 at
// 128^2 x 32; vqvae/layers.py:124-151 branch_conv2 and the Fixup conv2 of layers.py:28-36) --
// forward, backward-data and weight gradient -- on the VALU.
//
// With a handful of channels an MFMA tile is almost all padding (N = 2 of 16 columns, K = 6
// of 8 per tap row) and the LDS operand reads dominate, while the VALU work is small: 27 * CI *
// CO FMAs per voxel.  A workgroup owns an 8 x 8 x 32 brick; its 10 x 10 halo lines of 34
// positions are staged into LDS once (16-byte loads of the contiguous D-runs, wrap / zero
// padding resolved, the input prologue applied once per element); each thread computes 8
// consecutive voxels along D, so one (kh, kw) line read of 10 positions feeds 3 taps x 8
// voxels, with the wave-uniform weights in scalar registers.  Outputs leave as 16-byte
// vectors (8 voxels x CO channels are contiguous in channels-last memory).
//
// Weight gradient: workgroup (brick range, kh) accumulates the 9 (kw, kd) taps x CI x CO
// entries of its kh plane over its voxels in registers, reduces them across the workgroup
// (wave shuffles + LDS) into a per-workgroup partial, and a fixed-order kernel sums the
// partials (deterministic) into dw / dscale / dbias / dcbias.
#include "conv_epi.h"

#include <algorithm>
#include <cstdlib>

namespace vq3d {

namespace {

constexpr int BH = 8, BW = 8, BD = 32, DV = 8;        // brick; voxels per thread along D
constexpr int HL = BH + 2, WL = BW + 2, PL = BD + 2;  // halo lines, positions per line
constexpr int NTC = 256;
constexpr int kTcBlocks = 2048;  // persistent grid cap (bounds the partial buffers)

struct TcArgs {
    int B, H, W, D;  // grid (input == output)
    int circ;
    int nbh, nbw, nbd, nbricks;
    int LS, pad;  // LDS line stride (elements), elements before position 0
    int pro_kind;
    const float *pro_a, *pro_b;
};

template <typename T, int N>
__device__ __forceinline__ void vload(const T *__restrict__ p, float (&o)[N]) {
    if constexpr (sizeof(T) == 2 && (N % 8) == 0) {
#pragma unroll
        for (int q = 0; q < N / 8; ++q) {
            const uint4 u = reinterpret_cast<const uint4 *>(p)[q];
            const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[8 * q + 2 * j] = h2f_lo(w4[j]);
                o[8 * q + 2 * j + 1] = h2f_hi(w4[j]);
            }
        }
    } else if constexpr (sizeof(T) == 4 && (N % 4) == 0) {
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const float4 f = reinterpret_cast<const float4 *>(p)[q];
            o[4 * q] = f.x;
            o[4 * q + 1] = f.y;
            o[4 * q + 2] = f.z;
            o[4 * q + 3] = f.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = ld(p + j);
    }
}

template <typename T, int N>
__device__ __forceinline__ void vstore(T *__restrict__ p, const float (&v)[N]) {
    if constexpr (sizeof(T) == 2 && (N % 8) == 0) {
#pragma unroll
        for (int q = 0; q < N / 8; ++q) {
            uint32_t w4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                w4[j] = uint32_t(f2h(v[8 * q + 2 * j])) | (uint32_t(f2h(v[8 * q + 2 * j + 1])) << 16);
            reinterpret_cast<uint4 *>(p)[q] = uint4{w4[0], w4[1], w4[2], w4[3]};
        }
    } else if constexpr (sizeof(T) == 4 && (N % 4) == 0) {
#pragma unroll
        for (int q = 0; q < N / 4; ++q)
            reinterpret_cast<float4 *>(p)[q] = float4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) st(p + j, v[j]);
    }
}

__device__ __forceinline__ int wrap1(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

// the brick's halo: line (lh, lw) in [0, 10)^2, position p in [0, 34) holds input
// (oh0 - 1 + lh, ow0 - 1 + lw, od0 - 1 + p) at lines[line * LS + pad + p * CI + c]
template <typename T, int CI>
__device__ __forceinline__ void stage_tc(const TcArgs &a, const T *__restrict__ src, int b, int oh0, int ow0, int od0,
                                         const Prologue &pro, T *lines) {
    constexpr int E = 16 / sizeof(T);
    constexpr int UPL = BD * CI / E;  // 16-byte units of a line's main run (positions 1..32)
    const bool raw = pro.kind == VQ3D_PRO_NONE;
    for (int u = threadIdx.x; u < HL * WL * UPL; u += NTC) {
        const int line = u / UPL, r = u - line * UPL;
        const int lh = line / WL, lw = line - lh * WL;
        int ih = oh0 - 1 + lh, iw = ow0 - 1 + lw;
        bool ok = true;
        if (a.circ) {
            ih = wrap1(ih, a.H);
            iw = wrap1(iw, a.W);
        } else {
            ok = unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W);
        }
        uint4 q = uint4{0u, 0u, 0u, 0u};
        if (ok) {
            q = *reinterpret_cast<const uint4 *>(src + (((int64_t(b) * a.H + ih) * a.W + iw) * a.D + od0) * CI + r * E);
            if (!raw) {
                float f[E];
                vload<T, E>(reinterpret_cast<const T *>(&q), f);
#pragma unroll
                for (int j = 0; j < E; ++j) f[j] = pro.apply(f[j]);
                T tmp[E];
                vstore<T, E>(tmp, f);
                q = *reinterpret_cast<const uint4 *>(tmp);
            }
        }
        *reinterpret_cast<uint4 *>(lines + line * a.LS + a.pad + CI + r * E) = q;
    }
    // edge positions 0 and 33 (d = od0 - 1, od0 + 32): wrap or zero padding
    for (int u = threadIdx.x; u < HL * WL * 2 * CI; u += NTC) {
        const int line = u / (2 * CI), r = u - line * (2 * CI);
        const int side = r / CI, c = r - side * CI;
        const int lh = line / WL, lw = line - lh * WL;
        const int pos = side ? PL - 1 : 0;
        int ih = oh0 - 1 + lh, iw = ow0 - 1 + lw, id = od0 - 1 + pos;
        bool ok = true;
        if (a.circ) {
            ih = wrap1(ih, a.H);
            iw = wrap1(iw, a.W);
            id = wrap1(id, a.D);
        } else {
            ok = unsigned(ih) < unsigned(a.H) && unsigned(iw) < unsigned(a.W) && unsigned(id) < unsigned(a.D);
        }
        float v = 0.f;
        if (ok) {
            v = ld(src + (((int64_t(b) * a.H + ih) * a.W + iw) * a.D + id) * CI + c);
            if (!raw) v = pro.apply(v);
        }
        st(lines + line * a.LS + a.pad + pos * CI + c, v);
    }
}

__device__ __forceinline__ void brick_of(const TcArgs &a, int brick, int &b, int &oh0, int &ow0, int &od0) {
    int bi = brick;
    const int bzd = bi % a.nbd;
    bi /= a.nbd;
    const int bzw = bi % a.nbw;
    bi /= a.nbw;
    const int bzh = bi % a.nbh;
    b = bi / a.nbh;
    oh0 = bzh * BH;
    ow0 = bzw * BW;
    od0 = bzd * BD;
}

// the thread's 10 positions x CI of halo line (lh + kh, lw + kw), starting at position dg * 8
template <typename T, int CI>
__device__ __forceinline__ void read_line(const TcArgs &a, const T *lines, int line, int dg, float (&xv)[DV + 2][CI]) {
    const T *p = lines + line * a.LS + a.pad + dg * DV * CI;
#pragma unroll
    for (int q = 0; q < DV + 2; ++q)
#pragma unroll
        for (int c = 0; c < CI; ++c) xv[q][c] = ld(p + q * CI + c);
}

// DG = false: y = epi(conv(pro(x)));  DG = true: gx = bwd_epi(gscale * conv^T(g)) (flipped taps)
// CI / CO: channels of this pass's input / output
template <typename T, int CI, int CO, bool DG>
__global__ __launch_bounds__(NTC) void k_tc(TcArgs a, const T *__restrict__ in, const float *__restrict__ w,
                                           FwdEpi<T> fe, BwdEpi<T> be, const float *__restrict__ gscale,
                                           T *__restrict__ out, float *dpre, float *dpost, float *part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float red[8];
    T *lines = reinterpret_cast<T *>(smem);
    const int tid = threadIdx.x, dg = tid & 3, ln = tid >> 2, lh = ln >> 3, lw = ln & 7;
    const Prologue pro = make_prologue(DG ? VQ3D_PRO_NONE : a.pro_kind, a.pro_a, a.pro_b);
    const float sc = fe.scale ? *fe.scale : 1.f, bias = fe.bias ? *fe.bias : 0.f;
    const float aa = fe.act_a ? *fe.act_a : 0.f, ab = fe.act_b ? *fe.act_b : 0.f;
    const ActDeriv dv = make_deriv(be);
    const float gs = gscale ? *gscale : 1.f;
    float cb[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) cb[o] = (!DG && fe.cbias) ? fe.cbias[o] : 0.f;
    float pre = 0.f, post = 0.f;
    const TileSched bsc = xcd_sched(a.nbricks);
    for (int brick = bsc.t; brick < bsc.end; brick += bsc.step) {
        int b, oh0, ow0, od0;
        brick_of(a, brick, b, oh0, ow0, od0);
        __syncthreads();
        stage_tc<T, CI>(a, in, b, oh0, ow0, od0, pro, lines);
        __syncthreads();
        float acc[DV][CO];
#pragma unroll
        for (int v = 0; v < DV; ++v)
#pragma unroll
            for (int o = 0; o < CO; ++o) acc[v][o] = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                float xv[DV + 2][CI];
                read_line<T, CI>(a, lines, (lh + kh) * WL + lw + kw, dg, xv);
#pragma unroll
                for (int kd = 0; kd < 3; ++kd) {
                    const int tap = (kh * 3 + kw) * 3 + kd;
                    float wv[CO][CI];
#pragma unroll
                    for (int o = 0; o < CO; ++o)
#pragma unroll
                        for (int c = 0; c < CI; ++c)
                            wv[o][c] = DG ? w[(c * CO + o) * 27 + (26 - tap)] : w[(o * CI + c) * 27 + tap];
#pragma unroll
                    for (int v = 0; v < DV; ++v)
#pragma unroll
                        for (int o = 0; o < CO; ++o)
#pragma unroll
                            for (int c = 0; c < CI; ++c) acc[v][o] = fmaf(xv[v + kd][c], wv[o][c], acc[v][o]);
                }
            }
        // epilogue over the thread's 8 voxels x CO (contiguous in memory)
        const int64_t vox0 = ((int64_t(b) * a.H + oh0 + lh) * a.W + ow0 + lw) * a.D + od0 + dg * DV;
        float r[DV * CO];
#pragma unroll
        for (int v = 0; v < DV; ++v)
#pragma unroll
            for (int o = 0; o < CO; ++o) r[v * CO + o] = acc[v][o];
        if (!DG) {
            float res[DV * CO];
            if (fe.res) vload<T, DV * CO>(fe.res + vox0 * CO, res);
#pragma unroll
            for (int i = 0; i < DV * CO; ++i) {
                float val = r[i];
                if (fe.scale) val = val * sc;
                if (fe.bias) val = val + bias;
                if (fe.cbias) val = val + cb[i % CO];
                if (fe.res) val = val + res[i];
                r[i] = epi_act(fe.act, val, aa, ab);
            }
        } else {
            float ax[DV * CO], ad[DV * CO];
            if (dv.mode) vload<T, DV * CO>(be.aux + vox0 * CO, ax);
            if (be.addend) vload<T, DV * CO>(be.addend + vox0 * CO, ad);
#pragma unroll
            for (int i = 0; i < DV * CO; ++i) {
                float val = r[i];
                if (gscale) val = val * gs;
                pre += val;
                if (dv.mode) val = val * dv(ax[i]);
                post += val;
                if (be.addend) val = val + ad[i];
                r[i] = val;
            }
        }
        vstore<T, DV * CO>(out + vox0 * CO, r);
    }
    if (DG && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, NTC, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        if (tid == 0) {
            part[blockIdx.x] = pre;
            part[gridDim.x + blockIdx.x] = post;
        }
    }
}

// *dpre += sum(part[0..n)), *dpost += sum(part[n..2n)) in a fixed order
__global__ __launch_bounds__(256) void k_tc_sum(const float *__restrict__ part, int n, float *dpre, float *dpost) {
    __shared__ float red[8];
    float s0 = 0.f, s1 = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) {
        s0 += part[i];
        s1 += part[n + i];
    }
    {  // both sums in one barrier pair (bit-identical to two block_sum calls)
        float pp[2] = {s0, s1};
        block_sums<float, 256, 2, 4>(pp, red);
        s0 = pp[0];
        s1 = pp[1];
    }
    if (threadIdx.x == 0) {
        if (dpre) *dpre += s0;
        if (dpost) *dpost += s1;
    }
}

// weight gradient: workgroup (brick range, plane = blockIdx.y) with KW (kw, kd) rows per plane:
// KW = 3 -> plane = kh, KW = 1 -> plane = kh * 3 + kw (fewer accumulators for 4 x 4 channels);
// entries e = ((kw' * 3 + kd) * CI + ci) * CO + co, then CO g sums (conv / scalar bias; plane 0)
template <typename T, int CI, int CO, int KW>
__global__ __launch_bounds__(NTC) void k_tc_wgrad(TcArgs a, const T *__restrict__ x, const T *__restrict__ g,
                                                 float *__restrict__ part) {
    constexpr int NE = 3 * KW * CI * CO + CO;
    constexpr int NPL = 9 / KW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float wred[NTC / 64][NE];
    T *lines = reinterpret_cast<T *>(smem);
    const int tid = threadIdx.x, dg = tid & 3, ln = tid >> 2, lh = ln >> 3, lw = ln & 7;
    const int plane = blockIdx.y;
    const int kh = KW == 3 ? plane : plane / 3, kw0 = KW == 3 ? 0 : plane % 3;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    float acc[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) acc[e] = 0.f;
    const TileSched bsc = xcd_sched(a.nbricks);
    for (int brick = bsc.t; brick < bsc.end; brick += bsc.step) {
        int b, oh0, ow0, od0;
        brick_of(a, brick, b, oh0, ow0, od0);
        __syncthreads();
        stage_tc<T, CI>(a, x, b, oh0, ow0, od0, pro, lines);
        __syncthreads();
        const int64_t vox0 = ((int64_t(b) * a.H + oh0 + lh) * a.W + ow0 + lw) * a.D + od0 + dg * DV;
        float gv[DV * CO];
        vload<T, DV * CO>(g + vox0 * CO, gv);
        if (plane == 0) {
#pragma unroll
            for (int v = 0; v < DV; ++v)
#pragma unroll
                for (int o = 0; o < CO; ++o) acc[3 * KW * CI * CO + o] += gv[v * CO + o];
        }
#pragma unroll
        for (int kw = 0; kw < KW; ++kw) {
            float xv[DV + 2][CI];
            read_line<T, CI>(a, lines, (lh + kh) * WL + lw + kw0 + kw, dg, xv);
#pragma unroll
            for (int kd = 0; kd < 3; ++kd)
#pragma unroll
                for (int v = 0; v < DV; ++v)
#pragma unroll
                    for (int c = 0; c < CI; ++c)
#pragma unroll
                        for (int o = 0; o < CO; ++o) {
                            const int e = ((kw * 3 + kd) * CI + c) * CO + o;
                            acc[e] = fmaf(xv[v + kd][c], gv[v * CO + o], acc[e]);
                        }
        }
    }
    // workgroup reduction: xor-shuffle tree per wave, then the 4 waves in order
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        float s = acc[e];
        s = wave_sum(s);
        if (lane == 0) wred[wave][e] = s;
    }
    __syncthreads();
    float *pp = part + (int64_t(blockIdx.x) * NPL + plane) * NE;
    for (int e = tid; e < NE; e += NTC) pp[e] = ((wred[0][e] + wred[1][e]) + (wred[2][e] + wred[3][e]));
}

template <int CI, int CO, int KW, int LANES>
__global__ __launch_bounds__(256) void k_tc_wgrad_reduce(const float *__restrict__ part, int nblk,
                                                        const float *__restrict__ w, const float *__restrict__ escale,
                                                        float *dw, float *dscale, float *dbias, float *dcbias,
                                                        GridSum gsum) {
    constexpr int NE = 3 * KW * CI * CO + CO;
    constexpr int NPL = 9 / KW;
    __shared__ float red[8];
    const int lane = threadIdx.x % LANES;
    const int f = blockIdx.x * (256 / LANES) + threadIdx.x / LANES;  // f = plane * NE + e
    float sum = 0.f;
    if (f < NPL * NE) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int b0 = lane; b0 < nblk; b0 += 8 * LANES) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + u * LANES < nblk) acc[u] += part[int64_t(b0 + u * LANES) * NPL * NE + f];
        }
        sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    sum = group_sum<LANES>(sum);
    float wg = 0.f, bs = 0.f;
    if (f < NPL * NE && lane == 0) {
        const int plane = f / NE, e = f - plane * NE;
        if (e < 3 * KW * CI * CO) {
            const int o = e % CO, r = e / CO, c = r % CI, t = r / CI;  // t = kw' * 3 + kd
            const int tap = plane * 3 * KW + t;                         // (kh * 3 + kw) * 3 + kd
            const int64_t idx = (int64_t(o) * CI + c) * 27 + tap;
            if (dw) dw[idx] += escale ? sum * *escale : sum;
            if (dscale) wg = w[idx] * sum;
        } else if (plane == 0) {
            if (dcbias) dcbias[e - 3 * KW * CI * CO] += sum;
            bs = sum;
        }
    }
    if (dscale || dbias) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {wg, bs};
            block_sums<float, 256, 2, 4>(pp, red);
            wg = pp[0];
            bs = pp[1];
        }
        grid_sum2<256>(gsum, wg, bs, dscale, dbias, red);
    }
}

bool pow124(int c) { return c == 1 || c == 2 || c == 4; }

// (kw, kd) rows per weight-gradient plane: 3 (planes = kh) unless the accumulators would not fit
int tc_kw(int ci, int co) { return ci * co > 4 ? 1 : 3; }

TcArgs make_tc(const vq3d_conv_desc *d, const float *pa, const float *pb, int ci) {
    TcArgs a;
    a.B = d->batch;
    a.H = d->in_h;
    a.W = d->in_w;
    a.D = d->in_d;
    a.circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    a.nbh = a.H / BH;
    a.nbw = a.W / BW;
    a.nbd = a.D / BD;
    a.nbricks = a.B * a.nbh * a.nbw * a.nbd;
    const int esz = d->dtype == VQ3D_HALF ? 2 : 4;
    const int E = 16 / esz;
    a.pad = (E - ci % E) % E;  // position 1 (the main run) starts 16-B aligned
    a.LS = (a.pad + PL * ci + E - 1) / E * E;
    a.pro_kind = d->pro_kind;
    a.pro_a = pa;
    a.pro_b = pb;
    return a;
}

size_t lds_tc(const TcArgs &a, int esz) { return size_t(HL) * WL * a.LS * esz; }

unsigned grid_tc(const TcArgs &a) { return unsigned(std::min(a.nbricks, kTcBlocks)); }

}  // namespace

bool tc_applicable(const vq3d_conv_desc *d) {
    // measured: 1 -> 1 3x faster, 2 -> 2 1.2-2x faster than the MFMA engines; 4 -> 4 is slower
    // (27 x 16 wave-uniform weights per voxel group), so it stays on the MFMA engines
    return d->kernel == 3 && d->stride == 1 && d->pad == 1 && d->cin2 == 0 && pow124(d->cin) && pow124(d->cout) &&
           d->cin * d->cout <= 4 &&
           d->in_h == d->out_h && d->in_w == d->out_w && d->in_d == d->out_d && d->out_h % BH == 0 &&
           d->out_w % BW == 0 && d->out_d % BD == 0 && d->batch >= 1;
}

size_t tc_workspace(const vq3d_conv_desc *d, int pass) {
    if (!tc_applicable(d)) return 0;
    const TcArgs a = make_tc(d, nullptr, nullptr, pass == VQ3D_PASS_BWD_DATA ? d->cout : d->cin);
    const size_t nb = grid_tc(a);
    if (pass == VQ3D_PASS_FWD) return 0;
    if (pass == VQ3D_PASS_BWD_DATA) return 2 * nb * 4;
    const int kw = tc_kw(d->cin, d->cout);
    return nb * (9 / kw) * size_t(3 * kw * d->cin * d->cout + d->cout) * 4;
}

template <typename T>
int launch_tc(const vq3d_conv_desc *d, bool dgrad, const void *in, const float *w, const float *pa, const float *pb,
              const FwdEpi<T> &fe, const BwdEpi<T> &be, const float *gscale, void *out, float *dpre, float *dpost,
              void *ws, size_t ws_bytes, hipStream_t s) {
    const int ci = dgrad ? d->cout : d->cin, co = dgrad ? d->cin : d->cout;
    TcArgs a = make_tc(d, dgrad ? nullptr : pa, dgrad ? nullptr : pb, ci);
    if (dgrad) a.pro_kind = VQ3D_PRO_NONE;
    if (!dgrad && fe.res && fe.res_up2) return fail("conv3d(tiny channels): upsampled residual not supported");
    const unsigned nb = grid_tc(a);
    float *part = nullptr;
    if (dgrad && (dpre || dpost)) {
        if (!ws || ws_bytes < 2 * size_t(nb) * 4) return fail("conv3d_bwd_data(tiny channels): workspace too small");
        part = static_cast<float *>(ws);
    }
    const size_t lds = lds_tc(a, int(sizeof(T)));
#define TC(CI_, CO_)                                                                                         \
    if (ci == CI_ && co == CO_) {                                                                            \
        if (dgrad)                                                                                           \
            k_tc<T, CI_, CO_, true><<<nb, NTC, lds, s>>>(a, (const T *)in, w, fe, be, gscale, (T *)out, dpre, \
                                                         dpost, part);                                       \
        else                                                                                                 \
            k_tc<T, CI_, CO_, false><<<nb, NTC, lds, s>>>(a, (const T *)in, w, fe, be, nullptr, (T *)out,     \
                                                          nullptr, nullptr, nullptr);                        \
    } else
    TC(1, 1) TC(1, 2) TC(1, 4) TC(2, 1) TC(2, 2) TC(4, 1) {
        return fail("conv3d(tiny channels): channel pair not instantiated");
    }
#undef TC
    if (part) k_tc_sum<<<1, 256, 0, s>>>(part, int(nb), dpre, dpost);
    return check_launch(dgrad ? "conv3d_bwd_data(tiny channels)" : "conv3d_fwd(tiny channels)");
}

template <typename T>
int launch_tc_wgrad(const vq3d_conv_desc *d, const void *x, const void *g, const float *pa, const float *pb,
                    const float *w, const float *escale, float *dw, float *dscale, float *dbias, float *dcbias,
                    void *ws, size_t ws_bytes, hipStream_t s) {
    const int ci = d->cin, co = d->cout;
    TcArgs a = make_tc(d, pa, pb, ci);
    const unsigned nb = grid_tc(a);
    const int kw = tc_kw(ci, co), npl = 9 / kw;
    const size_t need = size_t(nb) * npl * (3 * kw * ci * co + co) * 4;
    if (!ws || ws_bytes < need) return fail("conv3d_bwd_weight(tiny channels): workspace too small");
    float *part = static_cast<float *>(ws);
    const size_t lds = lds_tc(a, int(sizeof(T)));
    const dim3 grid{nb, unsigned(npl), 1u};
    int lanes = 1;
    while (lanes < 64 && lanes * 32 < int(nb)) lanes *= 2;
#define RED(CI_, CO_, L)                                                                                        \
    k_tc_wgrad_reduce<CI_, CO_, (CI_ * CO_ > 4 ? 1 : 3), L>                                                    \
        <<<((9 / (CI_ * CO_ > 4 ? 1 : 3)) * (3 * (CI_ * CO_ > 4 ? 1 : 3) * CI_ * CO_ + CO_) + 256 / L - 1) /      \
               (256 / L),                                                                                       \
           256, 0, s>>>(part, int(nb), w, escale, dw, dscale, dbias, dcbias,                                   \
                        grid_sum_for(s, int64_t(npl) * (3 * kw * ci * co + co), dscale || dbias))
#define TW(CI_, CO_)                                                                                            \
    if (ci == CI_ && co == CO_) {                                                                               \
        k_tc_wgrad<T, CI_, CO_, (CI_ * CO_ > 4 ? 1 : 3)><<<grid, NTC, lds, s>>>(a, (const T *)x, (const T *)g,  \
                                                                                part);                          \
        switch (lanes) {                                                                                        \
        case 1: RED(CI_, CO_, 1); break;                                                                        \
        case 2: RED(CI_, CO_, 2); break;                                                                        \
        case 4: RED(CI_, CO_, 4); break;                                                                        \
        case 8: RED(CI_, CO_, 8); break;                                                                        \
        case 16: RED(CI_, CO_, 16); break;                                                                      \
        case 32: RED(CI_, CO_, 32); break;                                                                      \
        default: RED(CI_, CO_, 64); break;                                                                      \
        }                                                                                                       \
    } else
    TW(1, 1) TW(1, 2) TW(1, 4) TW(2, 1) TW(2, 2) TW(4, 1) {
        return fail("conv3d_bwd_weight(tiny channels): channel pair not instantiated");
    }
#undef TW
#undef RED
    return check_launch("conv3d_bwd_weight(tiny channels)");
}

template int launch_tc<float>(const vq3d_conv_desc *, bool, const void *, const float *, const float *, const float *,
                              const FwdEpi<float> &, const BwdEpi<float> &, const float *, void *, float *, float *,
                              void *, size_t, hipStream_t);
template int launch_tc<h16_t>(const vq3d_conv_desc *, bool, const void *, const float *, const float *,
                               const float *, const FwdEpi<h16_t> &, const BwdEpi<h16_t> &, const float *, void *,
                               float *, float *, void *, size_t, hipStream_t);
template int launch_tc_wgrad<float>(const vq3d_conv_desc *, const void *, const void *, const float *, const float *,
                                    const float *, const float *, float *, float *, float *, float *, void *, size_t,
                                    hipStream_t);
template int launch_tc_wgrad<h16_t>(const vq3d_conv_desc *, const void *, const void *, const float *,
                                     const float *, const float *, const float *, float *, float *, float *, float *,
                                     void *, size_t, hipStream_t);

}  // namespace vq3d
