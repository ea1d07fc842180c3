// Few-channel PreActFixupResBlocks (vqvae/layers.py:176-195, mode 'same', no skip conv) on the
// big grids: (block channels C, branch B) = (4, 2) at 512x512x128 (decoder post-upscale blocks),
// (2, 1) at 128x128x32 (50 encoder pre-quantize blocks), (8, 4) at 256x256x64; any grid with
// H % 8 == W % 8 == 0 and D % 16 == 0.  Forward in ONE launch, backward in THREE (fused kernel +
// two-stage fixed-order reduction), for the vq3d_preact_small_* entry points (preact_small.hip keeps its
// brick kernels for the small grids).
//
//   u1  = elu(x + b1a) + b1b      t2 = elu(W1 u1 + b2a) + b2b        (1x1, C -> B)
//   t3  = elu(W2 (*) t2 + b3a) + b3b                                   (3x3x3 circular, B -> B)
//   out = scale * (W3 t3) + b4 + x                                     (1x1, B -> C)
//
// A workgroup owns an 8 x 8 x 16 brick (1024 voxels, 256 threads, 4 voxels each along D: small
// enough LDS for 4-5 workgroups per CU).  The 1x1 convs and the
// activations run on the VALU, one voxel per work item, weights wave-uniform; the 3x3x3 conv and
// its backward run on the matrix cores (v_mfma_f32_16x16x32_bf16) with a "row-windowed" K: for a
// voxel and a tap row (kh, kw) the 3 kd taps x B channels are 3B consecutive bf16 of the halo line
// (position-major [line][pos][B]), padded to 8 (B <= 2) or 16 (B = 4) K entries whose extra
// weights are zero, so one k-step covers 4 (or 2) tap rows of 16 voxels.  Only B of the 16 MFMA
// columns are real: the k^3 conv is still ~2x cheaper on the matrix cores than on the VALU.
//
//   forward  A: t2 on the brick's circular halo (10 x 10 lines x 18 positions) into LDS
//            B: raw W2 (*) t2 per 16-voxel m-tile (matrix cores) into LDS
//            C: per thread 4 consecutive voxels: t2 / t3 (saved for the backward), out
//   backward A: gz3 = bf16(scale W3^T g * elu'(t3)) on the halo; the interior's scalar sums and
//               the W3 gradient (sum t3 (x) g) in registers; t2 on the halo channel-major
//            B: gt2 = W2^T (*) gz3 (flipped taps) per m-tile, and the W2 gradient
//               sum_v gz3[v][co] t2[v + tap][ci] with voxels as the MFMA reduction axis
//            C: per thread 4 voxels: gz1 = bf16(gt2 * elu'(t2)), gx = g + (W1^T gz1) * elu'(x + b1a),
//               the W1 gradient (sum gz1 (x) u1) and the b2 / b1 sums
//            per-workgroup partial rows [workgroup][entry] (the backward is persistent: a
//            workgroup walks a brick range, its sums in registers), summed in a fixed order by
//            k_col_reduce1 / 2.
// Rounding points are the unfused path's: t2, t3, gz3, gz1 rounded to bf16 (the conv operands), fp32
// accumulation; the W1 gradient reads u1 rounded to bf16 (the unfused wgrad's operand).  The
// residual stream x / out (and g / gx) is stored bf16 or fp32 per tensor (template TX / TO): a run
// of blocks keeps it fp32 between its blocks, as the reference's autocast blocks return fp32.
#include "engines.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#ifndef COL_UNROLL_F
#define COL_UNROLL_F 2  // m-tiles per unrolled step of the forward's phase B
#endif
#ifndef COL_UNROLL_B
#define COL_UNROLL_B 2  // ... and of the backward's phase B1
#endif
#ifndef COL_SWEIGHTS
#define COL_SWEIGHTS 1  // the backward's W1 / W3 held in SGPRs (0: plain loads, for A/B timing)
#endif
#ifdef COL_PROBE  // phase clocks of k_col_bwd's first brick per workgroup (tools/probes/col_probe.hip)
__device__ unsigned long long g_col_probe[4096][8];
#define CPROBE_DECL unsigned long long cprobe_t[8] = {};
#define CPROBE(k)                              \
    __builtin_amdgcn_sched_barrier(0);         \
    if (cprobe_t[k] == 0) cprobe_t[k] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);
#define CPROBE_DUMP                                                        \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                             \
        for (int i_ = 0; i_ < 8; ++i_) g_col_probe[blockIdx.x][i_] = cprobe_t[i_];
#else
#define CPROBE_DECL
#define CPROBE(k)
#define CPROBE_DUMP
#endif
#ifndef COL_VSTENCIL
#define COL_VSTENCIL 1  // (2, 1) backward: phase B as VALU stencils + an LDS-grouped reduction (0: MFMA, A/B)
#endif
#ifndef COL_NHB2
#define COL_NHB2 2  // load batches of the (2, 1) backward's halo phase
#endif
#ifndef COL_PAIRS
#define COL_PAIRS 1  // the backward's halo phase on position pairs (0: one position per item, A/B)
#endif
#ifndef FWD_PERSIST
#define FWD_PERSIST 1  // the forward walks brick ranges too (its grid: CArgs::nwg)
#endif

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BH = 8, BW = 8, BD = 16, DV = 4;  // brick; voxels per thread along D
constexpr int HL = BH + 2, WL = BW + 2, PL = BD + 2, NLN = HL * WL, HVX = NLN * PL;
constexpr int NV = BH * BW * BD, NMT = NV / 16;  // 1024 voxels, 64 m-tiles (one per brick line)
constexpr int NT = 256;
static_assert(BD == 16 && NT / (BD / DV) == BH * BW, "m-tile = brick line; thread = (line, D-group)");
#ifndef COL_TP
#define COL_TP 28  // 28: the W2-gradient window reads 2.25 -> 1.5-way (4,2) and 3.7 -> 1.3-way (8,4) bank conflicts (modelled); 24 measured 1.6 % / 6.5 % slower
#endif
constexpr int TP = COL_TP;    // channel-major halo line pitch (positions 0..17, zero pad)
constexpr int ZP = NV + 16;   // channel-major interior pitch
constexpr int PADE = 32;      // zero tail of the position-major halo buffers
constexpr int NSC = 8;        // scalar partials: b4, b3b, b3a, scale, b2b, b2a, b1b, b1a
constexpr int RPC = NT + 4;   // pitch (16-byte slots) of the (2, 1) backward's grouped partial row
// raw k^3 sums [voxel][B] fp32 with one pad float per brick line (16 voxels), so the per-thread
// epilogue reads of 16 lines do not share a bank
__host__ __device__ constexpr int acc_at(int v, int BR_) { return v * BR_ + v / BD; }
constexpr int acc_floats(int BR_) { return NV * BR_ + NV / BD; }

template <int BR>
struct K3 {
    static constexpr int EPR = 3 * BR <= 8 ? 8 : 16;  // K entries per tap row
    static constexpr int RPK = 32 / EPR;              // tap rows per k-step
    static constexpr int KS = (9 + RPK - 1) / RPK;    // k-steps
    static constexpr int NTN = (27 * BR + 15) / 16;   // W2-gradient column tiles
};
template <int C, int BR>
constexpr int n_entries() {
    return BR * C + 27 * BR * BR + BR * C + NSC;  // G3 [o][c], W2 [co][r][kd][ci], W1 [o][c], scalars
}

struct CArgs {
    int B, H, W, D;
    int nbh, nbw, nbd, nbricks;
    int nwg;  // persistent backward grid (workgroups walking brick ranges; its partial rows)
    int xcd;  // XCD-contiguous brick order (measured: faster up to 4096 bricks, slower at 32768)
};

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }
__device__ __forceinline__ float bf(uint32_t u16) { return h2f_lo(u16); }
__device__ __forceinline__ float rbf(float v) { return bf(f2h(v)); }
__device__ __forceinline__ float elu_f(float z) { return z > 0.f ? z : __expf(z) - 1.f; }
// N wave-uniform weights loaded once into SGPRs and laundered, so the compiler keeps them there: as
// plain loads it re-issued them inside the halo / epilogue loops (32 s_load_dword per 4 halo items
// of the (4, 2) backward, each with a lgkmcnt wait that also waited for the LDS stores)
template <int N>
struct SWeights {
    float v[N];
    __device__ __forceinline__ explicit SWeights(const float *__restrict__ w) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            float x = w[i];
            if constexpr (COL_SWEIGHTS) asm volatile("" : "+s"(x));
            v[i] = x;
        }
    }
    __device__ __forceinline__ float operator[](int i) const { return v[i]; }
};
__device__ __forceinline__ float elu_d_act(float t, float b) {
    const float z1 = t - b;
    return z1 > 0.f ? 1.f : z1 + 1.f;
}
__device__ __forceinline__ f32x4 mfma(hx8 a, hx8 b, f32x4 c) {
    return VQ3D_MFMA_16X16X32(a, b, c, 0, 0, 0);
}
// 8 consecutive bf16 from LDS at any element offset of a 4-byte aligned base
__device__ __forceinline__ hx8 read8(const h16_t *base, int off) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(base + (off & ~1));
    const uint32_t sh = uint32_t(off & 1) * 2u;
    const uint32_t u0 = q[0], u1 = q[1], u2 = q[2], u3 = q[3], u4 = q[4];
    const uint4 r = {__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                     __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
    return __builtin_bit_cast(hx8, r);
}
// 8 bf16 at an even element offset (4-byte aligned)
__device__ __forceinline__ hx8 read8e(const h16_t *p) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    return __builtin_bit_cast(hx8, uint4{q[0], q[1], q[2], q[3]});
}
__device__ __forceinline__ hx8 pack8(const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = uint32_t(f2h(v[2 * j])) | (uint32_t(f2h(v[2 * j + 1])) << 16);
    return __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]});
}

// NW dwords (2, 4 or 8) to global memory as 8- / 16-byte stores
template <int NW>
__device__ __forceinline__ void store_words(h16_t *__restrict__ p, const uint32_t (&w)[NW]) {
    if constexpr (NW == 2) {
        *reinterpret_cast<uint2 *>(p) = uint2{w[0], w[1]};
    } else {
        static_assert(NW % 4 == 0, "store width");
#pragma unroll
        for (int i = 0; i < NW / 4; ++i)
            reinterpret_cast<uint4 *>(p)[i] = uint4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
    }
}

// N bf16 <-> fp32 (N = 1, 2, 4, 8: one 2/4/8/16-byte access)
template <int N>
struct Vec {
    using U = typename std::conditional<N == 1, uint16_t,
              typename std::conditional<N == 2, uint32_t, typename std::conditional<N == 4, uint2, uint4>::type>::type>::type;
};
template <int N>
__device__ __forceinline__ void unpack(const typename Vec<N>::U &u, float (&o)[N]) {
    if constexpr (N == 1) {
        o[0] = bf(u);
    } else if constexpr (N == 2) {
        o[0] = h2f_lo(u);
        o[1] = h2f_hi(u);
    } else if constexpr (N == 4) {
        o[0] = h2f_lo(u.x);
        o[1] = h2f_hi(u.x);
        o[2] = h2f_lo(u.y);
        o[3] = h2f_hi(u.y);
    } else {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = h2f_lo(w[i]);
            o[2 * i + 1] = h2f_hi(w[i]);
        }
    }
}
// element i of N packed 16-bit values, as stored (no float round trip)
template <int N>
__device__ __forceinline__ h16_t half_of(const typename Vec<N>::U &u, int i) {
    if constexpr (N == 1) {
        return h16_t(u);
    } else if constexpr (N == 2) {
        return h16_t(i ? u >> 16 : u & 0xffffu);
    } else if constexpr (N == 4) {
        const uint32_t w = i < 2 ? u.x : u.y;
        return h16_t(i & 1 ? w >> 16 : w & 0xffffu);
    } else {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
        return h16_t(i & 1 ? w[i >> 1] >> 16 : w[i >> 1] & 0xffffu);
    }
}
template <int N>
__device__ __forceinline__ typename Vec<N>::U packv(const float (&v)[N]) {
    if constexpr (N == 1) {
        return f2h(v[0]);
    } else {
        uint32_t w[(N + 1) / 2];
#pragma unroll
        for (int i = 0; i < N / 2; ++i) w[i] = uint32_t(f2h(v[2 * i])) | (uint32_t(f2h(v[2 * i + 1])) << 16);
        if constexpr (N == 2) return w[0];
        else if constexpr (N == 4) return uint2{w[0], w[1]};
        else return uint4{w[0], w[1], w[2], w[3]};
    }
}
struct Scal {
    float b1a, b1b, b2a, b2b, b3a, b3b, sc, b4;
};
__device__ __forceinline__ Scal load_scal(const vq3d_preact_params &p) {
    return Scal{*p.bias1a, *p.bias1b, *p.bias2a, *p.bias2b, *p.bias3a, *p.bias3b, *p.scale, *p.bias4};
}

struct Org {
    int b, h0, w0, d0;
};
__device__ __forceinline__ Org brick_org(const CArgs &a, int t) {
    Org o;
    o.d0 = (t % a.nbd) * BD;
    t /= a.nbd;
    o.w0 = (t % a.nbw) * BW;
    t /= a.nbw;
    o.h0 = (t % a.nbh) * BH;
    o.b = t / a.nbh;
    return o;
}
// per halo line: global voxel index of (line, d = d0) (H / W wrapped)
__device__ __forceinline__ void line_table(const CArgs &a, const Org &o, int *lbase) {
    const int t = threadIdx.x;
    if (t < NLN) {
        const int lh = t / WL, lw = t - lh * WL;
        lbase[t] = ((o.b * a.H + wrapm(o.h0 - 1 + lh, a.H)) * a.W + wrapm(o.w0 - 1 + lw, a.W)) * a.D + o.d0;
    }
}
// global voxel of halo item q (line, pos), pos 0 = position -1 (D wrapped)
__device__ __forceinline__ int halo_voxel(const CArgs &a, const Org &o, const int *lbase, int q, int &line, int &pos) {
    line = q / PL;
    pos = q - line * PL;
    const int d = o.d0 - 1 + pos;
    return lbase[line] - o.d0 + (d < 0 ? d + a.D : (d >= a.D ? d - a.D : d));
}
__device__ __forceinline__ bool interior(int line, int pos) {
    const int lh = line / WL, lw = line - lh * WL;
    return lh >= 1 && lh <= BH && lw >= 1 && lw <= BW && pos >= 1 && pos <= BD;
}

// B fragment of k-step s of the row-windowed W2 (DGRAD: transposed, flipped taps)
template <int BR, bool DGRAD>
__device__ __forceinline__ hx8 w2_frag(const float *__restrict__ w2, int s, int lane) {
    using K = K3<BR>;
    const int n = lane & 15, kb = lane >> 4;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * kb + j, r = s * K::RPK + k / K::EPR, e = k % K::EPR, kd = e / BR, c = e - kd * BR;
        float x = 0.f;
        if (r < 9 && e < 3 * BR && n < BR) {
            const int tap = r * 3 + kd;
            x = DGRAD ? w2[(c * BR + n) * 27 + 26 - tap] : w2[(n * BR + c) * 27 + tap];
        }
        v[j] = x;
    }
    return pack8(v);
}

// A fragments of the row-windowed k^3 operand from the position-major halo buffer [line][pos][BR]:
// the lane's part of the element offset, per k-step (m-tile independent), and the m-tile's
// wave-uniform base.  Interior voxel v = 16 mt + row: brick line mt, d = row.
template <int BR>
__device__ __forceinline__ void win_offsets(int row, int kb, int (&off)[K3<BR>::KS]) {
    using K = K3<BR>;
#pragma unroll
    for (int s = 0; s < K::KS; ++s) {
        const int r = min(s * K::RPK + (8 * kb) / K::EPR, 8), e0 = (8 * kb) % K::EPR, kh = r / 3, kw = r - 3 * kh;
        off[s] = ((kh * WL + kw) * PL + row) * BR + e0;
    }
}
__device__ __forceinline__ int win_base(int mt, int BR) {  // m-tile mt = brick line mt
    return ((mt >> 3) * WL + (mt & 7)) * PL * BR;
}
template <int BR>
__device__ __forceinline__ hx8 win_frag(const h16_t *h, int off) {
    if constexpr (BR == 1) return read8(h, off);
    else return read8e(h + off);
}

// ============================================================================================ forward
// TX / TO: storage of the residual stream in / out (bf16 or fp32; a run of blocks carries it in
// fp32 between its blocks like the reference's autocast blocks, layers.py:187-193)
// CH (chained runs, vq3d_preact_small_fwd_chain): bit 0 -- this block's t2 was written by the
// previous block's epilogue (t2in): phase A loads it on the halo instead of forming it from x;
// bit 1 -- the epilogue also forms the NEXT block's t2 from this block's output (as stored, TO) with
// that block's W1 / biases (w1n, pn) and writes it to t2n, so the next launch skips its halo math.
// The formulas and their order are phase A's, so a chained run is bit-identical to an unchained one.
template <typename T>
__device__ __forceinline__ float as_stored(float v) {
    if constexpr (sizeof(T) == 4) return v;
    else return rbf(v);
}
template <int C, int BR>
__device__ __forceinline__ void t2_of(const float (&xf)[C], const float *__restrict__ w1, const Scal &s, float (&t)[BR]) {
    float u[C];
#pragma unroll
    for (int c = 0; c < C; ++c) u[c] = elu_f(xf[c] + s.b1a) + s.b1b;
#pragma unroll
    for (int oo = 0; oo < BR; ++oo) {
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) acc = fmaf(w1[oo * C + c], u[c], acc);
        t[oo] = elu_f(acc + s.b2a) + s.b2b;
    }
}
template <int C, int BR, typename TX, typename TO, int CH = 0>
__global__ __launch_bounds__(NT) void k_col_fwd(CArgs a, const TX *__restrict__ x, const float *__restrict__ w1,
                                                const float *__restrict__ w2, const float *__restrict__ w3,
                                                vq3d_preact_params p, TO *__restrict__ out,
                                                h16_t *__restrict__ t2o, h16_t *__restrict__ t3o,
                                                const h16_t *__restrict__ t2in, const float *__restrict__ w1n,
                                                vq3d_preact_params pn, h16_t *__restrict__ t2n) {
    using K = K3<BR>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *t2h = reinterpret_cast<h16_t *>(smem);            // [HVX][BR] + PADE
    float *accs = reinterpret_cast<float *>(t2h + HVX * BR + PADE);  // [NV][BR] raw W2 (*) t2
    int *lbase = reinterpret_cast<int *>(accs + acc_floats(BR));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kb = lane >> 4, row = lane & 15;
    const Scal s = load_scal(p);
    Scal sn{};
    if constexpr ((CH & 2) != 0) sn = load_scal(pn);
    // one branch channel (BR = 1): phase B as a VALU stencil over the thread's own 4 voxels
    constexpr bool VS = BR == 1 && COL_VSTENCIL;
    const SWeights<VS ? 27 : 1> w2s(w2);
    hx8 fw[K::KS];
#pragma unroll
    for (int k = 0; k < K::KS; ++k)
        if constexpr (!VS) fw[k] = w2_frag<BR, false>(w2, k, lane);  // MFMA path only
    for (int i = tid; i < PADE; i += NT) t2h[HVX * BR + i] = 0;
    int woff[K::KS];
    win_offsets<BR>(row, kb, woff);
    // persistent (FWD_PERSIST): the workgroup walks an XCD-contiguous brick range
    const TileSched sc = FWD_PERSIST ? xcd_sched(a.nbricks)
                                     : TileSched{a.xcd ? xcd_tile(a.nbricks) : int(blockIdx.x), a.nbricks, a.nbricks};
#pragma unroll 1
    for (int brick = sc.t; brick < sc.end; brick += sc.step) {
        const Org o = brick_org(a, brick);
        __syncthreads();  // the previous brick's readers of the LDS tiles are done
        line_table(a, o, lbase);
        __syncthreads();
        // A. t2 on the halo: loaded (chained), or formed from x with every x load issued first
        if constexpr ((CH & 1) != 0) {
            constexpr int P = (HVX + NT - 1) / NT;
            typename Vec<BR>::U tv[P];
#pragma unroll
            for (int u = 0; u < P; ++u) {
                int line, pos;
                const int vx = halo_voxel(a, o, lbase, min(tid + u * NT, HVX - 1), line, pos);
                tv[u] = *reinterpret_cast<const typename Vec<BR>::U *>(t2in + int64_t(vx) * BR);
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const int q = tid + u * NT;
                if (q < HVX) *reinterpret_cast<typename Vec<BR>::U *>(t2h + q * BR) = tv[u];
            }
        } else {
            constexpr int P = (HVX + NT - 1) / NT;
            Raw<TX, C> xv[P];
#pragma unroll
            for (int u = 0; u < P; ++u) {
                int line, pos;
                const int vx = halo_voxel(a, o, lbase, min(tid + u * NT, HVX - 1), line, pos);
                xv[u] = ldraw<TX, C>(x + int64_t(vx) * C);
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const int q = tid + u * NT;
                if (q < HVX) {
                    float xf[C], t[BR];
                    unraw<TX, C>(xv[u], xf);
                    t2_of<C, BR>(xf, w1, s, t);
                    *reinterpret_cast<typename Vec<BR>::U *>(t2h + q * BR) = packv<BR>(t);
                }
            }
        }
        __syncthreads();
        // this thread's 4 voxels (phase C): brick line ln, D-group dg; x in flight during phase B
        const int ln = tid / (BD / DV), dg = tid % (BD / DV);
        const int64_t vox0 = int64_t(lbase[((ln >> 3) + 1) * WL + (ln & 7) + 1]) + dg * DV;
        const Raw<TX, DV * C> xr = ldraw<TX, DV * C>(x + vox0 * C);
        float raw1[DV];  // VS: the thread's raw W2 (*) t2
        if constexpr (VS) {
            // B (BR = 1): voxel d takes positions d .. d + 2 of the 9 neighbour lines, one aligned
            // 6-position run (3 dwords) per line for the thread's 4 voxels; the taps rounded to the
            // 16-bit operands of the MFMA path
            const int lh = ln >> 3, lw = ln & 7, d0 = dg * DV;
            float wr[27];
#pragma unroll
            for (int t = 0; t < 27; ++t) wr[t] = rbf(w2s[t]);
#pragma unroll
            for (int i = 0; i < DV; ++i) raw1[i] = 0.f;
#pragma unroll
            for (int r = 0; r < 9; ++r) {
                const uint32_t *tp = reinterpret_cast<const uint32_t *>(t2h + ((lh + r / 3) * WL + lw + r % 3) * PL + d0);
                float tt[DV + 2];
#pragma unroll
                for (int k = 0; k < (DV + 2) / 2; ++k) {
                    const uint32_t tw = tp[k];
                    tt[2 * k] = bf(tw & 0xffffu);
                    tt[2 * k + 1] = bf(tw >> 16);
                }
#pragma unroll
                for (int kd = 0; kd < 3; ++kd)
#pragma unroll
                    for (int i = 0; i < DV; ++i) raw1[i] = fmaf(wr[3 * r + kd], tt[i + kd], raw1[i]);
            }
        } else {
            // B. raw W2 (*) t2 per m-tile (a fixed trip count, unrolled: the next m-tiles' window reads
            // are in flight during this one's MFMA chain)
#pragma unroll COL_UNROLL_F
            for (int i = 0; i < NMT / (NT / 64); ++i) {
                const int mt = wave + i * (NT / 64);
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                const int wb = win_base(mt, BR);
#pragma unroll
                for (int k = 0; k < K::KS; ++k) acc = mfma(win_frag<BR>(t2h, wb + woff[k]), fw[k], acc);
                if (row < BR) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) accs[acc_at(16 * mt + 4 * kb + j, BR) + row] = acc[j];
                }
            }
        }
        if constexpr (!VS) __syncthreads();  // accs complete
        // C. t3 and out of the thread's 4 voxels (and their t2, saved for the backward)
        const int v0 = ln * BD + dg * DV;
        if (t2o && (CH & 1) == 0) {  // chained: this block's t2 is already in memory
            const h16_t *src = t2h + ((((ln >> 3) + 1) * WL + (ln & 7) + 1) * PL + dg * DV + 1) * BR;
            uint32_t w[DV * BR / 2];
            if constexpr (BR == 1) {  // 4 positions at an odd element offset
                const uint4 u4 = __builtin_bit_cast(uint4, read8(t2h, int(src - t2h)));
                w[0] = u4.x, w[1] = u4.y;
            } else {
#pragma unroll
                for (int i = 0; i < DV * BR / 2; ++i) w[i] = reinterpret_cast<const uint32_t *>(src)[i];
            }
            store_words<DV * BR / 2>(t2o + vox0 * BR, w);
        }
        float t3v[DV][BR];
#pragma unroll
        for (int i = 0; i < DV; ++i)
#pragma unroll
            for (int oo = 0; oo < BR; ++oo)
                t3v[i][oo] = rbf(elu_f((VS ? raw1[i] : accs[acc_at(v0 + i, BR) + oo]) + s.b3a) + s.b3b);
        {
            uint32_t w[DV * BR / 2];
#pragma unroll
            for (int i = 0; i < DV * BR / 2; ++i) {
                const int e0 = 2 * i, e1 = 2 * i + 1;
                w[i] = uint32_t(f2h(t3v[e0 / BR][e0 % BR])) | (uint32_t(f2h(t3v[e1 / BR][e1 % BR])) << 16);
            }
            if (t3o) store_words<DV * BR / 2>(t3o + vox0 * BR, w);  // NULL: eval forward, nothing saved
        }
        float xf[DV * C];
        unraw<TX, DV * C>(xr, xf);
#pragma unroll
        for (int e = 0; e < DV * C; ++e) {
            const int vv = e / C, c = e - vv * C;
            float r = 0.f;
#pragma unroll
            for (int oo = 0; oo < BR; ++oo) r = fmaf(w3[c * BR + oo], t3v[vv][oo], r);
            xf[e] = r * s.sc + s.b4 + xf[e];
        }
        stvec<TO, DV * C>(out + vox0 * C, xf);
        if constexpr ((CH & 2) != 0) {  // the next block's t2 from this output as stored
            float tn[DV][BR];
#pragma unroll
            for (int vv = 0; vv < DV; ++vv) {
                float xs[C];
#pragma unroll
                for (int c = 0; c < C; ++c) xs[c] = as_stored<TO>(xf[vv * C + c]);
                t2_of<C, BR>(xs, w1n, sn, tn[vv]);
            }
            uint32_t w[DV * BR / 2];
#pragma unroll
            for (int i = 0; i < DV * BR / 2; ++i) {
                const int e0 = 2 * i, e1 = 2 * i + 1;
                w[i] = uint32_t(f2h(tn[e0 / BR][e0 % BR])) | (uint32_t(f2h(tn[e1 / BR][e1 % BR])) << 16);
            }
            store_words<DV * BR / 2>(t2n + vox0 * BR, w);
        }
    }  // bricks
}

// ============================================================================================ backward
// g has the storage of the forward's out (TO), x and gx that of its input (TX)
template <int C, int BR, typename TX, typename TO>
__global__ __launch_bounds__(NT) void k_col_bwd(CArgs a, const TO *__restrict__ g, const TX *__restrict__ x,
                                                const h16_t *__restrict__ t2, const h16_t *__restrict__ t3,
                                                const float *__restrict__ w1, const float *__restrict__ w2,
                                                const float *__restrict__ w3, vq3d_preact_params p,
                                                float *__restrict__ part, TX *__restrict__ gx) {
    using K = K3<BR>;
    constexpr int NE = n_entries<C, BR>();
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *z3h = reinterpret_cast<h16_t *>(smem);  // gz3 on the halo [HVX][BR] + PADE
    h16_t *t2T = z3h + HVX * BR + PADE;             // t2 on the halo, channel-major [BR][NLN][TP]
    h16_t *z3T = t2T + BR * NLN * TP;                // gz3 of the brick, channel-major [BR][ZP]
    float *accs = reinterpret_cast<float *>(z3T + BR * ZP);  // [NV][BR] raw W2^T (*) gz3
    int *lbase = reinterpret_cast<int *>(accs + acc_floats(BR));
    float *red = reinterpret_cast<float *>(lbase + NLN);  // [4 waves][NE]
    float *wred = reinterpret_cast<float *>(smem);        // after phase C: [4][NTN][64][4] over z3h / t2T
    static_assert(size_t(HVX * BR + PADE + BR * NLN * TP) * 2 >= size_t(4 * K::NTN * 256) * 4, "W2 sums fit z3h + t2T");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kb = lane >> 4, row = lane & 15;
    CPROBE_DECL
    CPROBE(0)
    const Scal s = load_scal(p);
    const SWeights<C * BR> w3s(w3), w1s(w1);
    const SWeights<(BR == 1 && COL_VSTENCIL) ? 27 : 1> w2s(w2);
    hx8 fw[K::KS];
#pragma unroll
    for (int k = 0; k < K::KS; ++k)
        if constexpr (!(BR == 1 && COL_VSTENCIL)) fw[k] = w2_frag<BR, true>(w2, k, lane);  // MFMA path only
    for (int i = tid; i < PADE; i += NT) z3h[HVX * BR + i] = 0;
    for (int i = tid; i < BR * NLN * (TP - PL) / 2; i += NT) {  // zero the channel-major line tails
        const int l = i / ((TP - PL) / 2), e = i - l * ((TP - PL) / 2);
        reinterpret_cast<uint32_t *>(t2T + l * TP + PL)[e] = 0u;
    }
    // every partial sum of the workgroup's bricks accumulates in registers (the W2 gradient in the
    // MFMA accumulators) and is reduced once, after the last brick
    float s4 = 0.f, s3b = 0.f, s3a = 0.f, ssc = 0.f, g3[BR][C];
    float s2b = 0.f, s2a = 0.f, s1b = 0.f, s1a = 0.f, dw1[BR][C];
#pragma unroll
    for (int oo = 0; oo < BR; ++oo)
#pragma unroll
        for (int c = 0; c < C; ++c) g3[oo][c] = dw1[oo][c] = 0.f;
    // one branch channel (BR = 1): phase B runs as VALU stencils over the thread's own 4 voxels
    // (no MFMA: a single W2 row / column would use 1 / 16 of each), the W2 sums in 27 registers
    constexpr bool VS = BR == 1 && COL_VSTENCIL;
    float dw2[VS ? 27 : 1];
#pragma unroll
    for (int i = 0; i < (VS ? 27 : 1); ++i) dw2[i] = 0.f;
    f32x4 aw[K::NTN];
    int toff[K::NTN];
#pragma unroll
    for (int n = 0; n < K::NTN; ++n) {
        aw[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int col = min(16 * n + row, 27 * BR - 1), r = col / (3 * BR), e = col - r * 3 * BR, kd = e / BR,
                  ci = e - kd * BR, kh = r / 3, kw = r - 3 * kh;
        toff[n] = (ci * NLN + kh * WL + kw) * TP + kd + 8 * (kb & 1);  // + line offset of the k-step
    }
    int woff[K::KS];
    win_offsets<BR>(row, kb, woff);
    // persistent: the workgroup walks a range of bricks (XCD-contiguous)
    const TileSched sc = xcd_sched(a.nbricks);
#pragma unroll 1
    for (int brick = sc.t; brick < sc.end; brick += sc.step) {
        const Org o = brick_org(a, brick);
        __syncthreads();  // the previous brick's readers of the LDS tiles are done
        line_table(a, o, lbase);
        __syncthreads();
        CPROBE(1)
        // A. gz3 on the halo; t2 on the halo (channel-major); interior sums and G3 = sum t3 (x) g.
#if COL_PAIRS
        // Work items are PAIRS of consecutive positions of a halo line (PL is even): one line /
        // position computation per pair, and the channel-major t2 copy and the position-major gz3
        // leave as whole-dword (pair) LDS stores instead of two 16-bit stores into one dword.
        // Two batches of pairs (COL_NHB2 = 1 for 2 channels measured no faster), every load of a
        // batch issued before its math.
        constexpr int NPAIR = HVX / 2, HP = PL / 2, NHB = C <= 2 ? COL_NHB2 : 2;
        static_assert(PL % 2 == 0 && TP % 2 == 0 && 2 * BR <= 8, "position pairs are dword aligned");
        constexpr int PH = ((NPAIR + NT - 1) / NT + NHB - 1) / NHB;
#pragma unroll 1
        for (int half = 0; half < NHB; ++half) {
            constexpr int P = PH;
            Raw<TO, C> gv[P][2];
            typename Vec<BR>::U tv3[P][2], tv2[P][2];
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const int qq = min(tid + (half * PH + u) * NT, NPAIR - 1), line = qq / HP, pos0 = 2 * (qq - line * HP);
                const int lb = lbase[line] - o.d0;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int d = o.d0 - 1 + pos0 + e;
                    const int vx = lb + (d < 0 ? d + a.D : (d >= a.D ? d - a.D : d));
                    gv[u][e] = ldraw<TO, C>(g + int64_t(vx) * C);
                    tv3[u][e] = *reinterpret_cast<const typename Vec<BR>::U *>(t3 + int64_t(vx) * BR);
                    tv2[u][e] = *reinterpret_cast<const typename Vec<BR>::U *>(t2 + int64_t(vx) * BR);
                }
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const int qp = tid + (half * PH + u) * NT;
                if (qp < NPAIR) {
                    const int line = qp / HP, pos0 = 2 * (qp - line * HP);
                    const int lh = line / WL, lw = line - lh * WL;
                    const bool lin = lh >= 1 && lh <= BH && lw >= 1 && lw <= BW;  // an interior line
                    const int vb = ((lh - 1) * BW + lw - 1) * BD - 1;            // interior index of position 0
                    float z[2][BR];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int pos = pos0 + e;
                        const bool in = lin && pos >= 1 && pos <= BD;
                        float gf[C], t3f[BR];
                        unraw<TO, C>(gv[u][e], gf);
                        unpack<BR>(tv3[u][e], t3f);
#pragma unroll
                        for (int oo = 0; oo < BR; ++oo) {
                            float acc = 0.f;
#pragma unroll
                            for (int c = 0; c < C; ++c) acc = fmaf(w3s[c * BR + oo], gf[c], acc);
                            const float gt3 = s.sc * acc;
                            z[e][oo] = gt3 * elu_d_act(t3f[oo], s.b3b);
                            if (in) {
                                s3b += gt3;
                                s3a += z[e][oo];
                                ssc = fmaf(acc, t3f[oo], ssc);
#pragma unroll
                                for (int c = 0; c < C; ++c) g3[oo][c] = fmaf(t3f[oo], gf[c], g3[oo][c]);
                            }
                        }
                        if (in) {
#pragma unroll
                            for (int c = 0; c < C; ++c) s4 += gf[c];
#pragma unroll
                            for (int oo = 0; oo < BR; ++oo) z3T[oo * ZP + vb + pos] = f2h(z[e][oo]);
                        }
                    }
#pragma unroll
                    for (int oo = 0; oo < BR; ++oo)  // the stored bits of the pair's t2, channel oo
                        *reinterpret_cast<uint32_t *>(t2T + (oo * NLN + line) * TP + pos0) =
                            uint32_t(half_of<BR>(tv2[u][0], oo)) | (uint32_t(half_of<BR>(tv2[u][1], oo)) << 16);
                    // gz3 of the pair: 2 BR contiguous 16-bit values at (line, pos0)
                    float zz[2 * BR];
#pragma unroll
                    for (int e = 0; e < 2; ++e)
#pragma unroll
                        for (int oo = 0; oo < BR; ++oo) zz[e * BR + oo] = z[e][oo];
                    *reinterpret_cast<typename Vec<2 * BR>::U *>(z3h + (line * PL + pos0) * BR) = packv<2 * BR>(zz);
                }
            }
        }
#else
        // two batches of halo items: every load of a batch issued before its math (registers)
        constexpr int PH = ((HVX + NT - 1) / NT + 1) / 2;
#pragma unroll 1
        for (int half = 0; half < 2; ++half) {
            constexpr int P = PH;
            Raw<TO, C> gv[P];
            typename Vec<BR>::U tv3[P], tv2[P];
#pragma unroll
            for (int u = 0; u < P; ++u) {
                int line, pos;
                const int vx = halo_voxel(a, o, lbase, min(tid + (half * PH + u) * NT, HVX - 1), line, pos);
                gv[u] = ldraw<TO, C>(g + int64_t(vx) * C);
                tv3[u] = *reinterpret_cast<const typename Vec<BR>::U *>(t3 + int64_t(vx) * BR);
                tv2[u] = *reinterpret_cast<const typename Vec<BR>::U *>(t2 + int64_t(vx) * BR);
            }
#pragma unroll
            for (int u = 0; u < P; ++u) {
                const int q = tid + (half * PH + u) * NT;
                if (q < HVX) {
                    const int line = q / PL, pos = q - line * PL;
                    const bool in = interior(line, pos);
                    float gf[C], t3f[BR], t2f[BR], z[BR];
                    unraw<TO, C>(gv[u], gf);
                    unpack<BR>(tv3[u], t3f);
                    unpack<BR>(tv2[u], t2f);
#pragma unroll
                    for (int oo = 0; oo < BR; ++oo) {
                        float acc = 0.f;
#pragma unroll
                        for (int c = 0; c < C; ++c) acc = fmaf(w3s[c * BR + oo], gf[c], acc);
                        const float gt3 = s.sc * acc;
                        z[oo] = gt3 * elu_d_act(t3f[oo], s.b3b);
                        if (in) {
                            s3b += gt3;
                            s3a += z[oo];
                            ssc = fmaf(acc, t3f[oo], ssc);
#pragma unroll
                            for (int c = 0; c < C; ++c) g3[oo][c] = fmaf(t3f[oo], gf[c], g3[oo][c]);
                        }
                        t2T[(oo * NLN + line) * TP + pos] = half_of<BR>(tv2[u], oo);  // the stored bits
                    }
                    const typename Vec<BR>::U zp = packv<BR>(z);
                    *reinterpret_cast<typename Vec<BR>::U *>(z3h + q * BR) = zp;
                    if (in) {
#pragma unroll
                        for (int c = 0; c < C; ++c) s4 += gf[c];
                        const int lh = line / WL, lw = line - lh * WL;
                        const int v = ((lh - 1) * BW + lw - 1) * BD + pos - 1;
#pragma unroll
                        for (int oo = 0; oo < BR; ++oo) z3T[oo * ZP + v] = f2h(z[oo]);
                    }
                }
            }
        }
#endif
        __syncthreads();
        CPROBE(2)
        // the thread's 4 voxels (phase C): g and x in flight during phase B
        const int ln = tid / (BD / DV), dg = tid % (BD / DV);
        const int64_t vox0 = int64_t(lbase[((ln >> 3) + 1) * WL + (ln & 7) + 1]) + dg * DV;
        constexpr int NXB = DV * C / 8;  // 8-element pieces of the thread's 4 voxels
        // phase C's first x / g piece: VS issues it before the stencils, the MFMA path after phase B
        // (registers: occupancy)
        const TX *xp = x + vox0 * C;
        const TO *gp = g + vox0 * C;
        Raw<TX, 8> xq;
        Raw<TO, 8> gq;
        if constexpr (VS) {
            xq = ldraw<TX, 8>(xp);
            gq = ldraw<TO, 8>(gp);
        }
        float raw1[DV];  // VS: the thread's raw W2^T (*) gz3
        if constexpr (VS) {
            // B (BR = 1). Voxel d of the thread's line takes positions d .. d + 2 of the 9 neighbour
            // lines: one aligned 6-position run (3 dwords) of gz3 and of t2 per line for all 4 voxels.
            const int lh = ln >> 3, lw = ln & 7, d0 = dg * DV;
            float wr[27];  // the flipped taps as the 16-bit operands the MFMA path rounds them to
#pragma unroll
            for (int t = 0; t < 27; ++t) wr[t] = rbf(w2s[26 - t]);
            const uint2 zq = *reinterpret_cast<const uint2 *>(z3T + ln * BD + d0);  // the 4 voxels' gz3
            const float gz[DV] = {bf(zq.x & 0xffffu), bf(zq.x >> 16), bf(zq.y & 0xffffu), bf(zq.y >> 16)};
#pragma unroll
            for (int i = 0; i < DV; ++i) raw1[i] = 0.f;
#pragma unroll
            for (int r = 0; r < 9; ++r) {
                const int L = (lh + r / 3) * WL + lw + r % 3;
                const uint32_t *zp = reinterpret_cast<const uint32_t *>(z3h + L * PL + d0);
                const uint32_t *tp = reinterpret_cast<const uint32_t *>(t2T + L * TP + d0);
                float zz[DV + 2], tt[DV + 2];
#pragma unroll
                for (int k = 0; k < (DV + 2) / 2; ++k) {
                    const uint32_t zw = zp[k], tw = tp[k];
                    zz[2 * k] = bf(zw & 0xffffu);
                    zz[2 * k + 1] = bf(zw >> 16);
                    tt[2 * k] = bf(tw & 0xffffu);
                    tt[2 * k + 1] = bf(tw >> 16);
                }
#pragma unroll
                for (int kd = 0; kd < 3; ++kd) {
                    const float wf = wr[3 * r + kd];
#pragma unroll
                    for (int i = 0; i < DV; ++i) {
                        raw1[i] = fmaf(wf, zz[i + kd], raw1[i]);
                        dw2[3 * r + kd] = fmaf(gz[i], tt[i + kd], dw2[3 * r + kd]);
                    }
                }
            }
        } else {
            // B1. raw W2^T (*) gz3 per m-tile (flipped taps; fixed trip count, unrolled as the forward's)
#pragma unroll COL_UNROLL_B
            for (int i = 0; i < NMT / (NT / 64); ++i) {
                const int mt = wave + i * (NT / 64);
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                const int wb = win_base(mt, BR);
#pragma unroll
                for (int k = 0; k < K::KS; ++k) acc = mfma(win_frag<BR>(z3h, wb + woff[k]), fw[k], acc);
                if (row < BR) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) accs[acc_at(16 * mt + 4 * kb + j, BR) + row] = acc[j];
                }
            }
            // B2. W2 gradient: D[co][col] += sum_v gz3[v][co] * t2win[v][col], col = r * 3B + kd * B + ci;
            // wave w takes the 32-voxel k-steps 8 w .. 8 w + 7 (two brick lines each; lane kb: line
            // 2 ks + kb / 2, d = 8 (kb & 1) + j)
#pragma unroll 2
            for (int ks = 8 * wave; ks < 8 * wave + 8; ++ks) {
                // rows >= B of the A operand only feed discarded D rows: read row B - 1 again
                const hx8 af = *reinterpret_cast<const hx8 *>(z3T + min(row, BR - 1) * ZP + 32 * ks + 8 * kb);
                const int lk = 2 * ks + (kb >> 1), lo = ((lk >> 3) * WL + (lk & 7)) * TP;
#pragma unroll
                for (int n = 0; n < K::NTN; ++n) aw[n] = mfma(af, read8(t2T, toff[n] + lo), aw[n]);
            }
        }
        if constexpr (!VS) __syncthreads();  // accs complete (VS: phase C reads registers and phase-A LDS)
        CPROBE(3)
        // C. gz1, gx, W1 gradient, b2 / b1 sums over the thread's 4 voxels
        const int v0 = ln * BD + dg * DV;
        // 8-element pieces of the thread's 4 voxels' x / g (PV voxels each), the next piece's loads in
        // flight during the current one's math (one piece of registers at a time: occupancy)
        constexpr int PV = 8 / C;
        const int hl0 = ((ln >> 3) + 1) * WL + (ln & 7) + 1;
        if constexpr (!VS) {
            xq = ldraw<TX, 8>(xp);
            gq = ldraw<TO, 8>(gp);
        }
#pragma unroll 1
        for (int pc = 0; pc < NXB; ++pc) {
            Raw<TX, 8> xn = xq;
            Raw<TO, 8> gn = gq;
            if (pc + 1 < NXB) {
                xn = ldraw<TX, 8>(xp + 8 * (pc + 1));
                gn = ldraw<TO, 8>(gp + 8 * (pc + 1));
            }
            float xe[8], ge[8], ov[8];
            unraw<TX, 8>(xq, xe);
            unraw<TO, 8>(gq, ge);
#pragma unroll
            for (int vi = 0; vi < PV; ++vi) {
                const int i = pc * PV + vi;
                float z1[BR];
#pragma unroll
                for (int oo = 0; oo < BR; ++oo) {
                    float gt2;
                    if constexpr (VS) gt2 = raw1[i];
                    else gt2 = accs[acc_at(v0 + i, BR) + oo];
                    const float t2v = bf(t2T[(oo * NLN + hl0) * TP + dg * DV + i + 1]);
                    const float zz = gt2 * elu_d_act(t2v, s.b2b);
                    s2b += gt2;
                    s2a += zz;
                    z1[oo] = rbf(zz);
                }
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    float gt1 = 0.f;
#pragma unroll
                    for (int oo = 0; oo < BR; ++oo) gt1 = fmaf(w1s[oo * C + c], z1[oo], gt1);
                    const int e = vi * C + c;
                    const float zx = xe[e] + s.b1a;
                    const float e1 = zx > 0.f ? 1.f : __expf(zx);
                    const float u1 = rbf((zx > 0.f ? zx : e1 - 1.f) + s.b1b);
                    s1b += gt1;
                    s1a = fmaf(gt1, e1, s1a);
                    ov[e] = ge[e] + gt1 * e1;
#pragma unroll
                    for (int oo = 0; oo < BR; ++oo) dw1[oo][c] = fmaf(z1[oo], u1, dw1[oo][c]);
                }
            }
            stvec<TX, 8>(gx + vox0 * C + 8 * pc, ov);
            xq = xn;
            gq = gn;
        }
    }  // bricks
    CPROBE(4)
    if constexpr (VS) {
        // every entry of the partial row, in row order, to LDS as groups of 4 ([group][RPC][4] over
        // the dead tiles; one 16-byte store per group), then a row of 16 threads per group sums its
        // NT slots and reduces on the DPP network: 10 short chains instead of 39 wave-wide DPP trees
        constexpr int NG = (NE + 3) / 4;
        float vals[NG * 4];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            vals[c] = g3[0][c];
            vals[C + 27 + c] = dw1[0][c];
        }
#pragma unroll
        for (int i = 0; i < 27; ++i) vals[C + i] = dw2[i];
        const float sc8[NSC] = {s4, s3b, s3a, ssc, s2b, s2a, s1b, s1a};
#pragma unroll
        for (int k = 0; k < NSC; ++k) vals[2 * C + 27 + k] = sc8[k];
#pragma unroll
        for (int i = NE; i < NG * 4; ++i) vals[i] = 0.f;
        float4 *grp = reinterpret_cast<float4 *>(smem);
        __syncthreads();  // every wave is past phase C (the LDS tiles are dead)
#pragma unroll
        for (int gi = 0; gi < NG; ++gi)
            grp[gi * RPC + tid] = make_float4(vals[4 * gi], vals[4 * gi + 1], vals[4 * gi + 2], vals[4 * gi + 3]);
        __syncthreads();
        CPROBE(4)
        CPROBE(5)
        for (int g0 = 0; g0 < NG; g0 += NT / 16) {
            const int gi = g0 + (tid >> 4), q = tid & 15;
            if (gi < NG) {
                float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int i = q; i < NT; i += 16) {
                    const float4 v = grp[gi * RPC + i];
                    t.x += v.x;
                    t.y += v.y;
                    t.z += v.z;
                    t.w += v.w;
                }
                const float tv[4] = {group_sum<16>(t.x), group_sum<16>(t.y), group_sum<16>(t.z), group_sum<16>(t.w)};
                if (q < 4 && 4 * gi + q < NE) part[int64_t(blockIdx.x) * NE + 4 * gi + q] = tv[q];
            }
        }
    } else {
        // partial row of this brick: per-wave shuffle sums, then the 4 waves in order
        {
            auto put = [&](int e, float v) {
                const float t = wave_sum(v);
                if (lane == 0) red[wave * NE + e] = t;
            };
#pragma unroll
            for (int oo = 0; oo < BR; ++oo)
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    put(oo * C + c, g3[oo][c]);
                    put(BR * C + 27 * BR * BR + oo * C + c, dw1[oo][c]);
                }
            const float sc8[NSC] = {s4, s3b, s3a, ssc, s2b, s2a, s1b, s1a};
#pragma unroll
            for (int k = 0; k < NSC; ++k) put(2 * BR * C + 27 * BR * BR + k, sc8[k]);
        }
        CPROBE(5)
        __syncthreads();  // every wave is past phase C (t2T) before the W2 sums go over it
        // W2 accumulators: D rows 4 kb + j = co, columns 16 n + row = col
#pragma unroll
        for (int n = 0; n < K::NTN; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) wred[((wave * K::NTN + n) * 64 + lane) * 4 + j] = aw[n][j];
        __syncthreads();
        for (int e = tid; e < NE; e += NT) {
            float t = 0.f;
            if (e >= BR * C && e < BR * C + 27 * BR * BR) {
                const int r2 = e - BR * C, co = r2 / (27 * BR), col = r2 - co * 27 * BR;
                const int n = col >> 4, l = 16 * (co >> 2) + (col & 15), j = co & 3;
#pragma unroll
                for (int w = 0; w < NT / 64; ++w) t += wred[((w * K::NTN + n) * 64 + l) * 4 + j];
            } else {
#pragma unroll
                for (int w = 0; w < NT / 64; ++w) t += red[w * NE + e];
            }
            part[int64_t(blockIdx.x) * NE + e] = t;  // the workgroup's row: one contiguous write
        }
    }
    CPROBE(6)
    CPROBE_DUMP
}

// Fixed-order sum of the partial rows [row][NE]: stage 1, workgroup r sums rows
// [r * RCH, (r + 1) * RCH) per entry (threads over entries: coalesced rows) into part2[r][e];
// stage 2 sums the stage-1 rows per entry in order and adds into the gradient buffers.
constexpr int RCH = 128;
template <int C, int BR>
__device__ __forceinline__ void col_reduce1(const float *__restrict__ part, int nb, float *__restrict__ part2) {
    constexpr int NE = n_entries<C, BR>();
    const int b0 = blockIdx.x * RCH, b1 = min(nb, b0 + RCH);
    for (int e = threadIdx.x; e < NE; e += 256) {
        float t = 0.f;
#pragma unroll 8
        for (int b = b0; b < b1; ++b) t += part[int64_t(b) * NE + e];
        part2[int64_t(blockIdx.x) * NE + e] = t;
    }
}
template <int C, int BR>
__global__ __launch_bounds__(256) void k_col_reduce1(const float *__restrict__ part, int nb, float *__restrict__ part2) {
    col_reduce1<C, BR>(part, nb, part2);
}
template <int C, int BR>
__device__ __forceinline__ void col_reduce2(const float *__restrict__ part2, int nr, const float *__restrict__ scale,
                                            const vq3d_preact_grads &gr);
template <int C, int BR>
__global__ __launch_bounds__(256) void k_col_reduce2(const float *__restrict__ part2, int nr, const float *__restrict__ scale,
                                                     vq3d_preact_grads gr) {
    col_reduce2<C, BR>(part2, nr, scale, gr);
}
// both stages for a whole run of blocks (blockIdx.y = block; its workspace at y * stride floats,
// its gradient / scale pointers from the run's [block][11] device tables)
template <int C, int BR>
__global__ __launch_bounds__(256) void k_col_reduce1_run(float *__restrict__ ws, size_t stride, int nb) {
    float *part = ws + blockIdx.y * stride;
    col_reduce1<C, BR>(part, nb, part + size_t(nb) * n_entries<C, BR>());
}
template <int C, int BR>
__global__ __launch_bounds__(256) void k_col_reduce2_run(const float *__restrict__ ws, size_t stride, int nb, int nr,
                                                         float *const *gtab, const float *const *ptab) {
    float *const *g = gtab + blockIdx.y * 11;
    const vq3d_preact_grads gr{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10]};
    col_reduce2<C, BR>(ws + blockIdx.y * stride + size_t(nb) * n_entries<C, BR>(), nr, ptab[blockIdx.y * 11 + 9], gr);
}
template <int C, int BR>
__device__ __forceinline__ void col_reduce2(const float *__restrict__ part2, int nr, const float *__restrict__ scale,
                                            const vq3d_preact_grads &gr) {
    constexpr int E1 = BR * C, E2 = 27 * BR * BR, E3 = BR * C, NE = n_entries<C, BR>();
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= NE) return;
    float t = 0.f;
#pragma unroll 8
    for (int r = 0; r < nr; ++r) t += part2[int64_t(r) * NE + e];
    if (e < E1) {  // G3 [o][c] -> dW3 [c][o] * scale
        const int oo = e / C, c = e - oo * C;
        gr.dw3[c * BR + oo] += *scale * t;
    } else if (e < E1 + E2) {  // [co][r][kd][ci] -> dW2 [co][ci][r * 3 + kd]
        const int r2 = e - E1, co = r2 / (27 * BR), col = r2 - co * 27 * BR, r = col / (3 * BR),
                  el = col - r * 3 * BR, kd = el / BR, ci = el - kd * BR;
        gr.dw2[(co * BR + ci) * 27 + r * 3 + kd] += t;
    } else if (e < E1 + E2 + E3) {
        gr.dw1[e - E1 - E2] += t;  // [o][c]
    } else {
        float *const sl[NSC] = {gr.dbias4, gr.dbias3b, gr.dbias3a, gr.dscale, gr.dbias2b, gr.dbias2a, gr.dbias1b, gr.dbias1a};
        *sl[e - E1 - E2 - E3] += t;
    }
}

template <int C, int BR>
constexpr size_t fwd_lds() {
    return size_t(HVX * BR + PADE) * 2 + size_t(acc_floats(BR)) * 4 + NLN * 4;
}
template <int C, int BR>
constexpr size_t bwd_lds() {
    const size_t tiles = size_t(HVX * BR + PADE + BR * NLN * TP + BR * ZP) * 2 + size_t(acc_floats(BR)) * 4 +
                         NLN * 4 + size_t(4 * n_entries<C, BR>()) * 4;
    if (BR == 1 && COL_VSTENCIL)  // + room for the grouped partial-row reduction over the tiles
        return std::max(tiles, size_t((n_entries<C, BR>() + 3) / 4) * RPC * 16);
    return tiles;
}

// persistent backward: max(512, bricks / 16) workgroups (a multiple of 8: XCD-contiguous ranges),
// each reducing its bricks' partial sums in registers into one partial row (measured: (4, 2) at
// 512^2 x 128, 32,768 bricks: 771 us one brick per workgroup, 746 at 1,024 workgroups, 641 at
// 2,048, 644 at 4,096; (8, 4) at 256^2 x 64, 4,096 bricks: 256 / 185 at 512 / 216 at 2,048)
int col_wg(int nbricks) {
    static const int env = [] {  // timing experiments only: VQ3D_COL_WG fixes the cap (read once)
        const char *e = std::getenv("VQ3D_COL_WG");
        return e ? std::atoi(e) : 0;
    }();
    return env > 0 ? env : std::max(512, (nbricks / 16) & ~7);
}

CArgs make_args(int B, int H, int W, int D) {
    CArgs a;
    a.B = B;
    a.H = H;
    a.W = W;
    a.D = D;
    a.nbh = H / BH;
    a.nbw = W / BW;
    a.nbd = D / BD;
    a.nbricks = B * a.nbh * a.nbw * a.nbd;
    a.xcd = a.nbricks <= 4096;
    a.nwg = std::min(a.nbricks, col_wg(a.nbricks));
    return a;
}

template <class Kern>
void allow(Kern k, size_t lds) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    (void)hipGetLastError();
}

// the chain links of one forward launch (CH bits: 1 chained in, 2 chained out)
struct FwdChain {
    int ch = 0;
    const h16_t *t2in = nullptr;
    const float *w1n = nullptr;
    vq3d_preact_params pn{};
    h16_t *t2n = nullptr;
};

template <int C, int BR, typename TX, typename TO, int CH>
void launch_fwd_ch(const CArgs &a, const void *x, const float *w1, const float *w2, const float *w3,
                   const vq3d_preact_params &p, void *out, h16_t *t2, h16_t *t3, const FwdChain &c, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        allow(k_col_fwd<C, BR, TX, TO, CH>, fwd_lds<C, BR>());
        attr = true;
    }
    k_col_fwd<C, BR, TX, TO, CH><<<FWD_PERSIST ? a.nwg : a.nbricks, NT, fwd_lds<C, BR>(), s>>>(
        a, static_cast<const TX *>(x), w1, w2, w3, p, static_cast<TO *>(out), t2, t3, c.t2in, c.w1n, c.pn, c.t2n);
}
template <int C, int BR, typename TX, typename TO>
void launch_fwd(const CArgs &a, const void *x, const float *w1, const float *w2, const float *w3,
                const vq3d_preact_params &p, void *out, h16_t *t2, h16_t *t3, const FwdChain &c, hipStream_t s) {
    switch (c.ch) {
    case 1: launch_fwd_ch<C, BR, TX, TO, 1>(a, x, w1, w2, w3, p, out, t2, t3, c, s); break;
    case 2: launch_fwd_ch<C, BR, TX, TO, 2>(a, x, w1, w2, w3, p, out, t2, t3, c, s); break;
    case 3: launch_fwd_ch<C, BR, TX, TO, 3>(a, x, w1, w2, w3, p, out, t2, t3, c, s); break;
    default: launch_fwd_ch<C, BR, TX, TO, 0>(a, x, w1, w2, w3, p, out, t2, t3, c, s); break;
    }
}
template <int C, int BR, typename TX, typename TO>
void launch_bwd(const CArgs &a, const void *g, const void *x, const h16_t *t2, const h16_t *t3, const float *w1,
                const float *w2, const float *w3, const vq3d_preact_params &p, const vq3d_preact_grads &gr, float *part,
                void *gx, int stages, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        allow(k_col_bwd<C, BR, TX, TO>, bwd_lds<C, BR>());
        attr = true;
    }
    if (stages & 1)
        k_col_bwd<C, BR, TX, TO><<<a.nwg, NT, bwd_lds<C, BR>(), s>>>(a, static_cast<const TO *>(g),
                                                                     static_cast<const TX *>(x), t2, t3, w1, w2, w3, p,
                                                                     part, static_cast<TX *>(gx));
    const int nr = (a.nwg + RCH - 1) / RCH;
    float *part2 = part + size_t(a.nwg) * n_entries<C, BR>();
    if (stages & 2) {
        k_col_reduce1<C, BR><<<nr, 256, 0, s>>>(part, a.nwg, part2);
        k_col_reduce2<C, BR><<<(n_entries<C, BR>() + 255) / 256, 256, 0, s>>>(part2, nr, p.scale, gr);
    }
}

// the (x, out) storage pair: VQ3D_HALF / VQ3D_F32 each
template <int C, int BR>
void fwd_io(int xdt, int odt, const CArgs &a, const void *x, const float *w1, const float *w2, const float *w3,
            const vq3d_preact_params &p, void *out, h16_t *t2, h16_t *t3, const FwdChain &c, hipStream_t s) {
    if (xdt == VQ3D_HALF && odt == VQ3D_HALF) launch_fwd<C, BR, h16_t, h16_t>(a, x, w1, w2, w3, p, out, t2, t3, c, s);
    else if (xdt == VQ3D_HALF) launch_fwd<C, BR, h16_t, float>(a, x, w1, w2, w3, p, out, t2, t3, c, s);
    else if (odt == VQ3D_HALF) launch_fwd<C, BR, float, h16_t>(a, x, w1, w2, w3, p, out, t2, t3, c, s);
    else launch_fwd<C, BR, float, float>(a, x, w1, w2, w3, p, out, t2, t3, c, s);
}
template <int C, int BR>
void bwd_io(int xdt, int odt, const CArgs &a, const void *g, const void *x, const h16_t *t2, const h16_t *t3,
            const float *w1, const float *w2, const float *w3, const vq3d_preact_params &p, const vq3d_preact_grads &gr,
            float *part, void *gx, int stages, hipStream_t s) {
    if (xdt == VQ3D_HALF && odt == VQ3D_HALF)
        launch_bwd<C, BR, h16_t, h16_t>(a, g, x, t2, t3, w1, w2, w3, p, gr, part, gx, stages, s);
    else if (xdt == VQ3D_HALF) launch_bwd<C, BR, h16_t, float>(a, g, x, t2, t3, w1, w2, w3, p, gr, part, gx, stages, s);
    else if (odt == VQ3D_HALF) launch_bwd<C, BR, float, h16_t>(a, g, x, t2, t3, w1, w2, w3, p, gr, part, gx, stages, s);
    else launch_bwd<C, BR, float, float>(a, g, x, t2, t3, w1, w2, w3, p, gr, part, gx, stages, s);
}

}  // namespace

template <int C, int BR>
void launch_reduce_run(const CArgs &a, int nblocks, float *ws, size_t stride_f, float *const *gtab,
                       const float *const *ptab, hipStream_t s) {
    const int nr = (a.nwg + RCH - 1) / RCH;
    k_col_reduce1_run<C, BR><<<dim3(nr, nblocks), 256, 0, s>>>(ws, stride_f, a.nwg);
    k_col_reduce2_run<C, BR><<<dim3((n_entries<C, BR>() + 255) / 256, nblocks), 256, 0, s>>>(ws, stride_f, a.nwg, nr,
                                                                                        gtab, ptab);
}

int col_reduce_run(int nblocks, int batch, int C, int BR, int h, int w, int d, void *workspaces, size_t stride,
                   float *const *gtab, const float *const *ptab, hipStream_t s) {
    const CArgs a = make_args(batch, h, w, d);
    float *ws = static_cast<float *>(workspaces);
    const size_t sf = stride / 4;
    if (C == 2) launch_reduce_run<2, 1>(a, nblocks, ws, sf, gtab, ptab, s);
    else if (C == 4) launch_reduce_run<4, 2>(a, nblocks, ws, sf, gtab, ptab, s);
    else launch_reduce_run<8, 4>(a, nblocks, ws, sf, gtab, ptab, s);
    return check_launch("preact_small_reduce_run (column kernels)");
}

bool col_supported(int batch, int C, int BR, int h, int w, int d) {
    const bool shape = (C == 2 && BR == 1) || (C == 4 && BR == 2) || (C == 8 && BR == 4);
    return shape && batch >= 1 && h >= BH && w >= BW && d >= BD && h % BH == 0 && w % BW == 0 && d % BD == 0 &&
           int64_t(batch) * h * w * d * C < (int64_t(1) << 31);
}

size_t col_workspace_bytes(int batch, int C, int BR, int h, int w, int d) {
    if (!col_supported(batch, C, BR, h, w, d)) return 0;
    const CArgs a = make_args(batch, h, w, d);
    const int ne = C == 2 ? n_entries<2, 1>() : C == 4 ? n_entries<4, 2>() : n_entries<8, 4>();
    return (size_t(a.nwg) + (a.nwg + RCH - 1) / RCH) * ne * 4;
}

int col_fwd(int xdt, int odt, int batch, int C, int BR, int h, int w, int d, const void *x, const float *w1,
            const float *w2, const float *w3, const vq3d_preact_params &p, void *out, void *t2, void *t3,
            hipStream_t s, int chain, const void *t2in, const float *w1n, const vq3d_preact_params *pn, void *t2n) {
    const CArgs a = make_args(batch, h, w, d);
    auto T2 = static_cast<h16_t *>(t2), T3 = static_cast<h16_t *>(t3);
    FwdChain c;
    c.ch = chain;
    c.t2in = static_cast<const h16_t *>(t2in);
    c.w1n = w1n;
    if (pn) c.pn = *pn;
    c.t2n = static_cast<h16_t *>(t2n);
    if (C == 2) fwd_io<2, 1>(xdt, odt, a, x, w1, w2, w3, p, out, T2, T3, c, s);
    else if (C == 4) fwd_io<4, 2>(xdt, odt, a, x, w1, w2, w3, p, out, T2, T3, c, s);
    else fwd_io<8, 4>(xdt, odt, a, x, w1, w2, w3, p, out, T2, T3, c, s);
    return check_launch("preact_small_fwd (column kernels)");
}

int col_bwd(int xdt, int odt, int batch, int C, int BR, int h, int w, int d, const void *g, const void *x,
            const void *t2, const void *t3, const float *w1, const float *w2, const float *w3,
            const vq3d_preact_params &p, const vq3d_preact_grads &gr, void *workspace, void *gx, int stages,
            hipStream_t s) {
    const CArgs a = make_args(batch, h, w, d);
    auto T2 = static_cast<const h16_t *>(t2), T3 = static_cast<const h16_t *>(t3);
    float *part = static_cast<float *>(workspace);
    if (C == 2) bwd_io<2, 1>(xdt, odt, a, g, x, T2, T3, w1, w2, w3, p, gr, part, gx, stages, s);
    else if (C == 4) bwd_io<4, 2>(xdt, odt, a, g, x, T2, T3, w1, w2, w3, p, gr, part, gx, stages, s);
    else bwd_io<8, 4>(xdt, odt, a, g, x, T2, T3, w1, w2, w3, p, gr, part, gx, stages, s);
    return check_launch("preact_small_bwd (column kernels)");
}

}  // namespace vq3d
