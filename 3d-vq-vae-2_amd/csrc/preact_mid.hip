// The 18-channel / branch-9 PreActFixupResBlock (vqvae/layers.py:176-195, mode 'same', no skip
// conv) of the published model's 128x128x32 level (50 decoder post-quantize blocks), forward in
// TWO launches and backward in THREE, all on resident bf16 channels-last tensors:
//
//   u1  = elu(x + b1a) + b1b      t2 = elu(W1 u1 + b2a) + b2b        (1x1, 18 -> 9)
//   t3  = elu(W2 (*) t2 + b3a) + b3b                                   (3x3x3 circular, 9 -> 9)
//   out = scale * (W3 t3) + b4 + x                                     (1x1, 9 -> 18)
//
// forward  k_pm_t2   : t2 from x, a streaming pointwise kernel (t2 is saved for the backward
//                      anyway, so computing it once beats recomputing it on every tile halo)
//          k_pm_fwd  : per tile, t2 on the tile's circular halo in LDS -> t3 on the matrix cores
//                      -> out = scale W3 t3 + b4 + x on the matrix cores; t3 / out leave in 16-B
//                      chunks.
// backward k_pm_bwd1 : gz3 = bf16(scale W3^T g * elu'(t3)) (pointwise) + the scale / b4 / b3
//                      partials
//          k_pm_bwd2 : per tile, gz3 and t2 on the halo in LDS -> gt2 = W2^T (*) gz3 (flipped
//                      taps, matrix cores) -> gz1 = bf16(gt2 * elu'(t2)) -> gx = g + (W1^T gz1)
//                      * elu'(x + b1a); gz1 to the workspace and the b2 / b1 partials
//          k_pm_w2grad, k_pm_w13grad: the W2 and the W1 / W3 gradient partials (matrix cores,
//                      voxels as the reduction axis, channel-major LDS copies); they only read,
//                      so the caller may run them on a second stream next to the next block's
//                      backward
//          k_pm_reduce: every gradient entry summed over the workgroups in a fixed order and
//                      added into the gradient buffers (deterministic, one adder per entry).
// Rounding points are the unfused per-conv path's (t2, t3, gz3, gz1, gx, out rounded to bf16,
// fp32 accumulation), except that the W1 gradient reads u1 rounded to bf16 and the backward's
// 1x1 data gradients (W1^T gz1, W3^T g) take W1 / W3 rounded to bf16 (the matrix-core operands).
//
// The k^3 convs use a "windowed" reduction order: for a voxel and a tap row (kh, kw) the three
// kd taps x 9 channels are 27 CONSECUTIVE elements of the halo D-line (channels-last, pitch 9),
// so one v_mfma_f32_16x16x32_bf16 k-step covers a whole tap row: 9 k-steps per 16 voxels
// instead of 14 with channel padding.  The five trailing elements of each window belong to the
// next position and meet zero weights.
#include "engines.h"

#include <cstdlib>

#include <algorithm>

// resident workgroups per CU of the forward / backward-data tile kernels: 0 = as many as fit
// (timing experiments set a cap: make exp EXP=N EXPDEF=PM_FWD_PER)
#ifndef PM_FWD_PER
#define PM_FWD_PER 0
#endif
#ifndef PM_BWD_PER
#define PM_BWD_PER 0
#endif
// 1: the D16 tile kernels keep one run's epilogue at a time (a scheduling barrier between runs)
#ifndef PM_DEPTH
#define PM_DEPTH 1  // tiles of operands in flight ahead of k_pm_bwd2's current tile (1 or 2)
#endif
#ifndef PM_SB
#define PM_SB 1
#endif
// minimum waves per SIMD the backward-data tile kernel is compiled for (2: at most 256 registers)
#ifndef PM_FREG
#define PM_FREG 1  // k_pm_bwd2: the 12 weight fragments in registers for the whole run (else one LDS read per use)
#endif
#ifndef PM_FREG_FWD
#define PM_FREG_FWD 0  // k_pm_fwd likewise (it runs 3 workgroups per CU on 64 VGPRs)
#endif
#ifndef PM_BWD_WPE
#define PM_BWD_WPE 2
#endif

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int C = 18, BR = 9, TD = 8;  // block channels, branch channels, tile depth (one D-run)
constexpr int NT = 256;                // threads per workgroup (every kernel)
constexpr int LSP = 104;               // halo line pitch (elements): [7 pad][pos -1][pos 0..7][pos 8][pad]
constexpr int LOFF = 7;                // element of halo position -1 (position p at LOFF + 9 (p + 1))
constexpr int LINT = 16;               // element of position 0: the interior run is 16-B aligned
constexpr int LEND = LINT + 9 * 9;     // first element after position 8 (97): zero padding
constexpr int SPAD = 40;               // zero tail of the pitch-9 / pitch-18 tile buffers

// scalar partials per workgroup: K1 b4, b3b, b3a, scale; K2 b2b, b2a, b1b, b1a
constexpr int NE1 = 4, NE2 = 4;
constexpr int NW2 = BR * BR * 27;  // W2 gradient [co][ci][tap]
// weight-gradient kernels: W2 over 512-voxel chunks (k_pm_w2grad), W1 / G3 over 128-voxel pieces
// (k_pm_w13grad)
constexpr int CHV = 512, ZP = CHV + 16;
constexpr int SUBV = 128, SP = SUBV + 8;
constexpr int NER = BR * 3 * BR;  // W2 entries of one tap row: co x (kd, ci)
constexpr int NEB = 2 * BR * C;   // W1 [o][c] then G3 [o][co]

struct PmArgs {
    int B, H, W, D;
    int nth, ntw, ntd, ntiles;
};

template <int TH, int TW>
struct Tile {
    static constexpr int LH = TH + 2, LW = TW + 2, NL = LH * LW;
    static constexpr int NRUN = TH * TW, TV = NRUN * TD, NMT = TV / 16;
    static constexpr int LINES = NL * LSP;                      // elements of one halo image
    static constexpr int S9 = (TV * BR + SPAD + 7) / 8 * 8;      // pitch-9 tile buffer
    static constexpr int S18 = (TV * C + SPAD + 7) / 8 * 8;      // pitch-18 tile buffer
    static_assert(TV % 64 == 0 && NRUN % 4 == 0, "tile");
};

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }
__device__ __forceinline__ float bf(uint32_t u16) { return h2f_lo(u16); }
// ELU on the hardware exp (v_exp_f32 of z log2 e: ~1e-7 relative, far inside the bf16 rounding that
// follows every use in the tile kernels; the libm expf is ~10 instructions)
__device__ __forceinline__ float elu_fast(float z) { return z > 0.f ? z : __expf(z) - 1.f; }
#ifndef PM_FAST_ELU
#define PM_FAST_ELU 1  // the first block's t2 stage and the W1-gradient staging's u1 on elu_fast too (as k_pm_fwd's u1)
#endif
#if PM_FAST_ELU
#define PM_ELU elu_fast
#else
#define PM_ELU elu
#endif
__device__ __forceinline__ float elu_d_act(float t, float b) {  // elu'(z) from t = elu(z) + b
    const float z1 = t - b;
    return z1 > 0.f ? 1.f : z1 + 1.f;
}

// 8 consecutive bf16 from LDS at element offset `off` (any parity; base 16-B aligned): five
// dwords + v_alignbyte when odd
__device__ __forceinline__ hx8 read8(const h16_t *base, int off) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(base + (off & ~1));
    const uint32_t sh = uint32_t(off & 1) * 2u;
    const uint32_t u0 = q[0], u1 = q[1], u2 = q[2], u3 = q[3], u4 = q[4];
    const uint4 r = {__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                     __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
    return __builtin_bit_cast(hx8, r);
}

// 8 bf16 at element offsets off + j * stride (j = 0..7) from LDS; zeros when !ok
__device__ __forceinline__ hx8 gather8(const h16_t *base, int off, int stride, bool ok) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (ok) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            w[j] = uint32_t(base[off + 2 * j * stride]) | (uint32_t(base[off + (2 * j + 1) * stride]) << 16);
    }
    return __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]});
}

__device__ __forceinline__ hx8 pack8(const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = uint32_t(f2h(v[2 * j])) | (uint32_t(f2h(v[2 * j + 1])) << 16);
    return __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]});
}

__device__ __forceinline__ f32x4 mfma(hx8 a, hx8 b, f32x4 c) {
    return VQ3D_MFMA_16X16X32(a, b, c, 0, 0, 0);
}

// copy n fp32 weights to LDS (coalesced; the fragments are then built from LDS instead of from
// scattered global loads)
__device__ __forceinline__ void stage_w(float *dst, const float *__restrict__ src, int n) {
    for (int i = threadIdx.x; i < n; i += NT) dst[i] = src[i];
}

// W2 B fragments (from the LDS copy), one per tap row kk = kh * 3 + kw: B[k = e][n] with
// e = kd * 9 + c (e < 27).
// Forward: n = co, c = ci, tap kk * 3 + kd.  Backward-data (transposed, flipped): n = ci,
// c = co, tap 26 - (kk * 3 + kd).
template <bool DGRAD>
__device__ __forceinline__ hx8 w2_frag(const float *w2, int kk, int lane) {
    const int n = lane & 15, kb = lane >> 4;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int e = 8 * kb + j, kd = e / 9, c = e - 9 * kd;
        float x = 0.f;
        if (n < BR && e < 27) {
            const int tap = kk * 3 + kd;
            x = DGRAD ? w2[(c * BR + n) * 27 + 26 - tap] : w2[(n * BR + c) * 27 + tap];
        }
        v[j] = x;
    }
    return pack8(v);
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
__device__ __forceinline__ Org tile_org(const PmArgs &a, int t, int TH, int TW) {
    Org o;
    o.d0 = (t % a.ntd) * TD;
    t /= a.ntd;
    o.w0 = (t % a.ntw) * TW;
    t /= a.ntw;
    o.h0 = (t % a.nth) * TH;
    o.b = t / a.nth;
    return o;
}
// global voxel index of D-run r (0 .. TH*TW-1) of the tile
template <int TW>
__device__ __forceinline__ int64_t run_vox(const PmArgs &a, const Org &o, int r) {
    return ((int64_t(o.b) * a.H + o.h0 + r / TW) * a.W + o.w0 + r % TW) * a.D + o.d0;
}

// Stage the (TH+2) x (TW+2) halo D-lines of a 9-channel tensor around the tile (circular wrap):
// per line the 8 interior positions (144 contiguous, 16-B aligned bytes) as 9 16-B chunks, and
// each edge position (position -1 / 8, 18 bytes, wrapped along D) inside two aligned 16-B chunks:
// the 32 bytes ending where position -1 ends land on line elements 0 .. 15 (position -1 at
// LOFF = 7 .. 15, the rest never read), the 32 bytes starting at position 8 on elements 88 .. 103
// (position 8 at LINT + 72 .. 96, the rest finite filler of the zero-weight window tails).  load()
// issues every global load into registers, store() writes them to LDS, so several tensors'
// loads are in flight together.
template <int TH, int TW>
struct LinesLd {
    using T = Tile<TH, TW>;
    static constexpr int NI = T::NL * 9, PI = (NI + NT - 1) / NT;
    static constexpr int NEG = T::NL * 4, PE = (NEG + NT - 1) / NT;  // (line, side, chunk)
    u32x4 vi[PI];
    u32x4 ve[PE];
    // every load is unconditional (indices past the end are clamped): a branch around a load
    // makes hipcc wait for it on the spot
    __device__ __forceinline__ void load(const PmArgs &a, const Org &o, const h16_t *__restrict__ src) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < PI; ++u) {
            const int i = min(tid + u * NT, NI - 1);
            const int line = i / 9, part = i - 9 * line, lh = line / T::LW, lw = line - lh * T::LW;
            const int gh = wrapm(o.h0 - 1 + lh, a.H), gw = wrapm(o.w0 - 1 + lw, a.W);
            const int64_t v0 = ((int64_t(o.b) * a.H + gh) * a.W + gw) * a.D + o.d0;
            vi[u] = reinterpret_cast<const u32x4 *>(src + v0 * BR)[part];
        }
#pragma unroll
        for (int u = 0; u < PE; ++u) {
            const int i = min(tid + u * NT, NEG - 1);
            const int line = i >> 2, side = (i >> 1) & 1, ch = i & 1;
            const int lh = line / T::LW, lw = line - lh * T::LW;
            const int gh = wrapm(o.h0 - 1 + lh, a.H), gw = wrapm(o.w0 - 1 + lw, a.W);
            const int64_t lb = ((int64_t(o.b) * a.H + gh) * a.W + gw) * a.D * BR;  // line start (elements)
            // left: the 32 bytes before position d0 (the line's end when d0 = 0); right: from
            // position d0 + 8 (the line's start when that wraps)
            const int e0 = side ? ((o.d0 + TD == a.D) ? 0 : (o.d0 + TD) * BR) : ((o.d0 == 0 ? a.D : o.d0) * BR - 16);
            ve[u] = *reinterpret_cast<const u32x4 *>(src + lb + e0 + 8 * ch);
        }
    }
    __device__ __forceinline__ void store(h16_t *lines) const {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < PI; ++u) {
            const int i = tid + u * NT;
            if (i < NI) {
                const int line = i / 9, part = i - 9 * line;
                reinterpret_cast<u32x4 *>(lines + line * LSP + LINT)[part] = vi[u];
            }
        }
#pragma unroll
        for (int u = 0; u < PE; ++u) {
            const int i = tid + u * NT;
            if (i < NEG) {
                const int line = i >> 2, side = (i >> 1) & 1, ch = i & 1;
                *reinterpret_cast<u32x4 *>(lines + line * LSP + (side ? LINT + 9 * TD : 0) + 8 * ch) = ve[u];
            }
        }
    }
};
static_assert(LOFF + 9 == LINT && LINT + 9 * TD + 16 == LSP - 0, "edge chunks fill elements 0..15 and 88..103");

// A tile of a channels-last tensor with CH channels (CH * 8 * 2 bytes per D-run, 16-B chunks)
// into LDS [voxel][CH]
template <int TH, int TW, int CH>
struct TileLd {
    using T = Tile<TH, TW>;
    static constexpr int PR = CH * TD / 8, N = T::NRUN * PR, P = (N + NT - 1) / NT;
    u32x4 v[P];
    __device__ __forceinline__ void load(const PmArgs &a, const Org &o, const h16_t *__restrict__ src) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int i = min(tid + u * NT, N - 1);
            const int r = i / PR, part = i - PR * r;
            v[u] = reinterpret_cast<const u32x4 *>(src + run_vox<TW>(a, o, r) * CH)[part];
        }
    }
    __device__ __forceinline__ void store(h16_t *dst) const {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int i = tid + u * NT;
            if (i < N) reinterpret_cast<u32x4 *>(dst)[i] = v[u];
        }
    }
};

template <int TH, int TW, int CH>
__device__ __forceinline__ void store_tile(const PmArgs &a, const Org &o, const h16_t *src, h16_t *__restrict__ dst) {
    using T = Tile<TH, TW>;
    constexpr int PR = CH * TD / 8, N = T::NRUN * PR;
    for (int i = threadIdx.x; i < N; i += NT) {
        const int r = i / PR, part = i - PR * r;
        reinterpret_cast<uint4 *>(dst + run_vox<TW>(a, o, r) * CH)[part] = reinterpret_cast<const uint4 *>(src)[i];
    }
}

// zero the never-staged tails of the halo lines and of the tile buffers (read by the windows /
// fragments that run past the valid data and meet zero weights: they must be finite)
template <int TH, int TW>
__device__ __forceinline__ void zero_pads(h16_t *lines, int nimg, h16_t *const *tails, const int *tail_at,
                                          int ntails) {
    using T = Tile<TH, TW>;
    for (int i = threadIdx.x; i < nimg * T::NL * (LSP - LEND); i += NT) {
        const int l = i / (LSP - LEND), e = i - l * (LSP - LEND);
        lines[l * LSP + LEND + e] = 0;
    }
    for (int t = 0; t < ntails; ++t)
        for (int i = threadIdx.x; i < SPAD; i += NT) tails[t][tail_at[t] + i] = 0;
}

// ============================================================================================ forward
// t2 = elu(W1 (elu(x + b1a) + b1b) + b2a) + b2b.  A thread owns a PAIR of voxels: 72 bytes of x
// (9 8-byte loads, all issued before any math) in, 36 bytes of t2 (9 dword stores) out; no LDS
// staging, no barriers.  W1 is broadcast from LDS.
__global__ __launch_bounds__(NT) void k_pm_t2(int64_t nvox, const h16_t *__restrict__ x,
                                              const float *__restrict__ w1, vq3d_preact_params p,
                                              h16_t *__restrict__ t2o) {
    __shared__ float w1s[BR * C];
    // W1 and u1 rounded to bf16: the operands of the chained forward's matrix-core t2 stage
    for (int i = threadIdx.x; i < BR * C; i += NT) w1s[i] = bf(f2h(w1[i]));
    __syncthreads();
    const Scal s = load_scal(p);
    const int64_t npair = nvox / 2;
    for (int64_t q = int64_t(blockIdx.x) * NT + threadIdx.x; q < npair; q += int64_t(gridDim.x) * NT) {
        uint2 v[C / 2];
        const uint2 *src = reinterpret_cast<const uint2 *>(x + q * 2 * C);
#pragma unroll
        for (int j = 0; j < C / 2; ++j) v[j] = src[j];
        uint32_t outw[BR];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            asm volatile("" ::: "memory");  // W1 re-read from LDS per voxel (not held in 162 registers)
            float uu[C];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int e = h * C + c;  // element of the 36 bf16 of the pair
                const uint2 w = v[e / 4];
                const uint32_t d = (e & 2) ? w.y : w.x;
                uu[c] = bf(f2h(PM_ELU(bf((e & 1) ? (d >> 16) : (d & 0xffffu)) + s.b1a) + s.b1b));
            }
            float t2v[BR];
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                asm volatile("" ::: "memory");  // one W1 row (18 floats) in registers at a time
                float acc = 0.f;
#pragma unroll
                for (int c = 0; c < C; ++c) acc = fmaf(w1s[o * C + c], uu[c], acc);
                t2v[o] = PM_ELU(acc + s.b2a) + s.b2b;
            }
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                const uint32_t hb = f2h(t2v[o]);
                const int e = h * BR + o;  // element of the 18 bf16 of the pair's t2
                if (e & 1) outw[e / 2] |= hb << 16;
                else outw[e / 2] = hb;
            }
        }
        uint32_t *dst = reinterpret_cast<uint32_t *>(t2o + q * 2 * BR);
#pragma unroll
        for (int j = 0; j < BR; ++j) dst[j] = outw[j];
    }
}

// ============================================================================================ backward
// K1: gz3 = bf16(scale * W3^T g * elu'(t3 - b3b)) and the sums of g (b4), of scale W3^T g (b3b),
// of gz3 (b3a) and of g . (W3 t3) (scale).  Blocks of 256 voxels; the next block's loads are in
// flight during the current one.  (The W3 gradient, sum t3 (x) g, is k_pm_w13grad's.)
__global__ __launch_bounds__(NT) void k_pm_bwd1(int64_t nvox, const h16_t *__restrict__ g,
                                                const h16_t *__restrict__ t3, const float *__restrict__ w3,
                                                vq3d_preact_params p, h16_t *__restrict__ gz3o,
                                                float *__restrict__ part) {
    __shared__ float w3s[C * BR];
    __shared__ __attribute__((aligned(16))) h16_t gs[NT * C];
    __shared__ __attribute__((aligned(16))) h16_t ts[NT * BR];
    __shared__ __attribute__((aligned(16))) h16_t zs[NT * BR];
    __shared__ float red[32];
    constexpr int NG = NT * C / 8, NTT = NT * BR / 8, PG = (NG + NT - 1) / NT, PT = (NTT + NT - 1) / NT;
    const int tid = threadIdx.x;
    // W3 rounded to bf16: the operand the chained stage of k_pm_bwd2 feeds the matrix cores
    for (int i = tid; i < C * BR; i += NT) w3s[i] = bf(f2h(w3[i]));
    const Scal s = load_scal(p);
    float s4 = 0.f, s3b = 0.f, s3a = 0.f, ssc = 0.f;
    const int64_t nblk = nvox / NT;
    u32x4 vg[PG], vt[PT];
    auto load = [&](int64_t blk) {
        const int64_t v0 = blk * NT;
#pragma unroll
        for (int u = 0; u < PG; ++u) vg[u] = reinterpret_cast<const u32x4 *>(g + v0 * C)[min(tid + u * NT, NG - 1)];
#pragma unroll
        for (int u = 0; u < PT; ++u) vt[u] = reinterpret_cast<const u32x4 *>(t3 + v0 * BR)[min(tid + u * NT, NTT - 1)];
    };
    if (blockIdx.x < nblk) load(blockIdx.x);
    for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const int64_t v0 = blk * NT;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PG; ++u)
            if (tid + u * NT < NG) reinterpret_cast<u32x4 *>(gs)[tid + u * NT] = vg[u];
#pragma unroll
        for (int u = 0; u < PT; ++u)
            if (tid + u * NT < NTT) reinterpret_cast<u32x4 *>(ts)[tid + u * NT] = vt[u];
        if (blk + gridDim.x < nblk) load(blk + gridDim.x);
        __syncthreads();
        {
            float gv[C], tv[BR];
            const uint32_t *gr = reinterpret_cast<const uint32_t *>(gs + tid * C);
#pragma unroll
            for (int j = 0; j < C / 2; ++j) {
                const uint32_t q = gr[j];
                gv[2 * j] = bf(q & 0xffffu);
                gv[2 * j + 1] = bf(q >> 16);
                s4 += gv[2 * j] + gv[2 * j + 1];
            }
#pragma unroll
            for (int o = 0; o < BR; ++o) tv[o] = bf(ts[tid * BR + o]);
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                float a3 = 0.f;
#pragma unroll
                for (int co = 0; co < C; ++co) a3 = fmaf(w3s[co * BR + o], gv[co], a3);
                const float gt3 = a3 * s.sc;
                const float z = gt3 * elu_d_act(tv[o], s.b3b);
                s3b += gt3;
                s3a += z;
                ssc = fmaf(a3, tv[o], ssc);  // sum_co g[co] (W3 t3)[co] == sum_o t3[o] (W3^T g)[o]
                zs[tid * BR + o] = f2h(z);
            }
        }
        __syncthreads();
        constexpr int NO = NT * BR / 8;
        for (int i = tid; i < NO; i += NT)
            reinterpret_cast<uint4 *>(gz3o + v0 * BR)[i] = reinterpret_cast<const uint4 *>(zs)[i];
    }
    float *dst = part + int64_t(blockIdx.x) * NE1;
    float q[4] = {s4, s3b, s3a, ssc};  // one barrier pair for the four (bit-identical)
    block_sums<float, NT, 4, 8>(q, red);
    if (tid == 0) {
        dst[0] = q[0];
        dst[1] = q[1];
        dst[2] = q[2];
        dst[3] = q[3];
    }
}

// ============================================================================================ D16 tiles
// The backward data tile kernel (k_pm_bwd2) works on tiles of 4 x 4 D-runs of 16 voxels (256
// voxels): an MFMA column block is one whole D-run and each of the 8 waves owns 2 runs.
//  * k^3: the gz3 halo D-lines are staged in LDS with a 10-element position pitch (9 channels + a
//    zero), so the window of a tap row (3 kd taps x 10 elements) is 4 aligned dwords per lane; the
//    WEIGHTS are the A operand and the window the B operand, and each staged window feeds both of
//    the wave's runs where both use its line (12 window reads for 18 MFMAs).
//  * With the weights in the A slot the accumulator of lane (n, kb) holds channels 4kb .. 4kb + 3
//    of voxel n.  The 1x1 convs that follow take exactly those 4 values as their own B operand
//    (their K axis is ordered to match: k = 8kb + i <-> channel 4kb + i), so gz1 and gx never leave
//    the registers; the epilogue operands (x, g, t2, the previous block's t3) are loaded straight
//    from HBM into that layout one tile ahead (no LDS staging), gx leaves as 8-byte stores and the
//    9-channel outputs through a per-wave 288-byte LDS image as 16-byte stores.
//  * One barrier per tile: the halo image is double-buffered.
constexpr int QTH = 4, QTW = 4, QTD = 16;
constexpr int QLW = QTW + 2, QNL = (QTH + 2) * QLW;  // 36 halo lines
constexpr int QPP = 10;                               // LDS elements per halo position
constexpr int QLP = 184;                              // LDS elements per halo line: 18 positions + zero tail (>= 182)
constexpr int QIMG = QNL * QLP;                       // one halo image (elements)
constexpr int QSTG = 576;                             // per-wave output image of a run: [16][18] + 2 x [16][9]
constexpr int QNT = 512, QNW = QNT / 64;              // threads / waves per workgroup: a wave owns 2 D-runs

PmArgs make_args_q(int B, int H, int W, int D) {
    PmArgs a;
    a.B = B;
    a.H = H;
    a.W = W;
    a.D = D;
    a.nth = H / QTH;
    a.ntw = W / QTW;
    a.ntd = D / QTD;
    a.ntiles = B * a.nth * a.ntw * a.ntd;
    return a;
}
__device__ __forceinline__ Org tile_org_q(const PmArgs &a, int t) {
    Org o;
    o.d0 = (t % a.ntd) * QTD;
    t /= a.ntd;
    o.w0 = (t % a.ntw) * QTW;
    t /= a.ntw;
    o.h0 = (t % a.nth) * QTH;
    o.b = t / a.nth;
    return o;
}

// The (QTH+2) x (QTW+2) halo D-lines of a 9-channel tensor around a tile (circular wrap), one work
// item per thread: the 8 interior position PAIRS of a line (positions d, d + 1 with d even: 36
// contiguous dword-aligned bytes, 9 dwords) or one of its 2 edge positions (d0 - 1 / d0 + 16,
// wrapped: the 20 bytes from the dword at or below the row).  load() issues the global loads
// into registers, store() writes each position as 5 dwords (9 channels + the zero pad) into the
// pitch-10 image with naturally aligned b32 / b64 stores (a position starts 4 or 0 mod 8).
constexpr int QPAIRS = QNL * 8, QITEMS = QPAIRS + QNL * 2;
static_assert(QITEMS <= QNT, "one halo item per thread");
struct HaloQ {
    uint32_t w[9];
    // element offsets fit 32 bits (vq3d_preact_mid_supported bounds the tensor)
    __device__ __forceinline__ void load(int tid, const PmArgs &a, const Org &o, const h16_t *__restrict__ src) {
        const int i = min(tid, QITEMS - 1);
        const bool pair = i < QPAIRS;
        const int line = pair ? i >> 3 : (i - QPAIRS) >> 1;
        const int lh = line / QLW, lw = line - lh * QLW;
        const uint32_t gh = wrapm(o.h0 - 1 + lh, a.H), gw = wrapm(o.w0 - 1 + lw, a.W);
        const uint32_t lb = ((uint32_t(o.b) * a.H + gh) * a.W + gw) * a.D;  // first voxel of the line
        const char *base = reinterpret_cast<const char *>(src);
        const int side = (i - QPAIRS) & 1;
        const int d = pair ? o.d0 + 2 * (i & 7)  // a 36-byte pair: dword aligned
                           : side ? (o.d0 + QTD == a.D ? 0 : o.d0 + QTD) : (o.d0 == 0 ? a.D - 1 : o.d0 - 1);
        const uint32_t off = ((lb + d) * (2 * BR)) & ~3u;  // an odd voxel's row starts at 2 mod 4
        // unconditional loads (a branch around a load makes hipcc wait for it on the spot)
        __builtin_memcpy(w, base + off, 20);
        __builtin_memcpy(w + 5, base + (pair ? off + 20 : off), 16);
    }
    __device__ __forceinline__ void store(int tid, h16_t *img) const {
        if (tid >= QITEMS) return;
        const bool pair = tid < QPAIRS;
        const int line = pair ? tid >> 3 : (tid - QPAIRS) >> 1;
        uint32_t *ln = reinterpret_cast<uint32_t *>(img + line * QLP);  // 16-B aligned (QLP * 2 = 368)
        if (pair) {
            // positions p = 2k + 1, 2k + 2 (d = 2k, 2k + 1) at dwords 5p .. 5p + 9: 5p = 4 mod 8 bytes
            const int q = 5 * (2 * (tid & 7) + 1);
            const uint32_t c[10] = {w[0], w[1], w[2], w[3], w[4] & 0xffffu, __builtin_amdgcn_alignbyte(w[5], w[4], 2),
                                    __builtin_amdgcn_alignbyte(w[6], w[5], 2), __builtin_amdgcn_alignbyte(w[7], w[6], 2),
                                    __builtin_amdgcn_alignbyte(w[8], w[7], 2), w[8] >> 16};
            ln[q] = c[0];
            *reinterpret_cast<u32x2 *>(ln + q + 1) = u32x2{c[1], c[2]};
            *reinterpret_cast<u32x2 *>(ln + q + 3) = u32x2{c[3], c[4]};
            *reinterpret_cast<u32x2 *>(ln + q + 5) = u32x2{c[5], c[6]};
            *reinterpret_cast<u32x2 *>(ln + q + 7) = u32x2{c[7], c[8]};
            ln[q + 9] = c[9];
        } else {
            // position 0 (dwords 0 .. 4): voxel d0 - 1 (or D - 1), odd, its row 2 bytes into w; position
            // 17 (dwords 85 .. 89): voxel d0 + 16 (or 0), even, its row at w
            const int side = (tid - QPAIRS) & 1;
            if (side) {  // dword 85: 4 mod 8 bytes
                ln[85] = w[0];
                *reinterpret_cast<u32x2 *>(ln + 86) = u32x2{w[1], w[2]};
                *reinterpret_cast<u32x2 *>(ln + 88) = u32x2{w[3], w[4] & 0xffffu};
            } else {
                *reinterpret_cast<u32x2 *>(ln) =
                    u32x2{__builtin_amdgcn_alignbyte(w[1], w[0], 2), __builtin_amdgcn_alignbyte(w[2], w[1], 2)};
                *reinterpret_cast<u32x2 *>(ln + 2) =
                    u32x2{__builtin_amdgcn_alignbyte(w[3], w[2], 2), __builtin_amdgcn_alignbyte(w[4], w[3], 2)};
                ln[4] = w[4] >> 16;
            }
        }
    }
};

// zero the line tails of n halo images (never staged; the last windows read them against zero
// weights); the channel pads are written with every position
__device__ __forceinline__ void zero_pads_q(h16_t *img, int n) {
    constexpr int PER = QLP - 18 * QPP;
    for (int i = threadIdx.x; i < n * QNL * PER; i += QNT) {
        const int l = i / PER, k = i - l * PER;
        img[l * QLP + 18 * QPP + k] = 0;
    }
}

// The window of one tap row for lane (n, kb): 8 elements at an even element offset (4 dwords)
__device__ __forceinline__ hx8 win8(const h16_t *p) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
    return __builtin_bit_cast(hx8, uint4{q[0], q[1], q[2], q[3]});
}

// k^3 weights as the A operand, one fragment per tap row kk = kh * 3 + kw: A[m][k] with
// k = kd * 10 + c (c < 9, kd < 3; the pad channel and k = 30, 31 zero).  Forward: m = co, c = ci,
// tap kk * 3 + kd.  Backward-data (transposed, flipped): m = ci, c = co, tap 26 - (kk * 3 + kd).
template <bool DGRAD>
__device__ __forceinline__ hx8 w2_afrag(const float *w2, int kk, int lane) {
    const int m = lane & 15, kb = lane >> 4;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * kb + j, kd = k / QPP, c = k - QPP * kd;
        float x = 0.f;
        if (m < BR && c < BR && kd < 3) {
            const int tap = kk * 3 + kd;
            x = DGRAD ? w2[(c * BR + m) * 27 + 26 - tap] : w2[(m * BR + c) * 27 + tap];
        }
        v[j] = x;
    }
    return pack8(v);
}

// The K order of the 1x1 convs fed from a k^3 / 1x1 accumulator: lane-group kb supplies channels
// 4kb .. 4kb + 3 as k = 8kb .. 8kb + 3 (9-channel inputs), and for 18-channel inputs (two
// accumulator tiles; the second tile's rows 12, 13 are channels 16, 17, so lane-group 3 holds
// channels 12 .. 17) kb = 3 also channels 16, 17 as k = 28, 29.  Channel of K entry k (-1: zero).
__device__ __forceinline__ int k_chan9(int k) {
    const int kb = k >> 3, i = k & 7;
    return (i < 4 && 4 * kb + i < BR) ? 4 * kb + i : -1;
}
__device__ __forceinline__ int k_chan18(int k) {
    const int kb = k >> 3, i = k & 7;
    return i < 4 ? 4 * kb + i : (kb == 3 && i < 6) ? 16 + i - 4 : -1;
}

// 9-channel voxel rows (18 bytes, only 2-byte aligned) in the accumulator layout: lane-group kb
// (< 2) needs channels 4kb .. 4kb + 3 of voxel v, kb = 2 channel 8.  Every lane loads the 3
// dwords around its values with one dword-aligned load that stays inside the tensor (the only
// voxel whose row ends the tensor is odd, and odd rows never read past their own end).
// (one native 3-dword vector: the register tuple a dwordx3 load writes is then the loop-carried
// value itself -- a struct of three scalars made the tile loop copy every prefetched operand at its
// back edge, which waits for the loads to land)
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
using Raw9 = u32x3;
__device__ __forceinline__ int q9_kb(int kb) { return kb == 3 ? 0 : kb; }
__device__ __forceinline__ Raw9 ld9(const h16_t *__restrict__ base, uint32_t v, int kb) {
    const int k = q9_kb(kb);
    const uint32_t s = v * (2 * BR) + 8 * k;
    const uint32_t a = (s & ~3u) - (k == 2 ? 8 : 0);
    u32x3 r;
    __builtin_memcpy(&r, reinterpret_cast<const char *>(base) + a, 12);
    return r;
}
// the 4 values of lane-group kb (kb 2: one value; kb 3: none) as floats.  The entries past channel 8
// are other finite elements of the tensor, not zeros: every use multiplies them by an accumulator
// row whose weights are zero (k_pm_bwd2), so they need no masks
__device__ __forceinline__ void ex9(const Raw9 &r, uint32_t v, int kb, float (&o)[4]) {
    const int k = q9_kb(kb);
    const uint32_t sub = uint32_t(v & 1) * 2u;  // 18 v mod 4
    const bool hi = k == 2;
    const uint32_t lo = hi ? r.z : r.x, mid = hi ? 0u : r.y, top = hi ? 0u : r.z;
    const uint32_t p0 = __builtin_amdgcn_alignbyte(mid, lo, sub), p1 = __builtin_amdgcn_alignbyte(top, mid, sub);
    o[0] = bf(p0 & 0xffffu);
    o[1] = bf(p0 >> 16);
    o[2] = bf(p1 & 0xffffu);
    o[3] = bf(p1 >> 16);
}
// 18-channel rows (36 bytes, dword aligned): channels 4kb .. 4kb + 5 (one dwordx3; lane-group 3
// uses all six: 12 .. 15 and 16, 17)
using Raw18 = u32x3;
__device__ __forceinline__ Raw18 ld18(const h16_t *__restrict__ base, uint32_t v, int kb) {
    u32x3 r;
    __builtin_memcpy(&r, reinterpret_cast<const char *>(base) + size_t(v * (2 * C) + 8 * kb), 12);
    return r;
}

// Outputs leave through a per-wave LDS image of the run (16 voxels: an 18-channel tensor's 576
// contiguous bytes, then two 9-channel tensors' 288 each = 72 16-byte chunks) and one pass of
// contiguous 16-byte stores: stored straight from the accumulator layout they would be 8-byte
// pieces at a 36-byte stride, which the store path moves several times slower.  The image is
// written and read by the same wave (LDS keeps a wave's accesses in order: no barrier).
constexpr int QO9A = 16 * C, QO9B = QO9A + 16 * BR;  // element offsets of the 9-channel images
__device__ __forceinline__ uint32_t pk2(float a, float b) { return uint32_t(f2h(a)) | (uint32_t(f2h(b)) << 16); }
// channels 4kb .. 4kb + 3 of voxel n (lane-group 3 also 16, 17) of the 18-channel image
__device__ __forceinline__ void put18(h16_t *st, int n, int kb, const float (&v)[6]) {
    uint32_t *p = reinterpret_cast<uint32_t *>(st + n * C + 4 * kb);  // 36 n + 8 kb bytes: dword aligned
    // separate b32 stores: merged into a b64 they would be misaligned for odd n (64-cycle replays)
    p[0] = pk2(v[0], v[1]);
    asm volatile("" ::: "memory");
    p[1] = pk2(v[2], v[3]);
    asm volatile("" ::: "memory");
    if (kb == 3) p[2] = pk2(v[4], v[5]);
}
// channels 4kb .. 4kb + 3 (kb 2: channel 8) of voxel n of a 9-channel image
__device__ __forceinline__ void put9(h16_t *st, int n, int kb, const float (&v)[4]) {
    h16_t *p = st + n * BR + 4 * kb;
    if (kb < 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j] = f2h(v[j]);
    } else if (kb == 2) {
        p[0] = f2h(v[0]);
    }
}
// the image to the run's rows (d18: 18-channel rows, d9a / d9b: 9-channel rows; null = absent)
__device__ __forceinline__ void flush_run(const h16_t *st, int lane, h16_t *__restrict__ d18,
                                          h16_t *__restrict__ d9a, h16_t *__restrict__ d9b) {
    const uint4 *src = reinterpret_cast<const uint4 *>(st);
    const uint4 q0 = src[lane];
    if (lane < 36) {
        reinterpret_cast<uint4 *>(d18)[lane] = q0;
    } else if (lane < 54) {
        if (d9a) reinterpret_cast<uint4 *>(d9a)[lane - 36] = q0;
    } else if (d9b) {
        reinterpret_cast<uint4 *>(d9b)[lane - 54] = q0;
    }
    if (lane < 8 && d9b) reinterpret_cast<uint4 *>(d9b)[10 + lane] = src[64 + lane];
}

// K2: per 4 x 4 x 16 tile: gt2 = W2^T (*) gz3 (flipped taps) -> gz1 = bf16(gt2 * elu'(t2)) ->
// gx = g + (W1^T gz1) * elu'(x + b1a); gz1 to the workspace (k_pm_w13grad) and the b2 / b1 sums.
// CHAIN (the chained backward of a run of blocks): the PREVIOUS block's K1 -- its gz3 and its four
// scalar partials, k_pm_bwd1's arithmetic -- from this tile's gx still in registers (gx is that
// block's g) and the previous block's t3, instead of a k_pm_bwd1 launch re-reading gx.
template <bool CHAIN>
__global__ __launch_bounds__(QNT) __attribute__((amdgpu_waves_per_eu(PM_BWD_WPE))) void k_pm_bwd2(
    PmArgs a, const h16_t *__restrict__ gz3, const h16_t *__restrict__ t2, const h16_t *__restrict__ x,
    const h16_t *__restrict__ g, const float *__restrict__ w1, const float *__restrict__ w2, vq3d_preact_params p,
    h16_t *__restrict__ gx, h16_t *__restrict__ gz1o, float *__restrict__ part, const h16_t *__restrict__ t3p,
    const float *__restrict__ w3p, vq3d_preact_params pp, h16_t *__restrict__ gz3p, float *__restrict__ part1p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *img = reinterpret_cast<h16_t *>(smem);              // 2 halo images [QNL][QLP]
    hx8 *frag = reinterpret_cast<hx8 *>(img + 2 * QIMG);  // A fragments [12][64]: W2 tap rows, W1^T x 2, W3^T
    h16_t *stg = reinterpret_cast<h16_t *>(frag + 12 * 64);    // [QNW waves][QSTG] output images
    float *red = reinterpret_cast<float *>(stg + QNW * QSTG);  // [32] block sums
    // prologue only: the fp32 weights W2 [NW2], W1 [o][c], previous W3 [co][o] over the halo images
    float *ws2 = reinterpret_cast<float *>(smem), *ws1 = ws2 + NW2, *ws3 = ws1 + BR * C;
    static_assert((2 * QIMG * 2) % 16 == 0 && (QNW * QSTG * 2) % 16 == 0, "carve alignment");
    static_assert(size_t(NW2 + 2 * BR * C) * 4 <= size_t(2 * QIMG) * 2, "weights fit the halo images");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = lane & 15, kb = lane >> 4;
    for (int i = tid; i < NW2; i += QNT) ws2[i] = w2[i];
    for (int i = tid; i < BR * C; i += QNT) ws1[i] = w1[i];
    if constexpr (CHAIN)
        for (int i = tid; i < C * BR; i += QNT) ws3[i] = w3p[i];
    __syncthreads();
    // the MFMA A fragments (lane-linear images, one ds_read_b128 per use: weights in VGPRs would
    // leave no room for the tile-ahead prefetch), fragment f built by wave f % 8
    for (int f = wave; f < 12; f += QNW) {
        hx8 fr = {};
        if (f < 9) {
            fr = w2_afrag<true>(ws2, f, lane);
        } else if (f < 11) {  // W1^T: A[m -> c][k -> o]; tile 1: rows 12, 13 = channels 16, 17
            float v[8];
            const int c = f == 10 ? (n >= 12 ? 16 + n - 12 : C) : n;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int o = k_chan9(8 * kb + j);
                v[j] = (o >= 0 && c < C) ? ws1[o * C + c] : 0.f;
            }
            fr = pack8(v);
        } else if (CHAIN) {  // previous W3^T: A[m = o][k -> co]
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int co = k_chan18(8 * kb + j);
                v[j] = (co >= 0 && n < BR) ? ws3[co * BR + n] : 0.f;
            }
            fr = pack8(v);
        }
        frag[f * 64 + lane] = fr;
    }
    __syncthreads();  // the weights are read: the halo images' pads can be zeroed
    // the A fragments in registers for the whole run (PM_FREG: 48 VGPRs; two waves per SIMD leave
    // room) -- an LDS read per use put a ~100-cycle wait in front of every 1x1 stage's MFMA
    hx8 fr[PM_FREG ? 12 : 1];
    if constexpr (PM_FREG) {
#pragma unroll
        for (int f = 0; f < 12; ++f) fr[f] = frag[f * 64 + lane];
    }
    auto wf = [&](int f, int l) -> hx8 {
        if constexpr (PM_FREG) return fr[f];
        else return frag[f * 64 + l];
    };
    zero_pads_q(img, 2);
    const Scal s = load_scal(p);
    Scal sp{};
    if constexpr (CHAIN) sp = load_scal(pp);
    float s2b = 0.f, s2a = 0.f, s1b = 0.f, s1a = 0.f;
    float q4 = 0.f, q3b = 0.f, q3a = 0.f, qsc = 0.f;  // CHAIN: the previous block's K1 sums
    // the wave's two D-runs: rows ph, ph + 1 of tile column pw (run coordinates inside the tile)
    const int ph = (wave >> 2) * 2, pw = wave & 3;
    // the operands of the tiles ahead of the current one, PM_DEPTH deep: with depth 2 the tile loop
    // is unrolled by two over two register sets (no loop-carried copies, which would wait for the
    // loads at the back edge), and each tile refills its set with the tile two steps ahead
    HaloQ hzA, hzB;
    Raw9 et2A[2], et3A[2], et2B[2], et3B[2];
    Raw18 exA[2], egA[2], exB[2], egB[2];
    // every per-thread index below derives from a copy of the thread index laundered once per tile:
    // the address arithmetic is then recomputed per tile (a few VALU ops) instead of being hoisted
    // out of the tile loop as dozens of live loop invariants
    auto launder = [](int v) {
        asm volatile("" : "+v"(v));
        return v;
    };
    auto run_vox0 = [&](const Org &o, int r) {  // first voxel of the wave's run r (0, 1)
        return ((uint32_t(o.b) * a.H + o.h0 + ph + r) * a.W + o.w0 + pw) * a.D + o.d0;
    };
    auto load_ep = [&](Raw9 (&et2)[2], Raw9 (&et3)[2], Raw18 (&ex)[2], Raw18 (&eg)[2], int ln, const Org &o, int r) {
        const int nn = ln & 15, kq = ln >> 4;
        const uint32_t v = run_vox0(o, r) + nn;
        et2[r] = ld9(t2, v, kq);
        ex[r] = ld18(x, v, kq);
        eg[r] = ld18(g, v, kq);
        if constexpr (CHAIN) et3[r] = ld9(t3p, v, kq);
    };
    const TileSched sc = xcd_sched(a.ntiles);
    constexpr int DEPTH = PM_DEPTH;
    static_assert(DEPTH == 1 || DEPTH == 2, "prefetch depth");
    if (sc.t < sc.end) {
        const Org o0 = tile_org_q(a, sc.t);
        hzA.load(tid, a, o0, gz3);
#pragma unroll
        for (int r = 0; r < 2; ++r) load_ep(et2A, et3A, exA, egA, lane, o0, r);
        if constexpr (DEPTH == 2) {
            const Org o1 = tile_org_q(a, sc.t + sc.step < sc.end ? sc.t + sc.step : sc.t);
            hzB.load(tid, a, o1, gz3);
#pragma unroll
            for (int r = 0; r < 2; ++r) load_ep(et2B, et3B, exB, egB, lane, o1, r);
        }
    }
    // o: the tile's origin (carried from the previous tile's `on` at depth 1: one set of runtime
    // divisions per tile); returns the origin of the tile DEPTH steps ahead
    auto body = [&](HaloQ &hz, Raw9 (&et2)[2], Raw9 (&et3)[2], Raw18 (&ex)[2], Raw18 (&eg)[2], int tile, int it,
                    const Org o) -> Org {
        const int tn = tile + DEPTH * sc.step;
        const Org on = tile_org_q(a, tn < sc.end ? tn : tile);
        const int tl = launder(tid), ln = tl & 63, nl = ln & 15, kl = ln >> 4;
        h16_t *hl = img + (it & 1) * QIMG;
        hz.store(tl, hl);
        hz.load(tl, a, on, gz3);
        __syncthreads();
        // gt2 of the wave's 2 runs: input line (i, j) of the 4 x 3 they need feeds run r through tap
        // row (i - r, j)
        f32x4 acc[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const hx8 bw = win8(hl + ((ph + i) * QLW + pw + j) * QLP + nl * QPP + 8 * kl);
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const int kh = i - r;
                        if (kh >= 0 && kh < 3) acc[r] = mfma(wf(kh * 3 + j, ln), bw, acc[r]);
                    }
                }
                asm volatile("" ::: "memory");  // one row of windows in registers at a time
            }
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t v0 = run_vox0(o, r), v = v0 + nl;
            h16_t *st = stg + wave * QSTG;
            // gz1 = bf16(gt2 * elu'(t2)) for channels 4kb + j
            float t2v[4], z1[4];
            ex9(et2[r], v, kl, t2v);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // channels past 8 (4 kb + j >= BR) need no masks here or below: their A rows are
                // zero, so acc, z, gt1 and the previous block's a3 are exactly 0 there (operands
                // finite), adding nothing to the sums and meeting zero weights as K entries
                const float z = acc[r][j] * elu_d_act(t2v[j], s.b2b);
                z1[j] = bf(f2h(z));
                s2b += acc[r][j];
                s2a += z;
            }
            // gt1 = W1^T gz1 (two channel tiles), gx = g + gt1 * elu'(x + b1a)
            float gxv[6];
            {
                const hx8 bz = pack8({z1[0], z1[1], z1[2], z1[3], 0.f, 0.f, 0.f, 0.f});
                const f32x4 a0 = mfma(wf(9, ln), bz, f32x4{0.f, 0.f, 0.f, 0.f});
                const f32x4 a1 = mfma(wf(10, ln), bz, f32x4{0.f, 0.f, 0.f, 0.f});
                const Raw18 &xr = ex[r], &gr = eg[r];
                const float xv[6] = {bf(xr.x & 0xffffu), bf(xr.x >> 16), bf(xr.y & 0xffffu), bf(xr.y >> 16),
                                     bf(xr.z & 0xffffu), bf(xr.z >> 16)};
                const float gv[6] = {bf(gr.x & 0xffffu), bf(gr.x >> 16), bf(gr.y & 0xffffu), bf(gr.y >> 16),
                                     bf(gr.z & 0xffffu), bf(gr.z >> 16)};
                const float gt1[6] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1]};
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const bool ok = j < 4 || kl == 3;  // channels 4kb + j, then (kb 3) 16 / 17
                    const float zx = xv[j] + s.b1a;
                    const float ez = zx > 0.f ? 1.f : __expf(zx);
                    s1b += gt1[j];
                    s1a += gt1[j] * ez;
                    gxv[j] = ok ? bf(f2h(gv[j] + gt1[j] * ez)) : 0.f;
                    if constexpr (CHAIN) q4 += gxv[j];  // the previous block's g = this gx
                }
            }
            {
                put18(st, nl, kl, gxv);
                put9(st + QO9A, nl, kl, z1);
            }
            if constexpr (CHAIN) {
                // previous block: gz3 = bf16(scale W3^T gx * elu'(t3)) (one MFMA, K = the 18 channels
                // of gx in the k_chan18 order)
                {
                    const hx8 bg = pack8({gxv[0], gxv[1], gxv[2], gxv[3], gxv[4], gxv[5], 0.f, 0.f});
                    const f32x4 a3 = mfma(wf(11, ln), bg, f32x4{0.f, 0.f, 0.f, 0.f});
                    float t3v[4], zq[4];
                    ex9(et3[r], v, kl, t3v);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float gt3 = a3[j] * sp.sc;
                        const float z = gt3 * elu_d_act(t3v[j], sp.b3b);
                        q3b += gt3;
                        q3a += z;
                        qsc += a3[j] * t3v[j];
                        zq[j] = z;
                    }
                    put9(st + QO9B, nl, kl, zq);
                }
            }
            flush_run(st, ln, gx + size_t(v0) * C, gz1o + size_t(v0) * BR, CHAIN ? gz3p + size_t(v0) * BR : nullptr);
            // the operands of the tile DEPTH steps ahead for this run (unconditional: on = this tile
            // at the end; a branch would keep the old values live)
            load_ep(et2, et3, ex, eg, ln, on, r);
            if constexpr (PM_SB) __builtin_amdgcn_sched_barrier(0);  // one run's epilogue at a time (no interleaving)
        }
        return on;
    };
    if constexpr (DEPTH == 1) {
        int it = 0;
        Org o = tile_org_q(a, sc.t < sc.end ? sc.t : 0);
        for (int tile = sc.t; tile < sc.end; tile += sc.step, ++it) o = body(hzA, et2A, et3A, exA, egA, tile, it, o);
    } else {
        int it = 0;
        for (int tile = sc.t; tile < sc.end; tile += 2 * sc.step, it += 2) {
            body(hzA, et2A, et3A, exA, egA, tile, it, tile_org_q(a, tile));
            if (tile + sc.step < sc.end)
                body(hzB, et2B, et3B, exB, egB, tile + sc.step, it + 1, tile_org_q(a, tile + sc.step));
        }
    }
    if constexpr (CHAIN) {
        float *dp = part1p + int64_t(blockIdx.x) * NE1;
        float q[4] = {q4, q3b, q3a, qsc};  // one barrier pair for the four (bit-identical)
        block_sums<float, QNT, 4, 8>(q, red);
        if (tid == 0) {
            dp[0] = q[0];
            dp[1] = q[1];
            dp[2] = q[2];
            dp[3] = q[3];
        }
    }
    float *dst = part + int64_t(blockIdx.x) * NE2;
    float q2[4] = {s2b, s2a, s1b, s1a};
    block_sums<float, QNT, 4, 8>(q2, red);
    if (tid == 0) {
        dst[0] = q2[0];
        dst[1] = q2[1];
        dst[2] = q2[2];
        dst[3] = q2[3];
    }
}

// The forward tile kernel on the same 4 x 4 x 16 tiles: t3 = elu(W2 (*) t2 + b3a) + b3b from t2 on
// the tile's halo, out = scale W3 t3 + b4 + x, and CHAIN: the next block's t2 = elu(W1' u1 + b2a')
// + b2b' with u1 = elu(out + b1a') + b1b' -- each stage's accumulator the next stage's B operand
// (the k_chan9 / k_chan18 K orders), x loaded straight into the accumulator layout a tile ahead.
// Rounding points: t3, out, u1 and the next t2 to bf16 (the per-conv path's; W2 / W3 / W1' as bf16
// matrix-core operands).
template <bool CHAIN>
__global__ __launch_bounds__(QNT) __attribute__((amdgpu_waves_per_eu(PM_BWD_WPE))) void k_pm_fwd(
    PmArgs a, const h16_t *__restrict__ t2, const h16_t *__restrict__ x, const float *__restrict__ w2,
    const float *__restrict__ w3, vq3d_preact_params p, h16_t *__restrict__ t3o, h16_t *__restrict__ out,
    const float *__restrict__ w1n, vq3d_preact_params pn, h16_t *__restrict__ t2n) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *img = reinterpret_cast<h16_t *>(smem);              // 2 halo images [QNL][QLP]
    hx8 *frag = reinterpret_cast<hx8 *>(img + 2 * QIMG);  // A fragments [12][64]: W2 tap rows, W3 x 2, W1'
    h16_t *stg = reinterpret_cast<h16_t *>(frag + 12 * 64);    // [QNW waves][QSTG] output images
    float *ws2 = reinterpret_cast<float *>(smem), *ws3 = ws2 + NW2, *ws1 = ws3 + C * BR;  // prologue only
    static_assert(size_t(NW2 + 2 * BR * C) * 4 <= size_t(2 * QIMG) * 2, "weights fit the halo images");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = lane & 15, kb = lane >> 4;
    for (int i = tid; i < NW2; i += QNT) ws2[i] = w2[i];
    for (int i = tid; i < C * BR; i += QNT) ws3[i] = w3[i];
    if constexpr (CHAIN)
        for (int i = tid; i < BR * C; i += QNT) ws1[i] = w1n[i];
    __syncthreads();
    for (int f = wave; f < 12; f += QNW) {
        hx8 fr = {};
        if (f < 9) {
            fr = w2_afrag<false>(ws2, f, lane);
        } else if (f < 11) {  // W3: A[m -> co][k -> o]; tile 1: rows 12, 13 = channels 16, 17
            float v[8];
            const int co = f == 10 ? (n >= 12 ? 16 + n - 12 : C) : n;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int o = k_chan9(8 * kb + j);
                v[j] = (o >= 0 && co < C) ? ws3[co * BR + o] : 0.f;
            }
            fr = pack8(v);
        } else if (CHAIN) {  // the next block's W1: A[m = o][k -> c]
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = k_chan18(8 * kb + j);
                v[j] = (c >= 0 && n < BR) ? ws1[n * C + c] : 0.f;
            }
            fr = pack8(v);
        }
        frag[f * 64 + lane] = fr;
    }
    __syncthreads();
    hx8 fr[PM_FREG_FWD ? 12 : 1];  // as k_pm_bwd2 (PM_FREG_FWD)
    if constexpr (PM_FREG_FWD) {
#pragma unroll
        for (int f = 0; f < 12; ++f) fr[f] = frag[f * 64 + lane];
    }
    auto wf = [&](int f, int l) -> hx8 {
        if constexpr (PM_FREG_FWD) return fr[f];
        else return frag[f * 64 + l];
    };
    zero_pads_q(img, 2);
    const Scal s = load_scal(p);
    Scal sn{};
    if constexpr (CHAIN) sn = load_scal(pn);
    const int ph = (wave >> 2) * 2, pw = wave & 3;
    HaloQ ht;
    Raw18 ex[2];
    auto launder = [](int v) {
        asm volatile("" : "+v"(v));
        return v;
    };
    auto run_vox0 = [&](const Org &o, int r) {
        return ((uint32_t(o.b) * a.H + o.h0 + ph + r) * a.W + o.w0 + pw) * a.D + o.d0;
    };
    const TileSched sc = xcd_sched(a.ntiles);
    if (sc.t < sc.end) {
        const Org o0 = tile_org_q(a, sc.t);
        ht.load(tid, a, o0, t2);
#pragma unroll
        for (int r = 0; r < 2; ++r) ex[r] = ld18(x, run_vox0(o0, r) + n, kb);
    }
    int it = 0;
    Org o = tile_org_q(a, sc.t < sc.end ? sc.t : 0);  // carried: one set of runtime divisions per tile
    for (int tile = sc.t; tile < sc.end; tile += sc.step, ++it) {
        const bool more = tile + sc.step < sc.end;
        const Org on = tile_org_q(a, more ? tile + sc.step : tile);
        const int tl = launder(tid), ln = tl & 63, nl = ln & 15, kl = ln >> 4;
        h16_t *hl = img + (it & 1) * QIMG;
        ht.store(tl, hl);
        ht.load(tl, a, on, t2);
        __syncthreads();
        f32x4 acc[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const hx8 bw = win8(hl + ((ph + i) * QLW + pw + j) * QLP + nl * QPP + 8 * kl);
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const int kh = i - r;
                        if (kh >= 0 && kh < 3) acc[r] = mfma(wf(kh * 3 + j, ln), bw, acc[r]);
                    }
                }
                asm volatile("" ::: "memory");  // one row of windows in registers at a time
            }
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t v0 = run_vox0(o, r);
            h16_t *st = stg + wave * QSTG;
            float t3v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)  // channels past 8 meet zero weights (finite: no masks)
                t3v[j] = bf(f2h(elu_fast(acc[r][j] + s.b3a) + s.b3b));
            float ov[6];
            {
                const hx8 bt = pack8({t3v[0], t3v[1], t3v[2], t3v[3], 0.f, 0.f, 0.f, 0.f});
                const f32x4 a0 = mfma(wf(9, ln), bt, f32x4{0.f, 0.f, 0.f, 0.f});
                const f32x4 a1 = mfma(wf(10, ln), bt, f32x4{0.f, 0.f, 0.f, 0.f});
                const Raw18 &xr = ex[r];
                const float xv[6] = {bf(xr.x & 0xffffu), bf(xr.x >> 16), bf(xr.y & 0xffffu), bf(xr.y >> 16),
                                     bf(xr.z & 0xffffu), bf(xr.z >> 16)};
                const float o3[6] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1]};
#pragma unroll
                for (int j = 0; j < 6; ++j) ov[j] = bf(f2h(o3[j] * s.sc + s.b4 + xv[j]));  // j >= 4 used by kb 3 only
            }
            {
                put18(st, nl, kl, ov);
                if (t3o) put9(st + QO9A, nl, kl, t3v);
            }
            if constexpr (CHAIN) {
                // the next block's u1 (k_pm_t2's rounding points) and t2
                float u1[6];
#pragma unroll
                for (int j = 0; j < 6; ++j) u1[j] = bf(f2h(elu_fast(ov[j] + sn.b1a) + sn.b1b));  // zero-weight K past 17
                const hx8 bu = pack8({u1[0], u1[1], u1[2], u1[3], u1[4], u1[5], 0.f, 0.f});
                const f32x4 a2 = mfma(wf(11, ln), bu, f32x4{0.f, 0.f, 0.f, 0.f});
                float tn[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) tn[j] = elu_fast(a2[j] + sn.b2a) + sn.b2b;
                put9(st + QO9B, nl, kl, tn);
            }
            flush_run(st, ln, out + size_t(v0) * C, t3o ? t3o + size_t(v0) * BR : nullptr,
                          CHAIN ? t2n + size_t(v0) * BR : nullptr);
            ex[r] = ld18(x, run_vox0(on, r) + nl, kl);  // next tile's x (unconditional)
            if constexpr (PM_SB) __builtin_amdgcn_sched_barrier(0);
        }
        o = on;
    }
}

// K3 (the weight gradients; may run on another stream after K1 / K2): voxels are the MFMA
// reduction axis, so both operands are staged channel-major in LDS -- 16-B global loads whose 8
// elements are scattered to their channel rows as they are written (no LDS gathers after).
//
// k_pm_w2grad: dW2[co][kk][kd, ci] += sum_v gz3[v][co] t2[v + tap][ci].  A chunk is a TH x TW
// tile of whole D-lines (512 voxels); the workgroup stages gz3 over the tile and t2 over its
// circular (TH + 2) x (TW + 2) halo (positions -1 .. D of each line), and wave kk (9 waves) owns
// tap row kk = (kh, kw): its 2 accumulators (co x the 27 (kd, ci) window entries) sum over the
// workgroup's npc chunks, the next chunk's loads in flight during the current one's MFMAs.
// Staging unit: an item = 8 consecutive voxels of a line x 9 channels (144 contiguous bytes).  The
// global loads are coalesced 16-B pieces (consecutive lanes, consecutive pieces) written as they
// come to a voxel-major LDS area; then each thread takes one item (nine conflict-free 16-B reads:
// the 144-B item stride walks all 16 bank slots), transposes it in registers (one v_perm_b32 per
// output dword) and writes 9 channel rows of 8 voxels (16-B stores; 2 x 8 B for t2).  The t2 rows hold position
// p at index p + 8 so every group lands aligned (position -1 at 7, D at D + 8: the circular
// wrap copies).  Chunks of one workgroup are consecutive and each XCD takes a contiguous eighth of
// them (the halo re-reads hit that XCD's L2).
constexpr int NT9 = 9 * 64;
// t2 is staged as THREE copies shifted by kd - 1 positions, copy kd holding position j + kd - 1
// (circular) at index j of each D-line, so the B operand of lane (kd, ci) -- 8 consecutive
// positions starting at d0 + kd - 1 -- is ONE aligned 16-byte read (a single unshifted copy needs
// five dword reads and four v_alignbyte per operand, 9 waves x 16 k-steps x 2 per chunk).  The
// channel stride CS has CS / 8 = 1 and the copy stride CK = 9 CS has CK / 8 = 9 (mod 16), so the 16
// lanes of a lane group read 16 distinct 16-byte bank slots.  Copy 1 is the items' transpose;
// copies 0 and 2 are built from it (dword reads + v_alignbyte once per row group, not per use).
#ifndef PM_W2ROWS
#define PM_W2ROWS 1  // D = 32: a wave per (tap row kh, chunk row), B fragments slid along the row (0: a wave per tap row)
#endif
template <int D>
struct W2c {
    // D = 32, 64 (PM_W2ROWS): 12 waves, wave (kh, r, s) sums taps (kh, 0..2) over chunk row r (line
    // segment s of 32 voxels) -- its TW
    // lines' A fragments are read once for 3 taps and the B fragments of halo columns c, c + 1,
    // c + 2 are shared by neighbouring lines (TW + 2 column reads instead of 3 TW): 192 instead of
    // 432 16-byte LDS reads per chunk for the same 288 MFMAs.  Otherwise 9 waves, one per tap row.
    static constexpr bool ROWS = PM_W2ROWS && (D == 32 || D == 64);
    static constexpr int SEG = D >= 32 ? D / 32 : 1;        // ROWS: 32-voxel k-steps per line
    static constexpr int NL = CHV / D;  // lines per chunk
    static constexpr int TH = NL >= 64 ? 8 : NL >= 16 ? 4 : NL >= 4 ? 2 : 1, TW = NL / TH;
    static constexpr int LW = TW + 2, HL = (TH + 2) * LW;  // halo lines
    static constexpr int GPL = D / 8;                       // 8-voxel groups per line
    static constexpr int CS = 8 * (HL * D / 8 + ((1 - HL * D / 8) % 16 + 16) % 16);  // channel stride
    static constexpr int CK = 9 * CS;                       // copy stride
    static constexpr int ZI = NL * GPL, TI = HL * GPL;      // staging items (gz3, t2)
    static constexpr int NPC = (ZI + TI) * 9;               // 16-B pieces per chunk
    static constexpr int NPART = TH * SEG;                  // ROWS: waves per tap row (chunk row, segment)
    static constexpr int NTW = ROWS ? 3 * NPART * 64 : NT9; // threads
    static constexpr int NP = (NPC + NTW - 1) / NTW;        // pieces per thread
    static constexpr int RAW = (ZI + TI) * 72;              // voxel-major staging area (elements)
    static constexpr int NRG = BR * HL * GPL;               // row groups of copies 0 / 2 to build
    // the raw area after the copies, or (when that would not fit) over copy 2: dead once the items
    // are transposed, before copy 2 is built (one more barrier per chunk then)
    static constexpr bool ALIAS = size_t(16 * ZP + 3 * CK + RAW) * 2 > 160 * 1024;
    static constexpr int RAWO = ALIAS ? 2 * CK : 3 * CK;    // raw offset in the t2 area
    static constexpr size_t LDS = size_t(16 * ZP + (ALIAS ? std::max(3 * CK, 2 * CK + RAW) : 3 * CK + RAW)) * 2;
    static_assert(NL * D == CHV && TH * TW == NL && D % 8 == 0, "chunk");
    static_assert(ZI + TI <= NTW, "one staging item per thread");
    static_assert(NTW <= 1024 && (!ROWS || size_t(NTW / 64) * 6 * 256 * 4 <= LDS), "row-wave partials fit");
    static_assert((CS / 8) % 16 == 1 && (CK / 8) % 16 == 9, "bank slots");
    static_assert(LDS <= 160 * 1024, "LDS");
};

// element e (0..71) of a staged 8-voxel x 9-channel item (voxel-major, 16-bit)
__device__ __forceinline__ uint32_t item_el(const uint32_t (&w)[36], int e) {
    return (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
}
// channel c of the item's 8 voxels as 4 dwords (voxels 2k, 2k + 1 in dword k): one byte permute each
__device__ __forceinline__ u32x4 item_row(const uint32_t (&w)[36], int c) {
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ea = 18 * k + c, eb = ea + 9;
        // v_perm_b32: selector values 0-3 pick bytes of the second source, 4-7 of the first
        const uint32_t sel = (ea & 1 ? 0x0302u : 0x0100u) | ((eb & 1 ? 0x0706u : 0x0504u) << 16);
        o[k] = __builtin_amdgcn_perm(w[eb >> 1], w[ea >> 1], sel);
    }
    return u32x4{o[0], o[1], o[2], o[3]};
}

template <int D>
__device__ __forceinline__ void pm_w2grad(const PmArgs &a, int nchunk, int npc, const h16_t *__restrict__ gz3,
                                          const h16_t *__restrict__ t2, float *__restrict__ p2a) {
    using K = W2c<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *zT = reinterpret_cast<h16_t *>(smem);  // gz3 [16][ZP] channel-major (rows >= 9 never read into results)
    h16_t *tT = zT + 16 * ZP;                      // t2 copies [3 (kd)][9][HL][D] (strides CK, CS)
    h16_t *raw = tT + K::RAWO;                     // [items][72] voxel-major (16-B aligned)
    const int tid = threadIdx.x, lane = tid & 63, kk = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int kh = kk / 3, kw = kk - 3 * kh;
    const int nth = a.H / K::TH, ntw = a.W / K::TW;
    // workgroup -> chunk range (XCD-aware when the grid is a multiple of 8)
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int slot = (nwg & 7) ? bid : (bid & 7) * (nwg >> 3) + (bid >> 3);
    const int c0 = slot * npc;
    int toff[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int e = min(16 * n + row, 26), kd = e / BR, ci = e - kd * BR;
        toff[n] = kd * K::CK + ci * K::CS;
    }
    u32x4 v[K::NP];
    auto load = [&](int c) {
        const int tw_i = c % ntw, r = c / ntw, th_i = r % nth, b = r / nth;
        const int h0 = th_i * K::TH, w0 = tw_i * K::TW;
#pragma unroll
        for (int u = 0; u < K::NP; ++u) {
            const int p = min(tid + u * K::NTW, K::NPC - 1), item = p / 9, j = p - item * 9;
            const bool z = item < K::ZI;
            const int it = z ? item : item - K::ZI, il = it / K::GPL, ig = it - il * K::GPL;
            int hh, ww;
            if (z) {
                hh = h0 + il / K::TW;
                ww = w0 + il % K::TW;
            } else {
                const int lh = il / K::LW, lw = il - lh * K::LW;
                hh = wrapm(h0 - 1 + lh, a.H);
                ww = wrapm(w0 - 1 + lw, a.W);
            }
            const h16_t *src = (z ? gz3 : t2) + (((int64_t(b) * a.H + hh) * a.W + ww) * D + 8 * ig) * BR;
            v[u] = reinterpret_cast<const u32x4 *>(src)[j];
        }
    };
    // this thread's staging item (transpose phase): gz3 line il (tid < ZI) or t2 halo line il, group ig
    const bool zitem = tid < K::ZI, titem = !zitem && tid < K::ZI + K::TI;
    const int it = zitem ? tid : min(tid - K::ZI, K::TI - 1);
    const int il = it / K::GPL, ig = it - il * K::GPL;
    h16_t *dst = zitem ? zT + il * D + 8 * ig : tT + K::CK + il * D + 8 * ig;  // copy 1
    const int pitch = zitem ? ZP : K::CS;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    // ROWS: wave kk = (rh * TH + rr) * SEG + sg (tap row rh, chunk row rr, line segment sg), taps (rh, 0..2)
    const int rh = kk / K::NPART, rr = (kk - rh * K::NPART) / K::SEG, sg = kk - rh * K::NPART - rr * K::SEG;
    f32x4 racc[K::ROWS ? 3 : 1][2];
#pragma unroll
    for (int t = 0; t < (K::ROWS ? 3 : 1); ++t) racc[t][0] = racc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int cend = min(c0 + npc, nchunk);
    if (c0 < cend) load(c0);
#pragma unroll 1
    for (int c = c0; c < cend; ++c) {
        if constexpr (K::ALIAS) __syncthreads();  // the previous chunk's readers of copy 2 (= raw) are done
#pragma unroll
        for (int u = 0; u < K::NP; ++u) {  // raw pieces (non-aliased: the area's readers passed the last barrier)
            const int p = tid + u * K::NTW;
            if (p < K::NPC) reinterpret_cast<u32x4 *>(raw)[p] = v[u];
        }
        __syncthreads();  // raw complete; the previous chunk's fragments are read
        if (zitem || titem) {
            uint32_t w[36];
            const u32x4 *src = reinterpret_cast<const u32x4 *>(raw) + (zitem ? tid : K::ZI + it) * 9;
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                const u32x4 q = src[j];
                w[4 * j] = q.x;
                w[4 * j + 1] = q.y;
                w[4 * j + 2] = q.z;
                w[4 * j + 3] = q.w;
            }
#pragma unroll
            for (int ch = 0; ch < BR; ++ch) *reinterpret_cast<u32x4 *>(dst + ch * pitch) = item_row(w, ch);
        }
        __syncthreads();  // copy 1 complete (and raw dead)
        // copies 0 and 2 of row group (channel, line, group) from copy 1: dwords 4g - 1 .. 4g + 4
        // of the line (circular), each output dword one v_alignbyte
        for (int q = tid; q < K::NRG; q += K::NTW) {
            const int g = q % K::GPL, lr = q / K::GPL;  // lr = channel * HL + line
            const uint32_t *r1 = reinterpret_cast<const uint32_t *>(tT + K::CK + (lr / K::HL) * K::CS + (lr % K::HL) * D);
            const u32x4 m = reinterpret_cast<const u32x4 *>(r1)[g];
            const uint32_t um = r1[g == 0 ? D / 2 - 1 : 4 * g - 1], up = r1[g == K::GPL - 1 ? 0 : 4 * g + 4];
            const size_t ro = size_t(lr / K::HL) * K::CS + (lr % K::HL) * D + 8 * g;
            *reinterpret_cast<u32x4 *>(tT + ro) =
                u32x4{__builtin_amdgcn_alignbyte(m.x, um, 2), __builtin_amdgcn_alignbyte(m.y, m.x, 2),
                      __builtin_amdgcn_alignbyte(m.z, m.y, 2), __builtin_amdgcn_alignbyte(m.w, m.z, 2)};
            *reinterpret_cast<u32x4 *>(tT + 2 * K::CK + ro) =
                u32x4{__builtin_amdgcn_alignbyte(m.y, m.x, 2), __builtin_amdgcn_alignbyte(m.z, m.y, 2),
                      __builtin_amdgcn_alignbyte(m.w, m.z, 2), __builtin_amdgcn_alignbyte(up, m.w, 2)};
        }
        __syncthreads();
        if (c + 1 < cend) load(c + 1);
        if constexpr (K::ROWS) {
            // wave (rh = tap row, rr = chunk row, sg = segment): line lw of the row takes halo columns
            // lw .. lw + 2 of halo row rr + rh; a line segment is one k-step
            const h16_t *bt = tT + (rr + rh) * K::LW * D + 32 * sg + 8 * kb;
            hx8 bw[3][2];
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int n = 0; n < 2; ++n) bw[c][n] = *reinterpret_cast<const hx8 *>(bt + toff[n] + c * D);
#pragma unroll
            for (int lw = 0; lw < K::TW; ++lw) {
#pragma unroll
                for (int n = 0; n < 2; ++n) bw[(lw + 2) % 3][n] = *reinterpret_cast<const hx8 *>(bt + toff[n] + (lw + 2) * D);
                const hx8 af = *reinterpret_cast<const hx8 *>(zT + row * ZP + (rr * K::TW + lw) * D + 32 * sg + 8 * kb);
#pragma unroll
                for (int t = 0; t < 3; ++t)
#pragma unroll
                    for (int n = 0; n < 2; ++n) racc[t][n] = mfma(af, bw[(lw + t) % 3][n], racc[t][n]);
            }
        } else {
#pragma unroll 4
            for (int ks = 0; ks < CHV / 32; ++ks) {
                const int vv = 32 * ks + 8 * kb, l = vv / D, d0 = vv - l * D;
                const int hl = (l / K::TW + kh) * K::LW + l % K::TW + kw;
                const hx8 af = *reinterpret_cast<const hx8 *>(zT + row * ZP + vv);
                const int off = hl * D + d0;  // copy kd: position d0 - 1 + kd at index d0
#pragma unroll
                for (int n = 0; n < 2; ++n) acc[n] = mfma(af, *reinterpret_cast<const hx8 *>(tT + toff[n] + off), acc[n]);
            }
        }
    }
    if constexpr (K::ROWS) {
        // the NPART waves of a tap row summed in wave order through LDS (over the dead tiles)
        float *red = reinterpret_cast<float *>(smem);  // [wave][tap t][n][lane][4]
        __syncthreads();  // every wave's last MFMA reads are done
#pragma unroll
        for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int n = 0; n < 2; ++n)
                *reinterpret_cast<f32x4 *>(red + (((kk * 3 + t) * 2 + n) * 64 + lane) * 4) = racc[t][n];
        __syncthreads();
        if (kk == rh * K::NPART) {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                float *dstp = p2a + (int64_t(bid) * 9 + rh * 3 + t) * NER;
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                    f32x4 v = racc[t][n];
                    for (int q = 1; q < K::NPART; ++q)
                        v += *reinterpret_cast<const f32x4 *>(red + ((((kk + q) * 3 + t) * 2 + n) * 64 + lane) * 4);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int co = 4 * kb + j, col = 16 * n + row;
                        if (co < BR && col < 27) dstp[co * 27 + col] = v[j];
                    }
                }
            }
        }
    } else {
        float *dstp = p2a + (int64_t(bid) * 9 + kk) * NER;
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = 4 * kb + j, col = 16 * n + row;
                if (co < BR && col < 27) dstp[co * 27 + col] = acc[n][j];
            }
    }
}
template <int D>
__global__ __launch_bounds__(W2c<D>::NTW) void k_pm_w2grad(PmArgs a, int nchunk, int npc, const h16_t *__restrict__ gz3,
                                                   const h16_t *__restrict__ t2, float *__restrict__ p2a) {
    pm_w2grad<D>(a, nchunk, npc, gz3, t2, p2a);
}
// A whole run's W2 gradients in ONE launch (round 6): grid.y = the run's blocks, each block's gz3 and
// partial rows in its workspace slice (base + i stride), its t2 from the pointer table.  Same
// workgroups and arithmetic per block as k_pm_w2grad (the partial rows are bit-identical); the
// chain of data kernels no longer waits behind 50 x 2 small weight-gradient launches, and one
// launch of 50 x the work fills the chip.
constexpr int MAXRUN = 64;
struct MidRunPtrs {
    const h16_t *t2[MAXRUN], *t3[MAXRUN], *x[MAXRUN], *g[MAXRUN];
};
struct MidRunWs {
    const char *base;
    size_t stride;
    int64_t ogz3, ogz1, op2a, op2b;  // byte offsets inside a block's workspace slice
};
template <int D>
__global__ __launch_bounds__(W2c<D>::NTW) void k_pm_w2grad_run(PmArgs a, int nchunk, int npc, MidRunWs w, MidRunPtrs r) {
    const int i = blockIdx.y;
    const char *b = w.base + size_t(i) * w.stride;
    pm_w2grad<D>(a, nchunk, npc, reinterpret_cast<const h16_t *>(b + w.ogz3), r.t2[i],
                 reinterpret_cast<float *>(const_cast<char *>(b + w.op2a)));
}

// k_pm_w13grad: W1 (sum gz1 (x) u1, u1 = bf16(elu(x + b1a) + b1b)) and G3 (sum t3 (x) g) over npb
// pieces of SUBV voxels per workgroup (the next piece's loads in flight); wave w: (W1 | G3,
// 16-column tile).  Staging as k_pm_w2grad's: the piece's gz1 | t3 | x | g arrive as coalesced 16-B
// pieces written as they come to a voxel-major LDS area (x already turned into u1 by the loading
// thread), then 96 threads each transpose one item -- 8 voxels x 9 channels of gz1 / t3, or 4
// voxels x 18 channels of u1 / g, 144 contiguous bytes -- into channel rows (16- / 8-B stores).
constexpr int W13_ZI = SUBV / 8, W13_XI = SUBV / 4;  // items per 9-channel / 18-channel array
constexpr int W13_RAW = (2 * SUBV * BR + 2 * SUBV * C);  // raw area (elements): gz1 | t3 | u1 | g
static_assert(2 * W13_ZI + 2 * W13_XI <= NT, "one staging item per thread");

__device__ __forceinline__ void pm_w13grad(int npb, const h16_t *__restrict__ gz1, const h16_t *__restrict__ t3,
                                           const h16_t *__restrict__ x, const h16_t *__restrict__ g, float b1a,
                                           float b1b, float *__restrict__ p2b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int ch = blockIdx.x;
    Scal s{};
    s.b1a = b1a;
    s.b1b = b1b;
    h16_t *z1T = reinterpret_cast<h16_t *>(smem);  // [16][SP] gz1
    h16_t *t3T = z1T + 16 * SP;                     // [16][SP] t3
    h16_t *u1T = t3T + 16 * SP;                     // [32][SP] u1
    h16_t *gT = u1T + 32 * SP;                      // [32][SP] g
    h16_t *raw = gT + 32 * SP;                      // [W13_RAW] voxel-major
    const int isG3 = wave >> 1, nt = wave & 1;
    const h16_t *aT = isG3 ? t3T : z1T, *bT = isG3 ? gT : u1T;
    // per piece: gz1 / t3 SUBV * 9 / 8 16-B pieces each, x / g SUBV * 18 / 8 each
    constexpr int N9 = SUBV * BR / 8, N18 = SUBV * C / 8, NQ = 2 * N9 + 2 * N18, PQ = (NQ + NT - 1) / NT;
    u32x4 vq[PQ];
    auto load = [&](int64_t v0) {
#pragma unroll
        for (int u = 0; u < PQ; ++u) {
            const int i = min(tid + u * NT, NQ - 1);
            const u32x4 *src;
            int k;
            if (i < N9) src = reinterpret_cast<const u32x4 *>(gz1 + v0 * BR), k = i;
            else if (i < 2 * N9) src = reinterpret_cast<const u32x4 *>(t3 + v0 * BR), k = i - N9;
            else if (i < 2 * N9 + N18) src = reinterpret_cast<const u32x4 *>(x + v0 * C), k = i - 2 * N9;
            else src = reinterpret_cast<const u32x4 *>(g + v0 * C), k = i - 2 * N9 - N18;
            vq[u] = src[k];
        }
    };
    // this thread's item: [0, ZI) gz1, [ZI, 2 ZI) t3 (8 voxels x 9), then u1, g (4 voxels x 18)
    const int nine = tid < 2 * W13_ZI, item = tid;
    const bool active = tid < 2 * W13_ZI + 2 * W13_XI;
    h16_t *dst;
    if (nine) dst = (item < W13_ZI ? z1T : t3T) + 8 * (item % W13_ZI);
    else dst = (item < 2 * W13_ZI + W13_XI ? u1T : gT) + 4 * ((item - 2 * W13_ZI) % W13_XI);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    load(int64_t(ch) * npb * SUBV);
#pragma unroll 1
    for (int pc = 0; pc < npb; ++pc) {
#pragma unroll
        for (int u = 0; u < PQ; ++u) {  // raw pieces (x as u1); the area's readers passed the last barrier
            const int i = tid + u * NT;
            if (i < NQ) {
                u32x4 q = vq[u];
                if (i >= 2 * N9 && i < 2 * N9 + N18) {
                    uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        w[j] = uint32_t(f2h(PM_ELU(h2f_lo(w[j]) + s.b1a) + s.b1b)) |
                               (uint32_t(f2h(PM_ELU(h2f_hi(w[j]) + s.b1a) + s.b1b)) << 16);
                    q = u32x4{w[0], w[1], w[2], w[3]};
                }
                reinterpret_cast<u32x4 *>(raw)[i] = q;
            }
        }
        __syncthreads();  // raw complete; the previous piece's fragments are read
        if (active) {
            uint32_t w[36];
            const u32x4 *src = reinterpret_cast<const u32x4 *>(raw) + 9 * item;  // every item is 144 B
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                const u32x4 q = src[j];
                w[4 * j] = q.x;
                w[4 * j + 1] = q.y;
                w[4 * j + 2] = q.z;
                w[4 * j + 3] = q.w;
            }
            if (nine) {
#pragma unroll
                for (int c = 0; c < BR; ++c) *reinterpret_cast<u32x4 *>(dst + c * SP) = item_row(w, c);
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    uint32_t o[2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {  // voxels 2k, 2k + 1 of channel c: elements 36 k + c, + 18
                        const int ea = 36 * k + c, eb = ea + 18;
                        const uint32_t sel = (ea & 1 ? 0x0302u : 0x0100u) | ((eb & 1 ? 0x0706u : 0x0504u) << 16);
                        o[k] = __builtin_amdgcn_perm(w[eb >> 1], w[ea >> 1], sel);
                    }
                    *reinterpret_cast<u32x2 *>(dst + c * SP) = u32x2{o[0], o[1]};
                }
            }
        }
        __syncthreads();
        if (pc + 1 < npb) load((int64_t(ch) * npb + pc + 1) * SUBV);
#pragma unroll
        for (int ks = 0; ks < SUBV / 32; ++ks) {
            const int ko = 32 * ks + 8 * kb;
            acc = mfma(*reinterpret_cast<const hx8 *>(aT + row * SP + ko),
                       *reinterpret_cast<const hx8 *>(bT + (16 * nt + row) * SP + ko), acc);
        }
    }
    float *dsto = p2b + int64_t(ch) * NEB + isG3 * BR * C;
    const int c = 16 * nt + row;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int oo = 4 * kb + j;
        if (oo < BR && c < C) dsto[oo * C + c] = acc[j];
    }
}
__global__ __launch_bounds__(NT) void k_pm_w13grad(int npb, const h16_t *__restrict__ gz1,
                                                   const h16_t *__restrict__ t3, const h16_t *__restrict__ x,
                                                   const h16_t *__restrict__ g, vq3d_preact_params p,
                                                   float *__restrict__ p2b) {
    pm_w13grad(npb, gz1, t3, x, g, *p.bias1a, *p.bias1b, p2b);
}
// the run's W1 / G3 gradients in one launch (grid.y = block; params: the run's [nblocks][11] table)
__global__ __launch_bounds__(NT) void k_pm_w13grad_run(int npb, MidRunWs w, MidRunPtrs r,
                                                       const float *const *__restrict__ params) {
    const int i = blockIdx.y;
    const char *b = w.base + size_t(i) * w.stride;
    pm_w13grad(npb, reinterpret_cast<const h16_t *>(b + w.ogz1), r.t3[i], r.x[i], r.g[i], *params[i * 11 + 3],
               *params[i * 11 + 4], reinterpret_cast<float *>(const_cast<char *>(b + w.op2b)));
}

// K4: every gradient entry summed over its partial rows in a fixed order and added into its
// gradient buffer.  A workgroup owns 32 consecutive entries of one partial array: 8 row groups
// x 32 entries (each row read one 128-B segment), then the 8 group sums in order.
struct RedOut {
    float *dw1, *dw2, *dw3, *db1a, *db1b, *db2a, *db2b, *db3a, *db3b, *dscale, *db4;
    const float *scale;
};

constexpr int NBA = (9 * NER + 31) / 32, NBB = (NEB + 31) / 32;

__device__ __forceinline__ void pm_reduce(const float *__restrict__ p1, int n1, const float *__restrict__ p2, int n2,
                                          const float *__restrict__ p2a, int nwa, const float *__restrict__ p2b,
                                          int nchb, const RedOut &o) {
    __shared__ float sm[8][32];
    const int el = threadIdx.x & 31, rg = threadIdx.x >> 5;
    const int blk = blockIdx.x;
    // blocks [0, NBA): W2 entries (kk, co, kd, ci) over the k_pm_w2grad workgroups; [NBA, NBA +
    // NBB): W1 / G3; the last: the 8 scalars over the K1 / K2 workgroups
    int e, n, stride;
    const float *P;
    if (blk < NBA) {
        e = blk * 32 + el;
        P = p2a + min(e, 9 * NER - 1);
        n = e < 9 * NER ? nwa : 0;
        stride = 9 * NER;
    } else if (blk < NBA + NBB) {
        e = (blk - NBA) * 32 + el;
        P = p2b + min(e, NEB - 1);
        n = e < NEB ? nchb : 0;
        stride = NEB;
    } else {
        e = el;
        const bool first = el < NE1;
        P = first ? p1 + el : p2 + (el - NE1);
        n = el < NE1 + NE2 ? (first ? n1 : n2) : 0;
        stride = first ? NE1 : NE2;
    }
    float t = 0.f;
#pragma unroll 4
    for (int r = rg; r < n; r += 8) t += P[int64_t(r) * stride];
    sm[rg][el] = t;
    __syncthreads();
    if (rg != 0 || n == 0) return;
    t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += sm[i][el];
    if (blk < NBA) {
        const int kk = e / NER, r = e - kk * NER, co = r / (3 * BR), col = r - co * 3 * BR, kd = col / BR,
                  ci = col - kd * BR;
        o.dw2[(co * BR + ci) * 27 + kk * 3 + kd] += t;
    } else if (blk < NBA + NBB) {
        if (e < BR * C) {
            o.dw1[e] += t;  // [o][c]
        } else {
            const int r = e - BR * C, oo = r / C, co = r - oo * C;
            o.dw3[co * BR + oo] += *o.scale * t;  // G3 [o][co] -> W3 [co][o]
        }
    } else {
        float *const sl[NE1 + NE2] = {o.db4, o.db3b, o.db3a, o.dscale, o.db2b, o.db2a, o.db1b, o.db1a};
        *sl[e] += t;
    }
}

__global__ __launch_bounds__(NT) void k_pm_reduce(const float *__restrict__ p1, int n1, const float *__restrict__ p2,
                                                  int n2, const float *__restrict__ p2a, int nwa,
                                                  const float *__restrict__ p2b, int nchb, RedOut o) {
    pm_reduce(p1, n1, p2, n2, p2a, nwa, p2b, nchb, o);
}

// K4 of a whole run of blocks in one launch (blockIdx.y = block): block y's workspace at
// base + y * stride (same layout for every block), its gradient / scale pointers from the run's
// device tables [block][11] (w1, w2, w3, bias1a, bias1b, bias2a, bias2b, bias3a, bias3b, scale,
// bias4).  Entry for entry the same fixed-order sums as k_pm_reduce.
__global__ __launch_bounds__(NT) void k_pm_reduce_run(const char *__restrict__ base, size_t stride, int64_t o1,
                                                      int n1, int64_t o2, int n2, int64_t oa, int nwa, int64_t ob,
                                                      int nchb, float *const *gtab, const float *const *ptab) {
    const char *ws = base + size_t(blockIdx.y) * stride;
    float *const *g = gtab + blockIdx.y * 11;
    const RedOut o{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], ptab[blockIdx.y * 11 + 9]};
    pm_reduce(reinterpret_cast<const float *>(ws + o1), n1, reinterpret_cast<const float *>(ws + o2), n2,
              reinterpret_cast<const float *>(ws + oa), nwa, reinterpret_cast<const float *>(ws + ob), nchb, o);
}

// ============================================================================================ host
constexpr int BTH = 4, BTW = 8;  // backward tile

// k_pm_fwd: the same carve as k_pm_bwd2 without the block sums
constexpr size_t fwd_lds() { return size_t(2 * QIMG) * 2 + size_t(12 * 64) * 16 + size_t(QNW * QSTG) * 2; }
// k_pm_bwd2: 2 halo images (the fp32 weights over them in the prologue), 12 A-fragment images, 8 waves' output
// images, 32 sums
constexpr size_t bwd_lds() { return size_t(2 * QIMG) * 2 + size_t(12 * 64) * 16 + size_t(QNW * QSTG) * 2 + 32 * 4; }

int n_cu() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    }
    return n;
}

template <class K>
int resident(K kern, size_t lds, int threads = NT) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, lds) != hipSuccess || per < 1) per = 1;
    (void)hipGetLastError();
    return per;
}

PmArgs make_args(int B, int H, int W, int D, int TH, int TW) {
    PmArgs a;
    a.B = B;
    a.H = H;
    a.W = W;
    a.D = D;
    a.nth = H / TH;
    a.ntw = W / TW;
    a.ntd = D / TD;
    a.ntiles = B * a.nth * a.ntw * a.ntd;
    return a;
}

// resident workgroups per CU of a tile kernel (dynamic LDS opted in once)
template <class K>
int per_cu(K kern, size_t lds, int threads = NT) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(lds));
    return resident(kern, lds, threads);
}
// K2 grid: both variants must give the same count (the chained variant writes the previous
// block's K1 partial rows, whose count the reduction assumes to be the K2 grid)
int bwd2_blocks(const PmArgs &a) {
    static int per = 0;
    if (!per)
        per = std::min(per_cu(k_pm_bwd2<false>, bwd_lds(), QNT), per_cu(k_pm_bwd2<true>, bwd_lds(), QNT));
    if (PM_BWD_PER > 0) per = std::min(per, PM_BWD_PER);
    return std::max(1, std::min(a.ntiles, per * n_cu()));
}

// k_pm_w13grad LDS: z1T, t3T [16][SP] + u1T, gT [32][SP] + raw
constexpr size_t w13_lds() { return size_t(96 * SP + W13_RAW) * 2; }  // + the raw area

template <int D>
void launch_w2(const PmArgs &a, int nwa, int npc, const h16_t *gz3, const h16_t *t2, float *p2a, hipStream_t s) {
    static bool init = false;
    if (!init) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad<D>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<D>::LDS));
        init = true;
    }
    k_pm_w2grad<D><<<nwa, W2c<D>::NTW, W2c<D>::LDS, s>>>(a, int(int64_t(a.B) * a.H * a.W * a.D / CHV), npc, gz3, t2, p2a);
}

void launch_fwd(int batch, int h, int w, int dd, const void *x, const float *w2, const float *w3,
                const vq3d_preact_params &p, void *out, const void *t2, void *t3, const float *w1n,
                const vq3d_preact_params *pn, void *t2n, hipStream_t s) {
    const PmArgs a = make_args_q(batch, h, w, dd);
    static int per = 0;
    if (!per) per = std::min(per_cu(k_pm_fwd<false>, fwd_lds(), QNT), per_cu(k_pm_fwd<true>, fwd_lds(), QNT));
    if (PM_FWD_PER > 0) per = std::min(per, PM_FWD_PER);
    const unsigned g2 = unsigned(std::max(1, std::min(a.ntiles, per * n_cu())));
    if (w1n)
        k_pm_fwd<true><<<g2, QNT, fwd_lds(), s>>>(a, (const h16_t *)t2, (const h16_t *)x, w2, w3, p, (h16_t *)t3,
                                                   (h16_t *)out, w1n, *pn, (h16_t *)t2n);
    else
        k_pm_fwd<false><<<g2, QNT, fwd_lds(), s>>>(a, (const h16_t *)t2, (const h16_t *)x, w2, w3, p, (h16_t *)t3,
                                                    (h16_t *)out, nullptr, p, nullptr);
}

// backward workspace: K1 / K2 scalar partial rows, the W2 partials [nwa][9][NER], the W1 / G3
// partials [nchb][NEB], then gz3 and gz1 (bf16 [nvox][9] each, 256-B aligned)
struct MidWs {
    float *p1, *p2, *p2a, *p2b;
    h16_t *gz3, *gz1;
    int n1, n2, nwa, nchb, npc, npb;
    size_t bytes;
};
constexpr int kW2Chunks = 4;  // 512-voxel chunks per k_pm_w2grad workgroup (when they divide; measured 2: 25.6, 4: 23.8 us)
constexpr int kW13Pieces = 4;  // SUBV-voxel pieces per k_pm_w13grad workgroup (when they divide)
// timing experiments only: VQ3D_W2_CHUNKS overrides the chunks per workgroup (read once)
int w2_chunks() {
    static const int n = [] {
        const char *e = std::getenv("VQ3D_W2_CHUNKS");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 ? v : kW2Chunks;
    }();
    return n;
}
int w13_pieces() {  // timing experiments only: VQ3D_W13_PIECES
    static const int n = [] {
        const char *e = std::getenv("VQ3D_W13_PIECES");
        const int v = e ? std::atoi(e) : 0;
        return v > 0 ? v : kW13Pieces;
    }();
    return n;
}

MidWs mid_ws(int B, int H, int W, int D, void *base) {
    MidWs m;
    const int64_t nvox = int64_t(B) * H * W * D;  // a multiple of 512 (H, W, D % 8 == 0)
    const PmArgs a = make_args(B, H, W, D, BTH, BTW);
    m.n2 = bwd2_blocks(a);
    m.n1 = m.n2;  // K1 rows: k_pm_bwd1's grid, or the next block's chained K2 grid
    m.npc = w2_chunks();
    while ((nvox / CHV) % m.npc) m.npc >>= 1;
    m.npb = w13_pieces();
    while ((nvox / SUBV) % m.npb) m.npb >>= 1;
    m.nwa = int(nvox / (int64_t(m.npc) * CHV));
    m.nchb = int(nvox / (int64_t(m.npb) * SUBV));
    auto al = [](size_t n) { return (n + 255) & ~size_t(255); };
    size_t off = 0;
    const size_t o1 = off;
    off = al(off + size_t(m.n1) * NE1 * 4);
    const size_t o2 = off;
    off = al(off + size_t(m.n2) * NE2 * 4);
    const size_t oa = off;
    off = al(off + size_t(9) * m.nwa * NER * 4);
    const size_t ob = off;
    off = al(off + size_t(m.nchb) * NEB * 4);
    const size_t oz3 = off;
    off = al(off + size_t(nvox) * BR * 2);
    const size_t oz1 = off;
    off = al(off + size_t(nvox) * BR * 2);
    m.bytes = off;
    char *c = static_cast<char *>(base);
    m.p1 = reinterpret_cast<float *>(c + o1);
    m.p2 = reinterpret_cast<float *>(c + o2);
    m.p2a = reinterpret_cast<float *>(c + oa);
    m.p2b = reinterpret_cast<float *>(c + ob);
    m.gz3 = reinterpret_cast<h16_t *>(c + oz3);
    m.gz1 = reinterpret_cast<h16_t *>(c + oz1);
    return m;
}

}  // namespace

// The W2-gradient kernel as the weight gradient of a plain 9 -> 9 3x3x3 circular conv (the up
// blocks' branch conv2 on the upsampled t2 at 256^2 x 64): dW[co][ci][tap] = sum_v g[v][co]
// x[v + tap][ci] is exactly k_pm_w2grad's gz3 (x) t2 window sum; its partials are summed by the
// W2 section of k_pm_reduce (fixed order, deterministic) straight into dw.
bool mid_w2grad_ok(const vq3d_conv_desc *d) {
    return d->dtype == VQ3D_HALF && d->cin == BR && d->cin2 == 0 && d->cout == BR && d->kernel == 3 &&
           d->stride == 1 && d->pad == 1 && d->pad_mode == VQ3D_PAD_CIRCULAR && d->pro_kind == VQ3D_PRO_NONE &&
           d->in_h == d->out_h && d->in_w == d->out_w && d->in_d == d->out_d && d->batch >= 1 && d->in_h % 8 == 0 &&
           d->in_w % 8 == 0 && d->in_d >= 8 && d->in_d <= 128 && (d->in_d & (d->in_d - 1)) == 0 &&
           int64_t(d->batch) * d->in_h * d->in_w * d->in_d * BR * 2 < (int64_t(1) << 31);  // k_pm_w2grad's tiles
}

namespace {
struct W2Plan {
    int nchunk, npc, nwa;
    size_t bytes;
};
W2Plan w2_plan(const vq3d_conv_desc *d) {
    W2Plan p;
    p.nchunk = int(int64_t(d->batch) * d->in_h * d->in_w * d->in_d / CHV);
    p.npc = w2_chunks();
    while (p.nchunk % p.npc) p.npc >>= 1;
    p.nwa = p.nchunk / p.npc;
    p.bytes = size_t(9) * p.nwa * NER * 4;
    return p;
}
}  // namespace

size_t mid_w2grad_ws(const vq3d_conv_desc *d) { return mid_w2grad_ok(d) ? w2_plan(d).bytes : 0; }

int mid_w2grad(const vq3d_conv_desc *d, const void *x, const void *g, float *dw, void *ws, size_t ws_bytes,
               hipStream_t s) {
    const W2Plan p = w2_plan(d);
    if (!mid_w2grad_ok(d) || !dw || !ws || ws_bytes < p.bytes) return fail("conv3d_bwd_weight(9->9 windowed): bad call");
    const PmArgs a = make_args(d->batch, d->in_h, d->in_w, d->in_d, BTH, BTW);
    float *p2a = static_cast<float *>(ws);
    const h16_t *gz = static_cast<const h16_t *>(g), *xt = static_cast<const h16_t *>(x);
    switch (d->in_d) {
        case 8: launch_w2<8>(a, p.nwa, p.npc, gz, xt, p2a, s); break;
        case 16: launch_w2<16>(a, p.nwa, p.npc, gz, xt, p2a, s); break;
        case 32: launch_w2<32>(a, p.nwa, p.npc, gz, xt, p2a, s); break;
        case 64: launch_w2<64>(a, p.nwa, p.npc, gz, xt, p2a, s); break;
        default: launch_w2<128>(a, p.nwa, p.npc, gz, xt, p2a, s); break;
    }
    RedOut o{};
    o.dw2 = dw;
    k_pm_reduce<<<NBA, NT, 0, s>>>(nullptr, 0, nullptr, 0, p2a, p.nwa, nullptr, 0, o);  // W2 blocks only
    return check_launch("conv3d_bwd_weight(9->9 windowed)");
}

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_mid_supported(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd) {
    // D a power of two in [16, 128]: the backward data tiles are 16 deep, the weight-gradient chunks
    // are tiles of whole D-lines
    return dtype == VQ3D_HALF && batch >= 1 && channels == C && branch == BR && h >= 8 && w >= 8 && h % 8 == 0 &&
           w % 8 == 0 && dd >= QTD && dd <= 128 && (dd & (dd - 1)) == 0 &&
           int64_t(batch) * h * w * dd * C * 2 < (int64_t(1) << 31);  // 32-bit byte offsets in the tile kernels
}

int vq3d_preact_mid_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                        int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                        const vq3d_preact_params *p, void *out, void *t2, void *t3, vq3d_stream_t stream) {
    return vq3d_preact_mid_fwd_stages(3, dtype, batch, channels, branch, h, w, dd, x, w1, w2, w3, p, out, t2, t3,
                                      stream);
}

int vq3d_preact_mid_fwd_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                               int32_t h, int32_t w, int32_t dd, const void *x, const float *w1, const float *w2,
                               const float *w3, const vq3d_preact_params *p, void *out, void *t2, void *t3,
                               vq3d_stream_t stream) {
    if (!vq3d_preact_mid_supported(dtype, batch, channels, branch, h, w, dd))
        return fail("preact_mid_fwd: shape outside the fused mid-level block kernels");
    if (!x || !w1 || !w2 || !w3 || !p || !out || !t2) return fail("preact_mid_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    const int64_t nvox = int64_t(batch) * h * w * dd;
    const unsigned g1 = unsigned(std::max<int64_t>(1, std::min<int64_t>(nvox / 2 / NT, 2048)));
    if (stages & 1) k_pm_t2<<<g1, NT, 0, s>>>(nvox, (const h16_t *)x, w1, *p, (h16_t *)t2);
    if (stages & 2) launch_fwd(batch, h, w, dd, x, w2, w3, *p, out, t2, t3, nullptr, nullptr, nullptr, s);
    return check_launch("preact_mid_fwd");
}

int vq3d_preact_mid_fwd_chain(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd, const void *x, const float *w2, const float *w3,
                              const vq3d_preact_params *p, const void *t2, void *out, void *t3,
                              const float *next_w1, const vq3d_preact_params *next_p, void *next_t2,
                              vq3d_stream_t stream) {
    if (!vq3d_preact_mid_supported(dtype, batch, channels, branch, h, w, dd))
        return fail("preact_mid_fwd_chain: shape outside the fused mid-level block kernels");
    if (!x || !w2 || !w3 || !p || !out || !t2) return fail("preact_mid_fwd_chain: null pointer");
    if (next_w1 && (!next_p || !next_t2)) return fail("preact_mid_fwd_chain: next_w1 needs next_p and next_t2");
    launch_fwd(batch, h, w, dd, x, w2, w3, *p, out, t2, t3, next_w1, next_p, next_t2, as_stream(stream));
    return check_launch("preact_mid_fwd_chain");
}

size_t vq3d_preact_mid_workspace_bytes(int32_t batch, int32_t h, int32_t w, int32_t dd) {
    return mid_ws(batch, h, w, dd, nullptr).bytes;
}

int vq3d_preact_mid_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                        int32_t dd, const void *g, const void *x, const void *t2, const void *t3, const float *w1,
                        const float *w2, const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                        void *workspace, size_t workspace_bytes, void *gx, vq3d_stream_t stream) {
    return vq3d_preact_mid_bwd_stages(31, dtype, batch, channels, branch, h, w, dd, g, x, t2, t3, w1, w2, w3, p, gr,
                                      workspace, workspace_bytes, gx, stream);
}

int vq3d_preact_mid_reduce_run(int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                               const void *workspaces, size_t workspace_stride, float *const *grads,
                               const float *const *params, vq3d_stream_t stream) {
    if (!vq3d_preact_mid_supported(VQ3D_HALF, batch, C, BR, h, w, dd))
        return fail("preact_mid_reduce_run: shape outside the fused mid-level block kernels");
    if (nblocks < 1 || nblocks > 65535 || !workspaces || !grads || !params)
        return fail("preact_mid_reduce_run: bad arguments");
    char *const b0 = static_cast<char *>(const_cast<void *>(workspaces));
    const MidWs m = mid_ws(batch, h, w, dd, b0);
    if (workspace_stride < m.bytes || workspace_stride % 256)
        return fail("preact_mid_reduce_run: workspace stride below vq3d_preact_mid_workspace_bytes or unaligned");
    auto off = [&](const void *p) { return int64_t(static_cast<const char *>(p) - b0); };
    k_pm_reduce_run<<<dim3(NBA + NBB + 1, unsigned(nblocks)), NT, 0, as_stream(stream)>>>(
        b0, workspace_stride, off(m.p1), m.n1, off(m.p2), m.n2, off(m.p2a), m.nwa, off(m.p2b), m.nchb, grads, params);
    return check_launch("preact_mid_reduce_run");
}

int vq3d_preact_mid_wgrad_run(int32_t dtype, int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                              const void *const *t2, const void *const *t3, const void *const *x,
                              const void *const *g, const float *const *params, void *workspaces,
                              size_t workspace_stride, vq3d_stream_t stream) {
    if (!vq3d_preact_mid_supported(dtype, batch, C, BR, h, w, dd))
        return fail("preact_mid_wgrad_run: shape / dtype outside the fused mid-level block kernels");
    if (nblocks < 1 || nblocks > 65535 || !t2 || !t3 || !x || !g || !params || !workspaces)
        return fail("preact_mid_wgrad_run: bad arguments");
    char *const b0 = static_cast<char *>(workspaces);
    const MidWs m = mid_ws(batch, h, w, dd, b0);
    if (workspace_stride < m.bytes || workspace_stride % 256)
        return fail("preact_mid_wgrad_run: workspace stride below vq3d_preact_mid_workspace_bytes or unaligned");
    for (int i = 0; i < nblocks; ++i)
        if (!t2[i] || !t3[i] || !x[i] || !g[i]) return fail("preact_mid_wgrad_run: null tensor pointer");
    hipStream_t s = as_stream(stream);
    const PmArgs a = make_args(batch, h, w, dd, BTH, BTW);
    const int nchunk = int(int64_t(batch) * h * w * dd / CHV);
    auto off = [&](const void *p) { return int64_t(static_cast<const char *>(p) - b0); };
    static bool init = false;
    if (!init) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad_run<8>), hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<8>::LDS));
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad_run<16>), hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<16>::LDS));
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad_run<32>), hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<32>::LDS));
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad_run<64>), hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<64>::LDS));
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad_run<128>), hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<128>::LDS));
        init = true;
    }
    for (int i0 = 0; i0 < nblocks; i0 += MAXRUN) {  // MAXRUN blocks per launch (kernel-argument tables)
        const int nb = std::min(MAXRUN, nblocks - i0);
        MidRunPtrs r{};
        for (int i = 0; i < nb; ++i) {
            r.t2[i] = static_cast<const h16_t *>(t2[i0 + i]);
            r.t3[i] = static_cast<const h16_t *>(t3[i0 + i]);
            r.x[i] = static_cast<const h16_t *>(x[i0 + i]);
            r.g[i] = static_cast<const h16_t *>(g[i0 + i]);
        }
        MidRunWs wr{b0 + size_t(i0) * workspace_stride, workspace_stride, off(m.gz3), off(m.gz1), off(m.p2a), off(m.p2b)};
        const dim3 ga(unsigned(m.nwa), unsigned(nb));
        switch (dd) {
            case 8: k_pm_w2grad_run<8><<<ga, W2c<8>::NTW, W2c<8>::LDS, s>>>(a, nchunk, m.npc, wr, r); break;
            case 16: k_pm_w2grad_run<16><<<ga, W2c<16>::NTW, W2c<16>::LDS, s>>>(a, nchunk, m.npc, wr, r); break;
            case 32: k_pm_w2grad_run<32><<<ga, W2c<32>::NTW, W2c<32>::LDS, s>>>(a, nchunk, m.npc, wr, r); break;
            case 64: k_pm_w2grad_run<64><<<ga, W2c<64>::NTW, W2c<64>::LDS, s>>>(a, nchunk, m.npc, wr, r); break;
            default: k_pm_w2grad_run<128><<<ga, W2c<128>::NTW, W2c<128>::LDS, s>>>(a, nchunk, m.npc, wr, r); break;
        }
        k_pm_w13grad_run<<<dim3(unsigned(m.nchb), unsigned(nb)), NT, w13_lds(), s>>>(m.npb, wr, r, params + size_t(i0) * 11);
    }
    return check_launch("preact_mid_wgrad_run");
}

int vq3d_preact_mid_bwd_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                               int32_t h, int32_t w, int32_t dd, const void *g, const void *x, const void *t2,
                               const void *t3, const float *w1, const float *w2, const float *w3,
                               const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *workspace,
                               size_t workspace_bytes, void *gx, vq3d_stream_t stream) {
    return vq3d_preact_mid_bwd_chain(stages, dtype, batch, channels, branch, h, w, dd, g, x, t2, t3, w1, w2, w3, p,
                                     gr, workspace, workspace_bytes, gx, nullptr, nullptr, nullptr, nullptr, 0,
                                     stream);
}

int vq3d_preact_mid_bwd_chain(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                              int32_t h, int32_t w, int32_t dd, const void *g, const void *x, const void *t2,
                              const void *t3, const float *w1, const float *w2, const float *w3,
                              const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *workspace,
                              size_t workspace_bytes, void *gx, const void *prev_t3, const float *prev_w3,
                              const vq3d_preact_params *prev_p, void *prev_workspace, size_t prev_workspace_bytes,
                              vq3d_stream_t stream) {
    if (!vq3d_preact_mid_supported(dtype, batch, channels, branch, h, w, dd))
        return fail("preact_mid_bwd: shape outside the fused mid-level block kernels");
    if (stages < 1 || stages > 31) return fail("preact_mid_bwd: stages must be a mask of 1 | 2 | 4 | 8 | 16");
    if (!g || !x || !t2 || !t3 || !w1 || !w2 || !w3 || !p || !gr || !workspace)
        return fail("preact_mid_bwd: null pointer");
    if ((stages & 2) && !gx) return fail("preact_mid_bwd: gx is required by the data stage");
    const bool chain = prev_t3 != nullptr;
    if (chain && (!prev_w3 || !prev_p || !prev_workspace))
        return fail("preact_mid_bwd_chain: prev_t3 needs prev_w3, prev_p and prev_workspace");
    if (chain && !(stages & 2)) return fail("preact_mid_bwd_chain: the chained K1 rides the data stage (2)");
    const vq3d_preact_grads &G = *gr;
    if (!G.dw1 || !G.dw2 || !G.dw3 || !G.dbias1a || !G.dbias1b || !G.dbias2a || !G.dbias2b || !G.dbias3a ||
        !G.dbias3b || !G.dscale || !G.dbias4)
        return fail("preact_mid_bwd: every gradient buffer is required");
    const MidWs m = mid_ws(batch, h, w, dd, workspace);
    if (workspace_bytes < m.bytes) return fail("preact_mid_bwd: workspace too small");
    MidWs mp{};
    if (chain) {
        mp = mid_ws(batch, h, w, dd, prev_workspace);
        if (prev_workspace_bytes < mp.bytes) return fail("preact_mid_bwd_chain: previous workspace too small");
    }
    hipStream_t s = as_stream(stream);
    const int64_t nvox = int64_t(batch) * h * w * dd;
    const PmArgs a = make_args(batch, h, w, dd, BTH, BTW);
    if (stages & 1) k_pm_bwd1<<<m.n1, NT, 0, s>>>(nvox, (const h16_t *)g, (const h16_t *)t3, w3, *p, m.gz3, m.p1);
    const PmArgs aq = make_args_q(batch, h, w, dd);
    if ((stages & 2) && chain)
        k_pm_bwd2<true><<<m.n2, QNT, bwd_lds(), s>>>(aq, m.gz3, (const h16_t *)t2, (const h16_t *)x, (const h16_t *)g,
                                                     w1, w2, *p, (h16_t *)gx, m.gz1, m.p2, (const h16_t *)prev_t3,
                                                     prev_w3, *prev_p, mp.gz3, mp.p1);
    else if (stages & 2)
        k_pm_bwd2<false><<<m.n2, QNT, bwd_lds(), s>>>(aq, m.gz3, (const h16_t *)t2, (const h16_t *)x,
                                                      (const h16_t *)g, w1, w2, *p, (h16_t *)gx, m.gz1, m.p2,
                                                      nullptr, nullptr, *p, nullptr, nullptr);
    if (stages & 4) {
        const h16_t *t2b = static_cast<const h16_t *>(t2);
        switch (dd) {
            case 8: launch_w2<8>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            case 16: launch_w2<16>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            case 32: launch_w2<32>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            case 64: launch_w2<64>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            default: launch_w2<128>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
        }
    }
    if (stages & 8) {
        k_pm_w13grad<<<m.nchb, NT, w13_lds(), s>>>(m.npb, m.gz1, (const h16_t *)t3, (const h16_t *)x,
                                                   (const h16_t *)g, *p, m.p2b);
    }
    RedOut o{G.dw1, G.dw2, G.dw3, G.dbias1a, G.dbias1b, G.dbias2a, G.dbias2b, G.dbias3a, G.dbias3b,
             G.dscale, G.dbias4, p->scale};
    if (stages & 16) k_pm_reduce<<<NBA + NBB + 1, NT, 0, s>>>(m.p1, m.n1, m.p2, m.n2, m.p2a, m.nwa, m.p2b, m.nchb, o);
    return check_launch("preact_mid_bwd");
}

}  // extern "C"
