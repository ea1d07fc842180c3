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

#include <algorithm>

// Timing experiments only (tools builds: make -C 3d-vq-vae-2_amd exp EXP=N): bit 0 skips the
// forward tile kernel's k^3 phase, 1 its 1x1 phase, 2 its stores, 3 its staging; bits 4 .. 8 the
// backward data tile kernel's staging (loads + LDS writes), k^3 dgrad phase, gx phase, chained
// previous-block phase and global stores.  The product library is built with PM_EXP = 0.
#ifndef PM_EXP
#define PM_EXP 0
#endif
// resident workgroups per CU of the forward / backward-data tile kernels: 0 = as many as fit
// (timing experiments set a cap: make exp EXP=N EXPDEF=PM_FWD_PER)
#ifndef PM_FWD_PER
#define PM_FWD_PER 0
#endif
#ifndef PM_BWD_PER
#define PM_BWD_PER 0
#endif
// minimum waves per SIMD the backward-data tile kernel is compiled for (1: the compiler's choice)
#ifndef PM_BWD_WPE
#define PM_BWD_WPE 1
#endif

namespace vq3d {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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
__device__ __forceinline__ float bf(uint32_t u16) { return __uint_as_float(u16 << 16); }
__device__ __forceinline__ float elu_d_act(float t, float b) {  // elu'(z) from t = elu(z) + b
    const float z1 = t - b;
    return z1 > 0.f ? 1.f : z1 + 1.f;
}

// 8 consecutive bf16 from LDS at element offset `off` (any parity; base 16-B aligned): five
// dwords + v_alignbyte when odd
__device__ __forceinline__ bf16x8 read8(const bf16_t *base, int off) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(base + (off & ~1));
    const uint32_t sh = uint32_t(off & 1) * 2u;
    const uint32_t u0 = q[0], u1 = q[1], u2 = q[2], u3 = q[3], u4 = q[4];
    const uint4 r = {__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                     __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
    return __builtin_bit_cast(bf16x8, r);
}

// 8 bf16 at element offsets off + j * stride (j = 0..7) from LDS; zeros when !ok
__device__ __forceinline__ bf16x8 gather8(const bf16_t *base, int off, int stride, bool ok) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (ok) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            w[j] = uint32_t(base[off + 2 * j * stride]) | (uint32_t(base[off + (2 * j + 1) * stride]) << 16);
    }
    return __builtin_bit_cast(bf16x8, uint4{w[0], w[1], w[2], w[3]});
}

__device__ __forceinline__ bf16x8 pack8(const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = uint32_t(f2bf(v[2 * j])) | (uint32_t(f2bf(v[2 * j + 1])) << 16);
    return __builtin_bit_cast(bf16x8, uint4{w[0], w[1], w[2], w[3]});
}

__device__ __forceinline__ f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
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
__device__ __forceinline__ bf16x8 w2_frag(const float *w2, int kk, int lane) {
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
    __device__ __forceinline__ void load(const PmArgs &a, const Org &o, const bf16_t *__restrict__ src) {
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
    __device__ __forceinline__ void store(bf16_t *lines) const {
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
    __device__ __forceinline__ void load(const PmArgs &a, const Org &o, const bf16_t *__restrict__ src) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int i = min(tid + u * NT, N - 1);
            const int r = i / PR, part = i - PR * r;
            v[u] = reinterpret_cast<const u32x4 *>(src + run_vox<TW>(a, o, r) * CH)[part];
        }
    }
    __device__ __forceinline__ void store(bf16_t *dst) const {
        const int tid = threadIdx.x;
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int i = tid + u * NT;
            if (i < N) reinterpret_cast<u32x4 *>(dst)[i] = v[u];
        }
    }
};

template <int TH, int TW, int CH>
__device__ __forceinline__ void store_tile(const PmArgs &a, const Org &o, const bf16_t *src, bf16_t *__restrict__ dst) {
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
__device__ __forceinline__ void zero_pads(bf16_t *lines, int nimg, bf16_t *const *tails, const int *tail_at,
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
__global__ __launch_bounds__(NT) void k_pm_t2(int64_t nvox, const bf16_t *__restrict__ x,
                                              const float *__restrict__ w1, vq3d_preact_params p,
                                              bf16_t *__restrict__ t2o) {
    __shared__ float w1s[BR * C];
    // W1 and u1 rounded to bf16: the operands of the chained forward's matrix-core t2 stage
    for (int i = threadIdx.x; i < BR * C; i += NT) w1s[i] = bf(f2bf(w1[i]));
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
                uu[c] = bf(f2bf(elu(bf((e & 1) ? (d >> 16) : (d & 0xffffu)) + s.b1a) + s.b1b));
            }
            float t2v[BR];
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                asm volatile("" ::: "memory");  // one W1 row (18 floats) in registers at a time
                float acc = 0.f;
#pragma unroll
                for (int c = 0; c < C; ++c) acc = fmaf(w1s[o * C + c], uu[c], acc);
                t2v[o] = elu(acc + s.b2a) + s.b2b;
            }
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                const uint32_t hb = f2bf(t2v[o]);
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

// t3 and out of a TH x TW x 8 tile from t2 on its halo and x; CHAIN: also the next block's t2
template <int TH, int TW, bool CHAIN>
__global__ __launch_bounds__(NT) void k_pm_fwd(PmArgs a, const bf16_t *__restrict__ t2, const bf16_t *__restrict__ x,
                                               const float *__restrict__ w2, const float *__restrict__ w3,
                                               vq3d_preact_params p, bf16_t *__restrict__ t3o,
                                               bf16_t *__restrict__ out, const float *__restrict__ w1n,
                                               vq3d_preact_params pn, bf16_t *__restrict__ t2n) {
    using T = Tile<TH, TW>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t *t2l = reinterpret_cast<bf16_t *>(smem);  // halo lines [NL][LSP]; CHAIN: then next t2 [TV][9]
    bf16_t *t3s = t2l + T::LINES;                     // [TV][9]
    bf16_t *xs = t3s + T::S9;                         // [TV][18]: x, then out in place
    float *w1ns = reinterpret_cast<float *>(xs + T::S18);  // CHAIN: next block's W1 [o][c]
    bf16_t *u1s = reinterpret_cast<bf16_t *>(w1ns + BR * C);  // CHAIN: next block's u1 [TV][18]
    static_assert(T::LINES >= T::TV * BR, "next t2 fits the halo image");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if constexpr (CHAIN) stage_w(w1ns, w1n, BR * C);
    const int row = lane & 15, kb = lane >> 4;
    bf16x8 bw2[9], bw3[2], bw1n[1] = {};
    {
        float *w2s = reinterpret_cast<float *>(smem), *w3s = w2s + NW2;  // scratch over the halo image
        static_assert(T::LINES * 2 >= (NW2 + C * BR) * 4, "weights fit the halo image");
        stage_w(w2s, w2, NW2);
        stage_w(w3s, w3, C * BR);
        __syncthreads();
        if constexpr (CHAIN) {  // the next block's W1 as B[k = c][n = o] (k >= 18, n >= 9 zero)
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = 8 * kb + j;
                v[j] = (c < C && row < BR) ? w1ns[row * C + c] : 0.f;
            }
            bw1n[0] = pack8(v);
        }
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) bw2[kk] = w2_frag<false>(w2s, kk, lane);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {  // W3 as B[k = o][n = co]
            float v[8];
            const int co = 16 * nt + row;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int o = 8 * kb + j;
                v[j] = (o < BR && co < C) ? w3s[co * BR + o] : 0.f;
            }
            bw3[nt] = pack8(v);
        }
        __syncthreads();
    }
    {
        bf16_t *tails[3] = {t3s, xs, u1s};
        const int at[3] = {T::TV * BR, T::TV * C, T::TV * C};
        zero_pads<TH, TW>(t2l, 1, tails, at, CHAIN ? 3 : 2);
    }
    const Scal s = load_scal(p);
    Scal sn{};
    if constexpr (CHAIN) sn = load_scal(pn);
    // the next tile's loads are in flight while the current tile computes
    LinesLd<TH, TW> lt;
    TileLd<TH, TW, C> lx;
    const TileSched sc = xcd_sched(a.ntiles);
    if (sc.t < sc.end) {
        const Org o0 = tile_org(a, sc.t, TH, TW);
        lt.load(a, o0, t2);
        lx.load(a, o0, x);
    }
    for (int tile = sc.t; tile < sc.end; tile += sc.step) {
        const Org o = tile_org(a, tile, TH, TW);
        __syncthreads();
        if constexpr (!(PM_EXP & 8)) {
            lt.store(t2l);
            lx.store(xs);
            if (tile + sc.step < sc.end) {
                const Org on = tile_org(a, tile + sc.step, TH, TW);
                lt.load(a, on, t2);
                lx.load(a, on, x);
            }
        }
        __syncthreads();
        // t3 = elu(W2 (*) t2 + b3a) + b3b: 16-voxel x 9-channel tiles, 9 windowed k-steps
        for (int mt = (PM_EXP & 1) ? T::NMT : wave; mt < T::NMT; mt += NT / 64) {
            const int vt = mt * 16 + row, r = vt >> 3, d = vt & 7;
            const int base = ((r / TW) * T::LW + r % TW) * LSP + LOFF + 9 * d + 8 * kb;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 9; ++kk)
                acc = mfma(read8(t2l, base + ((kk / 3) * T::LW + kk % 3) * LSP), bw2[kk], acc);
            if (row < BR) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    t3s[(mt * 16 + 4 * kb + j) * BR + row] = f2bf(elu(acc[j] + s.b3a) + s.b3b);
            }
        }
        __syncthreads();
        // out = scale * W3 t3 + b4 + x (in place over x); CHAIN: the wave also forms the next block's
        // u1 = bf16(elu(out + b1a) + b1b) of its 16 voxels (k_pm_t2's rounding points) and, reading
        // them back as the A fragment (its own LDS writes, in order: no barrier), the next block's
        // t2 = elu(W1 u1 + b2a) + b2b into the free halo image
        for (int mt = (PM_EXP & 2) ? T::NMT : wave; mt < T::NMT; mt += NT / 64) {
            const bf16x8 af = read8(t3s, (mt * 16 + row) * BR + 8 * kb);
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const f32x4 acc = mfma(af, bw3[nt], f32x4{0.f, 0.f, 0.f, 0.f});
                const int co = 16 * nt + row;
                if (co < C) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int xi = (mt * 16 + 4 * kb + j) * C + co;
                        const bf16_t ob = f2bf(acc[j] * s.sc + s.b4 + bf(xs[xi]));
                        xs[xi] = ob;
                        if constexpr (CHAIN) u1s[xi] = f2bf(elu(bf(ob) + sn.b1a) + sn.b1b);
                    }
                }
            }
            if constexpr (CHAIN && !(PM_EXP & 512)) {
                // K entries 18..31 are the next voxel's channels and meet zero weights, but they must
                // be finite: for row 15 they lie in the NEXT m-tile, which another wave may not have
                // written yet (on a workgroup's first tile: whatever the previous kernel left in LDS,
                // where a NaN bit pattern times the zero weight poisoned the next block's t2)
                uint4 q = kb == 3 ? uint4{0u, 0u, 0u, 0u}
                                  : __builtin_bit_cast(uint4, read8(u1s, (mt * 16 + row) * C + 8 * kb));
                if (kb == 2) q.y = q.z = q.w = 0u;
                const f32x4 acc = mfma(__builtin_bit_cast(bf16x8, q), bw1n[0], f32x4{0.f, 0.f, 0.f, 0.f});
                if (row < BR) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        t2l[(mt * 16 + 4 * kb + j) * BR + row] = f2bf(elu(acc[j] + sn.b2a) + sn.b2b);
                }
            }
        }
        __syncthreads();
        if constexpr (!(PM_EXP & 4)) {
            if (t3o) store_tile<TH, TW, BR>(a, o, t3s, t3o);
            store_tile<TH, TW, C>(a, o, xs, out);
        }
        if constexpr (CHAIN) store_tile<TH, TW, BR>(a, o, t2l, t2n);
    }
}

// ============================================================================================ backward
// K1: gz3 = bf16(scale * W3^T g * elu'(t3 - b3b)) and the sums of g (b4), of scale W3^T g (b3b),
// of gz3 (b3a) and of g . (W3 t3) (scale).  Blocks of 256 voxels; the next block's loads are in
// flight during the current one.  (The W3 gradient, sum t3 (x) g, is k_pm_w13grad's.)
__global__ __launch_bounds__(NT) void k_pm_bwd1(int64_t nvox, const bf16_t *__restrict__ g,
                                                const bf16_t *__restrict__ t3, const float *__restrict__ w3,
                                                vq3d_preact_params p, bf16_t *__restrict__ gz3o,
                                                float *__restrict__ part) {
    __shared__ float w3s[C * BR];
    __shared__ __attribute__((aligned(16))) bf16_t gs[NT * C];
    __shared__ __attribute__((aligned(16))) bf16_t ts[NT * BR];
    __shared__ __attribute__((aligned(16))) bf16_t zs[NT * BR];
    __shared__ float red[32];
    constexpr int NG = NT * C / 8, NTT = NT * BR / 8, PG = (NG + NT - 1) / NT, PT = (NTT + NT - 1) / NT;
    const int tid = threadIdx.x;
    // W3 rounded to bf16: the operand the chained stage of k_pm_bwd2 feeds the matrix cores
    for (int i = tid; i < C * BR; i += NT) w3s[i] = bf(f2bf(w3[i]));
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
                zs[tid * BR + o] = f2bf(z);
            }
        }
        __syncthreads();
        constexpr int NO = NT * BR / 8;
        for (int i = tid; i < NO; i += NT)
            reinterpret_cast<uint4 *>(gz3o + v0 * BR)[i] = reinterpret_cast<const uint4 *>(zs)[i];
    }
    float *dst = part + int64_t(blockIdx.x) * NE1;
    const float t4 = block_sum<float, NT>(s4, red);
    const float t3b = block_sum<float, NT>(s3b, red + 8);
    const float t3a = block_sum<float, NT>(s3a, red + 16);
    const float tsc = block_sum<float, NT>(ssc, red + 24);
    if (tid == 0) {
        dst[0] = t4;
        dst[1] = t3b;
        dst[2] = t3a;
        dst[3] = tsc;
    }
}

// K2: per TH x TW x 8 tile: gt2 = W2^T (*) gz3 (flipped taps) -> gz1 = bf16(gt2 * elu'(t2)) ->
// gx = g + (W1^T gz1) * elu'(x + b1a); gz1 to the workspace (k_pm_w13grad) and the b2 / b1 sums
// CHAIN (the chained backward of a run of blocks): the PREVIOUS block's K1 -- its gz3 and its four
// scalar partials, k_pm_bwd1's arithmetic -- from this tile's gx while it is still in LDS (gx is
// that block's g) and the previous block's t3, instead of a k_pm_bwd1 launch re-reading gx.
template <int TH, int TW, bool CHAIN>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(PM_BWD_WPE))) void k_pm_bwd2(PmArgs a, const bf16_t *__restrict__ gz3, const bf16_t *__restrict__ t2,
                                                const bf16_t *__restrict__ x, const bf16_t *__restrict__ g,
                                                const float *__restrict__ w1, const float *__restrict__ w2,
                                                vq3d_preact_params p, bf16_t *__restrict__ gx,
                                                bf16_t *__restrict__ gz1o, float *__restrict__ part,
                                                const bf16_t *__restrict__ t3p, const float *__restrict__ w3p,
                                                vq3d_preact_params pp, bf16_t *__restrict__ gz3p,
                                                float *__restrict__ part1p) {
    using T = Tile<TH, TW>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t *zl = reinterpret_cast<bf16_t *>(smem);  // gz3 halo lines; CHAIN: then the previous gz3 [TV][9]
    bf16_t *t2s = zl + T::LINES;                      // t2 of the tile [TV][9] (only elu'(t2) is needed)
    bf16_t *z1s = t2s + T::S9;                        // gz1 [TV][9]
    bf16_t *xs = z1s + T::S9;                         // x [TV][18]
    bf16_t *gs = xs + T::S18;                         // g [TV][18], then gx in place
    float *w1s = reinterpret_cast<float *>(gs + T::S18);  // W1 [o][c]
    float *red = w1s + BR * C;                            // [32] block sums
    float *w3ps = red + 32;                               // CHAIN: previous W3 [co][o]
    bf16_t *t3ps = reinterpret_cast<bf16_t *>(w3ps + C * BR);  // CHAIN: previous t3 [TV][9]
    static_assert(T::LINES >= T::TV * BR, "previous gz3 fits the halo image");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row = lane & 15, kb = lane >> 4;
    if constexpr (CHAIN) stage_w(w3ps, w3p, C * BR);
    bf16x8 bw2[9], bw1[2], bw3p = {};
    {
        float *w2s = reinterpret_cast<float *>(smem);  // scratch over the halo image
        static_assert(T::LINES * 2 >= NW2 * 4, "W2 fits the halo image");
        stage_w(w2s, w2, NW2);
        stage_w(w1s, w1, BR * C);
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) bw2[kk] = w2_frag<true>(w2s, kk, lane);
        // W1^T for gt1 = W1^T gz1 (B[k = o][n = c], two 16-channel n-tiles) and, chained, the
        // previous block's W3^T for its gz3 (B[k = co][n = o]); k >= 9 / 18 rows are zero
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int o = 8 * kb + j, c = 16 * nt + row;
                v[j] = (o < BR && c < C) ? w1s[o * C + c] : 0.f;
            }
            bw1[nt] = pack8(v);
        }
        if constexpr (CHAIN) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int co = 8 * kb + j;
                v[j] = (co < C && row < BR) ? w3ps[co * BR + row] : 0.f;
            }
            bw3p = pack8(v);
        }
        __syncthreads();
    }
    {
        bf16_t *tails[3] = {z1s, xs, gs};
        const int at[3] = {T::TV * BR, T::TV * C, T::TV * C};
        zero_pads<TH, TW>(zl, 1, tails, at, 3);
    }
    const Scal s = load_scal(p);
    float s2b = 0.f, s2a = 0.f, s1b = 0.f, s1a = 0.f;
    Scal sp{};
    if constexpr (CHAIN) sp = load_scal(pp);
    float q4 = 0.f, q3b = 0.f, q3a = 0.f, qsc = 0.f;  // CHAIN: the previous block's K1 sums
    // the next tile's gz3 halo and t2 loads are in flight while the current tile computes
    LinesLd<TH, TW> lz;
    TileLd<TH, TW, BR> lt;
    const TileSched sc = xcd_sched(a.ntiles);
    if (sc.t < sc.end) {
        const Org o0 = tile_org(a, sc.t, TH, TW);
        lz.load(a, o0, gz3);
        lt.load(a, o0, t2);
    }
    for (int tile = sc.t; tile < sc.end; tile += sc.step) {
        const Org o = tile_org(a, tile, TH, TW);
        __syncthreads();
        if constexpr (!(PM_EXP & 16)) {
            TileLd<TH, TW, C> lx, lg;
            TileLd<TH, TW, BR> l3;
            lx.load(a, o, x);
            lg.load(a, o, g);
            if constexpr (CHAIN) l3.load(a, o, t3p);
            lz.store(zl);
            lt.store(t2s);
            if (tile + sc.step < sc.end) {
                const Org on = tile_org(a, tile + sc.step, TH, TW);
                lz.load(a, on, gz3);
                lt.load(a, on, t2);
            }
            lx.store(xs);
            lg.store(gs);
            if constexpr (CHAIN) l3.store(t3ps);
        }
        __syncthreads();
        for (int mt = (PM_EXP & 32) ? T::NMT : wave; mt < T::NMT; mt += NT / 64) {
            const int vt = mt * 16 + row, r = vt >> 3, d = vt & 7;
            const int base = ((r / TW) * T::LW + r % TW) * LSP + LOFF + 9 * d + 8 * kb;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 9; ++kk)
                acc = mfma(read8(zl, base + ((kk / 3) * T::LW + kk % 3) * LSP), bw2[kk], acc);
            if (row < BR) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int v = mt * 16 + 4 * kb + j;
                    const float t2v = bf(t2s[v * BR + row]);
                    const float z1 = acc[j] * elu_d_act(t2v, s.b2b);
                    s2b += acc[j];
                    s2a += z1;
                    z1s[v * BR + row] = f2bf(z1);
                }
            }
        }
        __syncthreads();
        // gx = g + (W1^T gz1) * elu'(x + b1a): gt1 on the matrix cores (16 voxels x 2 16-channel
        // tiles per wave step, K = the 9 branch channels), the epilogue per (voxel, channel) lane
        for (int mt = (PM_EXP & 64) ? T::NMT : wave; mt < T::NMT; mt += NT / 64) {
            const bf16x8 af = read8(z1s, (mt * 16 + row) * BR + 8 * kb);
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const f32x4 acc = mfma(af, bw1[nt], f32x4{0.f, 0.f, 0.f, 0.f});
                const int c = 16 * nt + row;
                if (c < C) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = (mt * 16 + 4 * kb + j) * C + c;
                        const float gt1 = acc[j];
                        const float zx = bf(xs[i]) + s.b1a;
                        const float ez = zx > 0.f ? 1.f : expf(zx);
                        s1b += gt1;
                        s1a += gt1 * ez;
                        const bf16_t gb = f2bf(bf(gs[i]) + gt1 * ez);
                        gs[i] = gb;
                        if constexpr (CHAIN) q4 += bf(gb);  // the previous block's g = this gx
                    }
                }
            }
        }
        __syncthreads();
        if constexpr (CHAIN) {
            // previous block: gz3 = bf16(scale W3^T gx * elu'(t3)) into the free halo image (one
            // MFMA per 16 voxels, K = the 18 channels of gx)
            for (int mt = (PM_EXP & 128) ? T::NMT : wave; mt < T::NMT; mt += NT / 64) {
                const f32x4 acc = mfma(read8(gs, (mt * 16 + row) * C + 8 * kb), bw3p, f32x4{0.f, 0.f, 0.f, 0.f});
                if (row < BR) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int v = mt * 16 + 4 * kb + j;
                        const float a3 = acc[j], tv = bf(t3ps[v * BR + row]);
                        const float gt3 = a3 * sp.sc;
                        const float z = gt3 * elu_d_act(tv, sp.b3b);
                        q3b += gt3;
                        q3a += z;
                        qsc = fmaf(a3, tv, qsc);
                        zl[v * BR + row] = f2bf(z);
                    }
                }
            }
        }
        if constexpr (!(PM_EXP & 256)) {
            store_tile<TH, TW, C>(a, o, gs, gx);
            store_tile<TH, TW, BR>(a, o, z1s, gz1o);
        }
        if constexpr (CHAIN) {
            __syncthreads();
            if constexpr (!(PM_EXP & 256)) store_tile<TH, TW, BR>(a, o, zl, gz3p);
        }
    }
    if constexpr (CHAIN) {
        float *dp = part1p + int64_t(blockIdx.x) * NE1;
        const float t4 = block_sum<float, NT>(q4, red);
        const float t3b = block_sum<float, NT>(q3b, red + 8);
        const float t3a = block_sum<float, NT>(q3a, red + 16);
        const float tsc = block_sum<float, NT>(qsc, red + 24);
        if (tid == 0) {
            dp[0] = t4;
            dp[1] = t3b;
            dp[2] = t3a;
            dp[3] = tsc;
        }
    }
    float *dst = part + int64_t(blockIdx.x) * NE2;
    const float t2b = block_sum<float, NT>(s2b, red);
    const float t2a = block_sum<float, NT>(s2a, red + 8);
    const float t1b = block_sum<float, NT>(s1b, red + 16);
    const float t1a = block_sum<float, NT>(s1a, red + 24);
    if (tid == 0) {
        dst[0] = t2b;
        dst[1] = t2a;
        dst[2] = t1b;
        dst[3] = t1a;
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
// Chunks of one workgroup are consecutive and each XCD takes a contiguous eighth of them (the
// halo re-reads hit that XCD's L2).
constexpr int NT9 = 9 * 64;
template <int D>
struct W2c {
    static constexpr int NL = CHV / D;  // lines per chunk
    static constexpr int TH = NL >= 64 ? 8 : NL >= 16 ? 4 : NL >= 4 ? 2 : 1, TW = NL / TH;
    static constexpr int LW = TW + 2, HL = (TH + 2) * LW;  // halo lines
    static constexpr int RPD = D + 2;                       // positions -1 .. D
    static constexpr int CSTR = HL * RPD + 8;               // per channel (read8 reads one dword past)
    static constexpr int QL = D * BR / 8;                   // 16-B pieces of one 9-channel line
    static constexpr int ZQ = NL * QL, TQ = HL * QL;
    static constexpr int PZ = (ZQ + NT9 - 1) / NT9, PT = (TQ + NT9 - 1) / NT9;
    static constexpr size_t LDS = size_t(16 * ZP + BR * CSTR) * 2;
    static_assert(NL * D == CHV && TH * TW == NL, "chunk");
};

__device__ __forceinline__ void scatter9(bf16_t *dst, int pitch, int e0, u32x4 q, int base) {
    // the 8 elements e0 .. e0 + 7 of a 9-channel voxel-major run to dst[c * pitch + base + pos]
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int e = e0 + j, pos = e / BR, c = e - pos * BR;
        dst[c * pitch + base + pos] = bf16_t((w[j >> 1] >> ((j & 1) * 16)) & 0xffffu);
    }
}

template <int D>
__global__ __launch_bounds__(NT9) void k_pm_w2grad(PmArgs a, int nchunk, int npc, const bf16_t *__restrict__ gz3,
                                                   const bf16_t *__restrict__ t2, float *__restrict__ p2a) {
    using K = W2c<D>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t *zT = reinterpret_cast<bf16_t *>(smem);  // gz3 [16][ZP] channel-major (rows >= 9 never read into results)
    bf16_t *tT = zT + 16 * ZP;                      // t2 [9][HL][RPD] (+ tail)
    const int tid = threadIdx.x, lane = tid & 63, kk = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int kh = kk / 3, kw = kk - 3 * kh;
    const int nth = a.H / K::TH, ntw = a.W / K::TW;
    // workgroup -> chunk range (XCD-aware when the grid is a multiple of 8)
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int slot = (nwg & 7) ? bid : (bid & 7) * (nwg >> 3) + (bid >> 3);
    const int c0 = slot * npc;
    for (int i = tid; i < BR * 8; i += NT9) tT[(i >> 3) * K::CSTR + K::HL * K::RPD + (i & 7)] = 0;
    int toff[2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int e = min(16 * n + row, 26), kd = e / BR, ci = e - kd * BR;
        toff[n] = ci * K::CSTR + kd;
    }
    u32x4 vz[K::PZ], vt[K::PT];
    auto load = [&](int c) {
        const int tw_i = c % ntw, r = c / ntw, th_i = r % nth, b = r / nth;
        const int h0 = th_i * K::TH, w0 = tw_i * K::TW;
#pragma unroll
        for (int u = 0; u < K::PZ; ++u) {
            const int i = min(tid + u * NT9, K::ZQ - 1), l = i / K::QL, part = i - l * K::QL;
            const int64_t lv = ((int64_t(b) * a.H + h0 + l / K::TW) * a.W + w0 + l % K::TW) * D;
            vz[u] = reinterpret_cast<const u32x4 *>(gz3 + lv * BR)[part];
        }
#pragma unroll
        for (int u = 0; u < K::PT; ++u) {
            const int i = min(tid + u * NT9, K::TQ - 1), hl = i / K::QL, part = i - hl * K::QL;
            const int lh = hl / K::LW, lw = hl - lh * K::LW;
            const int64_t lv = ((int64_t(b) * a.H + wrapm(h0 - 1 + lh, a.H)) * a.W + wrapm(w0 - 1 + lw, a.W)) * D;
            vt[u] = reinterpret_cast<const u32x4 *>(t2 + lv * BR)[part];
        }
    };
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int cend = min(c0 + npc, nchunk);
    if (c0 < cend) load(c0);
#pragma unroll 1
    for (int c = c0; c < cend; ++c) {
        __syncthreads();  // the previous chunk's fragments are read
#pragma unroll
        for (int u = 0; u < K::PZ; ++u) {
            const int i = tid + u * NT9;
            if (i < K::ZQ) {
                const int l = i / K::QL, part = i - l * K::QL;
                scatter9(zT, ZP, part * 8, vz[u], l * D);
            }
        }
#pragma unroll
        for (int u = 0; u < K::PT; ++u) {
            const int i = tid + u * NT9;
            if (i < K::TQ) {
                const int hl = i / K::QL, part = i - hl * K::QL;
                const uint32_t w[4] = {vt[u].x, vt[u].y, vt[u].z, vt[u].w};
                bf16_t *ln = tT + hl * K::RPD;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int e = part * 8 + j, pos = e / BR, ci = e - pos * BR;
                    const bf16_t v = bf16_t((w[j >> 1] >> ((j & 1) * 16)) & 0xffffu);
                    ln[ci * K::CSTR + pos + 1] = v;
                    if (pos == 0) ln[ci * K::CSTR + D + 1] = v;  // position D wraps to 0
                    if (pos == D - 1) ln[ci * K::CSTR] = v;      // position -1 wraps to D - 1
                }
            }
        }
        __syncthreads();
        if (c + 1 < cend) load(c + 1);
#pragma unroll 4
        for (int ks = 0; ks < CHV / 32; ++ks) {
            const int v = 32 * ks + 8 * kb, l = v / D, d0 = v - l * D;
            const int hl = (l / K::TW + kh) * K::LW + l % K::TW + kw;
            const bf16x8 af = *reinterpret_cast<const bf16x8 *>(zT + row * ZP + v);
            const int off = hl * K::RPD + d0;
#pragma unroll
            for (int n = 0; n < 2; ++n) acc[n] = mfma(af, read8(tT, toff[n] + off), acc[n]);
        }
    }
    float *dst = p2a + (int64_t(bid) * 9 + kk) * NER;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * kb + j, col = 16 * n + row;
            if (co < BR && col < 27) dst[co * 27 + col] = acc[n][j];
        }
}

// k_pm_w13grad: W1 (sum gz1 (x) u1, u1 = bf16(elu(x + b1a) + b1b)) and G3 (sum t3 (x) g) over npb
// pieces of SUBV voxels per workgroup (the next piece's loads in flight); wave w: (W1 | G3,
// 16-column tile)
__global__ __launch_bounds__(NT) void k_pm_w13grad(int npb, const bf16_t *__restrict__ gz1,
                                                   const bf16_t *__restrict__ t3, const bf16_t *__restrict__ x,
                                                   const bf16_t *__restrict__ g, vq3d_preact_params p,
                                                   float *__restrict__ p2b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int ch = blockIdx.x;
    const Scal s = load_scal(p);
    bf16_t *z1T = reinterpret_cast<bf16_t *>(smem);  // [16][SP] gz1
    bf16_t *t3T = z1T + 16 * SP;                     // [16][SP] t3
    bf16_t *u1T = t3T + 16 * SP;                     // [32][SP] u1
    bf16_t *gT = u1T + 32 * SP;                      // [32][SP] g
    const int isG3 = wave >> 1, nt = wave & 1;
    const bf16_t *aT = isG3 ? t3T : z1T, *bT = isG3 ? gT : u1T;
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
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    load(int64_t(ch) * npb * SUBV);
#pragma unroll 1
    for (int pc = 0; pc < npb; ++pc) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PQ; ++u) {
            const int i = tid + u * NT;
            if (i < NQ) {
                const uint32_t w[4] = {vq[u].x, vq[u].y, vq[u].z, vq[u].w};
                if (i < 2 * N9) {
                    bf16_t *dT = i < N9 ? z1T : t3T;
                    const int e0 = (i < N9 ? i : i - N9) * 8;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int e = e0 + j, v = e / BR, c = e - v * BR;
                        dT[c * SP + v] = bf16_t((w[j >> 1] >> ((j & 1) * 16)) & 0xffffu);
                    }
                } else {
                    const bool isx = i < 2 * N9 + N18;
                    bf16_t *dT = isx ? u1T : gT;
                    const int e0 = (isx ? i - 2 * N9 : i - 2 * N9 - N18) * 8;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int e = e0 + j, v = e / C, c = e - v * C;
                        uint32_t h = (w[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
                        if (isx) h = f2bf(elu(bf(h) + s.b1a) + s.b1b);
                        dT[c * SP + v] = bf16_t(h);
                    }
                }
            }
        }
        __syncthreads();
        if (pc + 1 < npb) load((int64_t(ch) * npb + pc + 1) * SUBV);
#pragma unroll
        for (int ks = 0; ks < SUBV / 32; ++ks) {
            const int ko = 32 * ks + 8 * kb;
            acc = mfma(*reinterpret_cast<const bf16x8 *>(aT + row * SP + ko),
                       *reinterpret_cast<const bf16x8 *>(bT + (16 * nt + row) * SP + ko), acc);
        }
    }
    float *dst = p2b + int64_t(ch) * NEB + isG3 * BR * C;
    const int c = 16 * nt + row;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int oo = 4 * kb + j;
        if (oo < BR && c < C) dst[oo * C + c] = acc[j];
    }
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
constexpr int FTH = 4, FTW = 8;  // forward tile 4 x 8 x 8 (256 voxels)
constexpr int BTH = 4, BTW = 8;  // backward tile

template <int TH, int TW, bool CHAIN>
size_t fwd_lds() {
    using T = Tile<TH, TW>;
    return size_t(T::LINES + T::S9 + T::S18) * 2 + (CHAIN ? size_t(BR * C) * 4 + size_t(T::S18) * 2 : 0);
}
template <int TH, int TW, bool CHAIN>
size_t bwd_lds() {
    using T = Tile<TH, TW>;
    return size_t(T::LINES + 2 * T::S9 + 2 * T::S18) * 2 + size_t(BR * C + 32) * 4 +
           (CHAIN ? size_t(C * BR) * 4 + size_t(T::S9) * 2 : 0);
}

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
int resident(K kern, size_t lds) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, NT, lds) != hipSuccess || per < 1) per = 1;
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
int per_cu(K kern, size_t lds) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(lds));
    return resident(kern, lds);
}
// K2 grid: both variants must give the same count (the chained variant writes the previous
// block's K1 partial rows, whose count the reduction assumes to be the K2 grid)
int bwd2_blocks(const PmArgs &a) {
    static int per = 0;
    if (!per)
        per = std::min(per_cu(k_pm_bwd2<BTH, BTW, false>, bwd_lds<BTH, BTW, false>()),
                       per_cu(k_pm_bwd2<BTH, BTW, true>, bwd_lds<BTH, BTW, true>()));
    if (PM_BWD_PER > 0) per = std::min(per, PM_BWD_PER);
    return std::max(1, std::min(a.ntiles, per * n_cu()));
}

// k_pm_w13grad LDS: z1T, t3T [16][SP] + u1T, gT [32][SP]
constexpr size_t w13_lds() { return size_t(96 * SP) * 2; }

template <int D>
void launch_w2(const PmArgs &a, int nwa, int npc, const bf16_t *gz3, const bf16_t *t2, float *p2a, hipStream_t s) {
    static bool init = false;
    if (!init) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pm_w2grad<D>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(W2c<D>::LDS));
        init = true;
    }
    k_pm_w2grad<D><<<nwa, NT9, W2c<D>::LDS, s>>>(a, int(int64_t(a.B) * a.H * a.W * a.D / CHV), npc, gz3, t2, p2a);
}

void launch_fwd(int batch, int h, int w, int dd, const void *x, const float *w2, const float *w3,
                const vq3d_preact_params &p, void *out, const void *t2, void *t3, const float *w1n,
                const vq3d_preact_params *pn, void *t2n, hipStream_t s) {
    const PmArgs a = make_args(batch, h, w, dd, FTH, FTW);
    static int per = 0;
    if (!per)
        per = std::min(per_cu(k_pm_fwd<FTH, FTW, false>, fwd_lds<FTH, FTW, false>()),
                       per_cu(k_pm_fwd<FTH, FTW, true>, fwd_lds<FTH, FTW, true>()));
    if (PM_FWD_PER > 0) per = std::min(per, PM_FWD_PER);
    const unsigned g2 = unsigned(std::max(1, std::min(a.ntiles, per * n_cu())));
    if (w1n)
        k_pm_fwd<FTH, FTW, true><<<g2, NT, fwd_lds<FTH, FTW, true>(), s>>>(
            a, (const bf16_t *)t2, (const bf16_t *)x, w2, w3, p, (bf16_t *)t3, (bf16_t *)out, w1n, *pn,
            (bf16_t *)t2n);
    else
        k_pm_fwd<FTH, FTW, false><<<g2, NT, fwd_lds<FTH, FTW, false>(), s>>>(
            a, (const bf16_t *)t2, (const bf16_t *)x, w2, w3, p, (bf16_t *)t3, (bf16_t *)out, nullptr, p, nullptr);
}

// backward workspace: K1 / K2 scalar partial rows, the W2 partials [nwa][9][NER], the W1 / G3
// partials [nchb][NEB], then gz3 and gz1 (bf16 [nvox][9] each, 256-B aligned)
struct MidWs {
    float *p1, *p2, *p2a, *p2b;
    bf16_t *gz3, *gz1;
    int n1, n2, nwa, nchb, npc, npb;
    size_t bytes;
};
constexpr int kW2Chunks = 2;  // 512-voxel chunks per k_pm_w2grad workgroup (when they divide)
constexpr int kW13Pieces = 4;  // SUBV-voxel pieces per k_pm_w13grad workgroup (when they divide)

MidWs mid_ws(int B, int H, int W, int D, void *base) {
    MidWs m;
    const int64_t nvox = int64_t(B) * H * W * D;  // a multiple of 512 (H, W, D % 8 == 0)
    const PmArgs a = make_args(B, H, W, D, BTH, BTW);
    m.n2 = bwd2_blocks(a);
    m.n1 = m.n2;  // K1 rows: k_pm_bwd1's grid, or the next block's chained K2 grid
    m.npc = kW2Chunks;
    while ((nvox / CHV) % m.npc) m.npc >>= 1;
    m.npb = kW13Pieces;
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
    m.gz3 = reinterpret_cast<bf16_t *>(c + oz3);
    m.gz1 = reinterpret_cast<bf16_t *>(c + oz1);
    return m;
}

}  // namespace

// The W2-gradient kernel as the weight gradient of a plain 9 -> 9 3x3x3 circular conv (the up
// blocks' branch conv2 on the upsampled t2 at 256^2 x 64): dW[co][ci][tap] = sum_v g[v][co]
// x[v + tap][ci] is exactly k_pm_w2grad's gz3 (x) t2 window sum; its partials are summed by the
// W2 section of k_pm_reduce (fixed order, deterministic) straight into dw.
bool mid_w2grad_ok(const vq3d_conv_desc *d) {
    return d->dtype == VQ3D_BF16 && d->cin == BR && d->cin2 == 0 && d->cout == BR && d->kernel == 3 &&
           d->stride == 1 && d->pad == 1 && d->pad_mode == VQ3D_PAD_CIRCULAR && d->pro_kind == VQ3D_PRO_NONE &&
           d->in_h == d->out_h && d->in_w == d->out_w && d->in_d == d->out_d &&
           vq3d_preact_mid_supported(VQ3D_BF16, d->batch, C, BR, d->in_h, d->in_w, d->in_d);
}

namespace {
struct W2Plan {
    int nchunk, npc, nwa;
    size_t bytes;
};
W2Plan w2_plan(const vq3d_conv_desc *d) {
    W2Plan p;
    p.nchunk = int(int64_t(d->batch) * d->in_h * d->in_w * d->in_d / CHV);
    p.npc = kW2Chunks;
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
    const bf16_t *gz = static_cast<const bf16_t *>(g), *xt = static_cast<const bf16_t *>(x);
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
    // D a power of two in [8, 128]: the weight-gradient chunks are tiles of whole D-lines
    return dtype == VQ3D_BF16 && batch >= 1 && channels == C && branch == BR && h >= 8 && w >= 8 && h % 8 == 0 &&
           w % 8 == 0 && dd >= TD && dd <= 128 && (dd & (dd - 1)) == 0;
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
    if (stages & 1) k_pm_t2<<<g1, NT, 0, s>>>(nvox, (const bf16_t *)x, w1, *p, (bf16_t *)t2);
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
    if (!vq3d_preact_mid_supported(VQ3D_BF16, batch, C, BR, h, w, dd))
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
    if (stages & 1) k_pm_bwd1<<<m.n1, NT, 0, s>>>(nvox, (const bf16_t *)g, (const bf16_t *)t3, w3, *p, m.gz3, m.p1);
    if ((stages & 2) && chain)
        k_pm_bwd2<BTH, BTW, true><<<m.n2, NT, bwd_lds<BTH, BTW, true>(), s>>>(
            a, m.gz3, (const bf16_t *)t2, (const bf16_t *)x, (const bf16_t *)g, w1, w2, *p, (bf16_t *)gx, m.gz1, m.p2,
            (const bf16_t *)prev_t3, prev_w3, *prev_p, mp.gz3, mp.p1);
    else if (stages & 2)
        k_pm_bwd2<BTH, BTW, false><<<m.n2, NT, bwd_lds<BTH, BTW, false>(), s>>>(
            a, m.gz3, (const bf16_t *)t2, (const bf16_t *)x, (const bf16_t *)g, w1, w2, *p, (bf16_t *)gx, m.gz1, m.p2,
            nullptr, nullptr, *p, nullptr, nullptr);
    if (stages & 4) {
        const bf16_t *t2b = static_cast<const bf16_t *>(t2);
        switch (dd) {
            case 8: launch_w2<8>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            case 16: launch_w2<16>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            case 32: launch_w2<32>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            case 64: launch_w2<64>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
            default: launch_w2<128>(a, m.nwa, m.npc, m.gz3, t2b, m.p2a, s); break;
        }
    }
    if (stages & 8) {
        k_pm_w13grad<<<m.nchb, NT, w13_lds(), s>>>(m.npb, m.gz1, (const bf16_t *)t3, (const bf16_t *)x,
                                                   (const bf16_t *)g, *p, m.p2b);
    }
    RedOut o{G.dw1, G.dw2, G.dw3, G.dbias1a, G.dbias1b, G.dbias2a, G.dbias2b, G.dbias3a, G.dbias3b,
             G.dscale, G.dbias4, p->scale};
    if (stages & 16) k_pm_reduce<<<NBA + NBB + 1, NT, 0, s>>>(m.p1, m.n1, m.p2, m.n2, m.p2a, m.nwa, m.p2b, m.nchb, o);
    return check_launch("preact_mid_bwd");
}

}  // extern "C"
