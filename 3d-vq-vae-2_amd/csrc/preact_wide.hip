// The 72-channel / branch-36 PreActFixupResBlock (vqvae/layers.py:176-195, mode 'same', no skip
// conv): the published 3-layer model's 50 decoder post-quantize blocks at 32x32x8
// (Decoder.up[1], layers.py:395-405; 72 = embedding 8 + 64 conditioning channels).
//
//   u1  = elu(x + b1a) + b1b      t2 = elu(W1 u1 + b2a) + b2b        (1x1, 72 -> 36)
//   t3  = elu(W2 (*) t2 + b3a) + b3b                                   (3x3x3 circular, 36 -> 36)
//   out = scale * (W3 t3) + b4 + x                                     (1x1, 36 -> 72)
//
// On this grid (8192 voxels) every per-conv kernel is latency-bound, so the block runs as:
//   k_wide_pack      once per RUN of blocks: every block's W1 / W2 / W3 (and their transposed,
//                    tap-flipped backward forms) as bf16 MFMA B-fragment images, 1 KiB per
//                    fragment, lane-major, so a wave loads a fragment with one 16-B load per lane
//   k_wide_fwd       one launch per block: per 2x2x8 tile, u1 -> t2 on the tile's circular halo
//                    (matrix cores), t3 on the tile (windowed 3x3x3 on the matrix cores), out;
//                    t2 / t3 saved (bf16) for the backward
//   k_wide_bwd_data  one launch per block (the critical path): gz3 on the halo (W3^T g, matrix
//                    cores), gt2 = W2^T (*) gz3 (flipped taps), gz1, gt1 = W1^T gz1, gx; gz3 /
//                    gz1 and the 8 scalar-gradient partials to the workspace
//   k_wide_wgrad     (side stream) the W2 gradient per (tap row, 512-voxel chunk) and the W1 / W3
//                    gradients per chunk, voxels as the MFMA reduction axis (channel-major LDS
//                    copies), fixed-order partial rows
//   k_wide_reduce    (side stream) every gradient entry summed over its partial rows in a fixed
//                    order and added into the gradient buffers (deterministic)
// The residual stream (x, out, g, gx) is fp32 between the blocks of a run, as the reference's
// autocast blocks return fp32 (out * scale promotes); the matrix-core operands (u1, t2, t3, g,
// gz3, gz1, weights) are bf16, accumulation fp32.
//
// MFMA v_mfma_f32_16x16x32_bf16 layouts (lane l, row = l & 15, kb = l >> 4):
//   A: A[row][8 kb + j]   B: B[8 kb + j][row]   D: D[4 kb + j][row]   (j = 0..7 / 0..3)
// A wave owns one 16-column n-tile of the 36 branch channels and half of the m-tiles (6 waves),
// so no cross-wave sums.
#include "common.h"

#include <algorithm>


namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int C = 72, BR = 36;                         // block / branch channels
#ifndef WIDE_TW
#define WIDE_TW 2  // tile width: 2 x 2 x 8 tiles fill the chip at 32x32x8 (fwd 13.2 -> 10.3, bwd_data 16.3 -> 12.4 us vs 2 x 4 x 8)
#endif
constexpr int TH = 2, TW = WIDE_TW, TD = 8;            // tile (one D-run of 8 per (h, w))
constexpr int TV = TH * TW * TD, NMT = TV / 16;        // 32 voxels, 2 m-tiles
constexpr int MPW = NMT / 2;                           // m-tiles per wave (its half)
constexpr int LH = TH + 2, LW = TW + 2, NL = LH * LW;  // halo lines
constexpr int NP = TD + 2, HV = NL * NP, NHM = HV / 16;  // 10 positions, 240 halo voxels, 15 m-tiles
constexpr int NW = 6, NT = 64 * NW;                    // waves: (branch n-tile, half of the m-tiles)
constexpr int PADE = 32;                               // zero tail of each LDS buffer (K overrun)
static_assert(HV % 16 == 0, "halo m-tiles");

// fragment image (per block)
constexpr int KS1 = (C + 31) / 32, NTB = (BR + 15) / 16, NTC = (C + 15) / 16, KSB = (BR + 31) / 32;
constexpr int KSW = (3 * BR + 31) / 32;  // windowed k-steps per tap row (kd x 36 = 108 elements)
constexpr int OF1 = 0, OF2 = OF1 + KS1 * NTB, OF3 = OF2 + 9 * KSW * NTB, OG2 = OF3 + KSB * NTC,
              OG1 = OG2 + 9 * KSW * NTB, OG3 = OG1 + KSB * NTC, NFRAG = OG3 + KS1 * NTB;
static_assert(2 * NTB == NW && NMT % 2 == 0, "wave = (branch n-tile, m-tile half)");

// weight gradient decomposition
constexpr int CHV = 512, NRUNC = CHV / TD;  // voxels / D-runs per chunk
constexpr int ZP = CHV + 16;                // channel-major gz3 pitch (16-B rows, 8 banks apart)
constexpr int RP = 12;                      // t2 run pitch: positions -1..8 at 0..9, 2 pad
constexpr int CST = NRUNC * RP + 8;         // t2 channel pitch (4 banks apart)
constexpr int SUBV = 128, SP = SUBV + 8;    // W1 / W3 chunk and its pitch
constexpr int NE2 = BR * 3 * BR;            // W2 entries of one tap row (co x 108)
constexpr int NEB = 2 * BR * C;             // W1 [o][c] then G3 [o][co]
constexpr int NSC = 8;                      // scalar partials per tile

struct WArgs {
    int B, H, W, D;
    int nth, ntw, ntd, ntiles;
};

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }
__device__ __forceinline__ float bf(uint32_t u16) { return h2f_lo(u16); }
__device__ __forceinline__ float elu_d_act(float t, float b) {  // elu'(z) from t = elu(z) + b
    const float z1 = t - b;
    return z1 > 0.f ? 1.f : z1 + 1.f;
}
// elu with the hardware exp (v_exp_f32): every result is rounded to bf16 or feeds a bf16 operand
__device__ __forceinline__ float elu_f(float z) { return z > 0.f ? z : __expf(z) - 1.f; }
__device__ __forceinline__ f32x4 mfma(hx8 a, hx8 b, f32x4 c) {
    return VQ3D_MFMA_16X16X32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ uint32_t pk(float a, float b) { return uint32_t(f2h(a)) | (uint32_t(f2h(b)) << 16); }
// 8 bf16 from LDS, 8-byte aligned
__device__ __forceinline__ hx8 ld8(const h16_t *p) {
    const uint2 *q = reinterpret_cast<const uint2 *>(p);
    const uint2 a = q[0], b = q[1];
    return __builtin_bit_cast(hx8, uint4{a.x, a.y, b.x, b.y});
}
// 8 bf16 from LDS, 16-byte aligned
__device__ __forceinline__ hx8 ld16(const h16_t *p) { return *reinterpret_cast<const hx8 *>(p); }
// 8 consecutive bf16 at any element offset (4-byte aligned base): five dwords + v_alignbyte
__device__ __forceinline__ hx8 read8(const h16_t *base, int off) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(base + (off & ~1));
    const uint32_t sh = uint32_t(off & 1) * 2u;
    const uint32_t u0 = q[0], u1 = q[1], u2 = q[2], u3 = q[3], u4 = q[4];
    const uint4 r = {__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                     __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
    return __builtin_bit_cast(hx8, r);
}
// fragment f of a block image for this lane
__device__ __forceinline__ hx8 frag(const uint4 *__restrict__ img, int f, int lane) {
    return __builtin_bit_cast(hx8, img[f * 64 + lane]);
}
// two bf16 pairs (channels 2k, 2k+1 of voxels p and p + 1) -> the channel-major dword of channel
// 2k (lo) and 2k + 1 (hi)
__device__ __forceinline__ uint32_t tlo(uint32_t a, uint32_t b) { return (a & 0xffffu) | (b << 16); }
__device__ __forceinline__ uint32_t thi(uint32_t a, uint32_t b) { return (a >> 16) | (b & 0xffff0000u); }

struct Scal {
    float b1a, b1b, b2a, b2b, b3a, b3b, sc, b4;
};
__device__ __forceinline__ Scal load_scal(const vq3d_preact_params &p) {
    return Scal{*p.bias1a, *p.bias1b, *p.bias2a, *p.bias2b, *p.bias3a, *p.bias3b, *p.scale, *p.bias4};
}

struct Org {
    int b, h0, w0, d0;
};
__device__ __forceinline__ Org tile_org(const WArgs &a, int t) {
    Org o;
    o.d0 = (t % a.ntd) * TD;
    t /= a.ntd;
    o.w0 = (t % a.ntw) * TW;
    t /= a.ntw;
    o.h0 = (t % a.nth) * TH;
    o.b = t / a.nth;
    return o;
}
// global voxel of halo segment (line, pos) (pos 0 = position -1) and of the tile's run r
__device__ __forceinline__ int halo_vox(const WArgs &a, const Org &o, int line, int pos) {
    const int lh = line / LW, lw = line - lh * LW;
    const int gh = wrapm(o.h0 - 1 + lh, a.H), gw = wrapm(o.w0 - 1 + lw, a.W), gd = wrapm(o.d0 - 1 + pos, a.D);
    return ((o.b * a.H + gh) * a.W + gw) * a.D + gd;
}
__device__ __forceinline__ int run_vox(const WArgs &a, const Org &o, int r) {
    const int rh = r / TW, rw = r - rh * TW;
    return ((o.b * a.H + o.h0 + rh) * a.W + o.w0 + rw) * a.D + o.d0;
}
constexpr bool interior_hv(int hv) {
    const int line = hv / NP, pos = hv % NP, lh = line / LW, lw = line % LW;
    return pos >= 1 && pos <= TD && lh >= 1 && lh <= TH && lw >= 1 && lw <= TW;
}
// bit 4 m + j: halo voxel 16 m + 4 kb + j (an MFMA D row of m-tile m) is inside the tile
constexpr uint64_t interior_mask(int kb) {
    uint64_t msk = 0;
    for (int m = 0; m < NHM; ++m)
        for (int j = 0; j < 4; ++j)
            if (interior_hv(16 * m + 4 * kb + j)) msk |= uint64_t(1) << (4 * m + j);
    return msk;
}
// halo line of interior voxel v's tap row (kh, kw)
__device__ __forceinline__ int tap_line(int v, int kh, int kw) {
    const int r = v >> 3, rh = r / TW, rw = r - rh * TW;
    return (rh + kh) * LW + rw + kw;
}

// Voxel tables of the tile (LDS): segv[HV] halo segments, runv[TH * TW] tile runs.
__device__ __forceinline__ void make_tables(const WArgs &a, const Org &o, int *segv, int *runv) {
    const int tid = threadIdx.x;
    if (tid < HV) segv[tid] = halo_vox(a, o, tid / NP, tid - (tid / NP) * NP);
    if (tid < TH * TW) runv[tid] = run_vox(a, o, tid);
}

// Stage an fp32 [V][C] tensor on the tile halo into LDS as bf16 [HV][C]: u1 = elu(x + b1a) + b1b
// (ELU) or g rounded; returns the thread's sum of the interior values (fp32, unrounded) when !ELU.
// Every 16-B load is issued before any conversion.
template <bool ELU>
__device__ __forceinline__ float stage_halo_f32(const int *segv, const float *__restrict__ src, h16_t *dst, float b1a,
                                                float b1b, float *interior = nullptr) {
    constexpr int Q = C / 4, N4 = HV * Q, P = (N4 + NT - 1) / NT;
    const int tid = threadIdx.x;
    float4 v[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int i = min(tid + u * NT, N4 - 1), seg = i / Q, c4 = i - seg * Q;
        v[u] = reinterpret_cast<const float4 *>(src + int64_t(segv[seg]) * C)[c4];
    }
    float isum = 0.f;
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int i = tid + u * NT;
        if (i < N4) {
            const int seg = i / Q, c4 = i - seg * Q;
            float4 t = v[u];
            if (ELU) {
                t.x = elu_f(t.x + b1a) + b1b;
                t.y = elu_f(t.y + b1a) + b1b;
                t.z = elu_f(t.z + b1a) + b1b;
                t.w = elu_f(t.w + b1a) + b1b;
            } else {
                const int line = seg / NP, pos = seg - line * NP, lh = line / LW, lw = line - lh * LW;
                if (pos >= 1 && pos <= TD && lh >= 1 && lh <= TH && lw >= 1 && lw <= TW) {
                    isum += (t.x + t.y) + (t.z + t.w);  // and the fp32 value kept for the epilogue
                    reinterpret_cast<float4 *>(interior + (((lh - 1) * TW + lw - 1) * TD + pos - 1) * C)[c4] = t;
                }
            }
            *reinterpret_cast<uint2 *>(dst + seg * C + 4 * c4) = uint2{pk(t.x, t.y), pk(t.z, t.w)};
        }
    }
    return isum;
}

// Stage a bf16 [V][BR] tensor on the tile halo into LDS [HV][BR] (8-byte pieces, loads first)
__device__ __forceinline__ void stage_halo_br(const int *segv, const h16_t *__restrict__ src, h16_t *dst) {
    constexpr int Q = BR / 4, N = HV * Q, P = (N + NT - 1) / NT;
    const int tid = threadIdx.x;
    uint2 v[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int i = min(tid + u * NT, N - 1), seg = i / Q, q = i - seg * Q;
        v[u] = reinterpret_cast<const uint2 *>(src + int64_t(segv[seg]) * BR)[q];
    }
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int i = tid + u * NT;
        if (i < N) reinterpret_cast<uint2 *>(dst)[i] = v[u];
    }
}

// the tile's [64][BR] bf16 between LDS and global (8-byte pieces; LDS_HALO: the LDS side is the
// halo layout [HV][BR], otherwise [64][BR]); global -> LDS issues every load first
template <bool LDS_HALO>
__device__ __forceinline__ void tile_to_global(const int *runv, const h16_t *lds, h16_t *__restrict__ gl) {
    constexpr int Q = BR / 4, PR = TD * Q, N = TH * TW * PR;
    for (int i = threadIdx.x; i < N; i += NT) {
        const int r = i / PR, q = i - r * PR, rh = r / TW, rw = r - rh * TW;
        const int l0 = LDS_HALO ? (((rh + 1) * LW + rw + 1) * NP + 1) * BR : r * TD * BR;
        reinterpret_cast<uint2 *>(gl + int64_t(runv[r]) * BR)[q] = reinterpret_cast<const uint2 *>(lds + l0)[q];
    }
}
__device__ __forceinline__ void tile_from_global(const int *runv, const h16_t *__restrict__ gl, h16_t *lds) {
    constexpr int Q = BR / 4, PR = TD * Q, N = TH * TW * PR, P = (N + NT - 1) / NT;
    uint2 v[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int i = min(int(threadIdx.x) + u * NT, N - 1), r = i / PR, q = i - r * PR;
        v[u] = reinterpret_cast<const uint2 *>(gl + int64_t(runv[r]) * BR)[q];
    }
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const int i = threadIdx.x + u * NT;
        if (i < N) reinterpret_cast<uint2 *>(lds)[i] = v[u];
    }
}

// ============================================================================================ pack
// Per block (blockIdx.y), fragment blockIdx.x, lane threadIdx.x: 8 bf16 of the B operand.
__global__ __launch_bounds__(64) void k_wide_pack(const float *const *__restrict__ tab, uint4 *__restrict__ img) {
    const int f = blockIdx.x, blk = blockIdx.y, l = threadIdx.x, n = l & 15, kb = l >> 4;
    const float *w1 = tab[blk * 11 + 0], *w2 = tab[blk * 11 + 1], *w3 = tab[blk * 11 + 2];
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float x = 0.f;
        if (f < OF2) {  // t2 = W1 u1: B[c][o]
            const int s = f / NTB, nt = f - s * NTB, c = 32 * s + 8 * kb + j, o = 16 * nt + n;
            if (c < C && o < BR) x = w1[o * C + c];
        } else if (f < OF3) {  // t3 = W2 (*) t2, windowed: B[kd * 36 + ci][co]
            const int q = f - OF2, st = q / NTB, nt = q - st * NTB, kk = st / KSW, s = st - kk * KSW;
            const int e = 32 * s + 8 * kb + j, kd = e / BR, ci = e - kd * BR, co = 16 * nt + n;
            if (e < 3 * BR && co < BR) x = w2[(co * BR + ci) * 27 + kk * 3 + kd];
        } else if (f < OG2) {  // out = W3 t3: B[o][co]
            const int q = f - OF3, s = q / NTC, nt = q - s * NTC, o = 32 * s + 8 * kb + j, co = 16 * nt + n;
            if (o < BR && co < C) x = w3[co * BR + o];
        } else if (f < OG1) {  // gt2 = W2^T (*) gz3, flipped taps: B[kd' * 36 + co][ci]
            const int q = f - OG2, st = q / NTB, nt = q - st * NTB, kk = st / KSW, s = st - kk * KSW;
            const int e = 32 * s + 8 * kb + j, kd = e / BR, co = e - kd * BR, ci = 16 * nt + n;
            if (e < 3 * BR && ci < BR) x = w2[(co * BR + ci) * 27 + 26 - (kk * 3 + kd)];
        } else if (f < OG3) {  // gt1 = W1^T gz1: B[o][c]
            const int q = f - OG1, s = q / NTC, nt = q - s * NTC, o = 32 * s + 8 * kb + j, c = 16 * nt + n;
            if (o < BR && c < C) x = w1[o * C + c];
        } else {  // W3^T g: B[co][o]
            const int q = f - OG3, s = q / NTB, nt = q - s * NTB, co = 32 * s + 8 * kb + j, o = 16 * nt + n;
            if (co < C && o < BR) x = w3[co * BR + o];
        }
        v[j] = x;
    }
    img[(int64_t(blk) * NFRAG + f) * 64 + l] = uint4{pk(v[0], v[1]), pk(v[2], v[3]), pk(v[4], v[5]), pk(v[6], v[7])};
}

// ============================================================================================ forward
// Wave w: branch n-tile nt = w % 3 (channels 16 nt ..), m-tiles of parity / half hf = w / 3.
__global__ __launch_bounds__(NT) void k_wide_fwd(WArgs a, const float *__restrict__ x, const uint4 *__restrict__ img,
                                                 vq3d_preact_params p, float *__restrict__ out,
                                                 h16_t *__restrict__ t2o, h16_t *__restrict__ t3o) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *u1h = reinterpret_cast<h16_t *>(smem);  // [HV][C], then t3 [TV][BR]
    h16_t *t2h = u1h + HV * C + PADE;               // [HV][BR]
    int *segv = reinterpret_cast<int *>(t2h + HV * BR + PADE);
    int *runv = segv + HV;
    h16_t *t3s = u1h;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int nt = wave % NTB, hf = wave / NTB;
    // this wave's W1 and W2 fragments, in flight during the staging
    hx8 f1[KS1], f2[9 * KSW];
#pragma unroll
    for (int k = 0; k < KS1; ++k) f1[k] = frag(img, OF1 + k * NTB + nt, lane);
#pragma unroll
    for (int k = 0; k < 9 * KSW; ++k) f2[k] = frag(img, OF2 + k * NTB + nt, lane);
    const Org o = tile_org(a, blockIdx.x);
    const Scal s = load_scal(p);
    make_tables(a, o, segv, runv);
    for (int i = tid; i < PADE; i += NT) {
        u1h[HV * C + i] = 0;
        t2h[HV * BR + i] = 0;
    }
    __syncthreads();
    stage_halo_f32<true>(segv, x, u1h, s.b1a, s.b1b);
    __syncthreads();
    // t2 = elu(W1 u1 + b2a) + b2b on the halo
    const int ob = 16 * nt + row;
    for (int m = hf; m < NHM; m += 2) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS1; ++k) acc = mfma(ld16(u1h + (16 * m + row) * C + 32 * k + 8 * kb), f1[k], acc);
        if (ob < BR) {
#pragma unroll
            for (int j = 0; j < 4; ++j) t2h[(16 * m + 4 * kb + j) * BR + ob] = f2h(elu_f(acc[j] + s.b2a) + s.b2b);
        }
    }
    __syncthreads();
    if (t2o) tile_to_global<true>(runv, t2h, t2o);
    // x of this lane's output entries, in flight during the 3x3x3 phase: m-tiles 2 hf + mm,
    // channel tiles nt + 3 q; voxel 16 m + 4 kb + j = run 2 m + (kb >> 1), d = 4 (kb & 1) + j
    int vb[MPW];
#pragma unroll
    for (int mm = 0; mm < MPW; ++mm) vb[mm] = runv[2 * (MPW * hf + mm) + (kb >> 1)] + 4 * (kb & 1);
    float xv[2][MPW][4];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int co = min(16 * (nt + NTB * q) + row, C - 1);
#pragma unroll
        for (int mm = 0; mm < MPW; ++mm)
#pragma unroll
            for (int j = 0; j < 4; ++j) xv[q][mm][j] = x[int64_t(vb[mm] + j) * C + co];
    }
    // t3 = elu(W2 (*) t2 + b3a) + b3b on the tile
    f32x4 acc3[MPW];
#pragma unroll
    for (int mm = 0; mm < MPW; ++mm) {
        acc3[mm] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int v = 16 * (MPW * hf + mm) + row, d = v & 7;
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const h16_t *wbase = t2h + (tap_line(v, kk / 3, kk % 3) * NP + d) * BR + 8 * kb;
#pragma unroll
            for (int k = 0; k < KSW; ++k) acc3[mm] = mfma(ld8(wbase + 32 * k), f2[kk * KSW + k], acc3[mm]);
        }
    }
    __syncthreads();  // every wave is done with u1h (t3 goes over it)
    if (ob < BR) {
#pragma unroll
        for (int mm = 0; mm < MPW; ++mm)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                t3s[(16 * (MPW * hf + mm) + 4 * kb + j) * BR + ob] = f2h(elu_f(acc3[mm][j] + s.b3a) + s.b3b);
    }
    __syncthreads();
    if (t3o) tile_to_global<false>(runv, t3s, t3o);
    // out = x + scale * W3 t3 + b4
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ntc = nt + NTB * q;
        if (ntc < NTC) {
            hx8 f3[KSB];
#pragma unroll
            for (int k = 0; k < KSB; ++k) f3[k] = frag(img, OF3 + k * NTC + ntc, lane);
            const int co = 16 * ntc + row;
#pragma unroll
            for (int mm = 0; mm < MPW; ++mm) {
                const int m = MPW * hf + mm;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < KSB; ++k) acc = mfma(ld8(t3s + (16 * m + row) * BR + 32 * k + 8 * kb), f3[k], acc);
                if (co < C) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) out[int64_t(vb[mm] + j) * C + co] = xv[q][mm][j] + s.sc * acc[j] + s.b4;
                }
            }
        }
    }
}

// ============================================================================================ backward
// gx and the activation gradients of one tile; gz3 / gz1 (bf16) and 8 scalar partials out.
__global__ __launch_bounds__(NT) void k_wide_bwd_data(WArgs a, const float *__restrict__ g, const float *__restrict__ x,
                                                      const h16_t *__restrict__ t2, const h16_t *__restrict__ t3,
                                                      const uint4 *__restrict__ img, vq3d_preact_params p,
                                                      float *__restrict__ gx, h16_t *__restrict__ gz3o,
                                                      h16_t *__restrict__ gz1o, float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *gh = reinterpret_cast<h16_t *>(smem);  // g (bf16) on the halo [HV][C]
    h16_t *t3h = gh + HV * C + PADE;                // t3 on the halo [HV][BR]
    h16_t *z3h = t3h + HV * BR;                     // gz3 on the halo [HV][BR]
    h16_t *t2s = z3h + HV * BR + PADE;              // t2 on the tile [TV][BR]
    h16_t *z1s = t2s + TV * BR;                     // gz1 on the tile [TV][BR]
    float *gI = reinterpret_cast<float *>(z1s + TV * BR + PADE);  // g (fp32) on the tile [TV][C]
    float *xI = gI + TV * C;                                        // x (fp32) on the tile [TV][C]
    int *segv = reinterpret_cast<int *>(xI + TV * C);
    int *runv = segv + HV;
    float *red = reinterpret_cast<float *>(runv + TH * TW);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int nt = wave % NTB, hf = wave / NTB;
    const Org o = tile_org(a, blockIdx.x);
    const Scal s = load_scal(p);
    make_tables(a, o, segv, runv);
    for (int i = tid; i < PADE; i += NT) {
        gh[HV * C + i] = 0;
        z3h[HV * BR + i] = 0;
        z1s[TV * BR + i] = 0;
    }
    __syncthreads();
    // every staging load is issued before any LDS store: x (fp32) on the tile, t3 on the halo,
    // t2 on the tile, g (fp32) on the halo
    constexpr int QX = C / 4, NX = TV * QX, PX = (NX + NT - 1) / NT;
    constexpr int Q3 = BR / 4, N3 = HV * Q3, P3 = (N3 + NT - 1) / NT;
    constexpr int PR2 = TD * Q3, N2 = TH * TW * PR2, P2 = (N2 + NT - 1) / NT;
    constexpr int NG = HV * QX, PG = (NG + NT - 1) / NT;
    float4 vx[PX], vg[PG];
    uint2 v3[P3], v2[P2];
#pragma unroll
    for (int u = 0; u < PX; ++u) {
        const int i = min(tid + u * NT, NX - 1), vv = i / QX, c4 = i - vv * QX;
        vx[u] = reinterpret_cast<const float4 *>(x + int64_t(runv[vv >> 3] + (vv & 7)) * C)[c4];
    }
#pragma unroll
    for (int u = 0; u < P3; ++u) {
        const int i = min(tid + u * NT, N3 - 1), seg = i / Q3, q = i - seg * Q3;
        v3[u] = reinterpret_cast<const uint2 *>(t3 + int64_t(segv[seg]) * BR)[q];
    }
#pragma unroll
    for (int u = 0; u < P2; ++u) {
        const int i = min(tid + u * NT, N2 - 1), r = i / PR2, q = i - r * PR2;
        v2[u] = reinterpret_cast<const uint2 *>(t2 + int64_t(runv[r]) * BR)[q];
    }
#pragma unroll
    for (int u = 0; u < PG; ++u) {
        const int i = min(tid + u * NT, NG - 1), seg = i / QX, c4 = i - seg * QX;
        vg[u] = reinterpret_cast<const float4 *>(g + int64_t(segv[seg]) * C)[c4];
    }
    hx8 f3[KS1];
#pragma unroll
    for (int k = 0; k < KS1; ++k) f3[k] = frag(img, OG3 + k * NTB + nt, lane);
#pragma unroll
    for (int u = 0; u < PX; ++u)
        if (tid + u * NT < NX) reinterpret_cast<float4 *>(xI)[tid + u * NT] = vx[u];
#pragma unroll
    for (int u = 0; u < P3; ++u)
        if (tid + u * NT < N3) reinterpret_cast<uint2 *>(t3h)[tid + u * NT] = v3[u];
#pragma unroll
    for (int u = 0; u < P2; ++u)
        if (tid + u * NT < N2) reinterpret_cast<uint2 *>(t2s)[tid + u * NT] = v2[u];
    float s4 = 0.f;
#pragma unroll
    for (int u = 0; u < PG; ++u) {
        const int i = tid + u * NT;
        if (i < NG) {
            const int seg = i / QX, c4 = i - seg * QX;
            const float4 t = vg[u];
            const int line = seg / NP, pos = seg - line * NP, lh = line / LW, lw = line - lh * LW;
            if (pos >= 1 && pos <= TD && lh >= 1 && lh <= TH && lw >= 1 && lw <= TW) {
                s4 += (t.x + t.y) + (t.z + t.w);  // the fp32 value is kept for the gx epilogue
                reinterpret_cast<float4 *>(gI + (((lh - 1) * TW + lw - 1) * TD + pos - 1) * C)[c4] = t;
            }
            *reinterpret_cast<uint2 *>(gh + seg * C + 4 * c4) = uint2{pk(t.x, t.y), pk(t.z, t.w)};
        }
    }
    __syncthreads();
    hx8 f2[9 * KSW];
#pragma unroll
    for (int k = 0; k < 9 * KSW; ++k) f2[k] = frag(img, OG2 + k * NTB + nt, lane);
    // gz3 = bf16(scale * W3^T g * elu'(t3)) on the halo
    float s3b = 0.f, s3a = 0.f, ssc = 0.f;
    const int ob = 16 * nt + row;
    const uint64_t imsk = kb == 0 ? interior_mask(0) : kb == 1 ? interior_mask(1) : kb == 2 ? interior_mask(2)
                                                                                           : interior_mask(3);
    for (int m = hf; m < NHM; m += 2) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS1; ++k) acc = mfma(ld16(gh + (16 * m + row) * C + 32 * k + 8 * kb), f3[k], acc);
        if (ob < BR) {
            const uint32_t mj = uint32_t(imsk >> (4 * m)) & 15u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int hv = 16 * m + 4 * kb + j;
                const float t3v = bf(t3h[hv * BR + ob]), gt3 = s.sc * acc[j];
                const float z = gt3 * elu_d_act(t3v, s.b3b);
                z3h[hv * BR + ob] = f2h(z);
                if (mj & (1u << j)) {
                    s3b += gt3;
                    s3a += z;
                    ssc = fmaf(acc[j], t3v, ssc);
                }
            }
        }
    }
    __syncthreads();
    tile_to_global<true>(runv, z3h, gz3o);
    int vb[MPW];
#pragma unroll
    for (int mm = 0; mm < MPW; ++mm) vb[mm] = runv[2 * (MPW * hf + mm) + (kb >> 1)] + 4 * (kb & 1);
    // gt2 = W2^T (*) gz3 -> gz1 = bf16(gt2 * elu'(t2))
    float s2b = 0.f, s2a = 0.f;
#pragma unroll
    for (int mm = 0; mm < MPW; ++mm) {
        const int m = MPW * hf + mm;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int v = 16 * m + row, d = v & 7;
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const h16_t *wbase = z3h + (tap_line(v, kk / 3, kk % 3) * NP + d) * BR + 8 * kb;
#pragma unroll
            for (int k = 0; k < KSW; ++k) acc = mfma(ld8(wbase + 32 * k), f2[kk * KSW + k], acc);
        }
        if (ob < BR) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int vv = 16 * m + 4 * kb + j;
                const float z1 = acc[j] * elu_d_act(bf(t2s[vv * BR + ob]), s.b2b);
                s2b += acc[j];
                s2a += z1;
                z1s[vv * BR + ob] = f2h(z1);
            }
        }
    }
    __syncthreads();
    tile_to_global<false>(runv, z1s, gz1o);
    // gt1 = W1^T gz1; gx = g + gt1 * elu'(x + b1a)
    float s1b = 0.f, s1a = 0.f;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ntc = nt + NTB * q;
        if (ntc < NTC) {
            hx8 f1[KSB];
#pragma unroll
            for (int k = 0; k < KSB; ++k) f1[k] = frag(img, OG1 + k * NTC + ntc, lane);
            const int c = 16 * ntc + row;
#pragma unroll
            for (int mm = 0; mm < MPW; ++mm) {
                const int m = MPW * hf + mm;
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < KSB; ++k) acc = mfma(ld8(z1s + (16 * m + row) * BR + 32 * k + 8 * kb), f1[k], acc);
                if (c < C) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int vv = 16 * m + 4 * kb + j;
                        const float zx = xI[vv * C + c] + s.b1a, e1 = zx > 0.f ? 1.f : __expf(zx);
                        gx[int64_t(vb[mm] + j) * C + c] = gI[vv * C + c] + acc[j] * e1;
                        s1b += acc[j];
                        s1a = fmaf(acc[j], e1, s1a);
                    }
                }
            }
        }
    }
    // scalar partials: b4, b3b, b3a, scale, b2b, b2a, b1b, b1a
    // (all eight in one barrier pair: eight sequential block sums cost sixteen barriers on the
    // run's critical path)
    float sums[NSC] = {s4, s3b, s3a, ssc, s2b, s2a, s1b, s1a};
    block_sums<float, NT, NSC, 8>(sums, red);
    float *dst = part + int64_t(blockIdx.x) * NSC;
    if (tid == 0) {
#pragma unroll
        for (int k = 0; k < NSC; ++k) dst[k] = sums[k];
    }
}

// Weight gradients.  Workgroups [0, 9 * nch): the W2 gradient of tap row kk = wg / nch over
// chunk ch = wg % nch (512 voxels): dW2[co][kd * 36 + ci] += sum_v gz3[v][co] t2[v + tap][ci];
// wave (m-tile w % 3 of co, column tiles 4 (w / 3) ..).  Workgroups [9 * nch, 9 * nch + nchb):
// W1 (sum gz1 (x) u1) and G3 (sum t3 (x) g) over a 128-voxel chunk; wave (m-tile w % 3 of o,
// W1 or G3).  Voxels are the MFMA reduction axis: channel-major LDS copies.
__device__ __forceinline__ void wide_wgrad(const WArgs &a, int nch, const float *__restrict__ g,
                                           const float *__restrict__ x, const h16_t *__restrict__ t2,
                                           const h16_t *__restrict__ t3, const h16_t *__restrict__ gz3,
                                           const h16_t *__restrict__ gz1, const vq3d_preact_params &p,
                                           float *__restrict__ p2a, float *__restrict__ p2b) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int mt = wave % 3, hf = wave / 3;
    if (int(blockIdx.x) < 9 * nch) {
        const int kk = blockIdx.x / nch, ch = blockIdx.x - kk * nch, kh = kk / 3, kw = kk - 3 * kh;
        h16_t *zT = reinterpret_cast<h16_t *>(smem);  // gz3 channel-major [48][ZP]
        h16_t *tT = zT + 48 * ZP;                      // t2 shifted by the tap row, [36][CST]: [run][RP]
        int *rline = reinterpret_cast<int *>(tT + BR * CST);  // per run: source line base, d0
        int *rd0 = rline + NRUNC;
        const int v0 = ch * CHV;
        if (tid < NRUNC) {
            const int R = v0 / TD + tid, ndr = a.D / TD, dr = R % ndr, ln = R / ndr;
            const int w0 = ln % a.W, h0 = (ln / a.W) % a.H, bb = ln / (a.W * a.H);
            rline[tid] = ((bb * a.H + wrapm(h0 + kh - 1, a.H)) * a.W + wrapm(w0 + kw - 1, a.W)) * a.D;
            rd0[tid] = dr * TD;
        }
        __syncthreads();
        constexpr int Q = BR / 4;
        constexpr int NZ = (CHV / 2) * Q, PZ = (NZ + NT - 1) / NT;          // gz3 voxel pairs x quads
        constexpr int NTT = NRUNC * (NP / 2) * Q, PT = (NTT + NT - 1) / NT;  // t2 position pairs x quads
        uint2 zl[PZ], zh[PZ], tl[PT], th[PT];
#pragma unroll
        for (int u = 0; u < PZ; ++u) {
            const int i = min(tid + u * NT, NZ - 1), pr = i / Q, q = i - pr * Q;
            zl[u] = reinterpret_cast<const uint2 *>(gz3 + int64_t(v0 + 2 * pr) * BR)[q];
            zh[u] = reinterpret_cast<const uint2 *>(gz3 + int64_t(v0 + 2 * pr + 1) * BR)[q];
        }
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int i = min(tid + u * NT, NTT - 1), q = i % Q, rest = i / Q, pp = rest % (NP / 2),
                      run = rest / (NP / 2);
            const int lb = rline[run], d0 = rd0[run];
            const int da = wrapm(d0 - 1 + 2 * pp, a.D), db = wrapm(d0 + 2 * pp, a.D);
            tl[u] = reinterpret_cast<const uint2 *>(t2 + int64_t(lb + da) * BR)[q];
            th[u] = reinterpret_cast<const uint2 *>(t2 + int64_t(lb + db) * BR)[q];
        }
#pragma unroll
        for (int u = 0; u < PZ; ++u) {
            const int i = tid + u * NT;
            if (i < NZ) {
                const int pr = i / Q, q = i - pr * Q;
                uint32_t *dst = reinterpret_cast<uint32_t *>(zT + (4 * q) * ZP + 2 * pr);
                dst[0] = tlo(zl[u].x, zh[u].x);
                dst[ZP / 2] = thi(zl[u].x, zh[u].x);
                dst[ZP] = tlo(zl[u].y, zh[u].y);
                dst[3 * ZP / 2] = thi(zl[u].y, zh[u].y);
            }
        }
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int i = tid + u * NT;
            if (i < NTT) {
                const int q = i % Q, rest = i / Q, pp = rest % (NP / 2), run = rest / (NP / 2);
                uint32_t *dst = reinterpret_cast<uint32_t *>(tT + (4 * q) * CST + run * RP + 2 * pp);
                dst[0] = tlo(tl[u].x, th[u].x);
                dst[CST / 2] = thi(tl[u].x, th[u].x);
                dst[CST] = tlo(tl[u].y, th[u].y);
                dst[3 * CST / 2] = thi(tl[u].y, th[u].y);
            }
        }
        for (int i = tid; i < BR * NRUNC; i += NT) {
            const int ci = i / NRUNC, run = i - ci * NRUNC;
            reinterpret_cast<uint32_t *>(tT + ci * CST + run * RP + NP)[0] = 0u;
        }
        __syncthreads();
        constexpr int NTE = (3 * BR + 15) / 16;  // 7 column tiles of the 108-element window
        const int n0 = 4 * hf, nn = hf ? NTE - 4 : 4;
        f32x4 acc[4];
        int toff[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int e = 16 * min(n0 + n, NTE - 1) + row, kd = e / BR, ci = e - kd * BR;
            toff[n] = ci * CST + kd;
        }
#pragma unroll 2
        for (int ks = 0; ks < CHV / 32; ++ks) {
            const hx8 af = ld16(zT + (16 * mt + row) * ZP + 32 * ks + 8 * kb);
            const int roff = (4 * ks + kb) * RP;
#pragma unroll
            for (int n = 0; n < 4; ++n)
                if (n < nn) acc[n] = mfma(af, read8(tT, toff[n] + roff), acc[n]);
        }
        float *dst = p2a + (int64_t(kk) * nch + ch) * NE2;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int e = 16 * (n0 + n) + row;
            if (n < nn && e < 3 * BR) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = 16 * mt + 4 * kb + j;
                    if (co < BR) dst[co * 3 * BR + e] = acc[n][j];
                }
            }
        }
        return;
    }
    // W1 / G3 of a 128-voxel chunk
    const int ch = blockIdx.x - 9 * nch;
    const Scal s = load_scal(p);
    h16_t *z1T = reinterpret_cast<h16_t *>(smem);  // [48][SP] gz1
    h16_t *t3T = z1T + 48 * SP;                     // [48][SP] t3
    h16_t *u1T = t3T + 48 * SP;                     // [80][SP] u1
    h16_t *grT = u1T + 80 * SP;                     // [80][SP] g
    const int v0 = ch * SUBV;
    {
        constexpr int Q = BR / 4, N = 2 * (SUBV / 2) * Q, P = (N + NT - 1) / NT;
        constexpr int QC = C / 4, NC = 2 * (SUBV / 2) * QC, PC = (NC + NT - 1) / NT;
        uint2 bl[P], bh[P];
        float4 fl[PC], fh[PC];
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int i = min(tid + u * NT, N - 1), which = i / (N / 2), ii = i - which * (N / 2), pr = ii / Q,
                      q = ii - pr * Q;
            const h16_t *src = which ? t3 : gz1;
            bl[u] = reinterpret_cast<const uint2 *>(src + int64_t(v0 + 2 * pr) * BR)[q];
            bh[u] = reinterpret_cast<const uint2 *>(src + int64_t(v0 + 2 * pr + 1) * BR)[q];
        }
#pragma unroll
        for (int u = 0; u < PC; ++u) {
            const int i = min(tid + u * NT, NC - 1), which = i / (NC / 2), ii = i - which * (NC / 2), pr = ii / QC,
                      q = ii - pr * QC;
            const float *src = which ? g : x;
            fl[u] = reinterpret_cast<const float4 *>(src + int64_t(v0 + 2 * pr) * C)[q];
            fh[u] = reinterpret_cast<const float4 *>(src + int64_t(v0 + 2 * pr + 1) * C)[q];
        }
#pragma unroll
        for (int u = 0; u < P; ++u) {
            const int i = tid + u * NT;
            if (i < N) {
                const int which = i / (N / 2), ii = i - which * (N / 2), pr = ii / Q, q = ii - pr * Q;
                uint32_t *dst = reinterpret_cast<uint32_t *>((which ? t3T : z1T) + (4 * q) * SP + 2 * pr);
                dst[0] = tlo(bl[u].x, bh[u].x);
                dst[SP / 2] = thi(bl[u].x, bh[u].x);
                dst[SP] = tlo(bl[u].y, bh[u].y);
                dst[3 * SP / 2] = thi(bl[u].y, bh[u].y);
            }
        }
#pragma unroll
        for (int u = 0; u < PC; ++u) {
            const int i = tid + u * NT;
            if (i < NC) {
                const int which = i / (NC / 2), ii = i - which * (NC / 2), pr = ii / QC, q = ii - pr * QC;
                float l4[4] = {fl[u].x, fl[u].y, fl[u].z, fl[u].w}, h4[4] = {fh[u].x, fh[u].y, fh[u].z, fh[u].w};
                h16_t *dT = which ? grT : u1T;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float lv = l4[k], hv = h4[k];
                    if (!which) {
                        lv = elu_f(lv + s.b1a) + s.b1b;
                        hv = elu_f(hv + s.b1a) + s.b1b;
                    }
                    reinterpret_cast<uint32_t *>(dT + (4 * q + k) * SP + 2 * pr)[0] = pk(lv, hv);
                }
            }
        }
    }
    __syncthreads();
    // wave: o m-tile mt; hf 0: W1 [o][c] (gz1 x u1), hf 1: G3 [o][co] (t3 x g)
    const h16_t *aT = hf ? t3T : z1T, *bT = hf ? grT : u1T;
    f32x4 acc[NTC];
#pragma unroll
    for (int n = 0; n < NTC; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < SUBV / 32; ++ks) {
        const int ko = 32 * ks + 8 * kb;
        const hx8 af = ld16(aT + (16 * mt + row) * SP + ko);
#pragma unroll
        for (int n = 0; n < NTC; ++n) acc[n] = mfma(af, ld16(bT + (16 * n + row) * SP + ko), acc[n]);
    }
    float *dst = p2b + int64_t(ch) * NEB + hf * BR * C;
#pragma unroll
    for (int n = 0; n < NTC; ++n) {
        const int c = 16 * n + row;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int oo = 16 * mt + 4 * kb + j;
            if (oo < BR && c < C) dst[oo * C + c] = acc[n][j];
        }
    }
}

__global__ __launch_bounds__(NT) void k_wide_wgrad(WArgs a, int nch, const float *__restrict__ g,
                                                   const float *__restrict__ x, const h16_t *__restrict__ t2,
                                                   const h16_t *__restrict__ t3, const h16_t *__restrict__ gz3,
                                                   const h16_t *__restrict__ gz1, vq3d_preact_params p,
                                                   float *__restrict__ p2a, float *__restrict__ p2b) {
    wide_wgrad(a, nch, g, x, t2, t3, gz3, gz1, p, p2a, p2b);
}
// A whole run's weight-gradient partial rows in one launch (round 6, as preact_mid's
// k_pm_w2grad_run): grid.y = the run's blocks, their gz3 / gz1 / partial rows in their workspace
// slices, their g / x / t2 / t3 from kernel-argument tables, their scalars from the run's
// [nblocks][11] parameter table.  The same workgroups and arithmetic as k_wide_wgrad per block.
constexpr int WMAXRUN = 56;
struct WideRunPtrs {
    const float *g[WMAXRUN], *x[WMAXRUN];
    const h16_t *t2[WMAXRUN], *t3[WMAXRUN];
};
__global__ __launch_bounds__(NT) void k_wide_wgrad_run(WArgs a, int nch, const char *__restrict__ base, size_t stride,
                                                       int64_t ogz3, int64_t ogz1, int64_t op2a, int64_t op2b,
                                                       WideRunPtrs r, const float *const *__restrict__ params) {
    const int i = blockIdx.y;
    char *b = const_cast<char *>(base) + size_t(i) * stride;
    const float *const *t = params + size_t(i) * 11;
    const vq3d_preact_params p{t[3], t[4], t[5], t[6], t[7], t[8], t[9], t[10]};
    wide_wgrad(a, nch, r.g[i], r.x[i], r.t2[i], r.t3[i], reinterpret_cast<const h16_t *>(b + ogz3),
               reinterpret_cast<const h16_t *>(b + ogz1), p, reinterpret_cast<float *>(b + op2a),
               reinterpret_cast<float *>(b + op2b));
}

struct RedOut {
    float *dw1, *dw2, *dw3, *db1a, *db1b, *db2a, *db2b, *db3a, *db3b, *dscale, *db4;
    const float *scale;
};

// Every gradient entry: its partial rows summed in a fixed order, added into the gradient
// buffer.  The last workgroup sums the scalar partials of every tile.
constexpr int RNT = 256;
__device__ __forceinline__ void wide_reduce(int nch, int nchb, int ntiles, const float *__restrict__ p2a,
                                            const float *__restrict__ p2b, const float *__restrict__ p1,
                                            const RedOut &o) {
    constexpr int EA = 9 * NE2, EB = NEB;
    if (int(blockIdx.x) == int(gridDim.x) - 1) {
        __shared__ float sm[RNT];
        const int k = threadIdx.x & 7, part = threadIdx.x >> 3;
        float t = 0.f;
#pragma unroll 4
        for (int i = part; i < ntiles; i += RNT / 8) t += p1[int64_t(i) * NSC + k];
        sm[threadIdx.x] = t;
        __syncthreads();
        if (threadIdx.x < NSC) {
            float r = 0.f;
            for (int i = 0; i < RNT / 8; ++i) r += sm[i * 8 + threadIdx.x];
            float *dstp[NSC] = {o.db4, o.db3b, o.db3a, o.dscale, o.db2b, o.db2a, o.db1b, o.db1a};
            *dstp[threadIdx.x] += r;
        }
        return;
    }
    const int e = blockIdx.x * RNT + threadIdx.x;
    if (e < EA) {
        const int kk = e / NE2, rem = e - kk * NE2, co = rem / (3 * BR), el = rem - co * 3 * BR;
        const int kd = el / BR, ci = el - kd * BR;
        const float *src = p2a + int64_t(kk) * nch * NE2 + rem;
        float t = 0.f;
#pragma unroll 8
        for (int c = 0; c < nch; ++c) t += src[int64_t(c) * NE2];
        o.dw2[(co * BR + ci) * 27 + kk * 3 + kd] += t;
    } else if (e < EA + EB) {
        const int q = e - EA;
        float t = 0.f;
#pragma unroll 8
        for (int c = 0; c < nchb; ++c) t += p2b[int64_t(c) * NEB + q];
        if (q < BR * C) {
            o.dw1[q] += t;
        } else {
            const int r = q - BR * C, oo = r / C, co = r - oo * C;
            o.dw3[co * BR + oo] += *o.scale * t;
        }
    }
}
__global__ __launch_bounds__(RNT) void k_wide_reduce(int nch, int nchb, int ntiles, const float *__restrict__ p2a,
                                                     const float *__restrict__ p2b, const float *__restrict__ p1,
                                                     RedOut o) {
    wide_reduce(nch, nchb, ntiles, p2a, p2b, p1, o);
}
// a whole run of blocks (blockIdx.y = block; its workspace at base + y * stride, pointers from the
// run's [block][11] device tables)
__global__ __launch_bounds__(RNT) void k_wide_reduce_run(int nch, int nchb, int ntiles, const char *__restrict__ base,
                                                         size_t stride, int64_t oa, int64_t ob, int64_t o1,
                                                         float *const *gtab, const float *const *ptab) {
    const char *ws = base + size_t(blockIdx.y) * stride;
    float *const *g = gtab + blockIdx.y * 11;
    const RedOut o{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], ptab[blockIdx.y * 11 + 9]};
    wide_reduce(nch, nchb, ntiles, reinterpret_cast<const float *>(ws + oa), reinterpret_cast<const float *>(ws + ob),
                reinterpret_cast<const float *>(ws + o1), o);
}

// ============================================================================================ host
WArgs make_args(int B, int H, int W, int D) {
    WArgs a;
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
constexpr size_t kTables = size_t(HV + TH * TW) * 4;
constexpr size_t kFwdLds = size_t(HV * C + PADE + HV * BR + PADE) * 2 + kTables;
constexpr size_t kBwdLds =
    size_t(HV * C + PADE + 2 * HV * BR + PADE + 2 * TV * BR + PADE) * 2 + size_t(2 * TV * C) * 4 + kTables + 8 * NSC * 4;
constexpr size_t kWgLdsA = size_t(48 * ZP + BR * CST) * 2 + 2 * NRUNC * 4;
constexpr size_t kWgLdsB = size_t((48 + 48 + 80 + 80) * SP) * 2;
constexpr size_t kWgLds = kWgLdsA > kWgLdsB ? kWgLdsA : kWgLdsB;
static_assert(kFwdLds <= 160 * 1024 && kBwdLds <= 160 * 1024 && kWgLds <= 160 * 1024, "LDS");

void set_lds_limits() {
    static bool done = false;
    if (done) return;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_wide_fwd), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(kFwdLds));
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_wide_bwd_data),
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(kBwdLds));
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_wide_wgrad), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(kWgLds));
    done = true;
}

struct WsLayout {
    size_t gz3, gz1, p1, p2a, p2b, total;
};
WsLayout ws_layout(int B, int H, int W, int D) {
    const size_t nvox = size_t(B) * H * W * D, nch = nvox / CHV, nchb = nvox / SUBV, ntiles = nvox / TV;
    auto al = [](size_t n) { return (n + 255) & ~size_t(255); };
    WsLayout l;
    l.gz3 = 0;
    l.gz1 = l.gz3 + al(nvox * BR * 2);
    l.p1 = l.gz1 + al(nvox * BR * 2);
    l.p2a = l.p1 + al(ntiles * NSC * 4);
    l.p2b = l.p2a + al(9 * nch * NE2 * 4);
    l.total = l.p2b + al(nchb * NEB * 4);
    return l;
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_wide_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    return batch >= 1 && channels == C && branch == BR && h >= TH && w >= TW && dd >= TD && h % TH == 0 &&
           w % TW == 0 && dd % TD == 0 && (int64_t(batch) * h * w * dd) % CHV == 0 &&
           int64_t(batch) * h * w * dd * C < (int64_t(1) << 31);
}

size_t vq3d_preact_wide_image_bytes(int32_t channels, int32_t branch) {
    return (channels == C && branch == BR) ? size_t(NFRAG) * 64 * 16 : 0;
}

int vq3d_preact_wide_pack(int32_t dtype, int32_t nblocks, int32_t channels, int32_t branch, const float *const *params,
                          void *image, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_wide_pack: dtype must be the 16-bit format of this build");
    if (channels != C || branch != BR || nblocks < 1) return fail("preact_wide_pack: unsupported block shape");
    if (!params || !image) return fail("preact_wide_pack: null pointer");
    k_wide_pack<<<dim3(NFRAG, nblocks), 64, 0, as_stream(stream)>>>(params, static_cast<uint4 *>(image));
    return check_launch("preact_wide_pack");
}

int vq3d_preact_wide_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd,
                         const float *x, const void *image, const vq3d_preact_params *p, float *out, void *t2, void *t3,
                         vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_wide_fwd: dtype must be the 16-bit format of this build");
    if (!vq3d_preact_wide_supported(batch, channels, branch, h, w, dd))
        return fail("preact_wide_fwd: shape outside the fused wide-block kernels");
    if (!x || !image || !p || !out) return fail("preact_wide_fwd: null pointer");
    if (static_cast<const void *>(x) == static_cast<const void *>(out)) return fail("preact_wide_fwd: out aliases x");
    set_lds_limits();
    const WArgs a = make_args(batch, h, w, dd);
    k_wide_fwd<<<a.ntiles, NT, kFwdLds, as_stream(stream)>>>(a, x, static_cast<const uint4 *>(image), *p, out,
                                                             static_cast<h16_t *>(t2), static_cast<h16_t *>(t3));
    return check_launch("preact_wide_fwd");
}

size_t vq3d_preact_wide_workspace_bytes(int32_t batch, int32_t h, int32_t w, int32_t dd) {
    return ws_layout(batch, h, w, dd).total;
}

int vq3d_preact_wide_bwd_data(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd, const float *g, const float *x, const void *t2, const void *t3,
                              const void *image, const vq3d_preact_params *p, void *workspace, size_t workspace_bytes,
                              float *gx, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_wide_bwd_data: dtype must be the 16-bit format of this build");
    if (!vq3d_preact_wide_supported(batch, channels, branch, h, w, dd))
        return fail("preact_wide_bwd_data: shape outside the fused wide-block kernels");
    if (!g || !x || !t2 || !t3 || !image || !p || !workspace || !gx) return fail("preact_wide_bwd_data: null pointer");
    const WsLayout l = ws_layout(batch, h, w, dd);
    if (workspace_bytes < l.total) return fail("preact_wide_bwd_data: workspace too small");
    if (static_cast<const void *>(gx) == static_cast<const void *>(g)) return fail("preact_wide_bwd_data: gx aliases g");
    set_lds_limits();
    char *ws = static_cast<char *>(workspace);
    const WArgs a = make_args(batch, h, w, dd);
    k_wide_bwd_data<<<a.ntiles, NT, kBwdLds, as_stream(stream)>>>(
        a, g, x, static_cast<const h16_t *>(t2), static_cast<const h16_t *>(t3), static_cast<const uint4 *>(image),
        *p, gx, reinterpret_cast<h16_t *>(ws + l.gz3), reinterpret_cast<h16_t *>(ws + l.gz1),
        reinterpret_cast<float *>(ws + l.p1));
    return check_launch("preact_wide_bwd_data");
}

int vq3d_preact_wide_bwd_weight(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                                int32_t dd, const float *g, const float *x, const void *t2, const void *t3,
                                const vq3d_preact_params *p, const vq3d_preact_grads *gr, const void *workspace,
                                size_t workspace_bytes, vq3d_stream_t stream) {
    return vq3d_preact_wide_bwd_weight_stages(3, dtype, batch, channels, branch, h, w, dd, g, x, t2, t3, p, gr,
                                              workspace, workspace_bytes, stream);
}

int vq3d_preact_wide_reduce_run(int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                                const void *workspaces, size_t workspace_stride, float *const *grads,
                                const float *const *params, vq3d_stream_t stream) {
    if (!vq3d_preact_wide_supported(batch, C, BR, h, w, dd))
        return fail("preact_wide_reduce_run: shape outside the fused wide-block kernels");
    if (nblocks < 1 || nblocks > 65535 || !workspaces || !grads || !params)
        return fail("preact_wide_reduce_run: bad arguments");
    const WsLayout l = ws_layout(batch, h, w, dd);
    if (workspace_stride < l.total || workspace_stride % 256)
        return fail("preact_wide_reduce_run: stride below the workspace size or unaligned");
    const WArgs a = make_args(batch, h, w, dd);
    const int nch = int(int64_t(batch) * h * w * dd / CHV), nchb = int(int64_t(batch) * h * w * dd / SUBV);
    const int ne = 9 * NE2 + NEB;
    k_wide_reduce_run<<<dim3((ne + RNT - 1) / RNT + 1, unsigned(nblocks)), RNT, 0, as_stream(stream)>>>(
        nch, nchb, a.ntiles, static_cast<const char *>(workspaces), workspace_stride, int64_t(l.p2a), int64_t(l.p2b),
        int64_t(l.p1), grads, params);
    return check_launch("preact_wide_reduce_run");
}

int vq3d_preact_wide_wgrad_run(int32_t dtype, int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                               const float *const *g, const float *const *x, const void *const *t2,
                               const void *const *t3, const float *const *params, void *workspaces,
                               size_t workspace_stride, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_wide_wgrad_run: dtype must be the 16-bit format of this build");
    if (!vq3d_preact_wide_supported(batch, C, BR, h, w, dd))
        return fail("preact_wide_wgrad_run: shape outside the fused wide-block kernels");
    if (nblocks < 1 || nblocks > 65535 || !g || !x || !t2 || !t3 || !params || !workspaces)
        return fail("preact_wide_wgrad_run: bad arguments");
    const WsLayout l = ws_layout(batch, h, w, dd);
    if (workspace_stride < l.total || workspace_stride % 256)
        return fail("preact_wide_wgrad_run: stride below the workspace size or unaligned");
    for (int i = 0; i < nblocks; ++i)
        if (!g[i] || !x[i] || !t2[i] || !t3[i]) return fail("preact_wide_wgrad_run: null tensor pointer");
    set_lds_limits();
    static bool init = false;
    if (!init) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_wide_wgrad_run),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(kWgLds));
        init = true;
    }
    const WArgs a = make_args(batch, h, w, dd);
    const int nch = int(int64_t(batch) * h * w * dd / CHV), nchb = int(int64_t(batch) * h * w * dd / SUBV);
    const char *b0 = static_cast<const char *>(workspaces);
    for (int i0 = 0; i0 < nblocks; i0 += WMAXRUN) {
        const int nb = std::min(WMAXRUN, nblocks - i0);
        WideRunPtrs r{};
        for (int i = 0; i < nb; ++i) {
            r.g[i] = g[i0 + i];
            r.x[i] = x[i0 + i];
            r.t2[i] = static_cast<const h16_t *>(t2[i0 + i]);
            r.t3[i] = static_cast<const h16_t *>(t3[i0 + i]);
        }
        k_wide_wgrad_run<<<dim3(unsigned(9 * nch + nchb), unsigned(nb)), NT, kWgLds, as_stream(stream)>>>(
            a, nch, b0 + size_t(i0) * workspace_stride, workspace_stride, int64_t(l.gz3), int64_t(l.gz1),
            int64_t(l.p2a), int64_t(l.p2b), r, params + size_t(i0) * 11);
    }
    return check_launch("preact_wide_wgrad_run");
}

int vq3d_preact_wide_bwd_weight_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                                       int32_t h, int32_t w, int32_t dd, const float *g, const float *x, const void *t2,
                                       const void *t3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                                       const void *workspace, size_t workspace_bytes, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_wide_bwd_weight: dtype must be the 16-bit format of this build");
    if (stages < 1 || stages > 3) return fail("preact_wide_bwd_weight: stages must be a mask of 1 | 2");
    if (!vq3d_preact_wide_supported(batch, channels, branch, h, w, dd))
        return fail("preact_wide_bwd_weight: shape outside the fused wide-block kernels");
    if (!g || !x || !t2 || !t3 || !p || !gr || !workspace) return fail("preact_wide_bwd_weight: null pointer");
    const vq3d_preact_grads &G = *gr;
    if (!G.dw1 || !G.dw2 || !G.dw3 || !G.dbias1a || !G.dbias1b || !G.dbias2a || !G.dbias2b || !G.dbias3a ||
        !G.dbias3b || !G.dscale || !G.dbias4)
        return fail("preact_wide_bwd_weight: every gradient buffer is required");
    const WsLayout l = ws_layout(batch, h, w, dd);
    if (workspace_bytes < l.total) return fail("preact_wide_bwd_weight: workspace too small");
    set_lds_limits();
    const char *ws = static_cast<const char *>(workspace);
    const WArgs a = make_args(batch, h, w, dd);
    const int nch = int(int64_t(batch) * h * w * dd / CHV), nchb = int(int64_t(batch) * h * w * dd / SUBV);
    hipStream_t s = as_stream(stream);
    float *p2a = reinterpret_cast<float *>(const_cast<char *>(ws) + l.p2a);
    float *p2b = reinterpret_cast<float *>(const_cast<char *>(ws) + l.p2b);
    if (stages & 1)
        k_wide_wgrad<<<9 * nch + nchb, NT, kWgLds, s>>>(a, nch, g, x, static_cast<const h16_t *>(t2),
                                                   static_cast<const h16_t *>(t3),
                                                   reinterpret_cast<const h16_t *>(ws + l.gz3),
                                                   reinterpret_cast<const h16_t *>(ws + l.gz1), *p, p2a, p2b);
    if (!(stages & 2)) return check_launch("preact_wide_bwd_weight");
    RedOut o{G.dw1, G.dw2, G.dw3, G.dbias1a, G.dbias1b, G.dbias2a, G.dbias2b, G.dbias3a, G.dbias3b,
             G.dscale, G.dbias4, p->scale};
    const int ne = 9 * NE2 + NEB;
    k_wide_reduce<<<(ne + RNT - 1) / RNT + 1, RNT, 0, s>>>(nch, nchb, a.ntiles, p2a, p2b,
                                                           reinterpret_cast<const float *>(ws + l.p1), o);
    return check_launch("preact_wide_bwd_weight");
}

}  // extern "C"
