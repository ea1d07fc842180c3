// Forward of a whole PreActFixupResBlock (vqvae/layers.py:176-195, mode 'same', no skip conv)
// in ONE launch for the 18-channel / branch-9 blocks of the published model's 128x128x32 level
// (50 per step).  Unfused, the block forward is three launches that each stream activations
// through HBM (1x1 conv, 3x3x3 conv, 1x1 conv + residual); here a workgroup owns a 16 x 16 x 8
// brick and 768 threads (one D-run of 8 voxels x 3 channel groups):
//
//   A. t2 = elu(W1 (elu(x + b1a) + b1b) + b2a) + b2b on the brick's 18 x 18 x 10 halo
//      (circular wrap), straight from the x rows, bf16 in LDS (rows padded to 16 channels)
//   B. t3 = elu(W2 (*) t2 + b3a) + b3b: a thread owns a D-run of 8 voxels and 3 output channels,
//      so one halo line read (10 positions) feeds 3 taps x 8 voxels; W2 broadcast from LDS; the
//      line stride is an odd number of dwords (adjacent D-runs hit different banks)
//   C. out = scale * W3 t3 + b4 + x for the D-run's 8 voxels, 6 output channels per thread, on
//      the brick's x rows staged in LDS (over the dead t2 halo) and updated in place
//
// t2 (brick rows) and t3 go to HBM as bf16 for the backward, which is unchanged.  Every HBM
// access of the brick's rows (x in, out / t2 / t3 out) is a 16-B chunk per thread with
// consecutive threads on consecutive chunks: whole cache lines per wave, no partial-line writes.
// Rounding points are the unfused path's (t2 and t3 rounded to bf16 before the next conv), fp32
// accumulation; all three weight tensors are broadcast from LDS (fp32, rows padded to 48 B).
#include "engines.h"

#include <algorithm>
#include <cstdlib>

namespace vq3d {

namespace {

constexpr int C = 18, BR = 9;                 // block channels, branch channels
constexpr int BD = 8, HD = BD + 2;            // brick depth (one D-run of 8 voxels per thread)
constexpr int WS = 12;                        // weight row stride in LDS (fp32, 48 B)
constexpr int NG = 3;                         // thread groups: 3 output channels each in phase B
constexpr int W2R = 27 * 9 * 12 > 14 * 64 * 8 / 2 ? 27 * 9 * 12 : 14 * 64 * 8 / 2;  // W2 region (floats)

// Brick geometry (BH x BW x 8 voxels) and the t2 position row RS (bf16, >= 9): the 16 x 16
// brick with 16-wide rows needs 155 KB of LDS (one workgroup per CU, phases serialised on
// every CU); 8 x 16 with 10-wide rows fits two workgroups per CU (68 KB each).
template <int BH_, int BW_, int RS_>
struct Geo {
    static constexpr int BH = BH_, BW = BW_, RS = RS_;
    static constexpr int HH = BH + 2, HW = BW + 2, HP = HH * HW * HD;
    static constexpr int LSD = HD * RS + 2;   // t2 line stride (bf16): odd number of dwords -> no bank aliasing
    static constexpr int NR = BH * BW;        // D-runs per brick
    static constexpr int NTP = NR * NG;       // threads
    static constexpr int T2H = (HH * HW * LSD > NR * BD * C ? HH * HW * LSD : NR * BD * C + 0);  // t2 halo / x rows
    static constexpr int T2HA = (T2H + 7) / 8 * 8;
    static_assert(LSD / 2 % 2 == 1 && RS % 2 == 0 && RS >= BR, "odd dword line stride, paired rows");
    static_assert((W2R + 2 * C * WS) * 4 % 16 == 0, "t2h 16-B aligned");
    static size_t lds() { return (size_t(W2R) + 2 * size_t(C) * WS) * 4 + (size_t(T2HA) + 8 + size_t(NR) * BD * BR) * 2; }
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NPAIR = 14;  // MFMA k-steps of phase B: 27 taps in pairs x 16 (padded) channels

struct MidArgs {
    int B, H, W, D;
    int nbh, nbw, nbd, nbricks;
};

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

template <class G>
__global__ __launch_bounds__(G::NTP) void k_preact_mid_fwd(MidArgs a, const bf16_t *__restrict__ x,
                                                       const float *__restrict__ w1, const float *__restrict__ w2,
                                                       const float *__restrict__ w3, vq3d_preact_params p,
                                                       bf16_t *__restrict__ out, bf16_t *__restrict__ t2o,
                                                       bf16_t *__restrict__ t3o) {
    constexpr int BH = G::BH, BW = G::BW, RS = G::RS, HW = G::HW, HP = G::HP, LSD = G::LSD, NR = G::NR,
                  NTP = G::NTP;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *w2s = reinterpret_cast<float *>(smem);                      // [tap][c][WS] (o < 9)
    float *w1s = w2s + W2R;                                            // [c][WS]      (o < 9)
    float *w3s = w1s + C * WS;                                         // [co][WS]     (o < 9)
    bf16_t *t2h = reinterpret_cast<bf16_t *>(w3s + C * WS);            // [HH * HW lines][LSD]
    bf16_t *t3s = t2h + G::T2HA + 8;                             // [NR][BD * BR]
    const int tid = threadIdx.x;
    {
        // phase-B MFMA B fragments, bf16: [pair][lane][8], lane l holds B[k = 8 (l >> 4) + j][n = l & 15]
        // with k = 16 * (tap - 2 pair) + c (c < 16 padded, tap < 27), n = output channel (< 9)
        bf16_t *wf = reinterpret_cast<bf16_t *>(w2s);
        for (int i = tid; i < NPAIR * 64 * 8; i += NTP) {
            const int j = i & 7, l = (i >> 3) & 63, pr = i >> 9;
            const int k = 8 * (l >> 4) + j, n = l & 15, c = k & 15, tap = 2 * pr + (k >> 4);
            wf[i] = bf16_t(f2bf(n < BR && c < BR && tap < 27 ? w2[(n * BR + c) * 27 + tap] : 0.f));
        }
    }
    for (int i = tid; i < C * WS; i += NTP) {
        const int o = i % WS, c = i / WS;
        w1s[i] = o < BR ? w1[o * C + c] : 0.f;  // W1 [BR][C] -> [c][o]
        w3s[i] = o < BR ? w3[c * BR + o] : 0.f;  // W3 [C][BR] -> [co][o]
    }
    const float b1a = *p.bias1a, b1b = *p.bias1b, b2a = *p.bias2a, b2b = *p.bias2b;
    const float b3a = *p.bias3a, b3b = *p.bias3b, sc = *p.scale, b4 = *p.bias4;
    const int run = tid % NR, grp = tid / NR;  // D-run (lh, lw) and channel group (wave-uniform)


    for (int brick = blockIdx.x; brick < a.nbricks; brick += gridDim.x) {
        int bi = brick;
        const int bzd = bi % a.nbd;
        bi /= a.nbd;
        const int bzw = bi % a.nbw;
        bi /= a.nbw;
        const int bzh = bi % a.nbh;
        const int b = bi / a.nbh;
        const int oh0 = bzh * BH, ow0 = bzw * BW, od0 = bzd * BD;
        __syncthreads();
        // ---- A. t2 on the halo
        for (int q = tid; q < HP; q += NTP) {
            asm volatile("" ::: "memory");  // keep the W1 rows as per-iteration LDS reads (no hoisting)
            const int dd = q % HD, line = q / HD, ww = line % HW, hh = line / HW;
            const int gh = wrapm(oh0 - 1 + hh, a.H), gw = wrapm(ow0 - 1 + ww, a.W), gd = wrapm(od0 - 1 + dd, a.D);
            const uint32_t *s32 =
                reinterpret_cast<const uint32_t *>(x + (((int64_t(b) * a.H + gh) * a.W + gw) * a.D + gd) * C);
            float u[C];
#pragma unroll
            for (int j = 0; j < C / 2; ++j) {
                const uint32_t v = s32[j];
                u[2 * j] = elu(__uint_as_float(v << 16) + b1a) + b1b;
                u[2 * j + 1] = elu(__uint_as_float(v & 0xffff0000u) + b1a) + b1b;
            }
            float a9[WS];
#pragma unroll
            for (int o = 0; o < WS; ++o) a9[o] = 0.f;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const float4 *wr = reinterpret_cast<const float4 *>(w1s + c * WS);
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const float4 wq = wr[k];
                    a9[4 * k] = fmaf(u[c], wq.x, a9[4 * k]);
                    a9[4 * k + 1] = fmaf(u[c], wq.y, a9[4 * k + 1]);
                    a9[4 * k + 2] = fmaf(u[c], wq.z, a9[4 * k + 2]);
                    a9[4 * k + 3] = fmaf(u[c], wq.w, a9[4 * k + 3]);
                }
            }
            uint32_t *dst = reinterpret_cast<uint32_t *>(t2h + line * LSD + dd * RS);
#pragma unroll
            for (int o = 0; o < RS; o += 2) {
                const float lo = o < BR ? elu(a9[o] + b2a) + b2b : 0.f;
                const float hi = o + 1 < BR ? elu(a9[o + 1] + b2a) + b2b : 0.f;
                dst[o / 2] = uint32_t(f2bf(lo)) | (uint32_t(f2bf(hi)) << 16);
            }
        }
        __syncthreads();
        static_assert(G::RS == 16, "MFMA phase B reads 8-channel halves of 16-wide rows");
        {
        // ---- B (matrix cores). t3 = W2 (*) t2 as 16-voxel x 16-channel tiles (two D-runs of 8
        //      voxels; 9 of 16 output columns valid), K = 27 taps x 16 channels in 14 steps of
        //      v_mfma_f32_16x16x32_bf16; lane l reads its A row (voxel l & 15) straight from the
        //      t2 halo lines: 8 channels of one tap, 16 B in two dword pairs (lines are 4-B aligned)
            const int lane = tid & 63, wave = tid >> 6;
            const int ri = lane & 15, kb = lane >> 4, ts = kb >> 1, ch = (kb & 1) * 8;
            const bf16_t *wf = reinterpret_cast<const bf16_t *>(w2s);
            constexpr int NW = NTP / 64;
            // two tiles per iteration share each B fragment read and overlap their dependent
            // MFMA chains
            static_assert(NR % 4 == 0, "tile pairs");
            for (int tp = wave; tp < NR / 4; tp += NW) {
                const bf16_t *abase[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int run_i = 2 * (2 * tp + h) + (ri >> 3), d_i = ri & 7;
                    abase[h] = t2h + ((run_i / BW) * HW + run_i % BW) * LSD + d_i * RS + ch;
                }
                f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
                for (int pr = 0; pr < NPAIR; ++pr) {
                    constexpr auto toff = [](int tap) { return ((tap / 9) * HW + (tap / 3) % 3) * LSD + (tap % 3) * RS; };
                    const int ta = 2 * pr, tb = 2 * pr + 1;
                    const bool valid = ts == 0 || tb < 27;
                    const int off = ts ? toff(tb < 27 ? tb : ta) : toff(ta);
                    const bf16x8 bfr = *reinterpret_cast<const bf16x8 *>(wf + (pr * 64 + lane) * 8);
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t *ap = reinterpret_cast<const uint32_t *>(abase[h] + off);
                        uint32_t au[4] = {0u, 0u, 0u, 0u};
                        if (valid) {
                            au[0] = ap[0];
                            au[1] = ap[1];
                            au[2] = ap[2];
                            au[3] = ap[3];
                        }
                        bf16x8 af;
                        __builtin_memcpy(&af, au, 16);
                        acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[h], 0, 0, 0);
                    }
                }
                const int o = lane & 15;
                if (o < BR) {
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int row = kb * 4 + j, r = 2 * (2 * tp + h) + (row >> 3), v = row & 7;
                            t3s[r * BD * BR + v * BR + o] = bf16_t(f2bf(elu(acc[h][j] + b3a) + b3b));
                        }
                }
            }
        }
        __syncthreads();
        // t3 and the brick's t2 rows to HBM in 16-B chunks, consecutive threads on consecutive
        // chunks of a D-run's 144 contiguous bytes (whole cache lines per wave store)
        auto run_vox = [&](int r) {
            return ((int64_t(b) * a.H + oh0 + r / BW) * a.W + ow0 + r % BW) * a.D + od0;
        };
        constexpr int CH2 = BD * BR / 8;  // 9 chunks per D-run
        for (int j = tid; j < NR * CH2; j += NTP) {
            const int r = j / CH2, part = j - r * CH2;
            const int64_t v0 = run_vox(r);
            *reinterpret_cast<uint4 *>(t3o + v0 * BR + part * 8) =
                *reinterpret_cast<const uint4 *>(t3s + r * BD * BR + part * 8);
            const uint16_t *own = reinterpret_cast<const uint16_t *>(t2h + ((r / BW + 1) * HW + r % BW + 1) * LSD);
            uint32_t w4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int e0 = part * 8 + 2 * i, e1 = e0 + 1;
                w4[i] = uint32_t(own[(1 + e0 / BR) * RS + e0 % BR]) | (uint32_t(own[(1 + e1 / BR) * RS + e1 % BR]) << 16);
            }
            *reinterpret_cast<uint4 *>(t2o + v0 * BR + part * 8) = uint4{w4[0], w4[1], w4[2], w4[3]};
        }
        __syncthreads();  // t2h is reused below for the brick's x / out rows
        // ---- C. x rows into LDS (16-B chunks), out = scale * W3 t3 + b4 + x in place (thread:
        //      D-run x 6 output channels), out rows back to HBM in 16-B chunks
        bf16_t *obuf = t2h;               // [D-run][BD * C]
        constexpr int CH1 = BD * C / 8;  // 18 chunks per D-run
        for (int j = tid; j < NR * CH1; j += NTP) {
            const int r = j / CH1, part = j - r * CH1;
            *reinterpret_cast<uint4 *>(obuf + r * BD * C + part * 8) =
                *reinterpret_cast<const uint4 *>(x + run_vox(r) * C + part * 8);
        }
        __syncthreads();
        {
            const bf16_t *t3r = t3s + run * BD * BR;
            constexpr int CG = C / NG;  // 6 output channels per group
            for (int v = 0; v < BD; ++v) {
                asm volatile("" ::: "memory");  // W3 rows re-read from LDS per voxel (no hoisting)
                float t3v[BR];
#pragma unroll
                for (int o = 0; o < BR; ++o) t3v[o] = ld(t3r + v * BR + o);
                uint32_t *xr = reinterpret_cast<uint32_t *>(obuf + run * BD * C + v * C + grp * CG);
#pragma unroll
                for (int k = 0; k < CG / 2; ++k) {
                    const uint32_t xq = xr[k];
                    float r2[2];
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        const int co = grp * CG + 2 * k + s2;
                        const float4 *wr = reinterpret_cast<const float4 *>(w3s + co * WS);
                        const float4 wa = wr[0], wb = wr[1];
                        const float wc = w3s[co * WS + 8];
                        const float wv[BR] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w, wc};
                        float accv = 0.f;
#pragma unroll
                        for (int o = 0; o < BR; ++o) accv = fmaf(t3v[o], wv[o], accv);
                        const float xv = s2 ? __uint_as_float(xq & 0xffff0000u) : __uint_as_float(xq << 16);
                        r2[s2] = accv * sc + b4 + xv;
                    }
                    xr[k] = uint32_t(f2bf(r2[0])) | (uint32_t(f2bf(r2[1])) << 16);
                }
            }
        }
        __syncthreads();
        for (int j = tid; j < NR * CH1; j += NTP) {
            const int r = j / CH1, part = j - r * CH1;
            *reinterpret_cast<uint4 *>(out + run_vox(r) * C + part * 8) =
                *reinterpret_cast<const uint4 *>(obuf + r * BD * C + part * 8);
        }
    }
}

using GeoWide = Geo<16, 16, 16>;  // 256 bricks at 128 x 128 x 32
template <class G>
void launch_mid(const MidArgs &a0, hipStream_t s, const bf16_t *x, const float *w1, const float *w2, const float *w3,
                const vq3d_preact_params &p, bf16_t *out, bf16_t *t2, bf16_t *t3) {
    MidArgs a = a0;
    a.nbh = a.H / G::BH;
    a.nbw = a.W / G::BW;
    a.nbd = a.D / BD;
    a.nbricks = a.B * a.nbh * a.nbw * a.nbd;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_preact_mid_fwd<G>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024 - 256));
        (void)hipGetLastError();
        attr = true;
    }
    k_preact_mid_fwd<G><<<unsigned(a.nbricks), G::NTP, G::lds(), s>>>(a, x, w1, w2, w3, p, out, t2, t3);
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_mid_supported(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd) {
    return dtype == VQ3D_BF16 && batch >= 1 && channels == C && branch == BR && h % 16 == 0 && w % 16 == 0 &&
           dd % BD == 0 && h > 0 && w > 0 && dd > 0;
}

int vq3d_preact_mid_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                        int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                        const vq3d_preact_params *p, void *out, void *t2, void *t3, vq3d_stream_t stream) {
    if (!vq3d_preact_mid_supported(dtype, batch, channels, branch, h, w, dd))
        return fail("preact_mid_fwd: shape outside the fused mid-level block kernel");
    if (!x || !w1 || !w2 || !w3 || !p || !out || !t2 || !t3) return fail("preact_mid_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    MidArgs a;
    a.B = batch;
    a.H = h;
    a.W = w;
    a.D = dd;
    const bf16_t *xb = (const bf16_t *)x;
    bf16_t *ob = (bf16_t *)out, *t2b = (bf16_t *)t2, *t3b = (bf16_t *)t3;
    launch_mid<GeoWide>(a, s, xb, w1, w2, w3, *p, ob, t2b, t3b);
    return check_launch("preact_mid_fwd");
}

}  // extern "C"
