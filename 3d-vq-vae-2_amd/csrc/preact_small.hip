// A whole PreActFixupResBlock (vqvae/layers.py:176-195, mode 'same', no skip conv) with few
// channels, forward in ONE launch and backward in TWO, for the published model's narrow blocks:
// (block channels C, branch B) = (2, 1) at 128x128x32 (50 encoder pre-quantize blocks), (8, 4) at
// 32x32x8 (50) and 256x256x64 (post-up), (4, 2) at 512x512x128 (post-up).  Unfused, one block is
// ~20 launches (three convs fwd, three dgrads, three wgrads + reductions) whose few-channel
// operands never fill a wave; here every thread owns whole voxels and all channels:
//
//   u1  = elu(x + b1a) + b1b          t2 = elu(W1 u1 + b2a) + b2b            (1x1, C -> B)
//   t3  = elu(W2 (*) t2 + b3a) + b3b  (3x3x3 circular, B -> B)
//   out = scale * (W3 t3) + b4 + x                                           (1x1, B -> C)
//
// forward: a workgroup owns a brick of voxels; phase A computes t2 on the brick's circular halo
//   (one halo position per thread iteration, x read straight from HBM) into LDS, phase B the
//   voxel's t3 (27 taps from LDS, weights broadcast from LDS) and, from registers, out.
//   t2 / t3 are written (bf16) for the backward.  Rounding points are the unfused path's:
//   t2 and t3 rounded to bf16 before the next conv, fp32 accumulation.
// backward: per brick, gz3 = scale W3^T g * elu'(t3) on the halo (bf16, as the unfused conv3
//   dgrad writes it), then per voxel dL/dt2 = W2^T (*) gz3 (transposed taps), gz1 = dL/dt2 *
//   elu'(t2) (bf16), gx = g + (W1^T gz1) elu'(x + b1a); the brick's weight-gradient partials
//   (W3: sum g t3, W2: sum gz3 t2(shifted), W1: sum gz1 u1) and the eight scalar-gradient
//   partials go to the workspace [entry][brick]; a second launch sums every entry over the
//   bricks in a fixed order (deterministic, one adder per gradient entry).
#include "engines.h"

#include <algorithm>

namespace vq3d {

namespace {

constexpr int NT = 256;           // threads per workgroup (both kernels)
constexpr int kNScal = 8;         // scalar partials: b4, scale, b3b, b3a, b2b, b2a, b1b, b1a
constexpr int RP = NT + 4;        // pitch (16-byte slots) of the backward's per-thread sums in LDS
constexpr size_t kLdsTarget = 80 * 1024;
#ifdef SMALL_PROBE  // phase clocks of k_small_bwd (tools/probes/small_probe.hip), held in registers
__device__ unsigned long long g_small_probe[1024][12];  // and stored at the end (no stores in between)
#define SPROBE_DECL unsigned long long sprobe_t[12] = {};
#define SPROBE(k)                              \
    __builtin_amdgcn_sched_barrier(0);         \
    sprobe_t[k] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);
#define SPROBE_DUMP                                                        \
    if (threadIdx.x == 0 && blockIdx.x < 1024)                             \
        for (int i_ = 0; i_ < 12; ++i_) g_small_probe[blockIdx.x][i_] = sprobe_t[i_];
#else
#define SPROBE_DECL
#define SPROBE(k)
#define SPROBE_DUMP
#endif
#ifndef SMALL_TSPLIT
#define SMALL_TSPLIT 1  // bricks below NT voxels: the 27 taps over NT / nvb thread groups (0: one voxel per thread)
#endif
#ifndef SMALL_BPRE
#define SMALL_BPRE 1  // backward prologue: 0 weights staged first, 1 + halo loads before, 2 + the voxel x too
#endif
#ifndef SMALL_TU
#define SMALL_TU 1  // unroll of the per-voxel tap loops (timing experiments)
#endif
#ifndef SMALL_MINV
#define SMALL_MINV 64  // smallest brick halved to for more workgroups (timing experiments: EXPDEF=SMALL_MINV)
#endif

struct SArgs {
    int B, H, W, D;
    int bh, bw, bd, lbw, lbd;  // brick (powers of two)
    int hw, hd, hp;            // halo W / D extents, halo positions
    int nvb;                   // voxels per brick
    int nbh, nbw, nbd, nbricks;
};

constexpr int n_entries(int C, int BR) { return C * BR + 27 * BR * BR + BR * C; }
#ifndef SMALL_S2
#define SMALL_S2 16  // W2-gradient sub-streams of the 4-branch backward (timing experiments; 14 before)
#endif
constexpr int s2_of(int BR) { return BR >= 4 ? SMALL_S2 : 28; }  // W2-gradient sub-streams (9 each)

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }
__device__ __forceinline__ float rbf(float v) { return h2f_lo(uint32_t(f2h(v))); }
#ifndef SMALL_FASTEXP
#define SMALL_FASTEXP 1  // the brick kernels' elu on the hardware exp (v_exp_f32), as the column kernels' elu_f
#endif
__device__ __forceinline__ float belu(float z) {
    if constexpr (SMALL_FASTEXP) return z > 0.f ? z : __expf(z) - 1.f;
    else return elu(z);
}
__device__ __forceinline__ float belu_grad(float z) {
    if constexpr (SMALL_FASTEXP) return z > 0.f ? 1.f : __expf(z);
    else return elu_grad(z);
}
__device__ __forceinline__ float elu_d_act(float t, float b) {  // elu'(z) from t = elu(z) + b
    const float z1 = t - b;
    return z1 > 0.f ? 1.f : z1 + 1.f;
}

// N consecutive bf16 (N in 1, 2, 4, 8; the address is N * 2-byte aligned) <-> fp32 registers
template <int N>
__device__ __forceinline__ void ldv(const h16_t *__restrict__ p, float (&o)[N]) {
    if constexpr (N == 1) {
        o[0] = ld(p);
    } else if constexpr (N == 2) {
        const uint32_t u = *reinterpret_cast<const uint32_t *>(p);
        o[0] = h2f_lo(u);
        o[1] = h2f_hi(u);
    } else if constexpr (N == 4) {
        const uint2 u = *reinterpret_cast<const uint2 *>(p);
        const uint32_t w[2] = {u.x, u.y};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            o[2 * i] = h2f_lo(w[i]);
            o[2 * i + 1] = h2f_hi(w[i]);
        }
    } else {
        static_assert(N == 8, "channel count");
        const uint4 u = *reinterpret_cast<const uint4 *>(p);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = h2f_lo(w[i]);
            o[2 * i + 1] = h2f_hi(w[i]);
        }
    }
}

template <int N>
__device__ __forceinline__ void stv(h16_t *__restrict__ p, const float (&v)[N]) {
    if constexpr (N == 1) {
        *p = f2h(v[0]);
    } else {
        uint32_t w[N / 2];
#pragma unroll
        for (int i = 0; i < N / 2; ++i) w[i] = uint32_t(f2h(v[2 * i])) | (uint32_t(f2h(v[2 * i + 1])) << 16);
        if constexpr (N == 2) *reinterpret_cast<uint32_t *>(p) = w[0];
        else if constexpr (N == 4) *reinterpret_cast<uint2 *>(p) = uint2{w[0], w[1]};
        else *reinterpret_cast<uint4 *>(p) = uint4{w[0], w[1], w[2], w[3]};
    }
}

struct Brick {
    int b, oh0, ow0, od0;
};

__device__ __forceinline__ Brick brick_of(const SArgs &a, int brick) {
    Brick k;
    int bi = brick;
    const int bzd = bi % a.nbd;
    bi /= a.nbd;
    const int bzw = bi % a.nbw;
    bi /= a.nbw;
    const int bzh = bi % a.nbh;
    k.b = bi / a.nbh;
    k.oh0 = bzh * a.bh;
    k.ow0 = bzw * a.bw;
    k.od0 = bzd * a.bd;
    return k;
}

// halo position of brick voxel v, and the global voxel index of halo position q
__device__ __forceinline__ int halo_pos(const SArgs &a, int v) {
    const int ld_ = v & (a.bd - 1), lw = (v >> a.lbd) & (a.bw - 1), lh = v >> (a.lbd + a.lbw);
    return ((lh + 1) * a.hw + lw + 1) * a.hd + ld_ + 1;
}
__device__ __forceinline__ int64_t brick_vox(const SArgs &a, const Brick &k, int v) {
    const int ld_ = v & (a.bd - 1), lw = (v >> a.lbd) & (a.bw - 1), lh = v >> (a.lbd + a.lbw);
    return ((int64_t(k.b) * a.H + k.oh0 + lh) * a.W + k.ow0 + lw) * a.D + k.od0 + ld_;
}
// (global voxel, interior brick voxel or -1) of halo position q (circular wrap)
__device__ __forceinline__ int64_t halo_vox(const SArgs &a, const Brick &k, int q, int &vi) {
    const int dd = q % a.hd, r = q / a.hd, ww = r % a.hw, hh = r / a.hw;
    const int gh = wrapm(k.oh0 - 1 + hh, a.H), gw = wrapm(k.ow0 - 1 + ww, a.W), gd = wrapm(k.od0 - 1 + dd, a.D);
    vi = (hh >= 1 && hh <= a.bh && ww >= 1 && ww <= a.bw && dd >= 1 && dd <= a.bd)
             ? ((hh - 1) * a.bw + ww - 1) * a.bd + dd - 1
             : -1;
    return ((int64_t(k.b) * a.H + gh) * a.W + gw) * a.D + gd;
}
// halo offset of tap (kh, kw, kd), tap = (kh * 3 + kw) * 3 + kd (nn.Conv3d weight order)
__device__ __forceinline__ int tap_off(const SArgs &a, int tap) {
    const int kd = tap % 3, kw = (tap / 3) % 3, kh = tap / 9;
    return ((kh - 1) * a.hw + kw - 1) * a.hd + kd - 1;
}

struct Scal {
    float b1a, b1b, b2a, b2b, b3a, b3b, sc, b4;
};
__device__ __forceinline__ Scal load_scal(const vq3d_preact_params &p) {
    return Scal{*p.bias1a, *p.bias1b, *p.bias2a, *p.bias2b, *p.bias3a, *p.bias3b, *p.scale, *p.bias4};
}

// A workgroup's weights staged through registers: loaded (clamped, unconditional) before the
// kernel's first data loads, stored to LDS after them.  W2 goes to [tap][c][o] (forward) or
// [tap][o][c] (backward, transposed), W1 / W3 in torch order.
template <int C, int BR>
struct WStage {
    static constexpr int N2 = 27 * BR * BR, J2 = (N2 + NT - 1) / NT;
    static_assert(BR * C <= NT, "one W1 / W3 element per thread");
    float v2[J2], v1, v3;
    __device__ __forceinline__ WStage(const float *__restrict__ w1, const float *__restrict__ w2,
                                      const float *__restrict__ w3, int tid) {
#pragma unroll
        for (int j = 0; j < J2; ++j) v2[j] = w2[min(tid + j * NT, N2 - 1)];
        v1 = w1[min(tid, BR * C - 1)];
        v3 = w3[min(tid, BR * C - 1)];
    }
    __device__ __forceinline__ void store(float *w2s, float *w1s, float *w3s, int tid, bool transposed) const {
#pragma unroll
        for (int j = 0; j < J2; ++j) {
            const int i = tid + j * NT;
            if (i < N2) {
                const int tap = i % 27, r = i / 27, c = r % BR, o = r / BR;
                w2s[transposed ? (tap * BR + o) * BR + c : (tap * BR + c) * BR + o] = v2[j];
            }
        }
        if (tid < BR * C) {
            w1s[tid] = v1;
            w3s[tid] = v3;
        }
    }
};

// ------------------------------------------------------------------------------------ forward
// TX / TO: storage of the residual stream in / out (bf16 or fp32, as preact_col.hip)
template <int C, int BR, typename TX, typename TO, int UA = (C <= 4 ? 8 : 4)>
__global__ __launch_bounds__(NT) void k_small_fwd(SArgs a, const TX *__restrict__ x, const float *__restrict__ w1,
                                                 const float *__restrict__ w2, const float *__restrict__ w3,
                                                 vq3d_preact_params p, TO *__restrict__ out,
                                                 h16_t *__restrict__ t2o, h16_t *__restrict__ t3o) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *w2s = sm;                  // [tap][c][o]
    float *t2h = w2s + 27 * BR * BR;  // [halo position][BR]
    float *tps = t2h + a.hp * BR;     // [NT][BR] tap-group partials (bricks below NT voxels)
    __shared__ float w1s[BR * C], w3s[C * BR];  // W1 [o][c], W3 [co][o] (torch order)
    const int tid = threadIdx.x;
    const Brick k = brick_of(a, blockIdx.x);  // one brick per workgroup (grid = nbricks)
    // A. t2 on the halo, UA positions per thread.  The first batch's x loads are issued before the
    // weight staging and its barrier (raw words, converted after): the two load latencies overlap.
    int vi[UA];
    int64_t vox[UA];
    Raw<TX, C> xr[UA];
    auto loadA = [&](int q0) {
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const int q = q0 + u * NT;
            vox[u] = halo_vox(a, k, q < a.hp ? q : q0, vi[u]);
            xr[u] = ldraw<TX, C>(x + vox[u] * C);
        }
    };
    // weights first (registers), then the halo loads, then the weights' LDS stores: the stores wait
    // for the weight loads only (loads complete in order); every load unconditional (clamped)
    const WStage<C, BR> ws(w1, w2, w3, tid);
    loadA(min(tid, a.hp - 1));
    ws.store(w2s, w1s, w3s, tid, false);
    const Scal s = load_scal(p);
    __syncthreads();
    {
        for (int q0 = tid; q0 < a.hp; q0 += UA * NT) {
            if (q0 != tid) loadA(q0);
#pragma unroll
            for (int u = 0; u < UA; ++u) {
                const int q = q0 + u * NT;
                if (q >= a.hp) break;
                float xv[C];
                unraw<TX, C>(xr[u], xv);
#pragma unroll
                for (int c = 0; c < C; ++c) xv[c] = belu(xv[c] + s.b1a) + s.b1b;
                float t[BR];
#pragma unroll
                for (int o = 0; o < BR; ++o) {
                    float acc = 0.f;
#pragma unroll
                    for (int c = 0; c < C; ++c) acc = fmaf(w1s[o * C + c], xv[c], acc);
                    t[o] = rbf(belu(acc + s.b2a) + s.b2b);
                    t2h[q * BR + o] = t[o];
                }
                if (vi[u] >= 0 && t2o) stv<BR>(t2o + vox[u] * BR, t);
            }
        }
        __syncthreads();
        // B. t3 and out of the brick's voxels.  A brick smaller than the workgroup (the 64-voxel
        // bricks of a 32x32x8 grid) splits the 27 taps over G = NT / nvb thread groups: a quarter of
        // the dependent tap chain per thread, the partials summed by group 0 in group order.
        auto epi = [&](int v, const float (&acc)[BR], const float (&xv)[C]) {
            const int64_t vox = brick_vox(a, k, v);
            float t3v[BR], ov[C];
#pragma unroll
            for (int o = 0; o < BR; ++o) t3v[o] = rbf(belu(acc[o] + s.b3a) + s.b3b);
            if (t3o) stv<BR>(t3o + vox * BR, t3v);
#pragma unroll
            for (int co = 0; co < C; ++co) {
                float r = 0.f;
#pragma unroll
                for (int o = 0; o < BR; ++o) r = fmaf(w3s[co * BR + o], t3v[o], r);
                ov[co] = r * s.sc + s.b4 + xv[co];
            }
            stvec<TO, C>(out + vox * C, ov);
        };
        auto taps = [&](int pos, int t0, int t1, float (&acc)[BR]) {
#pragma unroll
            for (int o = 0; o < BR; ++o) acc[o] = 0.f;
#pragma unroll SMALL_TU
            for (int tap = t0; tap < t1; ++tap) {
                const float *tr = t2h + (pos + tap_off(a, tap)) * BR;
                const float *wr = w2s + tap * BR * BR;
#pragma unroll
                for (int c = 0; c < BR; ++c) {
                    const float tv = tr[c];
#pragma unroll
                    for (int o = 0; o < BR; ++o) acc[o] = fmaf(tv, wr[c * BR + o], acc[o]);
                }
            }
        };
        if (SMALL_TSPLIT && a.nvb < NT) {
            const int G = NT / a.nvb, v = tid & (a.nvb - 1), tg = tid / a.nvb;
            float xv[C], acc[BR];
            if (tg == 0) ldvec<TX, C>(x + brick_vox(a, k, v) * C, xv);  // in flight during the taps
            taps(halo_pos(a, v), 27 * tg / G, 27 * (tg + 1) / G, acc);
            if (tg > 0) {
#pragma unroll
                for (int o = 0; o < BR; ++o) tps[tid * BR + o] = acc[o];
            }
            __syncthreads();
            if (tg == 0) {
                for (int gi = 1; gi < G; ++gi)
#pragma unroll
                    for (int o = 0; o < BR; ++o) acc[o] += tps[(gi * a.nvb + v) * BR + o];
                epi(v, acc, xv);
            }
        } else {
            for (int v = tid; v < a.nvb; v += NT) {
                float xv[C], acc[BR];
                ldvec<TX, C>(x + brick_vox(a, k, v) * C, xv);  // in flight during the taps
                taps(halo_pos(a, v), 0, 27, acc);
                epi(v, acc, xv);
            }
        }
    }
}

// ------------------------------------------------------------------------------------ backward
// g has the forward out's storage (TO), x and gx the input's (TX)
template <int C, int BR, typename TX, typename TO, int UB = (C <= 4 ? 4 : 2), int S2 = s2_of(BR)>
__global__ __launch_bounds__(NT) void k_small_bwd(SArgs a, const TO *__restrict__ g, const TX *__restrict__ x,
                                                 const h16_t *__restrict__ t2, const h16_t *__restrict__ t3,
                                                 const float *__restrict__ w1, const float *__restrict__ w2,
                                                 const float *__restrict__ w3, vq3d_preact_params p,
                                                 float *__restrict__ part, TX *__restrict__ gx) {
    constexpr int E1 = C * BR, E2 = 27 * BR * BR, E = n_entries(C, BR);
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *w2t = sm;                      // [tap][o][c]
    float *gzh = w2t + 27 * BR * BR;      // [halo position][BR]  gz3 (bf16 values)
    float *t2h = gzh + a.hp * BR;         // [halo position][BR]
    float *gs = t2h + a.hp * BR;          // [brick voxel][C]   g
    float *t3s = gs + a.nvb * C;          // [brick voxel][BR]  t3
    float *scr = t3s + a.nvb * BR;        // [S2][E2] W2 sub-stream sums
    float *tps = scr + S2 * E2;           // [NT][BR] tap-group partials (bricks below NT voxels)
    float *rt = sm + ((tps + NT * BR - sm + 3) & ~3);  // [(2 C BR + 8) / 4][RP][4] per-thread W3 / W1 sums,
                                                        // scalar partials (16-byte aligned)
    __shared__ float w1s[BR * C], w3s[C * BR], g3s[C * BR];
    const int tid = threadIdx.x;
    SPROBE_DECL
    SPROBE(0)
    const Brick k = brick_of(a, blockIdx.x);
    // phase 1's first UB positions (and, split taps, phase 2's voxel x) are loaded before the weight
    // staging and its barrier as raw words: the load latencies overlap
    int vis[UB];
    Raw<TO, C> gr_[UB];
    Raw<h16_t, BR> t3r[UB], t2r[UB];
    auto load1 = [&](int q0) {
#pragma unroll
        for (int u = 0; u < UB; ++u) {  // UB positions' loads in flight before any compute
            const int q = q0 + u * NT;
            const int64_t vox = halo_vox(a, k, q < a.hp ? q : q0, vis[u]);
            gr_[u] = ldraw<TO, C>(g + vox * C);
            t3r[u] = ldraw<h16_t, BR>(t3 + vox * BR);
            t2r[u] = ldraw<h16_t, BR>(t2 + vox * BR);
        }
    };
    const WStage<C, BR> ws(w1, w2, w3, tid);  // weights first: their LDS stores wait for them only
    if (SMALL_BPRE == 0) {
        ws.store(w2t, w1s, w3s, tid, true);
        __syncthreads();
    }
    load1(min(tid, a.hp - 1));
    const bool split = SMALL_TSPLIT && a.nvb < NT;
    Raw<TX, C> xr2;
    if (split && SMALL_BPRE >= 2) xr2 = ldraw<TX, C>(x + brick_vox(a, k, tid & (a.nvb - 1)) * C);
    if (SMALL_BPRE != 0) ws.store(w2t, w1s, w3s, tid, true);
    const Scal s = load_scal(p);
    float sp[kNScal];
#pragma unroll
    for (int j = 0; j < kNScal; ++j) sp[j] = 0.f;
    __syncthreads();
    SPROBE(1)
    // 1. gz3 and t2 on the halo; g and t3 of the interior
    for (int q0 = tid; q0 < a.hp; q0 += UB * NT) {
      if (q0 != tid) load1(q0);
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int q = q0 + u * NT;
        if (q >= a.hp) break;
        const int vi = vis[u];
        float gv[C], t3v[BR], t2v[BR];
        unraw<TO, C>(gr_[u], gv);
        unraw<h16_t, BR>(t3r[u], t3v);
        unraw<h16_t, BR>(t2r[u], t2v);
#pragma unroll
        for (int o = 0; o < BR; ++o) {
            float h = 0.f;
#pragma unroll
            for (int co = 0; co < C; ++co) h = fmaf(w3s[co * BR + o], gv[co], h);
            h *= s.sc;
            const float z = h * elu_d_act(t3v[o], s.b3b);
            gzh[q * BR + o] = rbf(z);
            t2h[q * BR + o] = t2v[o];
            if (vi >= 0) {
                sp[2] += h;
                sp[3] += z;
                t3s[vi * BR + o] = t3v[o];
            }
        }
        if (vi >= 0) {
#pragma unroll
            for (int co = 0; co < C; ++co) {
                gs[vi * C + co] = gv[co];
                sp[0] += gv[co];
            }
        }
      }
    }
    __syncthreads();
    SPROBE(2)
    // 2. per voxel: dL/dt2 = W2^T (*) gz3, gz1, gx; W3 and W1 weight-gradient sums in registers
    float acc1[C][BR], acc3[BR][C];
#pragma unroll
    for (int i = 0; i < C; ++i)
#pragma unroll
        for (int j = 0; j < BR; ++j) acc1[i][j] = acc3[j][i] = 0.f;
    auto taps = [&](int pos, int t0, int t1, float (&dt)[BR]) {
#pragma unroll
        for (int c = 0; c < BR; ++c) dt[c] = 0.f;
#pragma unroll SMALL_TU
        for (int tap = t0; tap < t1; ++tap) {
            const float *zr = gzh + (pos - tap_off(a, tap)) * BR;
            const float *wr = w2t + tap * BR * BR;
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                const float zv = zr[o];
#pragma unroll
                for (int c = 0; c < BR; ++c) dt[c] = fmaf(zv, wr[o * BR + c], dt[c]);
            }
        }
    };
    auto epi = [&](int v, const float (&dt)[BR], const float (&xv)[C], float (&gxv)[C]) {
        const int pos = halo_pos(a, v);
        float z1[BR], t3v[BR];
#pragma unroll
        for (int c = 0; c < BR; ++c) {
            const float z = dt[c] * elu_d_act(t2h[pos * BR + c], s.b2b);
            sp[4] += dt[c];
            sp[5] += z;
            z1[c] = rbf(z);
            t3v[c] = t3s[v * BR + c];
        }
#pragma unroll
        for (int ci = 0; ci < C; ++ci) {
            float r = 0.f;
#pragma unroll
            for (int o = 0; o < BR; ++o) r = fmaf(w1s[o * C + ci], z1[o], r);
            sp[6] += r;
            const float e = r * belu_grad(xv[ci] + s.b1a);
            sp[7] += e;
            const float gv = gs[v * C + ci];
            gxv[ci] = gv + e;
            const float u = belu(xv[ci] + s.b1a) + s.b1b;
#pragma unroll
            for (int o = 0; o < BR; ++o) {
                acc1[ci][o] = fmaf(gv, t3v[o], acc1[ci][o]);
                acc3[o][ci] = fmaf(z1[o], u, acc3[o][ci]);
            }
        }
    };
    // the split path's gx goes out after the sums' LDS stores (4a): stores pending behind them
    // would make the compiler wait for their completion first
    float gxs[C];
    if (split) {  // the 27 taps over NT / nvb thread groups, as the forward's
        const int G = NT / a.nvb, v = tid & (a.nvb - 1), tg = tid / a.nvb;
        float xv[C], dt[BR];
        if (SMALL_BPRE >= 2) unraw<TX, C>(xr2, xv);
        else ldvec<TX, C>(x + brick_vox(a, k, v) * C, xv);  // every thread (exact wait counts)
        taps(halo_pos(a, v), 27 * tg / G, 27 * (tg + 1) / G, dt);
        if (tg > 0) {
#pragma unroll
            for (int c = 0; c < BR; ++c) tps[tid * BR + c] = dt[c];
        }
        SPROBE(8)
        __syncthreads();
        SPROBE(9)
        if (tg == 0) {
            for (int gi = 1; gi < G; ++gi)
#pragma unroll
                for (int c = 0; c < BR; ++c) dt[c] += tps[(gi * a.nvb + v) * BR + c];
            epi(v, dt, xv, gxs);
        }
    } else {
        for (int v = tid; v < a.nvb; v += NT) {
            float xv[C], dt[BR], gxv[C];
            ldvec<TX, C>(x + brick_vox(a, k, v) * C, xv);  // in flight during the taps
            taps(halo_pos(a, v), 0, 27, dt);
            epi(v, dt, xv, gxv);
            stvec<TX, C>(gx + brick_vox(a, k, v) * C, gxv);
        }
    }
    SPROBE(3)
    const int nb = gridDim.x;
    // 4a. the W3 / W1 sums and scalar partials into LDS in groups of 4 values, [group][thread][4]
    //     (one 16-byte store per group).  Group 16 (the phase-1 scalars) comes from every thread;
    //     the rest only from the phase-2 voxel threads (split taps: the first nvb threads).
    constexpr int NR2 = 2 * C * BR + kNScal, NG = NR2 / 4;
    static_assert(NR2 % 4 == 0 && (2 * C * BR) % 4 == 0, "groups of 4");
    const int nsrc = split ? a.nvb : NT;
    {
        float vals[NR2];
#pragma unroll
        for (int i = 0; i < C; ++i)
#pragma unroll
            for (int j = 0; j < BR; ++j) {
                vals[i * BR + j] = acc1[i][j];
                vals[E1 + j * C + i] = acc3[j][i];
            }
#pragma unroll
        for (int j = 0; j < kNScal; ++j) vals[2 * E1 + j] = sp[j];
        const bool vox = tid < nsrc;
#pragma unroll
        for (int gi = 0; gi < NG; ++gi)
            if (gi == NG - 2 || vox)
                *reinterpret_cast<float4 *>(rt + (gi * RP + tid) * 4) =
                    make_float4(vals[4 * gi], vals[4 * gi + 1], vals[4 * gi + 2], vals[4 * gi + 3]);
    }
    if (split && tid < a.nvb) stvec<TX, C>(gx + brick_vox(a, k, tid) * C, gxs);
    SPROBE(10)
    // 3. W2 weight-gradient partial: thread (g9 = (kh, kw), sub) runs over D-lines of the brick,
    //    3 kd taps x BR x BR sums in registers; the S2 sub-streams summed in a fixed order
    {
        float acc2[3][BR][BR];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int o = 0; o < BR; ++o)
#pragma unroll
                for (int c = 0; c < BR; ++c) acc2[i][o][c] = 0.f;
        const int g9 = tid % 9, sub = tid / 9;
        if (sub < S2) {
            const int kh = g9 / 3, kw = g9 - kh * 3;
            const int nr = a.bh * a.bw;
            for (int r = sub; r < nr; r += S2) {
                const int lh = r / a.bw, lw = r - lh * a.bw;
                const int base = ((lh + 1) * a.hw + lw + 1) * a.hd + 1;         // voxel j = 0
                const int tb = base + ((kh - 1) * a.hw + kw - 1) * a.hd - 1;    // its kd = 0 tap
                // a sliding window of the line's t2 rows: row j + 2 is the one new row per voxel
                float tw[3][BR];
#pragma unroll
                for (int c = 0; c < BR; ++c) {
                    tw[0][c] = t2h[tb * BR + c];
                    tw[1][c] = t2h[(tb + 1) * BR + c];
                }
#pragma unroll 2
                for (int j = 0; j < a.bd; ++j) {
                    float gz[BR];
#pragma unroll
                    for (int o = 0; o < BR; ++o) gz[o] = gzh[(base + j) * BR + o];
#pragma unroll
                    for (int c = 0; c < BR; ++c) tw[2][c] = t2h[(tb + j + 2) * BR + c];
#pragma unroll
                    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
                        for (int o = 0; o < BR; ++o)
#pragma unroll
                            for (int c = 0; c < BR; ++c) acc2[kd][o][c] = fmaf(gz[o], tw[kd][c], acc2[kd][o][c]);
#pragma unroll
                    for (int c = 0; c < BR; ++c) {
                        tw[0][c] = tw[1][c];
                        tw[1][c] = tw[2][c];
                    }
                }
            }
#pragma unroll
            for (int kd = 0; kd < 3; ++kd)
#pragma unroll
                for (int o = 0; o < BR; ++o)
#pragma unroll
                    for (int c = 0; c < BR; ++c) scr[sub * E2 + ((g9 * 3 + kd) * BR + o) * BR + c] = acc2[kd][o][c];
        }
        __syncthreads();
        SPROBE(4)
        for (int e = tid; e < E2; e += NT) {
            float t = 0.f;
            for (int j = 0; j < S2; ++j) t += scr[j * E2 + e];
            part[int64_t(E1 + e) * nb + blockIdx.x] = t;
        }
    }
    // 4b. a row of 16 threads per group: thread q of the row sums the group's words of threads
    //     16 i + q (16-byte reads; RP = 4 mod 8 spreads a half-wave's 8 group rows over the banks),
    //     then the row on the DPP network.  A fixed order: deterministic.
    for (int g0 = 0; g0 < NG; g0 += NT / 16) {
        const int gi = g0 + (tid >> 4), q = tid & 15;
        if (gi < NG) {
            const int cnt = gi == NG - 2 ? NT : nsrc;
            float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int i = q; i < cnt; i += 16) {
                const float4 v = *reinterpret_cast<const float4 *>(rt + (gi * RP + i) * 4);
                t.x += v.x;
                t.y += v.y;
                t.z += v.z;
                t.w += v.w;
            }
            const float tv[4] = {group_sum<16>(t.x), group_sum<16>(t.y), group_sum<16>(t.z), group_sum<16>(t.w)};
            if (q < 4) {
                const int n = 4 * gi + q;
                const float r = tv[q];
                if (n < E1) {
                    part[int64_t(n) * nb + blockIdx.x] = r;
                    g3s[n] = r;
                } else if (n < 2 * E1) {
                    part[int64_t(E1 + E2 + n - E1) * nb + blockIdx.x] = r;
                } else if (n != 2 * E1 + 1) {
                    part[int64_t(E + n - 2 * E1) * nb + blockIdx.x] = r;
                }
            }
        }
    }
    SPROBE(5)
    __syncthreads();
    SPROBE(6)
    if (tid == 0) {  // dscale partial: sum W3 o (sum_v g t3)
        float psc = 0.f;
        for (int n = 0; n < E1; ++n) psc = fmaf(w3s[n], g3s[n], psc);
        part[int64_t(E + 1) * nb + blockIdx.x] = psc;
    }
    SPROBE(7)
    SPROBE_DUMP
}

// sum of one gradient entry's per-brick partials (fixed order), added to its gradient
template <int C, int BR>
__device__ __forceinline__ void small_bwd_reduce(const float *__restrict__ part, int nb, const float *__restrict__ scale,
                                                 const vq3d_preact_grads &gr) {
    constexpr int E1 = C * BR, E2 = 27 * BR * BR, E = n_entries(C, BR);
    __shared__ float red[NT / 64];
    const int e = blockIdx.x;
    const float *pp = part + int64_t(e) * nb;
    float acc = 0.f;
    for (int i = threadIdx.x; i < nb; i += NT) acc += pp[i];
    const float t = block_sum<float, NT>(acc, red);
    if (threadIdx.x != 0) return;
    float *dst = nullptr;
    float v = t;
    if (e < E1) {
        dst = gr.dw3 ? gr.dw3 + e : nullptr;  // W3 [co][o]
        v = t * *scale;
    } else if (e < E1 + E2) {
        const int r = e - E1, tap = r / (BR * BR), o = (r / BR) % BR, c = r % BR;
        dst = gr.dw2 ? gr.dw2 + (o * BR + c) * 27 + tap : nullptr;
    } else if (e < E) {
        dst = gr.dw1 ? gr.dw1 + (e - E1 - E2) : nullptr;  // W1 [o][c]
    } else {
        float *const sl[kNScal] = {gr.dbias4, gr.dscale, gr.dbias3b, gr.dbias3a,
                                   gr.dbias2b, gr.dbias2a, gr.dbias1b, gr.dbias1a};
        dst = sl[e - E];
    }
    if (dst) *dst += v;
}
template <int C, int BR>
__global__ __launch_bounds__(NT) void k_small_bwd_reduce(const float *__restrict__ part, int nb,
                                                        const float *__restrict__ scale, vq3d_preact_grads gr) {
    small_bwd_reduce<C, BR>(part, nb, scale, gr);
}
// a whole run of blocks (blockIdx.y = block; workspace at y * stride floats, pointers from the
// run's [block][11] device tables)
template <int C, int BR>
__global__ __launch_bounds__(NT) void k_small_bwd_reduce_run(const float *__restrict__ ws, size_t stride, int nb,
                                                            float *const *gtab, const float *const *ptab) {
    float *const *g = gtab + blockIdx.y * 11;
    const vq3d_preact_grads gr{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10]};
    small_bwd_reduce<C, BR>(ws + blockIdx.y * stride, nb, ptab[blockIdx.y * 11 + 9], gr);
}

// ------------------------------------------------------------------------------------ planning
size_t lds_fwd(const SArgs &a, int BR) { return (size_t(27) * BR * BR + size_t(a.hp) * BR) * 4; }
size_t lds_bwd(const SArgs &a, int C, int BR) {
    return (size_t(27) * BR * BR * (1 + s2_of(BR)) + 2 * size_t(a.hp) * BR + size_t(a.nvb) * (C + BR)) * 4;
}
// what the backward launches with: + the tap-group partials and the per-thread sums
size_t lds_bwd_launch(const SArgs &a, int C, int BR) {
    return lds_bwd(a, C, BR) + (size_t(NT) * BR + 3 + size_t(2 * C * BR + kNScal) * RP) * 4;
}

int ilog2(int v) {
    int r = 0;
    while ((1 << r) < v) ++r;
    return r;
}

bool shape_ok(int C, int BR) { return (C == 2 && BR == 1) || (C == 4 && BR == 2) || (C == 8 && BR == 4); }

// Brick: up to 8 x 8 x 16 voxels (powers of two dividing the grid), halved while the backward's
// LDS exceeds ~80 KB (two workgroups per CU) or while there are fewer than 256 bricks.
bool plan(int batch, int C, int BR, int h, int w, int d, SArgs &a) {
    if (!shape_ok(C, BR) || batch < 1 || h < 1 || w < 1 || d < 1) return false;
    auto pow2 = [](int v) { return (v & (v - 1)) == 0; };
    if (!pow2(h) || !pow2(w) || !pow2(d)) return false;
    a.B = batch;
    a.H = h;
    a.W = w;
    a.D = d;
    auto set = [&](int bh, int bw, int bd) {
        a.bh = bh;
        a.bw = bw;
        a.bd = bd;
        a.lbw = ilog2(bw);
        a.lbd = ilog2(bd);
        a.hw = bw + 2;
        a.hd = bd + 2;
        a.hp = (bh + 2) * a.hw * a.hd;
        a.nvb = bh * bw * bd;
        a.nbh = h / bh;
        a.nbw = w / bw;
        a.nbd = d / bd;
        a.nbricks = batch * a.nbh * a.nbw * a.nbd;
    };
    set(std::min(h, 8), std::min(w, 8), std::min(d, 16));
    while (lds_bwd(a, C, BR) > kLdsTarget || lds_bwd_launch(a, C, BR) > 159 * 1024 ||
           (a.nbricks < 256 && a.nvb > SMALL_MINV)) {
        if (a.bd >= a.bh && a.bd >= a.bw && a.bd > 1) set(a.bh, a.bw, a.bd / 2);
        else if (a.bh >= a.bw && a.bh > 1) set(a.bh / 2, a.bw, a.bd);
        else if (a.bw > 1) set(a.bh, a.bw / 2, a.bd);
        else return false;
    }
    return true;
}

template <typename K>
void allow_lds(K kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(160 * 1024 - 1024));
    (void)hipGetLastError();
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_small_supported(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                                int32_t dd) {
    SArgs a;
    return dtype == VQ3D_HALF && (col_supported(batch, channels, branch, h, w, dd) ||
                                  plan(batch, channels, branch, h, w, dd, a))
               ? 1
               : 0;
}

int vq3d_preact_small_plan(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    SArgs a;
    if (col_supported(batch, channels, branch, h, w, dd)) return 2;
    return plan(batch, channels, branch, h, w, dd, a) ? 1 : 0;
}

size_t vq3d_preact_small_workspace_bytes(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                                         int32_t dd) {
    if (col_supported(batch, channels, branch, h, w, dd)) return col_workspace_bytes(batch, channels, branch, h, w, dd);
    SArgs a;
    if (!plan(batch, channels, branch, h, w, dd, a)) return 0;
    return size_t(a.nbricks) * (n_entries(channels, branch) + kNScal) * 4;
}

int vq3d_preact_small_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                          int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                          const vq3d_preact_params *p, void *out, void *t2, void *t3, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_small_fwd: the fused few-channel kernels take bf16 operands");
    return vq3d_preact_small_fwd_io(dtype, dtype, dtype, batch, channels, branch, h, w, dd, x, w1, w2, w3, p, out, t2,
                                    t3, stream);
}

namespace {
static bool io_ok(int32_t xdt, int32_t odt) {
    return (xdt == VQ3D_HALF || xdt == VQ3D_F32) && (odt == VQ3D_HALF || odt == VQ3D_F32);
}
}  // namespace

int vq3d_preact_small_fwd_io(int32_t dtype, int32_t x_dtype, int32_t out_dtype, int32_t batch, int32_t channels, int32_t branch,
                             int32_t h, int32_t w, int32_t dd, const void *x, const float *w1, const float *w2,
                             const float *w3, const vq3d_preact_params *p, void *out, void *t2, void *t3,
                             vq3d_stream_t stream) {
    SArgs a;
    if (!x || !w1 || !w2 || !w3 || !p || !out) return fail("preact_small_fwd: null pointer");
    if (dtype != VQ3D_HALF) return fail("preact_small_fwd: dtype must be the 16-bit format");
    if (!io_ok(x_dtype, out_dtype)) return fail("preact_small_fwd: stream storage must be dtype or VQ3D_F32");
    if (col_supported(batch, channels, branch, h, w, dd))
        return col_fwd(x_dtype, out_dtype, batch, channels, branch, h, w, dd, x, w1, w2, w3, *p, out, t2, t3,
                       as_stream(stream));
    if (!plan(batch, channels, branch, h, w, dd, a))
        return fail("preact_small_fwd: shape outside the fused few-channel block kernels");
    hipStream_t s = as_stream(stream);
    const size_t lds = lds_fwd(a, branch) + size_t(NT) * branch * 4;  // + the tap-group partials
#define F2(C_, B_, TX_, TO_)                                                                                   \
    {                                                                                                          \
        static bool attr = false;                                                                              \
        if (!attr) {                                                                                           \
            allow_lds(k_small_fwd<C_, B_, TX_, TO_>);                                                          \
            attr = true;                                                                                       \
        }                                                                                                      \
        k_small_fwd<C_, B_, TX_, TO_><<<unsigned(a.nbricks), NT, lds, s>>>(a, (const TX_ *)x, w1, w2, w3, *p,  \
                                                                          (TO_ *)out, (h16_t *)t2, (h16_t *)t3); \
    }
#define F(C_, B_)                                                                                              \
    if (channels == C_ && branch == B_) {                                                                      \
        if (x_dtype == VQ3D_HALF && out_dtype == VQ3D_HALF) F2(C_, B_, h16_t, h16_t)                         \
        else if (x_dtype == VQ3D_HALF) F2(C_, B_, h16_t, float)                                               \
        else if (out_dtype == VQ3D_HALF) F2(C_, B_, float, h16_t)                                             \
        else F2(C_, B_, float, float)                                                                          \
    }
    F(2, 1) else F(4, 2) else F(8, 4)
#undef F
#undef F2
    return check_launch("preact_small_fwd");
}

int vq3d_preact_small_fwd_chain(int32_t mode, int32_t dtype, int32_t x_dtype, int32_t out_dtype, int32_t batch, int32_t channels,
                                int32_t branch, int32_t h, int32_t w, int32_t dd, const void *x, const void *t2_in,
                                const float *w1, const float *w2, const float *w3, const vq3d_preact_params *p,
                                void *out, void *t2, void *t3, const float *w1_next,
                                const vq3d_preact_params *params_next, void *t2_next, vq3d_stream_t stream) {
    if (mode < 0 || mode > 3) return fail("preact_small_fwd_chain: mode must be a mask of 1 | 2");
    if (!col_supported(batch, channels, branch, h, w, dd))
        return fail("preact_small_fwd_chain: chained runs need the column kernels (vq3d_preact_small_plan == 2)");
    if (dtype != VQ3D_HALF) return fail("preact_small_fwd_chain: dtype must be the 16-bit format");
    if (!io_ok(x_dtype, out_dtype)) return fail("preact_small_fwd_chain: stream storage must be dtype or VQ3D_F32");
    if (!x || !w1 || !w2 || !w3 || !p || !out) return fail("preact_small_fwd_chain: null pointer");
    if ((mode & 1) && !t2_in) return fail("preact_small_fwd_chain: mode 1 needs t2_in");
    if ((mode & 2) && (!w1_next || !params_next || !t2_next)) return fail("preact_small_fwd_chain: mode 2 needs the next block");
    return col_fwd(x_dtype, out_dtype, batch, channels, branch, h, w, dd, x, w1, w2, w3, *p, out, (mode & 1) ? nullptr : t2,
                   t3, as_stream(stream), mode, t2_in, w1_next, params_next, t2_next);
}

int vq3d_preact_small_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                          int32_t dd, const void *g, const void *x, const void *t2, const void *t3, const float *w1,
                          const float *w2, const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                          void *workspace, size_t ws_bytes, void *gx, vq3d_stream_t stream) {
    return vq3d_preact_small_bwd_stages(3, dtype, batch, channels, branch, h, w, dd, g, x, t2, t3, w1, w2, w3, p, gr,
                                        workspace, ws_bytes, gx, stream);
}

int vq3d_preact_small_bwd_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                                 int32_t h, int32_t w, int32_t dd, const void *g, const void *x, const void *t2,
                                 const void *t3, const float *w1, const float *w2, const float *w3,
                                 const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *workspace,
                                 size_t ws_bytes, void *gx, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("preact_small_bwd: the fused few-channel kernels take bf16 operands");
    return vq3d_preact_small_bwd_stages_io(stages, dtype, dtype, dtype, batch, channels, branch, h, w, dd, g, x, t2,
                                           t3, w1, w2, w3, p, gr, workspace, ws_bytes, gx, stream);
}

int vq3d_preact_small_bwd_stages_io(int32_t stages, int32_t dtype, int32_t x_dtype, int32_t out_dtype, int32_t batch,
                                    int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd, const void *g,
                                    const void *x, const void *t2, const void *t3, const float *w1, const float *w2,
                                    const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                                    void *workspace, size_t ws_bytes, void *gx, vq3d_stream_t stream) {
    SArgs a;
    if (stages < 1 || stages > 3) return fail("preact_small_bwd: stages must be a mask of 1 | 2");
    if (!g || !x || !t2 || !t3 || !w1 || !w2 || !w3 || !p || !gr || !gx)
        return fail("preact_small_bwd: null pointer");
    if (dtype != VQ3D_HALF) return fail("preact_small_bwd: dtype must be the 16-bit format");
    if (!io_ok(x_dtype, out_dtype)) return fail("preact_small_bwd: stream storage must be dtype or VQ3D_F32");
    if (col_supported(batch, channels, branch, h, w, dd)) {
        const vq3d_preact_grads &G = *gr;
        if (!G.dw1 || !G.dw2 || !G.dw3 || !G.dbias1a || !G.dbias1b || !G.dbias2a || !G.dbias2b || !G.dbias3a ||
            !G.dbias3b || !G.dscale || !G.dbias4)
            return fail("preact_small_bwd: every gradient buffer is required");
        if (!workspace || ws_bytes < col_workspace_bytes(batch, channels, branch, h, w, dd))
            return fail("preact_small_bwd: workspace too small");
        return col_bwd(x_dtype, out_dtype, batch, channels, branch, h, w, dd, g, x, t2, t3, w1, w2, w3, *p, G,
                       workspace, gx, stages, as_stream(stream));
    }
    if (!plan(batch, channels, branch, h, w, dd, a))
        return fail("preact_small_bwd: shape outside the fused few-channel block kernels");
    const int ne = n_entries(channels, branch) + kNScal;
    if (!workspace || ws_bytes < size_t(a.nbricks) * ne * 4) return fail("preact_small_bwd: workspace too small");
    hipStream_t s = as_stream(stream);
    const size_t lds = lds_bwd_launch(a, channels, branch);
    float *part = static_cast<float *>(workspace);
#define B2(C_, B_, TX_, TO_)                                                                                   \
    {                                                                                                          \
        static bool attr = false;                                                                              \
        if (!attr) {                                                                                           \
            allow_lds(k_small_bwd<C_, B_, TX_, TO_>);                                                          \
            attr = true;                                                                                       \
        }                                                                                                      \
        if (stages & 1)                                                                                        \
            k_small_bwd<C_, B_, TX_, TO_><<<unsigned(a.nbricks), NT, lds, s>>>(                                \
                a, (const TO_ *)g, (const TX_ *)x, (const h16_t *)t2, (const h16_t *)t3, w1, w2, w3, *p, part,  \
                (TX_ *)gx);                                                                                    \
    }
#define Bk(C_, B_)                                                                                             \
    if (channels == C_ && branch == B_) {                                                                      \
        if (x_dtype == VQ3D_HALF && out_dtype == VQ3D_HALF) B2(C_, B_, h16_t, h16_t)                         \
        else if (x_dtype == VQ3D_HALF) B2(C_, B_, h16_t, float)                                               \
        else if (out_dtype == VQ3D_HALF) B2(C_, B_, float, h16_t)                                             \
        else B2(C_, B_, float, float)                                                                          \
        if (stages & 2) k_small_bwd_reduce<C_, B_><<<unsigned(ne), NT, 0, s>>>(part, a.nbricks, p->scale, *gr); \
    }
    Bk(2, 1) else Bk(4, 2) else Bk(8, 4)
#undef Bk
#undef B2
    return check_launch("preact_small_bwd");
}

int vq3d_preact_small_reduce_run(int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                                 int32_t w, int32_t dd, const void *workspaces, size_t workspace_stride,
                                 float *const *grads, const float *const *params, vq3d_stream_t stream) {
    if (nblocks < 1 || nblocks > 65535 || !workspaces || !grads || !params)
        return fail("preact_small_reduce_run: bad arguments");
    const size_t need = vq3d_preact_small_workspace_bytes(batch, channels, branch, h, w, dd);
    if (!need || workspace_stride < need || workspace_stride % 256)
        return fail("preact_small_reduce_run: shape unsupported, or stride below the workspace size / unaligned");
    void *ws = const_cast<void *>(workspaces);
    hipStream_t s = as_stream(stream);
    if (col_supported(batch, channels, branch, h, w, dd))
        return col_reduce_run(nblocks, batch, channels, branch, h, w, dd, ws, workspace_stride, grads, params, s);
    SArgs a;
    if (!plan(batch, channels, branch, h, w, dd, a)) return fail("preact_small_reduce_run: unsupported shape");
    const int ne = n_entries(channels, branch) + kNScal;
    const float *wsf = static_cast<const float *>(ws);
#define Rk(C_, B_)                                                                                             \
    if (channels == C_ && branch == B_)                                                                        \
        k_small_bwd_reduce_run<C_, B_><<<dim3(unsigned(ne), unsigned(nblocks)), NT, 0, s>>>(                    \
            wsf, workspace_stride / 4, a.nbricks, grads, params);
    Rk(2, 1) else Rk(4, 2) else Rk(8, 4)
#undef Rk
    return check_launch("preact_small_reduce_run");
}

}  // extern "C"
