// A STACK of consecutive PreActFixupResBlocks (vqvae/layers.py:102-216, mode 'same', no skip
// conv, identical channels) on a tiny grid, forward in ONE launch and backward in ONE launch:
// the 50 top-level pre-quantize blocks of the encoder and the 50 post-quantize blocks of the
// decoder of the published 3-layer model (8 x 8 x 2 = 128 voxels, 32 channels, branch 16).
// Per block, unfused, that level costs a forward and a two-launch backward whose grids hold a
// handful of workgroups; chained, one workgroup (1,024 threads) keeps the whole residual stream
// in LDS and walks the blocks:
//
//   u1  = elu(x + b1a) + b1b        t2 = elu(W1 u1 + b2a) + b2b          (1x1, C -> B)
//   t3  = elu(W2 (*) t2 + b3a) + b3b                                      (3x3x3 circular, B -> B)
//   x  <- scale * (W3 t3) + b4 + x                                        (1x1, B -> C)
//
// The residual stream stays fp32 between the blocks of the stack (the reference's blocks return
// fp32 under fp16 autocast: `out * self.scale` promotes); input and output are the caller's
// storage dtype.  The forward saves every block's input x and its t2 / t3 (fp32) to `saved`;
// the backward walks the blocks in reverse from them, writes gx and accumulates (+=) every
// parameter gradient of every block.  One workgroup owns all of it, so each gradient entry has
// exactly one adder and the scalar sums are fixed-order: deterministic.  Each block's weights
// are staged into LDS while the previous block computes (register prefetch).
#include "engines.h"

#include <algorithm>

namespace vq3d {

namespace {

constexpr int NT = 1024;                   // one workgroup, 16 waves
constexpr int MAXV = 256, MAXC = 32, MAXB = 16;
constexpr int NPRM = 11;                   // per block: w1, w2, w3, b1a, b1b, b2a, b2b, b3a, b3b, scale, b4
constexpr int WMAX = MAXB * MAXC * 2 + MAXB * MAXB * 27;

struct SkArgs {
    int nv, C, B, H, W, D;  // voxels (batch folded in), channels, branch, grid
    int nblk;
    int PC, PB;             // LDS row pitches (odd: lanes on consecutive voxels hit distinct banks)
};

__device__ __forceinline__ int nbr(const SkArgs &a, int v, int tap, int sgn) {
    const int kd = tap % 3, kw = (tap / 3) % 3, kh = tap / 9;
    int d = v % a.D, t = v / a.D;
    int w = t % a.W;
    t /= a.W;
    int h = t % a.H;
    const int b = t / a.H;
    h += sgn * (kh - 1);
    w += sgn * (kw - 1);
    d += sgn * (kd - 1);
    h = h < 0 ? h + a.H : (h >= a.H ? h - a.H : h);
    w = w < 0 ? w + a.W : (w >= a.W ? w - a.W : w);
    d = d < 0 ? d + a.D : (d >= a.D ? d - a.D : d);
    return ((b * a.H + h) * a.W + w) * a.D + d;
}

__device__ __forceinline__ float elu_d_act(float t, float b) {  // elu'(z) from t = elu(z) + b
    const float z1 = t - b;
    return z1 > 0.f ? 1.f : z1 + 1.f;
}

struct Scal {
    float b1a, b1b, b2a, b2b, b3a, b3b, sc, b4;
};
__device__ __forceinline__ Scal scal_of(const float *const *t) {
    return Scal{*t[3], *t[4], *t[5], *t[6], *t[7], *t[8], *t[9], *t[10]};
}

// LDS weight image of one block: w1s [C][B] (o fastest), w3s [B][C] (co fastest), w2s
// [tap][ci][co] (co fastest); `n` = total floats.  Prefetched into registers (<= 8 per thread)
// from the nn.Conv3d tensors, then stored.
struct WLd {
    float v[(WMAX + NT - 1) / NT];
    __device__ __forceinline__ void load(const SkArgs &a, const float *const *t) {
        const int nB1 = a.B * a.C, nB2 = a.B * a.B * 27;
#pragma unroll
        for (int u = 0; u < (WMAX + NT - 1) / NT; ++u) {
            const int i = threadIdx.x + u * NT;
            float x = 0.f;
            if (i < nB1) x = t[0][i];                       // W1 [o][c]
            else if (i < 2 * nB1) x = t[2][i - nB1];        // W3 [co][o]
            else if (i < 2 * nB1 + nB2) x = t[1][i - 2 * nB1];  // W2 [co][ci][tap]
            v[u] = x;
        }
    }
    __device__ __forceinline__ void store(const SkArgs &a, float *w1s, float *w3s, float *w2s) const {
        const int nB1 = a.B * a.C, nB2 = a.B * a.B * 27;
#pragma unroll
        for (int u = 0; u < (WMAX + NT - 1) / NT; ++u) {
            const int i = threadIdx.x + u * NT;
            if (i < nB1) {
                const int o = i / a.C, c = i - o * a.C;
                w1s[c * a.B + o] = v[u];
            } else if (i < 2 * nB1) {
                const int j = i - nB1, co = j / a.B, o = j - co * a.B;
                w3s[o * a.C + co] = v[u];
            } else if (i < 2 * nB1 + nB2) {
                const int j = i - 2 * nB1, tap = j % 27, r = j / 27, ci = r % a.B, co = r / a.B;
                w2s[(tap * a.B + ci) * a.B + co] = v[u];
            }
        }
    }
};

struct Lds {
    float *xs, *us, *t2s, *t3s, *gs, *z3s, *z1s, *w1s, *w3s, *w2s, *red;
    short *nb;
};

__device__ __forceinline__ Lds carve(const SkArgs &a, char *smem, bool bwd) {
    Lds l;
    float *p = reinterpret_cast<float *>(smem);
    auto take = [&](int n) {
        float *r = p;
        p += (n + 3) & ~3;
        return r;
    };
    l.w2s = take(a.B * a.B * 27);
    l.w1s = take(a.B * a.C);
    l.w3s = take(a.B * a.C);
    l.xs = take(a.nv * a.PC);
    l.us = take(a.nv * a.PC);
    l.t2s = take(a.nv * a.PB);
    l.t3s = take(a.nv * a.PB);
    l.red = take(16 * 8);
    l.gs = l.z3s = l.z1s = nullptr;
    if (bwd) {
        l.gs = take(a.nv * a.PC);
        l.z3s = take(a.nv * a.PB);
        l.z1s = take(a.nv * a.PB);
    }
    l.nb = reinterpret_cast<short *>(p);
    return l;
}

size_t lds_bytes(const SkArgs &a, bool bwd) {
    auto r4 = [](int n) { return size_t((n + 3) & ~3); };
    size_t f = r4(a.B * a.B * 27) + 2 * r4(a.B * a.C) + 2 * r4(a.nv * a.PC) + 2 * r4(a.nv * a.PB) + 16 * 8;
    if (bwd) f += r4(a.nv * a.PC) + 2 * r4(a.nv * a.PB);
    return f * 4 + size_t(a.nv) * 27 * 2;
}

// fixed-order sums of 8 per-thread partials over the workgroup (all threads get them)
__device__ __forceinline__ void sum8(float (&s)[8], float *red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = wave_sum(s[k]);
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 8; ++k) red[wid * 8 + k] = s[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float t = 0.f;
        for (int w = 0; w < NT / 64; ++w) t += red[w * 8 + k];
        s[k] = t;
    }
}

// t3[v][o] (4 outputs from o0) = W2 (*) src over the neighbours of v; sgn -1: transposed taps
// over [tap][ci][co] with the roles of ci / co swapped (backward-data)
template <bool DGRAD>
__device__ __forceinline__ void conv4(const SkArgs &a, const Lds &l, const float *src, int v, int o0, float (&acc)[4]) {
    acc[0] = acc[1] = acc[2] = acc[3] = 0.f;
    for (int tap = 0; tap < 27; ++tap) {
        const float *nrow = src + int(l.nb[v * 27 + (DGRAD ? 26 - tap : tap)]) * a.PB;
        const float *wt = l.w2s + tap * a.B * a.B;
        for (int c = 0; c < a.B; ++c) {
            const float u = nrow[c];
            if (!DGRAD) {
                const float4 w = *reinterpret_cast<const float4 *>(wt + c * a.B + o0);  // [ci = c][co = o0..]
                acc[0] = fmaf(u, w.x, acc[0]);
                acc[1] = fmaf(u, w.y, acc[1]);
                acc[2] = fmaf(u, w.z, acc[2]);
                acc[3] = fmaf(u, w.w, acc[3]);
            } else {  // gt2[v][ci = o0 + j] += W2[co = c][ci][tap] gz3[nbr(v, -tap)][c]
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = fmaf(u, wt[(o0 + j) * a.B + c], acc[j]);
            }
        }
    }
}

// ============================================================================================ forward
template <typename T>
__global__ __launch_bounds__(NT) void k_stack_fwd(SkArgs a, const T *__restrict__ x, const float *const *tab,
                                                  T *__restrict__ out, float *__restrict__ saved) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Lds l = carve(a, smem, false);
    const int tid = threadIdx.x;
    const int nvc = a.nv * a.C, nvb = a.nv * a.B, nog = a.B / 4;
    const size_t stride = size_t(a.nv) * (a.C + 2 * a.B);
    for (int i = tid; i < a.nv * 27; i += NT) l.nb[i] = short(nbr(a, i / 27, i % 27, 1));
    for (int i = tid; i < nvc; i += NT) l.xs[(i / a.C) * a.PC + i % a.C] = ld(x + i);
    WLd wl;
    wl.load(a, tab);
    for (int blk = 0; blk < a.nblk; ++blk) {
        const float *const *t = tab + blk * NPRM;
        const Scal s = scal_of(t);
        float *sx = saved + blk * stride, *st2 = sx + nvc, *st3 = st2 + nvb;
        __syncthreads();  // previous block's readers of the weight image / xs are done
        wl.store(a, l.w1s, l.w3s, l.w2s);
        if (blk + 1 < a.nblk) wl.load(a, tab + (blk + 1) * NPRM);
        for (int i = tid; i < nvc; i += NT) {
            const int v = i / a.C, c = i - v * a.C;
            const float xv = l.xs[v * a.PC + c];
            sx[i] = xv;
            l.us[v * a.PC + c] = elu(xv + s.b1a) + s.b1b;
        }
        __syncthreads();
        // t2 (items: voxel x 4 outputs)
        for (int i = tid; i < a.nv * nog; i += NT) {
            const int v = i % a.nv, o0 = (i / a.nv) * 4;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            for (int c = 0; c < a.C; ++c) {
                const float u = l.us[v * a.PC + c];
                const float4 w = *reinterpret_cast<const float4 *>(l.w1s + c * a.B + o0);
                acc[0] = fmaf(u, w.x, acc[0]);
                acc[1] = fmaf(u, w.y, acc[1]);
                acc[2] = fmaf(u, w.z, acc[2]);
                acc[3] = fmaf(u, w.w, acc[3]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float tv = elu(acc[j] + s.b2a) + s.b2b;
                l.t2s[v * a.PB + o0 + j] = tv;
                st2[v * a.B + o0 + j] = tv;
            }
        }
        __syncthreads();
        // t3
        for (int i = tid; i < a.nv * nog; i += NT) {
            const int v = i % a.nv, o0 = (i / a.nv) * 4;
            float acc[4];
            conv4<false>(a, l, l.t2s, v, o0, acc);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float tv = elu(acc[j] + s.b3a) + s.b3b;
                l.t3s[v * a.PB + o0 + j] = tv;
                st3[v * a.B + o0 + j] = tv;
            }
        }
        __syncthreads();
        // x <- scale * W3 t3 + b4 + x (items: voxel x 4 channels)
        for (int i = tid; i < a.nv * (a.C / 4); i += NT) {
            const int v = i % a.nv, c0 = (i / a.nv) * 4;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            for (int o = 0; o < a.B; ++o) {
                const float u = l.t3s[v * a.PB + o];
                const float4 w = *reinterpret_cast<const float4 *>(l.w3s + o * a.C + c0);
                acc[0] = fmaf(u, w.x, acc[0]);
                acc[1] = fmaf(u, w.y, acc[1]);
                acc[2] = fmaf(u, w.z, acc[2]);
                acc[3] = fmaf(u, w.w, acc[3]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) l.xs[v * a.PC + c0 + j] += acc[j] * s.sc + s.b4;
        }
    }
    __syncthreads();
    for (int i = tid; i < nvc; i += NT) st(out + i, l.xs[(i / a.C) * a.PC + i % a.C]);
}

// ============================================================================================ backward
template <typename T>
__global__ __launch_bounds__(NT) void k_stack_bwd(SkArgs a, const T *__restrict__ g, const float *const *tab,
                                                  float *const *gtab, const float *__restrict__ saved,
                                                  T *__restrict__ gx) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Lds l = carve(a, smem, true);
    const int tid = threadIdx.x;
    const int nvc = a.nv * a.C, nvb = a.nv * a.B, nog = a.B / 4, ncg = a.C / 4;
    const size_t stride = size_t(a.nv) * (a.C + 2 * a.B);
    for (int i = tid; i < a.nv * 27; i += NT) l.nb[i] = short(nbr(a, i / 27, i % 27, 1));
    for (int i = tid; i < nvc; i += NT) l.gs[(i / a.C) * a.PC + i % a.C] = ld(g + i);
    WLd wl;
    wl.load(a, tab + (a.nblk - 1) * NPRM);
    for (int blk = a.nblk - 1; blk >= 0; --blk) {
        const float *const *t = tab + blk * NPRM;
        float *const *gt = gtab + blk * NPRM;
        const Scal s = scal_of(t);
        const float *sx = saved + blk * stride, *st2 = sx + nvc, *st3 = st2 + nvb;
        __syncthreads();
        wl.store(a, l.w1s, l.w3s, l.w2s);
        if (blk > 0) wl.load(a, tab + (blk - 1) * NPRM);
        // saved block input -> u1 (us) and elu'(x + b1a) (xs); t2, t3
        for (int i = tid; i < nvc; i += NT) {
            const int v = i / a.C, c = i - v * a.C;
            const float z = sx[i] + s.b1a;
            const float e = z > 0.f ? 1.f : expf(z);
            l.us[v * a.PC + c] = (z > 0.f ? z : e - 1.f) + s.b1b;
            l.xs[v * a.PC + c] = e;
        }
        for (int i = tid; i < nvb; i += NT) {
            const int v = i / a.B, o = i - v * a.B;
            l.t2s[v * a.PB + o] = st2[i];
            l.t3s[v * a.PB + o] = st3[i];
        }
        __syncthreads();
        // scalar partials: 0 b4, 1 scale, 2 b3b, 3 b3a, 4 b2b, 5 b2a, 6 b1b, 7 b1a
        float ps[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // gz3 = scale W3^T g * elu'(t3 - b3b)
        for (int i = tid; i < a.nv * nog; i += NT) {
            const int v = i % a.nv, o0 = (i / a.nv) * 4;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            for (int c = 0; c < a.C; ++c) {
                const float gv = l.gs[v * a.PC + c];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = fmaf(gv, l.w3s[(o0 + j) * a.C + c], acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float g3 = acc[j] * s.sc;
                const float z = g3 * elu_d_act(l.t3s[v * a.PB + o0 + j], s.b3b);
                ps[2] += g3;
                ps[3] += z;
                l.z3s[v * a.PB + o0 + j] = z;
            }
        }
        // W3 gradient (entries co x o), dscale = sum W3 . G3, db4 = sum g
        for (int e = tid; e < a.C * a.B; e += NT) {
            const int co = e / a.B, o = e - co * a.B;
            float acc = 0.f, gsum = 0.f;
            for (int v = 0; v < a.nv; ++v) {
                const float gv = l.gs[v * a.PC + co];
                acc = fmaf(gv, l.t3s[v * a.PB + o], acc);
                if (o == 0) gsum += gv;
            }
            gt[2][e] += s.sc * acc;
            ps[1] = fmaf(l.w3s[o * a.C + co], acc, ps[1]);
            ps[0] += gsum;
        }
        __syncthreads();
        // gt2 = W2^T (*) gz3 -> gz1 = gt2 * elu'(t2 - b2b)
        for (int i = tid; i < a.nv * nog; i += NT) {
            const int v = i % a.nv, o0 = (i / a.nv) * 4;
            float acc[4];
            conv4<true>(a, l, l.z3s, v, o0, acc);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float z = acc[j] * elu_d_act(l.t2s[v * a.PB + o0 + j], s.b2b);
                ps[4] += acc[j];
                ps[5] += z;
                l.z1s[v * a.PB + o0 + j] = z;
            }
        }
        // W2 gradient: items (tap, ci group, co group) x 16 entries, sum over voxels
        for (int i = tid; i < 27 * nog * nog; i += NT) {
            const int tap = i % 27, r = i / 27, cig = r % nog, cog = r / nog;
            float acc[4][4];
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[p][q] = 0.f;
            for (int v = 0; v < a.nv; ++v) {
                const float *zr = l.z3s + v * a.PB + cog * 4;
                const float *tr = l.t2s + int(l.nb[v * 27 + tap]) * a.PB + cig * 4;
                float zz[4], tt[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    zz[q] = zr[q];
                    tt[q] = tr[q];
                }
#pragma unroll
                for (int p = 0; p < 4; ++p)
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[p][q] = fmaf(zz[p], tt[q], acc[p][q]);
            }
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    gt[1][((cog * 4 + p) * a.B + cig * 4 + q) * 27 + tap] += acc[p][q];
        }
        __syncthreads();
        // gx = g + (W1^T gz1) * elu'(x + b1a) (in place over g); W1 gradient
        for (int i = tid; i < a.nv * ncg; i += NT) {
            const int v = i % a.nv, c0 = (i / a.nv) * 4;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            for (int o = 0; o < a.B; ++o) {
                const float z = l.z1s[v * a.PB + o];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = fmaf(z, l.w1s[(c0 + j) * a.B + o], acc[j]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float e = l.xs[v * a.PC + c0 + j];
                ps[6] += acc[j];
                ps[7] += acc[j] * e;
                l.gs[v * a.PC + c0 + j] += acc[j] * e;
            }
        }
        for (int e = tid; e < a.B * a.C; e += NT) {
            const int o = e / a.C, c = e - o * a.C;
            float acc = 0.f;
            for (int v = 0; v < a.nv; ++v) acc = fmaf(l.z1s[v * a.PB + o], l.us[v * a.PC + c], acc);
            gt[0][e] += acc;
        }
        sum8(ps, l.red);
        if (tid == 0) {
            *gt[10] += ps[0];
            *gt[9] += ps[1];
            *gt[8] += ps[2];
            *gt[7] += ps[3];
            *gt[6] += ps[4];
            *gt[5] += ps[5];
            *gt[4] += ps[6];
            *gt[3] += ps[7];
        }
    }
    __syncthreads();
    for (int i = tid; i < nvc; i += NT) st(gx + i, l.gs[(i / a.C) * a.PC + i % a.C]);
}

// ============================================================================================ matrix cores
// bf16 storage with (C, B) = (32, 16) (the published top level): every contraction of the
// block on v_mfma_f32_16x16x32_bf16 (t2, t3, the block output, and in the backward gz3, the
// transposed conv, gx and the three weight gradients with the voxels as the reduction axis).
// Rounding points are the unfused bf16 path's (u1, t2, t3, gz3, gz1 rounded to bf16 as matrix
// operands, fp32 accumulation); the residual stream and the gradient stream stay fp32.
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int MC = 32, MB = 16;            // channels, branch
constexpr int PF = 36, PU = 40, PT = 24;   // row pitches: fp32 streams, u1 (bf16), branch tensors (bf16)
constexpr int MAXVM = 128;

__device__ __forceinline__ f32x4 mfma(hx8 a, hx8 b, f32x4 c) {
    return VQ3D_MFMA_16X16X32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ hx8 pack8(const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = uint32_t(f2h(v[2 * j])) | (uint32_t(f2h(v[2 * j + 1])) << 16);
    return __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]});
}
__device__ __forceinline__ hx8 rd8(const h16_t *p) { return __builtin_bit_cast(hx8, *reinterpret_cast<const uint4 *>(p)); }
__device__ __forceinline__ hx8 zero8() { return __builtin_bit_cast(hx8, uint4{0u, 0u, 0u, 0u}); }
// 8 bf16 at p[j * stride] (LDS)
__device__ __forceinline__ hx8 gat8(const h16_t *p, int stride) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = uint32_t(p[2 * j * stride]) | (uint32_t(p[(2 * j + 1) * stride]) << 16);
    return __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]});
}
// 8 fp32 at p[j * stride] (LDS), rounded to bf16
__device__ __forceinline__ hx8 gat8f(const float *p, int stride) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[j * stride];
    return pack8(v);
}
// 8 consecutive fp32 (16-B aligned), rounded to bf16
__device__ __forceinline__ hx8 rd8f(const float *p) {
    const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    return pack8(v);
}

struct Mk {
    float *xs, *gs, *part, *w;   // fp32: residual / gradient stream, conv partials [2][nv][16], weights
    h16_t *fr;                  // the block's weights as packed bf16 MFMA B fragments (FR_* below)
    h16_t *u1, *t2, *t3, *z3, *z1;
    short *nb;
    float *red;
};

// weight image (fp32): w1 [o][c] at 0, w3 [co][o] at 512, w2 [co][ci][tap] at 1024 (torch order)
constexpr int W1O = 0, W3O = MB * MC, W2O = 2 * MB * MC, WN = W2O + MB * MB * 27;

// Packed B-fragment images (bf16, [k-step / n-tile][lane = kb * 16 + n][8]; one 16-B LDS read per
// lane, no strided fp32 gathers -- those were bank-conflict bound).  Forward: FA = W1 (t2:
// k = c, n = o), FB = W2 (14 tap-pair k-steps: k = (tap, ci), n = co), FC = W3 (2 n-tiles: k = o
// (+ zero half), n = co).  Backward: FA = W3 (gz3: k = co, n = o), FB = W2 transposed (k = (tap,
// co), n = ci), FC = W1 (gx, 2 n-tiles: k = o (+ zero half), n = c).  Slots past tap 26 and the
// zero k-halves are cleared once per kernel.
constexpr int FRT = 512, FR_A = 0, FR_B = FRT, FR_C = 15 * FRT, FR_N = 17 * FRT;
__device__ __forceinline__ int frpos(int ktile, int kb, int n, int j) { return ktile * FRT + ((kb * 16 + n) << 3) + j; }

// weight element (torch-order image index i, value v) -> its fragment slots
template <bool BWD>
__device__ __forceinline__ void frag_store(h16_t *fr, int i, float v) {
    const h16_t b = f2h(v);
    if (i < W3O) {  // W1 [o][c]
        const int o = i / MC, c = i - o * MC;
        if (!BWD) fr[FR_A + frpos(0, c >> 3, o, c & 7)] = b;
        else fr[FR_C + frpos(c >> 4, o >> 3, c & 15, o & 7)] = b;
    } else if (i < W2O) {  // W3 [co][o]
        const int e = i - W3O, co = e / MB, o = e - co * MB;
        if (!BWD) fr[FR_C + frpos(co >> 4, o >> 3, co & 15, o & 7)] = b;
        else fr[FR_A + frpos(0, co >> 3, o, co & 7)] = b;
    } else {  // W2 [co][ci][tap]
        const int e = i - W2O, tap = e % 27, r = e / 27, ci = r % MB, co = r / MB;
        const int kc = BWD ? co : ci, n = BWD ? ci : co;
        fr[FR_B + frpos(tap >> 1, 2 * (tap & 1) + (kc >> 3), n, kc & 7)] = b;
    }
}
__device__ __forceinline__ void frag_zero(h16_t *fr) {
    // tap 27 (k-step 13, kb 2 / 3) and the k-halves o >= 16 of the two FC tiles (kb 2 / 3)
    for (int i = threadIdx.x; i < 3 * 32 * 8; i += NT) {
        const int t = i / 256, r = i - t * 256, lane = 32 + (r >> 3), j = r & 7;
        fr[(t == 0 ? FR_B + 13 * FRT : FR_C + (t - 1) * FRT) + lane * 8 + j] = 0;
    }
}
__device__ __forceinline__ hx8 frag(const h16_t *fr, int ktile, int lane) {
    return __builtin_bit_cast(hx8, *reinterpret_cast<const uint4 *>(fr + ktile * FRT + lane * 8));
}

__device__ __forceinline__ Mk carve_m(int nv, char *smem) {
    Mk m;
    float *p = reinterpret_cast<float *>(smem);
    m.w = p;
    p += WN;
    m.xs = p;
    p += nv * PF;
    m.gs = p;
    p += nv * PF;
    m.part = p;
    p += 2 * nv * MB;
    m.red = p;
    p += 16 * 8;
    h16_t *q = reinterpret_cast<h16_t *>(p);
    m.fr = q;
    q += FR_N;
    m.u1 = q;
    q += nv * PU;
    m.t2 = q;
    q += nv * PT + 32;
    m.t3 = q;
    q += nv * PT + 32;
    m.z3 = q;
    q += nv * PT + 32;
    m.z1 = q;
    q += nv * PT + 32;
    m.nb = reinterpret_cast<short *>(q);
    return m;
}
size_t lds_m(int nv) {
    return size_t(WN + 2 * nv * PF + 2 * nv * MB + 16 * 8) * 4 + size_t(FR_N + nv * PU + 4 * (nv * PT + 32)) * 2 +
           size_t(nv) * 27 * 2;
}

struct WReg {  // register prefetch of one block's weights (fp32, torch order)
    float v[(WN + NT - 1) / NT];
    __device__ __forceinline__ void load(const float *w1, const float *w2, const float *w3) {
#pragma unroll
        for (int u = 0; u < (WN + NT - 1) / NT; ++u) {
            const int i = min(int(threadIdx.x) + u * NT, WN - 1);
            v[u] = i < W3O ? w1[i] : (i < W2O ? w3[i - W3O] : w2[i - W2O]);
        }
    }
    template <bool BWD>
    __device__ __forceinline__ void store(float *w, h16_t *fr) const {
#pragma unroll
        for (int u = 0; u < (WN + NT - 1) / NT; ++u) {
            const int i = threadIdx.x + u * NT;
            if (i < WN) {
                w[i] = v[u];
                frag_store<BWD>(fr, i, v[u]);
            }
        }
    }
};

// Every block's packed fragment image, built once per run by k_stackm_pack (in parallel, one
// workgroup per block) so the chain kernels only copy 17 KiB per block from L2 into LDS (two
// 16-byte pieces per thread, fetched a block ahead) instead of converting and scattering the fp32
// weights on the chain's critical path (that staging was ~45 % of the forward chain's time).
constexpr int FR_CH = FR_N * 2 / 16;  // 16-byte pieces per image
constexpr int FR_CPT = (FR_CH + NT - 1) / NT;
static_assert((FR_N * 2) % 16 == 0, "image pieces");
template <bool BWD>
__global__ __launch_bounds__(NT) void k_stackm_pack(const float *const *tab, h16_t *__restrict__ img) {
    const int blk = blockIdx.x;
    const float *w1 = tab[blk * NPRM + 0], *w2 = tab[blk * NPRM + 1], *w3 = tab[blk * NPRM + 2];
    h16_t *fr = img + size_t(blk) * FR_N;
    for (int i = threadIdx.x; i < WN; i += NT)
        frag_store<BWD>(fr, i, i < W3O ? w1[i - W1O] : (i < W2O ? w3[i - W3O] : w2[i - W2O]));
    frag_zero(fr);
}
struct ImgReg {  // register prefetch of one block's packed image
    u32x4 v[FR_CPT];
    __device__ __forceinline__ void load(const h16_t *img, int blk) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(img + size_t(blk) * FR_N);
#pragma unroll
        for (int u = 0; u < FR_CPT; ++u) v[u] = src[min(int(threadIdx.x) + u * NT, FR_CH - 1)];
    }
    __device__ __forceinline__ void store(h16_t *fr) const {
#pragma unroll
        for (int u = 0; u < FR_CPT; ++u) {
            const int i = threadIdx.x + u * NT;
            if (i < FR_CH) reinterpret_cast<u32x4 *>(fr)[i] = v[u];
        }
    }
};

// A block's parameter-table row, lane-distributed in VECTOR registers: lane k (< NPRM) holds
// the row's k-th pointer, and after deref() lanes 3 .. 10 hold the scalar values.  Rows are
// fetched one block ahead, so the waits ride vmcnt a whole block after the issue (scalar loads
// would share lgkmcnt with every LDS access and stall at the next LDS wait).
__device__ __forceinline__ const float *row_ptr(const float *const *tab, int j, int lane) {
    return tab[j * NPRM + min(lane, NPRM - 1)];
}
__device__ __forceinline__ float *row_ptr(float *const *tab, int j, int lane) {
    return tab[j * NPRM + min(lane, NPRM - 1)];
}
template <typename P>
__device__ __forceinline__ P *bcast_ptr(P *p, int k) {
    const uint64_t u = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(u), k), hi = __builtin_amdgcn_readlane(uint32_t(u >> 32), k);
    return reinterpret_cast<P *>((uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ float bcastf(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
__device__ __forceinline__ Scal scal_lanes(float v) {
    return Scal{bcastf(v, 3), bcastf(v, 4), bcastf(v, 5), bcastf(v, 6),
                bcastf(v, 7), bcastf(v, 8), bcastf(v, 9), bcastf(v, 10)};
}

// conv2 (t3 from t2) or its transpose (gt2 from gz3): M-tile mt, k-steps of tap pairs
// [ks0, ks0 + 7); B[k][n] built from the fp32 image: forward n = co, k = (tap, ci); transposed
// n = ci, k = (tap, co) with the flipped tap
template <bool T>
__device__ __forceinline__ f32x4 conv_half(const Mk &m, const h16_t *src, int mt, int ks0, int lane) {
    const int row = lane & 15, kb = lane >> 4, v = mt * 16 + row;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // all 7 neighbour indices, then all 7 operand rows, then the MFMAs: one LDS round trip per
    // stage instead of two per k-step on the chain's critical path
    int nbi[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const int tap = 2 * (ks0 + k) + (kb >> 1);
        nbi[k] = tap < 27 ? int(m.nb[v * 27 + (T ? 26 - tap : tap)]) : -1;
    }
    hx8 af[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) af[k] = nbi[k] >= 0 ? rd8(src + nbi[k] * PT + 8 * (kb & 1)) : zero8();
#pragma unroll
    for (int k = 0; k < 7; ++k) acc = mfma(af[k], frag(m.fr + FR_B, ks0 + k, lane), acc);
    return acc;
}

__global__ __launch_bounds__(NT) void k_stackm_fwd(SkArgs a, const h16_t *__restrict__ x, const float *const *tab,
                                                   h16_t *__restrict__ out, float *__restrict__ saved,
                                                   const h16_t *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Mk m = carve_m(a.nv, smem);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int nv = a.nv, nmt = nv / 16, nvc = nv * MC, nvb = nv * MB;
    const size_t stride = size_t(nv) * (MC + 2 * MB);
    for (int i = tid; i < nv * 27; i += NT) m.nb[i] = short(nbr(a, i / 27, i % 27, 1));
    for (int i = tid; i < nvc; i += NT) m.xs[(i / MC) * PF + i % MC] = ld(x + i);
    for (int i = tid; i < 32; i += NT) m.t3[nv * PT + i] = 0;  // zero tail / row pads read by the fragments
    for (int i = tid; i < nv * (PT - MB); i += NT) m.t3[(i / (PT - MB)) * PT + MB + i % (PT - MB)] = 0;
    ImgReg ir;
    const float *pc = row_ptr(tab, 0, lane);
    float vc = *pc;
    ir.load(img, 0);
    const float *pn = row_ptr(tab, min(1, a.nblk - 1), lane);
    for (int blk = 0; blk < a.nblk; ++blk) {
        const Scal s = scal_lanes(vc);
        float *sx = saved + blk * stride, *st2 = sx + nvc, *st3 = st2 + nvb;
        __syncthreads();
        ir.store(m.fr);
        // the next block's weights and scalars, and the row after it
        if (blk + 1 < a.nblk) {
            ir.load(img, blk + 1);
            vc = *pn;
            pn = row_ptr(tab, min(blk + 2, a.nblk - 1), lane);
        }
        for (int i = tid; i < nvc; i += NT) {
            const int v = i / MC, c = i - v * MC;
            const float xv = m.xs[v * PF + c];
            sx[i] = xv;
            m.u1[v * PU + c] = f2h(elu(xv + s.b1a) + s.b1b);
        }
        __syncthreads();
        // t2: M-tile per wave, K = 32 channels, N = 16
        if (wave < nmt) {
            const f32x4 acc = mfma(rd8(m.u1 + (wave * 16 + row) * PU + 8 * kb), frag(m.fr + FR_A, 0, lane),
                                   f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int v = wave * 16 + 4 * kb + j;
                const h16_t tv = f2h(elu(acc[j] + s.b2a) + s.b2b);
                m.t2[v * PT + row] = tv;
                st2[v * MB + row] = ld(&tv);
            }
        }
        __syncthreads();
        // t3: (M-tile, half of the 14 tap-pair k-steps) per wave, partials summed in LDS
        if (wave < 2 * nmt) {
            const int mt = wave % nmt, half = wave / nmt;
            const f32x4 acc = conv_half<false>(m, m.t2, mt, 7 * half, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) m.part[(half * nv + mt * 16 + 4 * kb + j) * MB + row] = acc[j];
        }
        __syncthreads();
        for (int i = tid; i < nvb; i += NT) {
            const int v = i / MB, o = i - v * MB;
            const h16_t tv = f2h(elu(m.part[i] + m.part[nvb + i] + s.b3a) + s.b3b);
            m.t3[v * PT + o] = tv;
            st3[i] = ld(&tv);
        }
        __syncthreads();
        // x += scale * W3 t3 + b4: M-tile x 2 N-tiles per wave, K = 16 (+ zero half)
        if (wave < 2 * nmt) {
            const int mt = wave % nmt, nt = wave / nmt;
            const f32x4 acc = mfma(rd8(m.t3 + (mt * 16 + row) * PT + 8 * kb), frag(m.fr + FR_C, nt, lane),
                                   f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int j = 0; j < 4; ++j) m.xs[(mt * 16 + 4 * kb + j) * PF + 16 * nt + row] += acc[j] * s.sc + s.b4;
        }
    }
    __syncthreads();
    for (int i = tid; i < nvc; i += NT) out[i] = f2h(m.xs[(i / MC) * PF + i % MC]);
}

// SPLIT: the chain computes only the gradient stream and the scalar sums that ride it (gz3, gt2,
// gz1, gx; b1a .. b4 but scale) and records each block's bf16 matrix operands (g, gz3, gz1) in
// `rec`; the W1 / W2 / W3 and scale gradients, which nothing downstream in the chain needs, are
// k_stackm_wgrad's, one workgroup per block in parallel after the chain.
template <bool SPLIT>
__global__ __launch_bounds__(NT) void k_stackm_bwd(SkArgs a, const h16_t *__restrict__ g, const float *const *tab,
                                                   float *const *gtab, const float *__restrict__ saved,
                                                   h16_t *__restrict__ gx, h16_t *__restrict__ rec,
                                                   const h16_t *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const Mk m = carve_m(a.nv, smem);
    const int tid0 = threadIdx.x;
    const int nv = a.nv, nmt = nv / 16, nks = nv / 32, nvc = nv * MC, nvb = nv * MB;
    const size_t stride = size_t(nv) * (MC + 2 * MB);
    const int tid = tid0, lane = tid0 & 63;
    for (int i = tid; i < nv * 27; i += NT) m.nb[i] = short(nbr(a, i / 27, i % 27, 1));
    for (int i = tid; i < nvc; i += NT) m.gs[(i / MC) * PF + i % MC] = ld(g + i);
    for (int i = tid; i < nv * (PT - MB); i += NT) {  // zero row pads / tail read by the gx fragments
        const int v = i / (PT - MB), e = MB + i % (PT - MB);
        m.z1[v * PT + e] = 0;
    }
    for (int i = tid; i < 32; i += NT) m.z1[nv * PT + i] = 0;
    if constexpr (!SPLIT) frag_zero(m.fr);
    // prefetched one block ahead (the walk is in reverse): weights (SPLIT: the packed image, else
    // the fp32 weights, whose W3 the fused scale gradient reads), scalars, gradient pointers,
    // the saved x / t2 / t3; the current block's old gradient values at its top
    constexpr int SX = MAXVM * MC / NT, SB = MAXVM * MB / NT;
    WReg wr;
    ImgReg ir;
    const int last = a.nblk - 1;
    const float *pc = row_ptr(tab, last, lane);
    float vc = *pc;
    if constexpr (SPLIT) ir.load(img, last);
    else wr.load(bcast_ptr(pc, 0), bcast_ptr(pc, 1), bcast_ptr(pc, 2));
    const float *pn = row_ptr(tab, max(last - 1, 0), lane);
    float *gc = row_ptr(gtab, last, lane);
    float svx[SX], sv2[SB], sv3[SB];
    auto load_saved = [&](int b) {
        const float *sx = saved + b * stride, *st2 = sx + nvc, *st3 = st2 + nvb;
#pragma unroll
        for (int u = 0; u < SX; ++u) svx[u] = sx[min(tid + u * NT, nvc - 1)];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            sv2[u] = st2[min(tid + u * NT, nvb - 1)];
            sv3[u] = st3[min(tid + u * NT, nvb - 1)];
        }
    };
    load_saved(last);
    for (int blk = last; blk >= 0; --blk) {
        // the thread / lane indices are re-derived from an opaque copy each block, so the
        // compiler recomputes the per-phase LDS addresses instead of hoisting ~60 loop-invariant
        // ones out of the block loop and spilling them
        int tl = tid0;
        asm volatile("" : "+v"(tl));
        const int tid = tl, lane = tl & 63, wave = __builtin_amdgcn_readfirstlane(tl >> 6), row = lane & 15,
                  kb = lane >> 4;
        const Scal s = scal_lanes(vc);
        // this block's gradient pointers (fetched a block ago) and their old values: W3 entries of
        // waves nmt, nmt + 1, W2 entries of taps wave / wave + 16, W1 entries of waves 0, 1, the
        // scalars on lanes 3 .. 10 of wave 0 (every load unconditional, clamped indices)
        float *gw1 = bcast_ptr(gc, 0), *gw2 = bcast_ptr(gc, 1), *gw3 = bcast_ptr(gc, 2);
        float o3[4] = {}, o2[2][4] = {}, o1[4] = {};
        const int ct = min(max(wave - nmt, 0), 1), nt1 = min(wave, 1);
        if constexpr (!SPLIT) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o3[j] = gw3[(16 * ct + 4 * kb + j) * MB + row];
#pragma unroll
                for (int q = 0; q < 2; ++q) o2[q][j] = gw2[((4 * kb + j) * MB + row) * 27 + min(wave + 16 * q, 26)];
            }
        }
        h16_t *rg = rec + size_t(blk) * nv * (MC + 2 * MB), *rz3 = rg + nvc, *rz1 = rz3 + nvb;
        const float osc = *gc;
        float *const gsc = gc;  // lanes 3 .. 10: this block's scalar-gradient pointers
        if (blk > 0) gc = row_ptr(gtab, blk - 1, lane);
        __syncthreads();
        {
            if constexpr (SPLIT) ir.store(m.fr);
            else wr.store<true>(m.w, m.fr);
        }
#pragma unroll
        for (int u = 0; u < SX; ++u) {
            const int i = tid + u * NT;
            if (i < nvc) {
                const int v = i / MC, c = i - v * MC;
                const float z = svx[u] + s.b1a;
                const float e = z > 0.f ? 1.f : expf(z);
                m.u1[v * PU + c] = f2h((z > 0.f ? z : e - 1.f) + s.b1b);
                m.xs[v * PF + c] = e;
            }
        }
#pragma unroll
        for (int u = 0; u < SB; ++u) {
            const int i = tid + u * NT;
            if (i < nvb) {
                const int v = i / MB, o = i - v * MB;
                m.t2[v * PT + o] = f2h(sv2[u]);
                m.t3[v * PT + o] = f2h(sv3[u]);
            }
        }
        __syncthreads();
        float ps[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // b4, scale, b3b, b3a, b2b, b2a, b1b, b1a
        if (wave < nmt) {
            // gz3 = scale W3^T g * elu'(t3 - b3b): K = 32 channels of g, N = 16
            const f32x4 acc = mfma(rd8f(m.gs + (wave * 16 + row) * PF + 8 * kb), frag(m.fr + FR_A, 0, lane),
                                   f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int v = wave * 16 + 4 * kb + j;
                const float g3 = acc[j] * s.sc;
                const float z = g3 * elu_d_act(ld(&m.t3[v * PT + row]), s.b3b);
                ps[2] += g3;
                ps[3] += z;
                m.z3[v * PT + row] = f2h(z);
                if constexpr (SPLIT) rz3[v * MB + row] = f2h(z);
            }
        } else if (!SPLIT && wave < nmt + 2) {
            // W3 gradient: M = co tile (wave - nmt), N = o, K = voxels; dscale = sum W3 . G3
            const int ct = wave - nmt;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            for (int ks = 0; ks < nks; ++ks) {
                const int v0 = ks * 32 + 8 * kb;
                acc = mfma(gat8f(m.gs + v0 * PF + 16 * ct + row, PF), gat8(m.t3 + v0 * PT + row, PT), acc);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = 16 * ct + 4 * kb + j;
                gw3[co * MB + row] = o3[j] + s.sc * acc[j];
                ps[1] = fmaf(m.w[W3O + co * MB + row], acc[j], ps[1]);
            }
        }
        for (int i = tid; i < nvc; i += NT) {
            const float gv = m.gs[(i / MC) * PF + i % MC];
            ps[0] += gv;
            if constexpr (SPLIT) rg[i] = f2h(gv);
        }
        __syncthreads();
        // gt2 = W2^T (*) gz3 (M-tile x half of the k-steps per wave); W2 gradient per tap
        if (wave < 2 * nmt) {
            const int mt = wave % nmt, half = wave / nmt;
            const f32x4 acc = conv_half<true>(m, m.z3, mt, 7 * half, lane);
#pragma unroll
            for (int j = 0; j < 4; ++j) m.part[(half * nv + mt * 16 + 4 * kb + j) * MB + row] = acc[j];
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // M = co, N = ci, K = voxels: taps wave, wave + 16
            const int tap = wave + 16 * q;
            if (SPLIT || tap >= 27) continue;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
            for (int ks = 0; ks < nks; ++ks) {
                const int v0 = ks * 32 + 8 * kb;
                uint32_t w[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int va = v0 + 2 * j, vb = va + 1;
                    w[j] = uint32_t(m.t2[int(m.nb[va * 27 + tap]) * PT + row]) |
                           (uint32_t(m.t2[int(m.nb[vb * 27 + tap]) * PT + row]) << 16);
                }
                acc = mfma(gat8(m.z3 + v0 * PT + row, PT), __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]}),
                           acc);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) gw2[((4 * kb + j) * MB + row) * 27 + tap] = o2[q][j] + acc[j];
        }
        __syncthreads();
        // the next block's weights / scalars / saved tensors and this block's old W1 gradient
        // (issued here, after the register-heavy k^3 phases)
        if (blk > 0) {
            if constexpr (SPLIT) ir.load(img, blk - 1);
            else wr.load(bcast_ptr(pn, 0), bcast_ptr(pn, 1), bcast_ptr(pn, 2));
            vc = *pn;
            pn = row_ptr(tab, max(blk - 2, 0), lane);
            load_saved(blk - 1);
        }
        if constexpr (!SPLIT) {
#pragma unroll
            for (int j = 0; j < 4; ++j) o1[j] = gw1[(4 * kb + j) * MC + 16 * nt1 + row];
        }
        for (int i = tid; i < nvb; i += NT) {
            const int v = i / MB, o = i - v * MB;
            const float g2 = m.part[i] + m.part[nvb + i];
            const float z = g2 * elu_d_act(ld(&m.t2[v * PT + o]), s.b2b);
            ps[4] += g2;
            ps[5] += z;
            m.z1[v * PT + o] = f2h(z);
            if constexpr (SPLIT) rz1[i] = f2h(z);
        }
        __syncthreads();
        if (wave < 2 * nmt) {
            // gx = g + (W1^T gz1) * elu'(x + b1a): M-tile x 2 N-tiles (channels), K = 16 (+ zero half)
            const int mt = wave % nmt, nt = wave / nmt;
            const f32x4 acc = mfma(rd8(m.z1 + (mt * 16 + row) * PT + 8 * kb), frag(m.fr + FR_C, nt, lane),
                                   f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = (mt * 16 + 4 * kb + j) * PF + 16 * nt + row;
                const float e = m.xs[i];
                ps[6] += acc[j];
                ps[7] += acc[j] * e;
                m.gs[i] += acc[j] * e;
            }
        }
        if (!SPLIT && wave < 2) {
            // W1 gradient: M = o, N = channel tile (wave), K = voxels
            const int nt = wave;
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            for (int ks = 0; ks < nks; ++ks) {
                const int v0 = ks * 32 + 8 * kb;
                acc = mfma(gat8(m.z1 + v0 * PT + row, PT), gat8(m.u1 + v0 * PU + 16 * nt + row, PU), acc);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) gw1[(4 * kb + j) * MC + 16 * nt + row] = o1[j] + acc[j];
        }
        sum8(ps, m.red);
        if (wave == 0 && lane >= 3 && lane < NPRM && !(SPLIT && lane == 9)) {  // table slot k gets ps[10 - k]
            float add = ps[0];
#pragma unroll
            for (int k = 3; k < NPRM - 1; ++k) add = lane == k ? ps[10 - k] : add;
            *gsc = osc + add;
        }
    }
    __syncthreads();
    for (int i = tid; i < nvc; i += NT) gx[i] = f2h(m.gs[(i / MC) * PF + i % MC]);
}

// The weight gradients of a SPLIT backward: one workgroup per block, from its saved x / t2 / t3
// and the chain's record (g, gz3, gz1), with k_stackm_bwd's fragments and summation order, so the
// result equals the fused kernel's.  W2: waves own taps (wave, wave + 16); W1: waves 0, 1; W3 and
// the scale gradient (sum W3 . G3): waves 2, 3.  Each gradient entry has one adder.
constexpr int PG = 40;  // row pitch of the bf16 g record copy
#ifndef VQ3D_STACK_RCW
#define VQ3D_STACK_RCW 4
#endif
constexpr int RPART = VQ3D_STACK_RCW;  // k_stackr_bwd's scalar partials per block (one per compute wave)
__global__ __launch_bounds__(NT) void k_stackm_wgrad(SkArgs a, const float *const *tab, float *const *gtab,
                                                     const float *__restrict__ saved, const h16_t *__restrict__ rec,
                                                     const float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nv = a.nv, nks = nv / 32, nvc = nv * MC, nvb = nv * MB, blk = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    h16_t *t2 = reinterpret_cast<h16_t *>(smem), *t3 = t2 + nv * PT, *z3 = t3 + nv * PT, *z1 = z3 + nv * PT;
    h16_t *u1 = z1 + nv * PT, *gs = u1 + nv * PU;
    short *nb = reinterpret_cast<short *>(gs + nv * PG);
    float *red = reinterpret_cast<float *>(nb + ((nv * 27 + 7) & ~7));
    const float *pc = row_ptr(tab, blk, lane);
    const Scal s = scal_lanes(*pc);
    const float *w3 = bcast_ptr(pc, 2);
    float *gc = row_ptr(gtab, blk, lane);
    float *gw1 = bcast_ptr(gc, 0), *gw2 = bcast_ptr(gc, 1), *gw3 = bcast_ptr(gc, 2);
    const float *sx = saved + size_t(blk) * nv * (MC + 2 * MB), *st2 = sx + nvc, *st3 = st2 + nvb;
    const h16_t *rg = rec + size_t(blk) * nv * (MC + 2 * MB), *rz3 = rg + nvc, *rz1 = rz3 + nvb;
    for (int i = tid; i < nv * 27; i += NT) nb[i] = short(nbr(a, i / 27, i % 27, 1));
    for (int i = tid; i < nvc; i += NT) {
        const int v = i / MC, c = i - v * MC;
        const float z = sx[i] + s.b1a;
        u1[v * PU + c] = f2h((z > 0.f ? z : expf(z) - 1.f) + s.b1b);
        gs[v * PG + c] = rg[i];
    }
    for (int i = tid; i < nvb; i += NT) {
        const int v = i / MB, o = i - v * MB;
        t2[v * PT + o] = f2h(st2[i]);
        t3[v * PT + o] = f2h(st3[i]);
        z3[v * PT + o] = rz3[i];
        z1[v * PT + o] = rz1[i];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {  // W2: M = co, N = ci, K = voxels
        const int tap = wave + 16 * q;
        if (tap >= 27) continue;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int ks = 0; ks < nks; ++ks) {
            const int v0 = ks * 32 + 8 * kb;
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int va = v0 + 2 * j, vb = va + 1;
                w[j] = uint32_t(t2[int(nb[va * 27 + tap]) * PT + row]) | (uint32_t(t2[int(nb[vb * 27 + tap]) * PT + row]) << 16);
            }
            acc = mfma(gat8(z3 + v0 * PT + row, PT), __builtin_bit_cast(hx8, uint4{w[0], w[1], w[2], w[3]}), acc);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float *d = gw2 + ((4 * kb + j) * MB + row) * 27 + tap;
            *d = *d + acc[j];
        }
    }
    float dsc = 0.f;
    if (wave < 2) {  // W1: M = o, N = channel tile (wave), K = voxels
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < nks; ++ks) {
            const int v0 = ks * 32 + 8 * kb;
            acc = mfma(gat8(z1 + v0 * PT + row, PT), gat8(u1 + v0 * PU + 16 * wave + row, PU), acc);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float *d = gw1 + (4 * kb + j) * MC + 16 * wave + row;
            *d = *d + acc[j];
        }
    } else if (wave < 4) {  // W3: M = co tile, N = o, K = voxels; dscale = sum W3 . G3
        const int ct = wave - 2;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < nks; ++ks) {
            const int v0 = ks * 32 + 8 * kb;
            acc = mfma(gat8(gs + v0 * PG + 16 * ct + row, PG), gat8(t3 + v0 * PT + row, PT), acc);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 16 * ct + 4 * kb + j;
            float *d = gw3 + co * MB + row;
            *d = *d + s.sc * acc[j];
            dsc = fmaf(w3[co * MB + row], acc[j], dsc);
        }
        dsc = wave_sum(dsc);
        if (lane == 0) red[ct] = dsc;
    }
    __syncthreads();
    if (wave == 0 && lane == 9) *gc = *gc + (0.f + red[0] + red[1]);  // lane 9 holds the scale slot
    if (part && wave == 0 && lane >= 3 && lane < NPRM && lane != 9) {
        // k_stackr_bwd's scalar partials of this block: table slot k gets ps[10 - k], waves in order
        const float *pp = part + size_t(blk) * RPART * 8 + (10 - lane);  // [block][compute wave][8]
        float add = 0.f;
#pragma unroll
        for (int w = 0; w < RPART; ++w) add += pp[8 * w];
        *gc = *gc + add;
    }
}
// ============================================================================================ register chain
// The published top level's chains with ONE barrier per block (round 6; k_stackm_* above needed
// five per block plus the scalar-sum barriers).  Layout of one MFMA: the block's weights are the A
// operand and 16 voxels the N columns, so a lane's accumulator holds 4 consecutive output channels
// of ONE voxel; with the 1x1 stages' K axis ordered to match (rch: k = 8 kb + j <-> channel 4 kb + j
// for j < 4, 16 + 4 kb + j - 4 above) every stage's accumulator is the next stage's B operand and
// the residual / gradient stream (channels rch(kb, 0..7) of the lane's voxel) never leaves the
// registers.  Only the k^3 conv meets other voxels: t2 (forward) / gz3 (backward) go to LDS, one
// barrier, and each lane gathers its 14 neighbour rows (offsets precomputed once).
//
// Roles.  Waves 0..3 compute, each on two 16-voxel column blocks (w, w + 4), and hold the block's
// 17 A fragments (packed per lane by k_stackr_pack) in registers, each refilled with the next
// block's right after its last use.  Waves 4..7 only store: everything the chain saves (forward:
// x, t2, t3; backward: the record g, gz3, gz1 and the scalar partials) is written to an LDS ring by
// the compute waves and copied out by the store waves one block later.  The split is what makes
// the prefetch work: on gfx9 loads and stores share vmcnt and complete out of order with respect
// to each other, so a wave with a store in flight can only wait for a load with vmcnt(0) -- every
// use of a prefetched fragment then waited for the block's stores too (2.7 / 3.1 us per block
// forward / backward when the compute waves stored).  Compute waves without stores wait with
// exact counts.  The ring is 3 deep (block b's slot is rewritten in block b + 3, after the store
// waves' reads in block b + 1 and two barriers).  Rounding points are k_stackm_*'s.
#ifndef VQ3D_STACK_RCW
#define VQ3D_STACK_RCW 4
#endif
constexpr int RCW = VQ3D_STACK_RCW;      // compute waves; wave w owns column blocks w, w + RCW, ...
constexpr int RSW = 4;                   // store waves
constexpr int NH = MAXVM / 16 / RCW;     // column blocks per compute wave
constexpr int RNT = (RCW + RSW) * 64;
static_assert(NH * RCW * 16 == MAXVM, "column blocks");
constexpr int RF = 17;                   // A fragments per block
constexpr int RIMG = RF * 64 * 8;        // halves per block image
static_assert(RPART == RCW, "one scalar partial per compute wave");
static_assert(RIMG == FR_N, "the register chain's images fit the k_stackm image slots");
constexpr int RPS = 8;                   // scalar partials per compute wave and block (k_stackm_bwd's ps order)
constexpr int RRING = 3;
constexpr int RPF = 3;                   // store waves' L2 prefetch distance (blocks)
#if defined(VQ3D_STACK_EXP) && VQ3D_STACK_EXP == 2
#define FR_REFILL(k0, k1)
#else
#define FR_REFILL(k0, k1) fr.load(img, nx, lane, k0, k1)
#endif

// phase clock probe (tools/probes/stack_probe.hip builds this file with VQ3D_STACK_PROBE): wave 0
// stamps s_memtime at 5 points of every block into LDS and dumps them at the end
#ifdef VQ3D_STACK_PROBE
__device__ unsigned long long g_stack_probe[2][64][5];
#define RPROBE_DECL __shared__ unsigned long long rprobe[64][5];
#define RPROBE(b, k) \
    if (wave == 0 && lane == 0 && (b) < 64) rprobe[b][k] = __builtin_amdgcn_s_memtime();
#define RPROBE_DUMP(dir)                                          \
    if (wave == 0)                                                \
        for (int i = lane; i < 64 * 5; i += 64) g_stack_probe[dir][i / 5][i % 5] = rprobe[i / 5][i % 5];
#else
#define RPROBE_DECL
#define RPROBE(b, k)
#define RPROBE_DUMP(dir)
#endif

// a load through a pointer read from the parameter table, as a GLOBAL load: the generic (flat) load
// the compiler emits otherwise counts in both vmcnt and lgkmcnt, and its use then waits for every
// memory operation in flight (vmcnt(0) lgkmcnt(0)), prefetched fragments included
__device__ __forceinline__ float ldg(const float *p) {
    typedef const __attribute__((address_space(1))) float gfloat;
    return *(gfloat *)(p);
}

// vmcnt(0) once, after the prologue's loads: the compiler's wait counts at the loop top merge the
// prologue's issue order with the loop's, and a prologue load still pending there made every
// block's first wait vmcnt(2) (all of the previous block's refills, issued moments earlier)
__device__ __forceinline__ void drain_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

__device__ __forceinline__ int rch(int kb, int j) { return j < 4 ? 4 * kb + j : 16 + 4 * kb + (j - 4); }

// Fragment f of a block, lane l = kb * 16 + m, element j (k = 8 kb + j).  Forward: f 0 W1 (A[o][k] =
// W1[o][rch(k)]), f 1 .. 14 W2 tap pairs (A[co][k] = W2[co][ci][tap], tap = 2 (f - 1) + (kb >> 1),
// ci = 8 (kb & 1) + j), f 15 / 16 W3 tiles (A[co][k] = W3[co][4 kb + j], j < 4).  Backward: f 0 W3^T
// (A[o][k] = W3[rch(k)][o]), f 1 .. 14 W2 transposed (A[ci][k] = W2[co][ci][tap], co = 8 (kb & 1) +
// j; the B rows come from the flipped tap's neighbour), f 15 / 16 W1^T tiles (A[c][k] = W1[4 kb + j][c]).
template <bool BWD>
__global__ __launch_bounds__(256) void k_stackr_pack(const float *const *tab, h16_t *__restrict__ img) {
    const int blk = blockIdx.x;
    const float *w1 = tab[blk * NPRM + 0], *w2 = tab[blk * NPRM + 1], *w3 = tab[blk * NPRM + 2];
    h16_t *dst = img + size_t(blk) * RIMG;
    for (int i = threadIdx.x; i < RF * 64; i += 256) {
        const int f = i >> 6, lane = i & 63, m = lane & 15, kb = lane >> 4;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float x = 0.f;
            if (f == 0) {
                x = BWD ? w3[rch(kb, j) * MB + m] : w1[m * MC + rch(kb, j)];
            } else if (f < 15) {
                const int tap = 2 * (f - 1) + (kb >> 1), c = 8 * (kb & 1) + j;
                if (tap < 27) x = BWD ? w2[(c * MB + m) * 27 + tap] : w2[(m * MB + c) * 27 + tap];
            } else if (j < 4) {
                const int t = 16 * (f - 15) + m;
                x = BWD ? w1[(4 * kb + j) * MC + t] : w3[t * MB + 4 * kb + j];
            }
            v[j] = x;
        }
        *reinterpret_cast<uint4 *>(dst + size_t(i) * 8) = __builtin_bit_cast(uint4, pack8(v));
    }
}

struct RFrag {  // one block's 17 A fragments of this lane
    u32x4 f[RF];
    __device__ __forceinline__ void load(const h16_t *img, int blk, int lane, int k0 = 0, int k1 = RF) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(img + size_t(blk) * RIMG) + lane;
#pragma unroll
        for (int k = 0; k < RF; ++k)
            if (k >= k0 && k < k1) f[k] = src[64 * k];
    }
    __device__ __forceinline__ hx8 operator[](int k) const { return __builtin_bit_cast(hx8, f[k]); }
};

// Branch images (t2 / t3 forward, gz3 / gz1 backward) are PLANAR in the ring: channels 0..7 of every
// voxel (16 B rows) in plane 0, channels 8..15 in plane 1, PLN halves apart (a multiple of 256 B).  A
// gather's 16-lane LDS group then reads 16 distinct voxels' rows whose 16-B chunks are distinct mod
// 256 B (the 16 voxels of a column block are one (h) row, and a tap maps it onto another row):
// conflict-free.  The [voxel][PT] rows had 44 % of the chains' LDS cycles in bank conflicts.
constexpr int PLN = MAXVM * 8;
__device__ __forceinline__ int pl_off(int v, int c) { return (c >> 3) * PLN + v * 8 + (c & 7); }

// the 14 neighbour rows lane (voxel v, kb) gathers, as element offsets into a planar branch image
// packed two per dword: tap 2 s + (kb >> 1) (backward: its flip), channels 8 (kb & 1) .. + 7.  Tap
// 27 (s = 13, kb >= 2) has no row: those lanes read zeros.
template <bool BWD>
__device__ __forceinline__ void nbr_rows(const SkArgs &a, int v, int kb, uint32_t (&o)[7]) {
#pragma unroll
    for (int s = 0; s < 7; ++s) {
        uint32_t lo = 0, hi = 0;
        const int t0 = 4 * s + (kb >> 1), t1 = t0 + 2;
        lo = uint32_t(pl_off(nbr(a, v, BWD ? 26 - t0 : t0, 1), 8 * (kb & 1)));
        if (t1 < 27) hi = uint32_t(pl_off(nbr(a, v, BWD ? 26 - t1 : t1, 1), 8 * (kb & 1)));
        o[s] = lo | (hi << 16);
    }
}
__device__ __forceinline__ void gather14(const h16_t *src, const uint32_t (&o)[7], int kb, hx8 (&nb)[14]) {
#pragma unroll
    for (int s = 0; s < 14; ++s) {
        const uint32_t off = (o[s >> 1] >> (16 * (s & 1))) & 0xffffu;
        nb[s] = (s == 13 && kb >= 2) ? zero8() : rd8(src + off);
    }
}
// the two halves of the 14 tap-pair k-steps (k_stackm's summation order)
__device__ __forceinline__ f32x4 conv14(const RFrag &fr, const hx8 (&nb)[14]) {
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        c0 = mfma(fr[1 + k], nb[k], c0);
        c1 = mfma(fr[8 + k], nb[7 + k], c1);
    }
    return c0 + c1;
}
// exp through v_exp_f32 (2^x) directly: the chain is VALU-issue bound (one compute wave per SIMD,
// 4 cycles per instruction), and expf's range reduction was ~11 instructions per call, a third of
// the forward loop; the results are rounded to 16 bits (t2, t3) or feed fp32 gradients
#ifndef VQ3D_STACK_FAST_EXP
#define VQ3D_STACK_FAST_EXP 1
#endif
__device__ __forceinline__ float exp_f(float z) {
    if constexpr (VQ3D_STACK_FAST_EXP) return __builtin_amdgcn_exp2f(z * 1.44269504088896341f);
    else return expf(z);
}
__device__ __forceinline__ float elu_f(float z) { return z > 0.f ? z : exp_f(z) - 1.f; }
// elu(z + a) + b with the bias folds precomputed per block (EluB): one compare, one add, one fma,
// the exp and one add per element instead of two adds, a multiply, the exp, an add and the compare
struct EluB {
    float na, ab, al, bm;  // -a, a + b, a log2(e), b - 1
    __device__ __forceinline__ EluB(float a, float b) : na(-a), ab(a + b), al(a * 1.44269504088896341f), bm(b - 1.f) {}
    __device__ __forceinline__ float operator()(float z) const {
        float e;
        if constexpr (VQ3D_STACK_FAST_EXP) e = __builtin_amdgcn_exp2f(fmaf(z, 1.44269504088896341f, al)) + bm;
        else e = expf(z - na) + bm;
        return z > na ? z + ab : e;
    }
};
__device__ __forceinline__ uint32_t pk2h(float a, float b) { return uint32_t(f2h(a)) | (uint32_t(f2h(b)) << 16); }
__device__ __forceinline__ float lo_h(uint32_t u) { return h2f_lo(u & 0xffffu); }
__device__ __forceinline__ float hi_h(uint32_t u) { return h2f_lo(u >> 16); }

struct RfLds {  // the forward's LDS ring (RRING slots)
    float *xs;    // [nv][PF] the block's input x (fp32)
    h16_t *t2s;   // planar t2 (16-bit): the conv's gather source
    h16_t *t3s;   // planar t3 (16-bit)
};
__device__ __forceinline__ RfLds rf_slot(char *smem, int nv, int slot) {
    RfLds l;
    char *p = smem + size_t(slot) * (size_t(nv) * PF * 4 + size_t(PLN) * 8);
    l.xs = reinterpret_cast<float *>(p);
    l.t2s = reinterpret_cast<h16_t *>(p + size_t(nv) * PF * 4);
    l.t3s = l.t2s + 2 * PLN;
    return l;
}
size_t lds_rf(int nv) { return RRING * (size_t(nv) * PF * 4 + size_t(PLN) * 8); }

// store waves: block b's x / t2 / t3 from ring slot b % 3 to `saved` (fp32, k_stackm_fwd's layout)
__device__ __forceinline__ void rf_store(const RfLds &l, int nv, float *sx, int t) {
    float *st2 = sx + nv * MC, *st3 = st2 + nv * MB;
    for (int i = t; i < nv * (MC / 4); i += 256) {
        const int v = i >> 3, c = 4 * (i & 7);
        *reinterpret_cast<float4 *>(sx + v * MC + c) = *reinterpret_cast<const float4 *>(l.xs + v * PF + c);
    }
    for (int i = t; i < nv * (MB / 4); i += 256) {
        const int v = i >> 2, o = 4 * (i & 3);
        const u32x2 a = *reinterpret_cast<const u32x2 *>(l.t2s + pl_off(v, o));
        const u32x2 b = *reinterpret_cast<const u32x2 *>(l.t3s + pl_off(v, o));
        *reinterpret_cast<float4 *>(st2 + v * MB + o) = float4{lo_h(a[0]), hi_h(a[0]), lo_h(a[1]), hi_h(a[1])};
        *reinterpret_cast<float4 *>(st3 + v * MB + o) = float4{lo_h(b[0]), hi_h(b[0]), lo_h(b[1]), hi_h(b[1])};
    }
}

template <bool FULL>  // FULL: nv = 128, every column block active (the published top level)
__global__ __launch_bounds__(RNT) void k_stackr_fwd(SkArgs a, const h16_t *__restrict__ x, const float *const *tab,
                                                    h16_t *__restrict__ out, float *__restrict__ saved,
                                                    const h16_t *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    RPROBE_DECL
    // the wave index through readfirstlane: the compiler then knows it (and the column-block masks
    // below) wave-uniform and branches instead of masking exec around every load
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), n = lane & 15,
              kb = lane >> 4;
    const int nv = a.nv, nmt = nv / 16;
    const size_t stride = size_t(nv) * (MC + 2 * MB);
    if (wave >= RCW) {  // store waves: block b - 1's tensors after barrier b, the last block's after the loop
        const int t = tid - RCW * 64;  // 0 .. RSW * 64 - 1
        // and the L2 prefetch of the fragment images RPF blocks ahead (one dword per 128-B line; the
        // value is only "used" a block later, so this wave never waits on it)
        uint32_t pf = 0;
        auto touch = [&](int b) {
            return t < RIMG * 2 / 128 ? *reinterpret_cast<const uint32_t *>(img + size_t(b) * RIMG + t * 64) : 0u;
        };
        for (int b = 0; b < RPF && b < a.nblk; ++b) pf ^= touch(b);
        for (int blk = 0; blk < a.nblk; ++blk) {
            __syncthreads();
            asm volatile("" ::"v"(pf));
            if (blk > 0) rf_store(rf_slot(smem, nv, (blk - 1) % RRING), nv, saved + (blk - 1) * stride, t);
            pf = blk + RPF < a.nblk ? touch(blk + RPF) : 0u;
        }
        asm volatile("" ::"v"(pf));
        __syncthreads();
        rf_store(rf_slot(smem, nv, (a.nblk - 1) % RRING), nv, saved + (a.nblk - 1) * stride, t);
        return;
    }
    bool act[NH];
    int vv[NH];
    uint32_t nbo[NH][7];
    float xv[NH][8];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int cb = wave + RCW * h;
        act[h] = FULL || cb < nmt;
        vv[h] = min(cb, nmt - 1) * 16 + n;
        nbr_rows<false>(a, vv[h], kb, nbo[h]);
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[h][j] = ld(x + size_t(vv[h]) * MC + rch(kb, j));
    }
    RFrag fr;
    fr.load(img, 0, lane);
    float vc = ldg(row_ptr(tab, 0, lane));
    const float *pn = row_ptr(tab, min(1, a.nblk - 1), lane);
    drain_vmem();
    for (int blk = 0; blk < a.nblk; ++blk) {
        const Scal s = scal_lanes(vc);
        RPROBE(blk, 0)
        // the next block (the last block reloads itself: every load unconditional, so the
        // compiler's waits count exactly), its scalars a block ahead
#if defined(VQ3D_STACK_EXP) && VQ3D_STACK_EXP == 1
        const int nx = 0;
#else
        const int nx = min(blk + 1, a.nblk - 1);
#endif
        vc = ldg(pn);
        pn = row_ptr(tab, min(blk + 2, a.nblk - 1), lane);
        const RfLds l = rf_slot(smem, nv, blk % RRING);
        const EluB e1(s.b1a, s.b1b), e2(s.b2a, s.b2b), e3(s.b3a, s.b3b);
        // t2 = elu_f(W1 u1 + b2a) + b2b, u1 = elu_f(x + b1a) + b1b (K in the rch order)
        f32x4 a2[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const int v = vv[h];
            *reinterpret_cast<float4 *>(l.xs + v * PF + 4 * kb) = float4{xv[h][0], xv[h][1], xv[h][2], xv[h][3]};
            *reinterpret_cast<float4 *>(l.xs + v * PF + 16 + 4 * kb) = float4{xv[h][4], xv[h][5], xv[h][6], xv[h][7]};
            float u[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) u[j] = e1(xv[h][j]);
            a2[h] = mfma(fr[0], pack8(u), f32x4{0.f, 0.f, 0.f, 0.f});
        }
        FR_REFILL(0, 1);
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const f32x4 c = a2[h];
            *reinterpret_cast<u32x2 *>(l.t2s + pl_off(vv[h], 4 * kb)) =
                u32x2{pk2h(e2(c[0]), e2(c[1])), pk2h(e2(c[2]), e2(c[3]))};
        }
        RPROBE(blk, 1)
        __syncthreads();
        RPROBE(blk, 2)
        // t3 = elu_f(W2 (*) t2 + b3a) + b3b over the gathered neighbour rows
        // all column blocks' gathers and MFMAs first, then their epilogues: the next block's
        // LDS gathers are issued while the previous one's MFMA chain runs, and the epilogues
        // overlap the last MFMAs (in-order issue: an epilogue first would wait for its chain)
        u32x2 t3p[NH];
        f32x4 cc[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            hx8 nb[14];
            gather14(l.t2s, nbo[h], kb, nb);
            cc[h] = conv14(fr, nb);
        }
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const f32x4 c = cc[h];
            t3p[h] = u32x2{pk2h(e3(c[0]), e3(c[1])), pk2h(e3(c[2]), e3(c[3]))};
            *reinterpret_cast<u32x2 *>(l.t3s + pl_off(vv[h], 4 * kb)) = t3p[h];
        }
        RPROBE(blk, 3)
        FR_REFILL(1, 15);
        // x += scale * W3 t3 + b4 (two channel tiles; K = the lane's 4 t3 channels + zeros)
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const hx8 b3 = __builtin_bit_cast(hx8, u32x4{t3p[h][0], t3p[h][1], 0u, 0u});
            const f32x4 o0 = mfma(fr[15], b3, f32x4{0.f, 0.f, 0.f, 0.f});
            const f32x4 o1 = mfma(fr[16], b3, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xv[h][i] += o0[i] * s.sc + s.b4;
                xv[h][4 + i] += o1[i] * s.sc + s.b4;
            }
        }
        FR_REFILL(15, RF);
        RPROBE(blk, 4)
    }
    __syncthreads();  // the store waves' last block
    RPROBE_DUMP(0)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        if (!act[h]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) out[size_t(vv[h]) * MC + rch(kb, j)] = f2h(xv[h][j]);
    }
}

struct RbLds {  // the backward's LDS ring
    h16_t *gs;    // [nv][PG] the block's incoming gradient g (16-bit, the record)
    h16_t *z3s;   // planar gz3: the transposed conv's gather source
    h16_t *z1s;   // planar gz1
    float *ps;    // [RCW][64][RPS] the compute lanes' scalar partials
};
__device__ __forceinline__ RbLds rb_slot(char *smem, int nv, int slot) {
    RbLds l;
    char *p = smem + size_t(slot) * (size_t(nv) * PG * 2 + size_t(PLN) * 8 + RCW * 64 * RPS * 4);
    l.gs = reinterpret_cast<h16_t *>(p);
    l.z3s = l.gs + nv * PG;
    l.z1s = l.z3s + 2 * PLN;
    l.ps = reinterpret_cast<float *>(l.z1s + 2 * PLN);
    return l;
}
size_t lds_rb(int nv) { return RRING * (size_t(nv) * PG * 2 + size_t(PLN) * 8 + RCW * 64 * RPS * 4); }

// store waves: block b's record (g, gz3, gz1: k_stackm_bwd's layout) and scalar partials
__device__ __forceinline__ void rb_store(const RbLds &l, int nv, h16_t *rg, float *part, int t) {
    h16_t *rz3 = rg + nv * MC, *rz1 = rz3 + nv * MB;
    for (int i = t; i < nv * (MC / 8); i += 256) {
        const int v = i >> 2, c = 8 * (i & 3);
        *reinterpret_cast<u32x4 *>(rg + v * MC + c) = *reinterpret_cast<const u32x4 *>(l.gs + v * PG + c);
    }
    for (int i = t; i < nv * (MB / 4); i += 256) {
        const int v = i >> 2, o = 4 * (i & 3);
        *reinterpret_cast<u32x2 *>(rz3 + v * MB + o) = *reinterpret_cast<const u32x2 *>(l.z3s + pl_off(v, o));
        *reinterpret_cast<u32x2 *>(rz1 + v * MB + o) = *reinterpret_cast<const u32x2 *>(l.z1s + pl_off(v, o));
    }
    // store wave q sums compute waves q, q + RSW, ... (DPP, fixed order); part [block][wave][RPS]
    const int lane = t & 63;
    for (int cw = t >> 6; cw < RCW; cw += RSW) {
        const float *src = l.ps + (cw * 64 + lane) * RPS;
        const float4 pa = *reinterpret_cast<const float4 *>(src), pb = *reinterpret_cast<const float4 *>(src + 4);
        float ps[RPS] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
#pragma unroll
        for (int k = 0; k < RPS; ++k) ps[k] = wave_sum(ps[k]);
        if (lane < RPS) {
            float pv = ps[0];
#pragma unroll
            for (int k = 1; k < RPS; ++k) pv = lane == k ? ps[k] : pv;
            part[cw * RPS + lane] = pv;
        }
    }
}

// the backward chain: gradient stream in registers, gz3 through LDS for the transposed conv; the
// record and the per-wave scalar partials leave through the store waves
template <bool FULL>
__global__ __launch_bounds__(RNT) void k_stackr_bwd(SkArgs a, const h16_t *__restrict__ g, const float *const *tab,
                                                    const float *__restrict__ saved, h16_t *__restrict__ gx,
                                                    h16_t *__restrict__ rec, float *__restrict__ part,
                                                    const h16_t *__restrict__ img) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    RPROBE_DECL
    // the wave index through readfirstlane: the compiler then knows it (and the column-block masks
    // below) wave-uniform and branches instead of masking exec around every load
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), n = lane & 15,
              kb = lane >> 4;
    const int nv = a.nv, nmt = nv / 16, nvc = nv * MC, nvb = nv * MB;
    const size_t stride = size_t(nv) * (MC + 2 * MB);
    const int last = a.nblk - 1;
    if (wave >= RCW) {  // store waves (the walk is in reverse)
        const int t = tid - RCW * 64;  // 0 .. RSW * 64 - 1
        // L2 prefetch RPF blocks ahead: the fragment image (136 lines) and the saved x / t2 / t3
        // (nv / 2 lines of 128 B), one dword per line
        uint32_t pf = 0;
        const int sl = int(stride / 32);  // 128-B lines of one block's saved tensors
        auto touch = [&](int b) {
            uint32_t r = t < RIMG * 2 / 128 ? *reinterpret_cast<const uint32_t *>(img + size_t(b) * RIMG + t * 64) : 0u;
            for (int i = t; i < sl; i += 256) r ^= *reinterpret_cast<const uint32_t *>(saved + b * stride + i * 32);
            return r;
        };
        for (int b = last; b > last - RPF && b >= 0; --b) pf ^= touch(b);
        for (int blk = last; blk >= 0; --blk) {
            __syncthreads();
            asm volatile("" ::"v"(pf));
            pf = blk - RPF >= 0 ? touch(blk - RPF) : 0u;
            if (blk < last)
                rb_store(rb_slot(smem, nv, (blk + 1) % RRING), nv, rec + (blk + 1) * stride,
                         part + (blk + 1) * RCW * RPS, t);
        }
        __syncthreads();
        asm volatile("" ::"v"(pf));
        rb_store(rb_slot(smem, nv, 0), nv, rec, part, t);
        return;
    }
    bool act[NH];
    int vv[NH];
    uint32_t nbo[NH][7];
    float gv[NH][8];
    float4 s3[NH], s2[NH], sxa[NH], sxb[NH];  // the block's saved t3 / t2 (the lane's 4 branch channels), x (its 8)
    auto sv4 = [&](int b, int off) { return *reinterpret_cast<const float4 *>(saved + b * stride + off); };
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        const int cb = wave + RCW * h;
        act[h] = FULL || cb < nmt;
        vv[h] = min(cb, nmt - 1) * 16 + n;
        nbr_rows<true>(a, vv[h], kb, nbo[h]);
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[h][j] = ld(g + size_t(vv[h]) * MC + rch(kb, j));
        const int ox = vv[h] * MC + 4 * kb, ob = vv[h] * MB + 4 * kb;
        s3[h] = sv4(last, nvc + nvb + ob);
        s2[h] = sv4(last, nvc + ob);
        sxa[h] = sv4(last, ox);
        sxb[h] = sv4(last, ox + 16);
    }
    RFrag fr;
    fr.load(img, last, lane);
    float vc = ldg(row_ptr(tab, last, lane));
    const float *pn = row_ptr(tab, max(last - 1, 0), lane);
    drain_vmem();
    for (int blk = last; blk >= 0; --blk) {
        const Scal s = scal_lanes(vc);
        RPROBE(blk, 0)
        const int nx = max(blk - 1, 0);  // the next block (unconditional loads, as in the forward)
        vc = ldg(pn);
        pn = row_ptr(tab, max(blk - 2, 0), lane);
        const RbLds l = rb_slot(smem, nv, blk % RRING);
        const float nb1a = -s.b1a, b1al = s.b1a * 1.44269504088896341f;  // elu'(x + b1a) folds
        float ps[RPS] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // b4, (scale), b3b, b3a, b2b, b2a, b1b, b1a
        // gz3 = scale W3^T g * elu'(t3 - b3b)
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const int v = vv[h];
            const float *q = gv[h];
#pragma unroll
            for (int j = 0; j < 8; ++j) ps[0] += q[j];
            *reinterpret_cast<u32x2 *>(l.gs + v * PG + 4 * kb) = u32x2{pk2h(q[0], q[1]), pk2h(q[2], q[3])};
            *reinterpret_cast<u32x2 *>(l.gs + v * PG + 16 + 4 * kb) = u32x2{pk2h(q[4], q[5]), pk2h(q[6], q[7])};
            const f32x4 a3 = mfma(fr[0], pack8(gv[h]), f32x4{0.f, 0.f, 0.f, 0.f});
            const float t3v[4] = {s3[h].x, s3[h].y, s3[h].z, s3[h].w};
            float zq[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float g3 = a3[i] * s.sc;
                zq[i] = g3 * elu_d_act(t3v[i], s.b3b);
                ps[2] += g3;
                ps[3] += zq[i];
            }
            *reinterpret_cast<u32x2 *>(l.z3s + pl_off(v, 4 * kb)) = u32x2{pk2h(zq[0], zq[1]), pk2h(zq[2], zq[3])};
        }
        fr.load(img, nx, lane, 0, 1);
#pragma unroll
        for (int h = 0; h < NH; ++h) s3[h] = sv4(nx, nvc + nvb + vv[h] * MB + 4 * kb);
        RPROBE(blk, 1)
        __syncthreads();
        RPROBE(blk, 2)
        // gt2 = W2^T (*) gz3 over the flipped taps' neighbour rows; gz1 = gt2 * elu'(t2 - b2b)
        u32x2 z1p[NH];
        f32x4 cc[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) {  // gathers and MFMAs of every column block, then the epilogues
            if (!act[h]) continue;
            hx8 nb[14];
            gather14(l.z3s, nbo[h], kb, nb);
            cc[h] = conv14(fr, nb);
        }
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const f32x4 c = cc[h];
            const float t2v[4] = {s2[h].x, s2[h].y, s2[h].z, s2[h].w};
            float z[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                z[i] = c[i] * elu_d_act(t2v[i], s.b2b);
                ps[4] += c[i];
                ps[5] += z[i];
            }
            z1p[h] = u32x2{pk2h(z[0], z[1]), pk2h(z[2], z[3])};
            *reinterpret_cast<u32x2 *>(l.z1s + pl_off(vv[h], 4 * kb)) = z1p[h];
        }
        RPROBE(blk, 3)
        fr.load(img, nx, lane, 1, 15);
#pragma unroll
        for (int h = 0; h < NH; ++h) s2[h] = sv4(nx, nvc + vv[h] * MB + 4 * kb);
        // g += (W1^T gz1) * elu'(x + b1a), in the stream's channel order
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            if (!act[h]) continue;
            const hx8 bz = __builtin_bit_cast(hx8, u32x4{z1p[h][0], z1p[h][1], 0u, 0u});
            const f32x4 o0 = mfma(fr[15], bz, f32x4{0.f, 0.f, 0.f, 0.f});
            const f32x4 o1 = mfma(fr[16], bz, f32x4{0.f, 0.f, 0.f, 0.f});
            const float xs[8] = {sxa[h].x, sxa[h].y, sxa[h].z, sxa[h].w, sxb[h].x, sxb[h].y, sxb[h].z, sxb[h].w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float gt1 = j < 4 ? o0[j] : o1[j - 4];
                const float e = xs[j] > nb1a ? 1.f
                                : (VQ3D_STACK_FAST_EXP ? __builtin_amdgcn_exp2f(fmaf(xs[j], 1.44269504088896341f, b1al))
                                                       : expf(xs[j] - nb1a));
                ps[6] += gt1;
                ps[7] += gt1 * e;
                gv[h][j] += gt1 * e;
            }
        }
        fr.load(img, nx, lane, 15, RF);
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            sxa[h] = sv4(nx, vv[h] * MC + 4 * kb);
            sxb[h] = sv4(nx, vv[h] * MC + 16 + 4 * kb);
        }
        // this lane's scalar partials of the block: the store waves reduce them (fixed order)
        *reinterpret_cast<float4 *>(l.ps + (wave * 64 + lane) * RPS) = float4{ps[0], ps[1], ps[2], ps[3]};
        *reinterpret_cast<float4 *>(l.ps + (wave * 64 + lane) * RPS + 4) = float4{ps[4], ps[5], ps[6], ps[7]};
        RPROBE(blk, 4)
    }
    __syncthreads();  // the store waves' last block
    RPROBE_DUMP(1)
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        if (!act[h]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) gx[size_t(vv[h]) * MC + rch(kb, j)] = f2h(gv[h][j]);
    }
}

size_t lds_wgrad(int nv) { return size_t(nv) * (4 * PT + PU + PG) * 2 + size_t((nv * 27 + 7) & ~7) * 2 + 64; }

bool mfma_ok(const SkArgs &a) { return a.C == MC && a.B == MB && a.nv % 32 == 0 && a.nv <= MAXVM; }

bool lds_opt_in(const void *k) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
    (void)hipGetLastError();
    return true;
}

// which matrix-core chain runs: 'r' the register chain (default), 'm' the LDS-phase k_stackm_*
// (VQ3D_STACK_CHAIN=m, kept for A/B measurements)
char stack_chain() {
    static const char c = [] {
        const char *e = getenv("VQ3D_STACK_CHAIN");
        return e && e[0] == 'm' ? 'm' : 'r';
    }();
    return c;
}

int check(int32_t nblk, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd,
          SkArgs &a) {
    a.nv = batch * h * w * dd;
    a.C = channels;
    a.B = branch;
    a.H = h;
    a.W = w;
    a.D = dd;
    a.nblk = nblk;
    a.PC = channels + 1;
    a.PB = branch + 1;
    if (nblk < 1 || batch < 1 || h < 1 || w < 1 || dd < 1) return 1;
    if (a.nv > MAXV || channels > MAXC || branch > MAXB || channels % 4 || branch % 4) return 1;
    if (lds_bytes(a, true) > 160 * 1024) return 1;
    return 0;
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_stack_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    SkArgs a;
    return check(2, batch, channels, branch, h, w, dd, a) == 0 ? 1 : 0;
}

size_t vq3d_preact_stack_saved_floats(int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                                      int32_t w, int32_t dd) {
    // per block x / t2 / t3, then the matrix-core forward's packed fragment images (FR_N 16-bit each)
    return size_t(nblocks) * batch * h * w * dd * (channels + 2 * branch) + size_t(nblocks) * FR_N / 2;
}

int vq3d_preact_stack_fwd(int32_t dtype, int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                          int32_t w, int32_t dd, const void *x, const float *const *params, void *out, float *saved,
                          vq3d_stream_t stream) {
    SkArgs a;
    if (check(nblocks, batch, channels, branch, h, w, dd, a)) return fail("preact_stack_fwd: unsupported shape");
    if (!x || !params || !out || !saved) return fail("preact_stack_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    const size_t lds = lds_bytes(a, false);
    if (dtype == VQ3D_HALF && mfma_ok(a)) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stackm_fwd), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(160 * 1024));
        h16_t *img = reinterpret_cast<h16_t *>(saved + size_t(nblocks) * a.nv * (a.C + 2 * a.B));
        if (stack_chain() == 'r') {
            k_stackr_pack<false><<<nblocks, 256, 0, s>>>(params, img);
            static const bool opt = lds_opt_in(reinterpret_cast<const void *>(k_stackr_fwd<true>)) &&
                                    lds_opt_in(reinterpret_cast<const void *>(k_stackr_fwd<false>));
            (void)opt;
            if (a.nv == MAXVM)
                k_stackr_fwd<true><<<1, RNT, lds_rf(a.nv), s>>>(a, (const h16_t *)x, params, (h16_t *)out, saved, img);
            else
                k_stackr_fwd<false><<<1, RNT, lds_rf(a.nv), s>>>(a, (const h16_t *)x, params, (h16_t *)out, saved, img);
        } else {
            k_stackm_pack<false><<<nblocks, NT, 0, s>>>(params, img);
            k_stackm_fwd<<<1, NT, lds_m(a.nv), s>>>(a, (const h16_t *)x, params, (h16_t *)out, saved, img);
        }
    } else if (dtype == VQ3D_HALF) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stack_fwd<h16_t>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
        k_stack_fwd<h16_t><<<1, NT, lds, s>>>(a, (const h16_t *)x, params, (h16_t *)out, saved);
    } else if (dtype == VQ3D_F32) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stack_fwd<float>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
        k_stack_fwd<float><<<1, NT, lds, s>>>(a, (const float *)x, params, (float *)out, saved);
    } else {
        return fail("preact_stack_fwd: dtype");
    }
    return check_launch("preact_stack_fwd");
}

int vq3d_preact_stack_bwd(int32_t dtype, int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                          int32_t w, int32_t dd, const void *g, const float *const *params, float *const *grads,
                          const float *saved, void *gx, vq3d_stream_t stream) {
    SkArgs a;
    if (check(nblocks, batch, channels, branch, h, w, dd, a)) return fail("preact_stack_bwd: unsupported shape");
    if (!g || !params || !grads || !saved || !gx) return fail("preact_stack_bwd: null pointer");
    hipStream_t s = as_stream(stream);
    const size_t lds = lds_bytes(a, true);
    if (dtype == VQ3D_HALF && mfma_ok(a)) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stackm_bwd<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
        k_stackm_bwd<false><<<1, NT, lds_m(a.nv), s>>>(a, (const h16_t *)g, params, grads, saved, (h16_t *)gx, nullptr,
                                                       nullptr);
    } else if (dtype == VQ3D_HALF) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stack_bwd<h16_t>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
        k_stack_bwd<h16_t><<<1, NT, lds, s>>>(a, (const h16_t *)g, params, grads, saved, (h16_t *)gx);
    } else if (dtype == VQ3D_F32) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stack_bwd<float>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
        k_stack_bwd<float><<<1, NT, lds, s>>>(a, (const float *)g, params, grads, saved, (float *)gx);
    } else {
        return fail("preact_stack_bwd: dtype");
    }
    return check_launch("preact_stack_bwd");
}

size_t vq3d_preact_stack_bwd_workspace_bytes(int32_t nblocks, int32_t batch, int32_t channels, int32_t branch,
                                             int32_t h, int32_t w, int32_t dd) {
    SkArgs a;
    if (check(nblocks, batch, channels, branch, h, w, dd, a) || !mfma_ok(a)) return 0;
    // the record, the packed images, k_stackr_bwd's scalar partials (8 waves x 8 per block)
    return size_t(nblocks) * a.nv * (MC + 2 * MB) * 2 + size_t(nblocks) * FR_N * 2 + size_t(nblocks) * RCW * RPS * 4;
}

int vq3d_preact_stack_bwd_ws(int32_t dtype, int32_t nblocks, int32_t batch, int32_t channels, int32_t branch,
                             int32_t h, int32_t w, int32_t dd, const void *g, const float *const *params,
                             float *const *grads, const float *saved, void *gx, void *workspace, size_t ws_bytes,
                             vq3d_stream_t stream) {
    SkArgs a;
    if (check(nblocks, batch, channels, branch, h, w, dd, a)) return fail("preact_stack_bwd_ws: unsupported shape");
    const size_t need = vq3d_preact_stack_bwd_workspace_bytes(nblocks, batch, channels, branch, h, w, dd);
    if (dtype != VQ3D_HALF || need == 0)  // no split plan for this shape / dtype: the fused kernel
        return vq3d_preact_stack_bwd(dtype, nblocks, batch, channels, branch, h, w, dd, g, params, grads, saved, gx,
                                     stream);
    if (!g || !params || !grads || !saved || !gx || !workspace) return fail("preact_stack_bwd_ws: null pointer");
    if (ws_bytes < need) return fail("preact_stack_bwd_ws: workspace too small");
    hipStream_t s = as_stream(stream);
    h16_t *img = static_cast<h16_t *>(workspace) + size_t(nblocks) * a.nv * (MC + 2 * MB);
    float *part = reinterpret_cast<float *>(img + size_t(nblocks) * FR_N);
    if (stack_chain() == 'r') {
        k_stackr_pack<true><<<nblocks, 256, 0, s>>>(params, img);
        static const bool opt = lds_opt_in(reinterpret_cast<const void *>(k_stackr_bwd<true>)) &&
                                lds_opt_in(reinterpret_cast<const void *>(k_stackr_bwd<false>));
        (void)opt;
        if (a.nv == MAXVM)
            k_stackr_bwd<true><<<1, RNT, lds_rb(a.nv), s>>>(a, (const h16_t *)g, params, saved, (h16_t *)gx,
                                                            (h16_t *)workspace, part, img);
        else
            k_stackr_bwd<false><<<1, RNT, lds_rb(a.nv), s>>>(a, (const h16_t *)g, params, saved, (h16_t *)gx,
                                                             (h16_t *)workspace, part, img);
        k_stackm_wgrad<<<nblocks, NT, lds_wgrad(a.nv), s>>>(a, params, grads, saved, (const h16_t *)workspace, part);
    } else {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_stackm_bwd<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024));
        k_stackm_pack<true><<<nblocks, NT, 0, s>>>(params, img);
        k_stackm_bwd<true><<<1, NT, lds_m(a.nv), s>>>(a, (const h16_t *)g, params, grads, saved, (h16_t *)gx,
                                                      (h16_t *)workspace, img);
        k_stackm_wgrad<<<nblocks, NT, lds_wgrad(a.nv), s>>>(a, params, grads, saved, (const h16_t *)workspace,
                                                            nullptr);
    }
    return check_launch("preact_stack_bwd_ws");
}

}  // extern "C"
