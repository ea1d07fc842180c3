// One whole PreActFixupResBlock (vqvae/layers.py:102-216, mode 'same', no skip conv) on the
// tiny top-level grids (8x8x2 = 128 voxels at 32 channels: 100 of these blocks per training
// step in the published 3-layer model), forward in one launch and backward in two.  At this
// size every per-conv launch is pure fixed cost; here each launch keeps its operands in LDS
// (fp32) and splits the work over a handful of workgroups:
//
//   u1  = elu(x + b1a) + b1b                     t2 = elu(W1 u1 + b2a) + b2b        (1x1, C -> B)
//   t3  = elu(W2 * t2 + b3a) + b3b  (3x3x3 circular, B -> B)
//   out = scale * (W3 t3) + b4 + x                                                (1x1, B -> C)
//
// forward   (nv / 16 workgroups): every workgroup computes t2 on the whole grid (cheap 1x1),
//           then t3 and out for its 16 voxels; t2 / t3 are saved (fp32) for the backward.
// backward A (28 workgroups): all recompute gz3 = dL/d(W2 * t2) from g and t3; workgroup
//           `tap` < 27 forms dW2[:, :, tap] and that tap's share of dL/dt2 (partials in the
//           workspace), workgroup 27 the conv3 weight / scale / bias gradients.
// backward B (one workgroup): sums the 27 tap partials, then conv1: dW1, gx and the prologue /
//           activation scalar gradients.
// Scalar gradients are fixed-order block sums; weight gradients are added (+=) to the fp32
// gradient buffers, each entry by exactly one thread.
#include "engines.h"

#include <algorithm>

namespace vq3d {

namespace {

constexpr int MAXV = 256, MAXC = 32, MAXB = 16;
constexpr int VPW = 16;  // forward: voxels per workgroup

struct TArgs {
    int nv, C, B, H, W, D;  // voxels (batch folded in), channels, branch channels, grid
};

// circular neighbour of voxel v at tap (kh, kw, kd) in {0,1,2}^3; sgn = -1 for the transpose
__device__ __forceinline__ int nbr(const TArgs &a, int v, int tap, int sgn) {
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

// put(i, src[i]) for the n elements of a 16-byte aligned array: 16-byte loads, four of them in
// flight per thread before the (LDS) stores
template <typename T, typename F>
__device__ __forceinline__ void stage(const T *__restrict__ src, int n, F put) {
    constexpr int E = 16 / sizeof(T);
    const int nq = n / E;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    for (int b = threadIdx.x; b < nq; b += 4 * blockDim.x) {
        uint4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = b + u * blockDim.x;
            if (i < nq) r[u] = s4[i];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = b + u * blockDim.x;
            if (i >= nq) continue;
            const T *el = reinterpret_cast<const T *>(&r[u]);
#pragma unroll
            for (int j = 0; j < E; ++j) put(i * E + j, ld(el + j));
        }
    }
    for (int i = nq * E + threadIdx.x; i < n; i += blockDim.x) put(i, ld(src + i));
}

template <typename T>
__device__ __forceinline__ void load_act(const T *__restrict__ src, float *dst, int n) {
    stage(src, n, [&](int i, float v) { dst[i] = v; });
}

__device__ __forceinline__ void load_f(const float *__restrict__ src, float *dst, int n) {
    stage(src, n, [&](int i, float v) { dst[i] = v; });
}

struct Scal {
    float b1a, b1b, b2a, b2b, b3a, b3b, scale, b4;
};

__device__ __forceinline__ Scal load_scal(const vq3d_preact_params &p) {
    Scal s;
    s.b1a = *p.bias1a;
    s.b1b = *p.bias1b;
    s.b2a = *p.bias2a;
    s.b2b = *p.bias2b;
    s.b3a = *p.bias3a;
    s.b3b = *p.bias3b;
    s.scale = *p.scale;
    s.b4 = *p.bias4;
    return s;
}

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

__device__ __forceinline__ void fma4(float (&acc)[4], float u, const float4 w) {
    acc[0] = fmaf(u, w.x, acc[0]);
    acc[1] = fmaf(u, w.y, acc[1]);
    acc[2] = fmaf(u, w.z, acc[2]);
    acc[3] = fmaf(u, w.w, acc[3]);
}

// acc[j] += sum_k a[k] * W[(c0 + j) * ld + k], k over a 4-group (a, W rows contiguous in k)
__device__ __forceinline__ void dot4x4(float (&acc)[4], const float4 av, const float *wrow, int ld) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 w = ld4(wrow + j * ld);
        acc[j] = fmaf(av.x, w.x, fmaf(av.y, w.y, fmaf(av.z, w.z, fmaf(av.w, w.w, acc[j]))));
    }
}

template <int NTH>
__device__ __forceinline__ float bsum(float v, float *red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NTH / 64; ++i) t += red[i];
    return t;
}

// W1 [B][C] -> [C][B], W3 [C][B] -> [B][C] (output channels innermost)
__device__ __forceinline__ void load_w1t(const TArgs &a, const float *__restrict__ w1, float *w1t) {
    stage(w1, a.B * a.C, [&](int i, float v) {
        const int o = i / a.C, c = i - o * a.C;
        w1t[c * a.B + o] = v;
    });
}
__device__ __forceinline__ void load_w3t(const TArgs &a, const float *__restrict__ w3, float *w3t) {
    stage(w3, a.C * a.B, [&](int i, float v) {
        const int o = i / a.B, c = i - o * a.B;
        w3t[c * a.C + o] = v;
    });
}

// ------------------------------------------------------------------------------------ forward
constexpr int NTF = 256;

template <typename T>
__global__ __launch_bounds__(NTF) void k_tiny_fwd(TArgs a, const T *__restrict__ x, const float *__restrict__ w1,
                                                 const float *__restrict__ w2, const float *__restrict__ w3,
                                                 vq3d_preact_params p, T *__restrict__ out,
                                                 float *__restrict__ saved) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *xs = sm;                     // [nv][C]
    float *u1 = xs + a.nv * a.C;        // [nv][C]
    float *t2 = u1 + a.nv * a.C;        // [nv][B]
    float *t3 = t2 + a.nv * a.B;        // [VPW][B]
    float *w1t = t3 + VPW * a.B;        // [C][B]
    float *w2t = w1t + a.C * a.B;       // [tap][c][o]
    float *w3t = w2t + 27 * a.B * a.B;  // [B][C]
    int *nbt = reinterpret_cast<int *>(w3t + a.B * a.C);  // [VPW][27] neighbours of own voxels
    const int tid = threadIdx.x;
    const int v0 = blockIdx.x * VPW, nown = min(VPW, a.nv - v0);
    for (int i = tid; i < nown * 27; i += NTF) nbt[i] = nbr(a, v0 + i / 27, i % 27, 1);
    load_act(x, xs, a.nv * a.C);
    load_w1t(a, w1, w1t);
    stage(w2, a.B * a.B * 27, [&](int i, float v) {  // W2 [o][c][tap] -> [tap][c][o]
        const int tap = i % 27, r = i / 27, c = r % a.B, o = r / a.B;
        w2t[(tap * a.B + c) * a.B + o] = v;
    });
    load_w3t(a, w3, w3t);
    const Scal sc = load_scal(p);
    __syncthreads();
    for (int i = tid; i < a.nv * a.C; i += NTF) u1[i] = elu(xs[i] + sc.b1a) + sc.b1b;
    __syncthreads();
    const int B4 = a.B / 4;
    for (int e = tid; e < a.nv * B4; e += NTF) {  // t2 on the whole grid
        const int v = e / B4, o0 = (e - v * B4) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float *ur = u1 + v * a.C;
        for (int c = 0; c < a.C; ++c) fma4(acc, ur[c], ld4(w1t + c * a.B + o0));
#pragma unroll
        for (int j = 0; j < 4; ++j) t2[v * a.B + o0 + j] = elu(acc[j] + sc.b2a) + sc.b2b;
    }
    __syncthreads();
    for (int e = tid; e < nown * a.B; e += NTF) {  // t3 on this workgroup's voxels: (voxel, channel)
        const int vl = e / a.B, o = e - vl * a.B, v = v0 + vl;
        float acc = 0.f;
        for (int tap = 0; tap < 27; ++tap) {
            const float *tr = t2 + nbt[vl * 27 + tap] * a.B;
            const float *wr = w2t + tap * a.B * a.B + o;
            for (int c = 0; c < a.B; ++c) acc = fmaf(tr[c], wr[c * a.B], acc);
        }
        const float t = elu(acc + sc.b3a) + sc.b3b;
        t3[vl * a.B + o] = t;
        saved[a.nv * a.B + v * a.B + o] = t;
        saved[v * a.B + o] = t2[v * a.B + o];
    }
    __syncthreads();
    const int C4 = a.C / 4;
    for (int e = tid; e < nown * C4; e += NTF) {  // out = scale * W3 t3 + b4 + x
        const int vl = e / C4, o0 = (e - vl * C4) * 4, v = v0 + vl;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float *tr = t3 + vl * a.B;
        for (int c = 0; c < a.B; ++c) fma4(acc, tr[c], ld4(w3t + c * a.C + o0));
#pragma unroll
        for (int j = 0; j < 4; ++j)
            st(out + v * a.C + o0 + j, acc[j] * sc.scale + sc.b4 + xs[v * a.C + o0 + j]);
    }
}

// ------------------------------------------------------------------------------------ backward A
constexpr int NTA = 256;

template <typename T>
__global__ __launch_bounds__(NTA) void k_tiny_bwd_a(TArgs a, const T *__restrict__ g, const float *__restrict__ w2,
                                                   const float *__restrict__ w3, vq3d_preact_params p,
                                                   vq3d_preact_grads gr, const float *__restrict__ saved,
                                                   float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __shared__ float red[NTA / 64];
    float *gs = sm;                  // [nv][C]
    float *t2 = gs + a.nv * a.C;     // [nv][B]
    float *t3 = t2 + a.nv * a.B;     // [nv][B]
    float *gz3 = t3 + a.nv * a.B;    // [nv][B]
    float *w3t = gz3 + a.nv * a.B;   // [B][C]
    float *w2s = w3t + a.B * a.C;    // [c][o] of this tap
    int *nbf = reinterpret_cast<int *>(w2s + a.B * a.B);  // nbr(v, tap, +1)
    int *nbb = nbf + a.nv;                                 // nbr(v, tap, -1)
    const int tid = threadIdx.x;
    const int tap = blockIdx.x;  // 27: conv3 parameter gradients
    load_act(g, gs, a.nv * a.C);
    load_f(saved, t2, 2 * a.nv * a.B);  // t2 then t3
    load_w3t(a, w3, w3t);
    if (tap < 27) {
        for (int i = tid; i < a.B * a.B; i += NTA) {  // W2[o][c][tap] -> [c][o]
            const int o = i / a.B, c = i - o * a.B;
            w2s[c * a.B + o] = w2[i * 27 + tap];
        }
        for (int v = tid; v < a.nv; v += NTA) {
            nbf[v] = nbr(a, v, tap, 1);
            nbb[v] = nbr(a, v, tap, -1);
        }
    }
    const Scal sc = load_scal(p);
    __syncthreads();
    // gz3 = scale * W3^T g * elu'(t3) on the whole grid
    const int B4 = a.B / 4;
    float p_b3b = 0.f, p_b3a = 0.f;
    for (int e = tid; e < a.nv * B4; e += NTA) {
        const int v = e / B4, c0 = (e - v * B4) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int co = 0; co < a.C; co += 4) dot4x4(acc, ld4(gs + v * a.C + co), w3t + c0 * a.C + co, a.C);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float h3 = acc[j] * sc.scale;
            const float z = h3 * elu_d_act(t3[v * a.B + c0 + j], sc.b3b);
            p_b3b += h3;
            p_b3a += z;
            gz3[v * a.B + c0 + j] = z;
        }
    }
    __syncthreads();
    if (tap < 27) {
        // dW2[o][c][tap] = sum_v gz3[v][o] t2[nbf(v)][c]
        for (int e = tid; e < a.B * a.B; e += NTA) {
            const int o = e / a.B, c = e - o * a.B;
            float sum = 0.f;
            for (int v = 0; v < a.nv; ++v) sum = fmaf(gz3[v * a.B + o], t2[nbf[v] * a.B + c], sum);
            if (gr.dw2) atomicAdd(gr.dw2 + e * 27 + tap, sum);
        }
        // this tap's share of dL/dt2: part[tap][v][c] = sum_o W2[o][c][tap] gz3[nbb(v)][o]
        float *pp = part + int64_t(tap) * a.nv * a.B;
        for (int e = tid; e < a.nv * a.B; e += NTA) {
            const int v = e / a.B, c = e - v * a.B;
            const float *zr = gz3 + nbb[v] * a.B;
            const float *wr = w2s + c * a.B;
            float sum = 0.f;
            for (int o = 0; o < a.B; o += 4) {
                const float4 z = ld4(zr + o), w = ld4(wr + o);
                sum = fmaf(z.x, w.x, fmaf(z.y, w.y, fmaf(z.z, w.z, fmaf(z.w, w.w, sum))));
            }
            pp[e] = sum;
        }
        return;
    }
    // workgroup 27: dW3[co][c] = scale * sum_v g[v][co] t3[v][c]; dscale = sum W3 * G3; db4 = sum g
    float p_sc = 0.f, p_b4 = 0.f;
    for (int e = tid; e < a.C * a.B; e += NTA) {
        const int co = e / a.B, c = e - co * a.B;
        float sum = 0.f;
        for (int v = 0; v < a.nv; ++v) sum = fmaf(gs[v * a.C + co], t3[v * a.B + c], sum);
        if (gr.dw3) atomicAdd(gr.dw3 + e, sum * sc.scale);
        p_sc = fmaf(w3t[c * a.C + co], sum, p_sc);
    }
    for (int e = tid; e < a.nv * a.C; e += NTA) p_b4 += gs[e];
    const float t_b4 = bsum<NTA>(p_b4, red), t_sc = bsum<NTA>(p_sc, red), t_b3b = bsum<NTA>(p_b3b, red),
                t_b3a = bsum<NTA>(p_b3a, red);
    if (tid == 0) {
        if (gr.dbias4) atomicAdd(gr.dbias4, t_b4);
        if (gr.dscale) atomicAdd(gr.dscale, t_sc);
        if (gr.dbias3b) atomicAdd(gr.dbias3b, t_b3b);
        if (gr.dbias3a) atomicAdd(gr.dbias3a, t_b3a);
    }
}

// ------------------------------------------------------------------------------------ backward B
constexpr int NTB = 1024;

template <typename T>
__global__ __launch_bounds__(NTB) void k_tiny_bwd_b(TArgs a, const T *__restrict__ x, const T *__restrict__ g,
                                                   const float *__restrict__ w1, vq3d_preact_params p,
                                                   vq3d_preact_grads gr, const float *__restrict__ saved,
                                                   const float *__restrict__ part, T *__restrict__ gx) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __shared__ float red[NTB / 64];
    float *xs = sm;                // [nv][C]
    float *u1 = xs + a.nv * a.C;   // [nv][C]
    float *gz1 = u1 + a.nv * a.C;  // [nv][B]
    float *w1t = gz1 + a.nv * a.B;  // [C][B]
    const int tid = threadIdx.x;
    load_act(x, xs, a.nv * a.C);
    load_w1t(a, w1, w1t);
    const Scal sc = load_scal(p);
    float p_b2b = 0.f, p_b2a = 0.f, p_b1b = 0.f, p_b1a = 0.f;
    const int nvb = a.nv * a.B;
    for (int e = tid; e < nvb; e += NTB) {  // dL/dt2 = sum of the 27 tap partials (fixed order)
        float s = 0.f;
        for (int t = 0; t < 27; ++t) s += part[t * nvb + e];
        p_b2b += s;
        const float z = s * elu_d_act(saved[e], sc.b2b);
        p_b2a += z;
        gz1[e] = z;
    }
    __syncthreads();
    for (int i = tid; i < a.nv * a.C; i += NTB) u1[i] = elu(xs[i] + sc.b1a) + sc.b1b;
    __syncthreads();
    // dW1[o][c] = sum_v gz1[v][o] u1[v][c]  |  gx = g + (W1^T gz1) * elu'(x + b1a)
    const int C4 = a.C / 4;
    const int n1 = a.B * a.C, n2 = a.nv * C4;
    for (int e = tid; e < n1 + n2; e += NTB) {
        if (e < n1) {
            const int o = e / a.C, c = e - o * a.C;
            float sum = 0.f;
            for (int v = 0; v < a.nv; ++v) sum = fmaf(gz1[v * a.B + o], u1[v * a.C + c], sum);
            if (gr.dw1) atomicAdd(gr.dw1 + e, sum);
        } else {
            const int q = e - n1, v = q / C4, c0 = (q - v * C4) * 4;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
            for (int o = 0; o < a.B; o += 4) dot4x4(acc, ld4(gz1 + v * a.B + o), w1t + c0 * a.B + o, a.B);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = c0 + j;
                p_b1b += acc[j];
                const float gxp = acc[j] * elu_grad(xs[v * a.C + c] + sc.b1a);
                p_b1a += gxp;
                st(gx + v * a.C + c, ld(g + v * a.C + c) + gxp);
            }
        }
    }
    const float t_b2b = bsum<NTB>(p_b2b, red), t_b2a = bsum<NTB>(p_b2a, red), t_b1b = bsum<NTB>(p_b1b, red),
                t_b1a = bsum<NTB>(p_b1a, red);
    if (tid == 0) {
        if (gr.dbias2b) atomicAdd(gr.dbias2b, t_b2b);
        if (gr.dbias2a) atomicAdd(gr.dbias2a, t_b2a);
        if (gr.dbias1b) atomicAdd(gr.dbias1b, t_b1b);
        if (gr.dbias1a) atomicAdd(gr.dbias1a, t_b1a);
    }
}

constexpr size_t kLdsMax = 150 * 1024;

size_t lds_fwd(const TArgs &a) {
    return (2 * size_t(a.nv) * a.C + size_t(a.nv) * a.B + VPW * a.B + 2 * a.C * a.B + 27 * a.B * a.B + VPW * 27) * 4;
}
size_t lds_a(const TArgs &a) {
    return (size_t(a.nv) * a.C + 3 * size_t(a.nv) * a.B + a.B * a.C + a.B * a.B + 2 * size_t(a.nv)) * 4;
}
size_t lds_b(const TArgs &a) { return (2 * size_t(a.nv) * a.C + size_t(a.nv) * a.B + a.C * a.B) * 4; }

int check(int batch, int C, int B, int H, int W, int D, TArgs &a) {
    a.nv = batch * H * W * D;
    a.C = C;
    a.B = B;
    a.H = H;
    a.W = W;
    a.D = D;
    if (batch < 1 || H < 1 || W < 1 || D < 1 || a.nv > MAXV || C > MAXC || B > MAXB || C % 4 || B % 4 || C < 4 ||
        B < 4 || lds_fwd(a) > kLdsMax || lds_a(a) > kLdsMax || lds_b(a) > kLdsMax)
        return fail("preact_block: shape outside the tiny-grid fused kernels");
    return 0;
}

template <typename K>
void allow_lds(K kern) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(kLdsMax));
    (void)hipGetLastError();
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_tiny_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    TArgs a;
    return check(batch, channels, branch, h, w, dd, a) == 0 ? 1 : 0;
}

size_t vq3d_preact_tiny_saved_floats(int32_t batch, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    return size_t(2) * batch * h * w * dd * branch;
}

size_t vq3d_preact_tiny_workspace_floats(int32_t batch, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    return size_t(27) * batch * h * w * dd * branch;
}

int vq3d_preact_tiny_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                         int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                         const vq3d_preact_params *p, void *out, float *saved, vq3d_stream_t stream) {
    TArgs a;
    if (int r = check(batch, channels, branch, h, w, dd, a)) return r;
    if (!x || !w1 || !w2 || !w3 || !p || !out || !saved) return fail("preact_tiny_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    static bool attr = false;
    if (!attr) {
        allow_lds(k_tiny_fwd<h16_t>);
        allow_lds(k_tiny_fwd<float>);
        attr = true;
    }
    const unsigned nwg = unsigned((a.nv + VPW - 1) / VPW);
    if (dtype == VQ3D_HALF)
        k_tiny_fwd<h16_t><<<nwg, NTF, lds_fwd(a), s>>>(a, (const h16_t *)x, w1, w2, w3, *p, (h16_t *)out, saved);
    else
        k_tiny_fwd<float><<<nwg, NTF, lds_fwd(a), s>>>(a, (const float *)x, w1, w2, w3, *p, (float *)out, saved);
    return check_launch("preact_tiny_fwd");
}

int vq3d_preact_tiny_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                         int32_t dd, const void *x, const void *g, const float *w1, const float *w2, const float *w3,
                         const vq3d_preact_params *p, const vq3d_preact_grads *gr, const float *saved,
                         float *workspace, void *gx, vq3d_stream_t stream) {
    TArgs a;
    if (int r = check(batch, channels, branch, h, w, dd, a)) return r;
    if (!x || !g || !w1 || !w2 || !w3 || !p || !gr || !saved || !workspace || !gx)
        return fail("preact_tiny_bwd: null pointer");
    hipStream_t s = as_stream(stream);
    static bool attr = false;
    if (!attr) {
        allow_lds(k_tiny_bwd_a<h16_t>);
        allow_lds(k_tiny_bwd_a<float>);
        allow_lds(k_tiny_bwd_b<h16_t>);
        allow_lds(k_tiny_bwd_b<float>);
        attr = true;
    }
    if (dtype == VQ3D_HALF) {
        k_tiny_bwd_a<h16_t><<<28, NTA, lds_a(a), s>>>(a, (const h16_t *)g, w2, w3, *p, *gr, saved, workspace);
        k_tiny_bwd_b<h16_t><<<1, NTB, lds_b(a), s>>>(a, (const h16_t *)x, (const h16_t *)g, w1, *p, *gr, saved,
                                                      workspace, (h16_t *)gx);
    } else {
        k_tiny_bwd_a<float><<<28, NTA, lds_a(a), s>>>(a, (const float *)g, w2, w3, *p, *gr, saved, workspace);
        k_tiny_bwd_b<float><<<1, NTB, lds_b(a), s>>>(a, (const float *)x, (const float *)g, w1, *p, *gr, saved,
                                                     workspace, (float *)gx);
    }
    return check_launch("preact_tiny_bwd");
}

}  // extern "C"
