// One whole PreActFixupResBlock (vqvae/layers.py:102-216, mode 'same', no skip conv) in ONE
// workgroup, forward and backward, for the tiny top-level grids (8x8x2 = 128 voxels at 32
// channels: 100 of these blocks per training step in the published 3-layer model).  At this
// size every separate conv launch is pure fixed cost; here the block's activations, its three
// weight tensors and all intermediates stay in LDS (fp32) and the backward recomputes the
// forward intermediates instead of saving them.
//
//   u1  = elu(x + b1a) + b1b                     t2 = elu(W1 u1 + b2a) + b2b        (1x1, C -> B)
//   t3  = elu(W2 * t2 + b3a) + b3b  (3x3x3 circular, B -> B)
//   out = scale * (W3 t3) + b4 + x                                                (1x1, B -> C)
//
// Threads own (voxel, 4 output channels) for the convs and (4 x 4 weight entries) for the
// weight gradients; weights are stored with the 4-channel group innermost so operand reads are
// 16-byte LDS loads.  Scalar gradients are block reductions (fixed order); weight / scalar
// gradients are added to the fp32 gradient buffers.
#include "engines.h"

#include <algorithm>

namespace vq3d {

namespace {

constexpr int NT = 1024;  // threads per workgroup
constexpr int MAXV = 256, MAXC = 32, MAXB = 16;

struct TArgs {
    int nv, C, B, H, W, D;  // voxels (batch folded in), channels, branch channels, grid
};

__device__ __forceinline__ int nbr(const TArgs &a, int v, int tap, int sgn) {
    // circular neighbour of voxel v at tap (kh, kw, kd) in {0,1,2}^3; sgn = -1 for the transpose
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

template <typename T>
__device__ __forceinline__ void load_act(const T *__restrict__ src, float *dst, int n) {
    for (int i = threadIdx.x; i < n; i += NT) dst[i] = ld(src + i);
}

// LDS layouts (floats): activations [nv][C] / [nv][B]; W1t [C][B] (in-major, out innermost),
// W2t [tap][B in][B out], W3t [B][C] so output-channel groups of 4 are contiguous; the circular
// neighbour table nb[v][tap] (uint16) is built once per launch (no divides in the conv loops).
struct Smem {
    float *x, *u1, *t2, *t3, *w1, *w2, *w3, *end;
    uint16_t *nb;
};

__device__ __forceinline__ Smem carve(float *sm, const TArgs &a) {
    Smem s;
    // every region a multiple of 4 floats (C, B multiples of 4): float4 reads stay aligned
    s.x = sm;
    s.u1 = s.x + a.nv * a.C;
    s.t2 = s.u1 + a.nv * a.C;
    s.t3 = s.t2 + a.nv * a.B;
    s.w1 = s.t3 + a.nv * a.B;
    s.w2 = s.w1 + a.C * a.B;
    s.w3 = s.w2 + 27 * a.B * a.B;
    s.nb = reinterpret_cast<uint16_t *>(s.w3 + a.B * a.C);
    s.end = s.w3 + a.B * a.C + (a.nv * 27 + 7) / 8 * 4;
    return s;
}

__device__ __forceinline__ void load_weights(const TArgs &a, const float *w1, const float *w2, const float *w3,
                                             Smem &s) {
    for (int i = threadIdx.x; i < a.B * a.C; i += NT) {  // W1 [B][C] -> [C][B]
        const int o = i / a.C, c = i - o * a.C;
        s.w1[c * a.B + o] = w1[i];
    }
    for (int i = threadIdx.x; i < a.B * a.B * 27; i += NT) {  // W2 [o][c][tap] -> [tap][c][o]
        const int tap = i % 27, r = i / 27, c = r % a.B, o = r / a.B;
        s.w2[(tap * a.B + c) * a.B + o] = w2[i];
    }
    for (int i = threadIdx.x; i < a.C * a.B; i += NT) {  // W3 [C][B] -> [B][C]
        const int o = i / a.B, c = i - o * a.B;
        s.w3[c * a.C + o] = w3[i];
    }
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

// u1, the neighbour table, then t2 and t3 from x (all in LDS); x, weights loaded + synced
__device__ void forward_t2_t3(const TArgs &a, const Scal &sc, Smem &s) {
    for (int i = threadIdx.x; i < a.nv * a.C; i += NT) s.u1[i] = elu(s.x[i] + sc.b1a) + sc.b1b;
    for (int i = threadIdx.x; i < a.nv * 27; i += NT) {
        const int v = i / 27;
        s.nb[i] = uint16_t(nbr(a, v, i - v * 27, 1));
    }
    __syncthreads();
    const int B4 = a.B / 4;
    // t2 = elu(W1 u1 + b2a) + b2b
    for (int e = threadIdx.x; e < a.nv * B4; e += NT) {
        const int v = e / B4, o0 = (e - v * B4) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float *ur = s.u1 + v * a.C;
        for (int c = 0; c < a.C; ++c) fma4(acc, ur[c], ld4(s.w1 + c * a.B + o0));
#pragma unroll
        for (int j = 0; j < 4; ++j) s.t2[v * a.B + o0 + j] = elu(acc[j] + sc.b2a) + sc.b2b;
    }
    __syncthreads();
    // t3 = elu(W2 * t2 + b3a) + b3b
    for (int e = threadIdx.x; e < a.nv * B4; e += NT) {
        const int v = e / B4, o0 = (e - v * B4) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int tap = 0; tap < 27; ++tap) {
            const float *tr = s.t2 + int(s.nb[v * 27 + tap]) * a.B;
            const float *wr = s.w2 + tap * a.B * a.B + o0;
            for (int c = 0; c < a.B; c += 4) {
                const float4 t = ld4(tr + c);
                fma4(acc, t.x, ld4(wr + c * a.B));
                fma4(acc, t.y, ld4(wr + (c + 1) * a.B));
                fma4(acc, t.z, ld4(wr + (c + 2) * a.B));
                fma4(acc, t.w, ld4(wr + (c + 3) * a.B));
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) s.t3[v * a.B + o0 + j] = elu(acc[j] + sc.b3a) + sc.b3b;
    }
    __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(NT) void k_preact_tiny_fwd(TArgs a, const T *__restrict__ x, const float *w1,
                                                       const float *w2, const float *w3, vq3d_preact_params p,
                                                       T *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    Smem s = carve(sm, a);
    load_act(x, s.x, a.nv * a.C);
    load_weights(a, w1, w2, w3, s);
    const Scal sc = load_scal(p);
    __syncthreads();
    forward_t2_t3(a, sc, s);
    // out = scale * W3 t3 + b4 + x
    const int C4 = a.C / 4;
    for (int e = threadIdx.x; e < a.nv * C4; e += NT) {
        const int v = e / C4, o0 = (e - v * C4) * 4;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float *tr = s.t3 + v * a.B;
        for (int c = 0; c < a.B; ++c) fma4(acc, tr[c], ld4(s.w3 + c * a.C + o0));
#pragma unroll
        for (int j = 0; j < 4; ++j)
            st(out + v * a.C + o0 + j, acc[j] * sc.scale + sc.b4 + s.x[v * a.C + o0 + j]);
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

// Each phase runs its weight-gradient items and its data-gradient items side by side over one
// combined index range so all 16 waves stay busy.
template <typename T>
__global__ __launch_bounds__(NT) void k_preact_tiny_bwd(TArgs a, const T *__restrict__ x, const T *__restrict__ g,
                                                       const float *w1, const float *w2, const float *w3,
                                                       vq3d_preact_params p, vq3d_preact_grads gr,
                                                       T *__restrict__ gx) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __shared__ float red[NT / 64];
    Smem s = carve(sm, a);
    float *gs = s.end;              // g       [nv][C]
    float *gz3 = gs + a.nv * a.C;   // dL/dz3  [nv][B]
    float *gz1 = gz3 + a.nv * a.B;  // dL/dz1  [nv][B]
    load_act(x, s.x, a.nv * a.C);
    load_act(g, gs, a.nv * a.C);
    load_weights(a, w1, w2, w3, s);
    const Scal sc = load_scal(p);
    __syncthreads();
    forward_t2_t3(a, sc, s);
    const int B4 = a.B / 4, C4 = a.C / 4;
    float p_b4 = 0.f, p_b3b = 0.f, p_b3a = 0.f, p_b2b = 0.f, p_b2a = 0.f, p_b1b = 0.f, p_b1a = 0.f, p_sc = 0.f;

    // ---- conv3: gz3 = scale * W3^T g * elu'(t3)  |  dW3[co][c] = scale * sum_v g[v][co] t3[v][c],
    // dscale = sum W3 * G3, db4 = sum g
    {
        const int n1 = a.nv * B4, n2 = a.C * a.B;
        for (int e = threadIdx.x; e < n1 + n2; e += NT) {
            if (e < n1) {
                const int v = e / B4, c0 = (e - v * B4) * 4;
                float acc[4] = {0.f, 0.f, 0.f, 0.f};
                for (int co = 0; co < a.C; co += 4)
                    dot4x4(acc, ld4(gs + v * a.C + co), s.w3 + c0 * a.C + co, a.C);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float h3 = acc[j] * sc.scale;
                    p_b3b += h3;
                    const float z = h3 * elu_d_act(s.t3[v * a.B + c0 + j], sc.b3b);
                    p_b3a += z;
                    gz3[v * a.B + c0 + j] = z;
                }
            } else {
                const int q = e - n1, co = q / a.B, c = q - co * a.B;
                float sum = 0.f;
                for (int v = 0; v < a.nv; ++v) sum = fmaf(gs[v * a.C + co], s.t3[v * a.B + c], sum);
                if (gr.dw3) atomicAdd(gr.dw3 + q, sum * sc.scale);
                p_sc = fmaf(s.w3[c * a.C + co], sum, p_sc);
            }
        }
        for (int e = threadIdx.x; e < a.nv * a.C; e += NT) p_b4 += gs[e];
    }
    __syncthreads();

    // ---- conv2 (3x3x3 circular): dW2[o][c][tap] = sum_v gz3[v][o] t2[nbr(v,tap)][c]  |
    // gt2[v][c] = sum_tap sum_o W2[o][c][tap] gz3[nbr(v, 26 - tap)][o], gz1 = gt2 * elu'(t2)
    {
        const int n1 = 27 * B4 * B4, n2 = a.nv * B4;
        for (int e = threadIdx.x; e < n1 + n2; e += NT) {
            if (e < n1) {
                const int tap = e / (B4 * B4), r = e - tap * B4 * B4, og = r / B4, cg = r - og * B4;
                float acc[4][4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
                for (int v = 0; v < a.nv; ++v) {
                    const int n = s.nb[v * 27 + tap];
                    const float4 gq = ld4(gz3 + v * a.B + og * 4);
                    const float4 tq = ld4(s.t2 + n * a.B + cg * 4);
                    const float go[4] = {gq.x, gq.y, gq.z, gq.w};
#pragma unroll
                    for (int i = 0; i < 4; ++i) fma4(acc[i], go[i], tq);
                }
                if (gr.dw2) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            atomicAdd(gr.dw2 + ((og * 4 + i) * a.B + cg * 4 + j) * 27 + tap, acc[i][j]);
                }
            } else {
                const int q = e - n1, v = q / B4, c0 = (q - v * B4) * 4;
                float acc[4] = {0.f, 0.f, 0.f, 0.f};
                for (int tap = 0; tap < 27; ++tap) {
                    const float *zr = gz3 + int(s.nb[v * 27 + 26 - tap]) * a.B;
                    const float *wr = s.w2 + tap * a.B * a.B + c0 * a.B;  // [tap][c][o]
                    for (int o = 0; o < a.B; o += 4) dot4x4(acc, ld4(zr + o), wr + o, a.B);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float gt2 = acc[j];
                    p_b2b += gt2;
                    const float z = gt2 * elu_d_act(s.t2[v * a.B + c0 + j], sc.b2b);
                    p_b2a += z;
                    gz1[v * a.B + c0 + j] = z;
                }
            }
        }
    }
    __syncthreads();

    // ---- conv1: dW1[o][c] = sum_v gz1[v][o] u1[v][c]  |  gu1 = W1^T gz1, gx = g + gu1 * elu'(x + b1a)
    {
        const int n1 = a.B * a.C, n2 = a.nv * C4;
        for (int e = threadIdx.x; e < n1 + n2; e += NT) {
            if (e < n1) {
                const int o = e / a.C, c = e - o * a.C;
                float sum = 0.f;
                for (int v = 0; v < a.nv; ++v) sum = fmaf(gz1[v * a.B + o], s.u1[v * a.C + c], sum);
                if (gr.dw1) atomicAdd(gr.dw1 + e, sum);
            } else {
                const int q = e - n1, v = q / C4, c0 = (q - v * C4) * 4;
                float acc[4] = {0.f, 0.f, 0.f, 0.f};
                for (int o = 0; o < a.B; o += 4) dot4x4(acc, ld4(gz1 + v * a.B + o), s.w1 + c0 * a.B + o, a.B);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = c0 + j;
                    const float gu1 = acc[j];
                    p_b1b += gu1;
                    const float gxp = gu1 * elu_grad(s.x[v * a.C + c] + sc.b1a);
                    p_b1a += gxp;
                    st(gx + v * a.C + c, gs[v * a.C + c] + gxp);
                }
            }
        }
    }
    // ---- scalar gradients (fixed-order block sums)
    const float t_b4 = bsum<NT>(p_b4, red), t_sc = bsum<NT>(p_sc, red), t_b3b = bsum<NT>(p_b3b, red),
                t_b3a = bsum<NT>(p_b3a, red), t_b2b = bsum<NT>(p_b2b, red), t_b2a = bsum<NT>(p_b2a, red),
                t_b1b = bsum<NT>(p_b1b, red), t_b1a = bsum<NT>(p_b1a, red);
    if (threadIdx.x == 0) {
        if (gr.dbias4) atomicAdd(gr.dbias4, t_b4);
        if (gr.dscale) atomicAdd(gr.dscale, t_sc);
        if (gr.dbias3b) atomicAdd(gr.dbias3b, t_b3b);
        if (gr.dbias3a) atomicAdd(gr.dbias3a, t_b3a);
        if (gr.dbias2b) atomicAdd(gr.dbias2b, t_b2b);
        if (gr.dbias2a) atomicAdd(gr.dbias2a, t_b2a);
        if (gr.dbias1b) atomicAdd(gr.dbias1b, t_b1b);
        if (gr.dbias1a) atomicAdd(gr.dbias1a, t_b1a);
    }
}

constexpr size_t kLdsMax = 150 * 1024;

size_t lds_bytes(const TArgs &a, bool bwd) {
    const size_t act = size_t(a.nv) * a.C + 2 * size_t(a.nv) * a.B;
    const size_t nb = (size_t(a.nv) * 27 + 7) / 8 * 4;  // uint16 table in floats, 16-B multiple
    return (act + size_t(a.nv) * a.C + 2 * size_t(a.C) * a.B + 27 * size_t(a.B) * a.B + nb + (bwd ? act : 0)) * 4;
}

int check(int batch, int C, int B, int H, int W, int D, TArgs &a) {
    a.nv = batch * H * W * D;
    a.C = C;
    a.B = B;
    a.H = H;
    a.W = W;
    a.D = D;
    if (a.nv > MAXV || C > MAXC || B > MAXB || C % 4 || B % 4 || C < 4 || B < 4 || H < 1 || W < 1 || D < 1 ||
        batch < 1 || lds_bytes(a, true) > kLdsMax)
        return fail("preact_block: shape outside the tiny-grid fused kernel");
    return 0;
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_preact_tiny_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd) {
    TArgs a;
    return check(batch, channels, branch, h, w, dd, a) == 0 ? 1 : 0;
}

int vq3d_preact_tiny_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                         int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                         const vq3d_preact_params *p, void *out, vq3d_stream_t stream) {
    TArgs a;
    if (int r = check(batch, channels, branch, h, w, dd, a)) return r;
    if (!x || !w1 || !w2 || !w3 || !p || !out) return fail("preact_tiny_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    const size_t lds = lds_bytes(a, false);
    if (dtype == VQ3D_BF16)
        k_preact_tiny_fwd<bf16_t><<<1, NT, lds, s>>>(a, (const bf16_t *)x, w1, w2, w3, *p, (bf16_t *)out);
    else
        k_preact_tiny_fwd<float><<<1, NT, lds, s>>>(a, (const float *)x, w1, w2, w3, *p, (float *)out);
    return check_launch("preact_tiny_fwd");
}

int vq3d_preact_tiny_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                         int32_t dd, const void *x, const void *g, const float *w1, const float *w2, const float *w3,
                         const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *gx, vq3d_stream_t stream) {
    TArgs a;
    if (int r = check(batch, channels, branch, h, w, dd, a)) return r;
    if (!x || !g || !w1 || !w2 || !w3 || !p || !gr || !gx) return fail("preact_tiny_bwd: null pointer");
    hipStream_t s = as_stream(stream);
    const size_t lds = lds_bytes(a, true);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_preact_tiny_bwd<bf16_t>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsMax));
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_preact_tiny_bwd<float>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsMax));
        (void)hipGetLastError();
        attr = true;
    }
    if (dtype == VQ3D_BF16)
        k_preact_tiny_bwd<bf16_t><<<1, NT, lds, s>>>(a, (const bf16_t *)x, (const bf16_t *)g, w1, w2, w3, *p, *gr,
                                                     (bf16_t *)gx);
    else
        k_preact_tiny_bwd<float><<<1, NT, lds, s>>>(a, (const float *)x, (const float *)g, w1, w2, w3, *p, *gr,
                                                    (float *)gx);
    return check_launch("preact_tiny_bwd");
}

}  // extern "C"
