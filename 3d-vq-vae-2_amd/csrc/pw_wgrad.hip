// 1x1x1 convolution weight gradient (nn.Conv3d kernel_size=1 at the block convs 1 / 3 and
// the skip / proj / parse_input / out convs: vqvae/layers.py:134-171, 377, 490, 508, 535).
//
//   G[co][ci] = sum_v g[v][co] * pro(x)[v][ci]        (x channels then x2 channels: torch.cat)
//
// is a GEMM whose reduction runs over the voxels.  Channels-last slabs of `seg` consecutive
// voxels are contiguous for both x and g, so each workgroup streams them through LDS with
// 16-byte loads (all of a segment's loads in flight before the first is unpacked; the
// prologue elu(x + a) + b applied once per element) and every thread accumulates a 4x4
// (ci, co) tile over its voxel sub-stream.  A constant-1 column appended to x yields
// sum_v g[v][co] (conv-bias / scalar-bias gradients) from the same loop.
//
// Reduction is deterministic and atomic-free on the data: sub-streams are summed in a fixed
// order through LDS, each workgroup writes its partial G to the caller's workspace, and a
// second kernel sums the partials in workgroup order and adds them to the fp32 gradients
// (thousands of same-address atomics serialise at the L2 and were the bottleneck).
#include "engines.h"

#include <algorithm>
#include <cstdlib>

namespace vq3d {

namespace {

constexpr int TI = 4, TO = 4;  // thread tile: input x output channels
constexpr int kMaxBlocks = 2048;

struct PwwArgs {
    int64_t nvox;
    int Ca, Cb, N;
    int Xp, Gp;   // LDS row strides (floats) of the x and g slabs
    int ones;     // column of the constant-1 entry in the x slab (Ct)
    int ne;       // partial entries per workgroup: N x (Ct + 1)
    int seg;      // voxels per segment
    int nti;      // ci tiles
    int tpb;      // tiles per workgroup
    int S;        // voxel sub-streams per workgroup
    int vec;      // every slab base 16-B aligned
    FastDiv fa, fb, fn;
};

// Load a segment's slab (U x 16 B per thread in flight), then unpack:
// dst[v * P + off + c] = f(src[v * C + c]) for v < nv.
template <typename T, bool PRO, int U>
__device__ __forceinline__ void stage(float *__restrict__ dst, int P, int off, const T *__restrict__ src, int nv,
                                      int C, const FastDiv &fd, const Prologue &pro, bool vec) {
    constexpr int E = 16 / sizeof(T);
    const int n = nv * C;
    const int nq = vec ? n / E : 0;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    for (int q0 = threadIdx.x; q0 < nq; q0 += U * 256) {
        uint4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (q0 + u * 256 < nq) r[u] = s4[q0 + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = q0 + u * 256;
            if (q >= nq) break;
            const T *el = reinterpret_cast<const T *>(&r[u]);
            int v = int(fd.div(uint32_t(q * E))), c = q * E - v * C;
#pragma unroll
            for (int j = 0; j < E; ++j) {
                const float val = ld(el + j);
                dst[v * P + off + c] = PRO ? pro.apply(val) : val;
                if (++c == C) {
                    c = 0;
                    ++v;
                }
            }
        }
    }
    for (int e = nq * E + threadIdx.x; e < n; e += 256) {
        const int v = int(fd.div(uint32_t(e))), c = e - v * C;
        const float val = ld(src + e);
        dst[v * P + off + c] = PRO ? pro.apply(val) : val;
    }
}

// Final accumulation of one gradient entry e = co * (Ct + 1) + ci into the fp32 gradients
// (atomics: the reduce kernel owns an entry exclusively, direct-mode workgroups are few);
// the scale / scalar-bias contributions go to wg / bs for a block reduction.
struct WgOut {
    const float *w, *escale;
    float *dw, *dscale, *dbias, *dcbias;
    GridSum gsum;  // direct mode over several workgroups (the 2-D k_pw_wgrad grid): the scalar sums
};

__device__ __forceinline__ void finish_entry(const WgOut &o, int e, int Ct, float sum, float &wg, float &bs) {
    const int co = e / (Ct + 1), ci = e - co * (Ct + 1);
    if (ci < Ct) {
        const int64_t idx = int64_t(co) * Ct + ci;
        if (o.dw) atomicAdd(o.dw + idx, o.escale ? sum * *o.escale : sum);
        if (o.dscale) wg = fmaf(o.w[idx], sum, wg);
    } else {
        if (o.dcbias) atomicAdd(o.dcbias + co, sum);
        bs += sum;
    }
}

__device__ __forceinline__ void finish_block(const WgOut &o, float wg, float bs, float *red) {
    if (!o.dscale && !o.dbias) return;
    {  // both sums in one barrier pair (bit-identical to two block_sum calls)
        float pp[2] = {wg, bs};
        block_sums<float, 256, 2, 4>(pp, red);
        wg = pp[0];
        bs = pp[1];
    }
    grid_sum2<256>(o.gsum, wg, bs, o.dscale, o.dbias, red);
}

template <typename T>
__global__ __launch_bounds__(256) void k_pw_wgrad(PwwArgs a, const T *__restrict__ x, const T *__restrict__ x2,
                                                 const T *__restrict__ g, int pro_kind, const float *pro_a,
                                                 const float *pro_b, float *__restrict__ part, WgOut out) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    __shared__ float red[8];
    float *xs = sm;                     // [seg][Xp]
    float *gs = sm + a.seg * a.Xp;      // [seg][Gp]
    const int tid = threadIdx.x;
    const int Ct = a.Ca + a.Cb;
    const Prologue pro = make_prologue(pro_kind, pro_a, pro_b);
    const int tl = tid % a.tpb, sub = tid / a.tpb;
    const int tile = blockIdx.y * a.tpb + tl;
    const int ntiles = a.nti * (a.Gp / TO);
    const bool active = sub < a.S && tile < ntiles;
    const int ci0 = (tile % a.nti) * TI, co0 = (tile / a.nti) * TO;

    // columns the staging never writes: zero padding and the constant-1 column
    for (int e = tid; e < a.seg * a.Xp; e += 256) {
        const int c = e % a.Xp;
        if (c >= Ct) xs[e] = c == a.ones ? 1.f : 0.f;
    }
    for (int e = tid; e < a.seg * a.Gp; e += 256)
        if (e % a.Gp >= a.N) gs[e] = 0.f;

    float acc[TI][TO];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TO; ++j) acc[i][j] = 0.f;

    const int64_t nseg = (a.nvox + a.seg - 1) / a.seg;
    for (int64_t sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const int64_t v0 = sg * a.seg;
        const int nv = int(min<int64_t>(a.seg, a.nvox - v0));
        __syncthreads();
        if (pro.kind == VQ3D_PRO_NONE) {
            stage<T, false, 4>(xs, a.Xp, 0, x + v0 * a.Ca, nv, a.Ca, a.fa, pro, a.vec);
            if (a.Cb) stage<T, false, 2>(xs, a.Xp, a.Ca, x2 + v0 * a.Cb, nv, a.Cb, a.fb, pro, a.vec);
        } else {
            stage<T, true, 4>(xs, a.Xp, 0, x + v0 * a.Ca, nv, a.Ca, a.fa, pro, a.vec);
            if (a.Cb) stage<T, true, 2>(xs, a.Xp, a.Ca, x2 + v0 * a.Cb, nv, a.Cb, a.fb, pro, a.vec);
        }
        stage<T, false, 4>(gs, a.Gp, 0, g + v0 * a.N, nv, a.N, a.fn, pro, a.vec);
        __syncthreads();
        if (active) {
            for (int v = sub; v < nv; v += a.S) {
                const float4 xv = *reinterpret_cast<const float4 *>(xs + v * a.Xp + ci0);
                const float4 gv = *reinterpret_cast<const float4 *>(gs + v * a.Gp + co0);
                const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ga[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TO; ++j) acc[i][j] = fmaf(xa[i], ga[j], acc[i][j]);
            }
        }
    }
    // fixed-order reduction of the sub-streams (one thread per tile entry), partial -> workspace
    __syncthreads();
#pragma unroll
    for (int q = 0; q < TI * TO; ++q) sm[q * 256 + tid] = acc[q / TO][q % TO];
    __syncthreads();
    const int nblk = gridDim.x;
    float wg = 0.f, bs = 0.f;
    for (int idx = tid; idx < a.tpb * TI * TO; idx += 256) {
        const int q = idx / a.tpb, t = idx - q * a.tpb;
        const int tt = blockIdx.y * a.tpb + t;
        if (tt >= ntiles) continue;
        const int ci = (tt % a.nti) * TI + q / TO, co = (tt / a.nti) * TO + q % TO;
        if (co >= a.N || ci > Ct) continue;
        float sum = 0.f;
        for (int j = 0; j < a.S; ++j) sum += sm[q * 256 + j * a.tpb + t];
        if (part) part[int64_t(co * (Ct + 1) + ci) * nblk + blockIdx.x] = sum;
        else finish_entry(out, co * (Ct + 1) + ci, Ct, sum, wg, bs);
    }
    if (!part) finish_block(out, wg, bs, red);
}

// Few-channel convs (x: CX, g: CG channels, both in {1, 2, 4, 8}, one input): each thread
// streams whole voxel rows straight from HBM (one vector load per row, 4 voxels in flight) and
// keeps every (ci, co) product plus the bias column in registers; wave shuffles + one LDS
// pass reduce the workgroup, which writes its partials like k_pw_wgrad.
template <typename T, int C>
__device__ __forceinline__ void load_row(const T *__restrict__ p, float (&o)[C]) {
    if constexpr (sizeof(T) == 2) {
        if constexpr (C == 1) {
            o[0] = ld(p);
        } else if constexpr (C == 2) {
            const uint32_t u = *reinterpret_cast<const uint32_t *>(p);
            o[0] = h2f_lo(u);
            o[1] = h2f_hi(u);
        } else if constexpr (C == 4) {
            const uint2 u = *reinterpret_cast<const uint2 *>(p);
            const uint32_t w[2] = {u.x, u.y};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                o[2 * j] = h2f_lo(w[j]);
                o[2 * j + 1] = h2f_hi(w[j]);
            }
        } else if constexpr (C == 8) {
            const uint4 u = *reinterpret_cast<const uint4 *>(p);
            const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[2 * j] = h2f_lo(w[j]);
                o[2 * j + 1] = h2f_hi(w[j]);
            }
        } else if constexpr (C % 2 == 0) {  // rows 4-byte aligned
            const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
#pragma unroll
            for (int j = 0; j < C / 2; ++j) {
                const uint32_t u = q[j];
                o[2 * j] = h2f_lo(u);
                o[2 * j + 1] = h2f_hi(u);
            }
        } else {
#pragma unroll
            for (int j = 0; j < C; ++j) o[j] = ld(p + j);
        }
    } else {
#pragma unroll
        for (int j = 0; j < C; ++j) o[j] = p[j];
    }
}

template <typename T, int CX, int CG, int U = 4>
__global__ __launch_bounds__(256) void k_pw_wgrad_reg(int64_t nvox, const T *__restrict__ x,
                                                     const T *__restrict__ g, int pro_kind, const float *pro_a,
                                                     const float *pro_b, float *__restrict__ part, WgOut out) {
    constexpr int NE = CG * (CX + 1);
    __shared__ float wred[4][NE];
    __shared__ float red[8];
    const Prologue pro = make_prologue(pro_kind, pro_a, pro_b);
    float acc[CG][CX + 1];
#pragma unroll
    for (int j = 0; j < CG; ++j)
#pragma unroll
        for (int i = 0; i <= CX; ++i) acc[j][i] = 0.f;
    const int64_t stride = int64_t(gridDim.x) * 256;
    for (int64_t v0 = int64_t(blockIdx.x) * 256 + threadIdx.x; v0 < nvox; v0 += U * stride) {
        float xr[U][CX], gr[U][CG];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t v = v0 + u * stride;
            if (v < nvox) {
                load_row<T, CX>(x + v * CX, xr[u]);
                load_row<T, CG>(g + v * CG, gr[u]);
            } else {
#pragma unroll
                for (int i = 0; i < CX; ++i) xr[u][i] = 0.f;
#pragma unroll
                for (int j = 0; j < CG; ++j) gr[u][j] = 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int i = 0; i < CX; ++i) xr[u][i] = pro.apply(xr[u][i]);
#pragma unroll
            for (int j = 0; j < CG; ++j) {
#pragma unroll
                for (int i = 0; i < CX; ++i) acc[j][i] = fmaf(xr[u][i], gr[u][j], acc[j][i]);
                acc[j][CX] += gr[u][j];
            }
        }
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < CG; ++j)
#pragma unroll
        for (int i = 0; i <= CX; ++i) {
            const float t = wave_sum(acc[j][i]);
            if (lane == 0) wred[wv][j * (CX + 1) + i] = t;
        }
    __syncthreads();
    float wg = 0.f, bs = 0.f;
    if (threadIdx.x < NE) {
        const int e = threadIdx.x;
        const float sum = (wred[0][e] + wred[1][e]) + (wred[2][e] + wred[3][e]);
        if (part) part[int64_t(e) * gridDim.x + blockIdx.x] = sum;
        else finish_entry(out, e, CX, sum, wg, bs);
    }
    if (!part) finish_block(out, wg, bs, red);
}

// G = sum over the workgroup partials (part[entry][blk], fixed-order shuffle tree per entry);
// dw += escale * G, dscale += sum W*G, dcbias[co] += G[co][Ct], dbias += sum_co G[co][Ct].
// LANES lanes of a wave share one entry: each sums a strided slice of the partials (8 loads in
// flight), then the lanes combine with a fixed xor-shuffle tree.
template <int LANES>
__global__ __launch_bounds__(256) void k_pw_wgrad_reduce(const float *__restrict__ part, int nblk, int ne, int Ct,
                                                        const float *__restrict__ w, const float *__restrict__ escale,
                                                        float *dw, float *dscale, float *dbias, float *dcbias,
                                                        GridSum gsum) {
    __shared__ float red[8];
    const int lane = threadIdx.x % LANES;
    const int e = blockIdx.x * (256 / LANES) + threadIdx.x / LANES;
    float sum = 0.f;
    if (e < ne) {
        const float *p = part + int64_t(e) * nblk;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int b0 = lane; b0 < nblk; b0 += 8 * LANES) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + u * LANES < nblk) acc[u] += p[b0 + u * LANES];
        }
        sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    if constexpr (LANES > 64) {  // one entry per workgroup: waves, then the 4 wave sums in order
        __shared__ float wsum[LANES / 64];
        sum = wave_sum(sum);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = sum;
        __syncthreads();
        sum = 0.f;
#pragma unroll
        for (int i = 0; i < LANES / 64; ++i) sum += wsum[i];
    } else {
        sum = group_sum<LANES>(sum);
    }
    float wg = 0.f, bs = 0.f;
    if (e < ne && lane == 0) {
        const int co = e / (Ct + 1), ci = e - co * (Ct + 1);
        if (ci < Ct) {
            const int64_t o = int64_t(co) * Ct + ci;
            if (dw) dw[o] += escale ? sum * *escale : sum;
            if (dscale) wg = w[o] * sum;
        } else {
            if (dcbias) dcbias[co] += sum;
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

// ---- matrix cores (bf16): G^T = g^T x' over voxel chunks, v_mfma_f32_16x16x32_bf16 with
// M = output channels (co tiles), N = input channels + the constant-1 column (ci tiles), K = voxels.
// A chunk of VC voxels of x (prologue applied, rounded to bf16 as the reference's autocast conv
// input), x2 and g is staged channels-last in LDS with 16-byte loads (any channel count: a slab of
// VC voxels is contiguous); both operands come through the transposing ds_read_b64_tr_b16.  Waves
// split the co tiles (nwm of them) and the chunk's K-steps (4 / nwm); per-workgroup partials are
// combined over the K-split waves in a fixed order and written like k_pw_wgrad's.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ hx8 tr8(const h16_t *p0, const h16_t *p1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
    return __builtin_bit_cast(hx8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct WmArgs {
    int64_t nvox;
    int Ca, Cb, N, Ct;
    int VC;             // voxels per chunk (multiple of 32 x K-split)
    int XP, GP;         // LDS row pitches (elements)
    int MT, NT;         // co tiles, ci tiles (Ct + 1 columns)
    int nwm;            // waves over co tiles (1, 2, 4); 4 / nwm waves split the K-steps
    int ua, ub, ug;     // 16-byte units per chunk of x, x2, g
    int tr;             // partials workgroup-major part[blk][entry] (many entries, few workgroups)
};

constexpr int kWmU = 4;  // 16-byte units in flight per thread

template <int MPW, int NTT>
__global__ __launch_bounds__(256) void k_pw_wgrad_mma(WmArgs a, const h16_t *__restrict__ x,
                                                     const h16_t *__restrict__ x2, const h16_t *__restrict__ g,
                                                     int pro_kind, const float *pro_a, const float *pro_b,
                                                     float *__restrict__ part, WgOut out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float red[8];
    h16_t *xs = reinterpret_cast<h16_t *>(smem);  // [VC][XP]
    h16_t *gs = xs + a.VC * a.XP;                  // [VC][GP]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
    const int wm = wave % a.nwm, wk = wave / a.nwm, nwk = 4 / a.nwm;
    const Prologue pro = make_prologue(pro_kind, pro_a, pro_b);
    const bool raw = pro.kind == VQ3D_PRO_NONE;
    // columns staging never writes: the constant-1 column of x and the zero padding
    for (int v = tid; v < a.VC; v += 256) {
        for (int c = a.Ct; c < a.XP; ++c) xs[v * a.XP + c] = c == a.Ct ? f2h(1.f) : h16_t(0);
        for (int c = a.N; c < a.GP; ++c) gs[v * a.GP + c] = 0;
    }

    f32x4 acc[MPW][NTT];
#pragma unroll
    for (int i = 0; i < MPW; ++i)
#pragma unroll
        for (int t = 0; t < NTT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nu = a.ua + a.ub + a.ug;
    const int64_t nch = (a.nvox + a.VC - 1) / a.VC;
    // this thread's 16-byte units of a chunk (nu <= kWmU * 256: one round), held in registers so
    // the next chunk's loads are in flight while the current one is multiplied
    u32x4 r[kWmU];
    auto load = [&](int64_t ch) {
        const int64_t v0 = ch * a.VC;
        const int nv = int(min<int64_t>(a.VC, a.nvox - v0));
#pragma unroll
        for (int k = 0; k < kWmU; ++k) {
            const int u = tid + k * 256;
            r[k] = u32x4{0u, 0u, 0u, 0u};
            if (u >= nu) continue;
            const h16_t *src;
            int e, C;
            if (u < a.ua) src = x + v0 * a.Ca, e = 8 * u, C = a.Ca;
            else if (u < a.ua + a.ub) src = x2 + v0 * a.Cb, e = 8 * (u - a.ua), C = a.Cb;
            else src = g + v0 * a.N, e = 8 * (u - a.ua - a.ub), C = a.N;
            const int lim = nv * C;
            if (e + 8 <= lim) {
                r[k] = *reinterpret_cast<const u32x4 *>(src + e);
            } else {
                uint32_t t[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (e + j < lim) t[j >> 1] |= uint32_t(src[e + j]) << (16 * (j & 1));
                r[k] = u32x4{t[0], t[1], t[2], t[3]};
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int k = 0; k < kWmU; ++k) {
            const int u = tid + k * 256;
            if (u >= nu) continue;
            h16_t *dst;
            int e, C, off, P;
            bool isx = true;
            if (u < a.ua) e = 8 * u, C = a.Ca, off = 0, P = a.XP, dst = xs;
            else if (u < a.ua + a.ub) e = 8 * (u - a.ua), C = a.Cb, off = a.Ca, P = a.XP, dst = xs;
            else e = 8 * (u - a.ua - a.ub), C = a.N, off = 0, P = a.GP, dst = gs, isx = false;
            u32x4 w = r[k];
            if (isx && !raw)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float lo = pro.apply(h2f_lo(w[j]));
                    const float hi = pro.apply(h2f_hi(w[j]));
                    w[j] = uint32_t(f2h(lo)) | (uint32_t(f2h(hi)) << 16);
                }
            if (C % 8 == 0) {  // the unit is 8 channels of one voxel
                const int v = e / C, c = e - v * C;
                u32x2 *d2 = reinterpret_cast<u32x2 *>(dst + v * P + off + c);
                d2[0] = u32x2{w[0], w[1]};
                d2[1] = u32x2{w[2], w[3]};
            } else {
                int v = e / C, c = e - v * C;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (v < a.VC) dst[v * P + off + c] = h16_t(w[j >> 1] >> (16 * (j & 1)));
                    if (++c == C) c = 0, ++v;
                }
            }
        }
    };
    if (int64_t(blockIdx.x) < nch) load(blockIdx.x);
    for (int64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
        const int nv = int(min<int64_t>(a.VC, a.nvox - ch * a.VC));
        __syncthreads();
        store();
        if (ch + gridDim.x < nch) load(ch + gridDim.x);
        // a ragged last chunk: rows past the grid are zero (the prologue of a zero is not)
        if (nv < a.VC) {
            for (int e = tid; e < (a.VC - nv) * a.Ct; e += 256) xs[(nv + e / a.Ct) * a.XP + e % a.Ct] = 0;
            for (int e = tid; e < (a.VC - nv) * a.N; e += 256) gs[(nv + e / a.N) * a.GP + e % a.N] = 0;
        }
        __syncthreads();
        for (int ks = wk; ks < a.VC / 32; ks += nwk) {
            const int r0 = ks * 32 + 8 * grp + q;
            const h16_t *ga = gs + r0 * a.GP + 4 * p4;
            const h16_t *xa = xs + r0 * a.XP + 4 * p4;
            hx8 bfr[NTT];
#pragma unroll
            for (int t = 0; t < NTT; ++t)
                if (t < a.NT) bfr[t] = tr8(xa + 16 * t, xa + 16 * t + 4 * a.XP);
#pragma unroll
            for (int i = 0; i < MPW; ++i) {
                const int mt = wm + a.nwm * i;
                if (mt >= a.MT) break;
                const hx8 af = tr8(ga + 16 * mt, ga + 16 * mt + 4 * a.GP);
#pragma unroll
                for (int t = 0; t < NTT; ++t)
                    if (t < a.NT) acc[i][t] = VQ3D_MFMA_16X16X32(af, bfr[t], acc[i][t], 0, 0, 0);
            }
        }
    }
    // K-split waves: fixed-order sum through an LDS image [MT * 16][NT * 16]; then one pass writes
    // the partials (D[co = 16 mt + 4 grp + j][ci = 16 t + li])
    const int nblk = gridDim.x, W = a.NT * 16;
    float *img = reinterpret_cast<float *>(smem);
    float wg = 0.f, bs = 0.f;
    auto emit = [&](int co, int ci, float sum) {
        if (co >= a.N || ci > a.Ct) return;
        const int e = co * (a.Ct + 1) + ci;
        if (part) part[a.tr ? int64_t(blockIdx.x) * a.N * (a.Ct + 1) + e : int64_t(e) * nblk + blockIdx.x] = sum;
        else finish_entry(out, e, a.Ct, sum, wg, bs);
    };
    if (nwk == 1) {
#pragma unroll
        for (int i = 0; i < MPW; ++i) {
            const int mt = wm + a.nwm * i;
            if (mt >= a.MT) break;
#pragma unroll
            for (int t = 0; t < NTT; ++t)
                if (t < a.NT)
#pragma unroll
                    for (int j = 0; j < 4; ++j) emit(16 * mt + 4 * grp + j, 16 * t + li, acc[i][t][j]);
        }
    } else {
        for (int k = 0; k < nwk; ++k) {
            __syncthreads();
            if (wk == k) {
#pragma unroll
                for (int i = 0; i < MPW; ++i) {
                    const int mt = wm + a.nwm * i;
                    if (mt >= a.MT) break;
#pragma unroll
                    for (int t = 0; t < NTT; ++t)
                        if (t < a.NT)
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                float &d = img[(16 * mt + 4 * grp + j) * W + 16 * t + li];
                                d = k == 0 ? acc[i][t][j] : d + acc[i][t][j];
                            }
                }
            }
        }
        __syncthreads();
        for (int e = tid; e < a.MT * 16 * W; e += 256) emit(e / W, e % W, img[e]);
    }
    if (!part) finish_block(out, wg, bs, red);
}

// the plan of the matrix-core path, or false (fp32, > 16 accumulator tiles per wave, tiny grids)
bool plan_mma(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, WmArgs &m, int &mpw, int &ntt,
              int &nbx, size_t &lds) {
    auto al = [](const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (d->dtype != VQ3D_HALF || !al(x) || !al(x2) || !al(g)) return false;
    m = WmArgs{};
    m.nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    m.Ca = d->cin;
    m.Cb = d->cin2;
    m.N = d->cout;
    m.Ct = m.Ca + m.Cb;
    if (m.nvox < 256 || m.Ct > 255 || m.N > 128) return false;
    m.MT = (m.N + 15) / 16;
    m.NT = (m.Ct + 1 + 15) / 16;
    ntt = m.NT <= 1 ? 1 : m.NT <= 2 ? 2 : m.NT <= 4 ? 4 : m.NT <= 8 ? 8 : 16;
    m.nwm = m.MT >= 4 ? 4 : m.MT >= 2 ? 2 : 1;
    if (m.MT == 3) m.nwm = 4;
    mpw = (m.MT + m.nwm - 1) / m.nwm;
    if (mpw > 2 || mpw * ntt > 16) return false;
    if (mpw == 2 && ntt > 8) return false;
    m.XP = m.NT * 16 + 4;
    m.GP = m.MT * 16 + 4;
    const int nwk = 4 / m.nwm;
    // chunk: one round of kWmU 16-byte units per thread, at least one K-step per K-split wave,
    // at most 256 voxels
    m.VC = 256;
    while (m.VC > 32 * nwk && m.VC * (m.Ct + m.N) > kWmU * 256 * 8) m.VC /= 2;
    if (m.VC * (m.Ct + m.N) > kWmU * 256 * 8 || size_t(m.VC) * (m.XP + m.GP) * 2 > 48 * 1024) return false;
    m.ua = m.VC * m.Ca / 8;
    m.ub = m.VC * m.Cb / 8;
    m.ug = m.VC * m.N / 8;
    if ((m.VC * m.Ca) % 8 || (m.VC * m.Cb) % 8 || (m.VC * m.N) % 8) return false;
    lds = std::max(size_t(m.VC) * (m.XP + m.GP) * 2, nwk > 1 ? size_t(m.MT) * 16 * m.NT * 16 * 4 : size_t(0));
    // workgroups: enough chunks in flight, partial traffic (ne floats per workgroup) << the data
    const int64_t nch = (m.nvox + m.VC - 1) / m.VC;
    const int64_t ne = int64_t(m.N) * (m.Ct + 1);
    const int64_t data = m.nvox * (m.Ct + m.N) * 2;
    // workgroups: a chunk each on small grids (the chunk loop is load-latency bound), about 4 chunks
    // each on large ones (1024 .. 2048 workgroups; fewer partials)
    (void)data;
    (void)ne;
    nbx = int(nch <= 1024 ? nch : std::min<int64_t>(kMaxBlocks, std::max<int64_t>(1024, nch / 4)));
    // entry-major partials cost a scattered store per entry and workgroup
    m.tr = ne >= 64 * int64_t(nbx);
    return true;
}

// k_pw_wgrad_reduce for workgroup-major partials part[blk][entry]: a workgroup takes 64 entries,
// wave w sums blocks w, w + 4, ... (8 loads in flight, coalesced over the entries), the 4 wave sums
// are added in a fixed order
__global__ __launch_bounds__(256) void k_pw_wgrad_reduce_t(const float *__restrict__ part, int nblk, int ne, int Ct,
                                                          const float *__restrict__ w, const float *__restrict__ escale,
                                                          float *dw, float *dscale, float *dbias, float *dcbias,
                                                          GridSum gsum) {
    __shared__ float red[8];
    __shared__ float ws4[4][64];
    const int el = threadIdx.x & 63, bg = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + el;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (e < ne)
        for (int b0 = bg; b0 < nblk; b0 += 32) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + 4 * u < nblk) acc[u] += part[int64_t(b0 + 4 * u) * ne + e];
        }
    ws4[bg][el] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    float wg = 0.f, bs = 0.f;
    if (bg == 0 && e < ne) {
        const float sum = (ws4[0][el] + ws4[1][el]) + (ws4[2][el] + ws4[3][el]);
        const int co = e / (Ct + 1), ci = e - co * (Ct + 1);
        if (ci < Ct) {
            const int64_t o = int64_t(co) * Ct + ci;
            if (dw) dw[o] += escale ? sum * *escale : sum;
            if (dscale) wg = w[o] * sum;
        } else {
            if (dcbias) dcbias[co] += sum;
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

// ---- PixelSNAIL 1x1x1 conv weight gradient over voxel rows (the Conv3d(kernel_size=1) backward of
// pixel_model/layers.py:122-248, 650-703): dW[cg][cx] += sum_v g[v][cg] x[v][cx] and
// db[cg] += sum_v g[v][cg] for 16-bit channels-last rows of any channel count (multiples of 8).
// A workgroup owns one 64 x 64 (cg x cx) tile and a contiguous split of the rows; chunks of RW_VC
// rows are staged channels-last in LDS (16-byte loads, the next chunk's in registers while the
// current one is multiplied) and read through ds_read_b64_tr_b16 as in k_pw_wgrad_mma; each wave
// owns a 32 x 32 quadrant (2 x 2 v_mfma_f32_16x16x32 tiles) over all K-steps.  The bias sums ride
// on the cx-tile-0 workgroups (fixed-order column sums of the staged g rows).  Per-split partials
// part[split][cg][cx + 1] are summed in split order by k_pw_wgrad_reduce_t: deterministic.
constexpr int RW_VC = 128;  // rows per chunk
constexpr int RW_P = 68;    // LDS row pitch (halves)

struct RwArgs {
    int64_t nrows, rps;  // rows, rows per split (multiple of RW_VC)
    int cg, cx, ldg, ldx;
    int tx;  // cx tiles
};

__global__ __launch_bounds__(256) void k_rows_wgrad(RwArgs a, const h16_t *__restrict__ g,
                                                   const h16_t *__restrict__ x, float *__restrict__ part) {
    __shared__ __attribute__((aligned(16))) h16_t gs[RW_VC * RW_P];
    __shared__ __attribute__((aligned(16))) h16_t xs[RW_VC * RW_P];
    __shared__ float bred[4][64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
    const int wm = wave & 1, wn = wave >> 1;
    const int tcx = blockIdx.x % a.tx, tcg = blockIdx.x / a.tx;
    const int cg0 = 64 * tcg, cx0 = 64 * tcx;
    const int64_t r_begin = int64_t(blockIdx.y) * a.rps;
    const int64_t r_end = min<int64_t>(a.nrows, r_begin + a.rps);
    const bool with_bias = tcx == 0;

    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;

    // 2 x RW_VC rows x 8 units of 16 bytes per chunk: 8 per thread (unit u: operand u >> 10,
    // row (u & 1023) >> 3, channels 8 (u & 7) .. + 7 of the tile)
    u32x4 r[8];
    auto load = [&](int64_t row0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = tid + 256 * k;
            const bool isg = u < 1024;
            const int row = (u & 1023) >> 3, c = 8 * (u & 7);
            const int64_t v = row0 + row;
            const int ch = (isg ? cg0 : cx0) + c;
            r[k] = u32x4{0u, 0u, 0u, 0u};
            if (v < r_end && ch < (isg ? a.cg : a.cx))
                r[k] = *reinterpret_cast<const u32x4 *>(isg ? g + v * a.ldg + ch : x + v * a.ldx + ch);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int u = tid + 256 * k;
            const int row = (u & 1023) >> 3, c = 8 * (u & 7);
            u32x2 *d2 = reinterpret_cast<u32x2 *>((u < 1024 ? gs : xs) + row * RW_P + c);
            d2[0] = u32x2{r[k][0], r[k][1]};
            d2[1] = u32x2{r[k][2], r[k][3]};
        }
    };
    if (r_begin < r_end) load(r_begin);
    for (int64_t row0 = r_begin; row0 < r_end; row0 += RW_VC) {
        __syncthreads();
        store();
        if (row0 + RW_VC < r_end) load(row0 + RW_VC);
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < RW_VC / 32; ++ks) {
            const int r0 = ks * 32 + 8 * grp + q;
            const h16_t *ga = gs + r0 * RW_P + 4 * p4;
            const h16_t *xa = xs + r0 * RW_P + 4 * p4;
            hx8 af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int mt = 2 * wm + i, t = 2 * wn + i;
                af[i] = tr8(ga + 16 * mt, ga + 16 * mt + 4 * RW_P);
                bf[i] = tr8(xa + 16 * t, xa + 16 * t + 4 * RW_P);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = VQ3D_MFMA_16X16X32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (with_bias) {  // column lane, rows 32 wave .. 32 wave + 31 of the chunk, in order
            float s = 0.f;
#pragma unroll 8
            for (int rr = 0; rr < 32; ++rr) s += ld(gs + (32 * wave + rr) * RW_P + lane);
            bsum += s;
        }
    }
    const int ne1 = a.cx + 1;
    float *dst = part + int64_t(blockIdx.y) * a.cg * ne1;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ci = cx0 + 16 * (2 * wn + j) + li;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int co = cg0 + 16 * (2 * wm + i) + 4 * grp + e;
                if (co < a.cg && ci < a.cx) dst[int64_t(co) * ne1 + ci] = acc[i][j][e];
            }
        }
    if (with_bias) {
        bred[wave][lane] = bsum;
        __syncthreads();
        if (wave == 0 && cg0 + lane < a.cg)
            dst[int64_t(cg0 + lane) * ne1 + a.cx] = (bred[0][lane] + bred[1][lane]) + (bred[2][lane] + bred[3][lane]);
    }
}

struct RwPlan {
    RwArgs a;
    int tiles, splits;
};

RwPlan rows_wgrad_plan(int64_t nrows, int cg, int cx) {
    RwPlan p{};
    p.a.nrows = nrows;
    p.a.cg = cg;
    p.a.cx = cx;
    p.a.tx = (cx + 63) / 64;
    p.tiles = p.a.tx * ((cg + 63) / 64);
    const int64_t nch = std::max<int64_t>(1, (nrows + RW_VC - 1) / RW_VC);
    // about 256 workgroups: a chunk or more each, the split count bounded by the partial traffic
    const int64_t want = std::max<int64_t>(1, 256 / p.tiles);
    p.splits = int(std::min<int64_t>({nch, want, 1024}));
    p.a.rps = (nch + p.splits - 1) / p.splits * RW_VC;
    p.splits = int((nrows + p.a.rps - 1) / p.a.rps);
    if (p.splits < 1) p.splits = 1;
    return p;
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

bool reg_path(const vq3d_conv_desc *d) {
    auto p2 = [](int c) { return c == 1 || c == 2 || c == 4 || c == 8; };
    return d->cin2 == 0 && p2(d->cin) && p2(d->cout) && d->cout * (d->cin + 1) <= 40;
}

PwwArgs plan(const vq3d_conv_desc *d, int &ytiles, int &nbx, size_t &lds) {
    PwwArgs a = {};
    a.nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    a.Ca = d->cin;
    a.Cb = d->cin2;
    a.N = d->cout;
    const int Ct = a.Ca + a.Cb;
    a.ones = Ct;
    a.ne = a.N * (Ct + 1);
    a.Xp = round_up(Ct + 1, TI);
    a.Gp = round_up(a.N, TO);
    a.nti = a.Xp / TI;
    const int ntiles = a.nti * (a.Gp / TO);
    a.tpb = std::min(ntiles, 64);
    a.S = 256 / a.tpb;
    ytiles = (ntiles + a.tpb - 1) / a.tpb;
    // segment: ~16 KB of fp32 slabs (several workgroups per CU hide the load latency)
    const int row_bytes = (a.Xp + a.Gp) * 4;
    a.seg = 1024;
    while (a.seg > 16 && size_t(a.seg) * row_bytes > 16 * 1024) a.seg /= 2;
    a.fa = FastDiv(uint32_t(std::max(1, a.Ca)));
    a.fb = FastDiv(uint32_t(std::max(1, a.Cb)));
    a.fn = FastDiv(uint32_t(a.N));
    lds = std::max(size_t(a.seg) * row_bytes, size_t(256) * TI * TO * 4);
    const int64_t nseg = (a.nvox + a.seg - 1) / a.seg;
    nbx = int(std::max<int64_t>(1, std::min<int64_t>(nseg, std::max(1, kMaxBlocks / ytiles))));
    // mid-size grids: few workgroups striding over the segments, so the partials go straight
    // into the gradients (direct mode) instead of through a second reduction launch
    if (reg_path(d)) {  // 4 x 256 voxels per workgroup-iteration (wide rows: ~4 voxels per thread)
        ytiles = 1;
        nbx = int(std::max<int64_t>(1, std::min<int64_t>((a.nvox + 1023) / 1024, kMaxBlocks)));
    }
    return a;
}

}  // namespace

size_t pw_wgrad_workspace(const vq3d_conv_desc *d) {
    int ytiles, nbx;
    size_t lds;
    const PwwArgs a = plan(d, ytiles, nbx, lds);
    size_t bytes = size_t(nbx) * a.ne * 4;
    WmArgs m;
    int mpw, ntt;
    if (d->dtype == VQ3D_HALF && plan_mma(d, nullptr, nullptr, nullptr, m, mpw, ntt, nbx, lds))
        bytes = std::max(bytes, size_t(nbx) * m.N * (m.Ct + 1) * 4);
    return bytes;
}

int launch_pw_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pro_a,
                    const float *pro_b, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                    float *dcbias, void *workspace, size_t ws_bytes, hipStream_t s) {
    int ytiles, nbx;
    size_t lds;
    PwwArgs a = plan(d, ytiles, nbx, lds);
    if (!workspace || ws_bytes < size_t(nbx) * a.ne * 4) return fail("conv3d_bwd_weight: workspace too small");
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    a.vec = al(x) && al(g) && (!x2 || al(x2));
    WgOut out{w, escale, dw, dscale, dbias, dcbias, GridSum{}};
    const dim3 grid{unsigned(nbx), unsigned(ytiles), 1u};
    WmArgs m;
    int mpw, ntt, mbx;
    size_t mlds;
    const bool mma = !(reg_path(d) && a.vec) && plan_mma(d, x, x2, g, m, mpw, ntt, mbx, mlds) &&
                     size_t(mbx) * m.N * (m.Ct + 1) * 4 <= ws_bytes;
    if (mma) {
        nbx = mbx;
        a.ne = m.N * (m.Ct + 1);
    }
    // few workgroups: each adds its partial straight into the gradients (no reduce launch; the
    // matrix-core kernel's partials are whole co x ci images, so only a single workgroup goes direct)
    // one workgroup column (nbx == 1) adds its entries straight into the gradients (each entry has
    // one adder, so the sums stay deterministic); the scalar sums over the column's y tiles go
    // through the fixed-order in-grid sum
    const bool direct = nbx == 1;
    float *part = direct ? nullptr : static_cast<float *>(workspace);
    if (direct && !mma && !(reg_path(d) && a.vec)) out.gsum = grid_sum_for(s, ytiles, dscale || dbias);
    if (mma) {
#define WM(M_, N_)                                                                                              \
    else if (mpw == M_ && ntt == N_) k_pw_wgrad_mma<M_, N_><<<nbx, 256, mlds, s>>>(                            \
        m, (const h16_t *)x, (const h16_t *)x2, (const h16_t *)g, d->pro_kind, pro_a, pro_b, part, out);
        if (false) {
        }
        WM(1, 1) WM(1, 2) WM(1, 4) WM(1, 8) WM(1, 16) WM(2, 1) WM(2, 2) WM(2, 4) WM(2, 8)
        else return fail("conv3d_bwd_weight: no matrix-core instance");
#undef WM
    } else if (reg_path(d) && a.vec) {
        const int key = d->cin * 16 + d->cout;
        const bool bf = d->dtype == VQ3D_HALF;
#define REG(CX, CG)                                                                                            \
    case CX * 16 + CG:                                                                                         \
        if (bf)                                                                                                \
            k_pw_wgrad_reg<h16_t, CX, CG><<<nbx, 256, 0, s>>>(a.nvox, (const h16_t *)x, (const h16_t *)g,  \
                                                               d->pro_kind, pro_a, pro_b, part, out);         \
        else                                                                                                   \
            k_pw_wgrad_reg<float, CX, CG><<<nbx, 256, 0, s>>>(a.nvox, (const float *)x, (const float *)g,     \
                                                              d->pro_kind, pro_a, pro_b, part, out);          \
        break;
        switch (key) {
            REG(1, 1) REG(1, 2) REG(1, 4) REG(1, 8) REG(2, 1) REG(2, 2) REG(2, 4) REG(2, 8)
            REG(4, 1) REG(4, 2) REG(4, 4) REG(4, 8) REG(8, 1) REG(8, 2) REG(8, 4)
        default: return fail("conv3d_bwd_weight: no register-path kernel");
        }
#undef REG
    } else if (d->dtype == VQ3D_HALF)
        k_pw_wgrad<h16_t><<<grid, 256, lds, s>>>(a, (const h16_t *)x, (const h16_t *)x2, (const h16_t *)g,
                                                   d->pro_kind, pro_a, pro_b, part, out);
    else
        k_pw_wgrad<float><<<grid, 256, lds, s>>>(a, (const float *)x, (const float *)x2, (const float *)g,
                                                  d->pro_kind, pro_a, pro_b, part, out);
    if (direct) return check_launch("conv3d_bwd_weight(pointwise)");
    const int Ct = a.Ca + a.Cb;
    if (mma && m.tr) {
        const unsigned nr = unsigned((a.ne + 63) / 64);
        k_pw_wgrad_reduce_t<<<nr, 256, 0, s>>>(part, nbx, a.ne, Ct, w, escale, dw, dscale, dbias, dcbias,
                                               grid_sum_for(s, nr, dscale || dbias));
        return check_launch("conv3d_bwd_weight(pointwise)");
    }
    int lanes = 1;
    while (lanes < 64 && lanes * 8 < nbx) lanes *= 2;
    if (lanes == 64 && nbx > 512) lanes = 256;  // a workgroup per entry: one round of loads per thread
#define RED(L)                                                                                                 \
    k_pw_wgrad_reduce<L><<<(a.ne + 256 / L - 1) / (256 / L), 256, 0, s>>>(                                       \
        part, nbx, a.ne, Ct, w, escale, dw, dscale, dbias, dcbias,                                               \
        grid_sum_for(s, (a.ne + 256 / L - 1) / (256 / L), dscale || dbias))
    switch (lanes) {
    case 1: RED(1); break;
    case 2: RED(2); break;
    case 4: RED(4); break;
    case 8: RED(8); break;
    case 16: RED(16); break;
    case 32: RED(32); break;
    case 64: RED(64); break;
    default: RED(256); break;
    }
#undef RED
    return check_launch("conv3d_bwd_weight(pointwise)");
}

size_t rows_wgrad_workspace(int64_t nrows, int cg, int cx) {
    if (nrows <= 0 || cg <= 0 || cx <= 0) return 0;
    const RwPlan p = rows_wgrad_plan(nrows, cg, cx);
    return size_t(p.splits) * cg * (cx + 1) * sizeof(float);
}

int launch_rows_wgrad(int64_t nrows, int cg, int cx, const void *g, int64_t ldg, const void *x, int64_t ldx, float *dw,
                      float *db, void *workspace, size_t ws_bytes, hipStream_t s) {
    if (nrows <= 0) return 0;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (cg <= 0 || cx <= 0 || cg % 8 || cx % 8 || ldg % 8 || ldx % 8 || ldg < cg || ldx < cx)
        return fail("rows_wgrad: channel counts and row strides must be multiples of 8");
    if (!g || !x || !dw || !al(g) || !al(x)) return fail("rows_wgrad: g / x must be 16-byte aligned");
    RwPlan p = rows_wgrad_plan(nrows, cg, cx);
    p.a.ldg = int(ldg);
    p.a.ldx = int(ldx);
    const size_t need = size_t(p.splits) * cg * (cx + 1) * sizeof(float);
    if (!workspace || ws_bytes < need) return fail("rows_wgrad: workspace too small");
    float *part = static_cast<float *>(workspace);
    k_rows_wgrad<<<dim3(unsigned(p.tiles), unsigned(p.splits), 1u), 256, 0, s>>>(p.a, (const h16_t *)g,
                                                                               (const h16_t *)x, part);
    const int ne = cg * (cx + 1);
    const unsigned nr = unsigned((ne + 63) / 64);
    k_pw_wgrad_reduce_t<<<nr, 256, 0, s>>>(part, p.splits, ne, cx, nullptr, nullptr, dw, nullptr, nullptr, db,
                                           GridSum{});
    return check_launch("rows_wgrad");
}

}  // namespace vq3d
