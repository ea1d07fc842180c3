// Dense causal attention of the PixelSNAIL prior (pixel_model/layers.py:613-647,
// pixel_model/pixelsnail.py:295-298): for every (problem = stack x batch, head)
//
//   out[i] = sum_{j <= i} softmax_j(scale * q_i . k_j) v_j        (i, j over the n code positions)
//
// without ever forming the n x n logits (the reference materialises them, with the tril mask,
// per block: 3 x 8 x 8192^2 fp32 at the published mid level).  Head dims are tiny (model-dim
// 256 / bottleneck 4 / 8 heads = 8), so the contraction is per-thread VALU work: a thread owns
// one query row (fwd, dQ) or one key row (dK / dV) with its q / k / v / dO rows in registers;
// the opposite side streams through LDS in 64-row tiles that every lane reads as broadcasts.
// Causality bounds the tile loops (query tile t meets key tiles 0 .. t), the diagonal tile masks
// per lane.  The online softmax runs in base 2 on chunks of 8 scores (one rescale per chunk);
// the forward saves the per-row log-sum-exp (base 2) for the backward, which recomputes the
// probabilities (flash-attention style, fp32 arithmetic throughout, bf16 or fp32 storage).
// A workgroup owns 64 rows; its 4 waves split every staged 64-row tile of the other side four
// ways (4 waves per SIMD at the mid level's 8,192 positions x 8 heads) and merge at the end.
//
// Layout: q, k [P][n][nh * dk], v, out [P][n][nh * dv] -- channels-last rows with head-major
// channels (head h owns channels h * d .. h * d + d - 1, the reference's reshape(..., nh, d, n)).
#include "engines.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

namespace vq3d {

namespace {

constexpr int QR = 64;          // rows (queries, or keys in the dK / dV kernel) per workgroup
constexpr int NW = 4;           // waves per workgroup: each takes a quarter of every staged tile
constexpr int NT = QR * NW;     // 256 threads
constexpr int SUB = QR / NW;    // 16 staged rows per wave
constexpr int CH = 8;           // scores per online-softmax chunk
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
    int P, n, nh, dk, dv;
    float c2;  // scale * log2(e)
    // training-mode logit transform of the reference (layers.py:633-637): dropout(logits) -- kept
    // logits scaled by 1 / (1 - p), dropped ones 0 -- then logits == 0 -> -1e3.  train = 0: none.
    int train;
    uint32_t drop_below;      // a (problem, head, i, j) hash below this drops the logit (p * 2^32)
    float keep_scale;         // 1 / (1 - p)
    const uint64_t *seed;     // device seed of this forward (the backward reads the same value)
};

constexpr float ZERO_LOGIT2 = -1000.f * LOG2E;  // the reference's -1e3 logit, in log2 units

// counter-based hash of one logit's coordinates (lowbias32 mixing of a 64-bit seed, the
// problem / head and the two positions): the same value in the forward and both backward kernels
__device__ __forceinline__ uint32_t logit_hash(uint64_t seed, int ph, int i, int j) {
    uint32_t x = uint32_t(seed) ^ (uint32_t(seed >> 32) * 0x9E3779B1u) ^ (uint32_t(ph) * 0xC2B2AE3Du) ^
                 (uint32_t(i) * 0x85EBCA77u) ^ (uint32_t(j) * 0x27D4EB2Fu);
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// the training-mode transform of a raw (scaled, log2-unit) score s of logit (i, j); live = the
// logit keeps its gradient (kept by dropout and not replaced), with factor keep_scale
__device__ __forceinline__ float train_logit(const AttnArgs &a, uint64_t seed, int ph, int i, int j, float s,
                                             bool &live) {
    if (a.drop_below && logit_hash(seed, ph, i, j) < a.drop_below) {
        live = false;
        return ZERO_LOGIT2;
    }
    s *= a.keep_scale;
    live = s != 0.f;
    return live ? s : ZERO_LOGIT2;
}

template <typename T, int DM>
__device__ __forceinline__ void load_row(const T *__restrict__ src, int64_t base, int d, bool ok, float (&r)[DM]) {
#pragma unroll
    for (int c = 0; c < DM; ++c) r[c] = (ok && c < d) ? ld(src + base + c) : 0.f;
}

template <typename T, int DM>
__device__ __forceinline__ void store_row(T *__restrict__ dst, int64_t base, int d, const float (&r)[DM]) {
#pragma unroll
    for (int c = 0; c < DM; ++c)
        if (c < d) st(dst + base + c, r[c]);
}

// rows [r0, r0 + QR) of a [P][n][nh * d] tensor's head h into LDS [QR][DM] fp32 (zero past n / d),
// by the QR threads [t0, t0 + QR)
template <typename T, int DM>
__device__ __forceinline__ void stage(float *dst, const T *__restrict__ src, const AttnArgs &a, int p, int h, int d,
                                      int r0, int t0) {
    const int t = int(threadIdx.x) - t0;
    if (t < 0 || t >= QR) return;
    const int r = r0 + t;
    float v[DM];
    load_row<T, DM>(src, (int64_t(p) * a.n + min(r, a.n - 1)) * (a.nh * d) + h * d, d, r < a.n, v);
#pragma unroll
    for (int c = 0; c < DM; c += 4)
        *reinterpret_cast<float4 *>(dst + t * DM + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
}

template <int DM>
__device__ __forceinline__ float dot(const float (&a)[DM], const float *b) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < DM; c += 4) {
        const float4 q = *reinterpret_cast<const float4 *>(b + c);
        s = fmaf(a[c], q.x, s);
        s = fmaf(a[c + 1], q.y, s);
        s = fmaf(a[c + 2], q.z, s);
        s = fmaf(a[c + 3], q.w, s);
    }
    return s;
}

template <int DM>
__device__ __forceinline__ void axpy(float (&y)[DM], float a, const float *x) {
#pragma unroll
    for (int c = 0; c < DM; c += 4) {
        const float4 q = *reinterpret_cast<const float4 *>(x + c);
        y[c] = fmaf(a, q.x, y[c]);
        y[c + 1] = fmaf(a, q.y, y[c + 1]);
        y[c + 2] = fmaf(a, q.z, y[c + 2]);
        y[c + 3] = fmaf(a, q.w, y[c + 3]);
    }
}

// Forward.  Workgroup = QR query rows of one (problem, head); lane r of every wave owns query row
// r, wave w the keys w * SUB .. w * SUB + SUB - 1 of each staged QR-key tile (online softmax per
// wave), the 4 partial (m, l, o) merged at the end.  grid (query tiles, P * nh), heaviest first.
template <typename T, int DM>
__global__ __launch_bounds__(NT) void k_attn_fwd(AttnArgs a, const T *__restrict__ q, const T *__restrict__ k,
                                                 const T *__restrict__ v, T *__restrict__ out,
                                                 float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) float ks[QR * DM], vs[QR * DM];
    __shared__ __attribute__((aligned(16))) float pm[NW][QR], pl[NW][QR], po[NW][QR][DM];
    const int nqt = (a.n + QR - 1) / QR, qt = nqt - 1 - int(blockIdx.x);
    const int p = int(blockIdx.y) / a.nh, h = int(blockIdx.y) - p * a.nh;
    const int r = int(threadIdx.x) & (QR - 1), w = int(threadIdx.x) / QR;
    const int i = qt * QR + r;
    float qr[DM], o[DM];
    load_row<T, DM>(q, (int64_t(p) * a.n + min(i, a.n - 1)) * (a.nh * a.dk) + h * a.dk, a.dk, i < a.n, qr);
#pragma unroll
    for (int c = 0; c < DM; ++c) {
        qr[c] *= a.c2;
        o[c] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    const uint64_t seed = a.drop_below ? *a.seed : 0;
    // one staged key tile; FULL: every key of it precedes the wave's queries (no per-key masks --
    // all tiles but the diagonal one)
    auto tile = [&](auto fullc, int kt) {
        constexpr bool FULL = decltype(fullc)::value;
        const int jlim = FULL ? QR : r + 1;  // local keys j <= i
#pragma unroll
        for (int c0 = 0; c0 < SUB; c0 += CH) {
            const int j0 = w * SUB + c0;
            if (!FULL && j0 >= jlim) break;
            float s[CH], cm = m;
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const bool in = FULL || j0 + u < jlim;
                s[u] = in ? dot<DM>(qr, ks + (j0 + u) * DM) : -INFINITY;
                if (a.train && in) {
                    bool live;
                    s[u] = train_logit(a, seed, int(blockIdx.y), i, kt * QR + j0 + u, s[u], live);
                }
                cm = fmaxf(cm, s[u]);
            }
            const float alpha = exp2f(m - cm);  // m = -inf before the wave's first key: 0
            l *= alpha;
#pragma unroll
            for (int c = 0; c < DM; ++c) o[c] *= alpha;
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const float pr = exp2f(s[u] - cm);
                l += pr;
                axpy<DM>(o, pr, vs + (j0 + u) * DM);
            }
            m = cm;
        }
    };
    for (int kt = 0; kt <= qt; ++kt) {
        __syncthreads();
        stage<T, DM>(ks, k, a, p, h, a.dk, kt * QR, 0);
        stage<T, DM>(vs, v, a, p, h, a.dv, kt * QR, QR);
        __syncthreads();
        if (kt < qt) tile(std::true_type{}, kt);
        else tile(std::false_type{}, kt);
    }
    // merge the 4 waves' partial softmaxes (a wave that met no key has m = -inf, l = 0)
    pm[w][r] = m;
    pl[w][r] = l;
#pragma unroll
    for (int c = 0; c < DM; ++c) po[w][r][c] = o[c];
    __syncthreads();
    if (w == 0 && i < a.n) {
        float M = pm[0][r];
#pragma unroll
        for (int x = 1; x < NW; ++x) M = fmaxf(M, pm[x][r]);
        float Lt = 0.f, O[DM];
#pragma unroll
        for (int c = 0; c < DM; ++c) O[c] = 0.f;
#pragma unroll
        for (int x = 0; x < NW; ++x) {
            const float f = pm[x][r] == -INFINITY ? 0.f : exp2f(pm[x][r] - M);
            Lt = fmaf(pl[x][r], f, Lt);
#pragma unroll
            for (int c = 0; c < DM; ++c) O[c] = fmaf(po[x][r][c], f, O[c]);
        }
        const float inv = 1.f / Lt;
#pragma unroll
        for (int c = 0; c < DM; ++c) O[c] *= inv;
        store_row<T, DM>(out, (int64_t(p) * a.n + i) * (a.nh * a.dv) + h * a.dv, a.dv, O);
        lse[(int64_t(p) * a.nh + h) * a.n + i] = M + log2f(Lt);
    }
}

// backward, query side: delta_i = dO_i . O_i (to the workspace) and dQ_i = scale sum_j ds_ij k_j,
// ds_ij = p_ij (dO_i . v_j - delta_i); the waves split the keys as in the forward, the partial dQ
// summed at the end in wave order
template <typename T, int DM>
__global__ __launch_bounds__(NT) void k_attn_bwd_q(AttnArgs a, float scale, const T *__restrict__ q,
                                                   const T *__restrict__ k, const T *__restrict__ v,
                                                   const T *__restrict__ out, const T *__restrict__ gout,
                                                   const float *__restrict__ lse, float *__restrict__ delta,
                                                   T *__restrict__ gq) {
    __shared__ __attribute__((aligned(16))) float ks[QR * DM], vs[QR * DM];
    __shared__ __attribute__((aligned(16))) float pq[NW][QR][DM];
    const int nqt = (a.n + QR - 1) / QR, qt = nqt - 1 - int(blockIdx.x);
    const int p = int(blockIdx.y) / a.nh, h = int(blockIdx.y) - p * a.nh;
    const int r = int(threadIdx.x) & (QR - 1), w = int(threadIdx.x) / QR;
    const int i = qt * QR + r;
    const bool ok = i < a.n;
    const int ic = min(i, a.n - 1);
    float qr[DM], go[DM], orow[DM], dq[DM];
    load_row<T, DM>(q, (int64_t(p) * a.n + ic) * (a.nh * a.dk) + h * a.dk, a.dk, ok, qr);
    load_row<T, DM>(gout, (int64_t(p) * a.n + ic) * (a.nh * a.dv) + h * a.dv, a.dv, ok, go);
    load_row<T, DM>(out, (int64_t(p) * a.n + ic) * (a.nh * a.dv) + h * a.dv, a.dv, ok, orow);
    float dl = 0.f;
#pragma unroll
    for (int c = 0; c < DM; ++c) {
        dl = fmaf(go[c], orow[c], dl);
        qr[c] *= a.c2;
        dq[c] = 0.f;
    }
    const int64_t row = (int64_t(p) * a.nh + h) * a.n + ic;
    const float lz = ok ? lse[row] : 0.f;
    if (ok && w == 0) delta[row] = dl;
    const uint64_t seed = a.drop_below ? *a.seed : 0;
    for (int kt = 0; kt <= qt; ++kt) {
        __syncthreads();
        stage<T, DM>(ks, k, a, p, h, a.dk, kt * QR, 0);
        stage<T, DM>(vs, v, a, p, h, a.dv, kt * QR, QR);
        __syncthreads();
        auto tile = [&](auto fullc) {  // FULL: no per-key causal mask (every tile but the diagonal)
            constexpr bool FULL = decltype(fullc)::value;
            const int jlim = FULL ? QR : r + 1;
#pragma unroll 4
            for (int u = 0; u < SUB; ++u) {
                const int j = w * SUB + u;
                if (FULL || j < jlim) {
                    float sc = dot<DM>(qr, ks + j * DM), gf = 1.f;
                    if (a.train) {
                        bool live;
                        sc = train_logit(a, seed, int(blockIdx.y), i, kt * QR + j, sc, live);
                        gf = live ? a.keep_scale : 0.f;
                    }
                    const float pr = exp2f(sc - lz);
                    const float ds = gf * pr * (dot<DM>(go, vs + j * DM) - dl);
                    axpy<DM>(dq, ds, ks + j * DM);
                }
            }
        };
        if (kt < qt) tile(std::true_type{});
        else tile(std::false_type{});
    }
#pragma unroll
    for (int c = 0; c < DM; ++c) pq[w][r][c] = dq[c];
    __syncthreads();
    if (w == 0 && ok) {
#pragma unroll
        for (int c = 0; c < DM; ++c) dq[c] = scale * (((pq[0][r][c] + pq[1][r][c]) + pq[2][r][c]) + pq[3][r][c]);
        store_row<T, DM>(gq, (int64_t(p) * a.n + i) * (a.nh * a.dk) + h * a.dk, a.dk, dq);
    }
}

// backward, key side: dV_j = sum_{i >= j} p_ij dO_i, dK_j = scale sum_{i >= j} ds_ij q_i.
// Workgroup = QR key rows; wave w takes the queries w * SUB .. of each staged query tile.
template <typename T, int DM>
__global__ __launch_bounds__(NT) void k_attn_bwd_kv(AttnArgs a, float scale, const T *__restrict__ q,
                                                    const T *__restrict__ k, const T *__restrict__ v,
                                                    const T *__restrict__ gout, const float *__restrict__ lse,
                                                    const float *__restrict__ delta, T *__restrict__ gk,
                                                    T *__restrict__ gv) {
    __shared__ __attribute__((aligned(16))) float qs[QR * DM], gs[QR * DM];
    __shared__ float ls[QR], dls[QR];
    __shared__ __attribute__((aligned(16))) float pk[NW][QR][DM], pv[NW][QR][DM];
    [[maybe_unused]] const int nt = (a.n + QR - 1) / QR, kt = int(blockIdx.x);  // key tile 0 meets every query tile: first
    const int p = int(blockIdx.y) / a.nh, h = int(blockIdx.y) - p * a.nh;
    const int r = int(threadIdx.x) & (QR - 1), w = int(threadIdx.x) / QR;
    const int j = kt * QR + r;
    const bool ok = j < a.n;
    const int jc = min(j, a.n - 1);
    float kr[DM], vr[DM], dk[DM], dv[DM];
    load_row<T, DM>(k, (int64_t(p) * a.n + jc) * (a.nh * a.dk) + h * a.dk, a.dk, ok, kr);
    load_row<T, DM>(v, (int64_t(p) * a.n + jc) * (a.nh * a.dv) + h * a.dv, a.dv, ok, vr);
#pragma unroll
    for (int c = 0; c < DM; ++c) {
        kr[c] *= a.c2;
        dk[c] = dv[c] = 0.f;
    }
    const int64_t rb = (int64_t(p) * a.nh + h) * a.n;
    const uint64_t seed = a.drop_below ? *a.seed : 0;
    for (int qt = kt; qt < nt; ++qt) {
        __syncthreads();
        stage<T, DM>(qs, q, a, p, h, a.dk, qt * QR, 0);
        stage<T, DM>(gs, gout, a, p, h, a.dv, qt * QR, QR);
        if (threadIdx.x >= 2 * QR && threadIdx.x < 3 * QR) {
            const int t = int(threadIdx.x) - 2 * QR, rr = qt * QR + t;
            ls[t] = rr < a.n ? lse[rb + rr] : 0.f;
            dls[t] = rr < a.n ? delta[rb + rr] : 0.f;
        }
        __syncthreads();
        const int i0 = qt > kt ? 0 : r;  // local queries i >= j
        const int iend = min(QR, a.n - qt * QR);
        auto tile = [&](auto fullc) {  // FULL: every query of the tile follows every key (no masks)
            constexpr bool FULL = decltype(fullc)::value;
#pragma unroll 4
            for (int u = 0; u < SUB; ++u) {
                const int ii = w * SUB + u;
                if (FULL || (ii >= i0 && ii < iend)) {
                    float sc = dot<DM>(kr, qs + ii * DM), gf = 1.f;
                    if (a.train) {
                        bool live;
                        sc = train_logit(a, seed, int(blockIdx.y), qt * QR + ii, j, sc, live);
                        gf = live ? a.keep_scale : 0.f;
                    }
                    const float pr = exp2f(sc - ls[ii]);
                    axpy<DM>(dv, pr, gs + ii * DM);
                    const float ds = gf * pr * (dot<DM>(vr, gs + ii * DM) - dls[ii]);
                    axpy<DM>(dk, ds, qs + ii * DM);
                }
            }
        };
        if (qt > kt && iend == QR) tile(std::true_type{});
        else tile(std::false_type{});
    }
#pragma unroll
    for (int c = 0; c < DM; ++c) {
        pk[w][r][c] = dk[c];
        pv[w][r][c] = dv[c];
    }
    __syncthreads();
    if (w == 0 && ok) {
#pragma unroll
        for (int c = 0; c < DM; ++c) {
            dk[c] = scale * (((pk[0][r][c] + pk[1][r][c]) + pk[2][r][c]) + pk[3][r][c]);
            dv[c] = ((pv[0][r][c] + pv[1][r][c]) + pv[2][r][c]) + pv[3][r][c];
        }
        store_row<T, DM>(gk, (int64_t(p) * a.n + j) * (a.nh * a.dk) + h * a.dk, a.dk, dk);
        store_row<T, DM>(gv, (int64_t(p) * a.n + j) * (a.nh * a.dv) + h * a.dv, a.dv, dv);
    }
}

// ---------------------------------------------------------------------------- matrix-core forward
// 16-bit builds, head dims dk = dv = 8 (the published prior: model-dim 256 / bottleneck 4 / 8 heads).
// Workgroup = 128 queries of one (problem, head), a wave owns 32 of them; keys stream through LDS in
// 128-key tiles.  Per 32-key block a wave forms S^T = K Q^T on the matrix cores
// (v_mfma_f32_32x32x8, K = the 8 head dims): lane (column n = query, half h) holds the 16 keys
// (r & 3) + 8 (r >> 2) + 4 h of its query's column in accumulator r, so the online softmax's max is
// the lane's 16 values and its partner half's (one cross-half shuffle), and the probabilities are,
// unmoved, the B operand of O^T += V^T P^T (v_mfma_f32_32x32x16_f16, K = 16 keys: element j of lane
// half h <-> key (j & 3) + 8 (j >> 2) + 4 h; V^T is read in that key order).  O^T's rows are the 8
// value dims (rows 8 .. 31 of the A operand are zero): lane (n, h) ends with dims 4h .. 4h + 3 of
// query n.  Arithmetic: q . k products of the stored 16-bit values accumulated in fp32 and scaled in
// fp32 (the VALU kernel scales q first), P and V in the build's 16-bit format in the P V product
// with fp32 accumulation, l summed in fp32.
#ifndef ATTN_MQ
#define ATTN_MQ 128
#endif
constexpr int MQ = ATTN_MQ, MK = 128, VTP = MK + 8, MNT = 2 * MQ;  // MNT: threads (a wave per 32 queries)
typedef float f32x16 __attribute__((ext_vector_type(16)));
// the second products' operand format (P, V^T, dO^T, dS, K^T, Q^T): the build's own 16-bit format.
// bf16 builds run them on v_mfma_f32_32x32x16_bf16: bf16 keeps fp32's exponent range, so the small
// dO / dS of an unscaled bf16 loss (1e-5 .. 1e-8 per element) and large V rows stay representable
// (fp16 operands would flush them below 6.1e-5 / overflow above 65504).
typedef half_t f16x8v __attribute__((ext_vector_type(8)));
#ifdef VQ3D_FP16
#define ATT_MFMA_32X32X16 __builtin_amdgcn_mfma_f32_32x32x16_f16
#else
#define ATT_MFMA_32X32X16 __builtin_amdgcn_mfma_f32_32x32x16_bf16
#endif

// 2^x as the bare v_exp_f32 (results below 2^-126 flush to zero: probabilities below 2^-126 of the
// row's largest, which the fp16 build's P / dS operands flush anyway; -inf -> 0): the matrix-core
// kernels' per-score exps
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x16 mma_qk(u32x2 kf, u32x2 qf, f32x16 acc) {
#ifdef VQ3D_FP16
    typedef _Float16 f16x4v __attribute__((ext_vector_type(4)));
    return __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_bit_cast(f16x4v, kf), __builtin_bit_cast(f16x4v, qf), acc,
                                                0, 0, 0);
#else
    typedef short s16x4v __attribute__((ext_vector_type(4)));
    return __builtin_amdgcn_mfma_f32_32x32x8bf16_1k(__builtin_bit_cast(s16x4v, kf), __builtin_bit_cast(s16x4v, qf),
                                                    acc, 0, 0, 0);
#endif
}

__global__ __launch_bounds__(MNT) void k_attn_fwd_mma(AttnArgs a, const h16_t *__restrict__ q,
                                                      const h16_t *__restrict__ k, const h16_t *__restrict__ v,
                                                      h16_t *__restrict__ out, float *__restrict__ lse) {
    __shared__ __attribute__((aligned(16))) h16_t ks[MK * 8];    // [key][dim], the stored format
    __shared__ __attribute__((aligned(16))) half_t vt[8 * VTP];  // [dim][key], the 16-bit format
    const int nqt = (a.n + MQ - 1) / MQ, qt = nqt - 1 - int(blockIdx.x);
    const int p = int(blockIdx.y) / a.nh, hd = int(blockIdx.y) - p * a.nh;
    const int tid = int(threadIdx.x), lane = tid & 63, w = tid >> 6, col = lane & 31, hh = lane >> 5;
    const int qb = qt * (MQ / 32) + w;  // the wave's 32-query block
    const int i = qb * 32 + col;        // the lane's query
    const int rs = a.nh * 8;
    const u32x2 qf = *reinterpret_cast<const u32x2 *>(q + (int64_t(p) * a.n + min(i, a.n - 1)) * rs + hd * 8 + 4 * hh);
    f32x16 o = {};
    float m = -INFINITY, l = 0.f;
    const uint64_t seed = a.drop_below ? *a.seed : 0;
    const float c2k = a.train ? a.c2 * a.keep_scale : a.c2;  // train_logit's two factors in one
    const bool zrep = a.train != 0, drop = a.drop_below != 0;
    const int nkt = (qt * MQ + MQ + MK - 1) / MK;  // key tiles up to the workgroup's last query
    for (int kt = 0; kt < nkt; ++kt) {
        __syncthreads();
        for (int e = tid; e < 2 * MK; e += MNT) {  // K rows, then V rows (transposed V^T)
            const int t = e & (MK - 1), kc = min(kt * MK + t, a.n - 1);
            const u32x4 row = *reinterpret_cast<const u32x4 *>((e < MK ? k : v) + (int64_t(p) * a.n + kc) * rs + hd * 8);
            if (e < MK) {
                *reinterpret_cast<u32x4 *>(ks + t * 8) = row;
            } else {
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    vt[(2 * c) * VTP + t] = half_t(h2f_lo(row[c]));
                    vt[(2 * c + 1) * VTP + t] = half_t(h2f_hi(row[c]));
                }
            }
        }
        __syncthreads();
        const int b0 = kt * (MK / 32), nb = min(MK / 32, qb - b0 + 1);
        // one 32-key block; DIAG: the wave's own block (keys after the query masked).  The logit
        // transform of the VALU kernel, branch-free: t = c2 * ks * s, a zero t -> the -1e3 logit
        // (train mode), a dropped logit (hash below drop_below) -> the -1e3 logit
        auto block = [&](auto diagc, int bb) {
            constexpr bool DIAG = decltype(diagc)::value;
            const int kb = b0 + bb;
            f32x16 st = mma_qk(*reinterpret_cast<const u32x2 *>(ks + (bb * 32 + col) * 8 + 4 * hh), qf, f32x16{});
            float bm = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;  // key within the block
                float t = st[r] * c2k;
                if (zrep) t = t != 0.f ? t : ZERO_LOGIT2;
                if (drop && logit_hash(seed, int(blockIdx.y), i, kb * 32 + row) < a.drop_below) t = ZERO_LOGIT2;
                if (DIAG) t = row > col ? -INFINITY : t;
                st[r] = t;
                bm = fmaxf(bm, t);
            }
            bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
            const float mn = fmaxf(m, bm);  // finite: key 0 of the block precedes every query of it
            const float alpha = fexp2(m - mn);
            m = mn;
            l *= alpha;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] *= alpha;  // rows 8 .. 31 of O^T stay zero
            f16x8v pb0, pb1;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pr = fexp2(st[r] - mn);
                l += pr;
                if (r < 8) pb0[r] = half_t(pr);
                else pb1[r - 8] = half_t(pr);
            }
            u32x4 a0 = {0u, 0u, 0u, 0u}, a1 = {0u, 0u, 0u, 0u};  // V^T rows 8 .. 31: zero
            if (col < 8) {
                const half_t *vr = vt + col * VTP + bb * 32 + 4 * hh;  // 4 keys = one 8-byte read
                const u32x2 r0 = *reinterpret_cast<const u32x2 *>(vr), r1 = *reinterpret_cast<const u32x2 *>(vr + 8);
                const u32x2 r2 = *reinterpret_cast<const u32x2 *>(vr + 16), r3 = *reinterpret_cast<const u32x2 *>(vr + 24);
                a0 = u32x4{r0[0], r0[1], r1[0], r1[1]};
                a1 = u32x4{r2[0], r2[1], r3[0], r3[1]};
            }
            o = ATT_MFMA_32X32X16(__builtin_bit_cast(f16x8v, a0), pb0, o, 0, 0, 0);
            o = ATT_MFMA_32X32X16(__builtin_bit_cast(f16x8v, a1), pb1, o, 0, 0, 0);
        };
        for (int bb = 0; bb < nb; ++bb) {
            if (b0 + bb < qb) block(std::false_type{}, bb);
            else block(std::true_type{}, bb);
        }
    }
    l += __shfl_xor(l, 32, 64);
    if (i < a.n) {
        const float inv = 1.f / l;
        float ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = o[r] * inv;
        stvec<h16_t, 4>(out + (int64_t(p) * a.n + i) * rs + hd * 8 + 4 * hh, ov);
        if (hh == 0) lse[(int64_t(p) * a.nh + hd) * a.n + i] = m + log2f(l);
    }
}

// ---------------------------------------------------------------------------- matrix-core backward
// The same tiling as k_attn_fwd_mma (32 rows per wave, 128-row tiles of the other side through LDS,
// 16-bit builds, head dims 8).  Query side (dQ, and delta = dO . O to the workspace): lane (query n,
// half h) holds the 16 keys (r & 3) + 8 (r >> 2) + 4 h of S^T = K Q^T and of dP^T = V dO^T (both
// 32x32x8, the query's q / dO as the register-resident B operand), so lse_n and delta_n are the
// lane's own; dS^T feeds dQ^T += K^T dS^T (32x32x16 f16, K^T read in the accumulator's key order).
// Key side (dK, dV): lane (key n, half h) holds the 16 queries of S = Q K^T and dP = dO V^T, with
// lse / delta of those queries from LDS (four 16-byte reads each); dV^T += dO^T P and dK^T += Q^T dS
// (32x32x16).  P and dS are rounded to the 16-bit format for the products, accumulation fp32; the logit
// transform (dropout, zero -> -1e3, its gradient factor) is the VALU kernels'.
__device__ __forceinline__ f16x8v vt_frag(const half_t *base) {  // 4 + 4 keys in the accumulator's order
    const u32x2 r0 = *reinterpret_cast<const u32x2 *>(base), r1 = *reinterpret_cast<const u32x2 *>(base + 8);
    return __builtin_bit_cast(f16x8v, u32x4{r0[0], r0[1], r1[0], r1[1]});
}

// stage 128 rows of a [P][n][nh * 8] 16-bit tensor's head hd: native rows [row][8] (nat, may be
// null) and / or transposed [dim][row] (tr, may be null)
__device__ __forceinline__ void stage_rows(const h16_t *__restrict__ src, const AttnArgs &a, int p, int hd, int r0,
                                           int t, h16_t *nat, half_t *tr) {
    const int rc = min(r0 + t, a.n - 1);
    const u32x4 row = *reinterpret_cast<const u32x4 *>(src + (int64_t(p) * a.n + rc) * (a.nh * 8) + hd * 8);
    if (nat) *reinterpret_cast<u32x4 *>(nat + t * 8) = row;
    if (tr) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            tr[(2 * c) * VTP + t] = half_t(h2f_lo(row[c]));
            tr[(2 * c + 1) * VTP + t] = half_t(h2f_hi(row[c]));
        }
    }
}

// the logit transform + gradient factor of one score (raw q . k), as the VALU kernels apply it
__device__ __forceinline__ float tlogit(const AttnArgs &a, float c2k, bool zrep, bool drop, uint64_t seed, int ph,
                                        int i, int j, float raw, float &gf) {
    float t = raw * c2k;
    bool live = true;
    if (zrep) live = t != 0.f;
    if (drop && logit_hash(seed, ph, i, j) < a.drop_below) live = false;
    gf = zrep ? (live ? a.keep_scale : 0.f) : 1.f;
    return (zrep && !live) ? ZERO_LOGIT2 : t;
}

__global__ __launch_bounds__(MNT) void k_attn_bwd_q_mma(AttnArgs a, float scale, const h16_t *__restrict__ q,
                                                        const h16_t *__restrict__ k, const h16_t *__restrict__ v,
                                                        const h16_t *__restrict__ out, const h16_t *__restrict__ gout,
                                                        const float *__restrict__ lse, float *__restrict__ delta,
                                                        h16_t *__restrict__ gq) {
    __shared__ __attribute__((aligned(16))) h16_t ks[MK * 8], vs[MK * 8];
    __shared__ __attribute__((aligned(16))) half_t kt_[8 * VTP];
    const int nqt = (a.n + MQ - 1) / MQ, qt = nqt - 1 - int(blockIdx.x);
    const int p = int(blockIdx.y) / a.nh, hd = int(blockIdx.y) - p * a.nh;
    const int tid = int(threadIdx.x), lane = tid & 63, w = tid >> 6, col = lane & 31, hh = lane >> 5;
    const int qb = qt * (MQ / 32) + w, i = qb * 32 + col, ic = min(i, a.n - 1);
    const int rs = a.nh * 8;
    const int64_t rowo = (int64_t(p) * a.n + ic) * rs + hd * 8 + 4 * hh;
    const u32x2 qf = *reinterpret_cast<const u32x2 *>(q + rowo);
    const u32x2 gf2 = *reinterpret_cast<const u32x2 *>(gout + rowo);
    // delta_i = dO_i . O_i: the lane's 4 dims and its partner half's
    float dl;
    {
        const u32x2 of = *reinterpret_cast<const u32x2 *>(out + rowo);
        dl = h2f_lo(gf2[0]) * h2f_lo(of[0]);
        dl = fmaf(h2f_hi(gf2[0]), h2f_hi(of[0]), dl);
        dl = fmaf(h2f_lo(gf2[1]), h2f_lo(of[1]), dl);
        dl = fmaf(h2f_hi(gf2[1]), h2f_hi(of[1]), dl);
        dl += __shfl_xor(dl, 32, 64);
    }
    const int64_t lrow = (int64_t(p) * a.nh + hd) * a.n + ic;
    const float lz = lse[lrow];
    if (i < a.n && hh == 0) delta[lrow] = dl;
    const uint64_t seed = a.drop_below ? *a.seed : 0;
    const float c2k = a.train ? a.c2 * a.keep_scale : a.c2;
    const bool zrep = a.train != 0, drop = a.drop_below != 0;
    f32x16 dq = {};
    const int nkt = (qt * MQ + MQ + MK - 1) / MK;
    for (int kt = 0; kt < nkt; ++kt) {
        __syncthreads();
        for (int e = tid; e < 2 * MK; e += MNT) {
            const int t = e & (MK - 1);
            if (e < MK) stage_rows(k, a, p, hd, kt * MK, t, ks, kt_);
            else stage_rows(v, a, p, hd, kt * MK, t, vs, nullptr);
        }
        __syncthreads();
        const int b0 = kt * (MK / 32), nb = min(MK / 32, qb - b0 + 1);
        auto block = [&](auto diagc, int bb) {
            constexpr bool DIAG = decltype(diagc)::value;
            const int kb = b0 + bb;
            const f32x16 st = mma_qk(*reinterpret_cast<const u32x2 *>(ks + (bb * 32 + col) * 8 + 4 * hh), qf, f32x16{});
            const f32x16 dp = mma_qk(*reinterpret_cast<const u32x2 *>(vs + (bb * 32 + col) * 8 + 4 * hh), gf2, f32x16{});
            f16x8v d0, d1;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * hh;
                float g;
                const float t = tlogit(a, c2k, zrep, drop, seed, int(blockIdx.y), i, kb * 32 + row, st[r], g);
                float pr = fexp2(t - lz);
                if (DIAG) pr = row > col ? 0.f : pr;
                const half_t ds = half_t(g * pr * (dp[r] - dl));
                if (r < 8) d0[r] = ds;
                else d1[r - 8] = ds;
            }
            const half_t *kr = col < 8 ? kt_ + col * VTP + bb * 32 + 4 * hh : nullptr;
            const f16x8v a0 = kr ? vt_frag(kr) : f16x8v{}, a1 = kr ? vt_frag(kr + 16) : f16x8v{};
            dq = ATT_MFMA_32X32X16(a0, d0, dq, 0, 0, 0);
            dq = ATT_MFMA_32X32X16(a1, d1, dq, 0, 0, 0);
        };
        for (int bb = 0; bb < nb; ++bb) {
            if (b0 + bb < qb) block(std::false_type{}, bb);
            else block(std::true_type{}, bb);
        }
    }
    if (i < a.n) {
        float ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = scale * dq[r];
        stvec<h16_t, 4>(gq + rowo, ov);
    }
}

__global__ __launch_bounds__(MNT) void k_attn_bwd_kv_mma(AttnArgs a, float scale, const h16_t *__restrict__ q,
                                                         const h16_t *__restrict__ k, const h16_t *__restrict__ v,
                                                         const h16_t *__restrict__ gout,
                                                         const float *__restrict__ lse,
                                                         const float *__restrict__ delta, h16_t *__restrict__ gk,
                                                         h16_t *__restrict__ gv) {
    __shared__ __attribute__((aligned(16))) h16_t qs[MK * 8], gs[MK * 8];
    __shared__ __attribute__((aligned(16))) half_t qt_[8 * VTP], gt_[8 * VTP];
    __shared__ __attribute__((aligned(16))) float ls[MK], dls[MK];
    [[maybe_unused]] const int nt = (a.n + MQ - 1) / MQ, ktile = int(blockIdx.x);  // key tile 0 meets every query tile: first
    const int p = int(blockIdx.y) / a.nh, hd = int(blockIdx.y) - p * a.nh;
    const int tid = int(threadIdx.x), lane = tid & 63, w = tid >> 6, col = lane & 31, hh = lane >> 5;
    const int kbw = ktile * (MQ / 32) + w, j = kbw * 32 + col, jc = min(j, a.n - 1);
    const int rs = a.nh * 8;
    const int64_t rowk = (int64_t(p) * a.n + jc) * rs + hd * 8 + 4 * hh;
    const u32x2 kf = *reinterpret_cast<const u32x2 *>(k + rowk);
    const u32x2 vf = *reinterpret_cast<const u32x2 *>(v + rowk);
    const int64_t rb = (int64_t(p) * a.nh + hd) * a.n;
    const uint64_t seed = a.drop_below ? *a.seed : 0;
    const float c2k = a.train ? a.c2 * a.keep_scale : a.c2;
    const bool zrep = a.train != 0, drop = a.drop_below != 0;
    f32x16 dk = {}, dv = {};
    // query tiles from the workgroup's first key to the end (MK-row tiles)
    for (int qtile = (ktile * MQ) / MK; qtile * MK < a.n; ++qtile) {
        __syncthreads();
        for (int e = tid; e < 2 * MK; e += MNT) {
            const int t = e & (MK - 1);
            if (e < MK) {
                stage_rows(q, a, p, hd, qtile * MK, t, qs, qt_);
                const int r = qtile * MK + t;
                ls[t] = r < a.n ? lse[rb + r] : INFINITY;  // past the end: p = 0
                dls[t] = r < a.n ? delta[rb + r] : 0.f;
            } else {
                stage_rows(gout, a, p, hd, qtile * MK, t, gs, gt_);
            }
        }
        __syncthreads();
        const int b0 = qtile * (MK / 32);
        auto block = [&](auto diagc, int bb) {
            constexpr bool DIAG = decltype(diagc)::value;
            const int ib = b0 + bb;
            const f32x16 st = mma_qk(*reinterpret_cast<const u32x2 *>(qs + (bb * 32 + col) * 8 + 4 * hh), kf, f32x16{});
            const f32x16 dp = mma_qk(*reinterpret_cast<const u32x2 *>(gs + (bb * 32 + col) * 8 + 4 * hh), vf, f32x16{});
            f16x8v p0, p1, d0, d1;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int rb4 = bb * 32 + 8 * jj + 4 * hh;  // local rows (queries) of registers 4 jj .. 4 jj + 3
                const float4 l4 = *reinterpret_cast<const float4 *>(ls + rb4);
                const float4 d4 = *reinterpret_cast<const float4 *>(dls + rb4);
                const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = 4 * jj + u, row = u + 8 * jj + 4 * hh;  // query within the block
                    float g;
                    const float t = tlogit(a, c2k, zrep, drop, seed, int(blockIdx.y), ib * 32 + row, j, st[r], g);
                    float pr = fexp2(t - lv[u]);
                    if (DIAG) pr = row < col ? 0.f : pr;
                    const half_t ph = half_t(pr), ds = half_t(g * pr * (dp[r] - dv4[u]));
                    if (r < 8) {
                        p0[r] = ph;
                        d0[r] = ds;
                    } else {
                        p1[r - 8] = ph;
                        d1[r - 8] = ds;
                    }
                }
            }
            const half_t *gr = col < 8 ? gt_ + col * VTP + bb * 32 + 4 * hh : nullptr;
            const half_t *qr = col < 8 ? qt_ + col * VTP + bb * 32 + 4 * hh : nullptr;
            dv = ATT_MFMA_32X32X16(gr ? vt_frag(gr) : f16x8v{}, p0, dv, 0, 0, 0);
            dv = ATT_MFMA_32X32X16(gr ? vt_frag(gr + 16) : f16x8v{}, p1, dv, 0, 0, 0);
            dk = ATT_MFMA_32X32X16(qr ? vt_frag(qr) : f16x8v{}, d0, dk, 0, 0, 0);
            dk = ATT_MFMA_32X32X16(qr ? vt_frag(qr + 16) : f16x8v{}, d1, dk, 0, 0, 0);
        };
        for (int bb = 0; bb < MK / 32; ++bb) {
            const int ib = b0 + bb;
            if (ib < kbw) continue;  // queries before this wave's keys
            if (ib > kbw) block(std::false_type{}, bb);
            else block(std::true_type{}, bb);
        }
    }
    if (j < a.n) {
        float ok[4], ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ok[r] = scale * dk[r];
            ov[r] = dv[r];
        }
        const int64_t ro = (int64_t(p) * a.n + j) * rs + hd * 8 + 4 * hh;
        stvec<h16_t, 4>(gk + ro, ok);
        stvec<h16_t, 4>(gv + ro, ov);
    }
}

int dmax_of(int dk, int dv) {
    const int d = std::max(dk, dv);
    return d <= 4 ? 4 : d <= 8 ? 8 : d <= 16 ? 16 : 0;
}

template <typename T, int DM>
void launch_fwd(const AttnArgs &a, const void *q, const void *k, const void *v, void *out, float *lse,
                hipStream_t s) {
    if constexpr (std::is_same<T, h16_t>::value && DM == 8) {
        if (a.dk == 8 && a.dv == 8 && !std::getenv("VQ3D_ATTN_VALU")) {  // the matrix-core form (A/B switch)
            const dim3 mg((a.n + MQ - 1) / MQ, a.P * a.nh);
            k_attn_fwd_mma<<<mg, MNT, 0, s>>>(a, (const h16_t *)q, (const h16_t *)k, (const h16_t *)v, (h16_t *)out, lse);
            return;
        }
    }
    const dim3 grid((a.n + QR - 1) / QR, a.P * a.nh);
    k_attn_fwd<T, DM><<<grid, NT, 0, s>>>(a, (const T *)q, (const T *)k, (const T *)v, (T *)out, lse);
}

template <typename T, int DM>
void launch_bwd(const AttnArgs &a, float scale, const void *q, const void *k, const void *v, const void *out,
                const void *gout, const float *lse, float *delta, void *gq, void *gk, void *gv, hipStream_t s) {
    if constexpr (std::is_same<T, h16_t>::value && DM == 8) {
        if (a.dk == 8 && a.dv == 8 && !std::getenv("VQ3D_ATTN_VALU")) {  // the matrix-core forms (A/B switch)
            const dim3 mg((a.n + MQ - 1) / MQ, a.P * a.nh);
            k_attn_bwd_q_mma<<<mg, MNT, 0, s>>>(a, scale, (const h16_t *)q, (const h16_t *)k, (const h16_t *)v,
                                                (const h16_t *)out, (const h16_t *)gout, lse, delta, (h16_t *)gq);
            k_attn_bwd_kv_mma<<<mg, MNT, 0, s>>>(a, scale, (const h16_t *)q, (const h16_t *)k, (const h16_t *)v,
                                                 (const h16_t *)gout, lse, delta, (h16_t *)gk, (h16_t *)gv);
            return;
        }
    }
    const dim3 grid((a.n + QR - 1) / QR, a.P * a.nh);
    k_attn_bwd_q<T, DM><<<grid, NT, 0, s>>>(a, scale, (const T *)q, (const T *)k, (const T *)v, (const T *)out,
                                            (const T *)gout, lse, delta, (T *)gq);
    k_attn_bwd_kv<T, DM><<<grid, NT, 0, s>>>(a, scale, (const T *)q, (const T *)k, (const T *)v, (const T *)gout,
                                             lse, delta, (T *)gk, (T *)gv);
}

int check_args(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, AttnArgs &a,
               float scale, const vq3d_attn_train *train) {
    if (dtype != VQ3D_HALF && dtype != VQ3D_F32) return 1;
    if (nprob < 1 || n < 1 || nh < 1 || dk < 1 || dv < 1 || !dmax_of(dk, dv)) return 1;
    if (int64_t(nprob) * nh > 65535) return 1;
    a.P = nprob;
    a.n = n;
    a.nh = nh;
    a.dk = dk;
    a.dv = dv;
    a.c2 = scale * LOG2E;
    a.train = 0;
    a.drop_below = 0;
    a.keep_scale = 1.f;
    a.seed = nullptr;
    if (train) {
        const double p = train->dropout_p;
        if (!(p >= 0.0 && p < 1.0)) return 1;
        if (p > 0.0 && !train->seed) return 1;
        a.train = 1;
        a.drop_below = uint32_t(std::min(4294967295.0, p * 4294967296.0));
        a.keep_scale = float(1.0 / (1.0 - p));
        a.seed = train->seed;
    }
    return 0;
}

}  // namespace

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_causal_attn_supported(int32_t nh, int32_t dk, int32_t dv) {
    return nh >= 1 && dk >= 1 && dv >= 1 && dmax_of(dk, dv) ? 1 : 0;
}

size_t vq3d_causal_attn_workspace_bytes(int32_t nprob, int32_t n, int32_t nh) {
    return size_t(nprob) * nh * n * sizeof(float);
}

int vq3d_causal_attn_fwd(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                         const void *q, const void *k, const void *v, void *out, float *lse, vq3d_stream_t stream) {
    return vq3d_causal_attn_fwd_ex(dtype, nprob, n, nh, dk, dv, scale, q, k, v, nullptr, out, lse, stream);
}

int vq3d_causal_attn_fwd_ex(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                            const void *q, const void *k, const void *v, const vq3d_attn_train *train, void *out,
                            float *lse, vq3d_stream_t stream) {
    AttnArgs a;
    if (check_args(dtype, nprob, n, nh, dk, dv, a, scale, train))
        return fail("causal_attn_fwd: unsupported shape / dtype / dropout (p in [0, 1), a seed when p > 0)");
    if (!q || !k || !v || !out || !lse) return fail("causal_attn_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    const int dm = dmax_of(dk, dv);
    if (dtype == VQ3D_HALF) {
        if (dm == 4) launch_fwd<h16_t, 4>(a, q, k, v, out, lse, s);
        else if (dm == 8) launch_fwd<h16_t, 8>(a, q, k, v, out, lse, s);
        else launch_fwd<h16_t, 16>(a, q, k, v, out, lse, s);
    } else {
        if (dm == 4) launch_fwd<float, 4>(a, q, k, v, out, lse, s);
        else if (dm == 8) launch_fwd<float, 8>(a, q, k, v, out, lse, s);
        else launch_fwd<float, 16>(a, q, k, v, out, lse, s);
    }
    return check_launch("causal_attn_fwd");
}

int vq3d_causal_attn_bwd(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                         const void *q, const void *k, const void *v, const void *out, const void *gout,
                         const float *lse, void *workspace, size_t workspace_bytes, void *gq, void *gk, void *gv,
                         vq3d_stream_t stream) {
    return vq3d_causal_attn_bwd_ex(dtype, nprob, n, nh, dk, dv, scale, q, k, v, nullptr, out, gout, lse, workspace,
                                   workspace_bytes, gq, gk, gv, stream);
}

int vq3d_causal_attn_bwd_ex(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                            const void *q, const void *k, const void *v, const vq3d_attn_train *train,
                            const void *out, const void *gout, const float *lse, void *workspace,
                            size_t workspace_bytes, void *gq, void *gk, void *gv, vq3d_stream_t stream) {
    AttnArgs a;
    if (check_args(dtype, nprob, n, nh, dk, dv, a, scale, train))
        return fail("causal_attn_bwd: unsupported shape / dtype / dropout (p in [0, 1), a seed when p > 0)");
    if (!q || !k || !v || !out || !gout || !lse || !workspace || !gq || !gk || !gv)
        return fail("causal_attn_bwd: null pointer");
    if (workspace_bytes < vq3d_causal_attn_workspace_bytes(nprob, n, nh)) return fail("causal_attn_bwd: workspace too small");
    hipStream_t s = as_stream(stream);
    float *delta = static_cast<float *>(workspace);
    const int dm = dmax_of(dk, dv);
    if (dtype == VQ3D_HALF) {
        if (dm == 4) launch_bwd<h16_t, 4>(a, scale, q, k, v, out, gout, lse, delta, gq, gk, gv, s);
        else if (dm == 8) launch_bwd<h16_t, 8>(a, scale, q, k, v, out, gout, lse, delta, gq, gk, gv, s);
        else launch_bwd<h16_t, 16>(a, scale, q, k, v, out, gout, lse, delta, gq, gk, gv, s);
    } else {
        if (dm == 4) launch_bwd<float, 4>(a, scale, q, k, v, out, gout, lse, delta, gq, gk, gv, s);
        else if (dm == 8) launch_bwd<float, 8>(a, scale, q, k, v, out, gout, lse, delta, gq, gk, gv, s);
        else launch_bwd<float, 16>(a, scale, q, k, v, out, gout, lse, delta, gq, gk, gv, s);
    }
    return check_launch("causal_attn_bwd");
}

}  // extern "C"
