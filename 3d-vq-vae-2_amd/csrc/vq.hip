// Codebook kernels of the EMA vector quantiser (reference Quantizer, vqvae/layers.py:602-728).
//
//   nearest   : argmin_k cdist(z, E) with torch-CPU cdist arithmetic (bit-exact; SURVEY.md
//               App. B), gather q = E[idx], straight-through zst = x + (q - x), squared error.
//   ema_stats : counts = sum one_hot(idx), dw = one_hot^T z (layers.py:638-643), deterministic.
//   ema_update: decay / Laplace smoothing / normalise (layers.py:649-663).
//   moments + init_apply : first-pass codebook init (layers.py:665-683).
//
// Rows are channels-last voxels: row r = voxel (b, h, w, d), D contiguous values.
#include "common.h"

#include <algorithm>

namespace vq3d {

constexpr int kVqThreads = 256;
constexpr int kLdsCodebookFloats = 16384;  // 64 KiB: K*D up to 16384 staged in LDS

// exact torch-CPU cdist distance (no FMA on the first 4*floor(D/4) terms, FMA tail, IEEE sqrt)
template <int DM>
__device__ __forceinline__ float exact_dist(const float (&x)[DM], const float *e, int d) {
#pragma clang fp contract(off)
    const int b4 = d & ~3;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        if (i < b4) {
            const float t = x[i] - e[i];
            const float p = t * t;
            acc = acc + p;
        }
    }
#pragma unroll
    for (int i = 0; i < DM; ++i) {
        if (i >= b4 && i < d) {
            const float t = x[i] - e[i];
            acc = __builtin_fmaf(t, t, acc);
        }
    }
    return __builtin_sqrtf(acc);
}

template <typename TZ, typename TQ, int DM>
__global__ __launch_bounds__(kVqThreads) void k_vq_nearest(const TZ *__restrict__ z, int64_t n, int d,
                                                          const float *__restrict__ embed, int k,
                                                          int64_t *__restrict__ idx, TQ *__restrict__ zst,
                                                          float *__restrict__ sqpart) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float esh[];
    __shared__ float red[4];
    const bool in_lds = int64_t(k) * d <= kLdsCodebookFloats;
    if (in_lds) {
        for (int i = threadIdx.x; i < k * d; i += kVqThreads) esh[i] = embed[i];
        __syncthreads();
    }
    const float *E = in_lds ? esh : embed;
    const int64_t r = int64_t(blockIdx.x) * kVqThreads + threadIdx.x;
    float sq = 0.f;
    if (r < n) {
        float x[DM];
#pragma unroll
        for (int i = 0; i < DM; ++i) x[i] = i < d ? ld(z + r * d + i) : 0.f;
        float best = __builtin_inff();
        int bi = 0;
        for (int c = 0; c < k; ++c) {
            const float dv = exact_dist<DM>(x, E + c * d, d);
            if (dv < best) {
                best = dv;
                bi = c;
            }
        }
        idx[r] = bi;
        const float *q = E + bi * d;
#pragma unroll
        for (int i = 0; i < DM; ++i) {
            if (i < d) {
                const float diff = q[i] - x[i];
                st(zst + r * d + i, x[i] + diff);
                sq = __builtin_fmaf(diff, diff, sq);
            }
        }
    }
    sq = block_sum<float, kVqThreads>(sq, red);
    if (threadIdx.x == 0) sqpart[blockIdx.x] = sq;
}

// Few rows (the small top-level grids): the codebook is split into chunks over blockIdx.y so the
// search fills the chip.  Each (row, chunk) keeps the first strict minimum of its codes; the
// finish kernel scans the chunks in increasing code order with the same strict `<`, which
// reproduces the sequential first-index argmin exactly.
template <typename TZ, int DM>
__global__ __launch_bounds__(kVqThreads) void k_vq_nearest_part(const TZ *__restrict__ z, int64_t n, int d,
                                                               const float *__restrict__ embed, int k, int ck,
                                                               float *__restrict__ pbest, int *__restrict__ pidx) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) float esh[];
    const int c0 = blockIdx.y * ck, nc = min(ck, k - c0);
    for (int i = threadIdx.x; i < nc * d; i += kVqThreads) esh[i] = embed[int64_t(c0) * d + i];
    __syncthreads();
    const int64_t r = int64_t(blockIdx.x) * kVqThreads + threadIdx.x;
    if (r >= n) return;
    float x[DM];
#pragma unroll
    for (int i = 0; i < DM; ++i) x[i] = i < d ? ld(z + r * d + i) : 0.f;
    float best = __builtin_inff();
    int bi = c0;
    for (int c = 0; c < nc; ++c) {
        const float dv = exact_dist<DM>(x, esh + c * d, d);
        if (dv < best) {
            best = dv;
            bi = c0 + c;
        }
    }
    pbest[int64_t(blockIdx.y) * n + r] = best;
    pidx[int64_t(blockIdx.y) * n + r] = bi;
}

template <typename TZ, typename TQ>
__global__ __launch_bounds__(kVqThreads) void k_vq_nearest_finish(const TZ *__restrict__ z, int64_t n, int d,
                                                                 const float *__restrict__ embed, int nchunk,
                                                                 const float *__restrict__ pbest,
                                                                 const int *__restrict__ pidx,
                                                                 int64_t *__restrict__ idx, TQ *__restrict__ zst,
                                                                 float *__restrict__ sqpart) {
#pragma clang fp contract(off)
    __shared__ float red[4];
    const int64_t r = int64_t(blockIdx.x) * kVqThreads + threadIdx.x;
    float sq = 0.f;
    if (r < n) {
        float best = __builtin_inff();
        int bi = 0;
        for (int j = 0; j < nchunk; ++j) {
            const float v = pbest[int64_t(j) * n + r];
            if (v < best) {
                best = v;
                bi = pidx[int64_t(j) * n + r];
            }
        }
        idx[r] = bi;
        const float *q = embed + int64_t(bi) * d;
        for (int i = 0; i < d; ++i) {
            const float xv = ld(z + r * d + i);
            const float diff = q[i] - xv;
            st(zst + r * d + i, xv + diff);
            sq = __builtin_fmaf(diff, diff, sq);
        }
    }
    sq = block_sum<float, kVqThreads>(sq, red);
    if (threadIdx.x == 0) sqpart[blockIdx.x] = sq;
}

// generic-D fallback (D > 64): row read from memory for every codeword
template <typename TZ, typename TQ>
__global__ __launch_bounds__(kVqThreads) void k_vq_nearest_wide(const TZ *__restrict__ z, int64_t n, int d,
                                                               const float *__restrict__ embed, int k,
                                                               int64_t *__restrict__ idx, TQ *__restrict__ zst,
                                                               float *__restrict__ sqpart) {
#pragma clang fp contract(off)
    __shared__ float red[4];
    const int64_t r = int64_t(blockIdx.x) * kVqThreads + threadIdx.x;
    float sq = 0.f;
    if (r < n) {
        const TZ *x = z + r * d;
        const int b4 = d & ~3;
        float best = __builtin_inff();
        int bi = 0;
        for (int c = 0; c < k; ++c) {
            const float *e = embed + int64_t(c) * d;
            float acc = 0.f;
            for (int i = 0; i < b4; ++i) {
                const float t = ld(x + i) - e[i];
                const float p = t * t;
                acc = acc + p;
            }
            for (int i = b4; i < d; ++i) {
                const float t = ld(x + i) - e[i];
                acc = __builtin_fmaf(t, t, acc);
            }
            const float dv = __builtin_sqrtf(acc);
            if (dv < best) {
                best = dv;
                bi = c;
            }
        }
        idx[r] = bi;
        const float *q = embed + int64_t(bi) * d;
        for (int i = 0; i < d; ++i) {
            const float xv = ld(x + i);
            const float diff = q[i] - xv;
            st(zst + r * d + i, xv + diff);
            sq = __builtin_fmaf(diff, diff, sq);
        }
    }
    sq = block_sum<float, kVqThreads>(sq, red);
    if (threadIdx.x == 0) sqpart[blockIdx.x] = sq;
}

// sum nb partials in order into out[0] (one workgroup)
__global__ __launch_bounds__(256) void k_sum_partials(const float *__restrict__ part, int nb, float *__restrict__ out,
                                                     float coef, float *__restrict__ out2) {
    __shared__ float red[4];
    float s = 0.f;
    for (int j = threadIdx.x; j < nb; j += 256) s += part[j];
    s = block_sum<float, 256>(s, red);
    if (threadIdx.x == 0) {
        *out = s;
        if (out2) *out2 = coef * s;
    }
}

__global__ void k_commit_loss(const float *sq, float coef, float *loss) { *loss = coef * *sq; }

template <typename TZ, typename TG>
__global__ __launch_bounds__(256) void k_vq_bwd(const TZ *__restrict__ z, int64_t n, int d,
                                               const float *__restrict__ embed, const int64_t *__restrict__ idx,
                                               const TG *__restrict__ gzst, const float *__restrict__ gloss,
                                               float coef, TZ *__restrict__ gz) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n * d) return;
    const int64_t r = i / d;
    const int c = int(i - r * d);
    const float q = embed[idx[r] * d + c];
    const float x = ld(z + i);
    const float gl = gloss ? *gloss : 0.f;
    // d/dx [cc * mean((q - x)^2)] = coef * (x - q), coef = 2 cc / numel
    const float v = ld(gzst + i) + gl * (coef * (x - q));
    st(gz + i, v);
}

// ---------------------------------------------------------------- EMA statistics
// Workgroup (row chunk of kStatRows rows, tile of 256 (code, column) entries); entry
// e = c * (d + 1) + j: j < d sums z[r][j] over the chunk's rows with idx[r] == c, j == d counts
// them.  Every thread walks the chunk's rows in order (the row's code is wave-uniform, its z
// row is read by consecutive lanes), so partials are deterministic; part[chunk][k * (d + 1)].
constexpr int kStatRows = 256;

template <typename TZ>
__global__ __launch_bounds__(256) void k_vq_ema_stats(const TZ *__restrict__ z, int64_t n, int d,
                                                     const int64_t *__restrict__ idx, int k,
                                                     float *__restrict__ part) {
    const int64_t r0 = int64_t(blockIdx.x) * kStatRows;
    const int nr = int(min<int64_t>(kStatRows, n - r0));
    const int ne = k * (d + 1);
    const int e = blockIdx.y * 256 + threadIdx.x;
    const int c = e / (d + 1), j = e - c * (d + 1);
    float acc = 0.f;
    if (e < ne) {
        int rr = 0;
        for (; rr + 8 <= nr; rr += 8) {  // 8 rows' loads in flight, summed in row order
            int ci[8];
            float zv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t r = r0 + rr + u;
                ci[u] = int(idx[r]);
                zv[u] = j < d ? ld(z + r * d + j) : 1.f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (ci[u] == c) acc += zv[u];
        }
        for (; rr < nr; ++rr) {
            const int64_t r = r0 + rr;
            if (int(idx[r]) == c) acc += j < d ? ld(z + r * d + j) : 1.f;
        }
        part[int64_t(blockIdx.x) * ne + e] = acc;
    }
}

// counts / dw = sum of the per-block partials in block order: LANES lanes per entry sum
// strided slices (8 loads in flight), then a fixed xor-shuffle tree (deterministic)
template <int LANES>
__global__ __launch_bounds__(256) void k_vq_stats_reduce(int nb, int k, int d, const float *__restrict__ part,
                                                        float *__restrict__ counts, float *__restrict__ dw) {
    const int64_t ne = int64_t(k) * (d + 1);
    const int64_t f = int64_t(blockIdx.x) * (256 / LANES) + threadIdx.x / LANES;
    const int lane = threadIdx.x % LANES;
    float s = 0.f;
    if (f < ne) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int b0 = lane; b0 < nb; b0 += 8 * LANES) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + u * LANES < nb) acc[u] += part[int64_t(b0 + u * LANES) * ne + f];
        }
        s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    s = group_sum<LANES>(s);
    if (lane == 0 && f < ne) {
        const int c = int(f / (d + 1)), j = int(f - int64_t(c) * (d + 1));
        if (j < d) dw[int64_t(c) * d + j] = s;
        else counts[c] = s;
    }
}

__global__ __launch_bounds__(1024) void k_vq_ema_update(float *__restrict__ embed, float *__restrict__ embed_avg,
                                                       float *__restrict__ cs, const float *__restrict__ counts,
                                                       const float *__restrict__ dw, int k, int d, float decay,
                                                       float one_minus_decay, float alpha) {
#pragma clang fp contract(off)
    __shared__ float red[16];
    float part = 0.f;
    for (int c = threadIdx.x; c < k; c += 1024) {
        const float v = cs[c] * decay + counts[c] * one_minus_decay;
        cs[c] = v;
        part += v;
    }
    const float ntot = block_sum<float, 1024>(part, red);
    const float denom = ntot + float(k) * alpha;
    for (int64_t e = threadIdx.x; e < int64_t(k) * d; e += 1024) {
        const int c = int(e / d);
        const float ea = embed_avg[e] * decay + dw[e] * one_minus_decay;
        embed_avg[e] = ea;
        const float smoothed = ntot * ((cs[c] + alpha) / denom);
        embed[e] = ea / smoothed;
    }
}

// ---------------------------------------------------------------- first-pass init
// two-pass mean / unbiased variance per dimension, fixed-order partials (fp64 accumulate)
template <typename TZ>
__global__ __launch_bounds__(256) void k_vq_moments_part(const TZ *__restrict__ z, int64_t n, int d,
                                                        int64_t rows_per_blk, const float *__restrict__ mean,
                                                        double *__restrict__ part) {
    __shared__ double red[4];
    const int64_t r0 = int64_t(blockIdx.x) * rows_per_blk;
    const int64_t r1 = min(n, r0 + rows_per_blk);
    for (int j = 0; j < d; ++j) {
        const double mu = mean ? double(mean[j]) : 0.0;
        double s = 0.0;
        for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
            const double v = double(ld(z + r * d + j)) - mu;
            s += mean ? v * v : v;
        }
        s = block_sum<double, 256>(s, red);
        if (threadIdx.x == 0) part[int64_t(blockIdx.x) * d + j] = s;
    }
}

__global__ void k_vq_moments_fin(const double *__restrict__ part, int nb, int d, int64_t n, float *__restrict__ out,
                                 int is_var) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= d) return;
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += part[int64_t(b) * d + j];
    out[j] = is_var ? float(sqrt(s / double(n - 1))) : float(s / double(n));
}

__global__ __launch_bounds__(256) void k_vq_init_apply(float *__restrict__ embed, float *__restrict__ embed_avg,
                                                      float *__restrict__ cs, int64_t *__restrict__ first_pass,
                                                      const float *__restrict__ mean, const float *__restrict__ std,
                                                      int k, int d, float inv_world, float add) {
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e < int64_t(k) * d) {
        const int j = int(e % d);
        const float m = inv_world == 1.f ? mean[j] : mean[j] * inv_world;
        const float sd = inv_world == 1.f ? std[j] : std[j] * inv_world;
        const float v = embed[e] * sd + m;
        embed[e] = v;
        embed_avg[e] = v;
    }
    if (e < k) cs[e] += add;
    if (e == 0 && first_pass) *first_pass = 0;
}

// ---------------------------------------------------------------- host
struct VqPlan {
    int64_t nb_near, nb_stats;
    int nchunk, ck;  // codebook chunks of the split search (1: single pass)
    size_t off_sq, off_c, off_d, off_mom, off_pb, off_pi, bytes;
};

static VqPlan plan_vq(int64_t n, int d, int k) {
    VqPlan p;
    p.nb_near = (n + kVqThreads - 1) / kVqThreads;
    p.nb_stats = (n + kStatRows - 1) / kStatRows;
    p.off_sq = 0;
    p.off_c = (size_t(p.nb_near) * 4 + 255) / 256 * 256;
    p.off_d = p.off_c + (size_t(p.nb_stats) * k * 4 + 255) / 256 * 256;
    p.off_mom = p.off_d + (size_t(p.nb_stats) * k * d * 4 + 255) / 256 * 256;
    // split the codebook when the rows alone leave the chip idle (< 128 row blocks)
    p.nchunk = 1;
    p.ck = k;
    if (p.nb_near < 128 && d <= 64) {
        int nc = int(std::min<int64_t>(std::max<int64_t>(1, 512 / p.nb_near), std::max(1, k / 8)));
        p.ck = (k + nc - 1) / nc;
        p.nchunk = (k + p.ck - 1) / p.ck;
    }
    p.off_pb = p.off_mom + (size_t(1024) * d * 8 + 255) / 256 * 256;
    p.off_pi = p.off_pb + (size_t(p.nchunk) * n * 4 + 255) / 256 * 256;
    p.bytes = p.off_pi + size_t(p.nchunk) * n * 4 + 256;
    return p;
}

template <typename TZ, typename TQ>
static void launch_nearest(const void *z, int64_t n, int d, const float *embed, int k, int64_t *idx, void *zst,
                           float *sqpart, hipStream_t s) {
    const unsigned nb = unsigned((n + kVqThreads - 1) / kVqThreads);
    const size_t lds = (int64_t(k) * d <= kLdsCodebookFloats) ? size_t(k) * d * 4 : 0;
    const TZ *zz = static_cast<const TZ *>(z);
    TQ *q = static_cast<TQ *>(zst);
    if (d <= 2)
        k_vq_nearest<TZ, TQ, 2><<<nb, kVqThreads, lds, s>>>(zz, n, d, embed, k, idx, q, sqpart);
    else if (d <= 4)
        k_vq_nearest<TZ, TQ, 4><<<nb, kVqThreads, lds, s>>>(zz, n, d, embed, k, idx, q, sqpart);
    else if (d <= 8)
        k_vq_nearest<TZ, TQ, 8><<<nb, kVqThreads, lds, s>>>(zz, n, d, embed, k, idx, q, sqpart);
    else if (d <= 16)
        k_vq_nearest<TZ, TQ, 16><<<nb, kVqThreads, lds, s>>>(zz, n, d, embed, k, idx, q, sqpart);
    else if (d <= 32)
        k_vq_nearest<TZ, TQ, 32><<<nb, kVqThreads, lds, s>>>(zz, n, d, embed, k, idx, q, sqpart);
    else if (d <= 64)
        k_vq_nearest<TZ, TQ, 64><<<nb, kVqThreads, lds, s>>>(zz, n, d, embed, k, idx, q, sqpart);
    else
        k_vq_nearest_wide<TZ, TQ><<<nb, kVqThreads, 0, s>>>(zz, n, d, embed, k, idx, q, sqpart);
}

}  // namespace vq3d

using namespace vq3d;

extern "C" {

size_t vq3d_vq_workspace_size(int64_t n, int32_t d, int32_t k) {
    if (n <= 0 || d <= 0 || k <= 0) return 0;
    return plan_vq(n, d, k).bytes;
}

int vq3d_vq_nearest(int32_t z_dtype, const void *z, int64_t n, int32_t d, const float *embed, int32_t k,
                    int64_t *idx, int32_t zst_dtype, void *zst, float *sqerr_out, void *workspace,
                    vq3d_stream_t stream) {
    if (n <= 0 || d <= 0 || k <= 0) return fail("vq_nearest: bad sizes");
    if (!z || !embed || !idx || !zst || !sqerr_out || !workspace) return fail("vq_nearest: null pointer");
    hipStream_t s = as_stream(stream);
    VqPlan p = plan_vq(n, d, k);
    float *sqpart = reinterpret_cast<float *>(static_cast<char *>(workspace) + p.off_sq);
    const bool zf = z_dtype == VQ3D_F32, qf = zst_dtype == VQ3D_F32;
    if (p.nchunk > 1) {
        float *pb = reinterpret_cast<float *>(static_cast<char *>(workspace) + p.off_pb);
        int *pi = reinterpret_cast<int *>(static_cast<char *>(workspace) + p.off_pi);
        const dim3 g1{unsigned(p.nb_near), unsigned(p.nchunk), 1u};
        const size_t lds = size_t(p.ck) * d * 4;
        auto part = [&](auto tz) {
            using TZ = decltype(tz);
            const TZ *zz = static_cast<const TZ *>(z);
            if (d <= 8) k_vq_nearest_part<TZ, 8><<<g1, kVqThreads, lds, s>>>(zz, n, d, embed, k, p.ck, pb, pi);
            else if (d <= 16) k_vq_nearest_part<TZ, 16><<<g1, kVqThreads, lds, s>>>(zz, n, d, embed, k, p.ck, pb, pi);
            else if (d <= 32) k_vq_nearest_part<TZ, 32><<<g1, kVqThreads, lds, s>>>(zz, n, d, embed, k, p.ck, pb, pi);
            else k_vq_nearest_part<TZ, 64><<<g1, kVqThreads, lds, s>>>(zz, n, d, embed, k, p.ck, pb, pi);
        };
        const unsigned nb = unsigned(p.nb_near);
        if (zf) {
            part(float{});
            if (qf) k_vq_nearest_finish<float, float><<<nb, kVqThreads, 0, s>>>((const float *)z, n, d, embed, p.nchunk, pb, pi, idx, (float *)zst, sqpart);
            else k_vq_nearest_finish<float, h16_t><<<nb, kVqThreads, 0, s>>>((const float *)z, n, d, embed, p.nchunk, pb, pi, idx, (h16_t *)zst, sqpart);
        } else {
            part(h16_t{});
            if (qf) k_vq_nearest_finish<h16_t, float><<<nb, kVqThreads, 0, s>>>((const h16_t *)z, n, d, embed, p.nchunk, pb, pi, idx, (float *)zst, sqpart);
            else k_vq_nearest_finish<h16_t, h16_t><<<nb, kVqThreads, 0, s>>>((const h16_t *)z, n, d, embed, p.nchunk, pb, pi, idx, (h16_t *)zst, sqpart);
        }
        if (int r = check_launch("vq_nearest(split)")) return r;
        k_sum_partials<<<1, 256, 0, s>>>(sqpart, int(p.nb_near), sqerr_out, 0.f, nullptr);
        return check_launch("vq_nearest(sum)");
    }
    if (zf && qf) launch_nearest<float, float>(z, n, d, embed, k, idx, zst, sqpart, s);
    else if (zf) launch_nearest<float, h16_t>(z, n, d, embed, k, idx, zst, sqpart, s);
    else if (qf) launch_nearest<h16_t, float>(z, n, d, embed, k, idx, zst, sqpart, s);
    else launch_nearest<h16_t, h16_t>(z, n, d, embed, k, idx, zst, sqpart, s);
    if (int r = check_launch("vq_nearest")) return r;
    k_sum_partials<<<1, 256, 0, s>>>(sqpart, int(p.nb_near), sqerr_out, 0.f, nullptr);
    return check_launch("vq_nearest(sum)");
}

int vq3d_vq_commit_loss(const float *sqerr, float coef, float *loss, vq3d_stream_t stream) {
    if (!sqerr || !loss) return fail("vq_commit_loss: null pointer");
    k_commit_loss<<<1, 1, 0, as_stream(stream)>>>(sqerr, coef, loss);
    return check_launch("vq_commit_loss");
}

int vq3d_vq_bwd(int32_t z_dtype, const void *z, int64_t n, int32_t d, const float *embed, const int64_t *idx,
                int32_t g_dtype, const void *g_zst, const float *g_loss, float coef, void *gz,
                vq3d_stream_t stream) {
    if (n <= 0 || d <= 0) return fail("vq_bwd: bad sizes");
    if (!z || !embed || !idx || !g_zst || !gz) return fail("vq_bwd: null pointer");
    const unsigned nb = unsigned((n * d + 255) / 256);
    hipStream_t s = as_stream(stream);
    const bool zf = z_dtype == VQ3D_F32, gf = g_dtype == VQ3D_F32;
    if (zf && gf)
        k_vq_bwd<float, float><<<nb, 256, 0, s>>>((const float *)z, n, d, embed, idx, (const float *)g_zst, g_loss,
                                                  coef, (float *)gz);
    else if (zf)
        k_vq_bwd<float, h16_t><<<nb, 256, 0, s>>>((const float *)z, n, d, embed, idx, (const h16_t *)g_zst,
                                                   g_loss, coef, (float *)gz);
    else if (gf)
        k_vq_bwd<h16_t, float><<<nb, 256, 0, s>>>((const h16_t *)z, n, d, embed, idx, (const float *)g_zst,
                                                   g_loss, coef, (h16_t *)gz);
    else
        k_vq_bwd<h16_t, h16_t><<<nb, 256, 0, s>>>((const h16_t *)z, n, d, embed, idx, (const h16_t *)g_zst,
                                                    g_loss, coef, (h16_t *)gz);
    return check_launch("vq_bwd");
}

int vq3d_vq_ema_stats(int32_t z_dtype, const void *z, int64_t n, int32_t d, const int64_t *idx, int32_t k,
                      float *counts, float *dw, void *workspace, vq3d_stream_t stream) {
    if (n <= 0 || d <= 0 || k <= 0) return fail("vq_ema_stats: bad sizes");
    if (!z || !idx || !counts || !dw || !workspace) return fail("vq_ema_stats: null pointer");
    hipStream_t s = as_stream(stream);
    VqPlan p = plan_vq(n, d, k);
    float *part = reinterpret_cast<float *>(static_cast<char *>(workspace) + p.off_c);  // off_c..off_mom
    const int64_t ne = int64_t(k) * (d + 1);
    const dim3 grid{unsigned(p.nb_stats), unsigned((ne + 255) / 256), 1u};
    if (z_dtype == VQ3D_F32)
        k_vq_ema_stats<float><<<grid, 256, 0, s>>>((const float *)z, n, d, idx, k, part);
    else
        k_vq_ema_stats<h16_t><<<grid, 256, 0, s>>>((const h16_t *)z, n, d, idx, k, part);
    if (int r = check_launch("vq_ema_stats")) return r;
    int lanes = 1;
    while (lanes < 64 && lanes * 16 < p.nb_stats) lanes *= 2;
#define RED(L)                                                                                                 \
    k_vq_stats_reduce<L><<<unsigned((ne + 256 / L - 1) / (256 / L)), 256, 0, s>>>(int(p.nb_stats), k, d, part,  \
                                                                                  counts, dw)
    switch (lanes) {
    case 1: RED(1); break;
    case 2: RED(2); break;
    case 4: RED(4); break;
    case 8: RED(8); break;
    case 16: RED(16); break;
    case 32: RED(32); break;
    default: RED(64); break;
    }
#undef RED
    return check_launch("vq_ema_stats(reduce)");
}

int vq3d_vq_ema_update(float *embed, float *embed_avg, float *cluster_size, const float *counts, const float *dw,
                       int32_t k, int32_t d, float decay, float laplace_alpha, vq3d_stream_t stream) {
    if (k <= 0 || d <= 0) return fail("vq_ema_update: bad sizes");
    if (!embed || !embed_avg || !cluster_size || !counts || !dw) return fail("vq_ema_update: null pointer");
    // torch: mul_(decay).add_(x, alpha=1-decay) with both scalars cast to fp32
    const float omd = float(1.0 - double(decay));
    k_vq_ema_update<<<1, 1024, 0, as_stream(stream)>>>(embed, embed_avg, cluster_size, counts, dw, k, d, decay, omd,
                                                       laplace_alpha);
    return check_launch("vq_ema_update");
}

int vq3d_vq_moments(int32_t z_dtype, const void *z, int64_t n, int32_t d, float *mean, float *std, void *workspace,
                    vq3d_stream_t stream) {
    if (n <= 0 || d <= 0) return fail("vq_moments: bad sizes");
    if (!z || !mean || !std || !workspace) return fail("vq_moments: null pointer");
    hipStream_t s = as_stream(stream);
    VqPlan p = plan_vq(n, d, 1);
    double *part = reinterpret_cast<double *>(static_cast<char *>(workspace) + p.off_mom);
    const int64_t rpb = std::max<int64_t>(256, (n + 1023) / 1024);
    const int nb = int((n + rpb - 1) / rpb);
    const unsigned fb = unsigned((d + 63) / 64);
    for (int pass = 0; pass < 2; ++pass) {
        const float *mu = pass ? mean : nullptr;
        if (z_dtype == VQ3D_F32)
            k_vq_moments_part<float><<<nb, 256, 0, s>>>((const float *)z, n, d, rpb, mu, part);
        else
            k_vq_moments_part<h16_t><<<nb, 256, 0, s>>>((const h16_t *)z, n, d, rpb, mu, part);
        k_vq_moments_fin<<<fb, 64, 0, s>>>(part, nb, d, n, pass ? std : mean, pass);
    }
    return check_launch("vq_moments");
}

int vq3d_vq_init_apply(float *embed, float *embed_avg, float *cluster_size, int64_t *first_pass, const float *mean,
                       const float *std, int32_t k, int32_t d, float inv_world, float n_total,
                       vq3d_stream_t stream) {
    if (k <= 0 || d <= 0) return fail("vq_init_apply: bad sizes");
    if (!embed || !embed_avg || !cluster_size || !mean || !std) return fail("vq_init_apply: null pointer");
    const int64_t kd = std::max<int64_t>(int64_t(k) * d, k);
    k_vq_init_apply<<<unsigned((kd + 255) / 256), 256, 0, as_stream(stream)>>>(
        embed, embed_avg, cluster_size, first_pass, mean, std, k, d, inv_world, n_total / float(k));
    return check_launch("vq_init_apply");
}

}  // extern "C"
