// Reconstruction loss, EvoNorm-S0, Adam(amsgrad),
// casts, and the error plumbing of libvq3d.
#include "common.h"
#include "engines.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#ifndef VQ3D_FP16  // one error state for both builds (common.h: vq3d_rt)
namespace vq3d_rt {
static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
int fail(const std::string &msg) {
    set_error(msg);
    return -1;
}
int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(std::string(what) + ": " + hipGetErrorString(e));
    return 0;
}
const char *last_error() { return g_last_error.c_str(); }

// The ticket-slot table (common.h: keyed by stream; one table for both builds, so every ticketed
// launch of the library on one stream draws from that stream's region) and the pair storage the
// slots index.  A stream keeps its region for the life of the process: a region handed to another
// stream while its first owner still had launches in flight -- or baked into a captured graph that
// is replayed later -- would let two concurrent launches share a completion ticket.  torch hands out
// streams from fixed pools (32 per priority per device), so kTicketRegions covers every stream a
// process can create; beyond it, launches get kNoTicket and their grid sums fall back to float
// atomics (correct, not bitwise reproducible).
unsigned ticket_slot(hipStream_t st) {
    static std::mutex mu;
    static hipStream_t owner[kTicketRegions] = {};
    static unsigned next[kTicketRegions] = {}, nreg = 0;
    std::lock_guard<std::mutex> lk(mu);
    unsigned r = nreg;
    for (unsigned i = 0; i < nreg; ++i)
        if (owner[i] == st) {
            r = i;
            break;
        }
    if (r == nreg) {
        if (nreg == kTicketRegions) return kNoTicket;
        owner[nreg++] = st;
    }
    return r * kTicketSlots + (next[r]++ % kTicketSlots);
}
static __device__ uint64_t g_pair_pool[size_t(kTicketRegions) * kTicketSlots * kPairCap];
float *pair_pool(unsigned slot) {
    static std::mutex mu;
    static float *base[64] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    if (!base[dev]) {
        void *p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_pair_pool)) != hipSuccess) return nullptr;
        base[dev] = static_cast<float *>(p);
    }
    return base[dev] + size_t(slot) * kPairCap * 2;
}
}  // namespace vq3d_rt
#endif

namespace vq3d {

static unsigned grid_for(int64_t n) { return unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048))); }
static bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ============================================================================ reconstruction loss
__device__ __forceinline__ bool in_cylinder(int h, int w, int H, int W) {
    // dist((h,w), (H/2, W/2)) <= min(H,W)/2  <=>  (2h-H)^2 + (2w-W)^2 <= min(H,W)^2 (exact)
    const int64_t a = 2 * h - H, b = 2 * w - W, m = min(H, W);
    return a * a + b * b <= m * m;
}

__device__ __forceinline__ float huber(float d) {
    const float ad = fabsf(d);
    return ad < 1.f ? 0.5f * d * d : ad - 0.5f;
}
__device__ __forceinline__ float huber_grad(float d) {
    return d <= -1.f ? -1.f : (d >= 1.f ? 1.f : d);
}

// ---------------------------------------------------------------- Encoder2.parse_input
// Conv3d(1 -> C, k = 1, bias) on the fp32 input volume (layers.py:535): y[v][c] = w[c] x[v] + b[c],
// written in bf16 (the next conv's operand).  The volume is read in fp32, never rounded: under the
// reference's fp16 autocast this conv reads it with 11 mantissa bits, a bf16 copy would have 8.
// A thread owns 4 consecutive voxels (one 16-byte load, 4 C bf16 of output).
template <int C>
__global__ __launch_bounds__(256) void k_pin_fwd(const float *__restrict__ x, int64_t n4, const float *__restrict__ w,
                                                const float *__restrict__ b, h16_t *__restrict__ y) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n4) return;
    const float4 xv = reinterpret_cast<const float4 *>(x)[i];
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    float o[4 * C];
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int c = 0; c < C; ++c) o[v * C + c] = fmaf(w[c], xs[v], b[c]);
    stvec<h16_t, 4 * C>(y + i * 4 * C, o);
}
// weight / bias gradient partials per workgroup: [block][2 C] = (sum g x, sum g) per channel
template <int C>
__global__ __launch_bounds__(256) void k_pin_wgrad(const float *__restrict__ x, const h16_t *__restrict__ g, int64_t n4,
                                                  float *__restrict__ part) {
    __shared__ float red[4 * 2 * C];
    float sw[C], sb[C];
#pragma unroll
    for (int c = 0; c < C; ++c) sw[c] = sb[c] = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256) {
        const float4 xv = reinterpret_cast<const float4 *>(x)[i];
        const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
        float gv[4 * C];
        ldvec<h16_t, 4 * C>(g + i * 4 * C, gv);
#pragma unroll
        for (int v = 0; v < 4; ++v)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                sw[c] = fmaf(gv[v * C + c], xs[v], sw[c]);
                sb[c] += gv[v * C + c];
            }
    }
    float v[2 * C];  // all 2 C sums in one barrier pair (bit-identical to 2 C block_sum calls)
#pragma unroll
    for (int c = 0; c < C; ++c) {
        v[c] = sw[c];
        v[C + c] = sb[c];
    }
    block_sums<float, 256, 2 * C, 4>(v, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int e = 0; e < 2 * C; ++e) part[int64_t(blockIdx.x) * 2 * C + e] = v[e];
    }
}
// fixed-order sum of the partials (one workgroup per entry, a block tree), added into dw / db
template <int C>
__global__ __launch_bounds__(256) void k_pin_wgrad_fin(const float *__restrict__ part, int nb, float *__restrict__ dw,
                                                      float *__restrict__ db) {
    __shared__ float red[4];
    const int e = blockIdx.x;
    float t = 0.f;
    for (int j = threadIdx.x; j < nb; j += 256) t += part[int64_t(j) * 2 * C + e];
    t = block_sum<float, 256>(t, red);
    if (threadIdx.x == 0) {
        if (e < C) {
            if (dw) dw[e] += t;
        } else if (db) {
            db[e - C] += t;
        }
    }
}
static int pin_blocks(int64_t voxels) { return int(std::min<int64_t>(512, (voxels / 4 + 255) / 256)); }

template <typename T>
__global__ __launch_bounds__(256) void k_recon_fwd(const T *__restrict__ dec, const float *__restrict__ x,
                                                  const int64_t *__restrict__ nvs, int B, int H, int W, int D,
                                                  int cyl, float *__restrict__ part) {
    __shared__ float red[4];
    const int64_t n = int64_t(B) * H * W * D;
    float s = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        int64_t t = i;
        const int d = int(t % D); t /= D;
        const int w = int(t % W); t /= W;
        const int h = int(t % H);
        const int b = int(t / H);
        if (cyl && !in_cylinder(h, w, H, W)) continue;
        const float loc = (d >= nvs[b]) ? 0.f : elu(ld(dec + i));
        s += huber(loc - x[i]);
    }
    s = block_sum<float, 256>(s, red);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

struct CommitPtrs {
    const float *p[8];
};

__global__ __launch_bounds__(256) void k_recon_fin(const float *__restrict__ part, int nb, float inv_count,
                                                  CommitPtrs commit, int nc, float *recon, float *total) {
    __shared__ float red[4];
    float s = 0.f;
    for (int j = threadIdx.x; j < nb; j += 256) s += part[j];
    s = block_sum<float, 256>(s, red);
    if (threadIdx.x == 0) {
        const float r = s * inv_count;
        if (recon) *recon = r;
        float tot = r;
        for (int c = 0; c < nc; ++c) tot += *commit.p[c];
        if (total) *total = tot;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_recon_bwd(const T *__restrict__ dec, const float *__restrict__ x,
                                                  const int64_t *__restrict__ nvs, int B, int H, int W, int D,
                                                  int cyl, const float *__restrict__ gtot, float inv_count,
                                                  T *__restrict__ gdec) {
    const int64_t n = int64_t(B) * H * W * D;
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    int64_t t = i;
    const int d = int(t % D); t /= D;
    const int w = int(t % W); t /= W;
    const int h = int(t % H);
    const int b = int(t / H);
    float g = 0.f;
    if ((!cyl || in_cylinder(h, w, H, W)) && d < nvs[b]) {
        const float z = ld(dec + i);
        const float loc = elu(z);
        g = (*gtot * inv_count) * huber_grad(loc - x[i]) * elu_grad(z);
    }
    st(gdec + i, g);
}

// ============================================================================ EvoNorm-S0 (B = 1)
// stats[g] = {mean, std} with unbiased var over (C/G) x voxels; fp64 partial sums per block.
template <typename T>
__global__ __launch_bounds__(256) void k_evo_stats_part(const T *__restrict__ x, int C, int G, int64_t nvox,
                                                       int64_t vox_per_blk, const float *__restrict__ mean,
                                                       double *__restrict__ part) {
    __shared__ double red[4];
    const int cpg = C / G;
    const int64_t v0 = int64_t(blockIdx.x) * vox_per_blk, v1 = min(nvox, v0 + vox_per_blk);
    for (int g = 0; g < G; ++g) {
        const double mu = mean ? double(mean[2 * g]) : 0.0;
        double s = 0.0;
        for (int64_t e = v0 * cpg + threadIdx.x; e < v1 * cpg; e += 256) {
            const int64_t v = e / cpg;
            const int c = g * cpg + int(e - v * cpg);
            const double val = double(ld(x + v * C + c)) - mu;
            s += mean ? val * val : val;
        }
        s = block_sum<double, 256>(s, red);
        if (threadIdx.x == 0) part[int64_t(blockIdx.x) * G + g] = s;
    }
}

__global__ void k_evo_stats_fin(const double *__restrict__ part, int nb, int G, double m, float *__restrict__ stats,
                                int pass) {
    const int g = threadIdx.x;
    if (g >= G) return;
    double s = 0.0;
    for (int b = 0; b < nb; ++b) s += part[int64_t(b) * G + g];
    if (pass == 0) stats[2 * g] = float(s / m);
    else stats[2 * g + 1] = sqrtf(float(s / (m - 1.0)) + 1e-5f);
}

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + expf(-z)); }

template <typename T>
__global__ __launch_bounds__(256) void k_evo_apply(const T *__restrict__ x, int C, int G, int64_t nvox,
                                                  const float *__restrict__ v, const float *__restrict__ gamma,
                                                  const float *__restrict__ beta, const float *__restrict__ stats,
                                                  T *__restrict__ y) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= nvox * C) return;
    const int c = int(i % C);
    const int g = c / (C / G);
    const float xv = ld(x + i);
    const float num = xv * sigmoidf_(xv * v[c]);
    st(y + i, num * gamma[c] / stats[2 * g + 1] + beta[c]);
}

// per block partials: [G] sum(g * num * gamma) and per channel [C] dgamma, dbeta, dv
template <typename T>
__global__ __launch_bounds__(256) void k_evo_bwd_part(const T *__restrict__ x, const T *__restrict__ gy, int C, int G,
                                                     int64_t nvox, int64_t vox_per_blk, const float *__restrict__ v,
                                                     const float *__restrict__ gamma, const float *__restrict__ stats,
                                                     float *__restrict__ part) {
    __shared__ float red[4];
    const int64_t v0 = int64_t(blockIdx.x) * vox_per_blk, v1 = min(nvox, v0 + vox_per_blk);
    const int cpg = C / G;
    float *out = part + int64_t(blockIdx.x) * (G + 3 * C);
    for (int c = 0; c < C; ++c) {
        const float sd = stats[2 * (c / cpg) + 1];
        float sg = 0.f, sb = 0.f, sv = 0.f, ss = 0.f;
        for (int64_t vv = v0 + threadIdx.x; vv < v1; vv += 256) {
            const float xv = ld(x + vv * C + c), g = ld(gy + vv * C + c);
            const float xvv = xv * v[c];
            const float sgm = sigmoidf_(xvv);
            const float num = xv * sgm;
            sg += g * num / sd;
            sb += g;
            sv += (g * gamma[c] / sd) * (xv * xv * sgm * (1.f - sgm));
            ss += g * num * gamma[c];
        }
        sg = block_sum<float, 256>(sg, red);
        sb = block_sum<float, 256>(sb, red);
        sv = block_sum<float, 256>(sv, red);
        ss = block_sum<float, 256>(ss, red);
        if (threadIdx.x == 0) {
            out[G + 3 * c] = sg;
            out[G + 3 * c + 1] = sb;
            out[G + 3 * c + 2] = sv;
            if (c % cpg == 0) out[c / cpg] = 0.f;
            out[c / cpg] += ss;
        }
    }
}

__global__ void k_evo_bwd_fin(const float *__restrict__ part, int nb, int C, int G, float *__restrict__ red_out,
                              float *dv, float *dgamma, float *dbeta) {
    const int j = threadIdx.x;
    const int W = G + 3 * C;
    for (int e = j; e < W; e += blockDim.x) {
        float s = 0.f;
        for (int b = 0; b < nb; ++b) s += part[int64_t(b) * W + e];
        if (e < G) red_out[e] = s;
        else {
            const int c = (e - G) / 3, k = (e - G) % 3;
            if (k == 0 && dgamma) dgamma[c] += s;
            if (k == 1 && dbeta) dbeta[c] += s;
            if (k == 2 && dv) dv[c] += s;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_evo_bwd_apply(const T *__restrict__ x, const T *__restrict__ gy, int C, int G,
                                                      int64_t nvox, const float *__restrict__ v,
                                                      const float *__restrict__ gamma, const float *__restrict__ stats,
                                                      const float *__restrict__ gsum, T *__restrict__ gx) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= nvox * C) return;
    const int c = int(i % C);
    const int cpg = C / G;
    const int g = c / cpg;
    const float mu = stats[2 * g], sd = stats[2 * g + 1];
    const float m = float(nvox) * cpg;
    const float xv = ld(x + i), gv = ld(gy + i);
    const float xvv = xv * v[c];
    const float sgm = sigmoidf_(xvv);
    const float dnum = gv * gamma[c] / sd;
    // d/d sd of sum(g * num * gamma / sd) = -S / sd^2 ; d sd / d var = 1 / (2 sd)
    const float dvar = -gsum[g] / (sd * sd) / (2.f * sd);
    const float r = dnum * (sgm + xvv * sgm * (1.f - sgm)) + dvar * 2.f * (xv - mu) / (m - 1.f);
    st(gx + i, r);
}

// ============================================================================ Adam (amsgrad)
__global__ __launch_bounds__(256) void k_adam_amsgrad(float *__restrict__ p, const float *__restrict__ g,
                                                     float *__restrict__ m, float *__restrict__ v,
                                                     float *__restrict__ vmax, int64_t n, float beta1, float omb1,
                                                     float beta2, float omb2, float step_size, float bc2_sqrt,
                                                     float eps, const int64_t *__restrict__ step_dev, float lr,
                                                     const float *__restrict__ skip) {
#pragma clang fp contract(off)
    if (skip && *skip != 0.f) return;  // the loss scaler found a non-finite gradient: no step
    if (step_dev) {  // bias corrections of step *step_dev + 1, as the host path computes them (double)
        const double st = double(*step_dev + 1);
        const double bc1 = 1.0 - pow(double(beta1), st);
        const double bc2 = 1.0 - pow(double(beta2), st);
        step_size = float(double(lr) / bc1);
        bc2_sqrt = float(sqrt(bc2));
    }
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const float gi = g[i];
        float mi = m[i];
        mi = mi + omb1 * (gi - mi);  // torch lerp_ (weight < 0.5)
        float vi = v[i] * beta2 + omb2 * gi * gi;
        const float vm = fmaxf(vmax[i], vi);
        const float denom = sqrtf(vm) / bc2_sqrt + eps;
        p[i] = p[i] + (-step_size) * (mi / denom);
        m[i] = mi;
        v[i] = vi;
        vmax[i] = vm;
    }
}

__global__ void k_step_inc(int64_t *step, const float *skip) {
    if (!skip || *skip == 0.f) *step += 1;
}

// ============================================================================ dynamic loss scaling
// torch.cuda.amp.GradScaler's device work (the reference trains with PL native AMP, precision=16,
// vqvae/train.py:32): unscale the gradients in place and flag a non-finite one, then update the
// scale (backoff on a flagged step, growth after `interval` clean steps)
__global__ void k_zero1(float *p) { *p = 0.f; }
__global__ __launch_bounds__(256) void k_grad_unscale(float *__restrict__ g, int64_t n, const float *__restrict__ scale,
                                                      float *__restrict__ found_inf) {
    const float inv = float(1.0 / double(*scale));  // GradScaler: scale.double().reciprocal().float()
    bool bad = false;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const float v = g[i];
        bad |= !isfinite(v);
        g[i] = v * inv;
    }
    if (bad) *found_inf = 1.f;  // every writer stores the same value
}
__global__ void k_scale_update(float *scale, int32_t *tracker, const float *found_inf, float growth, float backoff,
                               int32_t interval) {
    if (*found_inf != 0.f) {
        *scale = *scale * backoff;
        *tracker = 0;
    } else {
        const int32_t t = *tracker + 1;
        if (t == interval) {
            const float ns = *scale * growth;
            if (isfinite(ns)) *scale = ns;
            *tracker = 0;
        } else {
            *tracker = t;
        }
    }
}

// ============================================================================ casts
template <typename S, typename D>
__global__ __launch_bounds__(256) void k_cast(const S *__restrict__ s, D *__restrict__ d, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
        st(d + i, ld(s + i));
}

template <typename T>
__global__ __launch_bounds__(256) void k_elu_bwd_out(const T *__restrict__ g, const T *__restrict__ y,
                                                    T *__restrict__ gz, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const float yv = ld(y + i);
        st(gz + i, ld(g + i) * (yv > 0.f ? 1.f : yv + 1.f));
    }
}

// Zero fill / device copy as KERNELS.  hipMemsetAsync / hipMemcpyAsync captured into a HIP graph
// become memset / memcpy nodes, and on this ROCm a replayed graph's memset nodes were measured NOT to
// be ordered with the kernels around them: a captured PixelSNAIL step whose zero fills were memset
// nodes gave different (growing) gradients on every replay, the same step with fill kernels replays
// bit for bit (tools/dbg/replay_bisect.py).  16-byte vectors when both ends allow, else dwords /
// bytes; grid-stride.
template <typename V>
__global__ __launch_bounds__(256) void k_fill0(V *__restrict__ p, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) p[i] = V{};
}
template <typename V>
__global__ __launch_bounds__(256) void k_copyv(V *__restrict__ d, const V *__restrict__ s, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) d[i] = s[i];
}

__global__ __launch_bounds__(256) void k_scale(float *__restrict__ x, float a, int64_t n) {
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) x[i] *= a;
}

// PixelSNAIL glue: y = elu(x + a) + b; its backward with the a / b sums (fixed order, grid_sum2)
template <typename TX, typename TY>
__global__ __launch_bounds__(256) void k_preact_act_fwd(int64_t n, const TX *__restrict__ x, const float *a,
                                                       const float *b, TY *__restrict__ y) {
    const float av = *a, bv = *b;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
        st(y + i, elu(ld(x + i) + av) + bv);
}
template <typename TG, typename TX>
__global__ __launch_bounds__(256) void k_preact_act_bwd(int64_t n, const TG *__restrict__ g, const TX *__restrict__ x,
                                                       const float *a, TX *__restrict__ gx, float *da, float *db,
                                                       GridSum gsum) {
    __shared__ float red[8];
    const float av = *a;
    float sa = 0.f, sb = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const float gv = ld(g + i), v = gv * elu_grad(ld(x + i) + av);
        if (gx) st(gx + i, v);
        sa += v;
        sb += gv;
    }
    {  // both sums in one barrier pair (bit-identical to two block_sum calls)
        float pp[2] = {sa, sb};
        block_sums<float, 256, 2, 4>(pp, red);
        sa = pp[0];
        sb = pp[1];
    }
    grid_sum2<256>(gsum, sa, sb, da, db, red);
}
// 4 consecutive elements (16-byte fp32 / 8-byte 16-bit accesses)
__device__ __forceinline__ void ld4(const float *p, float v[4]) {
    const float4 q = *reinterpret_cast<const float4 *>(p);
    v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
}
__device__ __forceinline__ void ld4(const h16_t *p, float v[4]) {
    const u32x2 q = *reinterpret_cast<const u32x2 *>(p);
    v[0] = h2f_lo(q[0]), v[1] = h2f_hi(q[0]), v[2] = h2f_lo(q[1]), v[3] = h2f_hi(q[1]);
}
__device__ __forceinline__ void st4(float *p, const float v[4]) {
    *reinterpret_cast<float4 *>(p) = float4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void st4(h16_t *p, const float v[4]) {
    *reinterpret_cast<u32x2 *>(p) = u32x2{uint32_t(f2h(v[0])) | (uint32_t(f2h(v[1])) << 16),
                                          uint32_t(f2h(v[2])) | (uint32_t(f2h(v[3])) << 16)};
}
// the backward glue reductions 4 elements per thread-step on <= 512 workgroups (fewer partials
// for the in-grid sum): n4 = n / 4
template <typename TG, typename TX>
__global__ __launch_bounds__(256) void k_preact_act_bwd4(int64_t n4, const TG *__restrict__ g,
                                                        const TX *__restrict__ x, const float *a,
                                                        TX *__restrict__ gx, float *da, float *db, GridSum gsum) {
    __shared__ float red[8];
    const float av = *a;
    float sa = 0.f, sb = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256) {
        float gv[4], xv[4], v[4];
        ld4(g + 4 * i, gv);
        ld4(x + 4 * i, xv);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = gv[j] * elu_grad(xv[j] + av);
            sa += v[j];
            sb += gv[j];
        }
        if (gx) st4(gx + 4 * i, v);
    }
    {  // both sums in one barrier pair (bit-identical to two block_sum calls)
        float pp[2] = {sa, sb};
        block_sums<float, 256, 2, 4>(pp, red);
        sa = pp[0];
        sb = pp[1];
    }
    grid_sum2<256>(gsum, sa, sb, da, db, red);
}
template <typename TO>
__global__ __launch_bounds__(256) void k_scale_bias_res_bwd4(int64_t n4, const float *__restrict__ g,
                                                            const TO *__restrict__ o, const float *scale,
                                                            TO *__restrict__ go, float *dscale, float *dbias,
                                                            GridSum gsum) {
    __shared__ float red[8];
    const float sc = *scale;
    float ss = 0.f, sb = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n4; i += int64_t(gridDim.x) * 256) {
        float gv[4], ov[4], v[4];
        ld4(g + 4 * i, gv);
        ld4(o + 4 * i, ov);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] = gv[j] * sc;
            ss = fmaf(gv[j], ov[j], ss);
            sb += gv[j];
        }
        if (go) st4(go + 4 * i, v);
    }
    {  // both sums in one barrier pair (bit-identical to two block_sum calls)
        float pp[2] = {ss, sb};
        block_sums<float, 256, 2, 4>(pp, red);
        ss = pp[0];
        sb = pp[1];
    }
    grid_sum2<256>(gsum, ss, sb, dscale, dbias, red);
}
static unsigned grid4_for(int64_t n4) { return unsigned(std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 512))); }

// out = o * scale + bias + s; backward go = g * scale, the scale / bias sums
template <typename TO>
__global__ __launch_bounds__(256) void k_scale_bias_res_fwd(int64_t n, const TO *__restrict__ o, const float *scale,
                                                           const float *bias, const float *__restrict__ s,
                                                           float *__restrict__ out) {
    const float sc = *scale, bv = *bias;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
        out[i] = (ld(o + i) * sc + bv) + s[i];
}
template <typename TO>
__global__ __launch_bounds__(256) void k_scale_bias_res_bwd(int64_t n, const float *__restrict__ g,
                                                           const TO *__restrict__ o, const float *scale,
                                                           TO *__restrict__ go, float *dscale, float *dbias,
                                                           GridSum gsum) {
    __shared__ float red[8];
    const float sc = *scale;
    float ss = 0.f, sb = 0.f;
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const float gv = g[i];
        if (go) st(go + i, gv * sc);
        ss = fmaf(gv, ld(o + i), ss);
        sb += gv;
    }
    {  // both sums in one barrier pair (bit-identical to two block_sum calls)
        float pp[2] = {ss, sb};
        block_sums<float, 256, 2, 4>(pp, red);
        ss = pp[0];
        sb = pp[1];
    }
    grid_sum2<256>(gsum, ss, sb, dscale, dbias, red);
}

// every 16-B slot of this workgroup's LDS allocation := all ones (a NaN in bf16 and fp32)
__global__ __launch_bounds__(256) void k_poison_lds(int nslots) {
    extern __shared__ __attribute__((aligned(16))) uint4 lds_slots[];
    for (int i = threadIdx.x; i < nslots; i += 256) lds_slots[i] = uint4{~0u, ~0u, ~0u, ~0u};
    __syncthreads();
}

}  // namespace vq3d

using namespace vq3d;

extern "C" {

#ifndef VQ3D_FP16  // format-independent, defined once (not renamed: abi_names.h)
const char *vq3d_last_error(void) { return vq3d_rt::last_error(); }
const char *vq3d_version(void) { return "vq3d 0.2 gfx950 (bf16 + fp16 builds)"; }
#endif

int vq3d_upsample2x_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd,
                        const void *x, int32_t pro_kind, const float *pro_a, const float *pro_b, void *y,
                        vq3d_stream_t stream) {
    if (batch <= 0 || channels <= 0 || h <= 0 || w <= 0 || dd <= 0) return fail("upsample2x_fwd: bad sizes");
    if (!x || !y || (pro_kind && !pro_a) || (pro_kind == VQ3D_PRO_ELU_ADD && !pro_b))
        return fail("upsample2x_fwd: null pointer");
    return launch_up2_fwd(dtype, batch, channels, h, w, dd, x, pro_kind, pro_a, pro_b, y, as_stream(stream));
}

int vq3d_upsample2x_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd,
                        const void *gy, int32_t pro_kind, const float *pro_a, const vq3d_dgrad_epilogue *epi,
                        void *gx, float *dpro_pre, float *dpro_post, vq3d_stream_t stream) {
    if (batch <= 0 || channels <= 0 || h <= 0 || w <= 0 || dd <= 0) return fail("upsample2x_bwd: bad sizes");
    if (!gy || !gx) return fail("upsample2x_bwd: null pointer");
    const void *aux = epi ? epi->aux : nullptr, *add = epi ? epi->addend : nullptr;
    int dmode = 0;
    const float *dparam = nullptr;
    if (aux && epi->aux_kind == 1) {
        dmode = 2;
        dparam = epi->aux_b;
    } else if (aux && pro_kind == VQ3D_PRO_ELU_ADD) {
        dmode = 1;
        dparam = pro_a;
    }
    if (dmode && !dparam) return fail("upsample2x_bwd: derivative needs its scalar (pro_a or aux_b)");
    return launch_up2_bwd(dtype, batch, channels, h, w, dd, gy, dmode, dparam, aux, add, gx, dpro_pre, dpro_post,
                          as_stream(stream));
}

int64_t vq3d_cylinder_count(int32_t h, int32_t w) {
    int64_t c = 0;
    const int64_t m = std::min(h, w);
    for (int64_t i = 0; i < h; ++i)
        for (int64_t j = 0; j < w; ++j) {
            const int64_t a = 2 * i - h, b = 2 * j - w;
            c += (a * a + b * b <= m * m);
        }
    return c;
}


int vq3d_parse_input_fwd(int32_t dtype, int64_t voxels, int32_t channels, const float *x, const float *w,
                         const float *b, void *y, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("parse_input_fwd: dtype must be the 16-bit format of this build");
    if (voxels <= 0 || voxels % 4 || !(channels == 2 || channels == 4 || channels == 8))
        return fail("parse_input_fwd: voxels % 4 == 0 and channels in {2, 4, 8}");
    if (!x || !w || !b || !y) return fail("parse_input_fwd: null pointer");
    // float4 input loads, 16- to 64-byte output stores
    if (!al16(x) || !al16(y)) return fail("parse_input_fwd: x and y must be 16-byte aligned");
    const int64_t n4 = voxels / 4;
    const unsigned nb = unsigned((n4 + 255) / 256);
    hipStream_t s = as_stream(stream);
    h16_t *Y = static_cast<h16_t *>(y);
    if (channels == 2) k_pin_fwd<2><<<nb, 256, 0, s>>>(x, n4, w, b, Y);
    else if (channels == 4) k_pin_fwd<4><<<nb, 256, 0, s>>>(x, n4, w, b, Y);
    else k_pin_fwd<8><<<nb, 256, 0, s>>>(x, n4, w, b, Y);
    return check_launch("parse_input_fwd");
}

size_t vq3d_parse_input_workspace_bytes(int64_t voxels, int32_t channels) {
    return size_t(pin_blocks(voxels)) * 2 * size_t(channels > 0 ? channels : 1) * 4;
}

int vq3d_parse_input_bwd(int32_t dtype, int64_t voxels, int32_t channels, const float *x, const void *g, float *dw,
                         float *db, void *workspace, size_t ws_bytes, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("parse_input_bwd: dtype must be the 16-bit format of this build");
    if (voxels <= 0 || voxels % 4 || !(channels == 2 || channels == 4 || channels == 8))
        return fail("parse_input_bwd: voxels % 4 == 0 and channels in {2, 4, 8}");
    if (!x || !g || !workspace) return fail("parse_input_bwd: null pointer");
    if (!al16(x) || !al16(g)) return fail("parse_input_bwd: x and g must be 16-byte aligned");
    if (ws_bytes < vq3d_parse_input_workspace_bytes(voxels, channels)) return fail("parse_input_bwd: workspace too small");
    const int nb = pin_blocks(voxels);
    const int64_t n4 = voxels / 4;
    hipStream_t s = as_stream(stream);
    const h16_t *G = static_cast<const h16_t *>(g);
    float *part = static_cast<float *>(workspace);
    if (channels == 2) {
        k_pin_wgrad<2><<<nb, 256, 0, s>>>(x, G, n4, part);
        k_pin_wgrad_fin<2><<<2 * 2, 256, 0, s>>>(part, nb, dw, db);
    } else if (channels == 4) {
        k_pin_wgrad<4><<<nb, 256, 0, s>>>(x, G, n4, part);
        k_pin_wgrad_fin<4><<<2 * 4, 256, 0, s>>>(part, nb, dw, db);
    } else {
        k_pin_wgrad<8><<<nb, 256, 0, s>>>(x, G, n4, part);
        k_pin_wgrad_fin<8><<<2 * 8, 256, 0, s>>>(part, nb, dw, db);
    }
    return check_launch("parse_input_bwd");
}

size_t vq3d_recon_loss_workspace_size(int32_t, int32_t, int32_t, int32_t) { return 4096 * 4; }

int vq3d_recon_loss_fwd(int32_t dtype, const void *dec, const float *x, const int64_t *nvs, int32_t batch, int32_t h,
                        int32_t w, int32_t dd, int32_t cylinder, const float *const *commit, int32_t n_commit,
                        float *recon, float *total, void *workspace, vq3d_stream_t stream) {
    if (batch <= 0 || h <= 0 || w <= 0 || dd <= 0) return fail("recon_loss_fwd: bad sizes");
    if (!dec || !x || !nvs || !workspace || (n_commit && !commit)) return fail("recon_loss_fwd: null pointer");
    if (n_commit < 0 || n_commit > 8) return fail("recon_loss_fwd: at most 8 commitment losses");
    CommitPtrs cp = {};
    for (int i = 0; i < n_commit; ++i) {
        if (!commit[i]) return fail("recon_loss_fwd: null commitment pointer");
        cp.p[i] = commit[i];
    }
    const int64_t n = int64_t(batch) * h * w * dd;
    const int nb = int(std::min<int64_t>(4096, (n + 255) / 256));
    const int64_t cnt = int64_t(batch) * dd * (cylinder ? vq3d_cylinder_count(h, w) : int64_t(h) * w);
    hipStream_t s = as_stream(stream);
    float *part = (float *)workspace;
    if (dtype == VQ3D_F32)
        k_recon_fwd<float><<<nb, 256, 0, s>>>((const float *)dec, x, nvs, batch, h, w, dd, cylinder, part);
    else
        k_recon_fwd<h16_t><<<nb, 256, 0, s>>>((const h16_t *)dec, x, nvs, batch, h, w, dd, cylinder, part);
    k_recon_fin<<<1, 256, 0, s>>>(part, nb, float(1.0 / double(cnt)), cp, n_commit, recon, total);
    return check_launch("recon_loss_fwd");
}

int vq3d_recon_loss_bwd(int32_t dtype, const void *dec, const float *x, const int64_t *nvs, int32_t batch, int32_t h,
                        int32_t w, int32_t dd, int32_t cylinder, const float *g_total, void *gdec,
                        vq3d_stream_t stream) {
    if (batch <= 0 || h <= 0 || w <= 0 || dd <= 0) return fail("recon_loss_bwd: bad sizes");
    if (!dec || !x || !nvs || !g_total || !gdec) return fail("recon_loss_bwd: null pointer");
    const int64_t n = int64_t(batch) * h * w * dd;
    const int64_t cnt = int64_t(batch) * dd * (cylinder ? vq3d_cylinder_count(h, w) : int64_t(h) * w);
    const unsigned nb = unsigned((n + 255) / 256);
    hipStream_t s = as_stream(stream);
    const float ic = float(1.0 / double(cnt));
    if (dtype == VQ3D_F32)
        k_recon_bwd<float><<<nb, 256, 0, s>>>((const float *)dec, x, nvs, batch, h, w, dd, cylinder, g_total, ic,
                                              (float *)gdec);
    else
        k_recon_bwd<h16_t><<<nb, 256, 0, s>>>((const h16_t *)dec, x, nvs, batch, h, w, dd, cylinder, g_total, ic,
                                               (h16_t *)gdec);
    return check_launch("recon_loss_bwd");
}

static int evo_groups(int c) { return std::max(c / 8, 1); }
static int64_t evo_blocks(int64_t nvox) { return std::min<int64_t>(1024, (nvox + 255) / 256); }

size_t vq3d_evonorm_workspace_size(int32_t channels, int64_t voxels) {
    const int64_t nb = evo_blocks(voxels);
    const int G = evo_groups(channels);
    return size_t(nb) * G * 8 + size_t(nb) * (G + 3 * channels) * 4 + size_t(G) * 4 + 1024;
}

int vq3d_evonorm_fwd(int32_t dtype, const void *x, int32_t channels, int64_t voxels, const float *v,
                     const float *gamma, const float *beta, void *y, float *stats, void *workspace,
                     vq3d_stream_t stream) {
    if (channels <= 0 || voxels <= 1) return fail("evonorm_fwd: bad sizes");
    if (!x || !v || !gamma || !beta || !y || !stats || !workspace) return fail("evonorm_fwd: null pointer");
    const int G = evo_groups(channels);
    if (channels % G) return fail("evonorm_fwd: channels not divisible by groups");
    const int64_t nb = evo_blocks(voxels);
    const int64_t vpb = (voxels + nb - 1) / nb;
    hipStream_t s = as_stream(stream);
    double *part = (double *)workspace;
    const double m = double(voxels) * (channels / G);
    for (int pass = 0; pass < 2; ++pass) {
        const float *mean = pass ? stats : nullptr;
        if (dtype == VQ3D_F32)
            k_evo_stats_part<float><<<unsigned(nb), 256, 0, s>>>((const float *)x, channels, G, voxels, vpb, mean,
                                                                 part);
        else
            k_evo_stats_part<h16_t><<<unsigned(nb), 256, 0, s>>>((const h16_t *)x, channels, G, voxels, vpb, mean,
                                                                  part);
        k_evo_stats_fin<<<1, 64 * ((G + 63) / 64), 0, s>>>(part, int(nb), G, m, stats, pass);
    }
    const unsigned na = unsigned((voxels * channels + 255) / 256);
    if (dtype == VQ3D_F32)
        k_evo_apply<float><<<na, 256, 0, s>>>((const float *)x, channels, G, voxels, v, gamma, beta, stats,
                                              (float *)y);
    else
        k_evo_apply<h16_t><<<na, 256, 0, s>>>((const h16_t *)x, channels, G, voxels, v, gamma, beta, stats,
                                               (h16_t *)y);
    return check_launch("evonorm_fwd");
}

int vq3d_evonorm_bwd(int32_t dtype, const void *x, const void *gy, int32_t channels, int64_t voxels, const float *v,
                     const float *gamma, const float *stats, void *gx, float *dv, float *dgamma, float *dbeta,
                     void *workspace, vq3d_stream_t stream) {
    if (channels <= 0 || voxels <= 1) return fail("evonorm_bwd: bad sizes");
    if (!x || !gy || !v || !gamma || !stats || !gx || !workspace) return fail("evonorm_bwd: null pointer");
    const int G = evo_groups(channels);
    const int64_t nb = evo_blocks(voxels);
    const int64_t vpb = (voxels + nb - 1) / nb;
    hipStream_t s = as_stream(stream);
    float *part = (float *)((char *)workspace + size_t(nb) * G * 8);
    float *gsum = part + size_t(nb) * (G + 3 * channels);
    if (dtype == VQ3D_F32)
        k_evo_bwd_part<float><<<unsigned(nb), 256, 0, s>>>((const float *)x, (const float *)gy, channels, G, voxels,
                                                           vpb, v, gamma, stats, part);
    else
        k_evo_bwd_part<h16_t><<<unsigned(nb), 256, 0, s>>>((const h16_t *)x, (const h16_t *)gy, channels, G,
                                                            voxels, vpb, v, gamma, stats, part);
    k_evo_bwd_fin<<<1, 256, 0, s>>>(part, int(nb), channels, G, gsum, dv, dgamma, dbeta);
    const unsigned na = unsigned((voxels * channels + 255) / 256);
    if (dtype == VQ3D_F32)
        k_evo_bwd_apply<float><<<na, 256, 0, s>>>((const float *)x, (const float *)gy, channels, G, voxels, v, gamma,
                                                  stats, gsum, (float *)gx);
    else
        k_evo_bwd_apply<h16_t><<<na, 256, 0, s>>>((const h16_t *)x, (const h16_t *)gy, channels, G, voxels, v,
                                                   gamma, stats, gsum, (h16_t *)gx);
    return check_launch("evonorm_bwd");
}

int vq3d_adam_amsgrad(float *p, const float *g, float *m, float *v, float *vmax, int64_t n, float lr, float beta1,
                      float beta2, float eps, int64_t step, vq3d_stream_t stream) {
    if (n <= 0 || step <= 0) return fail("adam: bad sizes/step");
    if (!p || !g || !m || !v || !vmax) return fail("adam: null pointer");
    const double bc1 = 1.0 - std::pow(double(beta1), double(step));
    const double bc2 = 1.0 - std::pow(double(beta2), double(step));
    const float step_size = float(double(lr) / bc1);
    const float bc2_sqrt = float(std::sqrt(bc2));
    k_adam_amsgrad<<<grid_for(n), 256, 0, as_stream(stream)>>>(p, g, m, v, vmax, n, beta1, float(1.0 - beta1), beta2,
                                                               float(1.0 - beta2), step_size, bc2_sqrt, eps,
                                                               nullptr, lr, nullptr);
    return check_launch("adam_amsgrad");
}

int vq3d_adam_amsgrad_dev(float *p, const float *g, float *m, float *v, float *vmax, int64_t n, float lr,
                          float beta1, float beta2, float eps, int64_t *step, const float *skip,
                          vq3d_stream_t stream) {
    if (n <= 0 || !step) return fail("adam: bad sizes/step");
    if (!p || !g || !m || !v || !vmax) return fail("adam: null pointer");
    hipStream_t s = as_stream(stream);
    k_adam_amsgrad<<<grid_for(n), 256, 0, s>>>(p, g, m, v, vmax, n, beta1, float(1.0 - beta1), beta2,
                                              float(1.0 - beta2), 0.f, 1.f, eps, step, lr, skip);
    k_step_inc<<<1, 1, 0, s>>>(step, skip);
    return check_launch("adam_amsgrad_dev");
}

int vq3d_grad_unscale(float *g, int64_t n, const float *scale, float *found_inf, vq3d_stream_t stream) {
    if (n <= 0 || !g || !scale || !found_inf) return fail("grad_unscale: bad arguments");
    hipStream_t s = as_stream(stream);
    k_zero1<<<1, 1, 0, s>>>(found_inf);
    k_grad_unscale<<<grid_for(n), 256, 0, s>>>(g, n, scale, found_inf);
    return check_launch("grad_unscale");
}

int vq3d_loss_scale_update(float *scale, int32_t *growth_tracker, const float *found_inf, float growth,
                           float backoff, int32_t interval, vq3d_stream_t stream) {
    if (!scale || !growth_tracker || !found_inf || interval < 1) return fail("loss_scale_update: bad arguments");
    k_scale_update<<<1, 1, 0, as_stream(stream)>>>(scale, growth_tracker, found_inf, growth, backoff, interval);
    return check_launch("loss_scale_update");
}

int vq3d_cast(int32_t src_dtype, const void *src, int32_t dst_dtype, void *dst, int64_t n, vq3d_stream_t stream) {
    if (n < 0 || (n && (!src || !dst))) return fail("cast: bad args");
    if (n == 0) return 0;
    hipStream_t s = as_stream(stream);
    const unsigned nb = grid_for(n);
    if (src_dtype == VQ3D_F32 && dst_dtype == VQ3D_HALF)
        k_cast<float, h16_t><<<nb, 256, 0, s>>>((const float *)src, (h16_t *)dst, n);
    else if (src_dtype == VQ3D_HALF && dst_dtype == VQ3D_F32)
        k_cast<h16_t, float><<<nb, 256, 0, s>>>((const h16_t *)src, (float *)dst, n);
    else if (src_dtype == dst_dtype)
        return vq3d_copy(dst, src, size_t(n) * (src_dtype == VQ3D_F32 ? 4 : 2), stream);
    else
        return fail("cast: bad dtype");
    return check_launch("cast");
}

int vq3d_zero(void *p, size_t bytes, vq3d_stream_t stream) {
    if (!bytes) return 0;
    if (!p) return fail("zero: null pointer");
    hipStream_t s = as_stream(stream);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p) | bytes;
    if (a % 16 == 0) k_fill0<u32x4><<<grid_for(int64_t(bytes / 16)), 256, 0, s>>>((u32x4 *)p, int64_t(bytes / 16));
    else if (a % 4 == 0) k_fill0<uint32_t><<<grid_for(int64_t(bytes / 4)), 256, 0, s>>>((uint32_t *)p, int64_t(bytes / 4));
    else k_fill0<uint8_t><<<grid_for(int64_t(bytes)), 256, 0, s>>>((uint8_t *)p, int64_t(bytes));
    return check_launch("zero");
}

int vq3d_copy(void *dst, const void *src, size_t bytes, vq3d_stream_t stream) {
    if (!bytes) return 0;
    if (!dst || !src) return fail("copy: null pointer");
    hipStream_t s = as_stream(stream);
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes;
    if (a % 16 == 0)
        k_copyv<u32x4><<<grid_for(int64_t(bytes / 16)), 256, 0, s>>>((u32x4 *)dst, (const u32x4 *)src, int64_t(bytes / 16));
    else if (a % 4 == 0)
        k_copyv<uint32_t><<<grid_for(int64_t(bytes / 4)), 256, 0, s>>>((uint32_t *)dst, (const uint32_t *)src,
                                                                     int64_t(bytes / 4));
    else
        k_copyv<uint8_t><<<grid_for(int64_t(bytes)), 256, 0, s>>>((uint8_t *)dst, (const uint8_t *)src, int64_t(bytes));
    return check_launch("copy");
}

int vq3d_poison_lds(vq3d_stream_t stream) {
    // 64 KB per workgroup, 8 x the CU count of workgroups: every CU hosts at least two at once
    // over its whole run, so its 160 KB are overwritten in every placement the allocator uses
    constexpr int kBytes = 64 * 1024;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_poison_lds),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kBytes);
        attr = true;
    }
    k_poison_lds<<<256 * 8, 256, kBytes, as_stream(stream)>>>(kBytes / 16);
    return check_launch("poison_lds");
}

int vq3d_elu_bwd_from_output(int32_t dtype, const void *g, const void *y, void *gz, int64_t n,
                             vq3d_stream_t stream) {
    if (n <= 0) return 0;
    if (!g || !y || !gz) return fail("elu_bwd_from_output: null pointer");
    if (dtype == VQ3D_F32)
        k_elu_bwd_out<float><<<grid_for(n), 256, 0, as_stream(stream)>>>((const float *)g, (const float *)y,
                                                                          (float *)gz, n);
    else
        k_elu_bwd_out<h16_t><<<grid_for(n), 256, 0, as_stream(stream)>>>((const h16_t *)g, (const h16_t *)y,
                                                                           (h16_t *)gz, n);
    return check_launch("elu_bwd_from_output");
}

int vq3d_scale(float *x, float a, int64_t n, vq3d_stream_t stream) {
    if (n <= 0) return 0;
    if (!x) return fail("scale: null pointer");
    k_scale<<<grid_for(n), 256, 0, as_stream(stream)>>>(x, a, n);
    return check_launch("scale");
}

static bool glue_dtype(int32_t d) { return d == VQ3D_F32 || d == VQ3D_HALF; }

int vq3d_preact_act_fwd(int32_t x_dtype, int32_t y_dtype, int64_t n, const void *x, const float *a, const float *b,
                        void *y, vq3d_stream_t stream) {
    if (n <= 0) return 0;
    if (!glue_dtype(x_dtype) || !glue_dtype(y_dtype)) return fail("preact_act_fwd: dtype");
    if (!x || !a || !b || !y) return fail("preact_act_fwd: null pointer");
    hipStream_t s = as_stream(stream);
#define PAF(TX, TY) k_preact_act_fwd<TX, TY><<<grid_for(n), 256, 0, s>>>(n, (const TX *)x, a, b, (TY *)y)
    if (x_dtype == VQ3D_F32) {
        if (y_dtype == VQ3D_F32) PAF(float, float);
        else PAF(float, h16_t);
    } else {
        if (y_dtype == VQ3D_F32) PAF(h16_t, float);
        else PAF(h16_t, h16_t);
    }
#undef PAF
    return check_launch("preact_act_fwd");
}

int vq3d_preact_act_bwd(int32_t g_dtype, int32_t x_dtype, int64_t n, const void *g, const void *x, const float *a,
                        void *gx, float *da, float *db, vq3d_stream_t stream) {
    if (n <= 0) return 0;
    if (!glue_dtype(g_dtype) || !glue_dtype(x_dtype)) return fail("preact_act_bwd: dtype");
    if (!g || !x || !a) return fail("preact_act_bwd: null pointer");
    hipStream_t s = as_stream(stream);
    if (n % 4 == 0 && al16(g) && al16(x) && (!gx || al16(gx))) {
        const unsigned nb4 = grid4_for(n / 4);
        const GridSum gs4 = grid_sum_for(s, nb4, da || db);
#define PAB4(TG, TX) k_preact_act_bwd4<TG, TX><<<nb4, 256, 0, s>>>(n / 4, (const TG *)g, (const TX *)x, a, (TX *)gx, da, db, gs4)
        if (g_dtype == VQ3D_F32) {
            if (x_dtype == VQ3D_F32) PAB4(float, float);
            else PAB4(float, h16_t);
        } else {
            if (x_dtype == VQ3D_F32) PAB4(h16_t, float);
            else PAB4(h16_t, h16_t);
        }
#undef PAB4
        return check_launch("preact_act_bwd");
    }
    const unsigned nb = grid_for(n);
    const GridSum gs = grid_sum_for(s, nb, da || db);
#define PAB(TG, TX) k_preact_act_bwd<TG, TX><<<nb, 256, 0, s>>>(n, (const TG *)g, (const TX *)x, a, (TX *)gx, da, db, gs)
    if (g_dtype == VQ3D_F32) {
        if (x_dtype == VQ3D_F32) PAB(float, float);
        else PAB(float, h16_t);
    } else {
        if (x_dtype == VQ3D_F32) PAB(h16_t, float);
        else PAB(h16_t, h16_t);
    }
#undef PAB
    return check_launch("preact_act_bwd");
}

int vq3d_scale_bias_res_fwd(int32_t o_dtype, int64_t n, const void *o, const float *scale, const float *bias,
                            const float *s_, float *out, vq3d_stream_t stream) {
    if (n <= 0) return 0;
    if (!glue_dtype(o_dtype)) return fail("scale_bias_res_fwd: dtype");
    if (!o || !scale || !bias || !s_ || !out) return fail("scale_bias_res_fwd: null pointer");
    hipStream_t s = as_stream(stream);
    if (o_dtype == VQ3D_F32) k_scale_bias_res_fwd<float><<<grid_for(n), 256, 0, s>>>(n, (const float *)o, scale, bias, s_, out);
    else k_scale_bias_res_fwd<h16_t><<<grid_for(n), 256, 0, s>>>(n, (const h16_t *)o, scale, bias, s_, out);
    return check_launch("scale_bias_res_fwd");
}

int vq3d_scale_bias_res_bwd(int32_t o_dtype, int64_t n, const float *g, const void *o, const float *scale, void *go,
                            float *dscale, float *dbias, vq3d_stream_t stream) {
    if (n <= 0) return 0;
    if (!glue_dtype(o_dtype)) return fail("scale_bias_res_bwd: dtype");
    if (!g || !o || !scale) return fail("scale_bias_res_bwd: null pointer");
    hipStream_t s = as_stream(stream);
    const unsigned nb = grid_for(n);
    const GridSum gs = grid_sum_for(s, nb, dscale || dbias);
    if (n % 4 == 0 && al16(g) && al16(o) && (!go || al16(go))) {
        const unsigned nb4 = grid4_for(n / 4);
        const GridSum gs4 = grid_sum_for(s, nb4, dscale || dbias);
        if (o_dtype == VQ3D_F32)
            k_scale_bias_res_bwd4<float><<<nb4, 256, 0, s>>>(n / 4, g, (const float *)o, scale, (float *)go, dscale,
                                                             dbias, gs4);
        else
            k_scale_bias_res_bwd4<h16_t><<<nb4, 256, 0, s>>>(n / 4, g, (const h16_t *)o, scale, (h16_t *)go, dscale,
                                                             dbias, gs4);
        return check_launch("scale_bias_res_bwd");
    }
    if (o_dtype == VQ3D_F32)
        k_scale_bias_res_bwd<float><<<nb, 256, 0, s>>>(n, g, (const float *)o, scale, (float *)go, dscale, dbias, gs);
    else
        k_scale_bias_res_bwd<h16_t><<<nb, 256, 0, s>>>(n, g, (const h16_t *)o, scale, (h16_t *)go, dscale, dbias, gs);
    return check_launch("scale_bias_res_bwd");
}

size_t vq3d_rows_wgrad_workspace_bytes(int64_t nrows, int32_t cg, int32_t cx) {
    return rows_wgrad_workspace(nrows, cg, cx);
}

int vq3d_rows_gemm(int32_t dtype, int64_t nrows, int32_t k, int32_t n, const void *x, int64_t ldx, const void *w,
                   int64_t ldw, int32_t trans_w, const float *bias, void *y, int64_t ldy, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("rows_gemm: 16-bit rows only");
    return launch_rows_gemm(nrows, k, n, x, ldx, w, ldw, trans_w, bias, y, ldy, as_stream(stream));
}

int vq3d_rows_wgrad(int32_t dtype, int64_t nrows, int32_t cg, int32_t cx, const void *g, int64_t ldg, const void *x,
                    int64_t ldx, float *dw, float *db, void *workspace, size_t ws_bytes, vq3d_stream_t stream) {
    if (dtype != VQ3D_HALF) return fail("rows_wgrad: 16-bit rows only");
    return launch_rows_wgrad(nrows, cg, cx, g, ldg, x, ldx, dw, db, workspace, ws_bytes, as_stream(stream));
}

}  // extern "C"
