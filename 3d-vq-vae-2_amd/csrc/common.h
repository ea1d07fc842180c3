// Device-side helpers shared by every libvq3d kernel (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <atomic>
#include <mutex>

// The kernel sources are compiled twice (Makefile): with bf16 as the 16-bit activation / matrix-
// core operand format, and with -DVQ3D_FP16 with IEEE fp16 (the reference trains with fp16 AMP,
// vqvae/train.py:32).  The fp16 build's C++ symbols live in namespace vq3d_fp16 and its C entry
// points carry the suffix __f16, the bf16 build's __bf16 (abi_names.h, generated from
// include/vq3d.h by tools/gen_abi.py); the public entry points (abi_dispatch.cpp, generated too)
// route each call to one build by its dtype arguments.  Error reporting is shared (vq3d_rt).
#ifdef VQ3D_FP16
#define vq3d vq3d_fp16
#endif
#include "abi_names.h"
#include "../../include/vq3d.h"

namespace vq3d_rt {
void set_error(const std::string &msg);
int fail(const std::string &msg);
int check_launch(const char *what);
constexpr int kPairCap = 65536;
constexpr unsigned kTicketRegions = 64, kTicketSlots = 4, kNoTicket = ~0u;
unsigned ticket_slot(hipStream_t st);
float *pair_pool(unsigned slot);
}  // namespace vq3d_rt

namespace vq3d {

constexpr int kWave = 64;

// ---------------------------------------------------------------- storage types
using h16_t = uint16_t;  // raw 16-bit activation bits (bf16, or fp16 in the fp16 build); arithmetic in fp32
#ifdef VQ3D_FP16
using half_t = _Float16;
constexpr int32_t VQ3D_HALF = VQ3D_F16;
#else
using half_t = __bf16;
constexpr int32_t VQ3D_HALF = VQ3D_BF16;
#endif
typedef half_t hx8 __attribute__((ext_vector_type(8)));  // one MFMA A / B fragment (8 elements)
#ifdef VQ3D_FP16
#define VQ3D_MFMA_16X16X32 __builtin_amdgcn_mfma_f32_16x16x32_f16
#else
#define VQ3D_MFMA_16X16X32 __builtin_amdgcn_mfma_f32_16x16x32_bf16
#endif

// the 16-bit value in the low / high half of a dword as fp32 (bf16: a shift or a mask; fp16:
// v_cvt_f32_f16)
__device__ __forceinline__ float h2f_lo(uint32_t u) {
#ifdef VQ3D_FP16
    return float(__builtin_bit_cast(_Float16, uint16_t(u)));
#else
    return __uint_as_float(u << 16);
#endif
}
__device__ __forceinline__ float h2f_hi(uint32_t u) {
#ifdef VQ3D_FP16
    return float(__builtin_bit_cast(_Float16, uint16_t(u >> 16)));
#else
    return __uint_as_float(u & 0xffff0000u);
#endif
}

__device__ __forceinline__ float ld(const float *p) { return *p; }
__device__ __forceinline__ float ld(const h16_t *p) { return h2f_lo(*p); }

// round-to-nearest-even f32 -> the 16-bit format (torch's conversion; NaN stays NaN): the hardware
// v_cvt_pk_bf16_f32 / v_cvt_f16_f32 on gfx950
__device__ __forceinline__ h16_t f2h(float f) { return __builtin_bit_cast(h16_t, static_cast<half_t>(f)); }

// n / d for 0 <= n < 2^31 without an integer divide (Granlund-Montgomery, host-built)
struct FastDiv {
    uint32_t m, s, d;
    __host__ __device__ FastDiv() : m(0), s(0), d(1) {}
    __host__ explicit FastDiv(uint32_t dd) : d(dd) {
        s = 0;
        while ((1u << s) < dd) ++s;
        m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << s) - dd)) / dd + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> s; }
};
__device__ __forceinline__ void st(float *p, float v) { *p = v; }
__device__ __forceinline__ void st(h16_t *p, float v) { *p = f2h(v); }

// Native 32-bit vectors for register-staged loads: an array of HIP's uint4 / uint2 (a class with
// union members) held across a loop is NOT promoted to registers by hipcc -- it lives in scratch
// memory, and every prefetch then waits on its scratch store -- while these are.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------- N-element vector moves
// N consecutive elements of storage type T (bf16 or fp32) as raw 32-bit words, so a kernel can
// issue a whole voxel's (or a run of voxels') loads before it converts anything.  N * sizeof(T)
// is 2, 4, 8 or a multiple of 16 bytes and the address is aligned to min(that, 16).
template <typename T, int N>
struct Raw {
    static constexpr int B = N * int(sizeof(T));
    static constexpr int W = (B + 3) / 4;
    uint32_t w[W];
};
template <typename T, int N>
__device__ __forceinline__ Raw<T, N> ldraw(const T *__restrict__ p) {
    Raw<T, N> r;
    constexpr int B = Raw<T, N>::B;
    if constexpr (B == 2) {
        r.w[0] = *reinterpret_cast<const uint16_t *>(p);
    } else if constexpr (B == 4) {
        r.w[0] = *reinterpret_cast<const uint32_t *>(p);
    } else if constexpr (B == 8) {
        const uint2 u = *reinterpret_cast<const uint2 *>(p);
        r.w[0] = u.x;
        r.w[1] = u.y;
    } else {
        static_assert(B % 16 == 0, "vector width");
#pragma unroll
        for (int i = 0; i < B / 16; ++i) {
            const uint4 u = reinterpret_cast<const uint4 *>(p)[i];
            r.w[4 * i] = u.x;
            r.w[4 * i + 1] = u.y;
            r.w[4 * i + 2] = u.z;
            r.w[4 * i + 3] = u.w;
        }
    }
    return r;
}
template <typename T, int N>
__device__ __forceinline__ void unraw(const Raw<T, N> &r, float (&o)[N]) {
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int i = 0; i < N; ++i) o[i] = __uint_as_float(r.w[i]);
    } else {
#pragma unroll
        for (int i = 0; i < N; ++i) o[i] = (i & 1) ? h2f_hi(r.w[i / 2]) : h2f_lo(r.w[i / 2]);
    }
}
template <typename T, int N>
__device__ __forceinline__ void ldvec(const T *__restrict__ p, float (&o)[N]) {
    unraw<T, N>(ldraw<T, N>(p), o);
}
// N values rounded to T (bf16: round-to-nearest-even) as 2 / 4 / 8 / 16n-byte stores
template <typename T, int N>
__device__ __forceinline__ void stvec(T *__restrict__ p, const float (&v)[N]) {
    Raw<T, N> r;
    constexpr int B = Raw<T, N>::B;
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int i = 0; i < N; ++i) r.w[i] = __float_as_uint(v[i]);
    } else if constexpr (N == 1) {
        r.w[0] = f2h(v[0]);
    } else {
#pragma unroll
        for (int i = 0; i < N / 2; ++i) r.w[i] = uint32_t(f2h(v[2 * i])) | (uint32_t(f2h(v[2 * i + 1])) << 16);
    }
    if constexpr (B == 2) {
        *reinterpret_cast<uint16_t *>(p) = uint16_t(r.w[0]);
    } else if constexpr (B == 4) {
        *reinterpret_cast<uint32_t *>(p) = r.w[0];
    } else if constexpr (B == 8) {
        *reinterpret_cast<uint2 *>(p) = uint2{r.w[0], r.w[1]};
    } else {
        static_assert(B % 16 == 0, "vector width");
#pragma unroll
        for (int i = 0; i < B / 16; ++i)
            reinterpret_cast<uint4 *>(p)[i] = uint4{r.w[4 * i], r.w[4 * i + 1], r.w[4 * i + 2], r.w[4 * i + 3]};
    }
}

// ---------------------------------------------------------------- activations
__device__ __forceinline__ float elu(float z) { return z > 0.f ? z : (expf(z) - 1.f); }
__device__ __forceinline__ float elu_grad(float z) { return z > 0.f ? 1.f : expf(z); }

struct Prologue {
    int kind;  // VQ3D_PRO_*
    float a, b;
    __device__ __forceinline__ float apply(float x) const {
        if (kind == VQ3D_PRO_NONE) return x;
        if (kind == VQ3D_PRO_ADD) return x + a;
        return elu(x + a) + b;
    }
    __device__ __forceinline__ float deriv(float x) const {
        return kind == VQ3D_PRO_ELU_ADD ? elu_grad(x + a) : 1.f;
    }
};

// derivative of the activation in front of a conv, applied in backward-data epilogues
// (vq3d_dgrad_epilogue): mode 1 from the pre-prologue input (elu'(aux + a)); mode 2 from an
// activated tensor t = elu(z) + b: elu'(z) = t - b > 0 ? 1 : t - b + 1.
struct ActDeriv {
    int mode;
    float p;
    __device__ __forceinline__ float operator()(float aux) const {
        if (mode == 1) return elu_grad(aux + p);
        const float z1 = aux - p;
        return z1 > 0.f ? 1.f : z1 + 1.f;
    }
};

__device__ __forceinline__ float epi_act(int act, float v, float a, float b) {
    if (act == VQ3D_ACT_ELU) return elu(v);
    if (act == VQ3D_ACT_ELU_AFFINE) return elu(v + a) + b;
    return v;
}

__device__ __forceinline__ Prologue make_prologue(int kind, const float *a, const float *b) {
    Prologue p;
    p.kind = kind;
    p.a = (kind != VQ3D_PRO_NONE && a) ? *a : 0.f;
    p.b = (kind == VQ3D_PRO_ELU_ADD && b) ? *b : 0.f;
    return p;
}

// ---------------------------------------------------------------- XCD-aware tile schedules
// The dispatcher places workgroup b on XCD b % 8 and every XCD has its own L2.  With a grid that
// is a multiple of 8, a persistent kernel gives each XCD a contiguous eighth of the tiles, and
// the XCD's workgroups walk that range side by side: the halo re-reads of neighbouring tiles and
// the cache lines their partial D-runs share are served by one L2 instead of eight.
struct TileSched {
    int t, end, step;
};
__device__ __forceinline__ TileSched xcd_sched(int ntiles) {
    const int G = gridDim.x, b = blockIdx.x;
    if ((G & 7) || ntiles < G) return TileSched{b, ntiles, G};
    const int per = (ntiles + 7) >> 3, start = (b & 7) * per;
    return TileSched{start + (b >> 3), min(ntiles, start + per), G >> 3};
}
// one tile per workgroup (non-persistent grids): consecutive tiles on one XCD
__device__ __forceinline__ int xcd_tile(int ntiles) {
    const int G = gridDim.x, b = blockIdx.x;
    if ((G & 7) || G != ntiles) return b;
    return (b & 7) * (G >> 3) + (b >> 3);
}

// ---------------------------------------------------------------- reductions
template <typename F>
__device__ __forceinline__ F wave_sum(F v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// fp32 wave sum on the DPP network (no LDS traffic, unlike the ds_bpermute behind __shfl_xor):
// pairs and quads by quad_perm, rows by rotation, then row_bcast:15 / row_bcast:31 carry the row
// totals into lane 63, whose value every lane receives.  A fixed order: deterministic.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xf, false));
}
template <>
__device__ __forceinline__ float wave_sum<float>(float v) {
    v += dpp_mov<0xb1>(v);        // quad_perm [1, 0, 3, 2]
    v += dpp_mov<0x4e>(v);        // quad_perm [2, 3, 0, 1]
    v += dpp_mov<0x124>(v);       // row_ror:4
    v += dpp_mov<0x128>(v);       // row_ror:8
    v += dpp_mov<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
    v += dpp_mov<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// fp32 sum over aligned groups of LANES lanes (a power of two <= 64), every lane of a group
// receiving its group's total: DPP within rows (quad_perm, half-mirror, mirror), one
// ds_bpermute step across rows for 32, the broadcast wave sum for 64.
template <int LANES>
__device__ __forceinline__ float group_sum(float v) {
    static_assert(LANES >= 1 && LANES <= 64 && (LANES & (LANES - 1)) == 0, "group width");
    if constexpr (LANES == 64) {
        return wave_sum(v);
    } else {
        if constexpr (LANES >= 2) v += dpp_mov<0xb1>(v);   // quad_perm [1, 0, 3, 2]
        if constexpr (LANES >= 4) v += dpp_mov<0x4e>(v);   // quad_perm [2, 3, 0, 1]
        if constexpr (LANES >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror: the other quad
        if constexpr (LANES >= 16) v += dpp_mov<0x140>(v); // row_mirror: the other half-row
        if constexpr (LANES >= 32) v += __shfl_xor(v, 16, 64);
        return v;
    }
}

// Deterministic block sum (fixed shuffle tree + fixed LDS order). All threads return the total.
template <typename F, int NT>
__device__ __forceinline__ F block_sum(F v, F *scratch /* >= NT/64 */) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    F t = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += scratch[i];
    return t;
}

// N deterministic block sums at once, each bit-identical to block_sum over scratch + k * S (the
// same wave trees and wave order), with one barrier pair for all N instead of one per value
template <typename F, int NT, int N, int S>
__device__ __forceinline__ void block_sums(F (&v)[N], F *scratch /* >= (N - 1) * S + NT / 64 */) {
    static_assert(S >= NT / 64, "scratch stride");
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    F w[N];
#pragma unroll
    for (int k = 0; k < N; ++k) w[k] = wave_sum(v[k]);
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < N; ++k) scratch[k * S + wid] = w[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) {
        F t = 0;
#pragma unroll
        for (int i = 0; i < NT / 64; ++i) t += scratch[k * S + i];
        v[k] = t;
    }
}

// ---------------------------------------------------------------- in-grid partial sums
// A grid's per-workgroup partials summed by its LAST workgroup to finish, in the order a separate
// one-workgroup pass over them would use (deterministic, bit-identical to that pass) without the
// extra launch.  The hand-off needs no release fence (which would write back the XCD's whole L2,
// the kernel's outputs included: measured 17.7 -> 44 us on a 1024-workgroup 1x1 conv): each
// workgroup's lane 0 stores its {pre, post} pair write-through (relaxed agent-scope 8-byte store),
// drains it, then takes a completion ticket (agent-scope adds); the workgroup whose add completes
// the grid reads every pair with agent-scope (L1-bypassing) loads -- MI355X_MICROARCH.md's
// hand-off table, first row.  The ticket is two-level: same-address atomics serialise (one
// counter for 1,024 workgroups added ~11 us), so workgroup b adds to shard b % 16 (counters a
// 128-B line apart) and the workgroup completing a shard adds to the top counter.  Tickets: a
// per-module array, the host hands each launch a slot (ticket_slot) and the finishing workgroup
// re-arms it to 0.
// Invariant: two launches holding the same slot must never run at the same time.  Slots are
// therefore keyed by STREAM: each stream that launches ticketed kernels owns a region of
// kTicketSlots slots for the life of the process and cycles through it; launches on one stream (or
// captured from one stream into a graph) are ordered, so a slot is free again by the time its
// stream reuses it, and launches on different streams -- a side stream, a second level chain, the
// PixelSNAIL lanes -- never share one.  A graph must be replayed on a stream that runs no ticketed
// launches concurrently with it (its slots are those of the streams it was captured from).
constexpr unsigned kTicketRegions = vq3d_rt::kTicketRegions, kTicketSlots = vq3d_rt::kTicketSlots,
                   kTickets = kTicketRegions * kTicketSlots;
constexpr unsigned kShards = 16, kTicketLine = 32;
static __device__ unsigned g_tickets[kTickets * (kShards + 1) * kTicketLine];
// the stream's next slot (misc.hip: ONE slot table for the library, both 16-bit builds)
inline unsigned ticket_slot(hipStream_t st) { return vq3d_rt::ticket_slot(st); }
// Pair storage for the in-grid sums: kPairCap {pre, post} pairs per slot, one device array for the
// library (misc.hip), so a kernel needs no workspace for them.  A slot is held by one launch at a
// time (the invariant above), so its pairs are too.
constexpr int kPairCap = vq3d_rt::kPairCap;
inline float *pair_pool(unsigned slot) { return vq3d_rt::pair_pool(slot); }
// every thread of the (1-D, NT-thread) workgroup calls this with the workgroup's sums in thread 0;
// part holds nb {pre, post} float pairs; *dpre += the pres' sum, *dpost += the posts'
template <int NT>
__device__ __forceinline__ void finish_partials(float *part, int nb, int bid, float pre, float post, float *dpre,
                                                float *dpost, unsigned slot, float *red /* >= 8 */) {
    static_assert(NT > int(kShards), "one re-arming thread per counter");
    __shared__ unsigned last;
    uint64_t *pp = reinterpret_cast<uint64_t *>(part);
    unsigned *tk = g_tickets + slot * (kShards + 1) * kTicketLine;
    const int nsh = min(nb, int(kShards));
    if (threadIdx.x == 0) {
        const uint64_t v = uint64_t(__float_as_uint(pre)) | (uint64_t(__float_as_uint(post)) << 32);
        __hip_atomic_store(pp + bid, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int sh = bid % int(kShards);
        const unsigned nin = unsigned((nb - sh + int(kShards) - 1) / int(kShards));  // workgroups of the shard
        bool l = atomicAdd(tk + sh * kTicketLine, 1u) == nin - 1;
        if (l) l = atomicAdd(tk + kShards * kTicketLine, 1u) == unsigned(nsh - 1);
        last = l;
    }
    __syncthreads();
    if (!last) return;
    // every load of a pass in flight before the first add (one dependent cross-XCD round trip per
    // strided load); summed in the strided order all the same
    constexpr int PASS = 8;
    float s0 = 0.f, s1 = 0.f;
    for (int i0 = threadIdx.x; i0 < nb; i0 += PASS * NT) {
        uint64_t v[PASS];
#pragma unroll
        for (int u = 0; u < PASS; ++u) {
            const int i = min(i0 + u * NT, nb - 1);
            v[u] = __hip_atomic_load(pp + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
        for (int u = 0; u < PASS; ++u)
            if (i0 + u * NT < nb) {
                s0 += __uint_as_float(uint32_t(v[u]));
                s1 += __uint_as_float(uint32_t(v[u] >> 32));
            }
    }
    float ss[2] = {s0, s1};  // one barrier pair (bit-identical to two block_sum calls)
    block_sums<float, NT, 2, 4>(ss, red);
    s0 = ss[0];
    s1 = ss[1];
    if (threadIdx.x == 0) {
        if (dpre) *dpre += s0;
        if (dpost) *dpost += s1;
    }
    if (threadIdx.x < nsh) atomicExch(tk + threadIdx.x * kTicketLine, 0u);
    if (threadIdx.x == kShards) atomicExch(tk + kShards * kTicketLine, 0u);
}

// The grid-wide {pre, post} sums of a kernel whose workgroups hold their block sums (every thread
// calls this; thread 0's values count): summed in fixed order by the last workgroup when the host
// passed pair storage (GridSum from grid_sum_for), else -- grids beyond kPairCap workgroups --
// float atomics.
struct GridSum {
    float *pairs;
    unsigned slot;
};
template <int NT>
__device__ __forceinline__ void grid_sum2(const GridSum &gs, float pre, float post, float *dpre, float *dpost,
                                          float *red /* >= 8 */) {
    if (!dpre && !dpost) return;
    if (gs.pairs) {
        const int nb = int(gridDim.x * gridDim.y * gridDim.z);
        const int bid = int(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
        finish_partials<NT>(gs.pairs, nb, bid, pre, post, dpre, dpost, gs.slot, red);
    } else if (threadIdx.x == 0) {
        if (dpre) atomicAdd(dpre, pre);
        if (dpost) atomicAdd(dpost, post);
    }
}
// host: the GridSum of a launch of nblocks workgroups on stream s that sums (want)
inline GridSum grid_sum_for(hipStream_t s, int64_t nblocks, bool want) {
    // one workgroup: its own sum is the total (a single add, deterministic)
    if (!want || nblocks <= 1 || nblocks > kPairCap) return GridSum{nullptr, 0u};
    const unsigned k = ticket_slot(s);
    if (k == vq3d_rt::kNoTicket) return GridSum{nullptr, 0u};  // regions exhausted: atomics
    return GridSum{pair_pool(k), k};
}

// ---------------------------------------------------------------- trilinear x2 (align_corners=False)
// Source index pair and weight of the upper neighbour for destination index j (size n source),
// as ATen's area_pixel_compute_source_index + upsample_trilinear3d compute it.
__device__ __forceinline__ void up_coeff(int j, int n, int &i0, int &i1, float &l1) {
    float src = 0.5f * (float(j) + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    i0 = int(src);
    i1 = i0 + ((i0 < n - 1) ? 1 : 0);
    l1 = src - float(i0);
}

}  // namespace vq3d

// ---------------------------------------------------------------- error plumbing (host)
namespace vq3d {
using vq3d_rt::check_launch;
using vq3d_rt::fail;
using vq3d_rt::set_error;
inline hipStream_t as_stream(vq3d_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace vq3d
