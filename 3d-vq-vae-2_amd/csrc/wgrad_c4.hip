// Weight gradient of the full-resolution 3x3x3 circular 4 -> 4 conv: the last up block's
// ResizeConv branch conv2 at 512x512x128 (vqvae/layers.py:124-151, 591-597),
//   dW[co][ci][kh][kw][kd] += sum_v g[v][co] x[v + (kh-1, kw-1, kd-1)][ci],
// on the matrix cores with D-SHIFTS: the voxels of a D-line in groups of four, v = 4m + s,
//   D_(kh,kw)[(s, co)][(pd, ci)] = sum_m g[4m + s][co] x_(kh,kw)[4m + pd - 1][ci]
// M = 16 = 4 shifts x 4 channels (every row real), N = 6 window positions x 4 channels (two
// 16-column tiles, 24 of 32 real), K = 32 groups = one whole 128-voxel D-line per
// v_mfma_f32_16x16x32_bf16; then dW[co][ci][kh][kw][kd] = sum_s D_(kh,kw)[(s, co)][(s + kd, ci)].
// In channels-last memory the g line IS the A^T image [m][16] and the x line, one position back,
// the B image [m][16]: both operands come through the transposing ds_read_b64_tr_b16 from lines
// staged with 16-byte loads.  (The generic MFMA weight-gradient engine pads this conv to 8 input
// and 16 output channels and stages per voxel: 780 us.)
//
// A workgroup walks 4 x 4-line tiles (XCD-contiguous), staging the 16 g lines and the 36 x lines
// of the tile's circular halo (positions -1 .. 130, wrapped) while the previous tile's MFMAs run
// (register prefetch); wave w owns g lines w, w+4, w+8, w+12 of every tile and the 9 x 2
// accumulators of all taps.  The per-workgroup sums go to the workspace in a fixed order and a
// second kernel adds them into dW in a fixed order: deterministic.
#include "engines.h"

#include <algorithm>

namespace vq3d {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int NT = 256;
constexpr int C = 4, D = 128, TH = 4, TW = 4;
constexpr int NG = TH * TW, XL = (TH + 2) * (TW + 2);  // g lines, x halo lines per tile
constexpr int GP = D * C;                              // g line pitch (elements)
constexpr int XOFF = 8;                                // element of x position 0 (position p at XOFF + 4p)
constexpr int XP = XOFF + (D + 4) * C;                 // x line pitch: positions -1 .. D + 2 (+ slack)
constexpr int NE = C * C * 27;                         // 432 weights
constexpr int GU = NG * GP / 8, XU = XL * GP / 8, EU = XL * 4;  // 16-B g / x units, 8-B edge units
constexpr int PG = (GU + NT - 1) / NT, PX = (XU + NT - 1) / NT, PE = (EU + NT - 1) / NT;
constexpr size_t LDS = size_t(NG * GP + XL * XP) * 2;
static_assert(XP % 8 == 0 && (XL * XP * 2) >= 16 * NE * 4, "x image holds the reduction image");

struct WArgs {
    int B, H, W;
    int nth, ntw, ntiles;
};

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

__device__ __forceinline__ bf16x8 tr8(const bf16_t *p0, const bf16_t *p1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct Org {
    int b, h0, w0;
};
__device__ __forceinline__ Org tile_org(const WArgs &a, int t) {
    Org o;
    o.w0 = (t % a.ntw) * TW;
    t /= a.ntw;
    o.h0 = (t % a.nth) * TH;
    o.b = t / a.nth;
    return o;
}

__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void k_wgrad_c4(
    WArgs a, const bf16_t *__restrict__ x, const bf16_t *__restrict__ g, float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t *gl = reinterpret_cast<bf16_t *>(smem);  // [NG][GP]
    bf16_t *xl = gl + NG * GP;                       // [XL][XP]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    // transposed-read offsets: image row (8 grp + q) [+ 4 rows], columns 4p (A) / 16t + 4p (B)
    const int ra = (8 * grp + q) * 16 + 4 * p;
    f32x4 acc[9][2];
#pragma unroll
    for (int kk = 0; kk < 9; ++kk) acc[kk][0] = acc[kk][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the next tile's g lines, x halo lines and x edge positions (-1, D, D + 1, D + 2, circular)
    // in registers while the current tile computes (every load unconditional, indices clamped)
    u32x4 gv[PG], xv[PX];
    u32x2 ev[PE];
    auto load = [&](const Org &o) {
#pragma unroll
        for (int u = 0; u < PG; ++u) {
            const int i = min(tid + u * NT, GU - 1), line = i / (GP / 8), part = i % (GP / 8);
            const int64_t v0 = ((int64_t(o.b) * a.H + o.h0 + line / TW) * a.W + o.w0 + line % TW) * D;
            gv[u] = reinterpret_cast<const u32x4 *>(g + v0 * C)[part];
        }
#pragma unroll
        for (int u = 0; u < PX; ++u) {
            const int i = min(tid + u * NT, XU - 1), line = i / (GP / 8), part = i % (GP / 8);
            const int gh = wrapm(o.h0 - 1 + line / (TW + 2), a.H), gw = wrapm(o.w0 - 1 + line % (TW + 2), a.W);
            xv[u] = reinterpret_cast<const u32x4 *>(x + ((int64_t(o.b) * a.H + gh) * a.W + gw) * D * C)[part];
        }
#pragma unroll
        for (int u = 0; u < PE; ++u) {
            const int i = min(tid + u * NT, EU - 1), line = i >> 2, k = i & 3;
            const int gh = wrapm(o.h0 - 1 + line / (TW + 2), a.H), gw = wrapm(o.w0 - 1 + line % (TW + 2), a.W);
            const int64_t v = ((int64_t(o.b) * a.H + gh) * a.W + gw) * D + (k == 0 ? D - 1 : k - 1);
            ev[u] = *reinterpret_cast<const u32x2 *>(x + v * C);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < PG; ++u) {
            const int i = tid + u * NT;
            if (i < GU) reinterpret_cast<u32x4 *>(gl)[i] = gv[u];
        }
#pragma unroll
        for (int u = 0; u < PX; ++u) {
            const int i = tid + u * NT;
            if (i < XU) reinterpret_cast<u32x4 *>(xl + (i / (GP / 8)) * XP + XOFF)[i % (GP / 8)] = xv[u];
        }
#pragma unroll
        for (int u = 0; u < PE; ++u) {
            const int i = tid + u * NT;
            if (i < EU) {
                const int line = i >> 2, k = i & 3;
                *reinterpret_cast<u32x2 *>(xl + line * XP + XOFF + C * (k == 0 ? -1 : D + k - 1)) = ev[u];
            }
        }
    };
    const TileSched sc = xcd_sched(a.ntiles);
    if (sc.t < sc.end) load(tile_org(a, sc.t));
    for (int tile = sc.t; tile < sc.end; tile += sc.step) {
        __syncthreads();
        store();
        if (tile + sc.step < sc.end) load(tile_org(a, tile + sc.step));
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NG / 4; ++j) {
            const int l = wave + 4 * j, lh = l / TW, lw = l % TW;
            const bf16_t *ga = gl + l * GP + ra;
            const bf16x8 af = tr8(ga, ga + 64);  // rows m = 8 grp + q and + 4
#pragma unroll
            for (int kk = 0; kk < 9; ++kk) {
                const bf16_t *xb = xl + ((lh + kk / 3) * (TW + 2) + lw + kk % 3) * XP + XOFF - C + ra;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const bf16x8 bf = tr8(xb + 16 * t, xb + 16 * t + 64);
                    acc[kk][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[kk][t], 0, 0, 0);
                }
            }
        }
    }
    // fold the shifts: lane (li, grp) holds D[(s = grp, co = i)][(pd = 4t + li / 4, ci = li % 4)]
    // of each tap row -> dW[co][ci][kk][kd = pd - s]; image [wave][s][432], summed in a fixed order
    __syncthreads();
    float *img = reinterpret_cast<float *>(xl);
#pragma unroll
    for (int kk = 0; kk < 9; ++kk)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int kd = 4 * t + (li >> 2) - grp, ci = li & 3;
            if (kd >= 0 && kd < 3) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    img[(wave * 4 + grp) * NE + ((i * C + ci) * 9 + kk) * 3 + kd] = acc[kk][t][i];
            }
        }
    __syncthreads();
    for (int e = tid; e < NE; e += NT) {
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) s += img[r * NE + e];
        part[int64_t(blockIdx.x) * NE + e] = s;
    }
}

// dW[e] += sum over the workgroups' partials in a fixed order: 32 lanes per entry stride the
// workgroups, then a fixed butterfly
__global__ __launch_bounds__(NT) void k_wgrad_c4_reduce(const float *__restrict__ part, int nwg,
                                                        float *__restrict__ dw) {
    const int e = blockIdx.x * (NT / 32) + (threadIdx.x >> 5), r = threadIdx.x & 31;
    float s = 0.f;
    if (e < NE)
        for (int b = r; b < nwg; b += 32) s += part[int64_t(b) * NE + e];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    if (e < NE && r == 0) dw[e] += s;
}

int nwg_of(const vq3d_conv_desc *d) {
    const int ntiles = d->batch * (d->in_h / TH) * (d->in_w / TW);
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1)
            n_cu = 256;
        (void)hipGetLastError();
    }
    // two resident workgroups per CU (LDS 55 KB each), a multiple of the 8 XCDs
    return std::max(1, std::min(ntiles, 2 * n_cu) & ~7) ;
}

}  // namespace

bool wgrad_c4_ok(const vq3d_conv_desc *d) {
    return d->dtype == VQ3D_BF16 && d->cin == C && d->cin2 == 0 && d->cout == C && d->kernel == 3 && d->stride == 1 &&
           d->pad == 1 && d->pad_mode == VQ3D_PAD_CIRCULAR && d->pro_kind == VQ3D_PRO_NONE && d->in_d == D &&
           d->out_d == D && d->in_h == d->out_h && d->in_w == d->out_w && d->in_h % TH == 0 && d->in_w % TW == 0 &&
           d->in_h >= TH && d->in_w >= TW && int64_t(d->batch) * d->in_h * d->in_w * D * C < (int64_t(1) << 31);
}

size_t wgrad_c4_ws(const vq3d_conv_desc *d) { return wgrad_c4_ok(d) ? size_t(nwg_of(d)) * NE * 4 : 0; }

int wgrad_c4(const vq3d_conv_desc *d, const void *x, const void *g, float *dw, void *ws, size_t ws_bytes,
             hipStream_t s) {
    if (!wgrad_c4_ok(d) || !ws || ws_bytes < wgrad_c4_ws(d)) return fail("conv(wgrad_c4): unsupported");
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_wgrad_c4), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(LDS));
        attr = true;
    }
    WArgs a;
    a.B = d->batch;
    a.H = d->in_h;
    a.W = d->in_w;
    a.nth = a.H / TH;
    a.ntw = a.W / TW;
    a.ntiles = a.B * a.nth * a.ntw;
    const int nwg = nwg_of(d);
    k_wgrad_c4<<<nwg, NT, LDS, s>>>(a, (const bf16_t *)x, (const bf16_t *)g, static_cast<float *>(ws));
    k_wgrad_c4_reduce<<<(NE + NT / 32 - 1) / (NT / 32), NT, 0, s>>>(static_cast<const float *>(ws), nwg, dw);
    return check_launch("conv3d_bwd_weight(wgrad_c4)");
}

}  // namespace vq3d
