// The 1x1x1 convs of the PixelSNAIL prior as GEMMs over voxel rows (pixel_model/layers.py:370-404
// branch / skip / aux convs, :225-248 ExpandRFConv, :665-675 key-value / query projections,
// pixelsnail.py:39-43 / 78-82 parse_input / parse_output -- every one a Conv3d(kernel_size=1) of a
// channels-last activation, i.e. a [voxels][cin] x [cin][cout] product):
//
//   forward        y[v][n]  = sum_k x[v][k] w[n][k] (+ bias[n])      (w: [cout][cin], trans_w = 0)
//   backward-data  gx[v][n] = sum_k g[v][k] w[k][n]                  (w: [cout][cin], trans_w = 1)
//
// fp32 accumulation on the matrix cores (v_mfma_f32_16x16x32, the build's 16-bit format), the
// result rounded once to that format (what the reference's autocast 1x1 convs store).  The weight
// slice of a workgroup's 64 outputs is staged once in LDS as [n][k] rows (transposed on the way in
// for the backward-data), so it is the MFMA A operand read with one ds_read_b128 per fragment; the
// voxel rows are the B operand, 16 contiguous bytes per lane straight from HBM, the next k-step's
// in flight while the current one multiplies.  With the weights in the A slot a lane's accumulator
// holds 4 consecutive output channels of one voxel: 8-byte vector stores, bias added in fp32.
// Workgroup: 4 waves x 16 voxels x 64 outputs; grid: voxel tiles x 64-output tiles.
#include "engines.h"

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int RG_M = 64;   // voxels per workgroup (4 waves x 16)
constexpr int RG_N = 64;   // outputs per workgroup (4 MFMA tiles)
constexpr int RG_KMAX = 1024;

struct RgArgs {
    int64_t nrows;
    int K, N, KS, pitch;  // reduction length, outputs, 32-wide k-steps, LDS row pitch (elements)
    int64_t ldx, ldw, ldy;
};

template <bool TW>
__global__ __launch_bounds__(256) void k_rows_gemm(RgArgs a, const h16_t *__restrict__ x, const h16_t *__restrict__ w,
                                                  const float *__restrict__ bias, h16_t *__restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *ws = reinterpret_cast<h16_t *>(smem);  // [RG_N][pitch]: W'[n0 + r][k]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, kb = lane >> 4;
    const int n0 = int(blockIdx.y) * RG_N;
    const int kc = a.K / 8;  // 16-byte chunks per W' row
    // the row tails K .. pitch - 1 meet the zero B chunks of the last k-step's lanes past K: they
    // must be finite (zero), not whatever the previous kernel left in LDS
    for (int i = tid; i < RG_N * (a.pitch - a.K); i += 256) {
        const int r = i / (a.pitch - a.K), c = i - r * (a.pitch - a.K);
        ws[r * a.pitch + a.K + c] = 0;
    }
    if constexpr (!TW) {
        // W'[n][k] = w[n][k]: 16-byte chunks of the rows
        for (int i = tid; i < RG_N * kc; i += 256) {
            const int r = i / kc, c = i - r * kc;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (n0 + r < a.N) v = *reinterpret_cast<const u32x4 *>(w + int64_t(n0 + r) * a.ldw + 8 * c);
            *reinterpret_cast<u32x4 *>(ws + r * a.pitch + 8 * c) = v;
        }
    } else {
        // W'[n][k] = w[k][n]: 16-byte chunks of w's rows (8 outputs of one k) scattered to 8 LDS rows
        for (int i = tid; i < (RG_N / 8) * a.K; i += 256) {
            const int k = i / (RG_N / 8), c = i - k * (RG_N / 8);
            u32x4 v = {0u, 0u, 0u, 0u};
            if (n0 + 8 * c < a.N) v = *reinterpret_cast<const u32x4 *>(w + int64_t(k) * a.ldw + n0 + 8 * c);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ws[(8 * c + 2 * j) * a.pitch + k] = h16_t(v[j] & 0xffffu);
                ws[(8 * c + 2 * j + 1) * a.pitch + k] = h16_t(v[j] >> 16);
            }
        }
    }
    __syncthreads();
    const int64_t v0 = int64_t(blockIdx.x) * RG_M + 16 * wave;
    const int64_t vr = min(v0 + col, a.nrows - 1);  // this lane's B row (clamped: masked at the store)
    const h16_t *xr = x + vr * a.ldx + 8 * kb;
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto ldb = [&](int ks) -> u32x4 {
        const int k0 = 32 * ks + 8 * kb;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (k0 < a.K) v = *reinterpret_cast<const u32x4 *>(xr + 32 * ks);
        return v;
    };
    u32x4 b0 = ldb(0), b1 = a.KS > 1 ? ldb(1) : u32x4{0u, 0u, 0u, 0u};
    for (int ks = 0; ks < a.KS; ks += 2) {
        // k-steps ks, ks + 1 with ks + 2, ks + 3 in flight
        const u32x4 c0 = b0, c1 = b1;
        if (ks + 2 < a.KS) b0 = ldb(ks + 2);
        if (ks + 3 < a.KS) b1 = ldb(ks + 3);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (ks + h >= a.KS) break;
            const int k0 = 32 * (ks + h) + 8 * kb;
            const hx8 bf = __builtin_bit_cast(hx8, h ? c1 : c0);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                // k0 >= K: the lane's B chunk is zero and the LDS row tail it meets is zero
                const hx8 af = __builtin_bit_cast(hx8, *reinterpret_cast<const u32x4 *>(ws + (16 * t + col) * a.pitch + k0));
                acc[t] = VQ3D_MFMA_16X16X32(af, bf, acc[t], 0, 0, 0);
            }
        }
    }
    // D[n][v]: lane (col = voxel, kb) holds outputs 16 t + 4 kb .. + 3 of voxel v0 + col
    const int64_t v = v0 + col;
    if (v < a.nrows) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int n = n0 + 16 * t + 4 * kb;
            if (n >= a.N) continue;
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = acc[t][j] + (bias ? bias[n + j] : 0.f);
            *reinterpret_cast<u32x2 *>(y + v * a.ldy + n) =
                u32x2{uint32_t(f2h(o[0])) | (uint32_t(f2h(o[1])) << 16), uint32_t(f2h(o[2])) | (uint32_t(f2h(o[3])) << 16)};
        }
    }
}

}  // namespace

int launch_rows_gemm(int64_t nrows, int k, int n, const void *x, int64_t ldx, const void *w, int64_t ldw, int trans_w,
                     const float *bias, void *y, int64_t ldy, hipStream_t s) {
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (nrows < 1 || k < 8 || n < 8 || k % 8 || n % 8 || ldx % 8 || ldw % 8 || ldy % 4 || k > RG_KMAX)
        return fail("rows_gemm: k, n and the row strides must be multiples of 8 (k <= 1024)");
    if (ldx < k || ldy < n || ldw < (trans_w ? n : k)) return fail("rows_gemm: row strides shorter than the rows");
    if (!x || !w || !y || !al(x) || !al(w) || (reinterpret_cast<uintptr_t>(y) & 7))
        return fail("rows_gemm: x / w must be 16-byte aligned, y 8-byte aligned");
    if (nrows > (int64_t(1) << 31) - RG_M) return fail("rows_gemm: too many rows");
    RgArgs a;
    a.nrows = nrows;
    a.K = k;
    a.N = n;
    a.KS = (k + 31) / 32;
    a.pitch = 32 * a.KS + 8;  // every k-step's fragment inside the row; +8: rows off the bank period
    a.ldx = ldx;
    a.ldw = ldw;
    a.ldy = ldy;
    const size_t lds = size_t(RG_N) * a.pitch * sizeof(h16_t);
    const dim3 grid{unsigned((nrows + RG_M - 1) / RG_M), unsigned((n + RG_N - 1) / RG_N), 1u};
    // above 64 KB of dynamic LDS (k > 472) the kernel must opt in (gfx950: 160 KB per workgroup)
    static const bool opt_in = [] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_rows_gemm<true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(RG_N * (RG_KMAX + 8) * 2));
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_rows_gemm<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(RG_N * (RG_KMAX + 8) * 2));
        (void)hipGetLastError();
        return true;
    }();
    (void)opt_in;
    if (trans_w)
        k_rows_gemm<true><<<grid, 256, lds, s>>>(a, (const h16_t *)x, (const h16_t *)w, bias, (h16_t *)y);
    else
        k_rows_gemm<false><<<grid, 256, lds, s>>>(a, (const h16_t *)x, (const h16_t *)w, bias, (h16_t *)y);
    return check_launch("rows_gemm");
}

}  // namespace vq3d
