// Trilinear x2 upsampling, align_corners=False (nn.Upsample inside ResizeConv3D,
// vqvae/layers.py:591-597), forward and adjoint, on channels-last tensors.
//
// Along one axis the destination j reads source floor(j/2 - 1/4) and its upper neighbour with
// weights (0.75, 0.25) or (0.25, 0.75), clamped at the edges (ATen's area_pixel source index).
// Hence source i receives from exactly the four destinations 2i-1 .. 2i+2 with weights
// 0.25, 0.75, 0.75, 0.25 -- the first 0.75 becomes 1 at i = 0 (j = 0 clamps onto it) and the
// second at i = n-1 -- which the adjoint applies in closed form, separably.  A thread owns one
// voxel and CV consecutive channels (8- or 16-byte rows), decomposes its index with 32-bit
// multiplicative division, and the backward fuses the activation derivative, the addend and the
// prologue-scalar partial sums of its consumer conv.
#include "common.h"

#include <algorithm>

// No FP contraction in this file: every kernel here (per-voxel and tiled, bf16 and fp32) then
// evaluates each interpolation with exactly the written multiplies and adds -- ATen's unfused
// arithmetic -- so the tiled kernels give the per-voxel kernels' bits (explicit fmaf stay fused).
#pragma clang fp contract(off)

namespace vq3d {

namespace {

template <typename T, int CV>
__device__ __forceinline__ void ldv(const T *__restrict__ p, float (&o)[CV]) {
    if constexpr (sizeof(T) == 2 && CV == 4) {
        const uint2 u = *reinterpret_cast<const uint2 *>(p);
        o[0] = h2f_lo(u.x);
        o[1] = h2f_hi(u.x);
        o[2] = h2f_lo(u.y);
        o[3] = h2f_hi(u.y);
    } else if constexpr (sizeof(T) == 2 && CV == 8) {
        const uint4 u = *reinterpret_cast<const uint4 *>(p);
        const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            o[2 * j] = h2f_lo(w4[j]);
            o[2 * j + 1] = h2f_hi(w4[j]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < CV; ++j) o[j] = ld(p + j);
    }
}

template <typename T, int CV>
__device__ __forceinline__ void stv(T *__restrict__ p, const float (&v)[CV]) {
    if constexpr (sizeof(T) == 2 && CV == 4) {
        *reinterpret_cast<uint2 *>(p) = uint2{uint32_t(f2h(v[0])) | (uint32_t(f2h(v[1])) << 16),
                                              uint32_t(f2h(v[2])) | (uint32_t(f2h(v[3])) << 16)};
    } else if constexpr (sizeof(T) == 2 && CV == 8) {
        uint32_t q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = uint32_t(f2h(v[2 * j])) | (uint32_t(f2h(v[2 * j + 1])) << 16);
        *reinterpret_cast<uint4 *>(p) = uint4{q[0], q[1], q[2], q[3]};
    } else {
#pragma unroll
        for (int j = 0; j < CV; ++j) st(p + j, v[j]);
    }
}

struct UArgs {
    int B, C, H, W, D;  // source grid (destination is 2H x 2W x 2D)
    int nchunk;         // C / CV
    FastDiv fch, f1, f2, f3;
};

// decompose e = (((b * n3 + i3) * n2 + i2) * n1 + i1) * nchunk + ch
__device__ __forceinline__ void split(const UArgs &a, uint32_t e, int n1, int n2, int n3, int &ch, int &i1, int &i2,
                                      int &i3, int &b) {
    uint32_t q = a.fch.div(e);
    ch = int(e - q * uint32_t(a.nchunk));
    uint32_t r = a.f1.div(q);
    i1 = int(q - r * uint32_t(n1));
    q = a.f2.div(r);
    i2 = int(r - q * uint32_t(n2));
    r = a.f3.div(q);
    i3 = int(q - r * uint32_t(n3));
    b = int(r);
}

// destination j -> (source i0, i1, weight of i1)
__device__ __forceinline__ void src_of(int j, int n, int &i0, int &i1, float &l1) { up_coeff(j, n, i0, i1, l1); }

template <typename T, int CV>
__global__ __launch_bounds__(256) void k_up2_fwd(UArgs a, const T *__restrict__ x, int pk, const float *pa,
                                                const float *pb, T *__restrict__ y) {
    const Prologue pro = make_prologue(pk, pa, pb);
    const uint32_t n = uint32_t(a.B) * 8u * a.H * a.W * a.D * a.nchunk;
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        int ch, od, ow, oh, b;
        split(a, e, 2 * a.D, 2 * a.W, 2 * a.H, ch, od, ow, oh, b);
        int h0, h1, w0, w1, d0, d1;
        float lh, lw, ldd;
        src_of(oh, a.H, h0, h1, lh);
        src_of(ow, a.W, w0, w1, lw);
        src_of(od, a.D, d0, d1, ldd);
        float v[8][CV];
        const int hs[2] = {h0, h1}, wsx[2] = {w0, w1}, ds[2] = {d0, d1};
#pragma unroll
        for (int q = 0; q < 8; ++q)
            ldv<T, CV>(x + (((int64_t(b) * a.H + hs[q >> 2]) * a.W + wsx[(q >> 1) & 1]) * a.D + ds[q & 1]) * a.C +
                           ch * CV,
                       v[q]);
        float out[CV];
#pragma unroll
        for (int c = 0; c < CV; ++c) {
            float X[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) X[q] = pro.apply(v[q][c]);
            out[c] = (1.f - lh) * ((1.f - lw) * ((1.f - ldd) * X[0] + ldd * X[1]) + lw * ((1.f - ldd) * X[2] + ldd * X[3])) +
                     lh * ((1.f - lw) * ((1.f - ldd) * X[4] + ldd * X[5]) + lw * ((1.f - ldd) * X[6] + ldd * X[7]));
        }
        const int64_t vo = ((int64_t(b) * 2 * a.H + oh) * 2 * a.W + ow) * 2 * a.D + od;
        stv<T, CV>(y + vo * a.C + ch * CV, out);
    }
}

// the four destinations of source i along an axis of source length n, with their weights
__device__ __forceinline__ void adj4(int i, int n, int (&j)[4], float (&wt)[4]) {
    j[0] = 2 * i - 1;
    wt[0] = i >= 1 ? 0.25f : 0.f;
    j[1] = 2 * i;
    wt[1] = i == 0 ? 1.f : 0.75f;
    j[2] = 2 * i + 1;
    wt[2] = i == n - 1 ? 1.f : 0.75f;
    j[3] = 2 * i + 2;
    wt[3] = i <= n - 2 ? 0.25f : 0.f;
    if (j[0] < 0) j[0] = 0;          // weight 0: any valid index
    if (j[3] > 2 * n - 1) j[3] = 2 * n - 1;
}

template <typename T, int CV>
__global__ __launch_bounds__(256) void k_up2_bwd(UArgs a, const T *__restrict__ gy, int dmode, const float *dparam,
                                                const T *__restrict__ aux, const T *__restrict__ addend,
                                                T *__restrict__ gx, float *dpre, float *dpost, GridSum gsum) {
    __shared__ float red[8];
    ActDeriv dv;
    dv.mode = aux ? dmode : 0;
    dv.p = (dv.mode && dparam) ? *dparam : 0.f;
    float pre = 0.f, post = 0.f;
    const uint32_t n = uint32_t(a.B) * a.H * a.W * a.D * a.nchunk;
    const int D2 = 2 * a.D, W2 = 2 * a.W, H2 = 2 * a.H;
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        int ch, id, iw, ih, b;
        split(a, e, a.D, a.W, a.H, ch, id, iw, ih, b);
        int jh[4], jw[4], jd[4];
        float wh[4], ww[4], wd[4];
        adj4(ih, a.H, jh, wh);
        adj4(iw, a.W, jw, ww);
        adj4(id, a.D, jd, wd);
        float acc[CV];
#pragma unroll
        for (int c = 0; c < CV; ++c) acc[c] = 0.f;
#pragma unroll
        for (int x0 = 0; x0 < 4; ++x0)
#pragma unroll
            for (int x1 = 0; x1 < 4; ++x1) {
                const float whw = wh[x0] * ww[x1];
                const int64_t rowb = ((int64_t(b) * H2 + jh[x0]) * W2 + jw[x1]) * D2;
                float r[4][CV];
#pragma unroll
                for (int x2 = 0; x2 < 4; ++x2) ldv<T, CV>(gy + (rowb + jd[x2]) * a.C + ch * CV, r[x2]);
#pragma unroll
                for (int c = 0; c < CV; ++c) {
                    const float sd = wd[0] * r[0][c] + wd[1] * r[1][c] + wd[2] * r[2][c] + wd[3] * r[3][c];
                    acc[c] = fmaf(whw, sd, acc[c]);
                }
            }
        const int64_t o = (((int64_t(b) * a.H + ih) * a.W + iw) * a.D + id) * a.C + ch * CV;
        float xa[CV], ad[CV];
        if (dv.mode) ldv<T, CV>(aux + o, xa);
        if (addend) ldv<T, CV>(addend + o, ad);
#pragma unroll
        for (int c = 0; c < CV; ++c) {
            float v = acc[c];
            pre += v;
            if (dv.mode) v *= dv(xa[c]);
            post += v;
            if (addend) v += ad[c];
            acc[c] = v;
        }
        stv<T, CV>(gx + o, acc);
    }
    if (dpre || dpost) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        grid_sum2<256>(gsum, pre, post, dpre, dpost, red);
    }
}

// 4 bf16 channels, D % 4 == 0: a thread owns a run of 4 source voxels along D.  Their destination
// rows 2 i0 - 1 .. 2 i0 + 8 of each (h, w) pair lie in one 96-byte window (destinations
// 2 i0 - 2 .. 2 i0 + 9, six 16-byte loads; the ends past the grid carry weight 0 and are zero
// here) instead of 16 separate 8-byte loads.  Same weights, same order of operations as k_up2_bwd,
// so the same bits.
__global__ __launch_bounds__(256) void k_up2_bwd_run4(UArgs a, const h16_t *__restrict__ gy, int dmode,
                                                     const float *dparam, const h16_t *__restrict__ aux,
                                                     const h16_t *__restrict__ addend, h16_t *__restrict__ gx,
                                                     float *dpre, float *dpost, GridSum gsum) {
    __shared__ float red[8];
    ActDeriv dv;
    dv.mode = aux ? dmode : 0;
    dv.p = (dv.mode && dparam) ? *dparam : 0.f;
    float pre = 0.f, post = 0.f;
    const int DQ = a.D / 4;
    const uint32_t n = uint32_t(a.B) * a.H * a.W * DQ;
    const int D2 = 2 * a.D, W2 = 2 * a.W, H2 = 2 * a.H;
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        int ch, q, iw, ih, b;
        split(a, e, DQ, a.W, a.H, ch, q, iw, ih, b);
        const int i0 = 4 * q;
        int jh[4], jw[4], jd[4];
        float wh[4], ww[4], wd[4][4];
        adj4(ih, a.H, jh, wh);
        adj4(iw, a.W, jw, ww);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) adj4(i0 + s4, a.D, jd, wd[s4]);
        float acc[4][4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[s4][c] = 0.f;
        // one h row of windows in flight (24 loads; all 96 would cap the occupancy at one wave,
        // 2 x 6 measured slower)
#pragma unroll 1
        for (int x0 = 0; x0 < 4; ++x0)
#pragma unroll 4
            for (int x1 = 0; x1 < 4; ++x1) {
                const float whw = wh[x0] * ww[x1];
                const int64_t rowb = ((int64_t(b) * H2 + jh[x0]) * W2 + jw[x1]) * D2;
                // destinations 2 i0 - 2 + k, k = 0 .. 11, 4 channels each
                float r[12][4];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const int j = 2 * i0 - 2 + 2 * k;
                    u32x4 u = u32x4{0u, 0u, 0u, 0u};
                    if (j >= 0 && j < D2) u = *reinterpret_cast<const u32x4 *>(gy + (rowb + j) * 4);
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2) {
                        r[2 * k + h2][0] = h2f_lo(u[2 * h2]);
                        r[2 * k + h2][1] = h2f_hi(u[2 * h2]);
                        r[2 * k + h2][2] = h2f_lo(u[2 * h2 + 1]);
                        r[2 * k + h2][3] = h2f_hi(u[2 * h2 + 1]);
                    }
                }
                // source i0 + s4 reads destinations 2 (i0 + s4) - 1 + t = window slot 2 s4 + 1 + t
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float *w4 = wd[s4];
                        const float sd = w4[0] * r[2 * s4 + 1][c] + w4[1] * r[2 * s4 + 2][c] + w4[2] * r[2 * s4 + 3][c] +
                                         w4[3] * r[2 * s4 + 4][c];
                        acc[s4][c] = fmaf(whw, sd, acc[s4][c]);
                    }
            }
        const int64_t o = (((int64_t(b) * a.H + ih) * a.W + iw) * a.D + i0) * 4;
        u32x4 xa[2] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}}, ad[2] = {xa[0], xa[1]};
        if (dv.mode) xa[0] = *reinterpret_cast<const u32x4 *>(aux + o), xa[1] = *reinterpret_cast<const u32x4 *>(aux + o + 8);
        if (addend) ad[0] = *reinterpret_cast<const u32x4 *>(addend + o), ad[1] = *reinterpret_cast<const u32x4 *>(addend + o + 8);
        u32x4 res[2];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            float v2[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint32_t wx = xa[s4 >> 1][2 * (s4 & 1) + (c >> 1)], wa = ad[s4 >> 1][2 * (s4 & 1) + (c >> 1)];
                const float xv = ((c & 1) ? h2f_hi(wx) : h2f_lo(wx));
                const float av = ((c & 1) ? h2f_hi(wa) : h2f_lo(wa));
                float v = acc[s4][c];
                pre += v;
                if (dv.mode) v *= dv(xv);
                post += v;
                if (addend) v += av;
                v2[c] = v;
            }
            res[s4 >> 1][2 * (s4 & 1)] = uint32_t(f2h(v2[0])) | (uint32_t(f2h(v2[1])) << 16);
            res[s4 >> 1][2 * (s4 & 1) + 1] = uint32_t(f2h(v2[2])) | (uint32_t(f2h(v2[3])) << 16);
        }
        *reinterpret_cast<u32x4 *>(gx + o) = res[0];
        *reinterpret_cast<u32x4 *>(gx + o + 8) = res[1];
    }
    if (dpre || dpost) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        grid_sum2<256>(gsum, pre, post, dpre, dpost, red);
    }
}

// The same adjoint with a thread owning 2 x 2 source lines (h, h + 1) x (w, w + 1) of 4 voxels along D
// (even H and W): the four lines' destination rows are the 6 x 6 (h, w) rows 2 h - 1 .. 2 h + 4 x
// 2 w - 1 .. 2 w + 4, each 96-byte D window loaded and reduced along D ONCE for all four lines
// (216 16-byte loads for 16 source voxels instead of 384).  Each line accumulates its 4 x 4 rows
// in run4's order (h row outer, w row inner; weight-0 clamped rows included), so the same bits.
__global__ __launch_bounds__(256) void k_up2_bwd_quad(UArgs a, const h16_t *__restrict__ gy, int dmode,
                                                     const float *dparam, const h16_t *__restrict__ aux,
                                                     const h16_t *__restrict__ addend, h16_t *__restrict__ gx,
                                                     float *dpre, float *dpost, GridSum gsum) {
    __shared__ float red[8];
    ActDeriv dv;
    dv.mode = aux ? dmode : 0;
    dv.p = (dv.mode && dparam) ? *dparam : 0.f;
    float pre = 0.f, post = 0.f;
    const int DQ = a.D / 4, HQ = a.H / 2, WQ = a.W / 2;
    const uint32_t n = uint32_t(a.B) * HQ * WQ * DQ;
    const int D2 = 2 * a.D, W2 = 2 * a.W, H2 = 2 * a.H;
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < n; e += gridDim.x * 256u) {
        int ch, q, iwq, ihq, b;
        split(a, e, DQ, WQ, HQ, ch, q, iwq, ihq, b);
        const int i0 = 4 * q, ih0 = 2 * ihq, iw0 = 2 * iwq;
        int jh[2][4], jw[2][4], jd[4];
        float wh[2][4], ww[2][4], wd[4][4];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            adj4(ih0 + r, a.H, jh[r], wh[r]);
            adj4(iw0 + r, a.W, jw[r], ww[r]);
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) adj4(i0 + s4, a.D, jd, wd[s4]);
        // the 6 destination rows per axis: slot x of line r is row index x + 2 r (adj4's clamped rows)
        int rowh[6], roww[6];
#pragma unroll
        for (int x = 0; x < 6; ++x) {
            rowh[x] = x < 4 ? jh[0][x] : jh[1][x - 2];
            roww[x] = x < 4 ? jw[0][x] : jw[1][x - 2];
        }
        float acc[2][2][4][4];
#pragma unroll
        for (int rh = 0; rh < 2; ++rh)
#pragma unroll
            for (int rw = 0; rw < 2; ++rw)
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[rh][rw][s4][c] = 0.f;
#pragma unroll 1
        for (int xh = 0; xh < 6; ++xh)
#pragma unroll 2
            for (int xw = 0; xw < 6; ++xw) {
                const int64_t rowb = ((int64_t(b) * H2 + rowh[xh]) * W2 + roww[xw]) * D2;
                float r[12][4];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const int j = 2 * i0 - 2 + 2 * k;
                    u32x4 u = u32x4{0u, 0u, 0u, 0u};
                    if (j >= 0 && j < D2) u = *reinterpret_cast<const u32x4 *>(gy + (rowb + j) * 4);
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2) {
                        r[2 * k + h2][0] = h2f_lo(u[2 * h2]);
                        r[2 * k + h2][1] = h2f_hi(u[2 * h2]);
                        r[2 * k + h2][2] = h2f_lo(u[2 * h2 + 1]);
                        r[2 * k + h2][3] = h2f_hi(u[2 * h2 + 1]);
                    }
                }
                float sd[4][4];
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const float *w4 = wd[s4];
                        sd[s4][c] = w4[0] * r[2 * s4 + 1][c] + w4[1] * r[2 * s4 + 2][c] + w4[2] * r[2 * s4 + 3][c] +
                                    w4[3] * r[2 * s4 + 4][c];
                    }
#pragma unroll
                for (int rh = 0; rh < 2; ++rh) {
                    const int x0 = xh - 2 * rh;
                    if (x0 < 0 || x0 > 3) continue;
#pragma unroll
                    for (int rw = 0; rw < 2; ++rw) {
                        const int x1 = xw - 2 * rw;
                        if (x1 < 0 || x1 > 3) continue;
                        const float whw = wh[rh][x0] * ww[rw][x1];
#pragma unroll
                        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                            for (int c = 0; c < 4; ++c) acc[rh][rw][s4][c] = fmaf(whw, sd[s4][c], acc[rh][rw][s4][c]);
                    }
                }
            }
#pragma unroll
        for (int rh = 0; rh < 2; ++rh)
#pragma unroll
            for (int rw = 0; rw < 2; ++rw) {
                const int64_t o = (((int64_t(b) * a.H + ih0 + rh) * a.W + iw0 + rw) * a.D + i0) * 4;
                u32x4 xa[2] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}}, ad[2] = {xa[0], xa[1]};
                if (dv.mode) xa[0] = *reinterpret_cast<const u32x4 *>(aux + o), xa[1] = *reinterpret_cast<const u32x4 *>(aux + o + 8);
                if (addend) ad[0] = *reinterpret_cast<const u32x4 *>(addend + o), ad[1] = *reinterpret_cast<const u32x4 *>(addend + o + 8);
                u32x4 res[2];
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) {
                    float v2[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const uint32_t wx = xa[s4 >> 1][2 * (s4 & 1) + (c >> 1)], wa = ad[s4 >> 1][2 * (s4 & 1) + (c >> 1)];
                        const float xv = ((c & 1) ? h2f_hi(wx) : h2f_lo(wx));
                        const float av = ((c & 1) ? h2f_hi(wa) : h2f_lo(wa));
                        float v = acc[rh][rw][s4][c];
                        pre += v;
                        if (dv.mode) v *= dv(xv);
                        post += v;
                        if (addend) v += av;
                        v2[c] = v;
                    }
                    res[s4 >> 1][2 * (s4 & 1)] = uint32_t(f2h(v2[0])) | (uint32_t(f2h(v2[1])) << 16);
                    res[s4 >> 1][2 * (s4 & 1) + 1] = uint32_t(f2h(v2[2])) | (uint32_t(f2h(v2[3])) << 16);
                }
                *reinterpret_cast<u32x4 *>(gx + o) = res[0];
                *reinterpret_cast<u32x4 *>(gx + o + 8) = res[1];
            }
    }
    if (dpre || dpost) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        grid_sum2<256>(gsum, pre, post, dpre, dpost, red);
    }
}

// ---------------------------------------------------------------------------------- LDS-tiled (bf16)
// A workgroup owns a SH x SW x SD brick of SOURCE voxels (all C channels) and writes its 8 x larger
// destination brick from the source brick + a one-voxel halo staged in LDS (each destination voxel
// 8 LDS reads instead of 8 scattered global loads).  Indices along every axis follow a fixed
// pattern in the tile (destination 2i + a reads source rows i - 1 + a, i + a) with the staged halo
// holding clamped copies at the grid's edges, where the weights (up_coeff) are exactly those of
// the per-voxel kernel: the arithmetic, and so every bit of the result, is its.
struct UT {
    int B, H, W, D;       // source grid
    int nth, ntw, ntd;    // bricks per axis
    int pro_kind;
    const float *pro_a, *pro_b;
};

// C consecutive bf16 at LDS element offset e (8-byte reads when C % 4 == 0) as fp32
template <int C>
__device__ __forceinline__ void lds_vox(const h16_t *s, int e, float (&o)[C]) {
    if constexpr (C % 4 == 0) {
#pragma unroll
        for (int j = 0; j < C / 4; ++j) {
            const u32x2 u = *reinterpret_cast<const u32x2 *>(s + e + 4 * j);
            o[4 * j] = h2f_lo(u[0]);
            o[4 * j + 1] = h2f_hi(u[0]);
            o[4 * j + 2] = h2f_lo(u[1]);
            o[4 * j + 3] = h2f_hi(u[1]);
        }
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) o[c] = h2f_lo(uint32_t(s[e + c]));
    }
}

// stage a (LH x LW x LD) box of a channels-last bf16 grid (n = H x W x D, rows clamped into it)
// whose first voxel is (h0, w0, d0) into LDS [LH][LW][LD][C]: 8-byte units when C % 4 == 0
template <int C, int LH, int LW, int LD>
__device__ __forceinline__ void stage_box(const h16_t *__restrict__ src, int b, int H, int W, int D, int h0, int w0,
                                          int d0, h16_t *s) {
    constexpr int U = C % 4 == 0 ? 4 : 1, NU = LH * LW * LD * C / U;
    for (int u = threadIdx.x; u < NU; u += 256) {
        const int e = u * U, v = e / C, c = e - v * C;
        const int ld_ = v % LD, lw_ = (v / LD) % LW, lh_ = v / (LD * LW);
        const int h = min(max(h0 + lh_, 0), H - 1), w = min(max(w0 + lw_, 0), W - 1), d = min(max(d0 + ld_, 0), D - 1);
        const int64_t g = (((int64_t(b) * H + h) * W + w) * D + d) * C + c;
        if constexpr (U == 4) *reinterpret_cast<u32x2 *>(s + e) = *reinterpret_cast<const u32x2 *>(src + g);
        else s[e] = src[g];
    }
}

template <int C, int SH, int SW, int SD>
__global__ __launch_bounds__(256) void k_up2t_fwd(UT a, const h16_t *__restrict__ x, h16_t *__restrict__ y) {
    constexpr int HH = SH + 2, HW = SW + 2, HD = SD + 2;
    constexpr int CG = C % 4 == 0 ? 4 : 1;  // channels per LDS read
    __shared__ __attribute__((aligned(16))) h16_t hs[HH * HW * HD * C];
    int t = blockIdx.x;
    const int td = t % a.ntd;
    t /= a.ntd;
    const int tw = t % a.ntw;
    t /= a.ntw;
    const int th = t % a.nth, b = t / a.nth;
    const int sh0 = th * SH, sw0 = tw * SW, sd0 = td * SD;
    stage_box<C, HH, HW, HD>(x, b, a.H, a.W, a.D, sh0 - 1, sw0 - 1, sd0 - 1, hs);
    __syncthreads();
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    // item = (destination line (oh, ow) of the brick, quad q of 4 destination voxels along D)
    constexpr int NQ = SD / 2, NITEM = 4 * SH * SW * NQ;
    for (int it = threadIdx.x; it < NITEM; it += 256) {
        const int q = it % NQ, line = it / NQ, ow = line % (2 * SW), oh = line / (2 * SW);
        const int r = oh >> 1, ah = oh & 1, cw = ow >> 1, aw = ow & 1;
        int i0, i1;
        float lh, lw;
        up_coeff(2 * (sh0 + r) + ah, a.H, i0, i1, lh);
        up_coeff(2 * (sw0 + cw) + aw, a.W, i0, i1, lw);
        const int64_t vo = ((int64_t(b) * 2 * a.H + 2 * sh0 + oh) * 2 * a.W + 2 * sw0 + ow) * 2 * a.D + 2 * sd0 + 4 * q;
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
            float ld;
            up_coeff(2 * (sd0 + 2 * q) + tt, a.D, i0, i1, ld);
            const int p0 = 2 * q + ((tt + 1) >> 1), p1 = p0 + 1;  // local positions (0,1) (1,2) (1,2) (2,3) + 2q
            float o[C];
#pragma unroll
            for (int cg = 0; cg < C / CG; ++cg) {
                float X[8][CG];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int lh_ = r + ah + (k >> 2), lw_ = cw + aw + ((k >> 1) & 1), ld_ = (k & 1) ? p1 : p0;
                    lds_vox<CG>(hs, ((lh_ * HW + lw_) * HD + ld_) * C + cg * CG, X[k]);
                }
#pragma unroll
                for (int c = 0; c < CG; ++c) {
                    float v[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = pro.apply(X[k][c]);
                    o[cg * CG + c] = (1.f - lh) * ((1.f - lw) * ((1.f - ld) * v[0] + ld * v[1]) + lw * ((1.f - ld) * v[2] + ld * v[3])) +
                                     lh * ((1.f - lw) * ((1.f - ld) * v[4] + ld * v[5]) + lw * ((1.f - ld) * v[6] + ld * v[7]));
                }
            }
            h16_t *dst = y + (vo + tt) * C;
            if constexpr (C % 8 == 0) {
#pragma unroll
                for (int j = 0; j < C / 8; ++j) {
                    float f[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) f[k] = o[8 * j + k];
                    stvec<h16_t, 8>(dst + 8 * j, f);
                }
            } else if constexpr (C == 4) {
                stvec<h16_t, 4>(dst, o);
            } else {
#pragma unroll
                for (int c = 0; c < C; ++c) st(dst + c, o[c]);
            }
        }
    }
}

// the tiled forward: used where measured faster than the per-voxel kernel (9 channels @128^2 x 32:
// 182 -> 88 us; 4 channels @256^2 x 64: 229 -> 219 us, 16 @64^2 x 16: 17 -> 45 us, not used; a tiled
// adjoint staging the destination gradient was slower for every channel count, 234 -> 324 us at 4)
template <int C, int SH, int SW, int SD>
bool up2_tiled_fwd(int batch, int h, int w, int dd, const void *x, int pro_kind, const float *pa, const float *pb,
                   void *y, hipStream_t s) {
    if (h % SH || w % SW || dd % SD) return false;
    if (int64_t(batch) * 8 * h * w * dd * C >= (int64_t(1) << 31)) return false;
    UT a;
    a.B = batch; a.H = h; a.W = w; a.D = dd;
    a.nth = h / SH; a.ntw = w / SW; a.ntd = dd / SD;
    a.pro_kind = pro_kind; a.pro_a = pa; a.pro_b = pb;
    const unsigned nb = unsigned(batch * a.nth * a.ntw * a.ntd);
    k_up2t_fwd<C, SH, SW, SD><<<nb, 256, 0, s>>>(a, (const h16_t *)x, (h16_t *)y);
    return true;
}

UArgs make_args(int B, int C, int H, int W, int D, int cv, bool fwd) {
    UArgs a;
    a.B = B; a.C = C; a.H = H; a.W = W; a.D = D;
    a.nchunk = C / cv;
    a.fch = FastDiv(uint32_t(a.nchunk));
    const int m = fwd ? 2 : 1;
    a.f1 = FastDiv(uint32_t(m * D));
    a.f2 = FastDiv(uint32_t(m * W));
    a.f3 = FastDiv(uint32_t(m * H));
    return a;
}

int pick_cv(int dtype, int C, const void *p0, const void *p1, const void *p2, const void *p3) {
    auto al = [](const void *p, int b) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % b) == 0; };
    if (dtype != VQ3D_HALF) return 1;
    if (C % 8 == 0 && al(p0, 16) && al(p1, 16) && al(p2, 16) && al(p3, 16)) return 8;
    if (C % 4 == 0 && al(p0, 8) && al(p1, 8) && al(p2, 8) && al(p3, 8)) return 4;
    return 1;
}

}  // namespace

int launch_up2_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd, const void *x,
                   int32_t pro_kind, const float *pro_a, const float *pro_b, void *y, hipStream_t s) {
    if (int64_t(batch) * 8 * h * w * dd * channels >= (int64_t(1) << 31)) return fail("upsample2x: tensor too large");
    if (dtype == VQ3D_HALF && channels == 9 && up2_tiled_fwd<9, 4, 8, 16>(batch, h, w, dd, x, pro_kind, pro_a, pro_b, y, s))
        return check_launch("upsample2x_fwd(tiled)");
    const int cv = pick_cv(dtype, channels, x, y, nullptr, nullptr);
    const UArgs a = make_args(batch, channels, h, w, dd, cv, true);
    const int64_t n = int64_t(batch) * 8 * h * w * dd * a.nchunk;
    const unsigned nb = unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)));
    if (dtype == VQ3D_F32)
        k_up2_fwd<float, 1><<<nb, 256, 0, s>>>(a, (const float *)x, pro_kind, pro_a, pro_b, (float *)y);
    else if (cv == 8)
        k_up2_fwd<h16_t, 8><<<nb, 256, 0, s>>>(a, (const h16_t *)x, pro_kind, pro_a, pro_b, (h16_t *)y);
    else if (cv == 4)
        k_up2_fwd<h16_t, 4><<<nb, 256, 0, s>>>(a, (const h16_t *)x, pro_kind, pro_a, pro_b, (h16_t *)y);
    else
        k_up2_fwd<h16_t, 1><<<nb, 256, 0, s>>>(a, (const h16_t *)x, pro_kind, pro_a, pro_b, (h16_t *)y);
    return check_launch("upsample2x_fwd");
}

int launch_up2_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd, const void *gy,
                   int dmode, const float *dparam, const void *aux, const void *add, void *gx, float *dpre,
                   float *dpost, hipStream_t s) {
    if (int64_t(batch) * 8 * h * w * dd * channels >= (int64_t(1) << 31)) return fail("upsample2x: tensor too large");
    const int cv = pick_cv(dtype, channels, gy, gx, aux, add);
    auto al16 = [](const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    // the run forms give a thread 4 (run4) or 16 (quad) source voxels: only grids that still fill the
    // chip take them (a 2-workgroup quad grid ran 49 us where the per-voxel kernel needs ~10)
    const int64_t nsrc = int64_t(batch) * h * w * dd;
    if (dtype == VQ3D_HALF && channels == 4 && dd % 4 == 0 && h % 2 == 0 && w % 2 == 0 && nsrc >= (int64_t(1) << 22) &&
        al16(gy) && al16(gx) && al16(aux) && al16(add)) {
        UArgs a = make_args(batch, channels, h, w, dd, 4, false);
        a.f1 = FastDiv(uint32_t(dd / 4));
        a.f2 = FastDiv(uint32_t(w / 2));
        a.f3 = FastDiv(uint32_t(h / 2));
        const int64_t n = int64_t(batch) * (h / 2) * (w / 2) * (dd / 4);
        const unsigned nb = unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024)));
        k_up2_bwd_quad<<<nb, 256, 0, s>>>(a, (const h16_t *)gy, dmode, dparam, (const h16_t *)aux,
                                          (const h16_t *)add, (h16_t *)gx, dpre, dpost,
                                          grid_sum_for(s, nb, dpre || dpost));
        return check_launch("upsample2x_bwd(quad)");
    }
    if (dtype == VQ3D_HALF && channels == 4 && dd % 4 == 0 && nsrc >= (int64_t(1) << 20) && al16(gy) && al16(gx) &&
        al16(aux) && al16(add)) {
        UArgs a = make_args(batch, channels, h, w, dd, 4, false);
        a.f1 = FastDiv(uint32_t(dd / 4));
        const int64_t n = int64_t(batch) * h * w * (dd / 4);
        const unsigned nb = unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024)));
        k_up2_bwd_run4<<<nb, 256, 0, s>>>(a, (const h16_t *)gy, dmode, dparam, (const h16_t *)aux,
                                          (const h16_t *)add, (h16_t *)gx, dpre, dpost,
                                          grid_sum_for(s, nb, dpre || dpost));
        return check_launch("upsample2x_bwd(run4)");
    }
    const UArgs a = make_args(batch, channels, h, w, dd, cv, false);
    const int64_t n = int64_t(batch) * h * w * dd * a.nchunk;
    // grid-stride, <= 1,024 workgroups
    const unsigned nb = unsigned(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024)));
#define UB(T, CV)                                                                                             \
    k_up2_bwd<T, CV><<<nb, 256, 0, s>>>(a, (const T *)gy, dmode, dparam, (const T *)aux, (const T *)add, (T *)gx, \
                                        dpre, dpost, grid_sum_for(s, nb, dpre || dpost))
    if (dtype == VQ3D_F32) UB(float, 1);
    else if (cv == 8) UB(h16_t, 8);
    else if (cv == 4) UB(h16_t, 4);
    else UB(h16_t, 1);
#undef UB
    return check_launch("upsample2x_bwd");
}

}  // namespace vq3d
