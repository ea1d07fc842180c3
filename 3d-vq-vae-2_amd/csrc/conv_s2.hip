// Backward-data of the stride-2 convolutions (PreAct down blocks: branch_conv2 4x4x4 stride 2
// circular, skip_conv 2x2x2 stride 2 -- vqvae/layers.py:124-126, 164-171).
//
// gx[i] = sum over taps t with 2o + t - p == i (mod n) of W[t]^T g[o].  Per dimension only the
// taps whose parity matches i + p contribute (k / 2 of them, each with a unique o), so a thread
// owning one input voxel visits (k/2)^3 taps instead of k^3, reading each contributing g row
// once; the weights of all taps sit in LDS.  The backward-data epilogue (activation derivative
// from aux, addend, prologue-scalar partial sums, split into gx / gx2) is fused.  VALU fp32: the
// stride-2 layers carry few channels on large grids (4..16 at 512^2..128^2) or few voxels.
#include "engines.h"


#include <algorithm>
#include <type_traits>

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct S2Args {
    int B, Cin1, Cin2, Cin, Cout;
    int iH, iW, iD, oH, oW, oD;
    int k, p, circ;
    FastDiv fD, fW, fH;  // 32-bit voxel index decomposition (no 64-bit divides in the loop)
    int rows;            // one input of exactly COT channels, 16-B aligned rows: vector epilogue
};

// the <= 2 (o, t) pairs of one dimension for input coordinate i (k in {2, 4}, stride 2)
__device__ __forceinline__ int taps_s2(int i, int k, int p, int n_in, int n_out, int circ, int (&o)[2], int (&t)[2]) {
    int cnt = 0;
    const int t0 = (i + p) & 1;  // taps with (i + p - t) even
    for (int tt = t0; tt < k; tt += 2) {
        int r = i + p - tt;
        if (circ) {
            r = r < 0 ? r + n_in : (r >= n_in ? r - n_in : r);
        } else if (r < 0) {
            continue;
        }
        r >>= 1;
        if (r >= n_out) continue;
        o[cnt] = r;
        t[cnt] = tt;
        ++cnt;
    }
    return cnt;
}

template <typename T, int N>
__device__ __forceinline__ void load_row(const T *__restrict__ p, float (&o)[N]) {
    if constexpr (sizeof(T) == 2 && (N % 8) == 0) {
#pragma unroll
        for (int q = 0; q < N / 8; ++q) {
            const uint4 u = reinterpret_cast<const uint4 *>(p)[q];
            const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[8 * q + 2 * j] = h2f_lo(w4[j]);
                o[8 * q + 2 * j + 1] = h2f_hi(w4[j]);
            }
        }
    } else if constexpr (sizeof(T) == 2 && N == 4) {
        const uint2 u = *reinterpret_cast<const uint2 *>(p);
        o[0] = h2f_lo(u.x);
        o[1] = h2f_hi(u.x);
        o[2] = h2f_lo(u.y);
        o[3] = h2f_hi(u.y);
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) o[j] = ld(p + j);
    }
}

template <typename T, int N>
__device__ __forceinline__ void store_row(T *__restrict__ p, const float (&v)[N]) {
    if constexpr (sizeof(T) == 2 && (N % 8) == 0) {
#pragma unroll
        for (int q = 0; q < N / 8; ++q) {
            uint32_t u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) u[j] = uint32_t(f2h(v[8 * q + 2 * j])) | (uint32_t(f2h(v[8 * q + 2 * j + 1])) << 16);
            reinterpret_cast<uint4 *>(p)[q] = uint4{u[0], u[1], u[2], u[3]};
        }
    } else {
#pragma unroll
        for (int j = 0; j < N; ++j) st(p + j, v[j]);
    }
}

// CO: g channels (conv Cout) when a compile-time row is used (0: runtime loop)
template <typename T, int COT, int CO>
__global__ __launch_bounds__(256) void k_dgrad_s2(S2Args a, const T *__restrict__ g, const float *__restrict__ gscale,
                                                 const float *__restrict__ w, BwdEpi<T> be, T *__restrict__ gx,
                                                 T *__restrict__ gx2, float *dpre, float *dpost, GridSum gsum) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];  // [tap][Cout][COT]
    __shared__ float red[8];
    const int K3 = a.k * a.k * a.k;
    const int c0 = blockIdx.y * COT;
    for (int e = threadIdx.x; e < K3 * a.Cout * COT; e += 256) {
        const int c = e % COT, r = e / COT, co = r % a.Cout, tap = r / a.Cout;
        const int ci = c0 + c;
        wsh[e] = ci < a.Cin ? w[(int64_t(co) * a.Cin + ci) * K3 + tap] : 0.f;
    }
    __syncthreads();
    ActDeriv dv;
    dv.mode = be.aux ? be.mode : 0;
    dv.p = (dv.mode && be.p) ? *be.p : 0.f;
    const float gs = gscale ? *gscale : 1.f;
    float pre = 0.f, post = 0.f;
    const int64_t nvox = int64_t(a.B) * a.iH * a.iW * a.iD;
    for (int64_t v = int64_t(blockIdx.x) * 256 + threadIdx.x; v < nvox; v += int64_t(gridDim.x) * 256) {
        uint32_t q = uint32_t(v);
        uint32_t q2 = a.fD.div(q);
        const int id = int(q - q2 * uint32_t(a.iD));
        q = a.fW.div(q2);
        const int iw = int(q2 - q * uint32_t(a.iW));
        q2 = a.fH.div(q);
        const int ih = int(q - q2 * uint32_t(a.iH));
        const int b = int(q2);
        int oh[2], th[2], ow[2], tw[2], od[2], td[2];
        const int nh = taps_s2(ih, a.k, a.p, a.iH, a.oH, a.circ, oh, th);
        const int nw = taps_s2(iw, a.k, a.p, a.iW, a.oW, a.circ, ow, tw);
        const int nd = taps_s2(id, a.k, a.p, a.iD, a.oD, a.circ, od, td);
        float acc[COT];
#pragma unroll
        for (int c = 0; c < COT; ++c) acc[c] = 0.f;
        if constexpr (CO > 0) {
            // all contributing g rows loaded first (up to 8 x CO values in flight)
            float gr[8][CO];
            int wt[8];
            int cnt = 0;
#pragma unroll
            for (int xh = 0; xh < 2; ++xh)
#pragma unroll
                for (int xw = 0; xw < 2; ++xw)
#pragma unroll
                    for (int xd = 0; xd < 2; ++xd) {
                        const int j = (xh * 2 + xw) * 2 + xd;
                        const bool live = xh < nh && xw < nw && xd < nd;
                        if (live) {
                            load_row<T, CO>(g + (((int64_t(b) * a.oH + oh[xh]) * a.oW + ow[xw]) * a.oD + od[xd]) * CO,
                                            gr[j]);
                            wt[j] = ((th[xh] * a.k + tw[xw]) * a.k + td[xd]) * CO * COT;
                        } else {
                            wt[j] = -1;
                        }
                    }
            (void)cnt;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (wt[j] < 0) continue;
                const float *wr = wsh + wt[j];
#pragma unroll
                for (int co = 0; co < CO; ++co)
#pragma unroll
                    for (int c = 0; c < COT; ++c) acc[c] = fmaf(gr[j][co], wr[co * COT + c], acc[c]);
            }
        } else {
            for (int xh = 0; xh < nh; ++xh)
                for (int xw = 0; xw < nw; ++xw)
                    for (int xd = 0; xd < nd; ++xd) {
                        const T *grp = g + (((int64_t(b) * a.oH + oh[xh]) * a.oW + ow[xw]) * a.oD + od[xd]) * a.Cout;
                        const float *wr = wsh + ((th[xh] * a.k + tw[xw]) * a.k + td[xd]) * a.Cout * COT;
                        for (int co = 0; co < a.Cout; ++co) {
                            const float gv = ld(grp + co);
#pragma unroll
                            for (int c = 0; c < COT; ++c) acc[c] = fmaf(gv, wr[co * COT + c], acc[c]);
                        }
                    }
        }
        if constexpr (sizeof(T) == 2 && (COT == 4 || COT == 8)) {
            if (a.rows) {  // all Cin (== COT) channels of one input: whole-row loads / stores
                float aux[COT], add[COT], o[COT];
                if (dv.mode) load_row<T, COT>(be.aux + v * COT, aux);
                if (be.addend) load_row<T, COT>(be.addend + v * COT, add);
#pragma unroll
                for (int c = 0; c < COT; ++c) {
                    float val = acc[c];
                    if (gscale) val = val * gs;
                    pre += val;
                    if (dv.mode) val = val * dv(aux[c]);
                    post += val;
                    if (be.addend) val = val + add[c];
                    o[c] = val;
                }
                uint32_t qv[COT / 2];
#pragma unroll
                for (int j = 0; j < COT / 2; ++j) qv[j] = uint32_t(f2h(o[2 * j])) | (uint32_t(f2h(o[2 * j + 1])) << 16);
                if constexpr (COT == 4) *reinterpret_cast<uint2 *>(gx + v * COT) = uint2{qv[0], qv[1]};
                else *reinterpret_cast<uint4 *>(gx + v * COT) = uint4{qv[0], qv[1], qv[2], qv[3]};
                continue;
            }
        }
#pragma unroll
        for (int c = 0; c < COT; ++c) {
            const int ci = c0 + c;
            if (ci >= a.Cin) break;
            float val = acc[c];
            if (gscale) val = val * gs;
            if (ci < a.Cin1) {
                const int64_t o = v * a.Cin1 + ci;
                pre += val;
                if (dv.mode) val = val * dv(ld(be.aux + o));
                post += val;
                if (be.addend) val = val + ld(be.addend + o);
                st(gx + o, val);
            } else {
                st(gx2 + v * a.Cin2 + (ci - a.Cin1), val);
            }
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

// Few-channel matrix-core form (CI, CO in {4, 8}; 4x4x4 circular p = 1 or 2x2x2 p = 0, one input,
// every extent even, 16-bit): the full-resolution down blocks' branch conv2 (4 -> 4 at 512^2 x 128,
// 8 -> 8 at 256^2 x 64) and skip conv (4 -> 8).  The input grid is cut into 2 x 2 x 2 CELLS; cell
// (mh, mw, md) holds the 8 input voxels i = 2 m + v that read the g rows o = m + e, e in {-1, 0, 1}^3
// (tap t = v + p - 2 e per dimension, 0 <= t < k; for k = 2 only e = 0).  So a cell's backward-data
// is one dense product gx[v][ci] = sum_(e, co) A[(v, ci)][(e, co)] g[m + e][co] with the tap weights
// (and zeros where t falls outside the kernel) as the MFMA A operand -- rows (v, ci) in 16-row tiles,
// staged once per workgroup in LDS -- and 16 cells along D as the B columns (lane (n, kb): the 8 k
// entries of g rows e for cell n, one 8- / 16-byte load per row).  Every lane's accumulator then
// holds 4 channels of one voxel of its cell, and lanes kb, kb + 1 own neighbouring voxels / channel
// halves: 16 cells x 16 (or 32) contiguous bytes per store.  The index math is one line (b, mh, mw)
// per tile of 16 cells (128 input voxels).  The epilogue is k_dgrad_s2's.
template <int CI, int CO, int K>
__global__ __launch_bounds__(256) void k_dgrad_s2_cell(S2Args a, const h16_t *__restrict__ g,
                                                      const float *__restrict__ gscale, const float *__restrict__ w,
                                                      BwdEpi<h16_t> be, h16_t *__restrict__ gx, float *dpre,
                                                      float *dpost, GridSum gsum) {
    constexpr int NR = K == 4 ? 27 : 1, K3 = K * K * K, NKS = (NR * CO + 31) / 32, NM = 8 * CI / 16;
    constexpr int EPL = CO == 4 ? 2 : 1;  // g rows per lane and k-step
    static_assert((CI == 4 || CI == 8) && (CO == 4 || CO == 8) && (K == 2 || K == 4), "few-channel form");
    __shared__ uint4 afr[NM * NKS * 64];  // packed A fragments [m-tile][k-step][lane]
    __shared__ float red[8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kb = lane >> 4, n = lane & 15;
    for (int idx = tid; idx < NM * NKS * 64; idx += 256) {
        const int l = idx & 63, ms = idx >> 6, st = ms % NKS, m = ms / NKS;
        const int R = 16 * m + (l & 15), v = R / CI, ci = R - v * CI;
        const int vh = v >> 2, vw = (v >> 1) & 1, vd = v & 1;
        uint32_t u[4];
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
            float x2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = 32 * st + 8 * (l >> 4) + 2 * e2 + h, r = k / CO, co = k - r * CO;
                float x = 0.f;
                if (r < NR) {
                    const int eh = K == 4 ? r / 9 - 1 : 0, ew = K == 4 ? (r / 3) % 3 - 1 : 0, ed = K == 4 ? r % 3 - 1 : 0;
                    const int th = vh + a.p - 2 * eh, tw = vw + a.p - 2 * ew, td = vd + a.p - 2 * ed;
                    if (th >= 0 && th < K && tw >= 0 && tw < K && td >= 0 && td < K)
                        x = w[(co * CI + ci) * K3 + (th * K + tw) * K + td];
                }
                x2[h] = x;
            }
            u[e2] = uint32_t(f2h(x2[0])) | (uint32_t(f2h(x2[1])) << 16);
        }
        afr[idx] = uint4{u[0], u[1], u[2], u[3]};
    }
    __syncthreads();
    ActDeriv dv;
    dv.mode = be.aux ? be.mode : 0;
    dv.p = (dv.mode && be.p) ? *be.p : 0.f;
    const float gs = gscale ? *gscale : 1.f;
    float pre = 0.f, post = 0.f;
    const int hh = a.iH >> 1, hw = a.iW >> 1, hd = a.iD >> 1;  // cells per dimension (= the g grid)
    const int ntl = (hd + 15) >> 4;                              // 16-cell tiles per line
    const int ntile = a.B * hh * hw * ntl;
    // one tile's operands: the B fragments, the epilogue's aux / addend rows, the output offsets
    struct Tile {
        uint4 bv[NKS];
        uint2 aux[NM], add[NM];
        int64_t ev[NM];
        bool live;
    };
    // tile coordinates (line (b, mh, mw), first cell md0), advanced incrementally along a wave's
    // contiguous tile range (no divisions per tile)
    struct Pos {
        int md0, mw, mh, b;
    };
    auto fetch = [&](const Pos &P, Tile &T) {
        const int md = P.md0 + n;
        T.live = md < hd;
        const int mdc = T.live ? md : hd - 1;  // dead lanes read a real row (never stored)
        // the g rows this lane's k entries read: o = m + e per dimension (circular on the g grid)
        int rowh[3], roww[3], rowd[3];
#pragma unroll
        for (int e = 0; e < 3; ++e) {
            const int oh_ = P.mh + e - 1, ow_ = P.mw + e - 1, od_ = mdc + e - 1;
            rowh[e] = oh_ < 0 ? oh_ + a.oH : (oh_ >= a.oH ? oh_ - a.oH : oh_);
            roww[e] = ow_ < 0 ? ow_ + a.oW : (ow_ >= a.oW ? ow_ - a.oW : ow_);
            rowd[e] = od_ < 0 ? od_ + a.oD : (od_ >= a.oD ? od_ - a.oD : od_);
        }
        const int64_t gb = int64_t(P.b) * a.oH;
#pragma unroll
        for (int st = 0; st < NKS; ++st) {
            uint32_t u[4];
#pragma unroll
            for (int h2 = 0; h2 < EPL; ++h2) {
                // k entries past the 27 rows meet zero weights: they read row NR - 1 (finite data)
                const int r = min((32 * st + 8 * kb) / CO + h2, NR - 1);
                const int eh = K == 4 ? r / 9 : 1, ew = K == 4 ? (r / 3) % 3 : 1, ed = K == 4 ? r % 3 : 1;
                const h16_t *src = g + (((gb + rowh[eh]) * a.oW + roww[ew]) * a.oD + rowd[ed]) * CO;
                if constexpr (CO == 8) {
                    const uint4 x = *reinterpret_cast<const uint4 *>(src);
                    u[0] = x.x, u[1] = x.y, u[2] = x.z, u[3] = x.w;
                } else {
                    const uint2 x = *reinterpret_cast<const uint2 *>(src);
                    u[2 * h2] = x.x, u[2 * h2 + 1] = x.y;
                }
            }
            if constexpr (CO == 4 && EPL == 1) u[2] = u[3] = 0u;
            T.bv[st] = uint4{u[0], u[1], u[2], u[3]};
        }
        // lane (n, kb) of m-tile m: rows 16 m + 4 kb .. + 3 = 4 channels of voxel v of cell n
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const int R = 16 * m + 4 * kb, v = R / CI, c0 = R - v * CI;
            const int vh = v >> 2, vw = (v >> 1) & 1, vd = v & 1;
            T.ev[m] = (((int64_t(P.b) * a.iH + 2 * P.mh + vh) * a.iW + 2 * P.mw + vw) * a.iD + 2 * mdc + vd) * CI + c0;
            T.aux[m] = dv.mode ? *reinterpret_cast<const uint2 *>(be.aux + T.ev[m]) : uint2{0u, 0u};
            T.add[m] = be.addend ? *reinterpret_cast<const uint2 *>(be.addend + T.ev[m]) : uint2{0u, 0u};
        }
    };
    auto advance = [&](Pos &P) {
        P.md0 += 16;
        if (P.md0 >= hd) {
            P.md0 = 0;
            if (++P.mw == hw) {
                P.mw = 0;
                if (++P.mh == hh) {
                    P.mh = 0;
                    ++P.b;
                }
            }
        }
    };
    auto compute = [&](const Tile &T) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int st = 0; st < NKS; ++st)
                acc = VQ3D_MFMA_16X16X32(__builtin_bit_cast(hx8, afr[(m * NKS + st) * 64 + lane]),
                                         __builtin_bit_cast(hx8, T.bv[st]), acc, 0, 0, 0);
            if (!T.live) continue;
            const float ax[4] = {h2f_lo(T.aux[m].x), h2f_hi(T.aux[m].x), h2f_lo(T.aux[m].y), h2f_hi(T.aux[m].y)};
            const float ad[4] = {h2f_lo(T.add[m].x), h2f_hi(T.add[m].x), h2f_lo(T.add[m].y), h2f_hi(T.add[m].y)};
            float o[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float val = acc[c];
                if (gscale) val = val * gs;
                pre += val;
                if (dv.mode) val = val * dv(ax[c]);
                post += val;
                if (be.addend) val = val + ad[c];
                o[c] = val;
            }
            *reinterpret_cast<uint2 *>(gx + T.ev[m]) = uint2{uint32_t(f2h(o[0])) | (uint32_t(f2h(o[1])) << 16),
                                                             uint32_t(f2h(o[2])) | (uint32_t(f2h(o[3])) << 16)};
        }
    };
    // each wave walks a contiguous range of tiles (consecutive 16-cell runs of the lines)
    const int nw = int(gridDim.x) * 4, wid = int(blockIdx.x) * 4 + wave;
    const int per = (ntile + nw - 1) / nw, t0 = min(wid * per, ntile), t1 = min(t0 + per, ntile);
    if (t0 >= t1) goto done;
    {
        Pos P;
        {
            const int line = t0 / ntl;
            P.md0 = (t0 - line * ntl) * 16;
            P.mw = line % hw;
            const int q = line / hw;
            P.mh = q % hh;
            P.b = q / hh;
        }
        // small tiles (<= 16 B-fragment registers x m-tiles): software-pipelined, the next tile's
        // loads in flight while this one computes; the wide ones keep one tile (their registers
        // would halve the occupancy)
        constexpr bool PIPE = CI * NKS <= 16;
        if constexpr (PIPE) {
            Tile nxt;
            fetch(P, nxt);
            for (int t = t0; t < t1; ++t) {
                const Tile T = nxt;
                if (t + 1 < t1) {
                    advance(P);
                    fetch(P, nxt);
                }
                compute(T);
            }
        } else {
            for (int t = t0; t < t1; ++t) {
                Tile T;
                fetch(P, T);
                compute(T);
                advance(P);
            }
        }
    }
done:
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

// Matrix-core form for the wide layers (one input, Cin % 16 == 0, Cout % 8 == 0: the down blocks'
// branch conv2 4x4x4 and skip conv 2x2x2 from 16 channels up, vqvae/layers.py:124-126,164-171).
// blockIdx.y = the (h, w, d) parity class of the input voxels: every voxel of a class meets the
// same (k/2)^3 taps, so per class the backward-data is one GEMM
//     gx^T[ci][v] = sum over (j, co) of W[co][ci][tap_j] * g[o_j(v)][co]
// with K = (k/2)^3 * Cout.  The weights are the MFMA A operand (so each lane's accumulator holds 4
// consecutive input channels of one voxel: one 8-byte store), packed per (channel tile, k-step)
// into LDS once per workgroup; the g rows are B (8 consecutive co of one tap: one 16-byte load per
// lane and k-step).  The epilogue is k_dgrad_s2's (activation derivative from aux, addend, gscale,
// prologue-scalar partial sums).
__device__ __forceinline__ int s2_src(int i, int t, int p, int n_in, int n_out, int circ) {
    int r = i + p - t;
    if (circ) r = r < 0 ? r + n_in : (r >= n_in ? r - n_in : r);
    else if (r < 0) return -1;
    r >>= 1;
    return r < n_out ? r : -1;
}

template <int K, int NTM>
__global__ __launch_bounds__(256) void k_dgrad_s2_mma(S2Args a, const h16_t *__restrict__ g,
                                                     const float *__restrict__ gscale, const float *__restrict__ w,
                                                     BwdEpi<h16_t> be, h16_t *__restrict__ gx, float *dpre,
                                                     float *dpost, int nks, GridSum gsum) {
    constexpr int NT_ = K / 2, NJ = NT_ * NT_ * NT_, K3 = K * K * K;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint4 *afr = reinterpret_cast<uint4 *>(smem);  // [NTM][nks][64] packed A fragments
    __shared__ float red[8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kb = lane >> 4, n = lane & 15;
    const int cls = int(blockIdx.y), rh = cls >> 2, rw = (cls >> 1) & 1, rd = cls & 1;
    const int t0h = (rh + a.p) & 1, t0w = (rw + a.p) & 1, t0d = (rd + a.p) & 1;  // the class's first taps
    const int c0 = int(blockIdx.z) * NTM * 16;
    for (int idx = tid; idx < NTM * nks * 64; idx += 256) {
        const int l = idx & 63, r = idx >> 6, s = r % nks, mt = r / nks;
        const int ci = c0 + 16 * mt + (l & 15);
        const int f0 = 32 * s + 8 * (l >> 4), j = f0 / a.Cout, co0 = f0 - j * a.Cout;
        uint32_t u[4] = {0u, 0u, 0u, 0u};
        if (j < NJ) {
            const int xd = j % NT_, xw = (j / NT_) % NT_, xh = j / (NT_ * NT_);
            const int tap = ((t0h + 2 * xh) * K + t0w + 2 * xw) * K + t0d + 2 * xd;
            const float *wp = w + (int64_t(co0) * a.Cin + ci) * K3 + tap;
            const int64_t st_ = int64_t(a.Cin) * K3;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                u[e] = uint32_t(f2h(wp[(2 * e) * st_])) | (uint32_t(f2h(wp[(2 * e + 1) * st_])) << 16);
        }
        afr[idx] = uint4{u[0], u[1], u[2], u[3]};
    }
    __syncthreads();
    ActDeriv dv;
    dv.mode = be.aux ? be.mode : 0;
    dv.p = (dv.mode && be.p) ? *be.p : 0.f;
    const float gs = gscale ? *gscale : 1.f;
    float pre = 0.f, post = 0.f;
    const int hh = a.iH >> 1, hw = a.iW >> 1, hd = a.iD >> 1;
    const int nvc = a.B * hh * hw * hd;  // voxels of the class
    const int ntile = (nvc + 15) >> 4;
    for (int t = int(blockIdx.x) * 4 + wave; t < ntile; t += int(gridDim.x) * 4) {
        const int vi = 16 * t + n;
        const bool live = vi < nvc;
        int q = live ? vi : 0;
        const int md = q % hd;
        q /= hd;
        const int mw = q % hw;
        q /= hw;
        const int mh = q % hh;
        const int b = q / hh;
        const int ih = 2 * mh + rh, iw = 2 * mw + rw, id = 2 * md + rd;
        int oh[NT_], ow[NT_], od[NT_];
#pragma unroll
        for (int x = 0; x < NT_; ++x) {
            oh[x] = s2_src(ih, t0h + 2 * x, a.p, a.iH, a.oH, a.circ);
            ow[x] = s2_src(iw, t0w + 2 * x, a.p, a.iW, a.oW, a.circ);
            od[x] = s2_src(id, t0d + 2 * x, a.p, a.iD, a.oD, a.circ);
        }
        f32x4 acc[NTM];
#pragma unroll
        for (int m = 0; m < NTM; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
        // the lane's k entries of step s: tap j, channels co .. co + 7 (advanced by 32 per step)
        int j = (8 * kb) / a.Cout, co = 8 * kb - j * a.Cout;
#pragma unroll 4
        for (int s = 0; s < nks; ++s) {
            uint4 bv = uint4{0u, 0u, 0u, 0u};
            if (live && j < NJ) {
                const int xd = j % NT_, xw = (j / NT_) % NT_, xh = j / (NT_ * NT_);
                const int hh_ = NT_ == 1 ? oh[0] : (xh ? oh[NT_ - 1] : oh[0]);
                const int ww_ = NT_ == 1 ? ow[0] : (xw ? ow[NT_ - 1] : ow[0]);
                const int dd_ = NT_ == 1 ? od[0] : (xd ? od[NT_ - 1] : od[0]);
                if (hh_ >= 0 && ww_ >= 0 && dd_ >= 0)
                    bv = *reinterpret_cast<const uint4 *>(
                        g + ((((int64_t(b) * a.oH + hh_) * a.oW + ww_) * a.oD + dd_) * a.Cout + co));
            }
            const hx8 bf = __builtin_bit_cast(hx8, bv);
#pragma unroll
            for (int m = 0; m < NTM; ++m)
                acc[m] = VQ3D_MFMA_16X16X32(__builtin_bit_cast(hx8, afr[(m * nks + s) * 64 + lane]), bf, acc[m], 0, 0, 0);
            co += 32;
            while (co >= a.Cout) {
                co -= a.Cout;
                ++j;
            }
        }
        if (!live) continue;
        const int64_t vox = ((int64_t(b) * a.iH + ih) * a.iW + iw) * a.iD + id;
#pragma unroll
        for (int m = 0; m < NTM; ++m) {
            const int64_t o = vox * a.Cin + c0 + 16 * m + 4 * kb;
            float aux[4], add[4], v[4];
            if (dv.mode) load_row<h16_t, 4>(be.aux + o, aux);
            if (be.addend) load_row<h16_t, 4>(be.addend + o, add);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float val = acc[m][c];
                if (gscale) val = val * gs;
                pre += val;
                if (dv.mode) val = val * dv(aux[c]);
                post += val;
                if (be.addend) val = val + add[c];
                v[c] = val;
            }
            *reinterpret_cast<uint2 *>(gx + o) = uint2{uint32_t(f2h(v[0])) | (uint32_t(f2h(v[1])) << 16),
                                                       uint32_t(f2h(v[2])) | (uint32_t(f2h(v[3])) << 16)};
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

}  // namespace

bool dgrad_s2_applicable(const vq3d_conv_desc *d) {
    return d->stride == 2 && (d->kernel == 2 || d->kernel == 4) && d->in_h % 2 == 0 && d->in_w % 2 == 0 &&
           d->in_d % 2 == 0;
}

template <typename T>
int launch_dgrad_s2(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w,
                    const BwdEpi<T> &be, void *gx, void *gx2, float *dpre, float *dpost, hipStream_t s) {
    S2Args a;
    a.B = d->batch;
    a.Cin1 = d->cin;
    a.Cin2 = d->cin2;
    a.Cin = d->cin + d->cin2;
    a.Cout = d->cout;
    a.iH = d->in_h; a.iW = d->in_w; a.iD = d->in_d;
    a.oH = d->out_h; a.oW = d->out_w; a.oD = d->out_d;
    a.k = d->kernel;
    a.p = d->pad;
    a.circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    a.fD = FastDiv(uint32_t(a.iD));
    a.fW = FastDiv(uint32_t(a.iW));
    a.fH = FastDiv(uint32_t(a.iH));
    if (int64_t(a.B) * a.iH * a.iW * a.iD >= (int64_t(1) << 31)) return fail("conv3d_bwd_data(s2): grid too large");
    {
        auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
        // few channels on the matrix cores over 2 x 2 x 2 cells (k_dgrad_s2_cell); k = 2, p = 0:
        // every tap lands inside the grid, so the padding mode does not matter (the down blocks'
        // zero-padded skip conv takes it too)
        if (std::is_same<T, h16_t>::value && (a.circ || (a.k == 2 && a.p == 0)) && a.Cin2 == 0 &&
            (a.Cin == 4 || a.Cin == 8) &&
            (a.Cout == 4 || a.Cout == 8) && a.p == a.k / 2 - 1 && a.iH == 2 * a.oH && a.iW == 2 * a.oW &&
            a.iD == 2 * a.oD && al16(g) && al16(gx) && (!be.aux || al16(be.aux)) && (!be.addend || al16(be.addend))) {
            // ~2,048 workgroups, each wave a contiguous range of 16-cell tiles
            const int64_t ntile = int64_t(a.B) * a.oH * a.oW * ((a.oD + 15) / 16);
            const dim3 fg(unsigned(std::max<int64_t>(1, std::min<int64_t>((ntile + 3) / 4, 2048))), 1u, 1u);
#define PK(CI_, CO_, K_)                                                                                      \
            if (a.Cin == CI_ && a.Cout == CO_ && a.k == K_) {                                                  \
                k_dgrad_s2_cell<CI_, CO_, K_><<<fg, 256, 0, s>>>(a, (const h16_t *)g, gscale, w,                \
                                                                 reinterpret_cast<const BwdEpi<h16_t> &>(be),    \
                                                                 (h16_t *)gx, dpre, dpost,               \
                                                                 grid_sum_for(s, fg.x, dpre || dpost));         \
                return check_launch("conv3d_bwd_data(s2 cell mma)");                                           \
            }
            PK(4, 4, 4) PK(4, 8, 4) PK(8, 4, 4) PK(8, 8, 4) PK(4, 4, 2) PK(4, 8, 2) PK(8, 4, 2) PK(8, 8, 2)
#undef PK
        }
    }
    if constexpr (std::is_same<T, h16_t>::value) {
        // matrix-core parity classes: one input, 16-channel input tiles, 8-channel g rows, K >= 32
        auto al16 = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
        const int nj = (a.k / 2) * (a.k / 2) * (a.k / 2);
        if (a.Cin2 == 0 && a.Cin % 16 == 0 && a.Cout % 8 == 0 && nj * a.Cout >= 32 && al16(g) && al16(gx) &&
            (!be.aux || al16(be.aux)) && (!be.addend || al16(be.addend)) &&
            int64_t(a.B) * a.oH * a.oW * a.oD * a.Cout < (int64_t(1) << 31)) {
            const int nks = (nj * a.Cout + 31) / 32;
            const int64_t nvc = int64_t(a.B) * (a.iH / 2) * (a.iW / 2) * (a.iD / 2);
            int ntm = 4;
            while (ntm > 1 && (a.Cin % (16 * ntm) || size_t(ntm) * nks * 1024 > 48 * 1024)) ntm /= 2;
            if (nvc <= 4096) ntm = 1;  // few voxels: spread the channel tiles over workgroups instead
            if (size_t(ntm) * nks * 1024 <= 48 * 1024) {
                const int nz = a.Cin / (16 * ntm);
                const int64_t ntile = (nvc + 15) / 16;
                // each workgroup packs its class's A fragments once (8 strided weight loads per entry):
                // with large packs ~256 workgroups amortise that (32 -> 32 @64^2x16 38.5 -> 31.0 us), with
                // small ones ~2,048 keep the big grids busy (16 -> 16 @128^2x32; r04f / r04g)
                const int wg_target = a.k == 4 && ntm * nks <= 8 ? 2048 : 256;  // 2x2x2: 256 (12.4 vs 20.8 us)
                const unsigned gxn = unsigned(std::max<int64_t>(
                    1, std::min<int64_t>((ntile + 3) / 4, std::max(1, wg_target / (8 * nz)))));
                const dim3 grid(gxn, 8u, unsigned(nz));
                const size_t lds = size_t(ntm) * nks * 1024;
#define MM(K_, NTM_)                                                                                          \
                if (a.k == K_ && ntm == NTM_) {                                                                  \
                    k_dgrad_s2_mma<K_, NTM_><<<grid, 256, lds, s>>>(a, (const h16_t *)g, gscale, w, be,           \
                                                                   (h16_t *)gx, dpre, dpost, nks,                 \
                                                                   grid_sum_for(s, int64_t(gxn) * 8 * nz,          \
                                                                                dpre || dpost));                 \
                    return check_launch("conv3d_bwd_data(s2 mma)");                                              \
                }
                MM(2, 1) MM(2, 2) MM(2, 4) MM(4, 1) MM(4, 2) MM(4, 4)
#undef MM
            }
        }
    }
    const int K3 = a.k * a.k * a.k;
    int cot = a.Cin <= 1 ? 1 : a.Cin <= 2 ? 2 : a.Cin <= 4 ? 4 : a.Cin <= 8 ? 8 : 16;
    while (cot > 1 && size_t(K3) * a.Cout * cot * 4 > 64 * 1024) cot /= 2;
    const size_t lds = size_t(K3) * a.Cout * cot * 4;
    if (lds > 64 * 1024) return fail("conv3d_bwd_data(s2): too many channels");
    const int64_t nvox = int64_t(a.B) * a.iH * a.iW * a.iD;
    const int ych = (a.Cin + cot - 1) / cot;
    const unsigned nbx = unsigned(std::max<int64_t>(1, std::min<int64_t>((nvox + 255) / 256, 4096 / ych + 1)));
    const dim3 grid{nbx, unsigned(ych), 1u};
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    a.rows = (ych == 1 && a.Cin2 == 0 && a.Cin == cot && (cot == 4 || cot == 8) && al(gx) &&
              (!be.aux || al(be.aux)) && (!be.addend || al(be.addend))) ? 1 : 0;
    const int co_t = (al(g) && (a.Cout == 4 || a.Cout == 8 || a.Cout == 16)) ? a.Cout : 0;
#define L(C, CO)                                                                                              \
    case C:                                                                                                   \
        k_dgrad_s2<T, C, CO><<<grid, 256, lds, s>>>(a, (const T *)g, gscale, w, be, (T *)gx, (T *)gx2, dpre,  \
                                                    dpost, grid_sum_for(s, int64_t(nbx) * ych, dpre || dpost)); \
        break;
#define LS(CO)                                                                                                \
    switch (cot) { L(1, CO) L(2, CO) L(4, CO) L(8, CO) L(16, CO) }
    switch (co_t) {
    case 4: LS(4) break;
    case 8: LS(8) break;
    case 16: LS(16) break;
    default: LS(0) break;
    }
#undef LS
#undef L
    return check_launch("conv3d_bwd_data(s2)");
}

template int launch_dgrad_s2<float>(const vq3d_conv_desc *, const void *, const float *, const float *,
                                    const BwdEpi<float> &, void *, void *, float *, float *, hipStream_t);
template int launch_dgrad_s2<h16_t>(const vq3d_conv_desc *, const void *, const float *, const float *,
                                     const BwdEpi<h16_t> &, void *, void *, float *, float *, hipStream_t);

}  // namespace vq3d
