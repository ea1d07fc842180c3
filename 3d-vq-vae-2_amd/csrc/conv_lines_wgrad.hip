// k^3 convolution weight gradient on v_mfma_f32_16x16x32_bf16 over staged D-lines (the layout of
// conv_lines.hip); the reduction runs over output voxels:
//
//   G[co][(kh, kw, kd, ci)] = sum_v g[v][co] * window(v, kh, kw)[(kd, ci)]
//   D[M = co][N = window column] += A[co][K = 32 voxels] * B[32 voxels][window column]
//
// Replaces the weight gradient of nn.Conv3d for the residual blocks' k^3 convs
// (vqvae/layers.py:124-151, 28-36, 239-247).
//
// Each brick's halo lines are staged once with channel stride CS = C rounded up to 4 (zero
// padding), so every voxel's window starts 8-byte aligned: both operands then come from LDS
// through the gfx950 transposing read ds_read_b64_tr_b16 -- A from the brick's g tile
// [voxel][co] (rows = voxels, columns = output channels), B straight from the lines (rows =
// the voxels' windows, columns = consecutive window elements) -- with no im2col copy.  A
// workgroup owns NPW column tiles per wave (blockIdx.y picks the column group), loops over
// bricks (grid-stride) accumulating in registers, and finally adds its partial G to the fp32
// gradient with one atomic per entry (workgroups per column group are capped, so each address
// sees a bounded number of adders).
#include "engines.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct WArgs {
    int B, Ca, Cb, C, CS, N;   // input channels (x, x2), LDS channel stride, output channels
    int iH, iW, iD, oH, oW, oD;
    int k, s, p, circ;
    int pro_kind;
    const float *pro_a, *pro_b;
    int bh, bw, bd, lbw, lbd;  // brick (power-of-two extents)
    int hh, hw, LP, LS, pad0;  // halo lines, positions per line, LDS line stride, head pad
    int nvb, nvp;              // brick voxels, padded to 32
    int GS;                    // g tile row stride (NTM * 16)
    int ncol;                  // window columns per (kh, kw): k * CS
    int ctile;                 // 16-wide column tiles per (kh, kw)
    int ntiles;                // k * k * ctile
    int nbh, nbw, nbd, nbricks;
    int wCt;                   // weight's 2nd dim
    int gvec;                  // g runs of bd*N elements are 16-B aligned multiples of 8
    int mc;                    // 8-element chunks per line run (C % 4 != 0 staging)
    int nent;                  // partial slots per workgroup: ntiles * NTM * 256 fragments + N g sums
    int64_t xtotal;            // elements of x
    FastDiv fC, fhw, fN, fCr, fmc;
    unsigned tapmask;          // 0, or the weight taps that may be nonzero (vq3d_conv_desc.tap_mask)
    int ntl;                   // column tiles computed: ntiles, or the live ones (tile_map order)
};

// column tile tt (t2 = kh*k + kw, 16 window columns from 16 jt) holds a live tap
__host__ __device__ inline bool wtile_live(int tt, const WArgs &a) {
    const int t2 = tt / a.ctile, jt = tt - t2 * a.ctile;
    const int e0 = 16 * jt;
    if (e0 >= a.k * a.CS) return false;
    const int e1 = (e0 + 15 < a.k * a.CS - 1) ? e0 + 15 : a.k * a.CS - 1;
    for (int kd = e0 / a.CS; kd <= e1 / a.CS; ++kd)
        if ((a.tapmask >> (t2 * a.k + kd)) & 1u) return true;
    return false;
}

// the live tiles in order into tmap[0 .. ntl): one wave (ballot prefix sums), caller synchronises
__device__ void live_tile_map(const WArgs &a, short *tmap, int lane) {
    int cnt = 0;
    for (int base = 0; base < a.ntiles; base += 64) {
        const int tt = base + lane;
        const bool lv = tt < a.ntiles && wtile_live(tt, a);
        const uint64_t bal = __ballot(lv);
        if (lv) tmap[cnt + __popcll(bal & ((uint64_t(1) << lane) - 1))] = short(tt);
        cnt += __popcll(bal);
    }
}
constexpr int kMaxMaskTiles = 1024;

__device__ __forceinline__ s16x4 tr_read(const h16_t *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p));
}

__device__ __forceinline__ hx8 cat8(s16x4 lo, s16x4 hi) {
    return __builtin_bit_cast(hx8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ int wrapw(int i, int n) {
    while (i < 0) i += n;
    while (i >= n) i -= n;
    return i;
}

template <int NTM, int NPW>
__global__ __launch_bounds__(256) void k_lines_wgrad(WArgs a, const h16_t *__restrict__ x,
                                                    const h16_t *__restrict__ x2, const h16_t *__restrict__ g,
                                                    float *__restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nlines = a.hh * a.hw;
    h16_t *lines = reinterpret_cast<h16_t *>(smem);                             // [nlines][LS]
    h16_t *gt = lines + ((nlines * a.LS + 7) / 8) * 8;                           // [nvp][GS]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const bool raw = pro.kind == VQ3D_PRO_NONE;
    const int tile0 = blockIdx.y * 4 * NPW;
    const bool do_bias = blockIdx.y == 0;
    short *tmap = reinterpret_cast<short *>(gt + a.nvp * a.GS);  // [ntiles] (tap mask only)
    if (a.tapmask) {
        if (wave == 0) live_tile_map(a, tmap, lane);
        __syncthreads();
    }

    // this lane's B column offset (element) per owned tile: (kh, kw) line delta + column chunk
    int coff[NPW];
#pragma unroll
    for (int t = 0; t < NPW; ++t) {
        int tt = tile0 + wave + 4 * t;  // index into the computed tiles
        if (tt >= a.ntl) tt = 0;        // padded tiles read valid addresses, are never written
        else if (a.tapmask) tt = tmap[tt];
        const int t2 = tt / a.ctile, jt = tt - t2 * a.ctile;
        const int kh = t2 / a.k, kw = t2 - kh * a.k;
        coff[t] = (kh * a.hw + kw) * a.LS + 16 * jt + 4 * pp;
    }
    f32x4 acc[NTM][NPW];
#pragma unroll
    for (int m = 0; m < NTM; ++m)
#pragma unroll
        for (int t = 0; t < NPW; ++t) acc[m][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float gsum = 0.f;

    for (int brick = blockIdx.x; brick < a.nbricks; brick += gridDim.x) {
        int bi = brick;
        const int bzd = bi % a.nbd; bi /= a.nbd;
        const int bzw = bi % a.nbw; bi /= a.nbw;
        const int bzh = bi % a.nbh;
        const int b = bi / a.nbh;
        const int oh0 = bzh * a.bh, ow0 = bzw * a.bw, od0 = bzd * a.bd;
        const int ih0 = oh0 * a.s - a.p, iw0 = ow0 * a.s - a.p, id0 = od0 * a.s - a.p;
        __syncthreads();
        // ---- lines: element (pos, c) at line*LS + pad0 + pos*CS + c; padding channels and
        // the slack are zero.
        if (a.Cb == 0 && (a.C & 3) != 0) {
            // C not a multiple of 4 (1, 2, 9 channels): a line's in-grid positions are one
            // contiguous run of x, read with 16-byte loads and scattered to the CS-padded slots
            for (int e = tid; e < nlines * a.LS / 8; e += 256) reinterpret_cast<uint4 *>(lines)[e] = uint4{0, 0, 0, 0};
            __syncthreads();
            const int pa = max(0, -id0), pb = min(a.LP, a.iD - id0);
            if (pb > pa) {
                for (int u = tid; u < nlines * a.mc; u += 256) {
                    const int ln = int(a.fmc.div(uint32_t(u))), ch = u - ln * a.mc;
                    const int lh_ = int(a.fhw.div(uint32_t(ln))), lw_ = ln - lh_ * a.hw;
                    int ih = ih0 + lh_, iw = iw0 + lw_;
                    if (a.circ) {
                        ih = wrapw(ih, a.iH);
                        iw = wrapw(iw, a.iW);
                    } else if (unsigned(ih) >= unsigned(a.iH) || unsigned(iw) >= unsigned(a.iW)) {
                        continue;
                    }
                    const int64_t lbase = ((int64_t(b) * a.iH + ih) * a.iW + iw) * a.iD * a.C;
                    const int64_t E0 = lbase + int64_t(pa + id0) * a.C, E1 = lbase + int64_t(pb + id0) * a.C;
                    const int64_t cs = (E0 & ~int64_t(7)) + int64_t(ch) * 8;
                    if (cs >= E1) continue;
                    h16_t el[8];
                    if (cs + 8 <= a.xtotal) {
                        const uint4 qv = *reinterpret_cast<const uint4 *>(x + cs);
                        const h16_t *q8 = reinterpret_cast<const h16_t *>(&qv);
#pragma unroll
                        for (int j = 0; j < 8; ++j) el[j] = q8[j];
                    } else {
#pragma unroll
                        for (int j = 0; j < 8; ++j) el[j] = cs + j < a.xtotal ? x[cs + j] : h16_t(0);
                    }
                    const int j0 = cs < E0 ? int(E0 - cs) : 0;
                    const int rel = int(cs + j0 - lbase);
                    int idd = int(a.fCr.div(uint32_t(rel))), c = rel - idd * a.C;
                    h16_t *dst = lines + ln * a.LS + a.pad0 + (idd - id0) * a.CS;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (j < j0 || cs + j >= E1) continue;
                        dst[c] = raw ? el[j] : f2h(pro.apply(h2f_lo(uint32_t(el[j]))));
                        if (++c == a.C) {
                            c = 0;
                            dst += a.CS;
                        }
                    }
                }
            }
            const int nw = pb > pa ? pa + (a.LP - pb) : a.LP;
            if (a.circ && nw > 0) {  // positions outside [pa, pb) wrap around D (zero padding: zeros)
                for (int u = tid; u < nlines * nw * a.C; u += 256) {
                    const int lk = int(a.fCr.div(uint32_t(u))), r = u - lk * a.C;  // r = channel
                    const int ln = lk / nw, k = lk - ln * nw;
                    const int pos = pb > pa ? (k < pa ? k : pb + (k - pa)) : k;
                    const int lh_ = int(a.fhw.div(uint32_t(ln))), lw_ = ln - lh_ * a.hw;
                    const int ih = wrapw(ih0 + lh_, a.iH), iw = wrapw(iw0 + lw_, a.iW), id = wrapw(id0 + pos, a.iD);
                    const h16_t v = x[(((int64_t(b) * a.iH + ih) * a.iW + iw) * a.iD + id) * a.C + r];
                    lines[ln * a.LS + a.pad0 + pos * a.CS + r] = raw ? v : f2h(pro.apply(ld(&v)));
                }
            }
        } else {
            {
                const int64_t bbase = int64_t(b) * a.iH * a.iW * a.iD;
                const int total = nlines * a.LP;
                for (int u = tid; u < total; u += 256) {
                    const int ln = u / a.LP, pos = u - ln * a.LP;
                    const int lh_ = int(a.fhw.div(uint32_t(ln))), lw_ = ln - lh_ * a.hw;
                    int ih = ih0 + lh_, iw = iw0 + lw_, id = id0 + pos;
                    bool ok;
                    if (a.circ) {
                        ih = wrapw(ih, a.iH);
                        iw = wrapw(iw, a.iW);
                        id = wrapw(id, a.iD);
                        ok = true;
                    } else {
                        ok = unsigned(ih) < unsigned(a.iH) && unsigned(iw) < unsigned(a.iW) && unsigned(id) < unsigned(a.iD);
                    }
                    const int64_t vox = bbase + (int64_t(ih) * a.iW + iw) * a.iD + id;
                    h16_t *dst = lines + ln * a.LS + a.pad0 + pos * a.CS;
                    if (ok && a.Cb == 0 && (a.C & 3) == 0) {
                        const uint2 *src = reinterpret_cast<const uint2 *>(x + vox * a.C);
                        for (int c4 = 0; c4 < a.C / 4; ++c4) {
                            uint2 qv = src[c4];
                            if (!raw) {
                                auto f = [&](uint32_t uu) {
                                    const float lo = pro.apply(h2f_lo(uu));
                                    const float hi = pro.apply(h2f_hi(uu));
                                    return uint32_t(f2h(lo)) | (uint32_t(f2h(hi)) << 16);
                                };
                                qv = uint2{f(qv.x), f(qv.y)};
                            }
                            reinterpret_cast<uint2 *>(dst)[c4] = qv;
                        }
                    } else {
                        for (int c = 0; c < a.CS; ++c) {
                            h16_t v = 0;
                            if (ok && c < a.C) {
                                const h16_t *src = c < a.Ca ? x + vox * a.Ca + c : x2 + vox * a.Cb + (c - a.Ca);
                                v = raw ? *src : f2h(pro.apply(ld(src)));
                            }
                            dst[c] = v;
                        }
                    }
                }
                const int tail0 = a.pad0 + a.LP * a.CS;
                const int z = a.LS - tail0 + a.pad0;
                for (int e = tid; e < nlines * z; e += 256) {
                    const int ln = e / z, r = e - ln * z;
                    lines[ln * a.LS + (r < a.pad0 ? r : tail0 + r - a.pad0)] = 0;
                }
            }
        }
        // ---- g tile [nvp][GS]: the brick's g is bh*bw contiguous runs of bd*N elements: 16-byte
        // loads when the runs allow, scattered into the padded rows; zero elsewhere
        for (int e = tid; e < a.nvp * a.GS; e += 256) gt[e] = 0;
        __syncthreads();
        {
            const int runlen = a.bd * a.N;
            const bool full = oh0 + a.bh <= a.oH && ow0 + a.bw <= a.oW && od0 + a.bd <= a.oD;
            if (full && a.gvec) {
                const int upr = runlen / 8;
                for (int u = tid; u < a.bh * a.bw * upr; u += 256) {
                    const int r = u / upr, e0 = (u - r * upr) * 8;
                    const int lh_ = r >> a.lbw, lw_ = r & (a.bw - 1);
                    const int64_t gb = ((((int64_t(b) * a.oH + oh0 + lh_) * a.oW) + ow0 + lw_) * a.oD + od0) * a.N;
                    const uint4 qv = *reinterpret_cast<const uint4 *>(g + gb + e0);
                    const h16_t *el = reinterpret_cast<const h16_t *>(&qv);
                    int ld_ = int(a.fN.div(uint32_t(e0))), co = e0 - ld_ * a.N;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        gt[((r << a.lbd) + ld_) * a.GS + co] = el[j];
                        if (++co == a.N) {
                            co = 0;
                            ++ld_;
                        }
                    }
                }
            } else {
                for (int e = tid; e < a.nvb * a.N; e += 256) {
                    const int v = int(a.fN.div(uint32_t(e))), co = e - v * a.N;
                    const int ld_ = v & (a.bd - 1), lw_ = (v >> a.lbd) & (a.bw - 1), lh_ = v >> (a.lbd + a.lbw);
                    const int oh = oh0 + lh_, ow = ow0 + lw_, od = od0 + ld_;
                    if (oh < a.oH && ow < a.oW && od < a.oD)
                        gt[v * a.GS + co] = g[((((int64_t(b) * a.oH + oh) * a.oW) + ow) * a.oD + od) * a.N + co];
                }
            }
        }
        __syncthreads();
        if (do_bias && tid < a.N)
            for (int v = 0; v < a.nvb; ++v) gsum += ld(gt + v * a.GS + tid);
        // ---- MFMA: K = 32 voxels per step
        for (int ks = 0; ks < a.nvp / 32; ++ks) {
            const int v1 = ks * 32 + 8 * grp + q, v2 = v1 + 4;
            hx8 af[NTM];
#pragma unroll
            for (int m = 0; m < NTM; ++m)
                af[m] = cat8(tr_read(gt + v1 * a.GS + m * 16 + 4 * pp), tr_read(gt + v2 * a.GS + m * 16 + 4 * pp));
            const int u1 = v1 < a.nvb ? v1 : 0, u2 = v2 < a.nvb ? v2 : 0;
            const int rb1 = (((u1 >> (a.lbd + a.lbw)) * a.s) * a.hw + ((u1 >> a.lbd) & (a.bw - 1)) * a.s) * a.LS +
                            a.pad0 + (u1 & (a.bd - 1)) * a.s * a.CS;
            const int rb2 = (((u2 >> (a.lbd + a.lbw)) * a.s) * a.hw + ((u2 >> a.lbd) & (a.bw - 1)) * a.s) * a.LS +
                            a.pad0 + (u2 & (a.bd - 1)) * a.s * a.CS;
#pragma unroll
            for (int t = 0; t < NPW; ++t) {
                const hx8 bfr = cat8(tr_read(lines + rb1 + coff[t]), tr_read(lines + rb2 + coff[t]));
#pragma unroll
                for (int m = 0; m < NTM; ++m)
                    acc[m][t] = VQ3D_MFMA_16X16X32(af[m], bfr, acc[m][t], 0, 0, 0);
            }
        }
    }
    // ---- this workgroup's partial G in MFMA fragment order (coalesced 16-byte stores):
    // part[blk][((tile * NTM + m) * 64 + lane) * 4 + i], then the N per-channel g sums; the
    // reduction maps each slot back to its weight entry
    float *pw = part + int64_t(blockIdx.x) * a.nent;
#pragma unroll
    for (int t = 0; t < NPW; ++t) {
        const int tt = tile0 + wave + 4 * t;
        if (tt >= a.ntl) continue;
#pragma unroll
        for (int m = 0; m < NTM; ++m)
            *reinterpret_cast<f32x4 *>(pw + ((tt * NTM + m) * 64 + lane) * 4) = acc[m][t];
    }
    if (do_bias && tid < a.N) pw[a.ntl * NTM * 256 + tid] = gsum;
}

// Sum the workgroup partials of every fragment slot (LANES lanes per slot, strided slices, 8
// loads in flight, fixed xor-shuffle tree: deterministic), map the slot to its weight entry
// (co, c, tap) and apply: dw += escale * G, dscale += sum W * G; the trailing N slots are
// the conv-bias / scalar-bias sums.
template <int LANES>
__global__ __launch_bounds__(256) void k_lines_wgrad_reduce(WArgs a, int ntm, const float *__restrict__ part,
                                                           int nblk, const float *__restrict__ w,
                                                           const float *__restrict__ escale, float *dw,
                                                           float *dscale, float *dbias, float *dcbias, GridSum gsum) {
    __shared__ float red[8];
    __shared__ short tmap[kMaxMaskTiles];
    if (a.tapmask) {
        if (threadIdx.x < 64) live_tile_map(a, tmap, threadIdx.x);
        __syncthreads();
    }
    const int lane = threadIdx.x % LANES;
    const int f = blockIdx.x * (256 / LANES) + threadIdx.x / LANES;
    const int ne = a.nent;
    float sum = 0.f;
    if (f < ne) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int b0 = lane; b0 < nblk; b0 += 8 * LANES) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (b0 + u * LANES < nblk) acc[u] += part[int64_t(b0 + u * LANES) * ne + f];
        }
        sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    sum = group_sum<LANES>(sum);
    float wg = 0.f, bs = 0.f;
    const int nfr = a.ntl * ntm * 256;
    if (f < ne && lane == 0) {
        if (f < nfr) {
            const int i = f & 3, ln = (f >> 2) & 63, q = f >> 8;  // q = tile * NTM + m
            int tt = q / ntm;
            const int m = q - tt * ntm;
            if (a.tapmask) tt = tmap[tt];
            const int co = m * 16 + (ln >> 4) * 4 + i;
            const int t2 = tt / a.ctile, jt = tt - t2 * a.ctile;
            const int e = 16 * jt + (ln & 15);
            const int kd = e / a.CS, c = e - kd * a.CS;
            if (co < a.N && kd < a.k && c < a.C) {
                const int K3 = a.k * a.k * a.k;
                const int64_t o = (int64_t(co) * a.wCt + c) * K3 + t2 * a.k + kd;
                if (dw) dw[o] += escale ? sum * *escale : sum;
                if (dscale) wg = w[o] * sum;
            }
        } else {
            if (dcbias) dcbias[f - nfr] += sum;
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

int ilog2w(int v) {
    int r = 0;
    while ((1 << r) < v) ++r;
    return r;
}
int pow2c(int v) {
    int r = 1;
    while (r < v) r *= 2;
    return r;
}

constexpr size_t kWLds = 160 * 1024 - 256;  // room for the static LDS

struct WPlan {
    WArgs a;
    int ntm, npw, ygroups, nbx;
    size_t lds;
    bool ok;
};

WPlan plan_w(const vq3d_conv_desc *d) {
    WPlan P = {};
    WArgs &a = P.a;
    if (d->dtype != VQ3D_HALF || d->kernel < 1 || d->cout > 64 || (d->cin2 && (d->cin + d->cin2) % 4)) return P;
    a.B = d->batch; a.Ca = d->cin; a.Cb = d->cin2; a.C = a.Ca + a.Cb; a.N = d->cout;
    a.CS = (a.C + 3) / 4 * 4;
    a.iH = d->in_h; a.iW = d->in_w; a.iD = d->in_d; a.oH = d->out_h; a.oW = d->out_w; a.oD = d->out_d;
    a.k = d->kernel; a.s = d->stride; a.p = d->pad; a.circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    a.wCt = a.C;
    P.ntm = (a.N + 15) / 16;
    a.GS = P.ntm * 16;
    a.ncol = a.k * a.CS;
    a.ctile = (a.ncol + 15) / 16;
    a.ntiles = a.k * a.k * a.ctile;
    a.tapmask = 0;
    a.ntl = a.ntiles;
    if (d->tap_mask && a.k <= 3 && a.ntiles <= kMaxMaskTiles) {  // only the tiles of live taps
        a.tapmask = d->tap_mask;
        int n = 0;
        for (int tt = 0; tt < a.ntiles; ++tt) n += wtile_live(tt, a);
        if (n > 0) a.ntl = n;
        else a.tapmask = 0;
    }
    // column tiles per wave: accumulators NTM * NPW * 4 VGPRs <= 112 (chosen after the bricks)
    const int cap = P.ntm == 1 ? 14 : (P.ntm == 2 ? 14 : 7);
    // brick: up to 512 voxels, full D when it fits
    auto set = [&](int bh, int bw, int bd) {
        a.bh = bh; a.bw = bw; a.bd = bd;
        a.lbw = ilog2w(bw); a.lbd = ilog2w(bd);
        a.hh = (bh - 1) * a.s + a.k; a.hw = (bw - 1) * a.s + a.k;
        a.LP = (bd - 1) * a.s + a.k;
        a.pad0 = (8 - (a.p * a.CS) % 8) % 8;
        a.LS = (a.pad0 + a.LP * a.CS + 16 + 7) / 8 * 8;
        a.nvb = bh * bw * bd;
        a.nvp = (a.nvb + 31) / 32 * 32;
    };
    auto lds_of = [&]() {  // lines, g tile, the live-tile map
        return ((size_t(a.hh) * a.hw * a.LS + 7) / 8 * 8) * 2 + size_t(a.nvp) * a.GS * 2 +
               (a.tapmask ? size_t(a.ntiles) * 2 : size_t(0));
    };
    int bd = std::min(pow2c(a.oD), 32);
    int bw = std::min(pow2c(a.oW), std::max(1, 512 / (bd * 4)));
    int bh = std::min(pow2c(a.oH), std::max(1, 512 / (bd * bw)));
    while (bh * bw * bd > 512) {
        if (bh > 1) bh /= 2; else if (bw > 1) bw /= 2; else bd /= 2;
    }
    set(bh, bw, bd);
    while (lds_of() > kWLds) {
        if (a.bh > 1) set(a.bh / 2, a.bw, a.bd);
        else if (a.bw > 1) set(a.bh, a.bw / 2, a.bd);
        else if (a.bd > 1) set(a.bh, a.bw, a.bd / 2);
        else return P;
    }
    // few bricks (small grids: the top levels' convs): smaller bricks, down to 64 voxels, until the
    // bricks x column groups cover the chip
    {
        const int cand[] = {1, 2, 4, 7, 14};
        int npw = 1;
        for (int c : cand) {
            if (c > cap) break;
            npw = c;
            if (4 * c >= a.ntl) break;
        }
        const int yg = (a.ntl + 4 * npw - 1) / (4 * npw);
        auto nbr = [&]() {
            return int64_t(a.B) * ((a.oH + a.bh - 1) / a.bh) * ((a.oW + a.bw - 1) / a.bw) * ((a.oD + a.bd - 1) / a.bd);
        };
        // (the partial rows the reduction reads grow with the bricks: at most ~8 MB of them)
        const int64_t nent = int64_t(a.ntl) * P.ntm * 256 + a.N;
        while (nbr() * yg < 256 && a.bh * a.bw * a.bd > 64 && 2 * nbr() * nent * 4 <= (int64_t(8) << 20)) {
            if (a.bh >= a.bw && a.bh > 1) set(a.bh / 2, a.bw, a.bd);
            else if (a.bw > 1) set(a.bh, a.bw / 2, a.bd);
            else set(a.bh, a.bw, a.bd / 2);
        }
    }
    a.nbh = (a.oH + a.bh - 1) / a.bh;
    a.nbw = (a.oW + a.bw - 1) / a.bw;
    a.nbd = (a.oD + a.bd - 1) / a.bd;
    a.nbricks = a.B * a.nbh * a.nbw * a.nbd;
    a.fC = FastDiv(uint32_t(a.CS));
    a.fhw = FastDiv(uint32_t(a.hw));
    a.fN = FastDiv(uint32_t(a.N));
    a.fCr = FastDiv(uint32_t(a.C));
    a.mc = (a.LP * a.C + 7) / 8 + 1;
    a.fmc = FastDiv(uint32_t(a.mc));
    a.xtotal = int64_t(a.B) * a.iH * a.iW * a.iD * a.C;
    a.gvec = (a.bd * a.N) % 8 == 0 && (int64_t(a.oD) * a.N) % 8 == 0;
    P.lds = lds_of();
    // Column tiles: as few column groups as the accumulator budget allows (each group
    // re-stages the bricks).  Bricks: ~1024 workgroups in all, each writing one partial G that
    // a fixed-order reduction sums (no atomics, deterministic).
    const int cands[] = {1, 2, 4, 7, 14};
    P.npw = 1;
    for (int c : cands) {
        if (c > cap) break;
        P.npw = c;
        if (4 * c >= a.ntl) break;
    }
    P.ygroups = (a.ntl + 4 * P.npw - 1) / (4 * P.npw);
    a.nent = a.ntl * P.ntm * 256 + a.N;
    int64_t nbx = std::max<int64_t>(1, std::min<int64_t>(a.nbricks, 1024 / P.ygroups));
    while (nbx > 1 && nbx * a.nent * 4 > (int64_t(16) << 20)) nbx /= 2;
    P.nbx = int(nbx);
    P.ok = true;
    if (std::getenv("VQ3D_VERBOSE"))
        std::fprintf(stderr, "[vq3d] lines wgrad C%d(CS%d)->N%d k%d s%d: brick %dx%dx%d ntm %d npw %d groups %d nbx %d lds %zu\n",
                     a.C, a.CS, a.N, a.k, a.s, a.bh, a.bw, a.bd, P.ntm, P.npw, P.ygroups, P.nbx, P.lds);
    return P;
}

}  // namespace

size_t lines_wgrad_workspace(const vq3d_conv_desc *d) {
    const WPlan P = plan_w(d);
    return P.ok ? size_t(P.nbx) * P.a.nent * 4 : 0;
}

namespace {


}  // namespace

bool lines_wgrad_applicable(const vq3d_conv_desc *d) { return plan_w(d).ok; }

int launch_lines_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pa,
                       const float *pb, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                       float *dcbias, void *ws, size_t ws_bytes, hipStream_t s) {
    WPlan P = plan_w(d);
    if (!P.ok) return fail("conv3d_bwd_weight(lines): geometry not supported");
    if (!ws || ws_bytes < size_t(P.nbx) * P.a.nent * 4) return fail("conv3d_bwd_weight(lines): workspace too small");
    float *part = static_cast<float *>(ws);
    P.a.pro_kind = d->pro_kind;
    P.a.pro_a = pa;
    P.a.pro_b = pb;
    const dim3 grid{unsigned(P.nbx), unsigned(P.ygroups), 1u};
    auto run = [&](auto ntm_c, auto npw_c) {
        constexpr int NTM = decltype(ntm_c)::value, NPW = decltype(npw_c)::value;
        auto kern = k_lines_wgrad<NTM, NPW>;
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      int(kWLds));
            (void)hipGetLastError();
            attr = true;
        }
        kern<<<grid, 256, P.lds, s>>>(P.a, (const h16_t *)x, (const h16_t *)x2, (const h16_t *)g, part);
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I7 = std::integral_constant<int, 7>;
    using I14 = std::integral_constant<int, 14>;
    auto by_npw = [&](auto ntm_c) {
        constexpr int NTM = decltype(ntm_c)::value;
        switch (P.npw) {
        case 1: run(ntm_c, I1{}); break;
        case 2: run(ntm_c, I2{}); break;
        case 4: run(ntm_c, I4{}); break;
        case 7: run(ntm_c, I7{}); break;
        default:
            if constexpr (NTM <= 2) run(ntm_c, I14{});
            else run(ntm_c, I7{});
            break;
        }
    };
    switch (P.ntm) {
    case 1: by_npw(I1{}); break;
    case 2: by_npw(I2{}); break;
    case 3: by_npw(I3{}); break;
    default: by_npw(I4{}); break;
    }
    int lanes = 1;
    while (lanes < 64 && lanes * 32 < P.nbx) lanes *= 2;
#define RED(L)                                                                                                 \
    k_lines_wgrad_reduce<L><<<(P.a.nent + 256 / L - 1) / (256 / L), 256, 0, s>>>(                                \
        P.a, P.ntm, part, P.nbx, w, escale, dw, dscale, dbias, dcbias,                                           \
        grid_sum_for(s, (P.a.nent + 256 / L - 1) / (256 / L), dscale || dbias))
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
    return check_launch("conv3d_bwd_weight(lines)");
}

}  // namespace vq3d
