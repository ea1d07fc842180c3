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

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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
    FastDiv fC, fhw, fN;
};

__device__ __forceinline__ s16x4 tr_read(const bf16_t *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 lo, s16x4 hi) {
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ int wrapw(int i, int n) {
    while (i < 0) i += n;
    while (i >= n) i -= n;
    return i;
}

template <int NTM, int NPW>
__global__ __launch_bounds__(256) void k_lines_wgrad(WArgs a, const bf16_t *__restrict__ x,
                                                    const bf16_t *__restrict__ x2, const bf16_t *__restrict__ g,
                                                    const float *__restrict__ w, const float *__restrict__ escale,
                                                    float *dw, float *dscale, float *dbias, float *dcbias) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ float red[8];
    const int nlines = a.hh * a.hw;
    bf16_t *lines = reinterpret_cast<bf16_t *>(smem);                             // [nlines][LS]
    bf16_t *gt = lines + ((nlines * a.LS + 7) / 8) * 8;                           // [nvp][GS]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const bool raw = pro.kind == VQ3D_PRO_NONE;
    const int tile0 = blockIdx.y * 4 * NPW;
    const bool do_bias = blockIdx.y == 0 && (dbias || dcbias);

    // this lane's B column offset (element) per owned tile: (kh, kw) line delta + column chunk
    int coff[NPW];
#pragma unroll
    for (int t = 0; t < NPW; ++t) {
        int tt = tile0 + wave + 4 * t;
        if (tt >= a.ntiles) tt = 0;  // padded tiles read valid addresses, are never written
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
        // the slack are zero.  Unit = one position's CS channels.
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
                bf16_t *dst = lines + ln * a.LS + a.pad0 + pos * a.CS;
                if (ok && a.Cb == 0 && (a.C & 3) == 0) {
                    const uint2 *src = reinterpret_cast<const uint2 *>(x + vox * a.C);
                    for (int c4 = 0; c4 < a.C / 4; ++c4) {
                        uint2 qv = src[c4];
                        if (!raw) {
                            auto f = [&](uint32_t uu) {
                                const float lo = pro.apply(__uint_as_float(uu << 16));
                                const float hi = pro.apply(__uint_as_float(uu & 0xffff0000u));
                                return uint32_t(f2bf(lo)) | (uint32_t(f2bf(hi)) << 16);
                            };
                            qv = uint2{f(qv.x), f(qv.y)};
                        }
                        reinterpret_cast<uint2 *>(dst)[c4] = qv;
                    }
                } else {
                    for (int c = 0; c < a.CS; ++c) {
                        bf16_t v = 0;
                        if (ok && c < a.C) {
                            const bf16_t *src = c < a.Ca ? x + vox * a.Ca + c : x2 + vox * a.Cb + (c - a.Ca);
                            v = raw ? *src : f2bf(pro.apply(ld(src)));
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
                    const bf16_t *el = reinterpret_cast<const bf16_t *>(&qv);
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
            bf16x8 af[NTM];
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
                const bf16x8 bfr = cat8(tr_read(lines + rb1 + coff[t]), tr_read(lines + rb2 + coff[t]));
#pragma unroll
                for (int m = 0; m < NTM; ++m)
                    acc[m][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr, acc[m][t], 0, 0, 0);
            }
        }
    }
    // ---- D[co][col]: lane column li -> window column, rows 4*grp + i -> co
    const float sc = escale ? *escale : 1.f;
    const int K3 = a.k * a.k * a.k;
    float wg = 0.f;
#pragma unroll
    for (int t = 0; t < NPW; ++t) {
        const int tt = tile0 + wave + 4 * t;
        if (tt >= a.ntiles) continue;
        const int t2 = tt / a.ctile, jt = tt - t2 * a.ctile;
        const int e = 16 * jt + li;  // window element (kd, c) with channel stride CS
        const int kd = int(a.fC.div(uint32_t(e))), c = e - kd * a.CS;
        if (kd >= a.k || c >= a.C) continue;
        const int tap = t2 * a.k + kd;
#pragma unroll
        for (int m = 0; m < NTM; ++m)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int co = m * 16 + grp * 4 + i;
                if (co >= a.N) continue;
                const int64_t o = (int64_t(co) * a.wCt + c) * K3 + tap;
                const float v = acc[m][t][i];
                if (dw) atomicAdd(dw + o, escale ? v * sc : v);
                if (dscale) wg = fmaf(w[o], v, wg);
            }
    }
    if (dscale) {
        wg = block_sum<float, 256>(wg, red);
        if (tid == 0) atomicAdd(dscale, wg);
    }
    if (do_bias) {
        if (dcbias && tid < a.N) atomicAdd(dcbias + tid, gsum);
        if (dbias) {
            const float tb = block_sum<float, 256>(tid < a.N ? gsum : 0.f, red + 4);
            if (tid == 0) atomicAdd(dbias, tb);
        }
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
    if (d->dtype != VQ3D_BF16 || d->kernel < 2 || d->cout > 64 || (d->cin + d->cin2) % 4) return P;
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
    auto lds_of = [&]() {
        return ((size_t(a.hh) * a.hw * a.LS + 7) / 8 * 8) * 2 + size_t(a.nvp) * a.GS * 2;
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
    a.nbh = (a.oH + a.bh - 1) / a.bh;
    a.nbw = (a.oW + a.bw - 1) / a.bw;
    a.nbd = (a.oD + a.bd - 1) / a.bd;
    a.nbricks = a.B * a.nbh * a.nbw * a.nbd;
    a.fC = FastDiv(uint32_t(a.CS));
    a.fhw = FastDiv(uint32_t(a.hw));
    a.fN = FastDiv(uint32_t(a.N));
    a.gvec = (a.bd * a.N) % 8 == 0 && (int64_t(a.oD) * a.N) % 8 == 0;
    P.lds = lds_of();
    // Every workgroup adds a partial of the whole (column-group slice of the) weight gradient,
    // so few voxels per workgroup means many atomics per voxel: give each workgroup >= 2
    // bricks (<= 64 adders per entry) and find parallelism in the column tiles instead
    // (fewer column tiles per wave -> more column groups).
    P.nbx = std::max(1, std::min(64, (a.nbricks + 1) / 2));
    const int cands[] = {1, 2, 4, 7, 14};
    P.npw = 1;
    for (int c : cands) {
        if (c > cap) break;
        P.npw = c;
        const int groups = (a.ntiles + 4 * c - 1) / (4 * c);
        if (int64_t(groups) * P.nbx <= 512) break;
    }
    P.ygroups = (a.ntiles + 4 * P.npw - 1) / (4 * P.npw);
    if (a.nbricks > 16 * P.nbx) return P;  // big grids: the brick-serial loop would be latency bound
    P.ok = true;
    if (std::getenv("VQ3D_VERBOSE"))
        std::fprintf(stderr, "[vq3d] lines wgrad C%d(CS%d)->N%d k%d s%d: brick %dx%dx%d ntm %d npw %d groups %d nbx %d lds %zu\n",
                     a.C, a.CS, a.N, a.k, a.s, a.bh, a.bw, a.bd, P.ntm, P.npw, P.ygroups, P.nbx, P.lds);
    return P;
}

bool wdisabled() {
    static const bool off = [] {
        const char *e = std::getenv("VQ3D_DISABLE_LINES_WGRAD");
        return e && e[0] == '1';
    }();
    return off;
}

}  // namespace

bool lines_wgrad_applicable(const vq3d_conv_desc *d) { return !wdisabled() && plan_w(d).ok; }

int launch_lines_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pa,
                       const float *pb, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                       float *dcbias, hipStream_t s) {
    WPlan P = plan_w(d);
    if (!P.ok) return fail("conv3d_bwd_weight(lines): geometry not supported");
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
        kern<<<grid, 256, P.lds, s>>>(P.a, (const bf16_t *)x, (const bf16_t *)x2, (const bf16_t *)g, w, escale, dw,
                                      dscale, dbias, dcbias);
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
    return check_launch("conv3d_bwd_weight(lines)");
}

}  // namespace vq3d
