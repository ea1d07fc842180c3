// 3-D convolution forward / backward-data / backward-weight for the VQ-VAE-2 path.
//
// Replaces nn.Conv3d (+ F.pad 'circular') at every reference call site
// (vqvae/layers.py:124-171 block convs, :535 parse_input, :377 / :490 proj, :508 out)
// together with the scalar glue around them (ELU(x+a)+b prologues, *scale + b
// epilogues, residual adds: layers.py:176-195, 277-290).
//
// Layout: activations channels-last [B][H][W][D][C] (fp32 or bf16 storage), fp32 math;
// weights fp32 [Cout][Cin][k][k][k] (reference layout, read straight from the param).
//
// Engines
//   pointwise (k = 1): a workgroup owns 256 consecutive voxels = one contiguous slab of
//     memory; input channels are staged through LDS in chunks (prologue applied once per
//     element), weights broadcast from LDS.  Forward and backward-data share the kernel.
//   k > 1: direct convolution, one thread = one output voxel x COT channels, all taps'
//     weights of the channel tile staged in LDS once.  Circular padding is index
//     arithmetic (out[o] = sum_t W[t] x[(s*o + t - p) mod H]); no padded copy exists.
//   weight gradient: thread = (row = (tap, ci), voxel sub-stream), g staged in LDS per
//     chunk of one output row; partial sums leave each workgroup as fp32 atomics straight
//     into the parameter-gradient buffer (no partial slabs, no finalize pass).
#include "common.h"
#include "conv_epi.h"
#include "engines.h"

#include <algorithm>
#include <map>
#include <utility>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "conv_mfma.inc"
namespace vq3d {

// ============================================================================ pointwise
constexpr int kMaxBlocksX = 2048;  // grid-stride cap (bounds the per-block scalar atomics)

// ============================================================================ forward, k > 1
// thread = one output voxel x COT channels (grid-stride over voxel blocks of 256)
template <typename T, int COT>
__global__ __launch_bounds__(256) void k_conv_fwd(ConvArgs a, const T *__restrict__ x, const T *__restrict__ x2,
                                                 const float *__restrict__ w, FwdEpi<T> fe, int all_taps,
                                                 T *__restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];  // [taps][Ct][COT]
    const int Ct = a.Cin + a.Cin2;
    const int K3 = a.k * a.k * a.k;
    const int64_t nvox = int64_t(a.B) * a.oH * a.oW * a.oD;
    const int co0 = blockIdx.y * COT;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);

    if (all_taps) {
        for (int i = threadIdx.x; i < K3 * Ct * COT; i += 256) {
            const int c = i % COT, r = i / COT, ci = r % Ct, tap = r / Ct;
            const int co = co0 + c;
            wsh[i] = co < a.Cout ? w[(int64_t(co) * Ct + ci) * K3 + tap] : 0.f;
        }
        __syncthreads();
    }
    for (int64_t vb = int64_t(blockIdx.x) * 256; vb < nvox; vb += int64_t(gridDim.x) * 256) {
        const int64_t v = vb + threadIdx.x;
        int od = 0, ow = 0, oh = 0, b = 0;
        if (v < nvox) {
            int64_t t = v;
            od = int(t % a.oD); t /= a.oD;
            ow = int(t % a.oW); t /= a.oW;
            oh = int(t % a.oH); b = int(t / a.oH);
        }
        float acc[COT];
#pragma unroll
        for (int c = 0; c < COT; ++c) acc[c] = 0.f;
        int tap = 0;
        for (int kh = 0; kh < a.k; ++kh) {
            const int ih = fwd_index(oh, kh, a.s, a.p, a.iH, a.circ);
            for (int kw = 0; kw < a.k; ++kw) {
                const int iw = fwd_index(ow, kw, a.s, a.p, a.iW, a.circ);
                for (int kd = 0; kd < a.k; ++kd, ++tap) {
                    const float *wt = wsh;
                    if (all_taps) {
                        wt = wsh + tap * Ct * COT;
                    } else {
                        __syncthreads();
                        for (int i = threadIdx.x; i < Ct * COT; i += 256) {
                            const int ci = i / COT, c = i - ci * COT;
                            const int co = co0 + c;
                            wsh[i] = co < a.Cout ? w[(int64_t(co) * Ct + ci) * K3 + tap] : 0.f;
                        }
                        __syncthreads();
                    }
                    if (v >= nvox) continue;
                    const int id = fwd_index(od, kd, a.s, a.p, a.iD, a.circ);
                    if ((ih | iw | id) < 0) continue;
                    const int64_t pos = ((int64_t(b) * a.iH + ih) * a.iW + iw) * a.iD + id;
                    const T *xp = x + pos * a.Cin;
                    for (int ci = 0; ci < a.Cin; ++ci) {
                        const float xv = pro.apply(ld(xp + ci));
                        const float *wr = wt + ci * COT;
#pragma unroll
                        for (int c = 0; c < COT; ++c) acc[c] = fmaf(xv, wr[c], acc[c]);
                    }
                    if (a.Cin2) {
                        const T *xq = x2 + pos * a.Cin2;
                        for (int ci = 0; ci < a.Cin2; ++ci) {
                            const float xv = pro.apply(ld(xq + ci));
                            const float *wr = wt + (a.Cin + ci) * COT;
#pragma unroll
                            for (int c = 0; c < COT; ++c) acc[c] = fmaf(xv, wr[c], acc[c]);
                        }
                    }
                }
            }
        }
        if (v < nvox) fwd_epilogue<T, COT>(a, fe, acc, v, co0, y + v * a.Cout);
    }
}

// ============================================================================ backward data, k > 1
template <typename T, int CIT>
__global__ __launch_bounds__(256) void k_conv_dgrad(ConvArgs a, const T *__restrict__ g, const float *__restrict__ gscale,
                                                   const float *__restrict__ w, BwdEpi<T> be, int all_taps,
                                                   T *__restrict__ gx, T *__restrict__ gx2, float *dpre,
                                                   float *dpost, GridSum gsum) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];  // [taps][Cout][CIT]
    __shared__ float red[8];
    const int Ct = a.Cin + a.Cin2;
    const int K3 = a.k * a.k * a.k;
    const int64_t nvox = int64_t(a.B) * a.iH * a.iW * a.iD;
    const int ci0 = blockIdx.y * CIT;
    const ActDeriv dv = make_deriv(be);
    const float gs = gscale ? *gscale : 1.f;
    float pre = 0.f, post = 0.f;

    if (all_taps) {
        for (int i = threadIdx.x; i < K3 * a.Cout * CIT; i += 256) {
            const int c = i % CIT, r = i / CIT, co = r % a.Cout, tap = r / a.Cout;
            const int ci = ci0 + c;
            wsh[i] = ci < Ct ? w[(int64_t(co) * Ct + ci) * K3 + tap] : 0.f;
        }
        __syncthreads();
    }
    for (int64_t vb = int64_t(blockIdx.x) * 256; vb < nvox; vb += int64_t(gridDim.x) * 256) {
        const int64_t v = vb + threadIdx.x;
        int id = 0, iw = 0, ih = 0, b = 0;
        if (v < nvox) {
            int64_t t = v;
            id = int(t % a.iD); t /= a.iD;
            iw = int(t % a.iW); t /= a.iW;
            ih = int(t % a.iH); b = int(t / a.iH);
        }
        float acc[CIT];
#pragma unroll
        for (int c = 0; c < CIT; ++c) acc[c] = 0.f;
        int tap = 0;
        for (int kh = 0; kh < a.k; ++kh) {
            const int oh = bwd_index(ih, kh, a.s, a.p, a.iH, a.oH, a.circ);
            for (int kw = 0; kw < a.k; ++kw) {
                const int ow = bwd_index(iw, kw, a.s, a.p, a.iW, a.oW, a.circ);
                for (int kd = 0; kd < a.k; ++kd, ++tap) {
                    const float *wt = wsh;
                    if (all_taps) {
                        wt = wsh + tap * a.Cout * CIT;
                    } else {
                        __syncthreads();
                        for (int i = threadIdx.x; i < a.Cout * CIT; i += 256) {
                            const int co = i / CIT, c = i - co * CIT;
                            const int ci = ci0 + c;
                            wsh[i] = ci < Ct ? w[(int64_t(co) * Ct + ci) * K3 + tap] : 0.f;
                        }
                        __syncthreads();
                    }
                    if (v >= nvox) continue;
                    const int od = bwd_index(id, kd, a.s, a.p, a.iD, a.oD, a.circ);
                    if ((oh | ow | od) < 0) continue;
                    const T *gp = g + (((int64_t(b) * a.oH + oh) * a.oW + ow) * a.oD + od) * a.Cout;
                    for (int co = 0; co < a.Cout; ++co) {
                        const float gv = ld(gp + co);
                        const float *wr = wt + co * CIT;
#pragma unroll
                        for (int c = 0; c < CIT; ++c) acc[c] = fmaf(gv, wr[c], acc[c]);
                    }
                }
            }
        }
        if (v < nvox)
            bwd_epilogue<T, CIT>(a, be, dv, gs, gscale != nullptr, acc, v, ci0, gx + v * a.Cin,
                                 gx2 ? gx2 + v * a.Cin2 : nullptr, pre, post);
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

// ============================================================================ backward weight
// Grid: x = voxel chunks, y = row tiles (row = ci * K3 + tap: the reference weight order, so a
// workgroup's atomics hit consecutive addresses; R rows per workgroup),
// z = co tiles of COT.  Thread = (row, voxel sub-stream vs), VS = 256 / R sub-streams.
// Each chunk is a run of consecutive output voxels inside one D-row, so the voxel
// coordinates advance without divisions.
constexpr int kWgChunk = 64;

template <typename T, int COT>
__global__ __launch_bounds__(256) void k_conv_wgrad(ConvArgs a, const T *__restrict__ x, const T *__restrict__ x2,
                                                   const T *__restrict__ g, int64_t rows_per_blk, int R,
                                                   const float *__restrict__ w, const float *__restrict__ escale,
                                                   float *dw, float *dscale, float *dbias, float *dcbias) {
    __shared__ __attribute__((aligned(16))) float gsh[kWgChunk][COT];
    __shared__ float racc[256][COT + 1];
    __shared__ float red[8];
    const int Ct = a.Cin + a.Cin2;
    const int K3 = a.k * a.k * a.k;
    const int Kt = Ct * K3;
    const int VS = 256 / R;
    const int tid = threadIdx.x;
    const int rl = tid % R, vs = tid / R;
    const int row = blockIdx.y * R + rl;
    const int co0 = blockIdx.z * COT;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const bool active = vs < VS && row < Kt;
    const int ci = active ? row / K3 : 0, tap = active ? row - (row / K3) * K3 : 0;
    const int kd = tap % a.k, kw = (tap / a.k) % a.k, kh = tap / (a.k * a.k);
    const bool second = ci >= a.Cin;
    const T *src = second ? x2 : x;
    const int srcC = second ? a.Cin2 : a.Cin;
    const int sci = second ? ci - a.Cin : ci;
    const bool pointwise = a.k == 1 && a.s == 1 && a.p == 0;

    float acc[COT];
#pragma unroll
    for (int c = 0; c < COT; ++c) acc[c] = 0.f;
    float gsum = 0.f;  // threads tid < COT of row tile 0 sum g[., co0 + tid]

    const int64_t nrows = int64_t(a.B) * a.oH * a.oW;  // output D-rows
    const int64_t r_begin = int64_t(blockIdx.x) * rows_per_blk;
    const int64_t r_end = min(nrows, r_begin + rows_per_blk);
    for (int64_t orow = r_begin; orow < r_end; ++orow) {
        const int ow = int(orow % a.oW);
        const int oh = int((orow / a.oW) % a.oH);
        const int b = int(orow / (int64_t(a.oW) * a.oH));
        const int ih = pointwise ? oh : fwd_index(oh, kh, a.s, a.p, a.iH, a.circ);
        const int iw = pointwise ? ow : fwd_index(ow, kw, a.s, a.p, a.iW, a.circ);
        const bool row_ok = (ih | iw) >= 0;
        const T *srow = src + ((int64_t(b) * a.iH + (ih < 0 ? 0 : ih)) * a.iW + (iw < 0 ? 0 : iw)) * a.iD * srcC;
        const int64_t gbase = orow * a.oD;
        for (int d0 = 0; d0 < a.oD; d0 += kWgChunk) {
            const int nv = min(kWgChunk, a.oD - d0);
            __syncthreads();
            for (int i = tid; i < kWgChunk * COT; i += 256) {
                const int vv = i / COT, c = i - vv * COT;
                gsh[vv][c] = (vv < nv && co0 + c < a.Cout) ? ld(g + (gbase + d0 + vv) * a.Cout + co0 + c) : 0.f;
            }
            __syncthreads();
            if (blockIdx.y == 0 && tid < COT) {
                for (int vv = 0; vv < nv; ++vv) gsum += gsh[vv][tid];
            }
            if (!active || !row_ok) continue;
            for (int vv = vs; vv < nv; vv += VS) {
                const int od = d0 + vv;
                const int id = pointwise ? od : fwd_index(od, kd, a.s, a.p, a.iD, a.circ);
                if (id < 0) continue;
                const float xv = pro.apply(ld(srow + int64_t(id) * srcC + sci));
#pragma unroll
                for (int c = 0; c < COT; ++c) acc[c] = fmaf(xv, gsh[vv][c], acc[c]);
            }
        }
    }
    // fixed-order reduction over the VS voxel sub-streams, then one atomic per entry
    __syncthreads();
#pragma unroll
    for (int c = 0; c < COT; ++c) racc[tid][c] = acc[c];
    __syncthreads();
    const float sc = escale ? *escale : 1.f;
    float wg = 0.f;
    if (vs == 0 && row < Kt) {
        const int ncot = min(COT, a.Cout - co0);
        for (int c = 0; c < ncot; ++c) {
            float s = 0.f;
            for (int j = 0; j < VS; ++j) s += racc[j * R + rl][c];
            const int64_t e = int64_t(co0 + c) * Kt + row;  // reference [co][ci][tap]: lanes contiguous
            if (dw) atomicAdd(dw + e, escale ? s * sc : s);
            if (dscale) wg = fmaf(w[e], s, wg);
        }
    }
    if (dscale) {
        wg = block_sum<float, 256>(wg, red);
        if (tid == 0) atomicAdd(dscale, wg);
    }
    if (blockIdx.y == 0) {
        if (dcbias && tid < COT && co0 + tid < a.Cout) atomicAdd(dcbias + co0 + tid, gsum);
        if (dbias) {
            const float t = block_sum<float, 256>(tid < COT && co0 + tid < a.Cout ? gsum : 0.f, red + 4);
            if (tid == 0) atomicAdd(dbias, t);
        }
    }
}

// ============================================================================ host side
static const int kTiles[] = {1, 2, 4, 8, 12, 16};

static int pick_tile(int c) {
    const int ntiles = (c + 15) / 16;
    const int per = (c + ntiles - 1) / ntiles;
    for (int o : kTiles)
        if (o >= per) return o;
    return 16;
}

// shrink the channel tile while the grid would leave the chip idle (tiny top-level grids)
static int pick_tile_for(int c, int64_t work_items, int64_t target = 65536) {
    int t = pick_tile(c);
    while (t > 1 && work_items * ((c + t - 1) / t) < target) {
        int smaller = 1;
        for (int o : kTiles)
            if (o < t) smaller = o;
        t = smaller;
    }
    return t;
}

static bool is_pointwise(const vq3d_conv_desc *d) { return d->kernel == 1 && d->stride == 1 && d->pad == 0; }

static int validate(const vq3d_conv_desc *d) {
    if (!d) return fail("conv: null descriptor");
    if (d->dtype != VQ3D_F32 && d->dtype != VQ3D_HALF) return fail("conv: bad dtype");
    if (d->batch <= 0 || d->cin <= 0 || d->cin2 < 0 || d->cout <= 0) return fail("conv: bad channel/batch");
    if (d->kernel <= 0 || d->stride <= 0 || d->pad < 0) return fail("conv: bad kernel/stride/pad");
    const int in[3] = {d->in_h, d->in_w, d->in_d}, out[3] = {d->out_h, d->out_w, d->out_d};
    for (int i = 0; i < 3; ++i) {
        if (in[i] <= 0 || out[i] <= 0) return fail("conv: bad spatial size");
        if ((in[i] + 2 * d->pad - d->kernel) / d->stride + 1 != out[i])
            return fail("conv: output size does not match (in + 2p - k)/s + 1");
        if (d->pad_mode == VQ3D_PAD_CIRCULAR && d->pad > in[i])
            return fail("conv: circular padding larger than the input");
        if (d->pad_mode == VQ3D_PAD_CIRCULAR && in[i] % d->stride)
            return fail("conv: circular strided conv needs size % stride == 0");
    }
    if (d->pro_kind < 0 || d->pro_kind > 2) return fail("conv: bad prologue");
    if ((int64_t(d->cin) + d->cin2) * 16 * 4 > 64 * 1024) return fail("conv: too many input channels");
    if (int64_t(d->cout) * 16 * 4 > 64 * 1024) return fail("conv: too many output channels");
    if (int64_t(d->batch) * d->in_h * d->in_w * d->in_d * (d->cin + d->cin2) > (int64_t(1) << 40))
        return fail("conv: tensor too large");
    return 0;
}

constexpr size_t kAllTapsLds = 48 * 1024;

static unsigned blocks_x(int64_t units) { return unsigned(std::max<int64_t>(1, std::min<int64_t>(units, kMaxBlocksX))); }

template <typename T>
static FwdEpi<T> make_fwd_epi(const vq3d_conv_epilogue *epi) {
    FwdEpi<T> e = {};
    if (epi) {
        e.scale = epi->scale;
        e.bias = epi->bias;
        e.cbias = epi->cbias;
        e.res = static_cast<const T *>(epi->residual);
        e.res_up2 = epi->residual_up2;
        e.act = epi->act;
        e.act_a = epi->act_a;
        e.act_b = epi->act_b;
    }
    return e;
}

template <typename T>
static BwdEpi<T> make_bwd_epi(const vq3d_dgrad_epilogue *epi, int pro_kind, const float *pro_a) {
    BwdEpi<T> e = {};
    if (epi) {
        e.aux = static_cast<const T *>(epi->aux);
        e.addend = static_cast<const T *>(epi->addend);
        if (epi->aux_kind == 1) {
            e.mode = 2;
            e.p = epi->aux_b;
        } else if (pro_kind == VQ3D_PRO_ELU_ADD) {
            e.mode = 1;
            e.p = pro_a;
        }
        if (!e.aux) e.mode = 0;
    }
    return e;
}

static bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// small grids with many channels: reduction split over workgroups (conv_small.hip)
static bool use_small(const vq3d_conv_desc *d, bool dgrad) {
    if (!small_applicable(d, dgrad)) return false;
    // measured: 9-20x faster than the lines / VALU engines at 128 voxels (8x8x2, 128 channels);
    // from 1024 voxels on only where the lines engine cannot take the shape
    const int64_t nv = dgrad ? int64_t(d->batch) * d->in_h * d->in_w * d->in_d
                             : int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    if (nv <= 512) return true;
    // matrix-core form up to VQ3D_SMALL_MMA_MAX voxels (default 512: the lines engine above)
    static const int64_t mma_max = [] {
        const char *e = std::getenv("VQ3D_SMALL_MMA_MAX");
        return e ? std::atoll(e) : int64_t(512);
    }();
    if (nv <= mma_max && small_mma_form(d, dgrad)) return true;
    if (dgrad && dgrad_s2_applicable(d)) return false;  // parity-tap engine measured 2x faster there
    return !lines_applicable(d, dgrad);
}

template <typename T>
static int launch_fwd(const vq3d_conv_desc *d, const void *x, const void *x2, const float *w, const float *pa,
                      const float *pb, const vq3d_conv_epilogue *epi, void *y, void *ws, size_t ws_bytes,
                      hipStream_t s) {
    ConvArgs a = make_args(d, pa, pb);
    const int64_t nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    FwdEpi<T> fe = make_fwd_epi<T>(epi);
    if (fe.res && fe.res_up2 && ((d->out_h | d->out_w | d->out_d) & 1))
        return fail("conv: residual_up2 needs even output");
    if (fe.act == VQ3D_ACT_ELU_AFFINE && (!fe.act_a || !fe.act_b)) return fail("conv: ELU_AFFINE needs act_a/b");
    if (is_pointwise(d)) {
        BwdEpi<T> be = {};
        return launch_pw1<T>(d, false, x, x2, w, pa, pb, fe, be, nullptr, y, nullptr, nullptr, nullptr, ws, ws_bytes,
                             s);
    }
    if (tc_applicable(d) && !(fe.res && fe.res_up2)) {
        BwdEpi<T> be = {};
        return launch_tc<T>(d, false, x, w, pa, pb, fe, be, nullptr, y, nullptr, nullptr, ws, ws_bytes, s);
    }
    if (use_small(d, false)) {
        BwdEpi<T> be = {};
        return launch_small<T>(d, false, x, x2, w, pa, pb, fe, be, nullptr, y, nullptr, nullptr, nullptr, ws, ws_bytes,
                               s);
    }
    if constexpr (std::is_same<T, h16_t>::value) {
        if (lines_applicable(d, false)) {
            BwdEpi<T> be = {};
            return launch_lines(d, false, x, x2, w, pa, pb, fe, be, nullptr, y, nullptr, nullptr, nullptr, ws,
                                ws_bytes, s);
        }
        {
            MPlan m = plan_mfma(d->batch, d->cin, d->cin2, d->cout, d->in_h, d->in_w, d->in_d, d->out_h, d->out_w,
                                d->out_d, d->kernel, d->stride, d->pad, d->pad_mode == VQ3D_PAD_CIRCULAR);
            if (m.ok) {
                m.a.pro_kind = d->pro_kind;
                m.a.pro_a = pa;
                m.a.pro_b = pb;
                m.a.wCt = d->cin + d->cin2;
                BwdEpi<T> be = {};
                return launch_mfma<false>(m, (const T *)x, (const T *)x2, w, fe, be, 0, nullptr, (T *)y, nullptr,
                                          nullptr, nullptr, s);
            }
        }
    }
    const int cot = pick_tile_for(d->cout, nvox);
    const int Ct = d->cin + d->cin2, K3 = d->kernel * d->kernel * d->kernel;
    const size_t all = size_t(K3) * Ct * cot * 4;
    const int all_taps = all <= kAllTapsLds;
    const size_t lds = all_taps ? all : size_t(Ct) * cot * 4;
    dim3 grid(blocks_x((nvox + 255) / 256), unsigned((d->cout + cot - 1) / cot));
#define L(C)                                                                                                   \
    case C:                                                                                                    \
        k_conv_fwd<T, C><<<grid, 256, lds, s>>>(a, (const T *)x, (const T *)x2, w, fe, all_taps, (T *)y);      \
        break;
    switch (cot) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch("conv3d_fwd");
}

template <typename T>
static int launch_dgrad(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w,
                        const float *pa, const vq3d_dgrad_epilogue *epi, void *gx, void *gx2, float *dpre,
                        float *dpost, void *ws, size_t ws_bytes, hipStream_t s) {
    ConvArgs a = make_args(d, pa, nullptr);
    const int Ct = d->cin + d->cin2;
    const int64_t nvox = int64_t(d->batch) * d->in_h * d->in_w * d->in_d;
    const int cit = pick_tile_for(Ct, nvox);
    BwdEpi<T> be = make_bwd_epi<T>(epi, d->pro_kind, pa);
    if (is_pointwise(d)) {
        FwdEpi<T> fe = {};
        return launch_pw1<T>(d, true, g, nullptr, w, pa, nullptr, fe, be, gscale, gx, gx2, dpre, dpost, ws, ws_bytes,
                             s);
    }
    if (tc_applicable(d)) {
        FwdEpi<T> fe = {};
        return launch_tc<T>(d, true, g, w, pa, nullptr, fe, be, gscale, gx, dpre, dpost, ws, ws_bytes, s);
    }
    if (use_small(d, true)) {
        FwdEpi<T> fe = {};
        return launch_small<T>(d, true, g, nullptr, w, pa, nullptr, fe, be, gscale, gx, gx2, dpre, dpost, ws, ws_bytes,
                               s);
    }
    if constexpr (std::is_same<T, h16_t>::value) {
        // stride-1 backward-data == forward conv of g with the flipped, transposed kernel
        if (lines_applicable(d, true)) {
            FwdEpi<T> fe = {};
            return launch_lines(d, true, g, nullptr, w, pa, nullptr, fe, be, gscale, gx, gx2, dpre, dpost, ws,
                                ws_bytes, s);
        }
        if (d->stride == 1) {
            const int pp = d->kernel - 1 - d->pad;
            MPlan m = plan_mfma(d->batch, d->cout, 0, Ct, d->out_h, d->out_w, d->out_d, d->in_h, d->in_w, d->in_d,
                                d->kernel, 1, pp, d->pad_mode == VQ3D_PAD_CIRCULAR);
            if (m.ok && pp >= 0) {
                m.a.pro_kind = VQ3D_PRO_NONE;
                m.a.wCt = Ct;
                FwdEpi<T> fe = {};
                return launch_mfma<true>(m, (const T *)g, nullptr, w, fe, be, d->cin, gscale, (T *)gx, (T *)gx2,
                                         dpre, dpost, s);
            }
        }
    }
    if (dgrad_s2_applicable(d)) return launch_dgrad_s2<T>(d, g, gscale, w, be, gx, gx2, dpre, dpost, s);
    const int K3 = d->kernel * d->kernel * d->kernel;
    const size_t all = size_t(K3) * d->cout * cit * 4;
    const int all_taps = all <= kAllTapsLds;
    const size_t lds = all_taps ? all : size_t(d->cout) * cit * 4;
    dim3 grid(blocks_x((nvox + 255) / 256), unsigned((Ct + cit - 1) / cit));
#define L(C)                                                                                                  \
    case C:                                                                                                   \
        k_conv_dgrad<T, C><<<grid, 256, lds, s>>>(a, (const T *)g, gscale, w, be, all_taps, (T *)gx, (T *)gx2,  \
                                                  dpre, dpost, grid_sum_for(s, int64_t(grid.x) * grid.y,     \
                                                                            dpre || dpost));                  \
        break;
    switch (cit) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch("conv3d_bwd_data");
}

// k^3 weight gradient engine choice (bf16): the lines engine for wide inputs (>= 32 channels:
// 36 -> 36 at 32x32x8 runs 4.7x faster than the direct MFMA engine) or where the direct engine
// does not apply; the direct engine for the few-channel large grids, where it is measured
// faster (9 -> 9 at 128^2 x 32 on par, 4 -> 4 at 256^2 x 64 1.9x).
static bool use_lines_wgrad(const vq3d_conv_desc *d) {
    if (d->dtype != VQ3D_HALF || !lines_wgrad_applicable(d)) return false;
    // grids up to VQ3D_WGRAD_MFMA_MAX output voxels go to the direct engine even when wide (A/B;
    // default 0: the lines engine for every wide input)
    static const int64_t mfma_max = [] {
        const char *e = std::getenv("VQ3D_WGRAD_MFMA_MAX");
        return e ? std::atoll(e) : int64_t(0);
    }();
    const int64_t nv = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    if (nv <= mfma_max && plan_mfma(d->batch, d->cin, d->cin2, d->cout, d->in_h, d->in_w, d->in_d, d->out_h, d->out_w,
                                    d->out_d, d->kernel, d->stride, d->pad, d->pad_mode == VQ3D_PAD_CIRCULAR, true)
                              .ok)
        return false;
    if (d->cin + d->cin2 >= 32) return true;
    return !plan_mfma(d->batch, d->cin, d->cin2, d->cout, d->in_h, d->in_w, d->in_d, d->out_h, d->out_w, d->out_d,
                      d->kernel, d->stride, d->pad, d->pad_mode == VQ3D_PAD_CIRCULAR, true)
                .ok;
}

// the generic engines' image workspace (deterministic path; without it they fall back to atomics)
static size_t generic_wgrad_ws(const vq3d_conv_desc *d) {
    if (d->dtype != VQ3D_HALF || use_lines_wgrad(d) || d->kernel == 1) return 0;
    MPlan m = plan_mfma(d->batch, d->cin, d->cin2, d->cout, d->in_h, d->in_w, d->in_d, d->out_h, d->out_w, d->out_d,
                        d->kernel, d->stride, d->pad, d->pad_mode == VQ3D_PAD_CIRCULAR, true);
    if (!m.ok) return 0;
    m.a.wCt = d->cin + d->cin2;
    return gen_wgrad_bytes(gen_wgrad_geom(m), d->cout);
}

template <typename T>
static int launch_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pa,
                        const float *pb, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                        float *dcbias, void *ws, size_t ws_bytes, hipStream_t s) {
    ConvArgs a = make_args(d, pa, pb);
    const int Ct = d->cin + d->cin2;
    const int K3 = d->kernel * d->kernel * d->kernel;
    const int Kt = Ct * K3;
    if (is_pointwise(d)) {
        return launch_pw_wgrad(d, x, x2, g, pa, pb, w, escale, dw, dscale, dbias, dcbias, ws, ws_bytes, s);
    }
    if (tc_applicable(d))
        return launch_tc_wgrad<T>(d, x, g, pa, pb, w, escale, dw, dscale, dbias, dcbias, ws, ws_bytes, s);
    if constexpr (std::is_same<T, h16_t>::value) {
        if (mid_w2grad_ok(d) && dw && !escale && !dscale && !dbias && !dcbias && ws && ws_bytes >= mid_w2grad_ws(d))
            return mid_w2grad(d, x, g, dw, ws, ws_bytes, s);
        if (wgrad_ds_ok(d) && dw && !escale && !dscale && !dcbias && ws && ws_bytes >= wgrad_ds_ws(d))
            return wgrad_ds(d, x, g, pa, pb, dw, dbias, ws, ws_bytes, s);
        if (use_lines_wgrad(d))
            return launch_lines_wgrad(d, x, x2, g, pa, pb, w, escale, dw, dscale, dbias, dcbias, ws, ws_bytes, s);
        {
            MPlan m = plan_mfma(d->batch, d->cin, d->cin2, d->cout, d->in_h, d->in_w, d->in_d, d->out_h, d->out_w,
                                d->out_d, d->kernel, d->stride, d->pad, d->pad_mode == VQ3D_PAD_CIRCULAR, true);
            if (m.ok) {
                m.a.pro_kind = d->pro_kind;
                m.a.pro_a = pa;
                m.a.pro_b = pb;
                m.a.wCt = Ct;
                // MFMA engine holds up to 4 tiles of 16 output channels; wider outputs (the top levels'
                // 128-channel convs on 128..1,024 voxels) stay on the VALU tiled kernel: 64-channel
                // chunks on the matrix cores measured slower there (r04f / r04g: 57 vs 48.7 us at
                // 128 -> 128 @8x8x2, 212 vs 155 us at 64 -> 128 k4 s2 @32x32x8)
                if (d->cout <= 64)
                    return launch_wgrad_mfma(m, (const T *)x, (const T *)x2, (const T *)g, w, escale, dw, dscale,
                                             dbias, dcbias, ws, ws_bytes, s);
                return launch_wgrad_tiled(m, (const T *)x, (const T *)x2, (const T *)g, w, escale, dw, dscale,
                                          dbias, dcbias, ws, ws_bytes, s);
            }
        }
    }
    // rows per workgroup: all rows when they fit (voxel sub-streams fill the rest), else 256
    const int R = Kt >= 256 ? 256 : (Kt > 128 ? Kt : std::max(1, Kt));
    const int ytiles = (Kt + R - 1) / R;
    const int64_t nrows = int64_t(d->batch) * d->out_h * d->out_w;
    const int64_t min_rows = std::max<int64_t>(1, 64 / std::max(1, d->out_d));
    const int64_t max_nbx = (nrows + min_rows - 1) / min_rows;
    // channel tile: shrink it while there are too few workgroups to fill the chip
    int cot = pick_tile(d->cout);
    while (cot > 1 && int64_t(ytiles) * ((d->cout + cot - 1) / cot) * std::min<int64_t>(max_nbx, 2048) < 512) {
        int smaller = 1;
        for (int o : kTiles)
            if (o < cot) smaller = o;
        cot = smaller;
    }
    const int ztiles = (d->cout + cot - 1) / cot;
    const int64_t tiles = int64_t(ytiles) * ztiles;
    int64_t nbx = std::max<int64_t>(1, 1024 / tiles);  // x tiles: bounds the atomic traffic (nbx * E)
    nbx = std::min<int64_t>(nbx, max_nbx);
    const int64_t rows_per_blk = (nrows + nbx - 1) / nbx;
    nbx = (nrows + rows_per_blk - 1) / rows_per_blk;
    dim3 grid((unsigned)nbx, (unsigned)ytiles, (unsigned)ztiles);
#define L(C)                                                                                                   \
    case C:                                                                                                    \
        k_conv_wgrad<T, C><<<grid, 256, 0, s>>>(a, (const T *)x, (const T *)x2, (const T *)g, rows_per_blk, R,  \
                                                w, escale, dw, dscale, dbias, dcbias);                         \
        break;
    switch (cot) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch("conv3d_bwd_weight");
}

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_conv3d_fwd(const vq3d_conv_desc *d, const void *x, const void *x2, const float *w, const float *pro_a,
                    const float *pro_b, const vq3d_conv_epilogue *epi, void *y, void *workspace,
                    size_t workspace_bytes, vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!x || !w || !y || (d->cin2 && !x2)) return fail("conv3d_fwd: null pointer");
    if (d->pro_kind != VQ3D_PRO_NONE && !pro_a) return fail("conv3d_fwd: prologue needs pro_a");
    if (d->pro_kind == VQ3D_PRO_ELU_ADD && !pro_b) return fail("conv3d_fwd: ELU prologue needs pro_b");
    hipStream_t s = as_stream(stream);
    return d->dtype == VQ3D_F32
               ? launch_fwd<float>(d, x, x2, w, pro_a, pro_b, epi, y, workspace, workspace_bytes, s)
               : launch_fwd<h16_t>(d, x, x2, w, pro_a, pro_b, epi, y, workspace, workspace_bytes, s);
}

int vq3d_conv3d_bwd_data(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w,
                         const float *pro_a, const vq3d_dgrad_epilogue *epi, void *gx, void *gx2, float *dpro_pre,
                         float *dpro_post, void *workspace, size_t workspace_bytes, vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!g || !w || !gx || (d->cin2 && !gx2)) return fail("conv3d_bwd_data: null pointer");
    if (d->pro_kind != VQ3D_PRO_NONE && !pro_a) return fail("conv3d_bwd_data: prologue needs pro_a");
    if (epi && epi->aux_kind == 1 && epi->aux && !epi->aux_b)
        return fail("conv3d_bwd_data: aux_kind 1 needs aux_b");
    hipStream_t s = as_stream(stream);
    return d->dtype == VQ3D_F32
               ? launch_dgrad<float>(d, g, gscale, w, pro_a, epi, gx, gx2, dpro_pre, dpro_post, workspace,
                                     workspace_bytes, s)
               : launch_dgrad<h16_t>(d, g, gscale, w, pro_a, epi, gx, gx2, dpro_pre, dpro_post, workspace,
                                      workspace_bytes, s);
}

size_t vq3d_conv3d_workspace_size(const vq3d_conv_desc *d, int32_t pass) {
    if (validate(d)) return 0;
    if (tc_applicable(d)) return tc_workspace(d, pass);
    if (pass != VQ3D_PASS_BWD_WEIGHT && !is_pointwise(d) && use_small(d, pass == VQ3D_PASS_BWD_DATA))
        return small_workspace(d, pass == VQ3D_PASS_BWD_DATA);
    if (pass == VQ3D_PASS_FWD) return lines_workspace(d, false);
    if (pass == VQ3D_PASS_BWD_DATA) return is_pointwise(d) ? pw_dgrad_workspace(d) : lines_workspace(d, true);
    if (is_pointwise(d)) return pw_wgrad_workspace(d);
    return std::max({use_lines_wgrad(d) ? lines_wgrad_workspace(d) : size_t(0), mid_w2grad_ws(d), wgrad_ds_ws(d),
                     generic_wgrad_ws(d)});
}

int vq3d_conv3d_bwd_weight(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pro_a,
                           const float *pro_b, const float *w, const float *epi_scale, float *dw, float *dscale,
                           float *dbias, float *dcbias, void *workspace, size_t workspace_bytes,
                           vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!x || !g || (d->cin2 && !x2)) return fail("conv3d_bwd_weight: null pointer");
    if (d->pro_kind != VQ3D_PRO_NONE && !pro_a) return fail("conv3d_bwd_weight: prologue needs pro_a");
    if (d->pro_kind == VQ3D_PRO_ELU_ADD && !pro_b) return fail("conv3d_bwd_weight: ELU prologue needs pro_b");
    if (dscale && (!w || !epi_scale)) return fail("conv3d_bwd_weight: dscale needs w and epi_scale");
    hipStream_t s = as_stream(stream);
    return d->dtype == VQ3D_F32 ? launch_wgrad<float>(d, x, x2, g, pro_a, pro_b, w, epi_scale, dw, dscale, dbias,
                                                      dcbias, workspace, workspace_bytes, s)
                                : launch_wgrad<h16_t>(d, x, x2, g, pro_a, pro_b, w, epi_scale, dw, dscale, dbias,
                                                       dcbias, workspace, workspace_bytes, s);
}

}  // extern "C"
