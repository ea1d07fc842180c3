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
// v1 engine: direct convolution on the VALU with the per-tap weight slice staged in LDS
// and broadcast to the wave; one thread = one output voxel x COT channels.  Circular
// padding is index arithmetic (out[o] = sum_t W[t] x[(s*o + t - p) mod H]), so no padded
// copy is ever materialised.
#include "common.h"

#include <algorithm>

namespace vq3d {

struct ConvArgs {
    int B, Cin, Cin2, Cout;
    int iH, iW, iD, oH, oW, oD;
    int k, s, p, circ;
    int pro_kind;
    const float *pro_a, *pro_b;
};

static ConvArgs make_args(const vq3d_conv_desc *d, const float *pa, const float *pb) {
    ConvArgs a;
    a.B = d->batch;
    a.Cin = d->cin;
    a.Cin2 = d->cin2;
    a.Cout = d->cout;
    a.iH = d->in_h; a.iW = d->in_w; a.iD = d->in_d;
    a.oH = d->out_h; a.oW = d->out_w; a.oD = d->out_d;
    a.k = d->kernel; a.s = d->stride; a.p = d->pad; a.circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    a.pro_kind = d->pro_kind;
    a.pro_a = pa;
    a.pro_b = pb;
    return a;
}

// forward tap: output coordinate o, kernel offset t -> input coordinate, or -1 if in zero padding
__device__ __forceinline__ int fwd_index(int o, int t, int s, int p, int n, int circ) {
    int i = o * s + t - p;
    if (circ) {
        i %= n;
        return i < 0 ? i + n : i;
    }
    return (i < 0 || i >= n) ? -1 : i;
}

// transposed tap: input coordinate i, kernel offset t -> output coordinate o with
// fwd_index(o, t) == i, or -1 if none (unique when it exists: see DESIGN.md §conv)
__device__ __forceinline__ int bwd_index(int i, int t, int s, int p, int n_in, int n_out, int circ) {
    int r = i - t + p;
    if (circ) {
        r %= n_in;
        if (r < 0) r += n_in;
    } else if (r < 0) {
        return -1;
    }
    if (r % s) return -1;
    r /= s;
    return r < n_out ? r : -1;
}

// ============================================================================ forward
template <typename T, int COT>
__global__ __launch_bounds__(256) void k_conv_fwd(ConvArgs a, const T *__restrict__ x, const T *__restrict__ x2,
                                                 const float *__restrict__ w, const float *__restrict__ e_scale,
                                                 const float *__restrict__ e_bias, const float *__restrict__ e_cbias,
                                                 const T *__restrict__ res, int res_up2, int post_elu,
                                                 T *__restrict__ y) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];  // [Ct][COT]
    const int Ct = a.Cin + a.Cin2;
    const int K3 = a.k * a.k * a.k;
    const int64_t nvox = int64_t(a.B) * a.oH * a.oW * a.oD;
    const int64_t v = int64_t(blockIdx.x) * 256 + threadIdx.x;
    const int co0 = blockIdx.y * COT;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);

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

    for (int tap = 0; tap < K3; ++tap) {
        __syncthreads();
        for (int i = threadIdx.x; i < Ct * COT; i += 256) {
            const int ci = i / COT, c = i - ci * COT;
            const int co = co0 + c;
            wsh[i] = co < a.Cout ? w[(int64_t(co) * Ct + ci) * K3 + tap] : 0.f;
        }
        __syncthreads();
        if (v >= nvox) continue;
        const int kd = tap % a.k, kw = (tap / a.k) % a.k, kh = tap / (a.k * a.k);
        const int ih = fwd_index(oh, kh, a.s, a.p, a.iH, a.circ);
        const int iw = fwd_index(ow, kw, a.s, a.p, a.iW, a.circ);
        const int id = fwd_index(od, kd, a.s, a.p, a.iD, a.circ);
        if ((ih | iw | id) < 0) continue;
        const int64_t pos = ((int64_t(b) * a.iH + ih) * a.iW + iw) * a.iD + id;
        const T *xp = x + pos * a.Cin;
        for (int ci = 0; ci < a.Cin; ++ci) {
            const float xv = pro.apply(ld(xp + ci));
            const float *wr = wsh + ci * COT;
#pragma unroll
            for (int c = 0; c < COT; ++c) acc[c] = fmaf(xv, wr[c], acc[c]);
        }
        if (a.Cin2) {
            const T *xq = x2 + pos * a.Cin2;
            for (int ci = 0; ci < a.Cin2; ++ci) {
                const float xv = pro.apply(ld(xq + ci));
                const float *wr = wsh + (a.Cin + ci) * COT;
#pragma unroll
                for (int c = 0; c < COT; ++c) acc[c] = fmaf(xv, wr[c], acc[c]);
            }
        }
    }
    if (v >= nvox) return;
    const float sc = e_scale ? *e_scale : 1.f;
    const float bi = e_bias ? *e_bias : 0.f;
    T *yp = y + v * a.Cout;
    // residual on the half grid, upsampled on the fly: 8-point trilinear stencil
    int h0 = 0, h1 = 0, w0 = 0, w1 = 0, d0 = 0, d1 = 0;
    float lh = 0.f, lw = 0.f, ldd = 0.f;
    int rH = a.oH / 2, rW = a.oW / 2, rD = a.oD / 2;
    if (res && res_up2) {
        up_coeff(oh, rH, h0, h1, lh);
        up_coeff(ow, rW, w0, w1, lw);
        up_coeff(od, rD, d0, d1, ldd);
    }
#pragma unroll
    for (int c = 0; c < COT; ++c) {
        const int co = co0 + c;
        if (co >= a.Cout) break;
        float val = acc[c];
        if (e_scale) val = val * sc;
        if (e_bias) val = val + bi;
        if (e_cbias) val = val + e_cbias[co];
        if (res) {
            if (!res_up2) {
                val = val + ld(res + v * a.Cout + co);
            } else {
                auto R = [&](int hh, int ww, int dd) {
                    return ld(res + (((int64_t(b) * rH + hh) * rW + ww) * rD + dd) * a.Cout + co);
                };
                const float r = (1.f - lh) * ((1.f - lw) * ((1.f - ldd) * R(h0, w0, d0) + ldd * R(h0, w0, d1)) +
                                              lw * ((1.f - ldd) * R(h0, w1, d0) + ldd * R(h0, w1, d1))) +
                                lh * ((1.f - lw) * ((1.f - ldd) * R(h1, w0, d0) + ldd * R(h1, w0, d1)) +
                                      lw * ((1.f - ldd) * R(h1, w1, d0) + ldd * R(h1, w1, d1)));
                val = val + r;
            }
        }
        if (post_elu) val = elu(val);
        st(yp + co, val);
    }
}

// ============================================================================ backward data
// thread = one input voxel x CIT input channels; partial sums of the epilogue scalars
// (pre, post) per block -> spart[block][2]
template <typename T, int CIT>
__global__ __launch_bounds__(256) void k_conv_dgrad(ConvArgs a, const T *__restrict__ g, const float *__restrict__ gscale,
                                                   const float *__restrict__ w, const T *__restrict__ aux,
                                                   const T *__restrict__ addend, T *__restrict__ gx,
                                                   T *__restrict__ gx2, float *__restrict__ spart) {
    extern __shared__ __attribute__((aligned(16))) float wsh[];  // [Cout][CIT]
    __shared__ float red[8];
    const int Ct = a.Cin + a.Cin2;
    const int K3 = a.k * a.k * a.k;
    const int64_t nvox = int64_t(a.B) * a.iH * a.iW * a.iD;
    const int64_t v = int64_t(blockIdx.x) * 256 + threadIdx.x;
    const int ci0 = blockIdx.y * CIT;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, nullptr);

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

    for (int tap = 0; tap < K3; ++tap) {
        __syncthreads();
        for (int i = threadIdx.x; i < a.Cout * CIT; i += 256) {
            const int co = i / CIT, c = i - co * CIT;
            const int ci = ci0 + c;
            wsh[i] = ci < Ct ? w[(int64_t(co) * Ct + ci) * K3 + tap] : 0.f;
        }
        __syncthreads();
        if (v >= nvox) continue;
        const int kd = tap % a.k, kw = (tap / a.k) % a.k, kh = tap / (a.k * a.k);
        const int oh = bwd_index(ih, kh, a.s, a.p, a.iH, a.oH, a.circ);
        const int ow = bwd_index(iw, kw, a.s, a.p, a.iW, a.oW, a.circ);
        const int od = bwd_index(id, kd, a.s, a.p, a.iD, a.oD, a.circ);
        if ((oh | ow | od) < 0) continue;
        const T *gp = g + (((int64_t(b) * a.oH + oh) * a.oW + ow) * a.oD + od) * a.Cout;
        for (int co = 0; co < a.Cout; ++co) {
            const float gv = ld(gp + co);
            const float *wr = wsh + co * CIT;
#pragma unroll
            for (int c = 0; c < CIT; ++c) acc[c] = fmaf(gv, wr[c], acc[c]);
        }
    }
    float pre = 0.f, post = 0.f;
    if (v < nvox) {
        const float gs = gscale ? *gscale : 1.f;
#pragma unroll
        for (int c = 0; c < CIT; ++c) {
            const int ci = ci0 + c;
            if (ci >= Ct) break;
            float val = acc[c];
            if (gscale) val = val * gs;
            if (ci < a.Cin) {
                const int64_t o = v * a.Cin + ci;
                pre += val;
                if (aux && pro.kind == VQ3D_PRO_ELU_ADD) val = val * pro.deriv(ld(aux + o));
                post += val;
                if (addend) val = val + ld(addend + o);
                st(gx + o, val);
            } else {
                st(gx2 + v * a.Cin2 + (ci - a.Cin), val);
            }
        }
    }
    pre = block_sum<float, 256>(pre, red);
    post = block_sum<float, 256>(post, red + 4);
    if (threadIdx.x == 0) {
        const int blk = blockIdx.y * gridDim.x + blockIdx.x;
        spart[2 * blk] = pre;
        spart[2 * blk + 1] = post;
    }
}

// ============================================================================ backward weight
// Grid: x = voxel chunks, y = row tiles (row = tap * Ct + ci), z = co tiles of COT.
// Thread = (row, voxel sub-stream vs); g for a chunk of voxels is staged in LDS and
// broadcast.  Output: wpart[bx][co][ci][tap] (fp32 partial slab of chunk bx), gpart[bx][co].
constexpr int kWgChunk = 64;

template <typename T, int COT>
__global__ __launch_bounds__(256) void k_conv_wgrad(ConvArgs a, const T *__restrict__ x, const T *__restrict__ x2,
                                                   const T *__restrict__ g, int64_t vox_per_blk, int rows_per_wg,
                                                   float *__restrict__ wpart, float *__restrict__ gpart) {
    __shared__ float gsh[kWgChunk][COT];
    __shared__ float racc[256][COT + 1];
    const int Ct = a.Cin + a.Cin2;
    const int K3 = a.k * a.k * a.k;
    const int Kt = Ct * K3;
    const int64_t nvox = int64_t(a.B) * a.oH * a.oW * a.oD;
    const int R = rows_per_wg, VS = 256 / rows_per_wg;
    const int rl = threadIdx.x % R, vs = threadIdx.x / R;
    const int row = blockIdx.y * R + rl;
    const int co0 = blockIdx.z * COT;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const bool active = row < Kt;
    const int tap = active ? row / Ct : 0, ci = active ? row - (row / Ct) * Ct : 0;
    const int kd = tap % a.k, kw = (tap / a.k) % a.k, kh = tap / (a.k * a.k);
    const bool second = ci >= a.Cin;
    const T *src = second ? x2 : x;
    const int srcC = second ? a.Cin2 : a.Cin;
    const int sci = second ? ci - a.Cin : ci;

    float acc[COT];
#pragma unroll
    for (int c = 0; c < COT; ++c) acc[c] = 0.f;
    float gsum = 0.f;  // thread c < COT of (blockIdx.y == 0) sums g[., co0 + c]

    const int64_t v_begin = int64_t(blockIdx.x) * vox_per_blk;
    const int64_t v_end = min(nvox, v_begin + vox_per_blk);
    for (int64_t v0 = v_begin; v0 < v_end; v0 += kWgChunk) {
        __syncthreads();
        for (int i = threadIdx.x; i < kWgChunk * COT; i += 256) {
            const int vv = i / COT, c = i - vv * COT;
            const int64_t vg = v0 + vv;
            gsh[vv][c] = (vg < v_end && co0 + c < a.Cout) ? ld(g + vg * a.Cout + co0 + c) : 0.f;
        }
        __syncthreads();
        if (blockIdx.y == 0 && threadIdx.x < COT) {
            for (int vv = 0; vv < kWgChunk; ++vv) gsum += gsh[vv][threadIdx.x];
        }
        if (!active) continue;
        const int nv = int(min<int64_t>(kWgChunk, v_end - v0));
        for (int vv = vs; vv < nv; vv += VS) {
            int64_t t = v0 + vv;
            const int od = int(t % a.oD); t /= a.oD;
            const int ow = int(t % a.oW); t /= a.oW;
            const int oh = int(t % a.oH);
            const int b = int(t / a.oH);
            const int ih = fwd_index(oh, kh, a.s, a.p, a.iH, a.circ);
            const int iw = fwd_index(ow, kw, a.s, a.p, a.iW, a.circ);
            const int id = fwd_index(od, kd, a.s, a.p, a.iD, a.circ);
            if ((ih | iw | id) < 0) continue;
            const float xv =
                pro.apply(ld(src + (((int64_t(b) * a.iH + ih) * a.iW + iw) * a.iD + id) * srcC + sci));
#pragma unroll
            for (int c = 0; c < COT; ++c) acc[c] = fmaf(xv, gsh[vv][c], acc[c]);
        }
    }
    // fixed-order reduction over the VS voxel sub-streams
    __syncthreads();
#pragma unroll
    for (int c = 0; c < COT; ++c) racc[threadIdx.x][c] = acc[c];
    __syncthreads();
    if (vs == 0 && active) {
        const int ncot = min(COT, a.Cout - co0);
        for (int c = 0; c < ncot; ++c) {
            float s = 0.f;
            for (int j = 0; j < VS; ++j) s += racc[j * R + rl][c];
            wpart[(int64_t(blockIdx.x) * a.Cout + co0 + c) * Kt + int64_t(ci) * K3 + tap] = s;  // reference [co][ci][tap]
        }
    }
    if (blockIdx.y == 0 && threadIdx.x < COT && co0 + threadIdx.x < a.Cout)
        gpart[int64_t(blockIdx.x) * a.Cout + co0 + threadIdx.x] = gsum;
}

// ============================================================================ finalize
// one workgroup per 256 weight entries (or a single workgroup when dscale is requested)
__global__ __launch_bounds__(256) void k_conv_finalize(int64_t E, int nbw, const float *__restrict__ wpart,
                                                      const float *__restrict__ w, const float *__restrict__ escale,
                                                      float *__restrict__ dw, float *__restrict__ dscale,
                                                      int Cout, const float *__restrict__ gpart,
                                                      float *__restrict__ dbias, float *__restrict__ dcbias,
                                                      int nbd, const float *__restrict__ spart,
                                                      float *__restrict__ dpre, float *__restrict__ dpost) {
    __shared__ float red[8];
    const float sc = escale ? *escale : 1.f;
    float wg = 0.f;
    const int64_t stride = int64_t(gridDim.x) * 256;
    for (int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x; e < E; e += stride) {
        float s = 0.f;
        for (int j = 0; j < nbw; ++j) s += wpart[int64_t(j) * E + e];
        if (dw) dw[e] += escale ? s * sc : s;
        if (dscale) wg = fmaf(w[e], s, wg);
    }
    if (dscale) {
        wg = block_sum<float, 256>(wg, red);
        if (threadIdx.x == 0) *dscale += wg;
    }
    if (blockIdx.x != 0) return;
    // per-channel bias and the scalar epilogue bias (sum of g), fixed order
    float tot = 0.f;
    for (int co = threadIdx.x; co < Cout; co += 256) {
        float s = 0.f;
        for (int j = 0; j < nbw; ++j) s += gpart[int64_t(j) * Cout + co];
        if (dcbias) dcbias[co] += s;
        tot += s;
    }
    if (dbias) {
        tot = block_sum<float, 256>(tot, red);
        if (threadIdx.x == 0) *dbias += tot;
    }
    if (dpre || dpost) {
        float p0 = 0.f, p1 = 0.f;
        for (int j = threadIdx.x; j < nbd; j += 256) {
            p0 += spart[2 * j];
            p1 += spart[2 * j + 1];
        }
        p0 = block_sum<float, 256>(p0, red);
        p1 = block_sum<float, 256>(p1, red + 4);
        if (threadIdx.x == 0) {
            if (dpre) *dpre += p0;
            if (dpost) *dpost += p1;
        }
    }
}

// ============================================================================ host side
static int pick_tile(int c) {
    // tiles of at most 16 channels, sized to waste as little as possible
    const int ntiles = (c + 15) / 16;
    const int per = (c + ntiles - 1) / ntiles;
    static const int opts[] = {1, 2, 4, 8, 12, 16};
    for (int o : opts)
        if (o >= per) return o;
    return 16;
}

struct BwdPlan {
    int64_t nvox_out, nvox_in, E;
    int Kt, rows_per_wg, ytiles, cot, ztiles, nbw, nbd, cit;
    int64_t vox_per_blk;
    size_t off_wpart, off_gpart, off_spart, bytes;
};

static BwdPlan plan_bwd(const vq3d_conv_desc *d) {
    BwdPlan p;
    const int Ct = d->cin + d->cin2;
    const int K3 = d->kernel * d->kernel * d->kernel;
    p.nvox_out = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    p.nvox_in = int64_t(d->batch) * d->in_h * d->in_w * d->in_d;
    p.Kt = Ct * K3;
    p.E = int64_t(d->cout) * p.Kt;
    int vsplit = 1;
    while (vsplit * 2 * p.Kt <= 256 && vsplit < 256) vsplit *= 2;
    p.rows_per_wg = 256 / vsplit;
    p.ytiles = (p.Kt + p.rows_per_wg - 1) / p.rows_per_wg;
    p.cot = pick_tile(d->cout);
    p.ztiles = (d->cout + p.cot - 1) / p.cot;
    const int64_t tiles = int64_t(p.ytiles) * p.ztiles;
    int64_t nbw = std::max<int64_t>(1, 1024 / tiles);
    nbw = std::min<int64_t>(nbw, (p.nvox_out + kWgChunk - 1) / kWgChunk);
    p.vox_per_blk = (p.nvox_out + nbw - 1) / nbw;
    p.vox_per_blk = (p.vox_per_blk + kWgChunk - 1) / kWgChunk * kWgChunk;
    p.nbw = int((p.nvox_out + p.vox_per_blk - 1) / p.vox_per_blk);
    p.cit = pick_tile(Ct);
    p.nbd = int(((p.nvox_in + 255) / 256) * ((Ct + p.cit - 1) / p.cit));
    p.off_wpart = 0;
    p.off_gpart = p.off_wpart + size_t(p.nbw) * p.E * 4;
    p.off_spart = p.off_gpart + size_t(p.nbw) * d->cout * 4;
    p.bytes = p.off_spart + size_t(p.nbd) * 2 * 4;
    p.bytes = (p.bytes + 255) / 256 * 256;
    return p;
}

static int validate(const vq3d_conv_desc *d) {
    if (!d) return fail("conv: null descriptor");
    if (d->dtype != VQ3D_F32 && d->dtype != VQ3D_BF16) return fail("conv: bad dtype");
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
    return 0;
}

template <typename T>
static int launch_fwd(const vq3d_conv_desc *d, const void *x, const void *x2, const float *w, const float *pa,
                      const float *pb, const vq3d_conv_epilogue *epi, void *y, hipStream_t s) {
    ConvArgs a = make_args(d, pa, pb);
    const int cot = pick_tile(d->cout);
    const int64_t nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    dim3 grid(unsigned((nvox + 255) / 256), unsigned((d->cout + cot - 1) / cot));
    const size_t lds = size_t(d->cin + d->cin2) * cot * 4;
    const float *es = epi ? epi->scale : nullptr;
    const float *eb = epi ? epi->bias : nullptr;
    const float *ec = epi ? epi->cbias : nullptr;
    const T *res = epi ? static_cast<const T *>(epi->residual) : nullptr;
    const int rup = epi ? epi->residual_up2 : 0, pe = epi ? epi->post_elu : 0;
    if (res && rup && ((d->out_h | d->out_w | d->out_d) & 1)) return fail("conv: residual_up2 needs even output");
#define L(C)                                                                                              \
    case C:                                                                                               \
        k_conv_fwd<T, C><<<grid, 256, lds, s>>>(a, (const T *)x, (const T *)x2, w, es, eb, ec, res, rup, pe, \
                                                (T *)y);                                                  \
        break;
    switch (cot) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch("conv3d_fwd");
}

template <typename T>
static int launch_dgrad(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w,
                        const float *pa, const vq3d_dgrad_epilogue *epi, void *gx, void *gx2, void *ws,
                        hipStream_t s) {
    ConvArgs a = make_args(d, pa, nullptr);
    BwdPlan p = plan_bwd(d);
    const int Ct = d->cin + d->cin2;
    dim3 grid(unsigned((p.nvox_in + 255) / 256), unsigned((Ct + p.cit - 1) / p.cit));
    const size_t lds = size_t(d->cout) * p.cit * 4;
    float *spart = reinterpret_cast<float *>(static_cast<char *>(ws) + p.off_spart);
    const T *aux = epi ? static_cast<const T *>(epi->aux) : nullptr;
    const T *add = epi ? static_cast<const T *>(epi->addend) : nullptr;
#define L(C)                                                                                            \
    case C:                                                                                             \
        k_conv_dgrad<T, C><<<grid, 256, lds, s>>>(a, (const T *)g, gscale, w, aux, add, (T *)gx, (T *)gx2, \
                                                  spart);                                               \
        break;
    switch (p.cit) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch("conv3d_bwd_data");
}

template <typename T>
static int launch_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pa,
                        const float *pb, void *ws, hipStream_t s) {
    ConvArgs a = make_args(d, pa, pb);
    BwdPlan p = plan_bwd(d);
    dim3 grid(unsigned(p.nbw), unsigned(p.ytiles), unsigned(p.ztiles));
    float *wpart = reinterpret_cast<float *>(static_cast<char *>(ws) + p.off_wpart);
    float *gpart = reinterpret_cast<float *>(static_cast<char *>(ws) + p.off_gpart);
#define L(C)                                                                                                   \
    case C:                                                                                                    \
        k_conv_wgrad<T, C><<<grid, 256, 0, s>>>(a, (const T *)x, (const T *)x2, (const T *)g, p.vox_per_blk,     \
                                                p.rows_per_wg, wpart, gpart);                                  \
        break;
    switch (p.cot) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch("conv3d_bwd_weight");
}

}  // namespace vq3d

using namespace vq3d;

extern "C" {

int vq3d_conv3d_fwd(const vq3d_conv_desc *d, const void *x, const void *x2, const float *w, const float *pro_a,
                    const float *pro_b, const vq3d_conv_epilogue *epi, void *y, vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!x || !w || !y || (d->cin2 && !x2)) return fail("conv3d_fwd: null pointer");
    if (d->pro_kind != VQ3D_PRO_NONE && !pro_a) return fail("conv3d_fwd: prologue needs pro_a");
    if (d->pro_kind == VQ3D_PRO_ELU_ADD && !pro_b) return fail("conv3d_fwd: ELU prologue needs pro_b");
    return d->dtype == VQ3D_F32 ? launch_fwd<float>(d, x, x2, w, pro_a, pro_b, epi, y, as_stream(stream))
                                : launch_fwd<bf16_t>(d, x, x2, w, pro_a, pro_b, epi, y, as_stream(stream));
}

size_t vq3d_conv3d_bwd_workspace_size(const vq3d_conv_desc *d) {
    if (validate(d)) return 0;
    return plan_bwd(d).bytes;
}

int vq3d_conv3d_bwd_data(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w,
                         const float *pro_a, const vq3d_dgrad_epilogue *epi, void *gx, void *gx2, void *workspace,
                         vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!g || !w || !gx || !workspace || (d->cin2 && !gx2)) return fail("conv3d_bwd_data: null pointer");
    if (d->pro_kind != VQ3D_PRO_NONE && !pro_a) return fail("conv3d_bwd_data: prologue needs pro_a");
    if (d->pro_kind == VQ3D_PRO_ELU_ADD && (!epi || !epi->aux))
        return fail("conv3d_bwd_data: ELU prologue derivative needs epi->aux");
    return d->dtype == VQ3D_F32
               ? launch_dgrad<float>(d, g, gscale, w, pro_a, epi, gx, gx2, workspace, as_stream(stream))
               : launch_dgrad<bf16_t>(d, g, gscale, w, pro_a, epi, gx, gx2, workspace, as_stream(stream));
}

int vq3d_conv3d_bwd_weight(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g,
                           const float *pro_a, const float *pro_b, void *workspace, vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!x || !g || !workspace || (d->cin2 && !x2)) return fail("conv3d_bwd_weight: null pointer");
    if (d->pro_kind != VQ3D_PRO_NONE && !pro_a) return fail("conv3d_bwd_weight: prologue needs pro_a");
    if (d->pro_kind == VQ3D_PRO_ELU_ADD && !pro_b) return fail("conv3d_bwd_weight: ELU prologue needs pro_b");
    return d->dtype == VQ3D_F32 ? launch_wgrad<float>(d, x, x2, g, pro_a, pro_b, workspace, as_stream(stream))
                                : launch_wgrad<bf16_t>(d, x, x2, g, pro_a, pro_b, workspace, as_stream(stream));
}

int vq3d_conv3d_bwd_finalize(const vq3d_conv_desc *d, const float *w, const float *epi_scale, const void *workspace,
                             float *dw, float *dscale, float *dbias, float *dcbias, float *dpro_pre,
                             float *dpro_post, vq3d_stream_t stream) {
    if (int r = validate(d)) return r;
    if (!workspace || (dscale && (!w || !epi_scale))) return fail("conv3d_bwd_finalize: null pointer");
    BwdPlan p = plan_bwd(d);
    const char *ws = static_cast<const char *>(workspace);
    unsigned nb = dscale ? 1u : unsigned(std::min<int64_t>((p.E + 255) / 256, 4096));
    if (nb == 0) nb = 1;
    k_conv_finalize<<<nb, 256, 0, as_stream(stream)>>>(
        p.E, p.nbw, reinterpret_cast<const float *>(ws + p.off_wpart), w, epi_scale, dw, dscale, d->cout,
        reinterpret_cast<const float *>(ws + p.off_gpart), dbias, dcbias, p.nbd,
        reinterpret_cast<const float *>(ws + p.off_spart), dpro_pre, dpro_post);
    return check_launch("conv3d_bwd_finalize");
}

}  // extern "C"
