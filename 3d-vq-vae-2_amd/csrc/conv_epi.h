// Conv geometry, circular / zero-pad index maps and the fused forward / backward-data
// epilogues shared by the direct conv engines (conv3d.hip, conv_small.hip).
#pragma once
#include "common.h"
#include "engines.h"

namespace vq3d {

struct ConvArgs {
    int B, Cin, Cin2, Cout;
    int iH, iW, iD, oH, oW, oD;
    int k, s, p, circ;
    int pro_kind;
    const float *pro_a, *pro_b;
};

inline ConvArgs make_args(const vq3d_conv_desc *d, const float *pa, const float *pb) {
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

// wrap into [0, n) for |i| < a few n (no integer division)
__device__ __forceinline__ int wrap(int i, int n) {
    while (i < 0) i += n;
    while (i >= n) i -= n;
    return i;
}

// forward tap: output coordinate o, kernel offset t -> input coordinate, or -1 if in zero padding
__device__ __forceinline__ int fwd_index(int o, int t, int s, int p, int n, int circ) {
    const int i = o * s + t - p;
    if (circ) return wrap(i, n);
    return (i < 0 || i >= n) ? -1 : i;
}

// transposed tap: input coordinate i, kernel offset t -> output coordinate o with
// fwd_index(o, t) == i, or -1 if none (unique when it exists: DESIGN.md §conv)
__device__ __forceinline__ int bwd_index(int i, int t, int s, int p, int n_in, int n_out, int circ) {
    int r = i - t + p;
    if (circ) r = wrap(r, n_in);
    else if (r < 0) return -1;
    if (s == 2) {
        if (r & 1) return -1;
        r >>= 1;
    } else if (s != 1) {
        if (r % s) return -1;
        r /= s;
    }
    return r < n_out ? r : -1;
}

__device__ __forceinline__ void atomic_add_f(float *p, float v) {
    if (p) atomicAdd(p, v);
}

template <typename T>
__device__ __forceinline__ ActDeriv make_deriv(const BwdEpi<T> &e) {
    ActDeriv d;
    d.mode = e.aux ? e.mode : 0;
    d.p = (d.mode && e.p) ? *e.p : 0.f;
    return d;
}

// y[v, co] for one voxel's accumulators (shared by the pointwise and the k > 1 forward)
template <typename T, int COT>
__device__ __forceinline__ void fwd_epilogue(const ConvArgs &a, const FwdEpi<T> &e, const float (&acc)[COT],
                                             int64_t v, int co0, T *__restrict__ yp) {
    const float sc = e.scale ? *e.scale : 1.f;
    const float bi = e.bias ? *e.bias : 0.f;
    const float aa = e.act_a ? *e.act_a : 0.f, ab = e.act_b ? *e.act_b : 0.f;
    int h0 = 0, h1 = 0, w0 = 0, w1 = 0, d0 = 0, d1 = 0, b = 0;
    float lh = 0.f, lw = 0.f, ldd = 0.f;
    const int rH = a.oH / 2, rW = a.oW / 2, rD = a.oD / 2;
    if (e.res && e.res_up2) {
        int64_t t = v;
        const int od = int(t % a.oD); t /= a.oD;
        const int ow = int(t % a.oW); t /= a.oW;
        const int oh = int(t % a.oH);
        b = int(t / a.oH);
        up_coeff(oh, rH, h0, h1, lh);
        up_coeff(ow, rW, w0, w1, lw);
        up_coeff(od, rD, d0, d1, ldd);
    }
#pragma unroll
    for (int c = 0; c < COT; ++c) {
        const int co = co0 + c;
        if (co >= a.Cout) break;
        float val = acc[c];
        if (e.scale) val = val * sc;
        if (e.bias) val = val + bi;
        if (e.cbias) val = val + e.cbias[co];
        if (e.res) {
            if (!e.res_up2) {
                val = val + ld(e.res + v * a.Cout + co);
            } else {
                auto R = [&](int hh, int ww, int dd) {
                    return ld(e.res + (((int64_t(b) * rH + hh) * rW + ww) * rD + dd) * a.Cout + co);
                };
                val = val + ((1.f - lh) * ((1.f - lw) * ((1.f - ldd) * R(h0, w0, d0) + ldd * R(h0, w0, d1)) +
                                          lw * ((1.f - ldd) * R(h0, w1, d0) + ldd * R(h0, w1, d1))) +
                             lh * ((1.f - lw) * ((1.f - ldd) * R(h1, w0, d0) + ldd * R(h1, w0, d1)) +
                                   lw * ((1.f - ldd) * R(h1, w1, d0) + ldd * R(h1, w1, d1))));
            }
        }
        st(yp + co, epi_act(e.act, val, aa, ab));
    }
}

// gx[v, ci] for one voxel's accumulators; returns the (pre, post) contributions
template <typename T, int CIT>
__device__ __forceinline__ void bwd_epilogue(const ConvArgs &a, const BwdEpi<T> &e, const ActDeriv &dv, float gs,
                                             bool has_gs, const float (&acc)[CIT], int64_t v, int ci0,
                                             T *__restrict__ gxr, T *__restrict__ gx2r, float &pre, float &post) {
    const int Ct = a.Cin + a.Cin2;
#pragma unroll
    for (int c = 0; c < CIT; ++c) {
        const int ci = ci0 + c;
        if (ci >= Ct) break;
        float val = acc[c];
        if (has_gs) val = val * gs;
        if (ci < a.Cin) {
            const int64_t o = v * a.Cin + ci;
            pre += val;
            if (dv.mode) val = val * dv(ld(e.aux + o));
            post += val;
            if (e.addend) val = val + ld(e.addend + o);
            st(gxr + ci, val);
        } else {
            st(gx2r + (ci - a.Cin), val);
        }
    }
}

}  // namespace vq3d
