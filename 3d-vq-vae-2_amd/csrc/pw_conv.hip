// 1x1x1 convolution forward and backward-data (nn.Conv3d kernel_size=1: PreAct branch_conv1 /
// branch_conv3 / skip_conv, proj, parse_input, out -- vqvae/layers.py:134-171, 377, 490, 508,
// 535) with the block glue fused: prologue elu(x + a) + b on the input, scale / bias / conv-bias
// / residual / ELU epilogue on the output (layers.py:176-195), or for backward-data the
// activation derivative, the residual-gradient addend and the prologue-scalar partial sums.
//
// At these channel counts (1..256 in, 1..128 out) the op streams voxel rows and is bound by
// memory, never by arithmetic.  Rows are 2..512 bytes and rarely 16-B aligned, and a per-lane
// row access (lanes 18..144 bytes apart) costs far more than its bytes, so EVERY per-voxel
// operand -- input(s), activation-derivative source, addend, residual, and the output -- moves
// between HBM and LDS as a contiguous slab of SEG voxels with 16-byte coalesced accesses.  One
// thread owns one voxel of the segment: it reads its rows from LDS, runs the channel GEMV in fp32
// against weights broadcast from LDS (16 output channels at a time), applies the epilogue and
// writes its output row back to the LDS out slab.
#include "conv_epi.h"
#include "engines.h"

#include <type_traits>

#include <algorithm>
#include <cstdlib>

namespace vq3d {

namespace {

constexpr int SEG = 256;  // threads per workgroup (= max voxels per segment)

struct PwArgs {
    int64_t nvox;
    int Ca, Cb;      // input channels (x then x2); dgrad: Ca = conv Cout (g), Cb = 0
    int Cin;         // Ca + Cb
    int CinP;        // weight row stride in LDS (multiple of 8)
    int N;           // output channels (fwd: Cout; dgrad: conv Cin + Cin2)
    int N1, N2;      // outputs to tensor 1 / 2 (dgrad: cin_split / Cin2; fwd: N / 0)
    int pro_kind;
    const float *pro_a, *pro_b;
    int vec;         // every slab base 16-B aligned
    int segv, tpv;   // voxels per segment, threads per voxel (segv * tpv == 256)
    // LDS slab offsets (elements of T) after the weights
    int o_x, o_x2, o_aux, o_add, o_res, o_out, o_out2;
};

// contiguous global <-> LDS copy of n elements, 16-byte units when `vec`
template <typename T>
__device__ __forceinline__ void copy_in(T *__restrict__ dst, const T *__restrict__ src, int n, bool vec) {
    constexpr int E = 16 / sizeof(T);
    int i0 = 0;
    if (vec) {
        const int nq = n / E;
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (int q = threadIdx.x; q < nq; q += SEG) d4[q] = s4[q];
        i0 = nq * E;
    }
    for (int i = i0 + threadIdx.x; i < n; i += SEG) dst[i] = src[i];
}

template <typename T>
__device__ __forceinline__ void copy_out(T *__restrict__ dst, const T *__restrict__ src, int n, bool vec) {
    copy_in<T>(dst, src, n, vec);
}

// copy_in with the input prologue applied once per element on the way into LDS (the staged
// slab then holds the conv's actual operand, as the k^3 engines stage theirs)
template <typename T>
__device__ __forceinline__ void copy_in_pro(T *__restrict__ dst, const T *__restrict__ src, int n, bool vec,
                                            const Prologue &pro) {
    if (pro.kind == VQ3D_PRO_NONE) {
        copy_in<T>(dst, src, n, vec);
        return;
    }
    constexpr int E = 16 / sizeof(T);
    int i0 = 0;
    if (vec) {
        const int nq = n / E;
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (int q = threadIdx.x; q < nq; q += SEG) {
            uint4 u = s4[q];
            if constexpr (sizeof(T) == 2) {
                uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float lo = pro.apply(h2f_lo(w4[j]));
                    const float hi = pro.apply(h2f_hi(w4[j]));
                    w4[j] = uint32_t(f2h(lo)) | (uint32_t(f2h(hi)) << 16);
                }
                u = uint4{w4[0], w4[1], w4[2], w4[3]};
            } else {
                u = uint4{__float_as_uint(pro.apply(__uint_as_float(u.x))), __float_as_uint(pro.apply(__uint_as_float(u.y))),
                          __float_as_uint(pro.apply(__uint_as_float(u.z))), __float_as_uint(pro.apply(__uint_as_float(u.w)))};
            }
            d4[q] = u;
        }
        i0 = nq * E;
    }
    for (int i = i0 + threadIdx.x; i < n; i += SEG) st(dst + i, pro.apply(ld(src + i)));
}

template <typename T, int COT, bool DGRAD>
__global__ __launch_bounds__(SEG) void k_pw2(PwArgs a, const T *__restrict__ in, const T *__restrict__ in2,
                                            const float *__restrict__ w, FwdEpi<T> fe, BwdEpi<T> be,
                                            const float *__restrict__ gscale, T *__restrict__ out,
                                            T *__restrict__ out2, float *dpre, float *dpost, float *part, unsigned slot) {
    extern __shared__ __attribute__((aligned(16))) float ws[];  // [N pad COT][CinP] then slabs
    __shared__ float red[8];
    const int tid = threadIdx.x;
    const int NP = (a.N + COT - 1) / COT * COT;
    const int Ct = DGRAD ? a.N : a.Cin;  // the weight's 2nd dim (conv input channels)
    for (int e = tid; e < NP * a.CinP; e += SEG) {
        const int o = e / a.CinP, c = e - o * a.CinP;
        float val = 0.f;
        if (o < a.N && c < a.Cin) val = DGRAD ? w[int64_t(c) * Ct + o] : w[int64_t(o) * Ct + c];
        ws[e] = val;
    }
    T *sl = reinterpret_cast<T *>(ws + NP * a.CinP);
    T *sx = sl + a.o_x, *sx2 = sl + a.o_x2, *saux = sl + a.o_aux, *sadd = sl + a.o_add, *sres = sl + a.o_res;
    T *sout = sl + a.o_out, *sout2 = sl + a.o_out2;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const float gs = gscale ? *gscale : 1.f;
    const float sc = fe.scale ? *fe.scale : 1.f, bias = fe.bias ? *fe.bias : 0.f;
    const float aa = fe.act_a ? *fe.act_a : 0.f, ab = fe.act_b ? *fe.act_b : 0.f;
    ActDeriv dv;
    dv.mode = (DGRAD && be.aux) ? be.mode : 0;
    dv.p = (dv.mode && be.p) ? *be.p : 0.f;
    const bool res_slab = !DGRAD && fe.res && !fe.res_up2;
    float pre = 0.f, post = 0.f;
    const int64_t nseg = (a.nvox + a.segv - 1) / a.segv;
    const int vt = tid / a.tpv, part_o = tid - vt * a.tpv;  // this thread's voxel and output-tile phase

    for (int64_t sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const int64_t v0 = sg * a.segv;
        const int nv = int(min<int64_t>(a.segv, a.nvox - v0));
        __syncthreads();
        copy_in_pro<T>(sx, in + v0 * a.Ca, nv * a.Ca, a.vec, pro);
        if (a.Cb) copy_in_pro<T>(sx2, in2 + v0 * a.Cb, nv * a.Cb, a.vec, pro);
        if (DGRAD && dv.mode) copy_in<T>(saux, be.aux + v0 * a.N1, nv * a.N1, a.vec);
        if (DGRAD && be.addend) copy_in<T>(sadd, be.addend + v0 * a.N1, nv * a.N1, a.vec);
        if (res_slab) copy_in<T>(sres, fe.res + v0 * a.N, nv * a.N, a.vec);
        __syncthreads();
        if (vt < nv) {
            const int tid = vt;  // slab row of this thread's voxel
            const int64_t v = v0 + vt;
            const T *xr = sx + tid * a.Ca;
            const T *xr2 = sx2 + tid * a.Cb;
            int h0 = 0, h1 = 0, w0i = 0, w1i = 0, d0 = 0, d1 = 0, b = 0;
            float lh = 0.f, lw = 0.f, ldd = 0.f;
            if (!DGRAD && fe.res && fe.res_up2) {
                int64_t t = v;
                const int od = int(t % fe.oD); t /= fe.oD;
                const int ow = int(t % fe.oW); t /= fe.oW;
                const int oh = int(t % fe.oH);
                b = int(t / fe.oH);
                up_coeff(oh, fe.oH / 2, h0, h1, lh);
                up_coeff(ow, fe.oW / 2, w0i, w1i, lw);
                up_coeff(od, fe.oD / 2, d0, d1, ldd);
            }
            for (int o0 = part_o * COT; o0 < a.N; o0 += a.tpv * COT) {
                float acc[COT];
#pragma unroll
                for (int j = 0; j < COT; ++j) acc[j] = 0.f;
                // full 8-channel chunks of one input (prologue already applied in the slab),
                // then the remaining channels one at a time
                const int full_a = a.Cb ? 0 : (a.Cin & ~7);
                for (int c0 = 0; c0 < full_a; c0 += 8) {
                    float xv[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) xv[j] = ld(xr + c0 + j);
#pragma unroll
                    for (int j = 0; j < COT; ++j) {
                        const float4 w0 = *reinterpret_cast<const float4 *>(ws + (o0 + j) * a.CinP + c0);
                        const float4 w1 = *reinterpret_cast<const float4 *>(ws + (o0 + j) * a.CinP + c0 + 4);
                        float s = acc[j];
                        s = fmaf(xv[0], w0.x, s);
                        s = fmaf(xv[1], w0.y, s);
                        s = fmaf(xv[2], w0.z, s);
                        s = fmaf(xv[3], w0.w, s);
                        s = fmaf(xv[4], w1.x, s);
                        s = fmaf(xv[5], w1.y, s);
                        s = fmaf(xv[6], w1.z, s);
                        s = fmaf(xv[7], w1.w, s);
                        acc[j] = s;
                    }
                }
                for (int c = full_a; c < a.Cin; ++c) {
                    const float xv = c < a.Ca ? ld(xr + c) : ld(xr2 + (c - a.Ca));
#pragma unroll
                    for (int j = 0; j < COT; ++j) acc[j] = fmaf(xv, ws[(o0 + j) * a.CinP + c], acc[j]);
                }
#pragma unroll
                for (int j = 0; j < COT; ++j) {
                    const int o = o0 + j;
                    if (o >= a.N) break;
                    float val = acc[j];
                    if (!DGRAD) {
                        if (fe.scale) val = val * sc;
                        if (fe.bias) val = val + bias;
                        if (fe.cbias) val = val + fe.cbias[o];
                        if (res_slab) {
                            val = val + ld(sres + tid * a.N + o);
                        } else if (fe.res) {
                            const int rH = fe.oH / 2, rW = fe.oW / 2, rD = fe.oD / 2;
                            auto R = [&](int hh, int ww, int dd) {
                                return ld(fe.res + (((int64_t(b) * rH + hh) * rW + ww) * rD + dd) * a.N + o);
                            };
                            val = val + ((1.f - lh) * ((1.f - lw) * ((1.f - ldd) * R(h0, w0i, d0) + ldd * R(h0, w0i, d1)) +
                                                      lw * ((1.f - ldd) * R(h0, w1i, d0) + ldd * R(h0, w1i, d1))) +
                                         lh * ((1.f - lw) * ((1.f - ldd) * R(h1, w0i, d0) + ldd * R(h1, w0i, d1)) +
                                               lw * ((1.f - ldd) * R(h1, w1i, d0) + ldd * R(h1, w1i, d1))));
                        }
                        st(sout + tid * a.N + o, epi_act(fe.act, val, aa, ab));
                    } else {
                        if (gscale) val = val * gs;
                        if (o < a.N1) {
                            const int e = tid * a.N1 + o;
                            pre += val;
                            if (dv.mode) val = val * dv(ld(saux + e));
                            post += val;
                            if (be.addend) val = val + ld(sadd + e);
                            st(sout + e, val);
                        } else {
                            st(sout2 + tid * a.N2 + (o - a.N1), val);
                        }
                    }
                }
            }
        }
        __syncthreads();
        copy_out<T>(out + v0 * a.N1, sout, nv * a.N1, a.vec);
        if (a.N2) copy_out<T>(out2 + v0 * a.N2, sout2, nv * a.N2, a.vec);
    }
    if (DGRAD && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, SEG, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        if (part) {  // per-workgroup partials, summed in order by the grid's last workgroup
            finish_partials<256>(part, int(gridDim.x), int(blockIdx.x), pre, post, dpre, dpost, slot, red);
        } else if (threadIdx.x == 0) {
            if (dpre) atomicAdd(dpre, pre);
            if (dpost) atomicAdd(dpost, post);
        }
    }
}

// Few-channel rows (Cin, N in {1, 2, 4, 8}, one input, no upsampled residual): each row is one
// naturally aligned 2..16-byte vector, so lanes read and write consecutive rows as one contiguous
// span -- no LDS staging; 4 voxels per thread in flight.
template <typename T, int C>
__device__ __forceinline__ void row_ld(const T *__restrict__ p, float (&o)[C]) {
    if constexpr (sizeof(T) == 2) {
        if constexpr (C == 1) {
            o[0] = ld(p);
        } else if constexpr (C == 2) {
            const uint32_t u = *reinterpret_cast<const uint32_t *>(p);
            o[0] = h2f_lo(u);
            o[1] = h2f_hi(u);
        } else if constexpr (C == 4) {
            const uint2 u = *reinterpret_cast<const uint2 *>(p);
            const uint32_t q[2] = {u.x, u.y};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                o[2 * j] = h2f_lo(q[j]);
                o[2 * j + 1] = h2f_hi(q[j]);
            }
        } else {
            const uint4 u = *reinterpret_cast<const uint4 *>(p);
            const uint32_t q[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o[2 * j] = h2f_lo(q[j]);
                o[2 * j + 1] = h2f_hi(q[j]);
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < C; ++j) o[j] = p[j];
    }
}

template <typename T, int C>
__device__ __forceinline__ void row_st(T *__restrict__ p, const float (&v)[C]) {
    if constexpr (sizeof(T) == 2) {
        if constexpr (C == 1) {
            st(p, v[0]);
        } else {
            uint32_t q[C / 2];
#pragma unroll
            for (int j = 0; j < C / 2; ++j) q[j] = uint32_t(f2h(v[2 * j])) | (uint32_t(f2h(v[2 * j + 1])) << 16);
            if constexpr (C == 2) *reinterpret_cast<uint32_t *>(p) = q[0];
            else if constexpr (C == 4) *reinterpret_cast<uint2 *>(p) = uint2{q[0], q[1]};
            else *reinterpret_cast<uint4 *>(p) = uint4{q[0], q[1], q[2], q[3]};
        }
    } else {
#pragma unroll
        for (int j = 0; j < C; ++j) p[j] = v[j];
    }
}

// bf16 storage: the activations' exp on the hardware v_exp_f32 (__expf; the result is rounded to
// bf16 anyway, as the fused block kernels do); fp32 storage keeps the accurate expf
template <typename T>
__device__ __forceinline__ float elu_st(float z) {
    if constexpr (sizeof(T) == 2) return z > 0.f ? z : __expf(z) - 1.f;
    else return elu(z);
}
template <typename T>
__device__ __forceinline__ float pro_fast(const Prologue &p, float x) {
    if (p.kind == VQ3D_PRO_NONE) return x;
    if (p.kind == VQ3D_PRO_ADD) return x + p.a;
    return elu_st<T>(x + p.a) + p.b;
}
template <typename T>
__device__ __forceinline__ float epi_act_fast(int act, float v, float a, float b) {
    if (act == VQ3D_ACT_ELU) return elu_st<T>(v);
    if (act == VQ3D_ACT_ELU_AFFINE) return elu_st<T>(v + a) + b;
    return v;
}

template <typename T, int CI, int CO, bool DGRAD>
__global__ __launch_bounds__(256) void k_pw_rows(int64_t nvox, const T *__restrict__ in, const float *__restrict__ w,
                                                int pro_kind, const float *pro_a, const float *pro_b,
                                                FwdEpi<T> fe, BwdEpi<T> be, const float *__restrict__ gscale,
                                                T *__restrict__ out, float *dpre, float *dpost, float *part, unsigned slot,
                                                FastDiv fD, FastDiv fW, FastDiv fH) {
    __shared__ float wsh[CO * CI];
    __shared__ float red[8];
    const int Ct = DGRAD ? CO : CI;
    for (int e = threadIdx.x; e < CO * CI; e += 256) {
        const int o = e / CI, c = e - o * CI;
        wsh[e] = DGRAD ? w[c * Ct + o] : w[o * Ct + c];
    }
    __syncthreads();
    float wr[CO][CI];
#pragma unroll
    for (int o = 0; o < CO; ++o)
#pragma unroll
        for (int c = 0; c < CI; ++c) wr[o][c] = wsh[o * CI + c];
    const Prologue pro = make_prologue(pro_kind, pro_a, pro_b);
    const float gs = gscale ? *gscale : 1.f;
    const float sc = fe.scale ? *fe.scale : 1.f, bias = fe.bias ? *fe.bias : 0.f;
    const float aa = fe.act_a ? *fe.act_a : 0.f, ab = fe.act_b ? *fe.act_b : 0.f;
    ActDeriv dv;
    dv.mode = (DGRAD && be.aux) ? be.mode : 0;
    dv.p = (dv.mode && be.p) ? *be.p : 0.f;
    float pre = 0.f, post = 0.f;
    const int64_t stride = int64_t(gridDim.x) * 256;
    for (int64_t vb = int64_t(blockIdx.x) * 256 + threadIdx.x; vb < nvox; vb += 4 * stride) {
        float xr[4][CI], er[4][CO], dr[4][CO];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t v = vb + u * stride;
            if (v < nvox) {
                row_ld<T, CI>(in + v * CI, xr[u]);
                if (!DGRAD && fe.res && fe.res_up2) {
                    // the half-grid residual upsampled x2 (trilinear, align_corners=False) on the
                    // fly: 8 neighbour rows of CO channels, the k_pw2 / k_up2_fwd weights and order
                    // voxel coordinates by magic-number division (three integer divisions per
                    // voxel were the kernel's largest VALU cost)
                    const uint32_t t0 = uint32_t(v), t1 = fD.div(t0), t2 = fW.div(t1), b = fH.div(t2);
                    const int od = int(t0 - t1 * uint32_t(fe.oD)), ow = int(t1 - t2 * uint32_t(fe.oW));
                    const int oh = int(t2 - b * uint32_t(fe.oH));
                    const int rH = fe.oH / 2, rW = fe.oW / 2, rD = fe.oD / 2;
                    int h0, h1, w0, w1, d0, d1;
                    float lh, lw, ld_;
                    up_coeff(oh, rH, h0, h1, lh);
                    up_coeff(ow, rW, w0, w1, lw);
                    up_coeff(od, rD, d0, d1, ld_);
                    float R[8][CO];
                    const int hs[2] = {h0, h1}, wsx[2] = {w0, w1}, dsx[2] = {d0, d1};
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        row_ld<T, CO>(fe.res + ((int64_t(int(b) * rH + hs[q >> 2]) * rW + wsx[(q >> 1) & 1]) * rD +
                                                dsx[q & 1]) * CO, R[q]);
#pragma unroll
                    for (int o = 0; o < CO; ++o)
                        er[u][o] = (1.f - lh) * ((1.f - lw) * ((1.f - ld_) * R[0][o] + ld_ * R[1][o]) +
                                                 lw * ((1.f - ld_) * R[2][o] + ld_ * R[3][o])) +
                                   lh * ((1.f - lw) * ((1.f - ld_) * R[4][o] + ld_ * R[5][o]) +
                                         lw * ((1.f - ld_) * R[6][o] + ld_ * R[7][o]));
                } else if (!DGRAD && fe.res) {
                    row_ld<T, CO>(fe.res + v * CO, er[u]);
                }
                if (DGRAD && dv.mode) row_ld<T, CO>(be.aux + v * CO, er[u]);
                if (DGRAD && be.addend) row_ld<T, CO>(be.addend + v * CO, dr[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t v = vb + u * stride;
            if (v >= nvox) break;
            float y[CO], xin[CI];
#pragma unroll
            for (int c = 0; c < CI; ++c) xin[c] = DGRAD ? xr[u][c] : pro_fast<T>(pro, xr[u][c]);
#pragma unroll
            for (int o = 0; o < CO; ++o) {
                float s = 0.f;
#pragma unroll
                for (int c = 0; c < CI; ++c) s = fmaf(xin[c], wr[o][c], s);
                if (!DGRAD) {
                    if (fe.scale) s = s * sc;
                    if (fe.bias) s = s + bias;
                    if (fe.cbias) s = s + fe.cbias[o];
                    if (fe.res) s = s + er[u][o];
                    s = epi_act_fast<T>(fe.act, s, aa, ab);
                } else {
                    if (gscale) s = s * gs;
                    pre += s;
                    if (dv.mode) s = s * dv(er[u][o]);
                    post += s;
                    if (be.addend) s = s + dr[u][o];
                }
                y[o] = s;
            }
            row_st<T, CO>(out + v * CO, y);
        }
    }
    if (DGRAD && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        if (part) {  // per-workgroup partials, summed in order by the grid's last workgroup
            finish_partials<256>(part, int(gridDim.x), int(blockIdx.x), pre, post, dpre, dpost, slot, red);
        } else if (threadIdx.x == 0) {
            if (dpre) atomicAdd(dpre, pre);
            if (dpost) atomicAdd(dpost, post);
        }
    }
}

}  // namespace

namespace {

constexpr int kMaxPwBlocks = 2048;


// Mid-size grids (a few thousand voxels, tens of channels: the 32x32x8 / 16x16x4 levels): the
// slab kernel's per-workgroup staging is pure latency there.  Here a thread owns one voxel and
// OPT consecutive output channels; every wave of a workgroup shares the same output group
// (blockIdx.y), so the weights are wave-uniform and come through the scalar cache (SGPR
// operands, no LDS); input rows are read per lane with 8/16-byte loads.
template <typename T, int N>
__device__ __forceinline__ void load_run(const T *__restrict__ p, int vw, float (&o)[N]) {
    if constexpr (sizeof(T) == 2) {
        if (vw == 8) {
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
            return;
        }
        if (vw == 4) {
#pragma unroll
            for (int q = 0; q < N / 4; ++q) {
                const uint2 u = reinterpret_cast<const uint2 *>(p)[q];
                o[4 * q] = h2f_lo(u.x);
                o[4 * q + 1] = h2f_hi(u.x);
                o[4 * q + 2] = h2f_lo(u.y);
                o[4 * q + 3] = h2f_hi(u.y);
            }
            return;
        }
    } else {
        if (vw >= 4) {
#pragma unroll
            for (int q = 0; q < N / 4; ++q) {
                const float4 f = reinterpret_cast<const float4 *>(p)[q];
                o[4 * q] = f.x;
                o[4 * q + 1] = f.y;
                o[4 * q + 2] = f.z;
                o[4 * q + 3] = f.w;
            }
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < N; ++j) o[j] = ld(p + j);
}

struct SgArgs {
    int64_t nvox;
    int Ca, Cb, Ct, N;  // row channels (x | x2, or g), weight 2nd dim, output channels
    int vwa, vwb;       // row vector width of in / in2 (8, 4 or 1 elements)
};

template <typename T, bool DG, int OPT>
__device__ __forceinline__ void sg_row(const SgArgs &s, const T *__restrict__ row, int n, int cbase, int vw,
                                       const Prologue &pro, const float *__restrict__ w, int o0, float (&acc)[OPT]) {
    // W(o, k): forward w[o * Ct + k], backward-data w[k * Ct + o]; o clamped in range (the
    // surplus accumulators of the last output group are never stored)
    int oc[OPT];
#pragma unroll
    for (int j = 0; j < OPT; ++j) oc[j] = min(o0 + j, s.N - 1);
    int c = 0;
    for (; c + 8 <= n; c += 8) {
        float xv[8];
        load_run<T, 8>(row + c, vw, xv);
        if (!DG && pro.kind != VQ3D_PRO_NONE) {
#pragma unroll
            for (int q = 0; q < 8; ++q) xv[q] = pro.apply(xv[q]);
        }
#pragma unroll
        for (int j = 0; j < OPT; ++j)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int k = cbase + c + q;
                const float wv = DG ? w[int64_t(k) * s.Ct + oc[j]] : w[int64_t(oc[j]) * s.Ct + k];
                acc[j] = fmaf(xv[q], wv, acc[j]);
            }
    }
    for (; c < n; ++c) {
        float xv = ld(row + c);
        if (!DG) xv = pro.apply(xv);
        const int k = cbase + c;
#pragma unroll
        for (int j = 0; j < OPT; ++j) {
            const float wv = DG ? w[int64_t(k) * s.Ct + oc[j]] : w[int64_t(oc[j]) * s.Ct + k];
            acc[j] = fmaf(xv, wv, acc[j]);
        }
    }
}

template <typename T, bool DG, int OPT>
__global__ __launch_bounds__(256) void k_pw_sg(SgArgs s, ConvArgs ca, const T *__restrict__ in,
                                              const T *__restrict__ in2, const float *__restrict__ w, FwdEpi<T> fe,
                                              BwdEpi<T> be, const float *__restrict__ gscale, T *__restrict__ out,
                                              T *__restrict__ out2, float *dpre, float *dpost, float *part, unsigned slot) {
    __shared__ float red[8];
    const int o0 = blockIdx.y * OPT;
    const Prologue pro = make_prologue(DG ? VQ3D_PRO_NONE : ca.pro_kind, ca.pro_a, ca.pro_b);
    const ActDeriv dv = make_deriv(be);
    const float gs = gscale ? *gscale : 1.f;
    float pre = 0.f, post = 0.f;
    for (int64_t v = int64_t(blockIdx.x) * 256 + threadIdx.x; v < s.nvox; v += int64_t(gridDim.x) * 256) {
        float acc[OPT];
#pragma unroll
        for (int j = 0; j < OPT; ++j) acc[j] = 0.f;
        sg_row<T, DG, OPT>(s, in + v * s.Ca, s.Ca, 0, s.vwa, pro, w, o0, acc);
        if (!DG && s.Cb) sg_row<T, DG, OPT>(s, in2 + v * s.Cb, s.Cb, s.Ca, s.vwb, pro, w, o0, acc);
        if (!DG)
            fwd_epilogue<T, OPT>(ca, fe, acc, v, o0, out + v * ca.Cout);
        else
            bwd_epilogue<T, OPT>(ca, be, dv, gs, gscale != nullptr, acc, v, o0, out + v * ca.Cin,
                                 out2 ? out2 + v * ca.Cin2 : nullptr, pre, post);
    }
    if (DG && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        if (part) {  // per-workgroup partials, summed in order by the grid's last workgroup
            finish_partials<256>(part, int(gridDim.x * gridDim.y), int(blockIdx.y * gridDim.x + blockIdx.x), pre, post, dpre, dpost, slot, red);
        } else if (threadIdx.x == 0) {
            if (dpre) atomicAdd(dpre, pre);
            if (dpost) atomicAdd(dpost, post);
        }
    }
}

bool rows_path(const vq3d_conv_desc *d, bool dgrad, const void *res_up2_flag) {
    auto p2 = [](int c) { return c == 1 || c == 2 || c == 4 || c == 8; };
    const int ci = dgrad ? d->cout : d->cin, co = dgrad ? d->cin : d->cout;
    // the half-grid residual (ResizeConv skip) is upsampled inside the forward row kernel
    return d->cin2 == 0 && p2(ci) && p2(co) && !(res_up2_flag && dgrad);
}

}  // namespace


template <typename T>
static int launch_pw_sg(const vq3d_conv_desc *d, bool dgrad, const void *in, const void *in2, const float *w,
                 const float *pa, const float *pb, const FwdEpi<T> &fe, const BwdEpi<T> &be, const float *gscale,
                 void *out, void *out2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t st) {
    const int64_t nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    SgArgs s;
    s.nvox = nvox;
    s.Ca = dgrad ? d->cout : d->cin;
    s.Cb = dgrad ? 0 : d->cin2;
    s.Ct = d->cin + d->cin2;
    s.N = dgrad ? s.Ct : d->cout;
    auto vw = [](const void *p, int ch) {
        const uintptr_t u = reinterpret_cast<uintptr_t>(p);
        const int esz = int(sizeof(T));
        if (ch % 8 == 0 && (u & 15) == 0 && (ch * esz) % 16 == 0) return 8;
        if (ch % 4 == 0 && (u & 7) == 0 && (ch * esz) % 8 == 0) return 4;
        return 1;
    };
    s.vwa = vw(in, s.Ca);
    s.vwb = s.Cb ? vw(in2, s.Cb) : 1;
    ConvArgs ca = make_args(d, pa, pb);
    // outputs per thread: enough (voxel, group) threads to fill the chip; an ELU prologue is
    // recomputed by every group, so it gets twice the outputs per thread
    const int64_t want = (!dgrad && d->pro_kind == VQ3D_PRO_ELU_ADD) ? 65536 : 131072;
    int opt = 16;
    while (opt > 1 && (opt / 2 >= s.N || nvox * ((s.N + opt - 1) / opt) < want)) opt /= 2;
    const int ny = (s.N + opt - 1) / opt;
    const unsigned nbx = unsigned(std::max<int64_t>(1, std::min<int64_t>((nvox + 255) / 256, kMaxPwBlocks / ny)));
    const dim3 grid{nbx, unsigned(ny), 1u};
    const bool want_part = dgrad && (dpre || dpost);
    const int nb = int(nbx) * ny;
    const GridSum gsm = grid_sum_for(st, nb, want_part);  // fixed-order sums (pair pool)
    float *part = gsm.pairs;
    const unsigned tk = gsm.slot;
#define SG(O)                                                                                                    \
    case O:                                                                                                      \
        if (dgrad)                                                                                               \
            k_pw_sg<T, true, O><<<grid, 256, 0, st>>>(s, ca, (const T *)in, nullptr, w, fe, be, gscale, (T *)out, \
                                                      (T *)out2, dpre, dpost, part, tk);                         \
        else                                                                                                     \
            k_pw_sg<T, false, O><<<grid, 256, 0, st>>>(s, ca, (const T *)in, (const T *)in2, w, fe, be, nullptr,  \
                                                       (T *)out, nullptr, nullptr, nullptr, nullptr, 0u);        \
        break;
    switch (opt) {
        SG(1)
        SG(2)
        SG(4)
        SG(8)
        SG(16)
    }
#undef SG
    return check_launch(dgrad ? "conv3d_bwd_data(pointwise sg)" : "conv3d_fwd(pointwise sg)");
}

// ---- matrix-core 1x1 conv for the up / down blocks' branch and skip convs on the mid grids
// (8 .. 256 channels, 128 .. 1M voxels): Y[v][n] = epi(sum_k X[v][k] W'[k][n]) as
// v_mfma_f32_16x16x32_bf16 over 16-voxel m-tiles.  The A fragment of lane (row, kb) is the 16
// contiguous bytes of voxel row v0 + row at channel 32 ks + 8 kb, loaded straight from HBM
// (channels-last rows, prologue applied in registers); W' (forward: W[n][k], backward-data:
// W[k][n]) lives in LDS as packed B fragments.  Operands are bf16, as the reference's autocast
// 1x1 convs run in fp16 (the VALU kernels above keep the weights fp32).
namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));

// 4 consecutive bf16 (8-byte aligned when `vec`) <-> fp32; `cnt` of them valid
__device__ __forceinline__ void ld4(const h16_t *p, bool vec, int cnt, float (&o)[4]) {
    if (vec) {
        const u32x2 u = *reinterpret_cast<const u32x2 *>(p);
        o[0] = h2f_lo(u[0]);
        o[1] = h2f_hi(u[0]);
        o[2] = h2f_lo(u[1]);
        o[3] = h2f_hi(u[1]);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = j < cnt ? ld(p + j) : 0.f;
    }
}
__device__ __forceinline__ void st4(h16_t *p, bool vec, int cnt, const float (&o)[4]) {
    if (vec) {
        *reinterpret_cast<u32x2 *>(p) = u32x2{uint32_t(f2h(o[0])) | (uint32_t(f2h(o[1])) << 16),
                                             uint32_t(f2h(o[2])) | (uint32_t(f2h(o[3])) << 16)};
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < cnt) st(p + j, o[j]);
    }
}

struct MmArgs {
    int64_t nvox;
    int Ca, Cb, K, N, KS;  // row channels (x | x2, or g), reduction length, outputs, 32-wide k-steps
};

template <int NTN, bool DG>
__global__ __launch_bounds__(256) void k_pw_mma(MmArgs m, ConvArgs ca, const h16_t *__restrict__ in,
                                               const h16_t *__restrict__ in2, const float *__restrict__ w,
                                               FwdEpi<h16_t> fe, BwdEpi<h16_t> be, const float *__restrict__ gscale,
                                               h16_t *__restrict__ out, h16_t *__restrict__ out2, float *dpre,
                                               float *dpost, float *part, unsigned slot) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    u32x4 *wB = reinterpret_cast<u32x4 *>(smem);  // [KS][NTN][64]: this workgroup's NTN n-tiles
    __shared__ float red[8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, row = lane & 15, kb = lane >> 4;
    const int Ct = ca.Cin + ca.Cin2, nt0 = int(blockIdx.y) * NTN;
    for (int i = tid; i < m.KS * NTN * 64; i += 256) {
        const int l = i & 63, t = (i >> 6) % NTN, ks = i / (64 * NTN);
        const int n = 16 * (nt0 + t) + (l & 15), k0 = 32 * ks + 8 * (l >> 4);
        uint32_t q[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float f2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = k0 + 2 * j + h;
                f2[h] = (k < m.K && n < m.N) ? (DG ? w[int64_t(k) * Ct + n] : w[int64_t(n) * Ct + k]) : 0.f;
            }
            q[j] = uint32_t(f2h(f2[0])) | (uint32_t(f2h(f2[1])) << 16);
        }
        wB[i] = u32x4{q[0], q[1], q[2], q[3]};
    }
    __syncthreads();
    const Prologue pro = make_prologue(DG ? VQ3D_PRO_NONE : ca.pro_kind, ca.pro_a, ca.pro_b);
    const bool raw = DG || pro.kind == VQ3D_PRO_NONE;
    const ActDeriv dv = make_deriv(be);
    const float gs = gscale ? *gscale : 1.f;
    const float sc = fe.scale ? *fe.scale : 1.f, bi = fe.bias ? *fe.bias : 0.f;
    const float aa = fe.act_a ? *fe.act_a : 0.f, ab = fe.act_b ? *fe.act_b : 0.f;
    float pre = 0.f, post = 0.f;
    const int64_t ntile = (m.nvox + 15) / 16;
    for (int64_t mt = int64_t(blockIdx.x) * 4 + wave; mt < ntile; mt += int64_t(gridDim.x) * 4) {
        const int64_t v0 = mt * 16, vr = min(v0 + row, m.nvox - 1);
        u32x4 av[8];  // every A fragment of the tile in flight together
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            av[ks] = u32x4{0u, 0u, 0u, 0u};
            const int k0 = 32 * ks + 8 * kb;
            if (ks < m.KS && k0 < m.K)
                av[ks] = k0 < m.Ca ? *reinterpret_cast<const u32x4 *>(in + vr * m.Ca + k0)
                                   : *reinterpret_cast<const u32x4 *>(in2 + vr * m.Cb + (k0 - m.Ca));
        }
        f32x4 acc[NTN];
#pragma unroll
        for (int t = 0; t < NTN; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (ks >= m.KS) break;
            u32x4 a = av[ks];
            if (!raw && 32 * ks + 8 * kb < m.K) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    a[j] = uint32_t(f2h(pro.apply(h2f_lo(a[j])))) |
                           (uint32_t(f2h(pro.apply(h2f_hi(a[j])))) << 16);
            }
            const hx8 af = __builtin_bit_cast(hx8, a);
            // D^T[n][v] = W'^T X^T: the weight fragment is the A operand, the voxel rows the B operand,
            // so a lane ends with 4 consecutive output channels of one voxel (vector epilogue)
#pragma unroll
            for (int t = 0; t < NTN; ++t)
                acc[t] = VQ3D_MFMA_16X16X32(__builtin_bit_cast(hx8, wB[(ks * NTN + t) * 64 + lane]),
                                                                 af, acc[t], 0, 0, 0);
        }
        // D^T[channel 16 t' + 4 kb + j][voxel v0 + row] of n-tile t' = nt0 + t
        const int64_t v = v0 + row;
        if (v < m.nvox) {
#pragma unroll
            for (int t = 0; t < NTN; ++t) {
                const int n0 = 16 * (nt0 + t) + 4 * kb;
                if (n0 >= m.N) continue;
                float val[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) val[j] = acc[t][j];
                if constexpr (!DG) {
                    const int cnt = min(4, m.N - n0);
                    const bool vec = cnt == 4 && (m.N & 3) == 0;
                    float r4[4] = {0.f, 0.f, 0.f, 0.f};
                    if (fe.res) ld4(fe.res + v * m.N + n0, vec, cnt, r4);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float x = val[j];
                        if (fe.scale) x = x * sc;
                        if (fe.bias) x = x + bi;
                        if (fe.cbias && j < cnt) x = x + fe.cbias[n0 + j];
                        if (fe.res) x = x + r4[j];
                        val[j] = epi_act(fe.act, x, aa, ab);
                    }
                    st4(out + v * m.N + n0, vec, cnt, val);
                } else {
                    if (gscale)
#pragma unroll
                        for (int j = 0; j < 4; ++j) val[j] = val[j] * gs;
                    if (n0 + 4 <= ca.Cin) {  // all 4 in gx
                        const int64_t o = v * ca.Cin + n0;
                        const bool vec = (ca.Cin & 3) == 0;
                        float x4[4], d4[4] = {0.f, 0.f, 0.f, 0.f};
                        if (dv.mode) ld4(be.aux + o, vec, 4, x4);
                        if (be.addend) ld4(be.addend + o, vec, 4, d4);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            pre += val[j];
                            if (dv.mode) val[j] = val[j] * dv(x4[j]);
                            post += val[j];
                            val[j] += d4[j];
                        }
                        st4(out + o, vec, 4, val);
                    } else if (n0 >= ca.Cin && ((ca.Cin2 | (n0 - ca.Cin)) & 3) == 0) {  // all in gx2
                        st4(out2 + v * ca.Cin2 + (n0 - ca.Cin), n0 + 4 <= ca.Cin + ca.Cin2, min(4, m.N - n0), val);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int n = n0 + j;
                            if (n >= m.N) break;
                            float x = val[j];
                            if (n < ca.Cin) {
                                const int64_t o = v * ca.Cin + n;
                                pre += x;
                                if (dv.mode) x = x * dv(ld(be.aux + o));
                                post += x;
                                if (be.addend) x = x + ld(be.addend + o);
                                st(out + o, x);
                            } else {
                                st(out2 + v * ca.Cin2 + (n - ca.Cin), x);
                            }
                        }
                    }
                }
            }
        }
    }
    if (DG && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        if (part) {  // per-workgroup partials, summed in order by the grid's last workgroup
            finish_partials<256>(part, int(gridDim.x * gridDim.y), int(blockIdx.y * gridDim.x + blockIdx.x), pre, post, dpre, dpost, slot, red);
        } else if (threadIdx.x == 0) {
            if (dpre) atomicAdd(dpre, pre);
            if (dpost) atomicAdd(dpost, post);
        }
    }
}
}  // namespace

// the matrix-core path, or false when the conv is not one of its shapes
static bool launch_pw_mma(const vq3d_conv_desc *d, bool dgrad, const void *in, const void *in2, const float *w,
                          const float *pa, const float *pb, const FwdEpi<h16_t> &fe, const BwdEpi<h16_t> &be,
                          const float *gscale, void *out, void *out2, float *dpre, float *dpost, void *ws,
                          size_t ws_bytes, hipStream_t s) {
    const int64_t nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    MmArgs m;
    m.nvox = nvox;
    m.Ca = dgrad ? d->cout : d->cin;
    m.Cb = dgrad ? 0 : d->cin2;
    m.K = m.Ca + m.Cb;
    m.N = dgrad ? d->cin + d->cin2 : d->cout;
    m.KS = (m.K + 31) / 32;
    auto al = [](const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    // 8 -> 8 on the big grids: the row kernel is faster
    if (m.K <= 8 && m.N <= 8) return false;
    if (m.K < 8 || m.K > 256 || m.N < 8 || m.N > 128 || m.Ca % 8 || m.Cb % 8 || nvox < 128 || nvox > (int64_t(1) << 20))
        return false;
    if (fe.res_up2 || !al(in) || !al(in2)) return false;
    // n-tiles per workgroup: all of them, halved while the grid has fewer than 512 workgroups
    // (small grids: the weight staging then splits over the second grid dimension)
    const int ntn = (m.N + 15) / 16;
    int NTN = ntn <= 1 ? 1 : ntn <= 2 ? 2 : ntn <= 4 ? 4 : 8;
    const int64_t ntile = (nvox + 15) / 16, nbx0 = (ntile + 3) / 4;
    while (NTN > 1 && nbx0 * ((ntn + NTN - 1) / NTN) < 512) NTN /= 2;
    const int ny = (ntn + NTN - 1) / NTN;
    const size_t lds = size_t(m.KS) * NTN * 64 * 16;
    const unsigned nbx = unsigned(std::max<int64_t>(1, std::min<int64_t>(nbx0, 1024 / ny)));
    const dim3 nb{nbx, unsigned(ny), 1u};
    const bool want_part = dgrad && (dpre || dpost);
    const GridSum gsm = grid_sum_for(s, int64_t(nbx) * ny, want_part);  // fixed-order sums (pair pool)
    float *part = gsm.pairs;
    const unsigned tk = gsm.slot;
    ConvArgs ca = make_args(d, pa, pb);
#define MM(NT_)                                                                                                 \
    if (dgrad)                                                                                                  \
        k_pw_mma<NT_, true><<<nb, 256, lds, s>>>(m, ca, (const h16_t *)in, nullptr, w, fe, be, gscale,         \
                                                 (h16_t *)out, (h16_t *)out2, dpre, dpost, part, tk);         \
    else                                                                                                        \
        k_pw_mma<NT_, false><<<nb, 256, lds, s>>>(m, ca, (const h16_t *)in, (const h16_t *)in2, w, fe, be,    \
                                                  nullptr, (h16_t *)out, nullptr, nullptr, nullptr, nullptr, 0u);
    switch (NTN) {
    case 1: MM(1) break;
    case 2: MM(2) break;
    case 4: MM(4) break;
    default: MM(8) break;
    }
#undef MM
    return true;
}

size_t pw_dgrad_workspace(const vq3d_conv_desc *) { return size_t(2) * kMaxPwBlocks * sizeof(float); }

template <typename T>
int launch_pw1(const vq3d_conv_desc *d, bool dgrad, const void *in, const void *in2, const float *w, const float *pa,
               const float *pb, const FwdEpi<T> &fe_in, const BwdEpi<T> &be, const float *gscale, void *out,
               void *out2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t s) {
    const int64_t nvox = int64_t(d->batch) * d->out_h * d->out_w * d->out_d;
    FwdEpi<T> fe = fe_in;
    fe.oH = d->out_h;
    fe.oW = d->out_w;
    fe.oD = d->out_d;
    auto al = [](const void *p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool want_part = dgrad && (dpre || dpost);
    // ---- 8 .. 256 channels on the mid grids: matrix cores
    if constexpr (std::is_same<T, h16_t>::value) {
        if (launch_pw_mma(d, dgrad, in, in2, w, pa, pb, fe, be, gscale, out, out2, dpre, dpost, ws, ws_bytes, s))
            return check_launch(dgrad ? "conv3d_bwd_data(pointwise mma)" : "conv3d_fwd(pointwise mma)");
    }
    // ---- mid-size grids: scalar-cache weights, one thread per (voxel, output group)
    if (nvox <= 65536)
        return launch_pw_sg<T>(d, dgrad, in, in2, w, pa, pb, fe, be, gscale, out, out2, dpre, dpost, ws, ws_bytes, s);
    // ---- few-channel rows: no LDS staging
    if (rows_path(d, dgrad, fe.res_up2 ? fe.res : nullptr) && al(in) && al(out) && al(fe.res) && al(be.aux) && al(be.addend)) {
        const int ci = dgrad ? d->cout : d->cin, co = dgrad ? d->cin : d->cout;
        const unsigned nbx = unsigned(std::max<int64_t>(1, std::min<int64_t>((nvox + 1023) / 1024, kMaxPwBlocks)));
        const GridSum gsm = grid_sum_for(s, nbx, want_part);  // fixed-order sums (pair pool)
        float *part = gsm.pairs;
        const unsigned tk = gsm.slot;
        const int key = ci * 16 + co;
        const int pk = dgrad ? VQ3D_PRO_NONE : d->pro_kind;
        const FastDiv fD(uint32_t(d->out_d)), fW(uint32_t(d->out_w)), fH(uint32_t(d->out_h));
#define R(CI, CO)                                                                                              \
    case CI * 16 + CO:                                                                                         \
        if (dgrad)                                                                                             \
            k_pw_rows<T, CI, CO, true><<<nbx, 256, 0, s>>>(nvox, (const T *)in, w, pk, pa, pb, fe, be, gscale, \
                                                           (T *)out, dpre, dpost, part, tk, fD, fW, fH);       \
        else                                                                                                   \
            k_pw_rows<T, CI, CO, false><<<nbx, 256, 0, s>>>(nvox, (const T *)in, w, pk, pa, pb, fe, be,       \
                                                            nullptr, (T *)out, nullptr, nullptr, nullptr, 0u, fD, \
                                                            fW, fH);                                           \
        break;
        switch (key) {
            R(1, 1) R(1, 2) R(1, 4) R(1, 8) R(2, 1) R(2, 2) R(2, 4) R(2, 8)
            R(4, 1) R(4, 2) R(4, 4) R(4, 8) R(8, 1) R(8, 2) R(8, 4) R(8, 8)
        default: return fail("conv(pointwise): no row kernel");
        }
#undef R
        return check_launch(dgrad ? "conv3d_bwd_data(pointwise rows)" : "conv3d_fwd(pointwise rows)");
    }
    // ---- LDS slabs
    PwArgs a = {};
    a.nvox = nvox;
    const int Ct = d->cin + d->cin2;
    if (!dgrad) {
        a.Ca = d->cin;
        a.Cb = d->cin2;
        a.N = d->cout;
        a.N1 = a.N;
        a.N2 = 0;
        a.pro_kind = d->pro_kind;
        a.pro_a = pa;
        a.pro_b = pb;
    } else {
        a.Ca = d->cout;
        a.Cb = 0;
        a.N = Ct;
        a.N1 = d->cin;
        a.N2 = d->cin2;
        a.pro_kind = VQ3D_PRO_NONE;
    }
    a.Cin = a.Ca + a.Cb;
    a.CinP = (a.Cin + 7) / 8 * 8;
    int cot = a.N <= 1 ? 1 : a.N <= 2 ? 2 : a.N <= 4 ? 4 : a.N <= 8 ? 8 : a.N <= 12 ? 12 : 16;
    if (nvox <= 8192 && cot > 4) cot = 4;  // tiny grids: split each voxel's outputs over more threads
    const int NP = (a.N + cot - 1) / cot * cot;
    // voxels per segment: 256 (one thread each) unless the grid would leave CUs idle; then
    // fewer voxels with several threads splitting each voxel's output tiles
    const int ntiles = NP / cot;
    a.segv = 256;
    while (a.segv > 32 && (nvox + a.segv - 1) / a.segv < 512 && 256 / (a.segv / 2) <= ntiles) a.segv /= 2;
    auto r8 = [](int v) { return (v + 7) / 8 * 8; };
    const bool aux = dgrad && be.aux && be.mode;
    size_t lds = 0;
    while (true) {  // shrink the segment until the slabs fit
        a.tpv = 256 / a.segv;
        const int S = a.segv;
        int off = 0;
        a.o_x = off; off += r8(S * a.Ca);
        a.o_x2 = off; off += r8(S * a.Cb);
        a.o_aux = off; off += aux ? r8(S * a.N1) : 0;
        a.o_add = off; off += (dgrad && be.addend) ? r8(S * a.N1) : 0;
        a.o_res = off; off += (!dgrad && fe.res && !fe.res_up2) ? r8(S * a.N) : 0;
        a.o_out = off; off += r8(S * a.N1);
        a.o_out2 = off; off += r8(S * a.N2);
        lds = size_t(NP) * a.CinP * 4 + size_t(off) * sizeof(T);
        if (lds <= 96 * 1024 || a.segv <= 8) break;
        a.segv /= 2;
    }
    if (lds > 150 * 1024) return fail("conv(pointwise): too many channels for the LDS slabs");
    a.vec = al(in) && al(in2) && al(out) && al(out2) && al(be.aux) && al(be.addend) && al(fe.res);
    const int64_t nseg = (a.nvox + a.segv - 1) / a.segv;
    const int slab_cap = std::min(kMaxPwBlocks, 1024);  // measured: 1024 >= 2048 > 512 workgroups
    const unsigned nbx = unsigned(std::max<int64_t>(1, std::min<int64_t>(nseg, slab_cap)));
    const GridSum gsm = grid_sum_for(s, nbx, want_part);  // fixed-order sums (pair pool)
    float *part = gsm.pairs;
    const unsigned tk = gsm.slot;
#define L(C)                                                                                                    \
    case C: {                                                                                                   \
        auto kern = dgrad ? k_pw2<T, C, true> : k_pw2<T, C, false>;                                             \
        static bool attr = false;                                                                               \
        if (!attr) {                                                                                            \
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pw2<T, C, true>),                        \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);                  \
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_pw2<T, C, false>),                       \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);                  \
            (void)hipGetLastError();                                                                            \
            attr = true;                                                                                        \
        }                                                                                                       \
        kern<<<nbx, SEG, lds, s>>>(a, (const T *)in, (const T *)in2, w, fe, be, gscale, (T *)out, (T *)out2,    \
                                   dpre, dpost, part, tk);                                                      \
    } break;
    switch (cot) { L(1) L(2) L(4) L(8) L(12) L(16) }
#undef L
    return check_launch(dgrad ? "conv3d_bwd_data(pointwise)" : "conv3d_fwd(pointwise)");
}

template int launch_pw1<float>(const vq3d_conv_desc *, bool, const void *, const void *, const float *, const float *,
                               const float *, const FwdEpi<float> &, const BwdEpi<float> &, const float *, void *,
                               void *, float *, float *, void *, size_t, hipStream_t);
template int launch_pw1<h16_t>(const vq3d_conv_desc *, bool, const void *, const void *, const float *,
                                const float *, const float *, const FwdEpi<h16_t> &, const BwdEpi<h16_t> &,
                                const float *, void *, void *, float *, float *, void *, size_t, hipStream_t);

}  // namespace vq3d
