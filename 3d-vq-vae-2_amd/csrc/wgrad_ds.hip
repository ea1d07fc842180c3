// Weight gradients of the few-channel k^3 convs on the large grids, on the matrix cores with
// D-SHIFTS (vqvae/layers.py:124-151 branch_conv2 / skip_conv, 591-597 ResizeConv):
//   dW[co][ci][kh][kw][kd] += sum_o g[o][co] x[s_ * o + (kh, kw, kd) - p][ci]
// With only CO = 4 / 8 / 16 output channels, S = 16 / CO consecutive output positions along D
// share one MFMA row block: o = S m + s,
//   D_(kh,kw)[(s, co)][(pd, ci)] = sum_m g[S m + s][co] x_(kh,kw)[s_ S m + pd - p][ci]
// (M = 16 = S x CO, every row real; N = the (s_ (S-1) + k) window positions x CI; K = 32 groups
// per v_mfma_f32_16x16x32_bf16, taken from one or more D-lines), then
//   dW[co][ci][kh][kw][kd] = sum_s D_(kh,kw)[(s, co)][(s_ s + kd, ci)].
// In channels-last memory a g line IS the A^T image [m][16] and an x line, read from position
// s_ S m - p, the B image [m][s_ S CI]: both operands come through the transposing
// ds_read_b64_tr_b16 from lines staged with 16-byte loads (prologue applied as they are written,
// circular wrap / zero padding resolved per line and per edge position).
//
// A workgroup walks TH x TW tiles of output lines (XCD-contiguous ranges), staging the tile's g
// lines and the (s_ (TH-1) + k) x (s_ (TW-1) + k) x lines under it while the previous tile's MFMAs
// run (register prefetch).  Wave w takes K-steps w, w + 4, ... with every tap row when the
// accumulators fit (3x3x3, 2x2x2), else tap rows w, w + 4, ... of every K-step (4x4x4).  The
// per-workgroup sums (and the sum of g for the conv's bias) go to the workspace and a second
// kernel adds them to dW in a fixed order: deterministic.
//
// Instances (3-layer published model, 512^2 x 128): the last up block's 3x3x3 4 -> 4 ResizeConv
// branch conv at 512^2 x 128 (generic engine 779 us), the down blocks' 4x4x4 stride-2 branch convs
// 4 -> 4 (512^2 -> 256^2), 8 -> 8 (256^2), 16 -> 16 (128^2; 619 us) and their 2x2x2 stride-2 skip
// convs 4 -> 8, 8 -> 16 (zero padding, + bias1c prologue, bias1d gradient).
#include "engines.h"

#include <algorithm>

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int NT = 256;

constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int rup(int v, int m) { return (v + m - 1) / m * m; }

template <int CI, int CO, int KS, int ST, int PAD, int DO, int TH, int TW>
struct Geo {
    static constexpr int S = 16 / CO;                  // output positions per MFMA row block
    static constexpr int MPL = DO / S;                 // groups per output line
    static constexpr int DI = DO * ST;                 // input line length
    static constexpr int NP = ST * (S - 1) + KS;       // window positions
    static constexpr int NTN = (NP * CI + 15) / 16;    // 16-column N tiles
    static constexpr int NL = TH * TW;                 // output lines per tile
    static constexpr int XH = ST * (TH - 1) + KS, XW = ST * (TW - 1) + KS, XL = XH * XW;
    static constexpr int NKS = NL * MPL / 32;          // K-steps per tile
    static constexpr int GLP = DO * CO;                // g line pitch (elements)
    static constexpr int MAXP = ST * S * (MPL - 1) - PAD + NTN * 16 / CI - 1;  // last position read
    static constexpr int RX = cmax(0, MAXP - (DI - 1));                        // positions past the line
    static constexpr int XOFF = rup(PAD * CI, 8);      // element of position 0 (16-B aligned)
    static constexpr int XP = rup(XOFF + (DI + RX) * CI, 8);
    static constexpr int NTAP = KS * KS;
    // wave partition: by K-steps (each wave all taps; A fragment reused over NTAP x NTN MFMAs) when
    // the accumulators fit, else by taps (wave w: taps w, w + 4, ...; every wave every K-step)
    static constexpr bool BYK = NTAP * NTN <= 24;
    static constexpr int TPW = BYK ? NTAP : (NTAP + 3) / 4, NIMG = BYK ? 4 : 1;
    static constexpr int NE = CO * CI * KS * KS * KS;
    static constexpr int GU = NL * GLP / 8, XU = XL * DI * CI / 8;     // 16-byte units
    static constexpr int EPL = (PAD + RX) * CI / 4, EU = XL * EPL;       // 8-byte edge units
    static constexpr int PG = (GU + NT - 1) / NT, PX = (XU + NT - 1) / NT, PE = cmax(1, (EU + NT - 1) / NT);
    static constexpr size_t LDS = size_t(cmax(NL * GLP + XL * XP, 2 * NIMG * S * NE + 2 * 8)) * 2;
    static_assert(MPL % 8 == 0 && (NL * MPL) % 32 == 0 && CI % 4 == 0 && 16 % CO == 0, "geometry");
    static_assert(KS > PAD, "padding");
};

struct WArgs {
    int B, Ho, Wo, Hi, Wi;
    int nth, ntw, ntiles;
    int circ;
    int pro_kind;
    const float *pro_a, *pro_b;
};

__device__ __forceinline__ int wrapm(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }

__device__ __forceinline__ hx8 tr8(const h16_t *p0, const h16_t *p1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
    return __builtin_bit_cast(hx8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// the prologue over 2 packed bf16 (zero padding stays zero: only loaded words come here)
__device__ __forceinline__ uint32_t pro2(uint32_t w, const Prologue &pro) {
    const float lo = pro.apply(h2f_lo(w)), hi = pro.apply(h2f_hi(w));
    return uint32_t(f2h(lo)) | (uint32_t(f2h(hi)) << 16);
}

template <int CI, int CO, int KS, int ST, int PAD, int DO, int TH, int TW>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void k_wgrad_ds(
    WArgs a, const h16_t *__restrict__ x, const h16_t *__restrict__ g, float *__restrict__ part, int want_gsum) {
    using Gm = Geo<CI, CO, KS, ST, PAD, DO, TH, TW>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    h16_t *gl = reinterpret_cast<h16_t *>(smem);  // [NL][GLP]
    h16_t *xl = gl + Gm::NL * Gm::GLP;              // [XL][XP]
    __shared__ float red[8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = lane >> 4, li = lane & 15, q = li >> 2, p4 = li & 3;
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const bool raw = a.pro_kind == VQ3D_PRO_NONE;
    f32x4 acc[Gm::TPW][Gm::NTN];
#pragma unroll
    for (int j = 0; j < Gm::TPW; ++j)
#pragma unroll
        for (int t = 0; t < Gm::NTN; ++t) acc[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float gsum = 0.f;

    // the next tile's g lines, x lines (main runs) and x edge positions in registers while the
    // current tile computes; every load unconditional (clamped index, zero when outside)
    u32x4 gv[Gm::PG], xv[Gm::PX];
    u32x2 ev[Gm::PE];
    uint32_t xok = 0, eok = 0;  // per unit: inside the grid (zero padding otherwise)
    auto x_line = [&](int b, int h0, int w0, int line, bool &ok) -> int64_t {
        int ih = h0 * ST - PAD + line / Gm::XW, iw = w0 * ST - PAD + line % Gm::XW;
        ok = a.circ || (unsigned(ih) < unsigned(a.Hi) && unsigned(iw) < unsigned(a.Wi));
        ih = wrapm(ih, a.Hi);
        iw = wrapm(iw, a.Wi);
        if (!ok) ih = iw = 0;
        return ((int64_t(b) * a.Hi + ih) * a.Wi + iw) * Gm::DI;
    };
    auto load = [&](int tile) {
        int t = tile;
        const int w0 = (t % a.ntw) * TW;
        t /= a.ntw;
        const int h0 = (t % a.nth) * TH, b = t / a.nth;
#pragma unroll
        for (int u = 0; u < Gm::PG; ++u) {
            const int i = min(tid + u * NT, Gm::GU - 1), line = i / (Gm::GLP / 8), part_ = i % (Gm::GLP / 8);
            const int64_t v0 = ((int64_t(b) * a.Ho + h0 + line / TW) * a.Wo + w0 + line % TW) * DO;
            gv[u] = reinterpret_cast<const u32x4 *>(g + v0 * CO)[part_];
        }
        xok = 0;
#pragma unroll
        for (int u = 0; u < Gm::PX; ++u) {
            const int i = min(tid + u * NT, Gm::XU - 1), line = i / (Gm::DI * CI / 8), part_ = i % (Gm::DI * CI / 8);
            bool ok;
            const int64_t v0 = x_line(b, h0, w0, line, ok);
            xv[u] = reinterpret_cast<const u32x4 *>(x + v0 * CI)[part_];
            xok |= ok ? (1u << u) : 0u;
        }
        eok = 0;
#pragma unroll
        for (int u = 0; u < Gm::PE; ++u) {
            ev[u] = u32x2{0u, 0u};
            if constexpr (Gm::EU > 0) {
                const int i = min(tid + u * NT, Gm::EU - 1), line = i / Gm::EPL, k = i % Gm::EPL;
                const int pos = k / (CI / 4), c4 = k % (CI / 4);  // pos < PAD: position pos - PAD; else DI + pos - PAD
                const int id = pos < PAD ? pos - PAD : Gm::DI + pos - PAD;
                bool ok;
                const int64_t v0 = x_line(b, h0, w0, line, ok);
                const bool inside = unsigned(id) < unsigned(Gm::DI);
                ok = ok && (a.circ || inside);
                ev[u] = *reinterpret_cast<const u32x2 *>(x + (v0 + wrapm(id, Gm::DI)) * CI + 4 * c4);
                eok |= ok ? (1u << u) : 0u;
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < Gm::PG; ++u) {
            const int i = tid + u * NT;
            if (i < Gm::GU) {
                reinterpret_cast<u32x4 *>(gl)[i] = gv[u];
                if (want_gsum) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        gsum += h2f_lo(gv[u][j]) + h2f_hi(gv[u][j]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < Gm::PX; ++u) {
            const int i = tid + u * NT;
            if (i < Gm::XU) {
                const int line = i / (Gm::DI * CI / 8), part_ = i % (Gm::DI * CI / 8);
                u32x4 v = xv[u];
                if (!((xok >> u) & 1u)) v = u32x4{0u, 0u, 0u, 0u};
                else if (!raw) v = u32x4{pro2(v[0], pro), pro2(v[1], pro), pro2(v[2], pro), pro2(v[3], pro)};
                reinterpret_cast<u32x4 *>(xl + line * Gm::XP + Gm::XOFF)[part_] = v;
            }
        }
        if constexpr (Gm::EU > 0) {
#pragma unroll
            for (int u = 0; u < Gm::PE; ++u) {
                const int i = tid + u * NT;
                if (i < Gm::EU) {
                    const int line = i / Gm::EPL, k = i % Gm::EPL;
                    const int pos = k / (CI / 4), c4 = k % (CI / 4);
                    const int id = pos < PAD ? pos - PAD : Gm::DI + pos - PAD;
                    u32x2 v = ev[u];
                    if (!((eok >> u) & 1u)) v = u32x2{0u, 0u};
                    else if (!raw) v = u32x2{pro2(v[0], pro), pro2(v[1], pro)};
                    *reinterpret_cast<u32x2 *>(xl + line * Gm::XP + Gm::XOFF + id * CI + 4 * c4) = v;
                }
            }
        }
    };

    const TileSched sc = xcd_sched(a.ntiles);
    if (sc.t < sc.end) load(sc.t);
    for (int tile = sc.t; tile < sc.end; tile += sc.step) {
        __syncthreads();
        store();
        if (tile + sc.step < sc.end) load(tile + sc.step);
        __syncthreads();
#pragma unroll 2
        for (int ks = Gm::BYK ? wave : 0; ks < Gm::NKS; ks += Gm::BYK ? 4 : 1) {
            // K rows 8 grp + q (and + 4) of this step: group G -> (line, m); 8 rows stay in one line
            const int G = ks * 32 + 8 * grp + q, line = G / Gm::MPL, m = G % Gm::MPL;
            const int lh = line / TW, lw = line % TW;
            const h16_t *ga = gl + line * Gm::GLP + m * 16 + 4 * p4;
            const hx8 af = tr8(ga, ga + 64);
            const h16_t *xb0 = xl + Gm::XOFF + (ST * Gm::S * m - PAD) * CI + 4 * p4;
#pragma unroll
            for (int j = 0; j < Gm::TPW; ++j) {
                const int kk = Gm::BYK ? j : wave + 4 * j;
                if (kk < Gm::NTAP) {
                    const int kh = kk / KS, kw = kk % KS;
                    const h16_t *xb = xb0 + ((lh * ST + kh) * Gm::XW + lw * ST + kw) * Gm::XP;
#pragma unroll
                    for (int t = 0; t < Gm::NTN; ++t) {
                        const hx8 bf = tr8(xb + 16 * t, xb + 16 * t + 4 * ST * Gm::S * CI);
                        acc[j][t] = VQ3D_MFMA_16X16X32(af, bf, acc[j][t], 0, 0, 0);
                    }
                }
            }
        }
    }
    // fold the shifts: lane (li, grp) holds D[(s, co) = 4 grp + i][(pd, ci) = 16 t + li] of its tap
    // rows -> image [wave (BYK)][s][NE], every entry written by one lane, summed in a fixed order
    __syncthreads();
    float *img = reinterpret_cast<float *>(smem);
#pragma unroll
    for (int j = 0; j < Gm::TPW; ++j) {
        const int kk = Gm::BYK ? j : wave + 4 * j;
        if (kk >= Gm::NTAP) continue;
        float *im = img + (Gm::BYK ? wave * Gm::S * Gm::NE : 0);
#pragma unroll
        for (int t = 0; t < Gm::NTN; ++t) {
            const int n = 16 * t + li, pd = n / CI, ci = n % CI;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * grp + i, s = r / CO, co = r % CO, kd = pd - ST * s;
                if (kd >= 0 && kd < KS) im[s * Gm::NE + ((co * CI + ci) * Gm::NTAP + kk) * KS + kd] = acc[j][t][i];
            }
        }
    }
    __syncthreads();
    float *dst = part + int64_t(blockIdx.x) * (Gm::NE + 1);
    for (int e = tid; e < Gm::NE; e += NT) {
        float v = 0.f;
#pragma unroll
        for (int s = 0; s < Gm::NIMG * Gm::S; ++s) v += img[s * Gm::NE + e];
        dst[e] = v;
    }
    if (want_gsum) {
        const float tot = block_sum<float, NT>(gsum, red);
        if (tid == 0) dst[Gm::NE] = tot;
    }
}

// dW[e] += sum over the workgroups' partial rows in a fixed order (32 lanes per entry stride the
// workgroups, then a fixed butterfly); entry NE (the sum of g) goes to dbias
__global__ __launch_bounds__(NT) void k_wgrad_ds_reduce(const float *__restrict__ part, int nwg, int ne,
                                                        float *__restrict__ dw, float *__restrict__ dbias) {
    const int e = blockIdx.x * (NT / 32) + (threadIdx.x >> 5), r = threadIdx.x & 31;
    const bool live = e < ne || (e == ne && dbias);
    float s = 0.f;
    if (live)
        for (int b = r; b < nwg; b += 32) s += part[int64_t(b) * (ne + 1) + e];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 32);
    if (live && r == 0) {
        if (e < ne) dw[e] += s;
        else *dbias += s;
    }
}

struct Inst {
    int ci, co, ks, st, pad, circ, dout;
    const void *kern;
    size_t lds;
    int ne, ntiles_h, ntiles_w;  // tile extents TH, TW
    void (*launch)(dim3, size_t, hipStream_t, const WArgs &, const h16_t *, const h16_t *, float *, int);
};

template <int CI, int CO, int KS, int ST, int PAD, int DO, int TH, int TW>
void launch_inst(dim3 grid, size_t lds, hipStream_t s, const WArgs &a, const h16_t *x, const h16_t *g, float *part,
                 int want_gsum) {
    k_wgrad_ds<CI, CO, KS, ST, PAD, DO, TH, TW><<<grid, NT, lds, s>>>(a, x, g, part, want_gsum);
}

template <int CI, int CO, int KS, int ST, int PAD, int DO, int TH, int TW>
Inst make_inst(int circ) {
    using Gm = Geo<CI, CO, KS, ST, PAD, DO, TH, TW>;
    return Inst{CI, CO, KS, ST, PAD, circ, DO, reinterpret_cast<const void *>(k_wgrad_ds<CI, CO, KS, ST, PAD, DO, TH, TW>),
                Gm::LDS, Gm::NE, TH, TW, launch_inst<CI, CO, KS, ST, PAD, DO, TH, TW>};
}

const Inst *find_inst(const vq3d_conv_desc *d) {
    static const Inst table[] = {
        make_inst<4, 4, 3, 1, 1, 128, 4, 4>(1),   // up block ResizeConv branch conv @512^2 x 128
        make_inst<4, 4, 4, 2, 1, 64, 2, 4>(1),    // down block branch conv 512^2 -> 256^2
        make_inst<8, 8, 4, 2, 1, 32, 2, 4>(1),    // 256^2 -> 128^2
        make_inst<16, 16, 4, 2, 1, 16, 2, 4>(1),  // 128^2 -> 64^2
        make_inst<4, 8, 2, 2, 0, 64, 2, 4>(0),    // down block skip conv 4 -> 8
        make_inst<8, 16, 2, 2, 0, 32, 2, 4>(0),   // 8 -> 16
    };
    if (d->dtype != VQ3D_HALF || d->cin2 != 0) return nullptr;
    const int circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    for (const Inst &in : table) {
        if (in.ci != d->cin || in.co != d->cout || in.ks != d->kernel || in.st != d->stride || in.pad != d->pad ||
            in.dout != d->out_d || (in.pad > 0 && in.circ != circ))
            continue;
        if (d->in_d != d->out_d * in.st || d->in_h != d->out_h * in.st || d->in_w != d->out_w * in.st) continue;
        if (d->out_h % in.ntiles_h || d->out_w % in.ntiles_w || d->out_h < in.ntiles_h || d->out_w < in.ntiles_w)
            continue;
        if (int64_t(d->batch) * d->in_h * d->in_w * d->in_d * d->cin >= (int64_t(1) << 31)) continue;
        return &in;
    }
    return nullptr;
}

int n_cu() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
        (void)hipGetLastError();
    }
    return n;
}

int nwg_of(const vq3d_conv_desc *d, const Inst &in) {
    const int ntiles = d->batch * (d->out_h / in.ntiles_h) * (d->out_w / in.ntiles_w);
    // <= 2 resident workgroups per CU; partial rows capped at ~8 MB (the 16 -> 16 conv has 16,384
    // weights); a multiple of the 8 XCDs
    const int cap = std::max(8, int((size_t(8) << 20) / (size_t(in.ne + 1) * 4)));
    return std::max(1, std::min({ntiles, 2 * n_cu(), cap}) & ~7);
}

}  // namespace

bool wgrad_ds_ok(const vq3d_conv_desc *d) { return find_inst(d) != nullptr; }

size_t wgrad_ds_ws(const vq3d_conv_desc *d) {
    const Inst *in = find_inst(d);
    return in ? size_t(nwg_of(d, *in)) * (in->ne + 1) * 4 : 0;
}

int wgrad_ds(const vq3d_conv_desc *d, const void *x, const void *g, const float *pro_a, const float *pro_b, float *dw,
             float *dbias, void *ws, size_t ws_bytes, hipStream_t s) {
    const Inst *in = find_inst(d);
    if (!in || !ws || ws_bytes < wgrad_ds_ws(d)) return fail("conv(wgrad_ds): unsupported");
    static const void *attr_done[8] = {};
    for (int i = 0; i < 8; ++i) {
        if (attr_done[i] == in->kern) break;
        if (!attr_done[i]) {
            (void)hipFuncSetAttribute(in->kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(in->lds));
            attr_done[i] = in->kern;
            break;
        }
    }
    WArgs a;
    a.B = d->batch;
    a.Ho = d->out_h;
    a.Wo = d->out_w;
    a.Hi = d->in_h;
    a.Wi = d->in_w;
    a.nth = a.Ho / in->ntiles_h;
    a.ntw = a.Wo / in->ntiles_w;
    a.ntiles = a.B * a.nth * a.ntw;
    a.circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    a.pro_kind = d->pro_kind;
    a.pro_a = pro_a;
    a.pro_b = pro_b;
    const int nwg = nwg_of(d, *in);
    in->launch(dim3(unsigned(nwg)), in->lds, s, a, static_cast<const h16_t *>(x), static_cast<const h16_t *>(g),
               static_cast<float *>(ws), dbias ? 1 : 0);
    const int ne1 = in->ne + 1;
    k_wgrad_ds_reduce<<<unsigned((ne1 + NT / 32 - 1) / (NT / 32)), NT, 0, s>>>(static_cast<const float *>(ws), nwg,
                                                                               in->ne, dw, dbias);
    return check_launch("conv3d_bwd_weight(wgrad_ds)");
}

}  // namespace vq3d
