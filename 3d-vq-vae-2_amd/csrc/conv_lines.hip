// k^3 convolution (forward, and stride-1 backward-data as the forward conv of g with the
// flipped, transposed kernel) as an implicit GEMM on v_mfma_f32_16x16x32_bf16, with the K
// dimension ordered (kh, kw, [kd, c]) so that one operand chunk is CONTIGUOUS in memory.
//
// Replaces nn.Conv3d + F.pad('circular') of the residual blocks' k^3 convs
// (vqvae/layers.py:124-151: PreAct branch_conv2 3x3x3 same / 4x4x4 stride-2 down; FixupResBlock
// and EvonormResBlock conv2, layers.py:28-36, 239-247) together with their scalar glue.
//
// Channels-last means a run of k positions along D of one (h, w) line is k*C consecutive
// elements.  A workgroup owns a brick of output voxels (bh x bw x bd) and stages, per halo
// line (hh, ww), the raw D-run of input positions [d0*s - p, (d0 + bd - 1)*s - p + k) into LDS
// (circular wrap / zero padding resolved, prologue applied once per element, 16/4/2-byte
// global loads).  Output voxel (lh, lw, ld) and tap row (kh, kw) then read their whole
// (kd, c) window as ceil(k*C/8) chunks of 8 bf16 starting at element
//     line(lh*s + kh, lw*s + kw) + ld*s*C + 8j
// which is one ds_read_b128 when s*C % 8 == 0 (else 2 x b64, 4 x b32, or 5 x b32 + v_alignbyte
// for odd C).  No channel padding: C = 9 costs 9 k-steps per 16 voxels, not 14.  Window
// elements beyond k*C multiply zero weights.
//
// The grid is persistent (workgroups resident at the kernel's occupancy, bricks strided over
// them): each workgroup packs its weight B-fragment image [chunk][NT*16][8] bf16 into LDS once,
// then per brick stages the lines, runs the MFMAs, parks the fp32 accumulators in LDS and
// applies the fused epilogue with 16-byte loads / stores over the brick's contiguous D-runs.
#include "engines.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <utility>

namespace vq3d {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct LArgs {
    int B, Ca, Cb, C, N;      // GEMM-conv input channels (x then x2), output channels
    int iH, iW, iD, oH, oW, oD;
    int k, s, p, circ;
    int pro_kind;
    const float *pro_a, *pro_b;
    int bh, bw, bd, lbw, lbd;  // brick (power-of-two extents), log2 of bw / bd
    int hh, hw;                // halo lines per brick
    int LP, LS;                // positions per line, LDS line stride (elements, multiple of 8)
    int nch, NCH, nks;         // chunks per (kh, kw), chunks total, 32-wide k steps
    int nbh, nbw, nbd, nbricks;
    int ntg, ntn;              // N-tile groups (grid.y), N columns per group (NT * 16)
    int vec;                   // staging unit (elements): 8, 2 or 1
    int upl;                   // staging units per line (generic path)
    int pad0;                  // LDS elements before each line's first position (main run 16-B aligned)
    int mvec, mupl;            // main-run copy unit (0: no main-run path) and units per line
    FastDiv fupl, fC, fhw, fmupl, frun, fN;
    int vec_out;               // 16-B epilogue path allowed (one N group, bd*N % 8 == 0, no y2 / res_up2)
    int region_lines;          // bytes of the lines region (weights follow)
    int cin_split;             // dgrad: output channels < cin_split go to y, the rest to y2
    int S;                     // D-shifts per A row: a row is S consecutive output voxels along D and
                               // column n = (shift n / N, channel n % N) (S * N = 16 when S > 1)
    unsigned tapmask;          // 0, or the weight taps that may be nonzero (vq3d_conv_desc.tap_mask):
                               // the k-steps then run over the live chunks only (S == 1)
};

// chunk c = ((kh*k + kw)*nch + j) of the window order holds a live tap (mask bit of tap
// (kh*k + kw)*k + kd, flipped for the backward-data kernel); chunks past the window are dead
__host__ __device__ inline bool chunk_live(int c, int nch, int k, int C, unsigned mask, bool dgrad) {
    const int t2 = c / nch, j = c - t2 * nch;
    const int e0 = 8 * j;
    if (e0 >= k * C) return false;
    const int e1 = (e0 + 7 < k * C - 1) ? e0 + 7 : k * C - 1;
    const int K3 = k * k * k;
    for (int kd = e0 / C; kd <= e1 / C; ++kd) {
        const int tap = t2 * k + kd;
        if ((mask >> (dgrad ? K3 - 1 - tap : tap)) & 1u) return true;
    }
    return false;
}

// the live chunks in order into cmap[0 .. nlive), padded with NCH (dead) up to `total`: one wave
// (ballot prefix sums), the caller synchronises
template <bool DGRAD>
__device__ void live_chunk_map(const LArgs &a, int *cmap, int total, int lane) {
    int cnt = 0;
    for (int base = 0; base < a.NCH; base += 64) {
        const int c = base + lane;
        const bool lv = c < a.NCH && chunk_live(c, a.nch, a.k, a.C, a.tapmask, DGRAD);
        const uint64_t bal = __ballot(lv);
        if (lv) cmap[cnt + __popcll(bal & ((uint64_t(1) << lane) - 1))] = c;
        cnt += __popcll(bal);
    }
    for (int i = cnt + lane; i < total; i += 64) cmap[i] = a.NCH;
}

__device__ __forceinline__ int wrapc(int i, int n) {
    while (i < 0) i += n;
    while (i >= n) i -= n;
    return i;
}

// 8 consecutive bf16 from LDS at element offset `off` of `base` (16-B aligned); the address is
// aligned to ALN bytes (odd offsets when ALN == 2: five dwords + v_alignbyte)
template <int ALN>
__device__ __forceinline__ hx8 read8(const h16_t *base, int off) {
    uint4 r;
    if constexpr (ALN == 16) {
        r = *reinterpret_cast<const uint4 *>(base + off);
    } else if constexpr (ALN == 8) {
        const uint2 a = *reinterpret_cast<const uint2 *>(base + off);
        const uint2 b = *reinterpret_cast<const uint2 *>(base + off + 4);
        r = uint4{a.x, a.y, b.x, b.y};
    } else if constexpr (ALN == 4) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(base + off);
        r = uint4{q[0], q[1], q[2], q[3]};
    } else {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(base + (off & ~1));
        const uint32_t sh = uint32_t(off & 1) * 2u;
        const uint32_t u0 = q[0], u1 = q[1], u2 = q[2], u3 = q[3], u4 = q[4];
        r = uint4{__builtin_amdgcn_alignbyte(u1, u0, sh), __builtin_amdgcn_alignbyte(u2, u1, sh),
                  __builtin_amdgcn_alignbyte(u3, u2, sh), __builtin_amdgcn_alignbyte(u4, u3, sh)};
    }
    return __builtin_bit_cast(hx8, r);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    return uint32_t(f2h(lo)) | (uint32_t(f2h(hi)) << 16);
}

// copy VEC consecutive bf16 (prologue applied unless raw; zeros when !ok)
template <int VEC>
__device__ __forceinline__ void copy_unit(const h16_t *__restrict__ src, h16_t *dst, bool ok, const Prologue &pro,
                                          bool raw) {
    if constexpr (VEC == 8) {
        uint4 q = {0u, 0u, 0u, 0u};
        if (ok) {
            q = *reinterpret_cast<const uint4 *>(src);
            if (!raw) {
                uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    w4[j] = pack2(pro.apply(h2f_lo(w4[j])), pro.apply(h2f_hi(w4[j])));
                q = uint4{w4[0], w4[1], w4[2], w4[3]};
            }
        }
        *reinterpret_cast<uint4 *>(dst) = q;
    } else if constexpr (VEC == 2) {
        uint32_t q = 0u;
        if (ok) {
            q = *reinterpret_cast<const uint32_t *>(src);
            if (!raw) q = pack2(pro.apply(h2f_lo(q)), pro.apply(h2f_hi(q)));
        }
        *reinterpret_cast<uint32_t *>(dst) = q;
    } else {
        h16_t q = 0;
        if (ok) q = raw ? *src : f2h(pro.apply(ld(src)));
        *dst = q;
    }
}

template <int NT>
struct MT {
    static constexpr int value = NT <= 2 ? 8 : 4;  // M tiles per wave (accumulators MT * NT * 4 VGPRs)
};

// one item of the weight image: 8 bf16 of chunk c for column gi*ntot + nn; chunk
// c = ((kh*k + kw)*nch + j) holds window elements e = 8j + t = (kd, ci)
template <bool DGRAD>
__device__ __forceinline__ uint4 pack_item(const LArgs &a, const float *__restrict__ w, int wCt, int gi, int ntot,
                                           int it, const int *cmap) {
    const int K3 = a.k * a.k * a.k;
    const int ci_ = it / ntot, nn = it - ci_ * ntot;
    const int c = cmap ? cmap[ci_] : ci_;  // the compacted k-step order's chunk
    const int n = gi * ntot + nn;
    const int t2 = c / a.nch, j = c - t2 * a.nch;
    // shift mode: column n = (shift sh, channel co) reads window position pd = kd + sh * s
    const int sh = a.S > 1 ? n / a.N : 0, co = a.S > 1 ? n - sh * a.N : n;
    const bool live = c < a.NCH && (a.S > 1 ? n < 16 : n < a.N);
    int e = 8 * j;
    int kd = int(a.fC.div(uint32_t(e))) - sh * a.s, ci = e - (kd + sh * a.s) * a.C;
    uint32_t pk[4];
#pragma unroll
    for (int t = 0; t < 8; t += 2) {
        float v2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float val = 0.f;
            if (live && kd >= 0 && kd < a.k) {
                const int tap = t2 * a.k + kd;  // t2 = kh * k + kw
                val = DGRAD ? w[(int64_t(ci) * wCt + co) * K3 + (K3 - 1 - tap)] : w[(int64_t(co) * wCt + ci) * K3 + tap];
            }
            v2[h] = val;
            if (++ci == a.C) {
                ci = 0;
                ++kd;
            }
        }
        pk[t / 2] = pack2(v2[0], v2[1]);
    }
    return uint4{pk[0], pk[1], pk[2], pk[3]};
}

// the whole image [group][chunk][ntot] into global memory (caller workspace), once per call
template <bool DGRAD>
__global__ __launch_bounds__(256) void k_lines_pack(LArgs a, const float *__restrict__ w, int wCt, int ntot,
                                                    uint4 *__restrict__ out) {
    __shared__ int cmap[1024];
    const int items = a.nks * 4 * ntot;
    if (a.tapmask) {
        if (threadIdx.x < 64) live_chunk_map<DGRAD>(a, cmap, a.nks * 4, threadIdx.x);
        __syncthreads();
    }
    const int it = blockIdx.x * 256 + threadIdx.x;
    if (it < items)
        out[int64_t(blockIdx.y) * items + it] = pack_item<DGRAD>(a, w, wCt, blockIdx.y, ntot, it, a.tapmask ? cmap : nullptr);
}

template <int NT, int ALN, bool DGRAD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((NT == 1 || NT == 3) ? 4 : 2))) void k_lines(LArgs a, const h16_t *__restrict__ x, const h16_t *__restrict__ x2,
                                              const float *__restrict__ w, int wCt, const uint4 *__restrict__ wpk,
                                              FwdEpi<h16_t> fe,
                                              BwdEpi<h16_t> be, const float *__restrict__ gscale,
                                              h16_t *__restrict__ y, h16_t *__restrict__ y2, float *dpre,
                                              float *dpost, GridSum gsum) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int MTW = MT<NT>::value;
    constexpr int NTOT = NT * 16;
    h16_t *lines = reinterpret_cast<h16_t *>(smem);                     // [nlines][LS]
    float *otile = reinterpret_cast<float *>(smem);                       // after the MFMAs: [nvb][nw] fp32
    uint4 *wl = reinterpret_cast<uint4 *>(smem + a.region_lines);         // [chunk][NTOT] fragments
    int *ctab = reinterpret_cast<int *>(wl + a.nks * 4 * NTOT);           // [chunk] element offsets
    __shared__ float red[8];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row = lane & 15, kq = lane >> 4;
    const int nlines = a.hh * a.hw;
    const int nvb = a.bh * a.bw * a.bd;
    const int nmt = (nvb / a.S + 15) / 16;  // m-tiles of 16 A rows (rows = groups of S voxels along D)
    const int gi = blockIdx.y;
    const int nw = min(NTOT, a.N - gi * NTOT);  // output channels of this group
    const int ncol = a.S > 1 ? 16 : nw;           // MFMA columns holding outputs

    // ---- once per workgroup: weight image of this N group + chunk offset table (with a tap mask:
    // the live chunks in order, ctab first holding their chunk indices)
    if (a.tapmask) {
        if (wave == 0) live_chunk_map<DGRAD>(a, ctab, a.nks * 4, lane);
        __syncthreads();
    }
    {
        const int items = a.nks * 4 * NTOT;
        if (wpk) {  // pre-packed image: 16-byte copies
            const uint4 *src = wpk + int64_t(gi) * items;
            for (int it = tid; it < items; it += 256) wl[it] = src[it];
        } else {
            for (int it = tid; it < items; it += 256)
                wl[it] = pack_item<DGRAD>(a, w, wCt, gi, NTOT, it, a.tapmask ? ctab : nullptr);
        }
    }
    if (a.tapmask) __syncthreads();  // the chunk indices are read above, rewritten as offsets below
    for (int i = tid; i < a.nks * 4; i += 256) {
        const int c = a.tapmask ? ctab[i] : i;
        int off = 0;  // padding chunks: zero weights, any valid window
        if (c < a.NCH) {
            const int t2 = c / a.nch, j = c - t2 * a.nch;
            const int kh = t2 / a.k, kw = t2 - kh * a.k;
            off = (kh * a.hw + kw) * a.LS + 8 * j;
        }
        ctab[i] = off;
    }
    // this lane's A-row window base per M tile (wave w owns tiles w, w + 4, ...)
    int rowbase[MTW];
#pragma unroll
    for (int m = 0; m < MTW; ++m) {
        int v = ((wave + 4 * m) * 16 + row) * a.S;
        if (v >= nvb) v = 0;
        const int ld_ = v & (a.bd - 1), lw_ = (v >> a.lbd) & (a.bw - 1), lh_ = v >> (a.lbd + a.lbw);
        rowbase[m] = ((lh_ * a.s) * a.hw + lw_ * a.s) * a.LS + a.pad0 + ld_ * a.s * a.C;
    }
    const Prologue pro = make_prologue(a.pro_kind, a.pro_a, a.pro_b);
    const float gs = gscale ? *gscale : 1.f;
    const float sc = fe.scale ? *fe.scale : 1.f, bias = fe.bias ? *fe.bias : 0.f;
    const float aa = fe.act_a ? *fe.act_a : 0.f, ab = fe.act_b ? *fe.act_b : 0.f;
    ActDeriv dv;
    dv.mode = (DGRAD && be.aux) ? be.mode : 0;
    dv.p = (dv.mode && be.p) ? *be.p : 0.f;
    float pre = 0.f, post = 0.f;
    const bool raw = pro.kind == VQ3D_PRO_NONE;

    const TileSched bsc = xcd_sched(a.nbricks);
    for (int brick = bsc.t; brick < bsc.end; brick += bsc.step) {
        int bi = brick;
        const int bzd = bi % a.nbd; bi /= a.nbd;
        const int bzw = bi % a.nbw; bi /= a.nbw;
        const int bzh = bi % a.nbh;
        const int b = bi / a.nbh;
        const int oh0 = bzh * a.bh, ow0 = bzw * a.bw, od0 = bzd * a.bd;
        const int ih0 = oh0 * a.s - a.p, iw0 = ow0 * a.s - a.p, id0 = od0 * a.s - a.p;
        __syncthreads();  // previous brick's epilogue is done with the LDS

        // ---- stage the halo lines.  Main run (when planned): the brick's own bd*s positions
        // are contiguous and 16-B aligned in HBM and land 16-B aligned in LDS (pad0), copied in
        // units of mvec elements; the p + (k - 1 - p) edge positions (wrap / zero padding) go
        // element-group wise.  Otherwise every position takes the generic unit path.
        {
            const int64_t bbase = int64_t(b) * a.iH * a.iW * a.iD;
            auto line_src = [&](int li, int id, bool &ok) -> int64_t {
                const int lh_ = int(a.fhw.div(uint32_t(li))), lw_ = li - lh_ * a.hw;
                int ih = ih0 + lh_, iw = iw0 + lw_;
                if (a.circ) {
                    ih = wrapc(ih, a.iH);
                    iw = wrapc(iw, a.iW);
                    id = wrapc(id, a.iD);
                    ok = true;
                } else {
                    ok = unsigned(ih) < unsigned(a.iH) && unsigned(iw) < unsigned(a.iW) &&
                         unsigned(id) < unsigned(a.iD);
                }
                return bbase + (int64_t(ih) * a.iW + iw) * a.iD + id;  // voxel index
            };
            if (a.mvec) {
                const int total = nlines * a.mupl;
                for (int u = tid; u < total; u += 256) {
                    const int li = int(a.fmupl.div(uint32_t(u))), r = u - li * a.mupl;
                    bool ok;
                    const int64_t vox = line_src(li, od0 * a.s, ok);
                    const h16_t *src = x + vox * a.C + r * a.mvec;
                    h16_t *dst = lines + li * a.LS + a.pad0 + a.p * a.C + r * a.mvec;
                    if (a.mvec == 8) copy_unit<8>(src, dst, ok, pro, raw);
                    else if (a.mvec == 2) copy_unit<2>(src, dst, ok, pro, raw);
                    else copy_unit<1>(src, dst, ok, pro, raw);
                }
                const int E = a.LP - a.bd * a.s;  // edge positions per line
                const int eupl = E * a.C / a.vec;
                const int tot_e = nlines * eupl;
                for (int u = tid; u < tot_e; u += 256) {
                    const int li = u / eupl, r = u - li * eupl;
                    const int e = r * a.vec;
                    const int pe = int(a.fC.div(uint32_t(e))), c = e - pe * a.C;
                    const int pos = pe < a.p ? pe : pe + a.bd * a.s;
                    bool ok;
                    const int64_t vox = line_src(li, id0 + pos, ok);
                    const h16_t *src = x + vox * a.C + c;
                    h16_t *dst = lines + li * a.LS + a.pad0 + pos * a.C + c;
                    if (a.vec == 8) copy_unit<8>(src, dst, ok, pro, raw);
                    else if (a.vec == 2) copy_unit<2>(src, dst, ok, pro, raw);
                    else copy_unit<1>(src, dst, ok, pro, raw);
                }
            } else {
                const int total = nlines * a.upl;
                for (int u = tid; u < total; u += 256) {
                    const int li = int(a.fupl.div(uint32_t(u))), r = u - li * a.upl;
                    const int e = r * a.vec;
                    const int pos = int(a.fC.div(uint32_t(e))), c = e - pos * a.C;
                    bool ok;
                    const int64_t vox = line_src(li, id0 + pos, ok);
                    h16_t *dst = lines + li * a.LS + a.pad0 + e;
                    const bool second = c >= a.Ca;
                    const h16_t *src = second ? x2 + vox * a.Cb + (c - a.Ca) : x + vox * a.Ca + c;
                    if (a.vec == 8) copy_unit<8>(src, dst, ok, pro, raw);
                    else if (a.vec == 2) copy_unit<2>(src, dst, ok, pro, raw);
                    else copy_unit<1>(src, dst, ok, pro, raw);
                }
            }
            // pad0 head and slack tail of each line (read by edge window chunks): zero
            const int tail0 = a.pad0 + a.LP * a.C;
            const int z = a.LS - tail0 + a.pad0;
            for (int e = tid; e < nlines * z; e += 256) {
                const int li = e / z, r = e - li * z;
                lines[li * a.LS + (r < a.pad0 ? r : tail0 + r - a.pad0)] = 0;
            }
        }
        __syncthreads();

        // ---- MFMA over the chunks
        f32x4 acc[MTW][NT];
#pragma unroll
        for (int m = 0; m < MTW; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int ks = 0; ks < a.nks; ++ks) {
            const int c = ks * 4 + kq;
            const int off = ctab[c];
            hx8 bfr[NT];
#pragma unroll
            for (int n = 0; n < NT; ++n) bfr[n] = __builtin_bit_cast(hx8, wl[c * NTOT + n * 16 + row]);
#pragma unroll
            for (int m = 0; m < MTW; ++m) {
                if (wave + 4 * m >= nmt) break;
                const hx8 afr = read8<ALN>(lines, rowbase[m] + off);
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    acc[m][n] = VQ3D_MFMA_16X16X32(afr, bfr[n], acc[m][n], 0, 0, 0);
            }
        }

        // ---- accumulators -> LDS tile [v][nw] fp32 (lane column co, rows kq*4 + i)
        __syncthreads();
#pragma unroll
        for (int m = 0; m < MTW; ++m) {
            if (wave + 4 * m >= nmt) break;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
                const int cl = n * 16 + row;
                if (cl >= ncol) continue;
#pragma unroll
                for (int i = 0; i < 4; ++i) {  // row g holds voxels g*S .. g*S + S-1: [v][nw] = [g][S*nw]
                    const int g = (wave + 4 * m) * 16 + kq * 4 + i;
                    if (g * a.S < nvb) otile[g * ncol + cl] = acc[m][n][i];
                }
            }
        }
        __syncthreads();

        // ---- epilogue over the tile.  Vector path: the brick is inside the grid, the group
        // holds every output channel, so the tile [v][N] is bh*bw contiguous runs of bd*N
        // elements in HBM: 8 elements (16 B) per thread-step.
        const int64_t ob = int64_t(b) * a.oH * a.oW * a.oD;
        const bool inside = oh0 + a.bh <= a.oH && ow0 + a.bw <= a.oW && od0 + a.bd <= a.oD;
        if (inside && a.vec_out) {
            const int runlen = a.bd * a.N;
            for (int q = tid; q < nvb * a.N / 8; q += 256) {
                const int e0 = 8 * q;
                const int r = int(a.frun.div(uint32_t(e0))), off = e0 - r * runlen;
                const int lh_ = r >> a.lbw, lw_ = r & (a.bw - 1);
                const int64_t gaddr = (ob + (int64_t(oh0 + lh_) * a.oW + ow0 + lw_) * a.oD + od0) * a.N + off;
                const float4 t0 = *reinterpret_cast<const float4 *>(otile + e0);
                const float4 t1 = *reinterpret_cast<const float4 *>(otile + e0 + 4);
                float v8[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
                int co = int(a.fN.div(uint32_t(off)));
                co = off - co * a.N;
                if (!DGRAD) {
                    float r8[8];
                    if (fe.res) {
                        const uint4 rq = *reinterpret_cast<const uint4 *>(fe.res + gaddr);
                        const uint32_t rw[4] = {rq.x, rq.y, rq.z, rq.w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            r8[2 * j] = h2f_lo(rw[j]);
                            r8[2 * j + 1] = h2f_hi(rw[j]);
                        }
                    }
                    uint32_t o4[4];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        float val = v8[t];
                        if (fe.scale) val = val * sc;
                        if (fe.bias) val = val + bias;
                        if (fe.cbias) val = val + fe.cbias[co];
                        if (fe.res) val = val + r8[t];
                        v8[t] = epi_act(fe.act, val, aa, ab);
                        if (++co == a.N) co = 0;
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) o4[j] = pack2(v8[2 * j], v8[2 * j + 1]);
                    *reinterpret_cast<uint4 *>(y + gaddr) = uint4{o4[0], o4[1], o4[2], o4[3]};
                } else {
                    float x8[8], d8[8];
                    if (dv.mode) {
                        const uint4 rq = *reinterpret_cast<const uint4 *>(be.aux + gaddr);
                        const uint32_t rw[4] = {rq.x, rq.y, rq.z, rq.w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            x8[2 * j] = h2f_lo(rw[j]);
                            x8[2 * j + 1] = h2f_hi(rw[j]);
                        }
                    }
                    if (be.addend) {
                        const uint4 rq = *reinterpret_cast<const uint4 *>(be.addend + gaddr);
                        const uint32_t rw[4] = {rq.x, rq.y, rq.z, rq.w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            d8[2 * j] = h2f_lo(rw[j]);
                            d8[2 * j + 1] = h2f_hi(rw[j]);
                        }
                    }
                    uint32_t o4[4];
#pragma unroll
                    for (int t = 0; t < 8; ++t) {
                        float val = v8[t];
                        if (gscale) val = val * gs;
                        pre += val;
                        if (dv.mode) val = val * dv(x8[t]);
                        post += val;
                        if (be.addend) val = val + d8[t];
                        v8[t] = val;
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) o4[j] = pack2(v8[2 * j], v8[2 * j + 1]);
                    *reinterpret_cast<uint4 *>(y + gaddr) = uint4{o4[0], o4[1], o4[2], o4[3]};
                }
            }
            continue;
        }
        // scalar path: any brick, any column group
        for (int e2 = tid; e2 < nvb * NTOT; e2 += 256) {
            const int v = e2 / NTOT, cl = e2 - v * NTOT;  // NTOT is a compile-time constant
            if (cl >= nw) continue;
            const int e = v * nw + cl;
            const int co = gi * NTOT + cl;
            const int ld_ = v & (a.bd - 1), lw_ = (v >> a.lbd) & (a.bw - 1), lh_ = v >> (a.lbd + a.lbw);
            const int oh = oh0 + lh_, ow = ow0 + lw_, od = od0 + ld_;
            if (oh >= a.oH || ow >= a.oW || od >= a.oD) continue;
            const int64_t vox = ob + (int64_t(oh) * a.oW + ow) * a.oD + od;
            float val = otile[e];
            if (!DGRAD) {
                if (fe.scale) val = val * sc;
                if (fe.bias) val = val + bias;
                if (fe.cbias) val = val + fe.cbias[co];
                if (fe.res) {
                    if (!fe.res_up2) {
                        val = val + ld(fe.res + vox * a.N + co);
                    } else {
                        const int rH = a.oH / 2, rW = a.oW / 2, rD = a.oD / 2;
                        int h0, h1, w0, w1, d0, d1;
                        float lh, lw, ldd;
                        up_coeff(oh, rH, h0, h1, lh);
                        up_coeff(ow, rW, w0, w1, lw);
                        up_coeff(od, rD, d0, d1, ldd);
                        auto R = [&](int hh, int ww, int dd) {
                            return ld(fe.res + (((int64_t(b) * rH + hh) * rW + ww) * rD + dd) * a.N + co);
                        };
                        val = val + ((1.f - lh) * ((1.f - lw) * ((1.f - ldd) * R(h0, w0, d0) + ldd * R(h0, w0, d1)) +
                                                  lw * ((1.f - ldd) * R(h0, w1, d0) + ldd * R(h0, w1, d1))) +
                                     lh * ((1.f - lw) * ((1.f - ldd) * R(h1, w0, d0) + ldd * R(h1, w0, d1)) +
                                           lw * ((1.f - ldd) * R(h1, w1, d0) + ldd * R(h1, w1, d1))));
                    }
                }
                st(y + vox * a.N + co, epi_act(fe.act, val, aa, ab));
            } else {
                if (gscale) val = val * gs;
                if (co < a.cin_split) {
                    const int64_t o = vox * a.cin_split + co;
                    pre += val;
                    if (dv.mode) val = val * dv(ld(be.aux + o));
                    post += val;
                    if (be.addend) val = val + ld(be.addend + o);
                    st(y + o, val);
                } else {
                    st(y2 + vox * (a.N - a.cin_split) + (co - a.cin_split), val);
                }
            }
        }
    }
    if (DGRAD && (dpre || dpost)) {
        {  // both sums in one barrier pair (bit-identical to two block_sum calls)
            float pp[2] = {pre, post};
            block_sums<float, 256, 2, 4>(pp, red);
            pre = pp[0];
            post = pp[1];
        }
        grid_sum2<256>(gsum, pre, post, dpre, dpost, red);
    }
}

// ------------------------------------------------------------------------------------------- host
int pow2_ceil(int v) {
    int r = 1;
    while (r < v) r *= 2;
    return r;
}
int ilog2(int v) {
    int r = 0;
    while ((1 << r) < v) ++r;
    return r;
}

constexpr size_t kLdsMax = 160 * 1024 - 256;  // room for the kernels' static LDS

struct Plan {
    LArgs a;
    int nt, aln;
    size_t lds;
    bool ok;
};

// region 0 holds the staged lines, then (after the MFMAs) the fp32 output tile
size_t region0_of(const LArgs &a, int nt) {
    const size_t lines = size_t(a.hh) * a.hw * a.LS * 2;
    const size_t tile = size_t(a.bh) * a.bw * a.bd * std::min(a.N, nt * 16) * 4;
    return (std::max(lines, tile) + 15) & ~size_t(15);
}

size_t lds_of(const LArgs &a, int nt) {
    return region0_of(a, nt) + size_t(a.nks) * 4 * nt * 16 * 16 + size_t(a.nks) * 4 * 4;
}

void set_brick(LArgs &a, int bh, int bw, int bd) {
    a.bh = bh;
    a.bw = bw;
    a.bd = bd;
    a.lbw = ilog2(bw);
    a.lbd = ilog2(bd);
    a.hh = (bh - 1) * a.s + a.k;
    a.hw = (bw - 1) * a.s + a.k;
    a.LP = (bd - 1) * a.s + a.k;
    a.pad0 = (8 - (a.p * a.C) % 8) % 8;
    a.LS = (a.pad0 + a.LP * a.C + 8 + 7) / 8 * 8;
}

// GEMM-conv geometry: input (B, Ca+Cb, iH, iW, iD) -> output (B, N, oH, oW, oD)
Plan plan(int B, int Ca, int Cb, int N, int iH, int iW, int iD, int oH, int oW, int oD, int k, int s, int p,
          int circ, int S, unsigned tapmask, bool dgrad) {
    Plan P = {};
    LArgs &a = P.a;
    a.B = B; a.Ca = Ca; a.Cb = Cb; a.C = Ca + Cb; a.N = N;
    a.iH = iH; a.iW = iW; a.iD = iD; a.oH = oH; a.oW = oW; a.oD = oD;
    a.k = k; a.s = s; a.p = p; a.circ = circ;
    if (s != 1 && s != 2) return P;
    if (int64_t(B) * iH * iW * iD * a.C >= (int64_t(1) << 31) || int64_t(B) * oH * oW * oD * N >= (int64_t(1) << 31))
        return P;
    a.S = S;
    a.nch = (((a.S - 1) * s + k) * a.C + 7) / 8;
    a.NCH = k * k * a.nch;
    a.nks = (a.NCH + 3) / 4;
    a.tapmask = 0;
    if (tapmask && S == 1 && k <= 3 && a.NCH <= 1016) {  // k-steps over the live chunks only
        int nlive = 0;
        for (int c = 0; c < a.NCH; ++c) nlive += chunk_live(c, a.nch, k, a.C, tapmask, dgrad);
        a.tapmask = tapmask;
        a.nks = std::max(1, (nlive + 3) / 4);
    }
    auto div = [](int v, int d) { return v % d == 0; };
    a.vec = (div(Ca, 8) && div(Cb, 8)) ? 8 : ((div(Ca, 2) && div(Cb, 2)) ? 2 : 1);
    const int ntr = (N + 15) / 16;
    static const bool verbose = std::getenv("VQ3D_VERBOSE") != nullptr;
    // N tiles per workgroup: all of them when they fit (<= 4), else groups of 4 / 2 / 1
    for (int nt : {4, 3, 2, 1}) {
        if (nt > ntr) continue;
        if (nt == 3 && ntr != 3) continue;
        const int mtw = nt <= 2 ? 8 : 4;
        const int target = 64 * mtw * a.S;
        int bd = std::min(pow2_ceil(oD), 32);
        int bw = std::min(pow2_ceil(oW), std::max(1, target / (bd * 4)));
        bw = 1 << ilog2(bw);
        int bh = std::min(pow2_ceil(oH), std::max(1, target / (bd * bw)));
        bh = std::max(1, 1 << (ilog2(bh + 1) - 1));
        while (bh * bw * bd > target) {
            if (bh > 1) bh /= 2;
            else if (bw > 1) bw /= 2;
            else bd /= 2;
        }
        set_brick(a, bh, bw, bd);
        // shrink the brick while it does not fit, or while the grid would leave CUs idle
        auto nwg = [&]() {
            return int64_t(B) * ((oH + a.bh - 1) / a.bh) * ((oW + a.bw - 1) / a.bw) * ((oD + a.bd - 1) / a.bd) *
                   ((ntr + nt - 1) / nt);
        };
        while (true) {
            const bool fits = lds_of(a, nt) <= kLdsMax;
            const bool small = a.bh * a.bw * a.bd <= 64;
            if (fits && (small || nwg() >= 512)) break;
            if (small && !fits) break;
            if (a.bh >= a.bw && a.bh > 1) set_brick(a, a.bh / 2, a.bw, a.bd);
            else if (a.bw > 1) set_brick(a, a.bh, a.bw / 2, a.bd);
            else if (a.bd > 1) set_brick(a, a.bh, a.bw, a.bd / 2);
            else break;
        }
        if (lds_of(a, nt) > kLdsMax) continue;
        P.nt = nt;
        break;
    }
    if (!P.nt || a.bd % a.S) return Plan{};
    a.ntg = (ntr + P.nt - 1) / P.nt;
    a.ntn = P.nt * 16;
    a.nbh = (oH + a.bh - 1) / a.bh;
    a.nbw = (oW + a.bw - 1) / a.bw;
    a.nbd = (oD + a.bd - 1) / a.bd;
    a.nbricks = B * a.nbh * a.nbw * a.nbd;
    a.upl = a.LP * a.C / a.vec;
    a.fupl = FastDiv(uint32_t(a.upl));
    {
        // window element offsets are pad0 + ld*s*C + 8j (+ multiples of LS)
        const int sc = s * a.C * a.S;
        int e = 8;
        while (e > 1 && (sc % e || a.pad0 % e)) e /= 2;
        P.aln = 2 * e;
        // main-run path: no brick overhang in D, one input tensor, aligned line bases
        const int mrun = a.bd * s * a.C;
        a.mvec = 0;
        if (Cb == 0 && oD % a.bd == 0 && int64_t(oD) * s <= iD) {
            if (mrun % 8 == 0 && (int64_t(iD) * a.C) % 8 == 0) a.mvec = 8;
            else if (mrun % 2 == 0 && (int64_t(iD) * a.C) % 2 == 0) a.mvec = 2;
            else a.mvec = 1;
        }
        a.mupl = a.mvec ? mrun / a.mvec : 1;
        a.fmupl = FastDiv(uint32_t(a.mupl));
    }
    a.fC = FastDiv(uint32_t(a.C));
    a.fhw = FastDiv(uint32_t(a.hw));
    a.region_lines = int(region0_of(a, P.nt));
    a.frun = FastDiv(uint32_t(a.bd * N));
    a.fN = FastDiv(uint32_t(N));
    a.vec_out = a.ntg == 1 && (a.bd * N) % 8 == 0;
    P.lds = lds_of(a, P.nt);
    P.ok = true;
    if (verbose)
        std::fprintf(stderr, "[vq3d] lines plan C%d->N%d k%d s%d: brick %dx%dx%d nt %d groups %d aln %d vec %d mvec %d lds %zu wg %d\n",
                     a.C, N, k, s, a.bh, a.bw, a.bd, P.nt, a.ntg, P.aln, a.vec, a.mvec, P.lds, a.nbricks * a.ntg);
    if (verbose && a.S > 1) std::fprintf(stderr, "[vq3d] lines plan: %d D-shifts per MFMA row\n", a.S);
    return P;
}

// S > 1 (several output voxels along D per MFMA row) when the 16 columns would otherwise hold
// only 4 or 8 output channels and the output depth holds whole groups; else S = 1.  4 -> 4 @512^2x128
// forward 719 -> 389 us, backward-data 828 -> 403 us (7 instead of 20 k-steps per 64 voxels)
Plan plan_s(int B, int Ca, int Cb, int N, int iH, int iW, int iD, int oH, int oW, int oD, int k, int s, int p,
            int circ, unsigned tapmask, bool dgrad) {
    if ((N == 4 || N == 8) && s == 1 && oD % (16 / N) == 0) {  // stride 2: measured slower (larger halo)
        const Plan P = plan(B, Ca, Cb, N, iH, iW, iD, oH, oW, oD, k, s, p, circ, 16 / N, 0u, dgrad);
        if (P.ok) return P;
    }
    return plan(B, Ca, Cb, N, iH, iW, iD, oH, oW, oD, k, s, p, circ, 1, tapmask, dgrad);
}

Plan plan_for(const vq3d_conv_desc *d, bool dgrad) {
    if (d->dtype != VQ3D_HALF || d->kernel < 2) return Plan{};
    const int circ = d->pad_mode == VQ3D_PAD_CIRCULAR;
    if (!dgrad)
        return plan_s(d->batch, d->cin, d->cin2, d->cout, d->in_h, d->in_w, d->in_d, d->out_h, d->out_w, d->out_d,
                      d->kernel, d->stride, d->pad, circ, d->tap_mask, false);
    const int pp = d->kernel - 1 - d->pad;
    if (d->stride != 1 || pp < 0) return Plan{};
    return plan_s(d->batch, d->cout, 0, d->cin + d->cin2, d->out_h, d->out_w, d->out_d, d->in_h, d->in_w, d->in_d,
                  d->kernel, 1, pp, circ, d->tap_mask, true);
}

// persistent grid: workgroups resident at the kernel's occupancy (per CU), bricks strided
template <typename K>
unsigned resident_blocks(K kernel, size_t lds, unsigned units) {
    static std::map<std::pair<const void *, size_t>, int> cache;
    const auto key = std::make_pair(reinterpret_cast<const void *>(kernel), lds);
    int per_cu;
    auto it = cache.find(key);
    if (it != cache.end()) {
        per_cu = it->second;
    } else {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds) != hipSuccess || per_cu < 1)
            per_cu = 1;
        (void)hipGetLastError();
        cache[key] = per_cu;
        if (std::getenv("VQ3D_VERBOSE")) std::fprintf(stderr, "[vq3d] lines occupancy %d blocks/CU at lds %zu\n", per_cu, lds);
    }
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1)
            n_cu = 256;
        (void)hipGetLastError();
    }
    return std::max(1u, std::min(units, unsigned(per_cu * n_cu)));
}

template <bool DGRAD>
void launch(const Plan &P, const h16_t *x, const h16_t *x2, const float *w, int wCt, const uint4 *wpk,
            const FwdEpi<h16_t> &fe,
            const BwdEpi<h16_t> &be, const float *gscale, h16_t *y, h16_t *y2, float *dpre, float *dpost,
            hipStream_t s) {
#define K(NT, ALN)                                                                                            \
    {                                                                                                         \
        auto kern = k_lines<NT, ALN, DGRAD>;                                                                  \
        static bool attr = false;                                                                             \
        if (!attr) {                                                                                          \
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),                                   \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsMax));              \
            (void)hipGetLastError();                                                                          \
            attr = true;                                                                                      \
        }                                                                                                     \
        const unsigned nb = resident_blocks(kern, P.lds, unsigned(P.a.nbricks));                              \
        const dim3 grid{nb, unsigned(P.a.ntg), 1u};                                                           \
        const GridSum gs = grid_sum_for(s, int64_t(nb) * P.a.ntg, DGRAD && (dpre || dpost));                    \
        kern<<<grid, 256, P.lds, s>>>(P.a, x, x2, w, wCt, wpk, fe, be, gscale, y, y2, dpre, dpost, gs);       \
    }
#define ALNS(NT)                                                                                              \
    switch (P.aln) {                                                                                          \
    case 16: K(NT, 16) break;                                                                                 \
    case 8: K(NT, 8) break;                                                                                   \
    case 4: K(NT, 4) break;                                                                                   \
    default: K(NT, 2) break;                                                                                  \
    }
    switch (P.nt) {
    case 1: ALNS(1) break;
    case 2: ALNS(2) break;
    case 3: ALNS(3) break;
    default: ALNS(4) break;
    }
#undef ALNS
#undef K
}

}  // namespace

static size_t ws_of(const Plan &P) { return size_t(P.a.ntg) * P.a.nks * 4 * P.a.ntn * 16; }

// packed B-fragment image of every N group (k_lines_pack), filled per call
size_t lines_workspace(const vq3d_conv_desc *d, bool dgrad) {
    const Plan P = plan_for(d, dgrad);
    return P.ok ? ws_of(P) : 0;
}

bool lines_applicable(const vq3d_conv_desc *d, bool dgrad) { return plan_for(d, dgrad).ok; }

int launch_lines(const vq3d_conv_desc *d, bool dgrad, const void *x, const void *x2, const float *w, const float *pa,
                 const float *pb, const FwdEpi<h16_t> &fe, const BwdEpi<h16_t> &be, const float *gscale, void *y,
                 void *y2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t s) {
    Plan P = plan_for(d, dgrad);
    if (!P.ok) return fail("conv(lines): geometry not supported");
    P.a.pro_kind = dgrad ? VQ3D_PRO_NONE : d->pro_kind;
    P.a.pro_a = pa;
    P.a.pro_b = pb;
    P.a.cin_split = d->cin;
    auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    // 16-B epilogue: one output tensor (no y2), no upsampled residual, aligned operands
    if (dgrad) {
        P.a.vec_out = P.a.vec_out && d->cin2 == 0 && al(y) && (!be.aux || al(be.aux)) && (!be.addend || al(be.addend));
    } else {
        P.a.vec_out = P.a.vec_out && !fe.res_up2 && al(y) && (!fe.res || al(fe.res));
    }
    const int wCt = d->cin + d->cin2;
    // pre-pack the weights once per call when the caller gave room (else each workgroup packs)
    const uint4 *wpk = nullptr;
    const int items_per_wg = P.a.nks * 4 * P.a.ntn;
    const bool want_pack = items_per_wg > 2048;
    if (want_pack && ws && ws_bytes >= ws_of(P)) {  // small images are packed in-kernel
        const int items = P.a.nks * 4 * P.a.ntn;
        const dim3 pg{unsigned((items + 255) / 256), unsigned(P.a.ntg), 1u};
        if (dgrad) k_lines_pack<true><<<pg, 256, 0, s>>>(P.a, w, wCt, P.a.ntn, static_cast<uint4 *>(ws));
        else k_lines_pack<false><<<pg, 256, 0, s>>>(P.a, w, wCt, P.a.ntn, static_cast<uint4 *>(ws));
        wpk = static_cast<const uint4 *>(ws);
    }
    if (dgrad)
        launch<true>(P, (const h16_t *)x, nullptr, w, wCt, wpk, fe, be, gscale, (h16_t *)y, (h16_t *)y2, dpre, dpost, s);
    else
        launch<false>(P, (const h16_t *)x, (const h16_t *)x2, w, wCt, wpk, fe, be, nullptr, (h16_t *)y, nullptr,
                      nullptr, nullptr, s);
    return check_launch(dgrad ? "conv3d_bwd_data(lines)" : "conv3d_fwd(lines)");
}

}  // namespace vq3d
