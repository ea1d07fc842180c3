// Host entry points of the specialised conv engines, each in its own translation unit so the
// big template files do not have to be rebuilt together.  Called from conv3d.hip's dispatch.
#pragma once
#include "common.h"

namespace vq3d {

// forward epilogue (vq3d_conv_epilogue), by value
template <typename T>
struct FwdEpi {
    const float *scale, *bias, *cbias;
    const T *res;
    int res_up2, act;
    const float *act_a, *act_b;
    int oH, oW, oD;  // output grid (filled by engines that need voxel coordinates)
};

// backward-data epilogue (vq3d_dgrad_epilogue) resolved on the host: mode 0 none,
// 1 elu'(aux + *p) (pre-prologue input), 2 from activated aux with offset *p
template <typename T>
struct BwdEpi {
    const T *aux;
    int mode;
    const float *p;
    const T *addend;
};


// 1x1x1 weight gradient (and the epilogue-parameter gradients of that conv), ACCUMULATED:
//   G[co][ci] = sum_v g[v][co] * pro(x|x2)[v][ci]
//   dw += escale * G ; dscale += sum W*G ; dbias += sum g ; dcbias[co] += sum_v g[v][co]
// Partials per workgroup go to `workspace` (pw_wgrad_workspace(d) bytes) and are summed in a
// fixed order by a second kernel: deterministic, no same-address atomics.
size_t pw_wgrad_workspace(const vq3d_conv_desc *d);
int launch_pw_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pro_a,
                    const float *pro_b, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                    float *dcbias, void *workspace, size_t ws_bytes, hipStream_t s);
// PixelSNAIL 1x1x1 weight gradient over 16-bit voxel rows (ACCUMULATED, deterministic):
//   dw[cg][cx] += sum_v g[v * ldg + co] x[v * ldx + ci], db[cg] += sum_v g[v * ldg + co] (db may be null)
size_t rows_wgrad_workspace(int64_t nrows, int cg, int cx);
int launch_rows_gemm(int64_t nrows, int k, int n, const void *x, int64_t ldx, const void *w, int64_t ldw, int trans_w,
                     const float *bias, void *y, int64_t ldy, hipStream_t s);
int launch_rows_wgrad(int64_t nrows, int cg, int cx, const void *g, int64_t ldg, const void *x, int64_t ldx, float *dw,
                      float *db, void *workspace, size_t ws_bytes, hipStream_t s);

// k^3 conv on the MFMA "lines" engine (conv_lines.hip): forward, or (dgrad) stride-1 backward-data.
// lines_applicable: bf16 and a geometry the engine plans; lines_workspace: packed-weight bytes.
bool lines_applicable(const vq3d_conv_desc *d, bool dgrad);
size_t lines_workspace(const vq3d_conv_desc *d, bool dgrad);
int launch_lines(const vq3d_conv_desc *d, bool dgrad, const void *x, const void *x2, const float *w, const float *pa,
                 const float *pb, const FwdEpi<h16_t> &fe, const BwdEpi<h16_t> &be, const float *gscale, void *y,
                 void *y2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t s);

// k^3 weight gradient on the lines layout (conv_lines_wgrad.hip), bf16, cout <= 64: per-workgroup
// partial G in the workspace (lines_wgrad_workspace bytes), summed in a fixed order
bool lines_wgrad_applicable(const vq3d_conv_desc *d);
size_t lines_wgrad_workspace(const vq3d_conv_desc *d);
int launch_lines_wgrad(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g, const float *pro_a,
                       const float *pro_b, const float *w, const float *escale, float *dw, float *dscale, float *dbias,
                       float *dcbias, void *ws, size_t ws_bytes, hipStream_t s);

// stride-2 (k = 2 or 4) backward-data visiting only the parity-matching taps (conv_s2.hip)
bool dgrad_s2_applicable(const vq3d_conv_desc *d);
template <typename T>
int launch_dgrad_s2(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w, const BwdEpi<T> &be,
                    void *gx, void *gx2, float *dpre, float *dpost, hipStream_t s);

// trilinear x2 upsample forward / adjoint (upsample.hip)
int launch_up2_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd, const void *x,
                   int32_t pro_kind, const float *pro_a, const float *pro_b, void *y, hipStream_t s);
int launch_up2_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd, const void *gy,
                   int dmode, const float *dparam, const void *aux, const void *add, void *gx, float *dpre,
                   float *dpost, hipStream_t s);

// 1x1x1 conv forward / backward-data (pw_conv.hip), both storage dtypes
// (dgrad with prologue-scalar partials on big grids: per-workgroup partials in `ws`,
// pw_dgrad_workspace(d) bytes, summed in order by a second kernel)
size_t pw_dgrad_workspace(const vq3d_conv_desc *d);
template <typename T>
int launch_pw1(const vq3d_conv_desc *d, bool dgrad, const void *in, const void *in2, const float *w, const float *pa,
               const float *pb, const FwdEpi<T> &fe, const BwdEpi<T> &be, const float *gscale, void *out,
               void *out2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t s);

// k > 1 forward / backward-data on small grids (<= 4096 voxels) with >= 32 reduction channels:
// reduction channels split over workgroups, partials [split][voxel][out] in the workspace
// (small_workspace bytes), summed in a fixed order by an epilogue kernel (conv_small.hip)
bool small_applicable(const vq3d_conv_desc *d, bool dgrad);
// the small-grid engine would run its matrix-core form (16-bit, 32-channel reduction chunks)
bool small_mma_form(const vq3d_conv_desc *d, bool dgrad);
size_t small_workspace(const vq3d_conv_desc *d, bool dgrad);
template <typename T>
int launch_small(const vq3d_conv_desc *d, bool dgrad, const void *in, const void *in2, const float *w,
                 const float *pa, const float *pb, const FwdEpi<T> &fe, const BwdEpi<T> &be, const float *gscale,
                 void *out, void *out2, float *dpre, float *dpost, void *ws, size_t ws_bytes, hipStream_t s);

// 3x3x3 stride-1 convs with 1 / 2 / 4 channels in and out on grids of 8 x 8 x 32 bricks
// (conv_tc.hip): VALU direct conv over a staged halo; weight gradient with per-workgroup
// partials (tc_workspace bytes per pass) and a fixed-order reduction
bool tc_applicable(const vq3d_conv_desc *d);
size_t tc_workspace(const vq3d_conv_desc *d, int pass);
template <typename T>
int launch_tc(const vq3d_conv_desc *d, bool dgrad, const void *in, const float *w, const float *pa, const float *pb,
              const FwdEpi<T> &fe, const BwdEpi<T> &be, const float *gscale, void *out, float *dpre, float *dpost,
              void *ws, size_t ws_bytes, hipStream_t s);
template <typename T>
int launch_tc_wgrad(const vq3d_conv_desc *d, const void *x, const void *g, const float *pa, const float *pb,
                    const float *w, const float *escale, float *dw, float *dscale, float *dbias, float *dcbias,
                    void *ws, size_t ws_bytes, hipStream_t s);

// few-channel blocks on the big grids (preact_col.hip), behind vq3d_preact_small_*
bool col_supported(int batch, int C, int BR, int h, int w, int d);
size_t col_workspace_bytes(int batch, int C, int BR, int h, int w, int d);
// xdt / odt: storage (VQ3D_HALF | VQ3D_F32) of the residual stream in (x, gx) and out (out, g)
// chain: vq3d_preact_small_fwd_chain's mode bits (0: an unchained launch, the rest unused)
int col_fwd(int xdt, int odt, int batch, int C, int BR, int h, int w, int d, const void *x, const float *w1,
            const float *w2, const float *w3, const vq3d_preact_params &p, void *out, void *t2, void *t3,
            hipStream_t s, int chain = 0, const void *t2in = nullptr, const float *w1n = nullptr,
            const vq3d_preact_params *pn = nullptr, void *t2n = nullptr);
int col_bwd(int xdt, int odt, int batch, int C, int BR, int h, int w, int d, const void *g, const void *x,
            const void *t2, const void *t3, const float *w1, const float *w2, const float *w3,
            const vq3d_preact_params &p, const vq3d_preact_grads &gr, void *workspace, void *gx, int stages,
            hipStream_t s);
bool mid_w2grad_ok(const vq3d_conv_desc *d);
size_t mid_w2grad_ws(const vq3d_conv_desc *d);
int mid_w2grad(const vq3d_conv_desc *d, const void *x, const void *g, float *dw, void *ws, size_t ws_bytes,
               hipStream_t s);
// few-channel k^3 weight gradients on the large grids (wgrad_ds.hip): D-shifted MFMA over whole
// D-lines for the instantiated (cin, cout, k, stride, pad, depth) shapes, optional prologue and
// sum-of-g (conv bias) gradient; per-workgroup partials in the workspace (wgrad_ds_ws bytes),
// fixed-order reduction
bool wgrad_ds_ok(const vq3d_conv_desc *d);
size_t wgrad_ds_ws(const vq3d_conv_desc *d);
int wgrad_ds(const vq3d_conv_desc *d, const void *x, const void *g, const float *pro_a, const float *pro_b, float *dw,
             float *dbias, void *ws, size_t ws_bytes, hipStream_t s);
int col_reduce_run(int nblocks, int batch, int C, int BR, int h, int w, int d, void *workspaces, size_t stride,
                   float *const *gtab, const float *const *ptab, hipStream_t s);

}  // namespace vq3d
