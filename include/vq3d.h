/*
 * vq3d.h — C-ABI of libvq3d.so, the MI355X (gfx950) kernels behind the 3D VQ-VAE-2
 * training step.  Plain pointers + sizes; no torch types.  The caller owns every
 * buffer (activations, gradients, workspaces); the library never allocates device
 * memory and never synchronises: every entry point enqueues work on `stream` and
 * returns.  Return value 0 = success, < 0 = error (message in vq3d_last_error(),
 * thread-local).  Entry points are stateless and re-entrant.
 *
 * The reference (sara-nl/3D-VQ-VAE-2) has no native code or FFI: its "operator API"
 * is nn.Module calls into ATen.  Each entry below replaces
 * the ATen work behind one reference call site, cited per function.
 *
 * Activation layout: channels-last NDHWC, i.e. the reference tensor (B, C, H, W, D)
 * stored as [B][H][W][D][C].  Storage dtype per call (VQ3D_F32, VQ3D_BF16 or VQ3D_F16);
 * arithmetic is fp32.  Weights are fp32 in the reference layout (Cout, Cin, k, k, k).
 * Wherever these comments say "bf16" for an activation or a matrix-core operand, a VQ3D_F16 call
 * uses IEEE fp16 instead (the reference's AMP precision, vqvae/train.py:32): the kernels exist in
 * both 16-bit formats and every entry point routes a call by its dtype arguments; one call's
 * 16-bit tensors share one format (mixing VQ3D_BF16 and VQ3D_F16 fails).
 */
#ifndef VQ3D_H
#define VQ3D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *vq3d_stream_t; /* == hipStream_t */

enum { VQ3D_F32 = 0, VQ3D_BF16 = 1, VQ3D_F16 = 2 };
enum { VQ3D_PAD_ZEROS = 0, VQ3D_PAD_CIRCULAR = 1 };
/* prologue applied to every input element as it is loaded (reference glue, layers.py:178-185) */
enum { VQ3D_PRO_NONE = 0, VQ3D_PRO_ADD = 1 /* x + a */, VQ3D_PRO_ELU_ADD = 2 /* elu(x + a) + b */ };

/* One 3-D convolution as nn.Conv3d computes it (padding_mode 'zeros' or 'circular';
 * circular == F.pad(x, p, 'circular') then a valid conv). */
typedef struct vq3d_conv_desc {
    int32_t dtype;      /* activation storage: VQ3D_F32 | VQ3D_BF16 | VQ3D_F16 */
    int32_t batch;
    int32_t cin;        /* channels of input 1 */
    int32_t cin2;       /* channels of input 2, concatenated after input 1 (torch.cat dim=1); 0 = none */
    int32_t cout;
    int32_t in_h, in_w, in_d;
    int32_t out_h, out_w, out_d;
    int32_t kernel, stride, pad, pad_mode;
    int32_t pro_kind;   /* VQ3D_PRO_* applied to the input on load */
    uint32_t tap_mask;  /* 0: dense kernel.  Else (kernel <= 3) bit (i0*k + i1)*k + i2 set for every
                           weight tap w[:, :, i0, i1, i2] that may be nonzero: the caller guarantees the
                           other taps are zero (e.g. a causal kernel embedded in a k^3 one), engines may
                           skip their products and leave their weight-gradient entries unwritten. */
} vq3d_conv_desc;

/* Forward epilogue: y = act( acc*scale + bias + cbias[co] + residual ) */
enum { VQ3D_ACT_NONE = 0, VQ3D_ACT_ELU = 1 /* elu(v) */, VQ3D_ACT_ELU_AFFINE = 2 /* elu(v + a) + b */ };
typedef struct vq3d_conv_epilogue {
    const float *scale;     /* device scalar or NULL (PreAct `scale`, layers.py:187) */
    const float *bias;      /* device scalar or NULL (`bias4`, `bias1d`, `bias2b`)  */
    const float *cbias;     /* device [cout] or NULL (nn.Conv3d bias)               */
    const void *residual;   /* NULL or activation tensor added before the activation */
    int32_t residual_up2;   /* 1: residual lives on the half-resolution grid and is
                               trilinearly upsampled x2 on the fly (ResizeConv skip)  */
    int32_t act;            /* VQ3D_ACT_*: ELU = FixupResBlock's post-activation
                               (layers.py:287-288); ELU_AFFINE = the NEXT PreAct conv's
                               "elu(x + a) + b" input glue fused here (layers.py:181-185) */
    const float *act_a, *act_b;  /* device scalars for VQ3D_ACT_ELU_AFFINE */
} vq3d_conv_epilogue;

/* Backward-data epilogue on the conv INPUT grid:
 *   v = acc;  pre += v;  v *= elu'(z);  post += v;  v += addend;  store
 * with elu'(z) from `aux`:
 *   aux_kind 0: aux = the conv input before its prologue elu(x + a) + b: z = aux + pro_a
 *   aux_kind 1: aux = an activated tensor t = elu(z) + b (b = *aux_b), as written by an
 *               ELU_AFFINE epilogue: elu'(z) = (t - b > 0) ? 1 : t - b + 1
 * pre / post are summed over every element (see vq3d_conv3d_bwd_data). */
typedef struct vq3d_dgrad_epilogue {
    const void *aux;        /* NULL: no derivative */
    int32_t aux_kind;
    const float *aux_b;
    const void *addend;     /* gradient added after the derivative, or NULL */
} vq3d_dgrad_epilogue;

/* --- 3-D convolution (replaces nn.Conv3d / F.pad circular, layers.py:124-171,535,377,490,508) ---
 * Every conv entry point takes a caller-owned scratch `workspace` of at least
 * vq3d_conv3d_workspace_size(d, pass) bytes (may be 0 -> NULL allowed): packed bf16 weight
 * fragments for the k^3 MFMA engine, per-workgroup partials for the weight gradient.  Its
 * contents are scratch; it must stay allocated until the launches on `stream` complete. */
enum { VQ3D_PASS_FWD = 0, VQ3D_PASS_BWD_DATA = 1, VQ3D_PASS_BWD_WEIGHT = 2 };
size_t vq3d_conv3d_workspace_size(const vq3d_conv_desc *d, int32_t pass);

int vq3d_conv3d_fwd(const vq3d_conv_desc *d, const void *x, const void *x2, const float *w,
                    const float *pro_a, const float *pro_b, const vq3d_conv_epilogue *epi,
                    void *y, void *workspace, size_t workspace_bytes, vq3d_stream_t stream);

/* Gradient w.r.t. the input(s).  g = dL/dy (y grid, cout channels); gscale: device scalar
 * multiplying g (the PreAct `scale`) or NULL.  gx (and gx2 for input 2) receive the result,
 * with the dgrad epilogue applied.  The prologue-scalar gradients are ACCUMULATED (fp32
 * atomics, one per workgroup) into dpro_pre (+= sum of v before the prologue derivative:
 * d/db of elu(x+a)+b, or d/da of x+a) and dpro_post (+= sum after it: d/da of elu(x+a)+b);
 * either may be NULL. */
int vq3d_conv3d_bwd_data(const vq3d_conv_desc *d, const void *g, const float *gscale, const float *w,
                         const float *pro_a, const vq3d_dgrad_epilogue *epi, void *gx, void *gx2,
                         float *dpro_pre, float *dpro_post, void *workspace, size_t workspace_bytes,
                         vq3d_stream_t stream);

/* Gradient w.r.t. the weight and the forward-epilogue parameters, ACCUMULATED (+=) into the
 * fp32 gradient buffers (any may be NULL):
 *   dw     += scale * G,  G[co,ci,t] = sum_v g[v,co] * prologue(x)[nbr(v,t),ci]
 *   dscale += sum(W * G)     (epilogue `scale`; needs w and epi_scale)
 *   dbias  += sum(g)         (epilogue scalar bias)
 *   dcbias += sum_v g[v,co]  (nn.Conv3d bias)
 * The workspace holds per-workgroup partials that a second kernel sums in a fixed order
 * (1x1x1 convs and the lines k^3 engine: deterministic); the direct k^3 engine used for
 * few-channel large grids accumulates with fp32 atomics, so its last bits are
 * order-dependent like cuDNN's wgrad. */
int vq3d_conv3d_bwd_weight(const vq3d_conv_desc *d, const void *x, const void *x2, const void *g,
                           const float *pro_a, const float *pro_b, const float *w, const float *epi_scale,
                           float *dw, float *dscale, float *dbias, float *dcbias, void *workspace,
                           size_t workspace_bytes, vq3d_stream_t stream);

/* --- trilinear x2 upsample, align_corners=False (nn.Upsample in ResizeConv3D, layers.py:591-597) --- */
int vq3d_upsample2x_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd,
                        const void *x, int32_t pro_kind, const float *pro_a, const float *pro_b, void *y,
                        vq3d_stream_t stream);
/* Adjoint of the upsample on the source grid, with the bwd_data epilogue (prologue
 * derivative w.r.t. aux, addend) and the same dpro_pre / dpro_post accumulation. */
int vq3d_upsample2x_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t h, int32_t w, int32_t dd,
                        const void *gy, int32_t pro_kind, const float *pro_a, const vq3d_dgrad_epilogue *epi,
                        void *gx, float *dpro_pre, float *dpro_post, vq3d_stream_t stream);

/* --- one whole PreActFixupResBlock, mode 'same', no skip conv (layers.py:102-216), on a tiny
 * grid with all operands in LDS: the 100 top-level blocks of the published model run on 8x8x2 voxels,
 * where per-conv launches are pure fixed cost (forward: one launch; backward: two).  Limits: batch*h*w*d <= 256, channels <= 32,
 * branch <= 16, both multiples of 4 (vq3d_preact_tiny_supported).  Weights are the fp32
 * nn.Conv3d tensors: w1 [branch][channels], w2 [branch][branch][3][3][3], w3 [channels][branch].
 *   out = scale * W3 t3 + bias4 + x,  t3 = elu(W2 (*) t2 + bias3a) + bias3b (3x3x3 circular),
 *   t2 = elu(W1 (elu(x + bias1a) + bias1b) + bias2a) + bias2b
 * The forward saves t2 / t3 (fp32) for the backward, which writes gx and accumulates (+=)
 * every parameter gradient (NULL pointers skipped). */
typedef struct vq3d_preact_params {
    const float *bias1a, *bias1b, *bias2a, *bias2b, *bias3a, *bias3b, *scale, *bias4;
} vq3d_preact_params;
typedef struct vq3d_preact_grads {
    float *dw1, *dw2, *dw3;
    float *dbias1a, *dbias1b, *dbias2a, *dbias2b, *dbias3a, *dbias3b, *dscale, *dbias4;
} vq3d_preact_grads;
int vq3d_preact_tiny_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd);
/* fp32 sizes of the forward's saved intermediates (t2, t3) and of the backward workspace */
size_t vq3d_preact_tiny_saved_floats(int32_t batch, int32_t branch, int32_t h, int32_t w, int32_t dd);
size_t vq3d_preact_tiny_workspace_floats(int32_t batch, int32_t branch, int32_t h, int32_t w, int32_t dd);
int vq3d_preact_tiny_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                         int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                         const vq3d_preact_params *p, void *out, float *saved, vq3d_stream_t stream);
int vq3d_preact_tiny_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                         int32_t dd, const void *x, const void *g, const float *w1, const float *w2,
                         const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                         const float *saved, float *workspace, void *gx, vq3d_stream_t stream);

/* One whole PreActFixupResBlock (mode 'same', no skip conv) on the 18-channel / branch-9 level
 * (bf16, h % 8 == w % 8 == 0, d % 8 == 0, batch*h*w*d % 256 == 0; the 50 decoder
 * post-quantize blocks of the published model at 128x128x32).  Replaces the per-conv calls of
 * layers.py:176-195 and their autograd backward for these blocks.
 * Forward (two launches): writes out and the intermediates t2 = elu(W1 u1 + bias2a) + bias2b and
 * t3 = elu(W2 (*) t2 + bias3a) + bias3b ([B][H][W][D][branch] bf16).
 * Backward (four launches): writes gx and accumulates (+=) every parameter gradient of *gr (all
 * required), deterministically (fixed-order workgroup partials), through a caller-owned
 * workspace of vq3d_preact_mid_workspace_bytes. */
int vq3d_preact_mid_supported(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd);
int vq3d_preact_mid_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                        int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                        const vq3d_preact_params *p, void *out, void *t2, void *t3, vq3d_stream_t stream);
size_t vq3d_preact_mid_workspace_bytes(int32_t batch, int32_t h, int32_t w, int32_t dd);
int vq3d_preact_mid_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                        int32_t dd, const void *g, const void *x, const void *t2, const void *t3, const float *w1,
                        const float *w2, const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                        void *workspace, size_t workspace_bytes, void *gx, vq3d_stream_t stream);
/* Staged entries: the same calls, launching only the kernels selected by `stages` (forward: bit 0
 * t2, bit 1 tile kernel; backward: bit 0 pointwise gz3 kernel, bit 1 data tile kernel (gx), bit 2
 * W2-gradient kernel, bit 3 W1 / W3-gradient kernel, bit 4 reduction).  Backward stages 4 | 8 | 16 read only g / x / t2 / t3 and
 * the workspace that stages 1 | 2 wrote, so a caller may issue them on a second stream ordered
 * after the first (the product's concurrent weight-gradient mode does); bench.py's roofline
 * probe and tools/block_micro.py time single stages. */
int vq3d_preact_mid_fwd_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                               int32_t h, int32_t w, int32_t dd, const void *x, const float *w1, const float *w2,
                               const float *w3, const vq3d_preact_params *p, void *out, void *t2, void *t3,
                               vq3d_stream_t stream);
int vq3d_preact_mid_bwd_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                               int32_t h, int32_t w, int32_t dd, const void *g, const void *x, const void *t2,
                               const void *t3, const float *w1, const float *w2, const float *w3,
                               const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *workspace,
                               size_t workspace_bytes, void *gx, vq3d_stream_t stream);
/* Chained entries for a RUN of these blocks (block i's out is block i+1's x), each fusing the
 * neighbouring block's pointwise stage into its tile kernel's epilogue, while the tile is in LDS:
 *  - fwd_chain: the tile kernel only (t2 is an INPUT: stage 1 of the first block, or the previous
 *    block's chained forward); with next_w1 != NULL it also writes the next block's t2 (next_w1,
 *    next_p: that block's W1 and scalars) -- stage 1's rounding points (u1 and W1 as bf16
 *    operands), summed on the matrix cores.
 *  - bwd_chain: vq3d_preact_mid_bwd_stages; with prev_t3 != NULL the data stage (2, required) also
 *    computes the PREVIOUS block's stage 1 (its gz3 and scalar partials, from this block's gx = its
 *    g, prev_t3 / prev_w3 / prev_p) into prev_workspace, whose own call then omits stage 1. */
int vq3d_preact_mid_fwd_chain(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd, const void *x, const float *w2, const float *w3,
                              const vq3d_preact_params *p, const void *t2, void *out, void *t3,
                              const float *next_w1, const vq3d_preact_params *next_p, void *next_t2,
                              vq3d_stream_t stream);
int vq3d_preact_mid_bwd_chain(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                              int32_t h, int32_t w, int32_t dd, const void *g, const void *x, const void *t2,
                              const void *t3, const float *w1, const float *w2, const float *w3,
                              const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *workspace,
                              size_t workspace_bytes, void *gx, const void *prev_t3, const float *prev_w3,
                              const vq3d_preact_params *prev_p, void *prev_workspace, size_t prev_workspace_bytes,
                              vq3d_stream_t stream);
/* Stage 16 (the fixed-order reduction) of a whole run in ONE launch: block i's workspace at
 * workspaces + i * workspace_stride (stride >= vq3d_preact_mid_workspace_bytes, a multiple of 256),
 * grads / params: device arrays [nblocks][11] of device pointers in the order of
 * vq3d_preact_stack_fwd's table (w1, w2, w3, bias1a, bias1b, bias2a, bias2b, bias3a, bias3b, scale,
 * bias4) -- gradient buffers (+=) and parameters (scale is read).  Same sums as per-block stage 16. */
int vq3d_preact_mid_reduce_run(int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                               const void *workspaces, size_t workspace_stride, float *const *grads,
                               const float *const *params, vq3d_stream_t stream);
/* Stages 4 and 8 (the W2 and W1 / G3 weight-gradient partial rows) of a whole run in one launch
 * each, after the run's data stages (bwd_chain with stages 2 | first): block i's gz3 / gz1 and
 * partial rows in its workspace slice (workspaces + i * workspace_stride, as for reduce_run), its
 * saved t2 / t3, its input x and its incoming gradient g given as HOST arrays [nblocks] of device
 * pointers, params the run's device table [nblocks][11] (bias1a / bias1b are read).  The partial
 * rows are bit-identical to per-block stages 4 | 8; vq3d_preact_mid_reduce_run then sums them.
 * dtype: the activations' 16-bit format (VQ3D_HALF with the build's format, as for the stages).
 * (Replaces the per-block reference call sites vqvae/layers.py:176-195's weight gradients, which
 * autograd runs interleaved with the data chain.) */
int vq3d_preact_mid_wgrad_run(int32_t dtype, int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                              const void *const *t2, const void *const *t3, const void *const *x,
                              const void *const *g, const float *const *params, void *workspaces,
                              size_t workspace_stride, vq3d_stream_t stream);

/* A RUN of nblocks identical PreActFixupResBlocks (mode 'same', no skip conv) on a tiny grid
 * (batch*h*w*d <= 256, channels <= 32, branch <= 16, both multiples of 4): forward in ONE launch,
 * backward in ONE launch, one workgroup walking the blocks with the residual stream in LDS (fp32).
 * Replaces, for the published model's 50 + 50 top-level blocks (8x8x2, 32 channels), the
 * per-block calls of layers.py:176-195 and their autograd backward.  bf16 with (32, 16) runs on the
 * matrix cores, everything else on fp32 VALU.
 * params: device array [nblocks][11] of device pointers, per block {w1, w2, w3, bias1a, bias1b,
 * bias2a, bias2b, bias3a, bias3b, scale, bias4}; grads: the same layout for the fp32 gradient
 * buffers, all accumulated (+=), deterministically.  saved: vq3d_preact_stack_saved_floats fp32
 * written by the forward (each block's input, t2, t3) and read by the backward. */
int vq3d_preact_stack_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd);
size_t vq3d_preact_stack_saved_floats(int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                                      int32_t w, int32_t dd);
int vq3d_preact_stack_fwd(int32_t dtype, int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                          int32_t w, int32_t dd, const void *x, const float *const *params, void *out, float *saved,
                          vq3d_stream_t stream);
int vq3d_preact_stack_bwd(int32_t dtype, int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                          int32_t w, int32_t dd, const void *g, const float *const *params, float *const *grads,
                          const float *saved, void *gx, vq3d_stream_t stream);
/* vq3d_preact_stack_bwd with the weight gradients taken off the block chain: the one-workgroup
 * chain carries only the gradient stream (and the scalar sums riding it) and records each block's
 * bf16 matrix operands in `workspace`; then one workgroup per block computes the W1 / W2 / W3 and
 * scale gradients in parallel.  Results equal vq3d_preact_stack_bwd's bit for bit.  Shapes or
 * dtypes without a split plan (workspace_bytes 0) run the fused kernel. */
size_t vq3d_preact_stack_bwd_workspace_bytes(int32_t nblocks, int32_t batch, int32_t channels, int32_t branch,
                                             int32_t h, int32_t w, int32_t dd);
int vq3d_preact_stack_bwd_ws(int32_t dtype, int32_t nblocks, int32_t batch, int32_t channels, int32_t branch,
                             int32_t h, int32_t w, int32_t dd, const void *g, const float *const *params,
                             float *const *grads, const float *saved, void *gx, void *workspace, size_t ws_bytes,
                             vq3d_stream_t stream);

/* The 72-channel / branch-36 PreActFixupResBlock (mode 'same', no skip conv) of the published
 * model's decoder level 1 (50 blocks at 32x32x8, layers.py:176-195, Decoder.up layers.py:395-405):
 * h % 2 == 0, w % 4 == 0, dd % 8 == 0, batch*h*w*dd % 512 == 0.  The residual stream (x, out, g,
 * gx) is fp32 [B][H][W][D][72]; t2 / t3 are saved bf16 [B][H][W][D][36]; weights are read from a
 * packed bf16 fragment image (vq3d_preact_wide_pack, per RUN of blocks, params as for
 * vq3d_preact_stack_fwd; each block's image is vq3d_preact_wide_image_bytes long).
 * Forward: one launch.  Backward: bwd_data (one launch: gx, plus gz3 / gz1 / scalar partials in
 * the workspace) then bwd_weight (two launches reading the workspace: every parameter gradient,
 * accumulated (+=) deterministically); bwd_weight may run on another stream after bwd_data. */
int vq3d_preact_wide_supported(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd);
size_t vq3d_preact_wide_image_bytes(int32_t channels, int32_t branch);
/* dtype (VQ3D_BF16 | VQ3D_F16): the format of the fragment image and of t2 / t3 */
int vq3d_preact_wide_pack(int32_t dtype, int32_t nblocks, int32_t channels, int32_t branch, const float *const *params,
                          void *image, vq3d_stream_t stream);
int vq3d_preact_wide_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd,
                         const float *x, const void *image, const vq3d_preact_params *p, float *out, void *t2,
                         void *t3, vq3d_stream_t stream);
size_t vq3d_preact_wide_workspace_bytes(int32_t batch, int32_t h, int32_t w, int32_t dd);
int vq3d_preact_wide_bwd_data(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                              int32_t dd,
                              const float *g, const float *x, const void *t2, const void *t3, const void *image,
                              const vq3d_preact_params *p, void *workspace, size_t workspace_bytes, float *gx,
                              vq3d_stream_t stream);
int vq3d_preact_wide_bwd_weight(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                                int32_t dd,
                                const float *g, const float *x, const void *t2, const void *t3,
                                const vq3d_preact_params *p, const vq3d_preact_grads *gr, const void *workspace,
                                size_t workspace_bytes, vq3d_stream_t stream);
/* bwd_weight in stages: 1 = the weight-gradient partial kernel, 2 = the fixed-order reduction;
 * reduce_run = stage 2 of a whole RUN in one launch (block i's workspace at workspaces + i *
 * workspace_stride, stride >= vq3d_preact_wide_workspace_bytes and a multiple of 256; grads /
 * params as for vq3d_preact_mid_reduce_run). */
int vq3d_preact_wide_bwd_weight_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                                       int32_t h,
                                       int32_t w, int32_t dd, const float *g, const float *x, const void *t2,
                                       const void *t3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                                       const void *workspace, size_t workspace_bytes, vq3d_stream_t stream);
/* The weight-gradient stage (1 of vq3d_preact_wide_bwd_weight_stages) of a whole run in one
 * launch, after the run's data kernels: block i's gz3 / gz1 and partial rows in its workspace slice
 * (workspaces + i * workspace_stride, as for vq3d_preact_wide_reduce_run), its incoming gradient g
 * and input x (fp32) and its saved t2 / t3 as HOST arrays [nblocks] of device pointers, params the
 * run's device table [nblocks][11].  Partial rows bit-identical to the per-block stage. */
int vq3d_preact_wide_wgrad_run(int32_t dtype, int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                               const float *const *g, const float *const *x, const void *const *t2,
                               const void *const *t3, const float *const *params, void *workspaces,
                               size_t workspace_stride, vq3d_stream_t stream);
int vq3d_preact_wide_reduce_run(int32_t nblocks, int32_t batch, int32_t h, int32_t w, int32_t dd,
                                const void *workspaces, size_t workspace_stride, float *const *grads,
                                const float *const *params, vq3d_stream_t stream);

/* Whole PreActFixupResBlock (mode 'same', no skip conv) on few channels: (channels, branch) in
 * {(2, 1), (4, 2), (8, 4)}, bf16, power-of-two grid.  Forward in one launch writes out, t2 and t3
 * ([B][H][W][D][branch] bf16, as the unfused convs' epilogues write them); backward in two
 * launches writes gx and accumulates (+=) every parameter gradient of *gr (NULL skipped),
 * deterministically, through a caller-owned workspace of vq3d_preact_small_workspace_bytes.
 * Replaces, for these blocks, the per-conv calls of layers.py:176-195 (fwd) and their autograd
 * backward. */
int vq3d_preact_small_supported(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                                int32_t dd);
/* 0: unsupported; 1: brick kernels (small grids); 2: column kernels (H % 8 == W % 8 == 0,
 * D % 16 == 0: one-launch forward, fused backward + fixed-order reduction, preact_col.hip) */
int vq3d_preact_small_plan(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd);
size_t vq3d_preact_small_workspace_bytes(int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                                         int32_t dd);
int vq3d_preact_small_fwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                          int32_t dd, const void *x, const float *w1, const float *w2, const float *w3,
                          const vq3d_preact_params *p, void *out, void *t2, void *t3, vq3d_stream_t stream);
int vq3d_preact_small_bwd(int32_t dtype, int32_t batch, int32_t channels, int32_t branch, int32_t h, int32_t w,
                          int32_t dd, const void *g, const void *x, const void *t2, const void *t3, const float *w1,
                          const float *w2, const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                          void *workspace, size_t ws_bytes, void *gx, vq3d_stream_t stream);
/* the same in stages: 1 = the fused data / partial-sum kernel (gx, per-brick partial rows in the
 * workspace), 2 = the fixed-order reduction of the partial rows into the gradient buffers.  Stage 2
 * only reads the workspace, so a caller may issue it on a second stream (after stage 1). */
int vq3d_preact_small_bwd_stages(int32_t stages, int32_t dtype, int32_t batch, int32_t channels, int32_t branch,
                                 int32_t h, int32_t w, int32_t dd, const void *g, const void *x, const void *t2,
                                 const void *t3, const float *w1, const float *w2, const float *w3,
                                 const vq3d_preact_params *p, const vq3d_preact_grads *gr, void *workspace,
                                 size_t ws_bytes, void *gx, vq3d_stream_t stream);
/* The same blocks with the residual stream stored per tensor: x (and gx) as x_dtype, out (and g) as
 * out_dtype, each dtype (the 16-bit format, VQ3D_BF16 | VQ3D_F16, of t2 / t3 and of every conv
 * operand) or VQ3D_F32.  A run of blocks carries its stream in fp32 between blocks (16-bit -> fp32,
 * fp32 -> fp32, ..., fp32 -> 16-bit), as the reference's autocast blocks return fp32
 * (`out * self.scale` with fp32 parameters, layers.py:187-193); the plain entries above are
 * (dtype, dtype). */
int vq3d_preact_small_fwd_io(int32_t dtype, int32_t x_dtype, int32_t out_dtype, int32_t batch, int32_t channels, int32_t branch,
                             int32_t h, int32_t w, int32_t dd, const void *x, const float *w1, const float *w2,
                             const float *w3, const vq3d_preact_params *p, void *out, void *t2, void *t3,
                             vq3d_stream_t stream);
int vq3d_preact_small_bwd_stages_io(int32_t stages, int32_t dtype, int32_t x_dtype, int32_t out_dtype, int32_t batch,
                                    int32_t channels, int32_t branch, int32_t h, int32_t w, int32_t dd, const void *g,
                                    const void *x, const void *t2, const void *t3, const float *w1, const float *w2,
                                    const float *w3, const vq3d_preact_params *p, const vq3d_preact_grads *gr,
                                    void *workspace, size_t ws_bytes, void *gx, vq3d_stream_t stream);
/* Chained RUNS of the column-kernel blocks (vq3d_preact_small_plan == 2): links between consecutive
 * blocks that skip the halo recompute (each block's t2 is formed once per voxel, in the previous
 * block's epilogue, instead of on every brick's halo).  Forward, mode bit 0: this
 * block's t2 was written by the previous block's launch (t2_in; the t2 argument is then not
 * written); bit 1: the launch also writes the NEXT block's t2 (t2_next) from this block's out as
 * stored, with that block's W1 (w1_next) and params_next.  Bit-identical to unchained launches. */
int vq3d_preact_small_fwd_chain(int32_t mode, int32_t dtype, int32_t x_dtype, int32_t out_dtype, int32_t batch, int32_t channels,
                                int32_t branch, int32_t h, int32_t w, int32_t dd, const void *x, const void *t2_in,
                                const float *w1, const float *w2, const float *w3, const vq3d_preact_params *p,
                                void *out, void *t2, void *t3, const float *w1_next,
                                const vq3d_preact_params *params_next, void *t2_next, vq3d_stream_t stream);
/* Stage 2 of a whole RUN of these blocks in one launch pair: block i's workspace at
 * workspaces + i * workspace_stride (stride >= vq3d_preact_small_workspace_bytes, a multiple of
 * 256), grads / params as for vq3d_preact_mid_reduce_run ([nblocks][11] device pointer tables). */
int vq3d_preact_small_reduce_run(int32_t nblocks, int32_t batch, int32_t channels, int32_t branch, int32_t h,
                                 int32_t w, int32_t dd, const void *workspaces, size_t workspace_stride,
                                 float *const *grads, const float *const *params, vq3d_stream_t stream);

/* --- codebook (Quantizer.forward / _update_ema / _init_ema, layers.py:636-728) --- */
/* Nearest codeword with torch-CPU cdist arithmetic (bit-exact),
 * q = E[idx], zst = fl(x + fl(q - x)) stored as zst_dtype, and the squared-error sum
 * for the commitment loss (layers.py:716) reduced into *sqerr_out (fp32 scalar).
 * z: n rows of d fp32-or-bf16 values (z_dtype), row order (b, h, w, d) = channels-last. */
size_t vq3d_vq_workspace_size(int64_t n, int32_t d, int32_t k);
int vq3d_vq_nearest(int32_t z_dtype, const void *z, int64_t n, int32_t d, const float *embed, int32_t k,
                    int64_t *idx, int32_t zst_dtype, void *zst, float *sqerr_out, void *workspace,
                    vq3d_stream_t stream);
/* loss = coef * (*sqerr) ; writes a device scalar (coef = commitment_cost / numel) */
int vq3d_vq_commit_loss(const float *sqerr, float coef, float *loss, vq3d_stream_t stream);
/* gz = g_zst + (*g_loss) * coef * (x - q)    (coef = 2 * commitment_cost / numel) */
int vq3d_vq_bwd(int32_t z_dtype, const void *z, int64_t n, int32_t d, const float *embed, const int64_t *idx,
                int32_t g_dtype, const void *g_zst, const float *g_loss, float coef, void *gz,
                vq3d_stream_t stream);
/* counts[k] = #rows with idx == k ; dw[k, :] = sum of those rows   (deterministic) */
int vq3d_vq_ema_stats(int32_t z_dtype, const void *z, int64_t n, int32_t d, const int64_t *idx, int32_t k,
                      float *counts, float *dw, void *workspace, vq3d_stream_t stream);
/* cluster_size = cs*decay + counts*(1-decay); embed_avg likewise with dw; Laplace smoothing;
 * embed = embed_avg / smoothed  (layers.py:649-663). counts/dw already world-summed. */
int vq3d_vq_ema_update(float *embed, float *embed_avg, float *cluster_size, const float *counts,
                       const float *dw, int32_t k, int32_t d, float decay, float laplace_alpha,
                       vq3d_stream_t stream);
/* mean[d] and unbiased std[d] over the n rows (layers.py:666-667) */
int vq3d_vq_moments(int32_t z_dtype, const void *z, int64_t n, int32_t d, float *mean, float *std,
                    void *workspace, vq3d_stream_t stream);
/* embed = embed*(std/world) + mean/world ; embed_avg = embed ; cluster_size += n_total/k ;
 * *first_pass = 0   (layers.py:670-683; mean/std already world-summed) */
int vq3d_vq_init_apply(float *embed, float *embed_avg, float *cluster_size, int64_t *first_pass,
                       const float *mean, const float *std, int32_t k, int32_t d, float inv_world,
                       float n_total, vq3d_stream_t stream);

/* --- Encoder2.parse_input (layers.py:535): Conv3d(1 -> channels, k = 1, bias) on the fp32 input
 * volume [voxels] with a 16-bit output [voxels][channels] (dtype VQ3D_BF16 | VQ3D_F16; channels in {2, 4,
 * 8}, voxels % 4 == 0).
 * The volume stays fp32 (the reference's autocast rounds it to fp16, never to bf16).  The backward
 * accumulates (+=) the weight [channels] and bias [channels] gradients, deterministically (fixed-
 * order partial sums through a workspace of vq3d_parse_input_workspace_bytes); the input has no
 * gradient. --- */
int vq3d_parse_input_fwd(int32_t dtype, int64_t voxels, int32_t channels, const float *x, const float *w,
                         const float *b, void *y, vq3d_stream_t stream);
size_t vq3d_parse_input_workspace_bytes(int64_t voxels, int32_t channels);
int vq3d_parse_input_bwd(int32_t dtype, int64_t voxels, int32_t channels, const float *x, const void *g, float *dw,
                         float *db, void *workspace, size_t ws_bytes, vq3d_stream_t stream);

/* --- reconstruction loss (VQVAE.loc_metric with F.smooth_l1_loss, model.py:115-163) ---
 * loc = elu(dec); loc[..., s >= nvs[b]] = 0; optional centre-cylinder gather
 * (ExtractCenterCylinder, load_nrrd_dataset.py:258-300); smooth-L1 (beta 1) mean. */
size_t vq3d_recon_loss_workspace_size(int32_t batch, int32_t h, int32_t w, int32_t dd);
/* total = recon + sum_i *commit[i]  (commit: host array of n_commit <= 8 device scalars) */
int vq3d_recon_loss_fwd(int32_t dtype, const void *dec, const float *x, const int64_t *nvs, int32_t batch,
                        int32_t h, int32_t w, int32_t dd, int32_t cylinder, const float *const *commit,
                        int32_t n_commit, float *recon, float *total, void *workspace, vq3d_stream_t stream);
int vq3d_recon_loss_bwd(int32_t dtype, const void *dec, const float *x, const int64_t *nvs, int32_t batch,
                        int32_t h, int32_t w, int32_t dd, int32_t cylinder, const float *g_total,
                        void *gdec, vq3d_stream_t stream);
/* number of (h, w) pixels inside the cylinder (host function) */
int64_t vq3d_cylinder_count(int32_t h, int32_t w);

/* --- EvoNorm-S0 (evonorm.py:8-76), batch 1 --- */
size_t vq3d_evonorm_workspace_size(int32_t channels, int64_t voxels);
int vq3d_evonorm_fwd(int32_t dtype, const void *x, int32_t channels, int64_t voxels, const float *v,
                     const float *gamma, const float *beta, void *y, float *stats, void *workspace,
                     vq3d_stream_t stream);
int vq3d_evonorm_bwd(int32_t dtype, const void *x, const void *gy, int32_t channels, int64_t voxels,
                     const float *v, const float *gamma, const float *stats, void *gx, float *dv,
                     float *dgamma, float *dbeta, void *workspace, vq3d_stream_t stream);

/* --- optimizer: torch.optim.Adam(amsgrad=True) over one flat fp32 buffer (model.py:91-93) --- */
int vq3d_adam_amsgrad(float *p, const float *g, float *m, float *v, float *vmax, int64_t n, float lr,
                      float beta1, float beta2, float eps, int64_t step, vq3d_stream_t stream);
/* Same update with the step count on the device: uses *step + 1 for the bias corrections, then
 * increments *step -- no host value baked into the launch, so a captured HIP graph of the
 * training step replays correctly.  skip (NULL: never): a device flag; when *skip != 0 (the loss
 * scaler found a non-finite gradient) neither the parameters nor *step change (GradScaler.step). */
int vq3d_adam_amsgrad_dev(float *p, const float *g, float *m, float *v, float *vmax, int64_t n, float lr,
                          float beta1, float beta2, float eps, int64_t *step, const float *skip,
                          vq3d_stream_t stream);
/* --- dynamic loss scaling: torch.cuda.amp.GradScaler's device work for the fp16 path (the
 * reference's PL native AMP, vqvae/train.py:32).  grad_unscale: g *= 1 / *scale over the flat
 * gradient, *found_inf = 1 when any value was inf / NaN (else 0).  loss_scale_update: on a flagged
 * step *scale *= backoff and *growth_tracker = 0, else after `interval` clean steps in a row
 * *scale *= growth (if finite).  All state on the device (graph-capturable). --- */
int vq3d_grad_unscale(float *g, int64_t n, const float *scale, float *found_inf, vq3d_stream_t stream);
int vq3d_loss_scale_update(float *scale, int32_t *growth_tracker, const float *found_inf, float growth,
                           float backoff, int32_t interval, vq3d_stream_t stream);

/* --- utilities --- */
int vq3d_cast(int32_t src_dtype, const void *src, int32_t dst_dtype, void *dst, int64_t n,
              vq3d_stream_t stream);
int vq3d_zero(void *p, size_t bytes, vq3d_stream_t stream);
int vq3d_copy(void *dst, const void *src, size_t bytes, vq3d_stream_t stream);
/* Test support: fill the LDS of every CU with all-ones words (bf16 / fp32 NaN) so a kernel that
 * reads LDS it never wrote -- even only to multiply it by a zero weight -- shows up as NaN in its
 * output instead of depending on what the previous kernel left behind. */
int vq3d_poison_lds(vq3d_stream_t stream);
/* gz = g * elu'(z) recovered from the OUTPUT y = elu(z): 1 if y > 0 else y + 1 (FixupResBlock's
 * post-activation, layers.py:287-288); n elements of dtype */
int vq3d_elu_bwd_from_output(int32_t dtype, const void *g, const void *y, void *gz, int64_t n,
                             vq3d_stream_t stream);
/* x *= a over n fp32 values (gradient averaging after the all-reduce uses a = 1/world) */
int vq3d_scale(float *x, float a, int64_t n, vq3d_stream_t stream);

/* --- PixelSNAIL block glue (pixel_model/layers.py:425-465), the elementwise steps around the
 * 1x1 causal convs, each one launch with its scalar-parameter gradient sums (fixed order) ---
 * pre-activation of a conv input: y = elu(x + *a) + *b (x: x_dtype, y: y_dtype, n elements); its
 * backward gx = g * elu'(x + a) (gx: x_dtype, may be NULL), *da += sum gx, *db += sum g */
int vq3d_preact_act_fwd(int32_t x_dtype, int32_t y_dtype, int64_t n, const void *x, const float *a, const float *b,
                        void *y, vq3d_stream_t stream);
int vq3d_preact_act_bwd(int32_t g_dtype, int32_t x_dtype, int64_t n, const void *g, const void *x, const float *a,
                        void *gx, float *da, float *db, vq3d_stream_t stream);
/* the block's output out = o * *scale + *bias + s (o: o_dtype, s / out fp32); its backward
 * go = g * scale (o_dtype), *dscale += sum g * o, *dbias += sum g (the skip's gradient is g) */
int vq3d_scale_bias_res_fwd(int32_t o_dtype, int64_t n, const void *o, const float *scale, const float *bias,
                            const float *s, float *out, vq3d_stream_t stream);
int vq3d_scale_bias_res_bwd(int32_t o_dtype, int64_t n, const float *g, const void *o, const float *scale, void *go,
                            float *dscale, float *dbias, vq3d_stream_t stream);
/* the 1x1x1 convs' forward and backward-data over voxel rows (Conv3d(kernel_size=1) of
 * pixel_model/layers.py:225-248 / 370-404 / 665-675 and pixelsnail.py:39-43 / 78-82 on
 * channels-last activations; replaces the GEMM those convs run as torch F.linear / matmul):
 * y[v][j] = sum_i x[v][i] w'[j][i] (+ bias[j], fp32, may be NULL) for v < nrows, j < n, i < k, with
 * w' = w (trans_w = 0: w[n][k] rows at stride ldw -- the forward, w = [cout][cin]) or w' = w^T
 * (trans_w = 1: w[k][n] -- the backward-data gx = g W).  x, w, y 16-bit (dtype BF16 / F16), fp32
 * accumulation on the matrix cores, y rounded once; k, n, ldx, ldw multiples of 8, ldy of 4, k <= 1024,
 * x / w 16-byte and y 8-byte aligned. */
int vq3d_rows_gemm(int32_t dtype, int64_t nrows, int32_t k, int32_t n, const void *x, int64_t ldx, const void *w,
                   int64_t ldw, int32_t trans_w, const float *bias, void *y, int64_t ldy, vq3d_stream_t stream);
/* the 1x1x1 convs' weight gradient over voxel rows (the Conv3d(kernel_size=1) backward of
 * layers.py:122-248 / 650-703, the GEMMs' K = voxels side): dw[cg][cx] += sum_v g[v][co] x[v][ci]
 * and (db != NULL) db[co] += sum_v g[v][co], fp32 accumulation in a fixed order.  g: nrows rows of
 * cg channels at row stride ldg, x: rows of cx channels at stride ldx, both 16-bit (dtype BF16 / F16),
 * 16-byte aligned, channel counts and strides multiples of 8; workspace of
 * vq3d_rows_wgrad_workspace_bytes bytes. */
size_t vq3d_rows_wgrad_workspace_bytes(int64_t nrows, int32_t cg, int32_t cx);
int vq3d_rows_wgrad(int32_t dtype, int64_t nrows, int32_t cg, int32_t cx, const void *g, int64_t ldg, const void *x,
                    int64_t ldx, float *dw, float *db, void *workspace, size_t ws_bytes, vq3d_stream_t stream);

/* --- PixelSNAIL prior: dense causal attention (pixel_model/layers.py:613-647) ---
 * For each of nprob problems (stack x batch) and nh heads: out[i] = sum_{j <= i} softmax_j(scale *
 * q_i . k_j) v_j over n positions, without the n x n logits.  q, k: [nprob][n][nh * dk], v, out:
 * [nprob][n][nh * dv] (rows channels-last, head h owns channels h*d .. h*d + d - 1), dtype bf16 or
 * fp32, fp32 arithmetic; head dims up to 16.  The forward saves lse [nprob][nh][n] (fp32, base-2
 * log-sum-exp of the scaled scores); the backward recomputes the probabilities from it and writes
 * gq, gk, gv (same layouts as q, k, v) through a workspace of vq3d_causal_attn_workspace_bytes.
 * The reference's CausalAttentionPixelBlock binds its projected queries to the parameter named
 * `keys` and vice versa (layers.py:694 vs 619); callers pass q = that block's keys projection. */
/* Training mode (CausalAttention with its nn.Dropout in training, layers.py:633-637): the logits go
 * through dropout (each dropped with probability dropout_p, the kept ones scaled by 1 / (1 - p)) and
 * then every logit equal to 0 -- the dropped ones and any exact zero -- is replaced by -1e3 before
 * the causal mask and the softmax; the replaced logits pass no gradient.  The drop decision is a
 * counter-based hash of (*seed, problem * nh + head, i, j), recomputed by the backward, so one
 * seed value must serve a forward and its backward (the caller keeps it on the device and
 * advances it between forwards: HIP-graph replays draw fresh masks).  train == NULL: eval mode
 * (the plain entries). */
typedef struct vq3d_attn_train {
    double dropout_p;       /* in [0, 1); 0 keeps every logit (the zero replacement still applies) */
    const uint64_t *seed;   /* device scalar, required when dropout_p > 0 */
} vq3d_attn_train;
int vq3d_causal_attn_supported(int32_t nh, int32_t dk, int32_t dv);
size_t vq3d_causal_attn_workspace_bytes(int32_t nprob, int32_t n, int32_t nh);
int vq3d_causal_attn_fwd(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                         const void *q, const void *k, const void *v, void *out, float *lse, vq3d_stream_t stream);
int vq3d_causal_attn_bwd(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                         const void *q, const void *k, const void *v, const void *out, const void *gout,
                         const float *lse, void *workspace, size_t workspace_bytes, void *gq, void *gk, void *gv,
                         vq3d_stream_t stream);

int vq3d_causal_attn_fwd_ex(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                            const void *q, const void *k, const void *v, const vq3d_attn_train *train, void *out,
                            float *lse, vq3d_stream_t stream);
int vq3d_causal_attn_bwd_ex(int32_t dtype, int32_t nprob, int32_t n, int32_t nh, int32_t dk, int32_t dv, float scale,
                            const void *q, const void *k, const void *v, const vq3d_attn_train *train,
                            const void *out, const void *gout, const float *lse, void *workspace,
                            size_t workspace_bytes, void *gq, void *gk, void *gv, vq3d_stream_t stream);

const char *vq3d_last_error(void);
const char *vq3d_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VQ3D_H */
