"""autograd Functions of the VQ-VAE-2 hot path, each a fixed sequence of libvq3d kernels.

Parameter gradients are written by the kernels straight into `param.grad` (fp32, one flat
buffer per model, see flat.py) with += semantics, and the Functions return None for those
inputs: no torch accumulate kernels, no extra allocations.  Every tensor in and out is a
GPU tensor; the activations are channels-last (ops.py).
"""
import ctypes

import torch

from . import _lib as L
from . import ops
from .ops import ConvGeom
from . import flat as _flat
from .parallel import grads_ready, sum_allreduce

CL = torch.channels_last_3d


_BINDING = ["ctypes"]


def set_binding(name):
    """How the model's layers reach the kernels: "ctypes" (default) -- the autograd Functions below
    call the C-ABI; "library" -- through the registered `torch.ops.vq3d.*` operators (vq3d.library),
    which run the same Function bodies, so the two give bit-identical steps."""
    if name not in ("ctypes", "library"):
        raise ValueError(f"binding must be 'ctypes' or 'library', not {name!r}")
    if name == "library":
        from . import library  # noqa: F401  (registers the operators)
    _BINDING[0] = name


def binding():
    return _BINDING[0]


def _library():
    if _BINDING[0] != "library":
        return None
    from . import library
    return library


def preact_block(x, blk):
    lb = _library()
    if lb is not None:
        return lb.block(x, blk)
    return PreActBlockFn.apply(x, blk, *param_edges(blk._fn_params, x))


def preact_run(fn, x, plan):
    lb = _library()
    if lb is not None:
        return lb.run(fn, x, plan)
    return fn.apply(x, plan, *param_edges(plan.params, x))


def upsample(x):
    lb = _library()
    if lb is not None:
        return lb.upsample(x)
    return UpsampleFn.apply(x)


def parse_input(x, w, b, half):
    lb = _library()
    if lb is not None:
        return lb.parse_input(x, w, b, half)
    return ParseInputFn.apply(x, w, b, half)


def quantize(z, q):
    lb = _library()
    if lb is not None:
        return lb.quantize(z, q)
    return QuantizeFn.apply(z, q)


def recon_loss(dec, x, nvs, cylinder, *commit):
    lb = _library()
    if lb is not None:
        total, recon = lb.recon_loss(dec, x, nvs, cylinder, *commit)
        return total, recon
    return ReconLossFn.apply(dec, x, nvs, cylinder, *commit)


def param_edges(params, *acts):
    """The parameters as autograd inputs of a Function only when no activation input already ties
    it into the graph.  The kernels accumulate parameter gradients straight into the flat buffer
    (backward returns None for them), so an edge per parameter only costs the autograd engine time
    (a 50-block run has 550 of them); a node fed by data alone keeps them so its backward runs."""
    for a in acts:
        if a is not None and a.requires_grad:
            return ()
    return params


def grad_buf(p):
    """fp32 gradient buffer of parameter p (allocated zeroed if the caller set it to None)."""
    if p is None:
        return None
    if p.grad is None:
        p.grad = ops.zero_(torch.empty_like(p))
    return p.grad


def _cl(g):
    if g.is_contiguous(memory_format=CL) or (g.shape[1] == 1 and g.is_contiguous()):
        return g
    return g.contiguous(memory_format=CL)


def mode_geometry(mode):
    """branch conv2 of a residual block (layers.py:124-132 / 239-247 / 28-36)."""
    if mode == "down":
        return 4, 2, 1, False
    if mode in ("same", "out"):
        return 3, 1, 1, False
    return 3, 1, 1, True


# ============================================================================================ PreAct block
class PreActBlockFn(torch.autograd.Function):
    """PreActFixupResBlock.forward (layers.py:176-195), circular padding (layers.py:109).

    Each conv's epilogue writes the NEXT conv's activated input, so no kernel recomputes an
    ELU for a k^3 gather:
        t2  = elu(conv1(elu(x + b1a) + b1b) + b2a) + b2b      (1x1, prologue + ELU_AFFINE epilogue)
        t3  = elu(conv2(t2 | up(t2)) + b3a) + b3b            (k^3 circular, ELU_AFFINE epilogue)
        s   = skip(x + b1c) + b1d                              (if present; half grid in up mode)
        out = conv3(t3) * scale + b4 + (s | up(s) | x)        (1x1)
    Backward recovers elu'(z) from the saved activated tensors (t - b > 0 ? 1 : t - b + 1).
    Saved: x, t2, t3 (+ up(t2) in up mode)."""

    @staticmethod
    def forward(ctx, x, blk, *params):
        ctx.n_params = len(params)
        k, s, p, up = mode_geometry(blk.mode)
        g1 = ConvGeom(1)
        x = ops.as_cl(x)
        ctx.tiny = (blk.skip_conv is None and not up and k == 3 and s == 1 and ops.tiny_blocks_enabled()
                    and ops.preact_tiny_supported(x.shape, blk.branch_conv1.weight.shape[0]))
        if ctx.tiny:
            # whole block in one launch (tiny_block.hip); t2 / t3 saved in fp32
            out, saved = ops.preact_tiny_fwd(x, blk)
            ctx.blk = blk
            ctx.save_for_backward(x, saved)
            return out
        ctx.small = False
        # no backward follows (eval / no_grad: the encode-only extraction path): the fused
        # kernels skip writing the saved intermediates
        save = any(ctx.needs_input_grad)
        if (blk.skip_conv is None and not up and k == 3 and s == 1
                and ops.preact_small_supported(x, blk.branch_conv1.weight.shape[0])):
            # few-channel blocks: fused forward (preact_small.hip / preact_col.hip); t2 / t3 saved
            # in bf16 as the unfused convs write them, so either backward applies
            out, t2, t3 = ops.preact_small_fwd(x, blk, save=save)
            ctx.blk = blk
            ctx.small = ops.small_backward_fused(x)
            ctx.save_for_backward(x, t2, t3, None)
            return out
        if (blk.skip_conv is None and not up and k == 3 and s == 1
                and ops.preact_mid_supported(x, blk.branch_conv1.weight.shape[0])):
            # 18-channel level: fused forward (2 launches) and backward (3 launches),
            # preact_mid.hip
            out, t2, t3 = ops.preact_mid_fwd(x, blk, save=save)
            ctx.blk = blk
            ctx.mid = True
            ctx.save_for_backward(x, t2, t3, None)
            return out
        t2 = ops.conv_fwd(x, blk.branch_conv1.weight, g1, pro=(blk.bias1a, blk.bias1b), act=(blk.bias2a, blk.bias2b))
        if up:
            tup = ops.upsample2x(t2)
            t3 = ops.conv_fwd(tup, blk.branch_conv2.weight, ConvGeom(3, 1, 1, True), act=(blk.bias3a, blk.bias3b))
        else:
            tup = None
            t3 = ops.conv_fwd(t2, blk.branch_conv2.weight, ConvGeom(k, s, p, True), act=(blk.bias3a, blk.bias3b))
        if blk.skip_conv is not None:
            gs = ConvGeom(2, 2, 0) if blk.mode == "down" else g1
            # up mode: W (up(x + b1c)) + b1d == up(W (x + b1c) + b1d) (both linear, weights sum to 1),
            # so the skip runs on the half grid and is upsampled inside conv3's epilogue
            res = ops.conv_fwd(x, blk.skip_conv.weight, gs, pro=(blk.bias1c,), bias=blk.bias1d)
        else:
            res = x
        out = ops.conv_fwd(t3, blk.branch_conv3.weight, g1, scale=blk.scale, bias=blk.bias4, residual=res,
                           residual_up2=up)
        ctx.blk = blk
        ctx.save_for_backward(x, t2, t3, tup)
        return out

    @staticmethod
    def backward(ctx, g):
        blk = ctx.blk
        g = _cl(g)
        if ctx.tiny:
            x, saved = ctx.saved_tensors
            gb = grad_buf
            names = {"dw1": blk.branch_conv1.weight, "dw2": blk.branch_conv2.weight, "dw3": blk.branch_conv3.weight,
                     "dbias1a": blk.bias1a, "dbias1b": blk.bias1b, "dbias2a": blk.bias2a, "dbias2b": blk.bias2b,
                     "dbias3a": blk.bias3a, "dbias3b": blk.bias3b, "dscale": blk.scale, "dbias4": blk.bias4}
            g_x = ops.preact_tiny_bwd(g, x, saved, blk, {n: gb(t) for n, t in names.items()})
            grads_ready(blk._fn_params)
            return (g_x, None) + (None,) * ctx.n_params
        x, t2, t3, tup = ctx.saved_tensors
        if ctx.small or getattr(ctx, "mid", False):
            names = {"dw1": blk.branch_conv1.weight, "dw2": blk.branch_conv2.weight, "dw3": blk.branch_conv3.weight,
                     "dbias1a": blk.bias1a, "dbias1b": blk.bias1b, "dbias2a": blk.bias2a, "dbias2b": blk.bias2b,
                     "dbias3a": blk.bias3a, "dbias3b": blk.bias3b, "dscale": blk.scale, "dbias4": blk.bias4}
            bwd = ops.preact_small_bwd if ctx.small else ops.preact_mid_bwd
            g_x = bwd(g, x, t2, t3, blk, {n: grad_buf(t) for n, t in names.items()})
            grads_ready(blk._fn_params)
            return (g_x, None) + (None,) * ctx.n_params
        k, s, p, up = mode_geometry(blk.mode)
        g1 = ConvGeom(1)
        gb = grad_buf
        # conv3 (1x1): g_h2 = scale * W3^T g * elu'(h2 + b3a), elu' from t3
        g_h2, _ = ops.conv_bwd(g, t3, blk.branch_conv3.weight, g1, gscale=blk.scale, aux=t3, aux_b=blk.bias3b,
                               dw=gb(blk.branch_conv3.weight), dscale=gb(blk.scale), dbias=gb(blk.bias4),
                               dpro_pre=gb(blk.bias3b), dpro_post=gb(blk.bias3a), escale=blk.scale)
        # conv2
        if up:
            g_tup, _ = ops.conv_bwd(g_h2, tup, blk.branch_conv2.weight, ConvGeom(3, 1, 1, True),
                                    dw=gb(blk.branch_conv2.weight))
            g_h1 = ops.upsample2x_bwd(g_tup, t2.shape, aux=t2, aux_b=blk.bias2b, dpro_pre=gb(blk.bias2b),
                                      dpro_post=gb(blk.bias2a))
        else:
            g_h1, _ = ops.conv_bwd(g_h2, t2, blk.branch_conv2.weight, ConvGeom(k, s, p, True), aux=t2,
                                   aux_b=blk.bias2b, dw=gb(blk.branch_conv2.weight), dpro_pre=gb(blk.bias2b),
                                   dpro_post=gb(blk.bias2a))
        # skip path
        if blk.skip_conv is not None:
            gs = ConvGeom(2, 2, 0) if blk.mode == "down" else g1
            g_s = ops.upsample2x_bwd(g, x.shape[:1] + (blk.skip_conv.weight.shape[0],) + x.shape[2:]) if up else g
            addend, _ = ops.conv_bwd(g_s, x, blk.skip_conv.weight, gs, pro=(blk.bias1c,),
                                     dw=gb(blk.skip_conv.weight), dbias=gb(blk.bias1d), dpro_pre=gb(blk.bias1c))
        else:
            addend = g
        # conv1 (1x1 on the input grid) + residual gradient; elu'(x + b1a) from x
        g_x, _ = ops.conv_bwd(g_h1, x, blk.branch_conv1.weight, g1, pro=(blk.bias1a, blk.bias1b), aux=x,
                              addend=addend, dw=gb(blk.branch_conv1.weight), dpro_pre=gb(blk.bias1b),
                              dpro_post=gb(blk.bias1a))
        grads_ready(blk._fn_params)
        return (g_x, None) + (None,) * ctx.n_params


# ============================================================================================ block stack
_PRM = ("branch_conv1", "branch_conv2", "branch_conv3", "bias1a", "bias1b", "bias2a", "bias2b", "bias3a", "bias3b",
        "scale", "bias4")


def _prm_tensor(blk, n):
    return getattr(blk, n).weight if n.startswith("branch_conv") else getattr(blk, n)


class StackPlan:
    """Device tables of the parameter / gradient pointers of a run of blocks ([block][11], the
    order of vq3d_preact_stack_fwd), rebuilt when the parameters move (flat.py re-views)."""

    def __init__(self, blocks, out_dtype=None):
        self.blocks = list(blocks)
        self.params = [_prm_tensor(b, n) for b in self.blocks for n in _PRM]
        self.key = None
        self.out_dtype = out_dtype  # a run Function's output storage (None: its input's)

    def grad_ptrs(self, i):
        """gradient buffer addresses of block i (in the table order), after tables()"""
        return self.gptrs[i * len(_PRM): (i + 1) * len(_PRM)]

    def tables(self, dev):
        # fast path: no view was re-attached since the last build (flat.VERSION) and every .grad is set
        if (self.key is not None and self.key[0] == _flat.VERSION[0] and self.key[1] == dev
                and all(p.grad is not None for p in self.params)):
            return self.ptab, self.gtab
        for p in self.params:
            grad_buf(p)
        key = (_flat.VERSION[0], dev) + tuple(p.data_ptr() for p in self.params) + \
            tuple(p.grad.data_ptr() for p in self.params)
        if key != self.key:
            self.gptrs = [p.grad.data_ptr() for p in self.params]
            n = len(self.params)
            self.ptab = torch.tensor([p.data_ptr() for p in self.params], dtype=torch.int64).to(dev)
            self.gtab = torch.tensor([p.grad.data_ptr() for p in self.params], dtype=torch.int64).to(dev)
            assert self.ptab.numel() == n
            self.key = key
        return self.ptab, self.gtab


class PreActStackFn(torch.autograd.Function):
    """A run of identical PreActFixupResBlocks ('same', no skip) on a tiny grid: forward and
    backward in one launch each (preact_stack.hip), the residual stream fp32 inside the run."""

    @staticmethod
    def forward(ctx, x, plan, *params):
        ctx.n_params = len(params)
        x = ops.as_cl(x)
        b, c, h, w, d = x.shape
        nb = plan.blocks[0].branch_conv1.weight.shape[0]
        nblk = len(plan.blocks)
        ptab, _ = plan.tables(x.device)
        saved = torch.empty(L.query("vq3d_preact_stack_saved_floats", nblk, b, c, nb, h, w, d), dtype=torch.float32,
                            device=x.device)
        out = torch.empty_like(x, memory_format=ops.CL)
        ops._timed("k_stackm_fwd", lambda: L.call("vq3d_preact_stack_fwd", L.dtype_code(x), nblk, b, c, nb, h, w, d,
                                                  L.ptr(x), L.ptr(ptab), L.ptr(out), L.ptr(saved), L.stream()))
        ctx.plan = plan
        ctx.save_for_backward(saved)
        ctx.shape = (b, c, nb, h, w, d)
        return out

    @staticmethod
    def backward(ctx, g):
        (saved,) = ctx.saved_tensors
        plan = ctx.plan
        b, c, nb, h, w, d = ctx.shape
        g = _cl(g)
        ptab, gtab = plan.tables(g.device)
        gx = torch.empty_like(g, memory_format=ops.CL)
        nblk = len(plan.blocks)
        nws = L.query("vq3d_preact_stack_bwd_workspace_bytes", nblk, b, c, nb, h, w, d)
        ws = ops.workspace(nws, g.device)
        ops._timed("k_stackm_bwd", lambda: L.call("vq3d_preact_stack_bwd_ws", L.dtype_code(g), nblk, b, c, nb, h, w, d,
                                                  L.ptr(g), L.ptr(ptab), L.ptr(gtab), L.ptr(saved), L.ptr(gx),
                                                  L.ptr(ws), max(nws, 256), L.stream()))
        grads_ready(plan.params)
        return (gx, None) + (None,) * ctx.n_params


class PreActWideFn(torch.autograd.Function):
    """A run of 72-channel / branch-36 PreActFixupResBlocks (preact_wide.hip): the weights of the
    whole run packed once (one launch), then one fused launch per block forward and two per block
    backward (data path, weight-gradient partials into a slice of one run workspace) plus one
    fixed-order reduction launch for the whole run;
    the residual and gradient streams fp32 inside the run."""

    @staticmethod
    def forward(ctx, x, plan, *params):
        ctx.n_params = len(params)
        x = ops.as_cl(x)
        b, c, h, w, d = x.shape
        nb = plan.blocks[0].branch_conv1.weight.shape[0]
        ptab, _ = plan.tables(x.device)
        img, per = ops.preact_wide_pack(ptab, len(plan.blocks), c, nb, x.device, dtype=x.dtype)
        base = img.data_ptr()
        xs = ops.cast(x, torch.float32)
        save = any(ctx.needs_input_grad)
        saved = []
        for i, blk in enumerate(plan.blocks):
            out, t2, t3 = ops.preact_wide_fwd(xs, base + i * per, blk, save=save, dtype=x.dtype)
            if save:
                saved += [xs, t2, t3]
            xs = out
        ctx.plan, ctx.per, ctx.in_dtype = plan, per, x.dtype
        ctx.save_for_backward(img, *saved)
        return ops.cast(xs, x.dtype)

    @staticmethod
    def backward(ctx, g):
        img, *saved = ctx.saved_tensors
        plan = ctx.plan
        base = img.data_ptr()
        gs = ops.cast(_cl(g), torch.float32)
        run_ws, wbase, stride = ops.preact_wide_run_workspace(plan, gs.shape, gs.device)
        batched = ops.batched_wgrad() and not ops.concurrent_wgrad()
        run = [None] * len(plan.blocks)  # batched: (g, x, t2, t3) per block for one weight launch
        for i in reversed(range(len(plan.blocks))):
            blk = plan.blocks[i]
            xs, t2, t3 = saved[3 * i: 3 * i + 3]
            names = {"dw1": blk.branch_conv1.weight, "dw2": blk.branch_conv2.weight, "dw3": blk.branch_conv3.weight,
                     "dbias1a": blk.bias1a, "dbias1b": blk.bias1b, "dbias2a": blk.bias2a, "dbias2b": blk.bias2b,
                     "dbias3a": blk.bias3a, "dbias3b": blk.bias3b, "dscale": blk.scale, "dbias4": blk.bias4}
            if batched:
                run[i] = (gs, xs, t2, t3)
            gs = ops.preact_wide_bwd(gs, xs, t2, t3, base + i * ctx.per, blk,
                                     {n: grad_buf(t) for n, t in names.items()}, ws_ptr=wbase + i * stride,
                                     reduce=False, weights=not batched)
        if batched:
            ops.preact_wide_wgrad_run(plan, gs.shape, run_ws, stride, *[list(v) for v in zip(*run)])
        ops.preact_wide_reduce_run(plan, gs.shape, run_ws, stride)
        grads_ready(plan.params)
        return (ops.cast(gs, ctx.in_dtype), None) + (None,) * ctx.n_params


class PreActMidRunFn(torch.autograd.Function):
    """A run of 18-channel / branch-9 PreActFixupResBlocks (preact_mid.hip), chained: each block's
    tile kernel also writes the next block's t2 (forward) / the previous block's gz3 (backward)
    from the tile it holds in LDS, and the fixed-order gradient reductions of all blocks run as one
    launch, so a run of n blocks costs n + 1 forward and 3n + 2 backward launches instead of 2n and
    5n, and the out / gx round trips through the pointwise kernels are gone.  Numerics are the per-block path's (bit-identical t2 / gz3; only the scalar partial-sum
    grouping of the fused stage differs)."""

    @staticmethod
    def forward(ctx, x, plan, *params):
        ctx.n_params = len(params)
        save = any(ctx.needs_input_grad)
        out, saved = ops.preact_mid_run_fwd(x, plan.blocks, save=save)
        ctx.plan = plan
        if save:
            ctx.save_for_backward(*[t for trio in saved for t in trio])
        return out

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        flat = ctx.saved_tensors
        saved = [flat[3 * i: 3 * i + 3] for i in range(len(plan.blocks))]

        gx = ops.preact_mid_run_bwd(g, plan, saved, on_done=lambda: grads_ready(plan.params))
        return (gx, None) + (None,) * ctx.n_params


class PreActSmallRunFn(torch.autograd.Function):
    """A run of few-channel PreActFixupResBlocks ((C, branch) = (2, 1), (4, 2), (8, 4); preact_small.hip /
    preact_col.hip): the fused forward per block, the fused backward per block into slices of one
    run workspace, and the fixed-order gradient reductions of all blocks as one launch pair at the
    end (instead of one or two small launches per block).  The residual stream between the run's
    blocks is fp32 (ops.fp32_stream(); the reference's autocast blocks return fp32,
    layers.py:187-193); the run returns its input's dtype, or fp32 when plan.out_dtype says so (the
    encoder's pre-quantize runs feed the fp32 Quantizer, layers.py:685-687)."""

    @staticmethod
    def forward(ctx, x, plan, *params):
        ctx.n_params = len(params)
        save = any(ctx.needs_input_grad)
        saved = []
        n = len(plan.blocks)
        last_dt = plan.out_dtype or x.dtype
        odts = [last_dt if i == n - 1 else (torch.float32 if ops.fp32_stream() else x.dtype) for i in range(n)]
        if ops.small_chain_ok(x, n):  # column kernels: each launch hands the next block its t2
            x, runs = ops.preact_small_run_fwd(x, plan.blocks, save, odts)
            saved = [t for r in runs for t in r]
        else:
            fmt = ops._fmt16(x)
            for i, blk in enumerate(plan.blocks):
                out, t2, t3 = ops.preact_small_fwd(x, blk, save=save, out_dtype=odts[i], fmt=fmt)
                if save:
                    saved += [x, t2, t3]
                x = out
        ctx.plan = plan
        if save:
            ctx.save_for_backward(*saved)
        return x

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        flat = ctx.saved_tensors
        saved = [flat[3 * i: 3 * i + 3] for i in range(len(plan.blocks))]
        gx = ops.preact_small_run_bwd(g, plan, saved, on_done=lambda: grads_ready(plan.params))
        return (gx, None) + (None,) * ctx.n_params


def small_run_eligible(x, blk):
    k, s, _, up = mode_geometry(blk.mode)
    return (stack_eligible(blk) and k == 3 and s == 1 and not up and x.is_cuda and x.dim() == 5
            and x.shape[1] == blk.in_channels and ops.preact_small_supported(x, blk.branch_conv1.weight.shape[0])
            and ops.small_backward_fused(x))


def mid_run_eligible(x, blk):
    k, s, _, up = mode_geometry(blk.mode)
    return (stack_eligible(blk) and k == 3 and s == 1 and not up and x.is_cuda and x.dim() == 5
            and x.shape[1] == blk.in_channels and ops.preact_mid_supported(x, blk.branch_conv1.weight.shape[0]))


def wide_eligible(x, blk):
    return (stack_eligible(blk) and x.is_cuda and x.dim() == 5 and x.shape[1] == blk.in_channels
            and ops.preact_wide_supported(x, blk.branch_conv1.weight.shape[0]))


def stack_eligible(blk):
    return (type(blk).__name__ == "PreActFixupResBlock" and blk.skip_conv is None and blk.mode in ("same", "out"))


# ============================================================================================ generic conv
class ConvFn(torch.autograd.Function):
    """One nn.Conv3d call with the fused prologue / epilogue (regular + EvoNorm blocks,
    parse_input / proj / out, layers.py:535,377,490,508).  `spec` carries the geometry and
    the Parameter objects whose .grad the kernels accumulate into."""

    @staticmethod
    def forward(ctx, x, x2, residual, spec, *tensors):
        ctx.n_params = len(tensors)
        y = ops.conv_fwd(x, spec.w, spec.geom, pro=spec.pro, x2=x2, scale=spec.scale, bias=spec.bias,
                         cbias=spec.cbias, residual=residual, residual_up2=spec.residual_up2,
                         act="elu" if spec.post_elu else None)
        ctx.spec = spec
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, x2, y if spec.post_elu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        spec = ctx.spec
        x, x2, y = ctx.saved_tensors
        g = _cl(g)
        if spec.post_elu:
            gz = torch.empty_like(g)
            L.call("vq3d_elu_bwd_from_output", L.dtype_code(g), L.ptr(g), L.ptr(y), L.ptr(gz), g.numel(),
                   L.stream())
            g = gz
        g_res = None
        if ctx.has_res and ctx.needs_input_grad[2]:
            if spec.residual_up2:
                b, c, h, w, d = g.shape
                g_res = ops.upsample2x_bwd(g, (b, c, h // 2, w // 2, d // 2))
            else:
                g_res = g
        gb = grad_buf
        pro_pre = pro_post = None
        if spec.pro is not None:
            if len(spec.pro) == 1:
                pro_pre = gb(spec.pro_params[0])
            else:
                pro_pre, pro_post = gb(spec.pro_params[1]), gb(spec.pro_params[0])
        want = ctx.needs_input_grad[0] or (x2 is not None and ctx.needs_input_grad[1])
        gx, gx2 = ops.conv_bwd(g, x, spec.w, spec.geom, pro=spec.pro, x2=x2, gscale=spec.scale, aux=x,
                               want_gx=want, dw=gb(spec.w), dscale=gb(spec.scale), dbias=gb(spec.bias),
                               dcbias=gb(spec.cbias), dpro_pre=pro_pre, dpro_post=pro_post, escale=spec.scale)
        if not want:
            gx = gx2 = None
        grads_ready(spec.tensors)
        return (gx, gx2, g_res, None) + (None,) * ctx.n_params


class ConvSpec:
    __slots__ = ("w", "geom", "pro", "pro_params", "scale", "bias", "cbias", "residual_up2", "post_elu",
                 "tensors")

    def __init__(self, w, geom, pro=None, scale=None, bias=None, cbias=None, residual_up2=False, post_elu=False):
        self.w, self.geom, self.scale, self.bias, self.cbias = w, geom, scale, bias, cbias
        self.pro = pro
        self.pro_params = pro
        self.residual_up2, self.post_elu = residual_up2, post_elu
        self.tensors = tuple(t for t in (w, scale, bias, cbias) + tuple(pro or ()) if t is not None)


def conv(x, spec, x2=None, residual=None):
    lb = _library()
    if lb is not None:
        return lb.conv(x, spec, x2, residual)
    return ConvFn.apply(x, x2, residual, spec, *param_edges(spec.tensors, x, x2, residual))


# ============================================================================================ parse_input
class ParseInputFn(torch.autograd.Function):
    """Encoder2.parse_input (layers.py:535): Conv3d(1 -> C, k = 1, bias) reading the fp32 input
    volume and writing the 16-bit activation (half: bf16 or fp16; vq3d_parse_input_*): the volume is
    never rounded to bf16 (the reference's autocast rounds it to fp16).  Weight / bias gradients
    only."""

    @staticmethod
    def forward(ctx, x, w, b, half):
        bsz, _, h, wd, d = x.shape
        c = w.shape[0]
        nv = bsz * h * wd * d
        y = ops.new_act(bsz, c, h, wd, d, half, x.device)
        L.call("vq3d_parse_input_fwd", L.dtype_code(half), nv, c, L.ptr(x), L.ptr(w), L.ptr(b), L.ptr(y), L.stream())
        ctx.save_for_backward(x)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        w, b = ctx.params
        g = _cl(g)
        c = w.shape[0]
        nv = x.numel()
        nws = int(L.query("vq3d_parse_input_workspace_bytes", nv, c))
        ws = ops.workspace(nws, x.device)
        L.call("vq3d_parse_input_bwd", L.dtype_code(g), nv, c, L.ptr(x), L.ptr(g), L.ptr(grad_buf(w)), L.ptr(grad_buf(b)), L.ptr(ws),
               nws, L.stream())
        grads_ready((w, b))
        return None, None, None, None


def parse_input_fused(x, conv, compute_dtype):
    """True when the fp32 volume can go through ParseInputFn (1 input channel, bf16 activations)."""
    return (compute_dtype in (torch.bfloat16, torch.float16) and x.dtype == torch.float32 and x.is_cuda and x.dim() == 5
            and x.shape[1] == 1 and conv.in_channels == 1 and conv.out_channels in (2, 4, 8)
            and conv.bias is not None and x.is_contiguous() and (x.numel() // max(x.shape[0], 1)) % 4 == 0
            and _aligned16(x))  # k_pin_fwd / k_pin_wgrad: float4 loads, 16- to 64-B stores


def _aligned16(x):
    try:
        return x.data_ptr() % 16 == 0
    except RuntimeError:  # a traced (fake) tensor has no storage: the operator checks at run time
        return True


# ============================================================================================ upsample
class UpsampleFn(torch.autograd.Function):
    """nn.Upsample(trilinear, x2, align_corners=False) of ResizeConv3D (layers.py:591-597)."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = tuple(x.shape)
        return ops.upsample2x(x)

    @staticmethod
    def backward(ctx, g):
        return ops.upsample2x_bwd(_cl(g), ctx.shape)


# ============================================================================================ EvoNorm-S0
class EvoNormFn(torch.autograd.Function):
    """EvoNorm3DS0 (evonorm.py:59-76): x*sigmoid(v x)*gamma / group_std(x) + beta, batch 1."""

    @staticmethod
    def forward(ctx, x, mod, v, gamma, beta):
        x = ops.as_cl(x)
        b, c = x.shape[:2]
        if b != 1:
            # the reference's group_std reshapes its std to batch 1 (evonorm.py:24) and fails
            raise RuntimeError("EvoNorm3DS0 supports batch size 1 only (reference semantics, evonorm.py:24)")
        nvox = x.numel() // c
        y = torch.empty_like(x)
        groups = max(c // 8, 1)
        stats = torch.empty(2 * groups, dtype=torch.float32, device=x.device)
        ws = ops.workspace(L.query("vq3d_evonorm_workspace_size", c, nvox), x.device)
        L.call("vq3d_evonorm_fwd", L.dtype_code(x), L.ptr(x), c, nvox, L.ptr(v), L.ptr(gamma), L.ptr(beta),
               L.ptr(y), L.ptr(stats), L.ptr(ws), L.stream())
        ctx.mod = mod
        ctx.save_for_backward(x, stats)
        return y

    @staticmethod
    def backward(ctx, g):
        x, stats = ctx.saved_tensors
        mod = ctx.mod
        g = _cl(g)
        c = x.shape[1]
        nvox = x.numel() // c
        gx = torch.empty_like(x)
        ws = ops.workspace(L.query("vq3d_evonorm_workspace_size", c, nvox), x.device)
        L.call("vq3d_evonorm_bwd", L.dtype_code(x), L.ptr(x), L.ptr(g), c, nvox, L.ptr(mod.v), L.ptr(mod.gamma),
               L.ptr(stats), L.ptr(gx), L.ptr(grad_buf(mod.v)), L.ptr(grad_buf(mod.gamma)),
               L.ptr(grad_buf(mod.beta)), L.ptr(ws), L.stream())
        grads_ready((mod.v, mod.gamma, mod.beta))
        return gx, None, None, None, None


# ============================================================================================ quantizer
def vq_init(z, q):
    """_init_ema (layers.py:665-683) on the first training pass: mean / unbiased std of this rank's
    rows, summed over the ranks in one all-reduce (C3) and divided by the world size in the init
    kernel."""
    b, d, h, w, dz = z.shape
    n = b * h * w * dz
    k = q.num_embeddings
    dev = z.device
    st = L.stream()
    ws = ops.workspace(L.query("vq3d_vq_workspace_size", n, d, k), dev)
    ms = torch.empty(2 * d, dtype=torch.float32, device=dev)
    mean, std = ms[:d], ms[d:]
    L.call("vq3d_vq_moments", L.dtype_code(z), L.ptr(z), n, d, L.ptr(mean), L.ptr(std), L.ptr(ws), st)
    world = sum_allreduce(ms)
    n_tot = float(n) * world
    L.call("vq3d_vq_init_apply", L.ptr(q.embed), L.ptr(q.embed_avg), L.ptr(q.cluster_size),
           L.ptr(q.first_pass), L.ptr(mean), L.ptr(std), k, d, 1.0 / world, n_tot, st)
    q.first_pass_host = False


def vq_search(z, embed, commitment_cost, zst_dtype=None):
    """The codebook search (exact torch-CPU cdist arithmetic), the straight-through output (in
    zst_dtype: the model's conv operand storage, its consumers are convs / the decoder's runs) and
    the commitment loss: returns loss, zst, idx."""
    b, d, h, w, dz = z.shape
    n = b * h * w * dz
    k = embed.shape[0]
    dev = z.device
    st = L.stream()
    ws = ops.workspace(L.query("vq3d_vq_workspace_size", n, d, k), dev)
    idx = torch.empty((b, h, w, dz), dtype=torch.int64, device=dev)
    zst = torch.empty_like(z, dtype=zst_dtype or z.dtype)
    sq = torch.empty((), dtype=torch.float32, device=dev)
    L.call("vq3d_vq_nearest", L.dtype_code(z), L.ptr(z), n, d, L.ptr(embed), k, L.ptr(idx), L.dtype_code(zst),
           L.ptr(zst), L.ptr(sq), L.ptr(ws), st)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    L.call("vq3d_vq_commit_loss", L.ptr(sq), commitment_cost / float(n * d), L.ptr(loss), st)
    return loss, zst, idx


def vq_ema(z, idx, q):
    """_update_ema (layers.py:636-663).  Inside Encoder2 the statistics land in the encoder's fused
    buffer (q.ema_slot) and the update waits for its single all-reduce."""
    b, d, h, w, dz = z.shape
    n = b * h * w * dz
    k = q.num_embeddings
    ws = ops.workspace(L.query("vq3d_vq_workspace_size", n, d, k), z.device)
    slot = q.ema_slot
    stats = torch.empty(k * (d + 1), dtype=torch.float32, device=z.device) if slot is None else slot
    counts, dw = stats[:k], stats[k:]
    L.call("vq3d_vq_ema_stats", L.dtype_code(z), L.ptr(z), n, d, L.ptr(idx), k, L.ptr(counts), L.ptr(dw), L.ptr(ws),
           L.stream())
    if slot is None:
        sum_allreduce(stats)
        ema_update(q, stats)


def vq_backward(z, embed, idx, coef, g_loss, g_zst):
    """Straight-through gradient plus the commitment term 2 cc (z - e_idx) / (n d) (layers.py:713-728)."""
    b, d, h, w, dz = z.shape
    n = b * h * w * dz
    if g_zst is None:
        g_zst = ops.zero_(torch.empty_like(z))
    g_zst = _cl(g_zst)
    gz = torch.empty_like(z)
    L.call("vq3d_vq_bwd", L.dtype_code(z), L.ptr(z), n, d, L.ptr(embed), L.ptr(idx), L.dtype_code(g_zst),
           L.ptr(g_zst), None if g_loss is None else L.ptr(g_loss), coef, L.ptr(gz), L.stream())
    return gz


class QuantizeFn(torch.autograd.Function):
    """Quantizer.forward (layers.py:685-728): fp32 codebook search (exact torch-CPU cdist
    arithmetic), EMA update in train mode, commitment loss, straight-through output."""

    @staticmethod
    def forward(ctx, z, q):
        z = ops.as_cl(z)
        b, d, h, w, dz = z.shape
        if q.training and q.first_pass_host:
            vq_init(z, q)
        embed = q.embed
        if q.training:
            # the pre-update codebook for q / backward (the updated one is first read by the NEXT step)
            embed = ops.copy_(torch.empty_like(q.embed), q.embed)
        loss, zst, idx = vq_search(z, embed, q.commitment_cost, getattr(q, "zst_dtype", None))
        if q.training:
            vq_ema(z, idx, q)
        ctx.coef = 2.0 * q.commitment_cost / float(b * h * w * dz * d)
        ctx.save_for_backward(z, embed, idx)
        ctx.mark_non_differentiable(idx)
        return loss, zst, idx

    @staticmethod
    def backward(ctx, g_loss, g_zst, g_idx):
        z, embed, idx = ctx.saved_tensors
        return vq_backward(z, embed, idx, ctx.coef, g_loss, g_zst), None


def ema_update(q, stats):
    """EMA decay + Laplace smoothing of one Quantizer from its (all-reduced) statistics
    [counts (K) | dw (K x D)] (layers.py:649-663)."""
    k, d = q.num_embeddings, q.embedding_dim
    L.call("vq3d_vq_ema_update", L.ptr(q.embed), L.ptr(q.embed_avg), L.ptr(q.cluster_size), L.ptr(stats[:k]),
           L.ptr(stats[k:]), k, d, q.decay, q.laplace_alpha, L.stream())


# ============================================================================================ loss
class ReconLossFn(torch.autograd.Function):
    """VQVAE.loc_metric with F.smooth_l1_loss (model.py:115-163): returns (total, recon) with
    total = recon + sum(commitment losses)."""

    @staticmethod
    def forward(ctx, dec, x, nvs, cylinder, *commit):
        dec = ops.as_cl(dec)
        b, c, h, w, d = dec.shape
        if c != 1:
            # the loss kernels index (B, H, W, D) volumes; the published runs use one input channel
            raise NotImplementedError(f"recon loss kernels take --input-channels 1 (got {c} channels)")
        if tuple(x.shape) != tuple(dec.shape) or not x.is_contiguous():
            raise ValueError(f"target volume {tuple(x.shape)} must be a contiguous {tuple(dec.shape)} tensor")
        dev = dec.device
        recon = torch.empty((), dtype=torch.float32, device=dev)
        total = torch.empty((), dtype=torch.float32, device=dev)
        ws = ops.workspace(L.query("vq3d_recon_loss_workspace_size", b, h, w, d), dev)
        arr = (ctypes.c_void_p * 8)(*[c.data_ptr() for c in commit])
        L.call("vq3d_recon_loss_fwd", L.dtype_code(dec), L.ptr(dec), L.ptr(x), L.ptr(nvs), b, h, w, d,
               int(cylinder), arr, len(commit), L.ptr(recon), L.ptr(total), L.ptr(ws), L.stream())
        ctx.cyl = int(cylinder)
        ctx.ncommit = len(commit)
        ctx.save_for_backward(dec, x, nvs)
        ctx.mark_non_differentiable(recon)
        return total, recon

    @staticmethod
    def backward(ctx, g_total, g_recon):
        dec, x, nvs = ctx.saved_tensors
        b, _, h, w, d = dec.shape
        gdec = torch.empty_like(dec)
        L.call("vq3d_recon_loss_bwd", L.dtype_code(dec), L.ptr(dec), L.ptr(x), L.ptr(nvs), b, h, w, d, ctx.cyl,
               L.ptr(g_total), L.ptr(gdec), L.stream())
        return (gdec, None, None, None) + (g_total,) * ctx.ncommit
