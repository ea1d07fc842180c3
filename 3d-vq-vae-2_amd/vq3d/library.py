"""torch.library binding of the hot path: the libvq3d entry points as registered PyTorch operators
(namespace `vq3d`) with autograd registrations, so the model's step can run through
`torch.ops.vq3d.*` (SURVEY.md 8(b) "Binding"; the reference's ops are ATen calls,
vqvae/layers.py:134-171 nn.Conv3d, :685-728 the Quantizer, model.py:115-163 the loss).

    vq3d::conv3d / conv3d_backward            one nn.Conv3d with its fused prologue / epilogue
    vq3d::preact_block / preact_block_backward one PreActFixupResBlock (layers.py:176-195)
    vq3d::preact_run / preact_run_backward    a fused run of identical blocks (kind: stack | wide |
                                              mid | small, the engines of vq3d.functional)
    vq3d::vq_nearest / vq_nearest_backward    codebook search + commitment loss + straight-through
                                              output (layers.py:700-728)
    vq3d::vq_init, vq3d::vq_ema               the codebook's first-pass init and EMA statistics /
                                              update (mutating, no autograd; layers.py:636-683)
    vq3d::parse_input / parse_input_backward  the fp32 volume into the 16-bit activation (layers.py:535)
    vq3d::upsample2x / upsample2x_backward    trilinear x2 (layers.py:591-597)
    vq3d::recon_loss / recon_loss_backward    smooth-L1 reconstruction + commitment sum (model.py:115-163)

Each operator runs exactly the kernels of the ctypes path (the same autograd.Function bodies of
vq3d.functional, driven through a stand-in context), so `vq3d.functional.set_binding("library")`
gives a bit-identical step (tests/test_gpu_library.py).  Operator contracts:
  * a forward operator returns [outputs..., meta, saved...]: `meta` (int64, host) holds the path
    flags the forward chose and, per saved tensor of the backward, a code: -1 none, k >= 0 the k-th
    `saved` tensor, -2 - i the i-th of the forward's tensor inputs / outputs (outputs never alias
    inputs, as torch.library requires);
  * a backward operator takes the resolved saved list and the parameter gradient buffers
    (`grads`, mutated: the kernels accumulate into them, `param.grad` of vq3d.flat) and returns
    [codes, new...] for the input gradients in the same encoding over its own tensor inputs;
  * parameters are operator inputs, so autograd sees every edge; their gradients arrive through
    `grads`, and the autograd formulas return None for them.
The model's layers (set_binding("library")) reach the operators through `_Call`: the operator
dispatched below the autograd key, its registered formula applied by one autograd.Function (a
direct torch.ops.vq3d call under autograd uses the same formula through register_autograd).
No fake (meta-device) kernels are registered: the operators are for eager execution and HIP-graph
capture of it, not for tracing compilers."""
from typing import List, Optional

import torch

from . import _lib as L
from . import functional as Fn
from . import ops
from .ops import ConvGeom

Tensor = torch.Tensor
_FLAGS = ("tiny", "small", "mid")  # PreActBlockFn's path choice (the only forward-chosen state)


# ------------------------------------------------------------------------------------------------ plumbing
class _Ctx:
    """Stands in for an autograd context inside an operator body."""

    def __init__(self, needs=(True,)):
        self.needs_input_grad = tuple(needs)
        self.saved_tensors = ()

    def save_for_backward(self, *ts):
        self.saved_tensors = ts

    def mark_non_differentiable(self, *ts):
        pass


def _flat(items):
    out = []
    for t in items:
        if isinstance(t, (list, tuple)):
            out.extend(t)
        elif isinstance(t, torch.Tensor) or t is None:
            out.append(t)
    return out


def _pack(ts, pool):
    """tensors (or None) -> (codes, new): -1 None, -2 - i the pool's i-th tensor (by identity), k the
    k-th of `new`"""
    codes, new = [], []
    for t in ts:
        if t is None:
            codes.append(-1)
            continue
        hit = next((i for i, p in enumerate(pool) if p is t), None)
        if hit is not None:
            codes.append(-2 - hit)
            continue
        k = next((i for i, p in enumerate(new) if p is t), None)  # outputs may not alias each other either
        if k is None:
            k = len(new)
            new.append(t)
        codes.append(k)
    return codes, new


def _unpack(codes, new, pool):
    return [None if c == -1 else (pool[-2 - c] if c < -1 else new[c]) for c in codes]


def _forward(fn, nout, pool_in, needs, *args):
    """Run an autograd.Function's forward body; returns the forward operator's tensor list."""
    ctx = _Ctx(needs)
    res = fn.forward(ctx, *args)
    outs = list(res) if isinstance(res, tuple) else [res]
    assert len(outs) == nout
    flags = [int(getattr(ctx, f)) if hasattr(ctx, f) else -1 for f in _FLAGS]
    codes, new = _pack(ctx.saved_tensors, pool_in + outs)
    return outs + [torch.tensor(flags + codes, dtype=torch.int64)] + new


def _saved(ctx, inputs, output, nout, pool_fn):
    """setup_context helper: the backward's saved list and the forward's path flags."""
    outs, meta, new = list(output[:nout]), output[nout], list(output[nout + 1:])
    m = meta.tolist()
    ctx.flags = m[:len(_FLAGS)]
    ctx.saved = _unpack(m[len(_FLAGS):], new, pool_fn(inputs) + outs)
    ctx.mark_non_differentiable(meta, *new)
    ctx.set_materialize_grads(False)  # no zero-filled gradients for the saved-tensor outputs


def _backward(fn, ctx, pool, grads_out):
    """Run an autograd.Function's backward body on a stand-in context; returns [codes, new...]."""
    res = fn.backward(ctx, *grads_out)
    codes, new = _pack(res, pool)
    return [torch.tensor(codes, dtype=torch.int64)] + new


def _grads_of(res, pool):
    return _unpack(res[0].tolist(), list(res[1:]), pool)


def _check_grads(params, grads):
    for p, g in zip(params, grads):
        if g is not None and p.grad is not g:
            raise ValueError("vq3d: `grads` must be the parameters' .grad buffers (vq3d.flat.FlatParams)")


def _needs(ctx, n):
    """needs_input_grad of the first n inputs (under _Call: of its differentiable inputs)"""
    return list(ctx.needs) if hasattr(ctx, "needs") else list(ctx.needs_input_grad[:n])


def _save_flag(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in _flat(ts))


# ------------------------------------------------------------------------------------------------ calls
_BELOW = torch._C._AutoDispatchBelowAutograd
_FORMULAS = {}  # operator -> (setup_context, backward, differentiable input positions)


class _Call(torch.autograd.Function):
    """One differentiable operator of this module, dispatched BELOW the autograd key, with its
    registered formula (the setup_context / backward given to torch.library.register_autograd)
    applied by this Function: the same gradients as calling torch.ops.vq3d.<op> under autograd,
    without the custom-op autograd layer's Python cost (~30 us of a ~45 us call; the step's ~700
    calls otherwise outrun the GPU).  `tracked`: the operator's differentiable inputs (in
    `_FORMULAS` order), then the parameter edges (Fn.param_edges) the node needs to exist."""

    @staticmethod
    def forward(ctx, name, args, *tracked):
        setup, _, diff = _FORMULAS[name]
        ctx.name, ctx.ntr = name, len(tracked)
        ctx.needs = [t is not None and t.requires_grad for t in tracked[:3]]  # conv3d's x, x2, residual
        with _BELOW():
            out = getattr(torch.ops.vq3d, name)(*args)
        setup(ctx, args, out)
        return tuple(out) if isinstance(out, (list, tuple)) else out

    @staticmethod
    def backward(ctx, *grads):
        _, bwd, diff = _FORMULAS[ctx.name]
        with _BELOW():
            res = bwd(ctx, list(grads) if len(grads) > 1 or ctx.name != "upsample2x" else grads[0])
        res = res if isinstance(res, tuple) else (res,)
        gs = []
        for i in diff:  # a list input (recon_loss's commitment losses) contributes one gradient per tensor
            gs.extend(res[i] if isinstance(res[i], list) else [res[i]])
        return (None, None) + tuple(gs) + (None,) * (ctx.ntr - len(gs))


def _register(name, bwd, setup, diff):
    torch.library.register_autograd(f"vq3d::{name}", bwd, setup_context=setup)
    _FORMULAS[name] = (setup, bwd, diff)


def _call(name, args, diff_inputs, params=()):
    """torch.ops.vq3d.<name>(*args) with autograd through _Call; with gradients off (eval,
    torch.no_grad: the traceable inference path) the operator itself."""
    if not torch.is_grad_enabled():
        out = getattr(torch.ops.vq3d, name)(*args)
        return tuple(out) if isinstance(out, (list, tuple)) else out
    return _Call.apply(name, args, *diff_inputs, *Fn.param_edges(params, *diff_inputs))


# ------------------------------------------------------------------------------------------------ block views
class _W:
    __slots__ = ("weight",)

    def __init__(self, w):
        self.weight = w


class BlockView:
    """The attributes of a PreActFixupResBlock the engines read, from its parameter list in
    PreActFixupResBlock._fn_params order (bias1a, bias1b, bias2a, bias2b, bias3a, bias3b, bias4,
    scale, conv1, conv2, conv3 [, bias1c, bias1d, skip])."""

    def __init__(self, params, mode):
        (self.bias1a, self.bias1b, self.bias2a, self.bias2b, self.bias3a, self.bias3b, self.bias4, self.scale,
         w1, w2, w3) = params[:11]
        self.branch_conv1, self.branch_conv2, self.branch_conv3 = _W(w1), _W(w2), _W(w3)
        if len(params) == 14:
            self.bias1c, self.bias1d = params[11], params[12]
            self.skip_conv = _W(params[13])
        else:
            self.skip_conv = None
        self.mode = mode
        self.in_channels = w1.shape[1]
        self._fn_params = list(params)


_VIEWS = {}


def _views(params, mode, per):
    key = (mode, per) + tuple(id(p) for p in params)
    v = _VIEWS.get(key)
    if v is None or any(a is not b for a, b in zip(v[1], params)):
        blocks = [BlockView(params[i:i + per], mode) for i in range(0, len(params), per)]
        v = _VIEWS[key] = (blocks, list(params), {})
    return v


def _plan(params, out_fp32):
    blocks, _, cache = _views(params, "same", 11)
    plan = cache.get("plan")
    if plan is None:
        plan = cache["plan"] = Fn.StackPlan(blocks)
    plan.out_dtype = torch.float32 if out_fp32 else None
    return plan


_RUNS = {"stack": Fn.PreActStackFn, "wide": Fn.PreActWideFn, "mid": Fn.PreActMidRunFn, "small": Fn.PreActSmallRunFn}
RUN_KINDS = {v: k for k, v in _RUNS.items()}


# ------------------------------------------------------------------------------------------------ conv3d
def _spec(weight, scale, bias, cbias, pro, geom, residual_up2, post_elu):
    return Fn.ConvSpec(weight, ConvGeom(*geom), pro=tuple(pro) if pro else None, scale=scale, bias=bias,
                       cbias=cbias, residual_up2=residual_up2, post_elu=post_elu)


def _conv_pool(inputs):
    return _flat(inputs[:3])  # x, x2, residual


@torch.library.custom_op("vq3d::conv3d", mutates_args=())
def conv3d(x: Tensor, x2: Optional[Tensor], residual: Optional[Tensor], weight: Tensor, scale: Optional[Tensor],
           bias: Optional[Tensor], cbias: Optional[Tensor], pro: List[Tensor], geom: List[int], residual_up2: bool,
           post_elu: bool, save: bool) -> List[Tensor]:
    spec = _spec(weight, scale, bias, cbias, pro, geom, residual_up2, post_elu)
    return _forward(Fn.ConvFn, 1, [x, x2, residual], (save,), x, x2, residual, spec)


@torch.library.custom_op("vq3d::conv3d_backward", mutates_args=("grads",))
def conv3d_backward(g: Tensor, saved: List[Optional[Tensor]], weight: Tensor, scale: Optional[Tensor],
                    bias: Optional[Tensor], cbias: Optional[Tensor], pro: List[Tensor], geom: List[int],
                    residual_up2: bool, post_elu: bool, has_res: bool, needs: List[bool],
                    grads: List[Tensor]) -> List[Tensor]:
    spec = _spec(weight, scale, bias, cbias, pro, geom, residual_up2, post_elu)
    _check_grads(spec.tensors, grads)
    ctx = _Ctx(needs)
    ctx.saved_tensors, ctx.spec, ctx.has_res, ctx.n_params = tuple(saved), spec, has_res, 0
    return _backward(Fn.ConvFn, ctx, [g], (g,))


def _conv_setup(ctx, inputs, output):
    _saved(ctx, inputs, output, 1, _conv_pool)
    ctx.args = inputs[3:11]
    ctx.has_res = inputs[2] is not None


def _conv_bwd(ctx, grads):
    weight, scale, bias, cbias, pro, geom, residual_up2, post_elu = ctx.args
    spec = _spec(weight, scale, bias, cbias, pro, geom, residual_up2, post_elu)
    g = grads[0]
    res = torch.ops.vq3d.conv3d_backward(g, ctx.saved, weight, scale, bias, cbias, pro, geom, residual_up2, post_elu,
                                         ctx.has_res, _needs(ctx, 3),
                                         [Fn.grad_buf(t) for t in spec.tensors])
    gx, gx2, gres = _grads_of(res, [g])[:3]
    return gx, gx2, gres, None, None, None, None, [None] * len(pro), None, None, None, None


_register("conv3d", _conv_bwd, _conv_setup, (0, 1, 2))


def conv(x, spec, x2=None, residual=None):
    """Fn.conv through the registered operator."""
    pro = list(spec.pro) if spec.pro else []
    save = _save_flag(x, x2, residual, *spec.tensors)
    g = spec.geom
    args = (x, x2, residual, spec.w, spec.scale, spec.bias, spec.cbias, pro, [g.k, g.s, g.p, int(g.circular)],
            spec.residual_up2, spec.post_elu, save)
    return _call("conv3d", args, (x, x2, residual), spec.tensors)[0]


# ------------------------------------------------------------------------------------------------ blocks
@torch.library.custom_op("vq3d::preact_block", mutates_args=())
def preact_block(x: Tensor, params: List[Tensor], mode: str, save: bool) -> List[Tensor]:
    blk = _views(params, mode, len(params))[0][0]
    return _forward(Fn.PreActBlockFn, 1, [x], (save,), x, blk)


@torch.library.custom_op("vq3d::preact_block_backward", mutates_args=("grads",))
def preact_block_backward(g: Tensor, saved: List[Optional[Tensor]], flags: List[int], params: List[Tensor],
                          mode: str, grads: List[Tensor]) -> List[Tensor]:
    _check_grads(params, grads)
    ctx = _Ctx()
    ctx.saved_tensors, ctx.blk, ctx.n_params = tuple(saved), _views(params, mode, len(params))[0][0], 0
    for f, v in zip(_FLAGS, flags):
        if v >= 0:
            setattr(ctx, f, bool(v))
    return _backward(Fn.PreActBlockFn, ctx, [g], (g,))


def _block_setup(ctx, inputs, output):
    _saved(ctx, inputs, output, 1, lambda i: [i[0]])
    ctx.params, ctx.mode = inputs[1], inputs[2]


def _block_bwd(ctx, grads):
    g = grads[0]
    res = torch.ops.vq3d.preact_block_backward(g, ctx.saved, ctx.flags, ctx.params, ctx.mode,
                                               [Fn.grad_buf(p) for p in ctx.params])
    return _grads_of(res, [g])[0], [None] * len(ctx.params), None, None


_register("preact_block", _block_bwd, _block_setup, (0,))


def block(x, blk):
    """Fn.PreActBlockFn through the registered operator."""
    params = list(blk._fn_params)
    return _call("preact_block", (x, params, blk.mode, _save_flag(x, *params)), (x,), params)[0]


@torch.library.custom_op("vq3d::preact_run", mutates_args=())
def preact_run(x: Tensor, params: List[Tensor], kind: str, out_fp32: bool, save: bool) -> List[Tensor]:
    return _forward(_RUNS[kind], 1, [x], (save,), x, _plan(params, out_fp32))


@torch.library.custom_op("vq3d::preact_run_backward", mutates_args=("grads",))
def preact_run_backward(g: Tensor, saved: List[Optional[Tensor]], params: List[Tensor], kind: str, out_fp32: bool,
                        in_dtype: torch.dtype, grads: List[Tensor]) -> List[Tensor]:
    _check_grads(params, grads)
    plan = _plan(params, out_fp32)
    ctx = _Ctx()
    ctx.saved_tensors, ctx.plan, ctx.n_params = tuple(saved), plan, 0
    nb, c = params[8].shape[0], params[8].shape[1]
    if kind == "wide":  # PreActWideFn's per-block image stride and the run's input storage
        ctx.per, ctx.in_dtype = int(L.query("vq3d_preact_wide_image_bytes", c, nb)), in_dtype
    elif kind == "stack":
        b, _, h, w, d = g.shape
        ctx.shape = (b, c, nb, h, w, d)
    return _backward(_RUNS[kind], ctx, [g], (g,))


def _run_setup(ctx, inputs, output):
    _saved(ctx, inputs, output, 1, lambda i: [i[0]])
    ctx.params, ctx.kind, ctx.out_fp32, ctx.in_dtype = inputs[1], inputs[2], inputs[3], inputs[0].dtype


def _run_bwd(ctx, grads):
    g = grads[0]
    res = torch.ops.vq3d.preact_run_backward(g, ctx.saved, ctx.params, ctx.kind, ctx.out_fp32, ctx.in_dtype,
                                             [Fn.grad_buf(p) for p in ctx.params])
    return _grads_of(res, [g])[0], [None] * len(ctx.params), None, None, None


_register("preact_run", _run_bwd, _run_setup, (0,))


def run(fn, x, plan):
    """A run Function (Fn.PreAct{Stack,Wide,MidRun,SmallRun}Fn) through the registered operator."""
    params = [p for b in plan.blocks for p in b._fn_params]
    args = (x, params, RUN_KINDS[fn], plan.out_dtype is torch.float32, _save_flag(x, *params))
    return _call("preact_run", args, (x,), params)[0]


# ------------------------------------------------------------------------------------------------ quantizer
class QuantizerView:
    """The Quantizer attributes the codebook stages read (layers.py:600-634)."""

    def __init__(self, embed, embed_avg, cluster_size, first_pass=None, ema_slot=None, decay=0.0, laplace_alpha=0.0):
        self.embed, self.embed_avg, self.cluster_size, self.first_pass = embed, embed_avg, cluster_size, first_pass
        self.ema_slot, self.decay, self.laplace_alpha = ema_slot, decay, laplace_alpha
        self.num_embeddings, self.embedding_dim = embed.shape


@torch.library.custom_op("vq3d::vq_init", mutates_args=("embed", "embed_avg", "cluster_size", "first_pass"))
def vq_init(z: Tensor, embed: Tensor, embed_avg: Tensor, cluster_size: Tensor, first_pass: Tensor) -> None:
    """The codebook's data-dependent initialisation on the first training pass (layers.py:665-683)."""
    Fn.vq_init(z, QuantizerView(embed, embed_avg, cluster_size, first_pass))


@torch.library.custom_op("vq3d::vq_nearest", mutates_args=())
def vq_nearest(z: Tensor, embed: Tensor, commitment_cost: float, zst_dtype: Optional[torch.dtype]) -> List[Tensor]:
    """The codebook search: [commitment loss, straight-through output, codes] (layers.py:700-728)."""
    loss, zst, idx = Fn.vq_search(z, embed, commitment_cost, zst_dtype)
    return [loss, zst, idx]


@torch.library.custom_op("vq3d::vq_nearest_backward", mutates_args=())
def vq_nearest_backward(z: Tensor, embed: Tensor, idx: Tensor, coef: float, g_loss: Optional[Tensor],
                        g_zst: Optional[Tensor]) -> Tensor:
    return Fn.vq_backward(z, embed, idx, coef, g_loss, g_zst)


def _vq_setup(ctx, inputs, output):
    z, embed, cc = inputs[0], inputs[1], inputs[2]
    b, d, h, w, dz = z.shape
    ctx.coef = 2.0 * cc / float(b * h * w * dz * d)
    ctx.save_for_backward(z, embed, output[2])
    ctx.mark_non_differentiable(output[2])
    ctx.set_materialize_grads(False)


def _vq_bwd(ctx, grads):
    z, embed, idx = ctx.saved_tensors
    return torch.ops.vq3d.vq_nearest_backward(z, embed, idx, ctx.coef, grads[0], grads[1]), None, None, None


_register("vq_nearest", _vq_bwd, _vq_setup, (0,))


@torch.library.custom_op("vq3d::vq_ema", mutates_args=("embed", "embed_avg", "cluster_size", "ema_slot"))
def vq_ema(z: Tensor, idx: Tensor, embed: Tensor, embed_avg: Tensor, cluster_size: Tensor, ema_slot: Optional[Tensor],
           decay: float, laplace_alpha: float) -> None:
    """EMA statistics of the step's codes (into ema_slot, the encoder's fused all-reduce buffer) or,
    without a slot, statistics + all-reduce + EMA update (layers.py:636-663)."""
    Fn.vq_ema(z, idx, QuantizerView(embed, embed_avg, cluster_size, ema_slot=ema_slot, decay=decay,
                                    laplace_alpha=laplace_alpha))


def quantize(z, q):
    """Fn.QuantizeFn through the registered operators: init (first training pass), search (the
    autograd-registered operator, on the pre-update codebook), EMA statistics."""
    z = ops.as_cl(z)
    if q.training and q.first_pass_host:
        with _BELOW():  # mutating, no autograd formula
            torch.ops.vq3d.vq_init(z.detach(), q.embed, q.embed_avg, q.cluster_size, q.first_pass)
        q.first_pass_host = False
    embed = ops.copy_(torch.empty_like(q.embed), q.embed) if q.training else q.embed
    loss, zst, idx = _call("vq_nearest", (z, embed, float(q.commitment_cost), getattr(q, "zst_dtype", None)), (z,))
    if q.training:
        with _BELOW():
            torch.ops.vq3d.vq_ema(z.detach(), idx, q.embed, q.embed_avg, q.cluster_size, q.ema_slot, float(q.decay),
                                  float(q.laplace_alpha))
    return loss, zst, idx


# ------------------------------------------------------------------------------------------------ parse_input / upsample / loss
@torch.library.custom_op("vq3d::parse_input", mutates_args=())
def parse_input(x: Tensor, weight: Tensor, bias: Tensor, half: torch.dtype) -> List[Tensor]:
    return _forward(Fn.ParseInputFn, 1, [x, weight, bias], (True,), x, weight, bias, half)


@torch.library.custom_op("vq3d::parse_input_backward", mutates_args=("grads",))
def parse_input_backward(g: Tensor, saved: List[Optional[Tensor]], weight: Tensor, bias: Tensor,
                         grads: List[Tensor]) -> List[Tensor]:
    _check_grads((weight, bias), grads)
    ctx = _Ctx()
    ctx.saved_tensors, ctx.params = tuple(saved), (weight, bias)
    return _backward(Fn.ParseInputFn, ctx, [g], (g,))


def _pi_setup(ctx, inputs, output):
    _saved(ctx, inputs, output, 1, lambda i: [i[0], i[1], i[2]])
    ctx.w, ctx.b = inputs[1], inputs[2]


def _pi_bwd(ctx, grads):
    torch.ops.vq3d.parse_input_backward(grads[0], ctx.saved, ctx.w, ctx.b, [Fn.grad_buf(ctx.w), Fn.grad_buf(ctx.b)])
    return None, None, None, None


_register("parse_input", _pi_bwd, _pi_setup, (0, 1, 2))


@torch.library.custom_op("vq3d::upsample2x", mutates_args=())
def upsample2x(x: Tensor) -> Tensor:
    return ops.upsample2x(x)


@torch.library.custom_op("vq3d::upsample2x_backward", mutates_args=())
def upsample2x_backward(g: Tensor, src_shape: List[int]) -> Tensor:
    ctx = _Ctx()
    ctx.shape = tuple(src_shape)
    return Fn.UpsampleFn.backward(ctx, g)


def _up_setup(ctx, inputs, output):
    ctx.shape = list(inputs[0].shape)


def _up_bwd(ctx, g):
    return torch.ops.vq3d.upsample2x_backward(g, ctx.shape)


_register("upsample2x", _up_bwd, _up_setup, (0,))


@torch.library.custom_op("vq3d::recon_loss", mutates_args=())
def recon_loss(dec: Tensor, x: Tensor, nvs: Tensor, cylinder: bool, commit: List[Tensor]) -> List[Tensor]:
    return _forward(Fn.ReconLossFn, 2, [dec, x, nvs], (True,), dec, x, nvs, cylinder, *commit)


@torch.library.custom_op("vq3d::recon_loss_backward", mutates_args=())
def recon_loss_backward(g_total: Tensor, saved: List[Optional[Tensor]], cylinder: bool, ncommit: int) -> List[Tensor]:
    ctx = _Ctx()
    ctx.saved_tensors, ctx.cyl, ctx.ncommit = tuple(saved), int(cylinder), ncommit
    return _backward(Fn.ReconLossFn, ctx, [g_total], (g_total, None))


def _loss_setup(ctx, inputs, output):
    _saved(ctx, inputs, output, 2, lambda i: [i[0], i[1], i[2]])
    ctx.mark_non_differentiable(output[1])  # recon: a logged value (ReconLossFn)
    ctx.cyl, ctx.ncommit = inputs[3], len(inputs[4])


def _loss_bwd(ctx, grads):
    g_total = grads[0]
    gs = _grads_of(torch.ops.vq3d.recon_loss_backward(g_total, ctx.saved, ctx.cyl, ctx.ncommit), [g_total])
    return gs[0], None, None, None, list(gs[4:])


_register("recon_loss", _loss_bwd, _loss_setup, (0, 4))


def upsample(x):
    return _call("upsample2x", (x,), (x,))


def parse_input(x, w, b, half):
    return _call("parse_input", (x, w, b, half), (x, w, b))[0]


def recon_loss(dec, x, nvs, cylinder, *commit):
    return _call("recon_loss", (dec, x, nvs, bool(cylinder), list(commit)), (dec, *commit))[:2]


# ------------------------------------------------------------------------------------------------ fake kernels
# Shape / dtype / stride propagation for tracing (torch.compile, torch.export): every operator has
# a fake implementation.  The forward operators' outputs are [result(s), meta, saved...]: with
# save=False (inference: eval / torch.no_grad, what a traced deployment runs) no intermediate is
# saved and the structure is fixed, [result, meta (3 path flags)].  With save=True the saved set
# depends on the engine the forward picks at run time (tiny / few-channel / mid / per-conv paths),
# so a training-mode forward is not traceable: its fake says so.  The backward operators (called by
# the registered autograd formulas only) return engine-dependent lists too and are likewise
# eager-only.
_CL = torch.channels_last_3d


def _act_like(ref, shape, dtype=None):
    return torch.empty(tuple(shape), dtype=dtype or ref.dtype, device=ref.device).contiguous(memory_format=_CL)


def _meta(ref, nsaved=0):
    return torch.empty(len(_FLAGS) + nsaved, dtype=torch.int64)


def _inference_only(name, save):
    if save:
        raise NotImplementedError(f"vq3d::{name}: a gradient-recording forward saves engine-dependent intermediates "
                                  "and is not traceable; trace the model in eval mode / under torch.no_grad()")


def _eager_only(name):
    def fake(*args, **kw):
        raise NotImplementedError(f"vq3d::{name} runs inside the eager backward only (engine-dependent outputs)")
    return fake


@torch.library.register_fake("vq3d::conv3d")
def _conv3d_fake(x, x2, residual, weight, scale, bias, cbias, pro, geom, residual_up2, post_elu, save):
    _inference_only("conv3d", save)
    k, st, pd, _ = geom
    b, _, h, w, d = x.shape
    out = [(n + 2 * pd - k) // st + 1 for n in (h, w, d)]
    return [_act_like(x, (b, weight.shape[0], *out)), _meta(x)]


@torch.library.register_fake("vq3d::preact_block")
def _preact_block_fake(x, params, mode, save):
    _inference_only("preact_block", save)
    b, _, h, w, d = x.shape
    f = 0.5 if mode == "down" else (2 if mode == "up" else 1)
    return [_act_like(x, (b, params[10].shape[0], int(h * f), int(w * f), int(d * f))), _meta(x)]


@torch.library.register_fake("vq3d::preact_run")
def _preact_run_fake(x, params, kind, out_fp32, save):
    _inference_only("preact_run", save)
    return [_act_like(x, x.shape, torch.float32 if out_fp32 else x.dtype), _meta(x)]


@torch.library.register_fake("vq3d::vq_nearest")
def _vq_nearest_fake(z, embed, commitment_cost, zst_dtype):
    b, _, h, w, d = z.shape
    return [torch.empty((), dtype=torch.float32, device=z.device), _act_like(z, z.shape, zst_dtype or z.dtype),
            torch.empty((b, h, w, d), dtype=torch.int64, device=z.device)]


@torch.library.register_fake("vq3d::vq_nearest_backward")
def _vq_nearest_backward_fake(z, embed, idx, coef, g_loss, g_zst):
    return _act_like(z, z.shape)


@torch.library.register_fake("vq3d::vq_init")
def _vq_init_fake(z, embed, embed_avg, cluster_size, first_pass):
    return None


@torch.library.register_fake("vq3d::vq_ema")
def _vq_ema_fake(z, idx, embed, embed_avg, cluster_size, ema_slot, decay, laplace_alpha):
    return None


@torch.library.register_fake("vq3d::parse_input")
def _parse_input_fake(x, weight, bias, half):
    b, _, h, w, d = x.shape
    return [_act_like(x, (b, weight.shape[0], h, w, d), half), _meta(x, 1)]  # saves x (an input)


@torch.library.register_fake("vq3d::upsample2x")
def _upsample2x_fake(x):
    b, c, h, w, d = x.shape
    return _act_like(x, (b, c, 2 * h, 2 * w, 2 * d))


@torch.library.register_fake("vq3d::upsample2x_backward")
def _upsample2x_backward_fake(g, src_shape):
    return _act_like(g, src_shape)


@torch.library.register_fake("vq3d::recon_loss")
def _recon_loss_fake(dec, x, nvs, cylinder, commit):
    s = torch.empty((), dtype=torch.float32, device=dec.device)
    return [s, torch.empty_like(s), _meta(dec, 3)]  # saves dec, x, nvs (inputs)


for _n in ("conv3d_backward", "preact_block_backward", "preact_run_backward", "parse_input_backward",
           "recon_loss_backward"):
    torch.library.register_fake(f"vq3d::{_n}")(_eager_only(_n))


OPS = ("conv3d", "conv3d_backward", "preact_block", "preact_block_backward", "preact_run", "preact_run_backward",
       "vq_init", "vq_nearest", "vq_nearest_backward", "vq_ema", "parse_input", "parse_input_backward", "upsample2x",
       "upsample2x_backward", "recon_loss", "recon_loss_backward")
