"""PixelSNAIL prior over VQ-VAE codes (reference pixel_model/pixelsnail.py + pixel_model/layers.py),
module API and state_dict of the reference, GPU path through libvq3d:

* the masked k = 3 causal 3-stack convs (CausalConv3dAdd, layers.py:122-222) run on the
  hand-written conv engines (conv3d.hip): the (k-1, k, k) depth, (1, k-1, k) height and
  (1, 1, k//2 + 1) width kernels are embedded in a zero-padded k^3 kernel whose dead taps are
  exactly zero, so the causal front padding becomes the engines' symmetric zero padding; the
  PreAct pre-activation elu(x + a) + b runs as the conv's fused prologue;
* the 1x1x1 convs (branch 1 / 3, expand_rf, the attention projections, skip / aux, parse_input /
  parse_output) are plain GEMMs over the voxel rows of the channels-last tensors: hipBLASLt via
  torch.nn.functional.linear (mask 'A' shifts its pre-activated input by one position first);
* the dense causal attention (CausalAttention, layers.py:613-647) is attention.hip: no n x n
  logits, fp32 online softmax, recomputing backward;
* elementwise glue (shifts, residual adds, ELU of the attention aux input, Dropout3d, the
  cross-entropy) is plain torch on the same stream.

A stack is the reference's (3, b, c, d, h, w) tensor (depth-, height-, width-wise streams); inside
the model it travels as a list of three channels-last (b, c, d, h, w) tensors.  Dropout: the
causal Dropout3d runs per stream as in the reference; the attention's training-mode logits
(dropout, then zero logits -> -1e3, layers.py:633-637) are computed inside the attention kernels
from a device seed (CausalAttentionFn).  Mixup (pixelsnail.py:136-138, train_helpers.py:20-63)
blends the one-hot inputs and the two targets' losses as the reference does.
"""
import contextlib
import ctypes
import math
from random import randrange
from argparse import ArgumentParser, Namespace
from functools import partial
from operator import attrgetter

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import _lib as L
from . import ops
from .ops import ConvGeom

CL = torch.channels_last_3d


def cl(t):
    return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)


def _zeros_like(t):
    return ops.zero_(torch.empty_like(t))


def _is_param(p):
    return isinstance(p, nn.Parameter) and p.is_leaf


def _param_grad(p):
    """the gradient buffer a kernel may add into directly: a leaf parameter's own .grad (the flat
    buffer's view); anything else gets a zeroed temporary that autograd then accumulates"""
    if _is_param(p):
        from .functional import grad_buf
        return grad_buf(p)
    return _zeros_like(p)


# the conv operand dtype of the model being run (PixelSNAIL.logits sets it): the residual streams
# stay fp32 between blocks as under the reference's fp16 autocast (`out * self.scale` with the
# fp32 parameter promotes, layers.py:463-465); every conv reads its operand in this dtype
_compute = [torch.float32]


def _operand(x):
    return cl(x if x.dtype == _compute[0] else x.to(_compute[0]))


def _fused_glue():
    """16-bit runs put the block glue on the libvq3d kernels below; fp32 runs (the exact-parity
    path against the reference goldens) keep torch's elementwise ops"""
    return _compute[0] != torch.float32


# ---- lanes: 16-bit GPU runs put the three stack streams (depth / height / width) on three HIP
# streams.  The streams meet only in ExpandRFConv (height and width add projections of the depth
# / height branches) and at the output, so each stream's chain of small kernels runs concurrently
# with the other two's; autograd runs every backward op on its forward's stream and synchronises
# the gradient hand-offs between them.
#
# The one-element parameters (the blocks' bias1a .. bias4, scale) are shared by the three streams:
# their gradient sums would be added into the same address from three streams at once.  Under
# lanes each lane adds into its own row of a [3][n] buffer and one callback at the end of the
# backward adds the rows in lane order into the gradients: race-free and deterministic.
_lanes_on = [False]  # off: a captured lanes step's gradients differ between replays
_LANES = [None]
_CUR = [0]       # the lane the current code runs on
_LSTATE = [None]  # the forward's _LaneGrads


def set_lanes(enabled="graph"):
    """per-stack-stream HIP streams in 16-bit GPU runs: "graph" inside HIP-graph captures only, True
    also in eager runs, False never (the default: see DESIGN.md 9 -- a captured lanes step's
    gradients differ between replays, a cross-stream race not yet found)"""
    _lanes_on[0] = enabled if enabled == "graph" else bool(enabled)


@contextlib.contextmanager
def _lane(i):
    """run on stream i's lane (no stream switch without lanes)"""
    lanes = _LANES[0]
    prev = _CUR[0]
    _CUR[0] = i
    try:
        if lanes is None:
            yield
        else:
            with torch.cuda.stream(lanes[i]):
                yield
    finally:
        _CUR[0] = prev


class _LaneGrads:
    """per-lane gradient rows of the shared one-element parameters of one forward"""

    def __init__(self, params, lanes, device):
        self.params = params
        self.slot = {id(p): j for j, p in enumerate(params)}
        self.lanes = lanes
        self.buf = torch.zeros((3, max(1, len(params))), dtype=torch.float32, device=device)
        self.queued = False

    def row(self, lane, p):
        """lane's gradient slot of p (queues the flush of this backward on first use)"""
        if not self.queued:
            self.queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self.flush)
        j = self.slot[id(p)]
        return self.buf[lane, j:j + 1]

    def flush(self):
        """on the forward's main lane (the callback may run on autograd's device thread, whose
        current stream is not the caller's): wait for the other lanes, add the rows in order"""
        from .functional import grad_buf
        main = self.lanes[0]
        with torch.cuda.stream(main):
            for s in self.lanes[1:]:
                main.wait_stream(s)
            sums = self.buf.sum(0).view(-1, 1)
            torch._foreach_add_([grad_buf(p) for p in self.params], list(sums[:len(self.params)].unbind()))
        self.queued = False


def _lane_ctx():
    """(the forward's _LaneGrads, this op's lane) for an autograd Function's ctx, or None"""
    st = _LSTATE[0]
    return None if st is None else (st, _CUR[0])


def _sgrad(lst, p):
    """the buffer a kernel adds p's gradient into: the lane row of a shared one-element parameter
    under lanes, else _param_grad(p)"""
    if lst is not None and id(p) in lst[0].slot:
        return lst[0].row(lst[1], p)
    return _param_grad(p)



class _Handoff(torch.autograd.Function):
    """a tensor crossing from lane j to lane i (applied on lane i).  Backward runs on lane i and hands
    the gradient back to lane j: the gradient's memory (allocated on lane i) is recorded on lane j,
    so the allocator cannot give it to lane i's next allocation while lane j still reads it (the
    cross-stream reuse hazard autograd leaves to the caller)."""

    @staticmethod
    def forward(ctx, t, src):
        ctx.src = src
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        if g is not None:
            g.record_stream(ctx.src)
        return g, None


def _take(i, j, *ts):
    """lane i is about to use tensors made on lane j: it waits for lane j's work so far, the
    allocator keeps the tensors' memory until lane i's use is done, and the tensors that need a
    gradient come back wrapped in _Handoff (their gradients cross back to lane j).  Returns the
    tensors (unchanged without lanes)."""
    lanes = _LANES[0]
    if lanes is None or i == j:
        return ts if len(ts) != 1 else ts[0]
    lanes[i].wait_stream(lanes[j])
    out = []
    with torch.cuda.stream(lanes[i]):
        for t in ts:
            if t is not None:
                t.record_stream(lanes[i])
                if t.requires_grad:
                    t = _Handoff.apply(t, lanes[j])
            out.append(t)
    return out if len(out) != 1 else out[0]


class PreActFn(torch.autograd.Function):
    """elu(x + a) + b straight into the conv operand format (layers.py:425-432 pre-activation +
    the autocast of the conv input): one launch; backward one launch with the a / b gradient sums
    added into the parameters' gradient buffers (fixed order)."""

    @staticmethod
    def forward(ctx, x, a, b):
        x = cl(x)
        y = torch.empty_like(x, dtype=_compute[0], memory_format=CL)
        L.call("vq3d_preact_act_fwd", L.dtype_code(x), L.dtype_code(y), x.numel(), L.ptr(x), L.ptr(a), L.ptr(b),
               L.ptr(y), L.stream())
        ctx.save_for_backward(x)
        ctx.prm = (a, b)
        ctx.lst = _lane_ctx()
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        a, b = ctx.prm
        g = cl(g)
        gx = torch.empty_like(x, memory_format=CL) if ctx.needs_input_grad[0] else None
        da, db = _sgrad(ctx.lst, a), _sgrad(ctx.lst, b)
        L.call("vq3d_preact_act_bwd", L.dtype_code(g), L.dtype_code(x), x.numel(), L.ptr(g), L.ptr(x), L.ptr(a),
               None if gx is None else L.ptr(gx), L.ptr(da), L.ptr(db), L.stream())
        return gx, None if _is_param(a) else da, None if _is_param(b) else db


class ScaleBiasResFn(torch.autograd.Function):
    """out = o * scale + bias4 + skip (layers.py:463-465, fp32 as the 1-element fp32 parameters
    promote): one launch; backward one launch (go = g * scale and the two sums), skip's gradient g."""

    @staticmethod
    def forward(ctx, o, scale, bias, s):
        o, s = cl(o), cl(s)
        if s.dtype != torch.float32:
            s = s.float().contiguous(memory_format=CL)
        out = torch.empty_like(o, dtype=torch.float32, memory_format=CL)
        L.call("vq3d_scale_bias_res_fwd", L.dtype_code(o), o.numel(), L.ptr(o), L.ptr(scale), L.ptr(bias), L.ptr(s),
               L.ptr(out), L.stream())
        ctx.save_for_backward(o)
        ctx.prm = (scale, bias)
        ctx.lst = _lane_ctx()
        return out

    @staticmethod
    def backward(ctx, g):
        (o,) = ctx.saved_tensors
        scale, bias = ctx.prm
        g = cl(g).float()
        go = torch.empty_like(o, memory_format=CL) if ctx.needs_input_grad[0] else None
        ds, dbi = _sgrad(ctx.lst, scale), _sgrad(ctx.lst, bias)
        L.call("vq3d_scale_bias_res_bwd", L.dtype_code(o), o.numel(), L.ptr(g), L.ptr(o), L.ptr(scale),
               None if go is None else L.ptr(go), L.ptr(ds), L.ptr(dbi), L.stream())
        return (go, None if _is_param(scale) else ds, None if _is_param(bias) else dbi,
                (g if ctx.needs_input_grad[3] else None))


def _preact(x, pro):
    """the conv operand of elu(x + a) + b"""
    if _fused_glue():
        return PreActFn.apply(x, pro[0], pro[1])
    return _operand(F.elu(x + pro[0]) + pro[1])


# ============================================================================================ conv
class CausalConvFn(torch.autograd.Function):
    """y = conv(prologue(x), w) + cbias on the libvq3d engines; w is the (embedded) k^3 weight.
    Gradients of w / cbias / the prologue scalars come back as tensors (torch autograd maps them
    onto the reference-shaped parameters through the embedding)."""

    @staticmethod
    def forward(ctx, x, w, cbias, pa, pb, k, taps=0):
        geom = ConvGeom(k, 1, k // 2, False)
        pro = None if pa is None else (pa, pb)
        y = ops.conv_fwd(x, w, geom, pro=pro, cbias=cbias, taps=taps)
        ctx.geom, ctx.pro, ctx.taps = geom, pro, taps
        ctx.lst = _lane_ctx()
        ctx.has_bias = cbias is not None
        ctx.cbias = cbias
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = cl(g)
        dw = _zeros_like(w)
        # the conv bias and the prologue scalars are parameters themselves: their sums go straight
        # into their gradient buffers (the kernels add), no zeroed temporaries and accumulations
        dcb = da = db = None
        if ctx.has_bias:
            dcb = _sgrad(ctx.lst, ctx.cbias)
        if ctx.pro is not None:
            da, db = _sgrad(ctx.lst, ctx.pro[0]), _sgrad(ctx.lst, ctx.pro[1])
        gx, _ = ops.conv_bwd(g, x, w, ctx.geom, pro=ctx.pro, aux=x, want_gx=ctx.needs_input_grad[0], dw=dw,
                             dcbias=dcb, dpro_pre=db, dpro_post=da, taps=ctx.taps)
        return (gx, dw, None if dcb is None or _is_param(ctx.cbias) else dcb,
                None if da is None or _is_param(ctx.pro[0]) else da,
                None if db is None or _is_param(ctx.pro[1]) else db, None, None)


# the 16-bit weight shadow of the current forward: (FlatParams, dtype) when the parameters live in
# a flat buffer (PixelSNAIL.logits refreshes it once per forward), else None (per-call casts)
_shadow = [None]


def _w16(p, dtype):
    """parameter p as a GEMM operand of dtype: its slice of the refreshed flat shadow, or a cast"""
    sh = _shadow[0]
    if sh is not None and sh[1] == dtype and p.dtype == torch.float32 and sh[0].owns(p):
        return sh[0].shadow_view(p, dtype)
    return p.to(dtype)


def _rows_ok(t):
    return (t.dtype in (torch.bfloat16, torch.float16) and t.dim() == 2 and t.stride(1) == 1
            and t.shape[1] % 8 == 0 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0)


class PointwiseFn(torch.autograd.Function):
    """1x1x1 conv of a channels-last (b, c, d, h, w) tensor as GEMMs over its voxel rows
    (hipBLASLt, fp32 accumulation) for y and gx.  The weight gradient sum_v g[v] (x) x[v] has the
    voxels as its K dimension and only co x ci outputs: on 16-bit rows it is vq3d_rows_wgrad
    (matrix cores, split K, fixed-order sum, bias sums included) adding straight into the
    parameters' gradient buffers; fp32 rows (the reference-parity path) run a batched fp32 GEMM over
    256-voxel slices plus one sum over the slices."""

    @staticmethod
    def forward(ctx, x, w, b):
        xv = x.permute(0, 2, 3, 4, 1).reshape(-1, x.shape[1])
        w2 = _w16(w, x.dtype).reshape(w.shape[0], -1)
        y = F.linear(xv, w2, None if b is None else _w16(b, x.dtype))
        ctx.save_for_backward(xv, w2)
        ctx.shape = (x.shape[0],) + tuple(x.shape[2:])
        ctx.prm = (w, b)
        return y.reshape(ctx.shape + (w.shape[0],)).permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        xv, w2 = ctx.saved_tensors
        w, b = ctx.prm
        co = w2.shape[0]
        gv = g.permute(0, 2, 3, 4, 1).reshape(-1, co)
        if not gv.is_contiguous():
            gv = gv.contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            gx = (gv @ w2.to(gv.dtype)).reshape(ctx.shape + (w2.shape[1],)).permute(0, 4, 1, 2, 3)
        n = gv.shape[0]
        if gv.dtype == xv.dtype and _rows_ok(gv) and _rows_ok(xv):
            dw = _param_grad(w)
            db = None if b is None else _param_grad(b)
            nws = int(L.query("vq3d_rows_wgrad_workspace_bytes", n, co, xv.shape[1]))
            ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=gv.device)
            L.call("vq3d_rows_wgrad", L.dtype_code(gv), n, co, xv.shape[1], L.ptr(gv), gv.stride(0), L.ptr(xv),
                   xv.stride(0), L.ptr(dw), L.ptr(db), L.ptr(ws), ctypes_size(nws), L.stream())
            return gx, None if _is_param(w) else dw, None if b is None or _is_param(b) else db
        sk = 256 if n % 256 == 0 and n >= 4096 else n
        gw = torch.bmm(gv.reshape(-1, sk, co).transpose(1, 2).float(), xv.reshape(-1, sk, xv.shape[1]).float()).sum(0)
        gb = gv.float().sum(0) if b is not None else None
        return gx, gw.reshape(w.shape), gb


def pointwise(x, w, b):
    return PointwiseFn.apply(x, w, b)


def _embed(depth_w, height_w, width_w, k):
    """the three causal kernels inside k^3 kernels (k = 3): taps the reference never reads are 0.
    depth (k-1, k, k) at kd = 0 .. k-2 (front pad k-2 = offsets -1, 0); height (1, k-1, k) at
    kd = 1, kh = 0 .. k-2; width (1, 1, wk) at kd = kh = 1, kw = 0 .. wk-1."""
    return tuple(_embed_one(i, w, k) for i, w in enumerate((depth_w, height_w, width_w)))


def _embed_one(i, w, k):
    """stream i's kernel of _embed"""
    if k == 1:
        return w
    if i == 0:
        return F.pad(w, (0, 0, 0, 0, 0, 1))
    if i == 1:
        return F.pad(w, (0, 0, 0, 1, 1, 1))
    return F.pad(w, (0, 3 - w.shape[-1], 1, 1, 1, 1))


def _tap_mask(stream, k, wk):
    """vq3d_conv_desc.tap_mask of the embedded kernel of stream 0 / 1 / 2 (_embed): bit
    (i0*k + i1)*k + i2 for the taps the causal kernel occupies; the conv engines skip the others"""
    live = {0: lambda a, b, c: a <= k - 2,
            1: lambda a, b, c: a == 1 and b <= k - 2,
            2: lambda a, b, c: a == 1 and b == 1 and c < wk}[stream]
    return sum(1 << ((a * k + b) * k + c) for a in range(k) for b in range(k) for c in range(k) if live(a, b, c))


def _shift(t, axis):
    """front-pad spatial axis (0 = d, 1 = h, 2 = w) by one and drop the last slice (the mask 'A'
    shifts, layers.py:13-100)"""
    pad = [0, 0, 0, 0, 0, 0]
    pad[2 * (2 - axis)] = 1
    t = F.pad(t, tuple(pad))
    sl = [slice(None)] * 5
    sl[2 + axis] = slice(0, -1)
    return cl(t[tuple(sl)])


class CausalConv3dAdd(nn.Module):
    """layers.py:122-222 (parameters: depth_conv / height_conv / width_conv nn.Conv3d)."""

    def __init__(self, mask: str = "B", **conv_kwargs):
        super().__init__()
        assert "padding" not in conv_kwargs
        assert mask in ("A", "B")
        self.mask = mask
        kernel_size = conv_kwargs.pop("kernel_size")
        assert kernel_size > 0 and kernel_size % 2 == 1, "even kernel sizes are not supported"
        if conv_kwargs.get("groups", 1) != 1:
            raise NotImplementedError("grouped causal convs (concat_activation) are not implemented")
        self.kernel_size = kernel_size
        depth_size = max(kernel_size - 1, 1)
        height_size = max(kernel_size - 1, 1)
        width_size = max(kernel_size // 2 + (1 if mask == "B" else 0), 1)
        self.depth_conv = nn.Conv3d(kernel_size=(depth_size, kernel_size, kernel_size), **conv_kwargs)
        self.height_conv = nn.Conv3d(kernel_size=(1, height_size, kernel_size), **conv_kwargs)
        self.width_conv = nn.Conv3d(kernel_size=(1, 1, width_size), **conv_kwargs)

    def run(self, stack, pro=None):
        """stack: list of 3 channels-last tensors; pro = (a, b): every input goes through
        elu(x + a) + b first (fused as the conv prologue unless mask 'A' has to shift it).
        Stream i runs on its lane."""
        out = []
        for i, x in enumerate(stack):
            with _lane(i):
                out.append(self.run_one(i, x, pro))
        return out

    def run_one(self, i, x, pro=None):
        """stream i (0 depth, 1 height, 2 width) of run, on the current stream"""
        k = self.kernel_size
        if k not in (1, 3):
            raise NotImplementedError("causal conv kernel sizes 1 and 3 (the reference's default) are supported")
        conv = (self.depth_conv, self.height_conv, self.width_conv)[i]
        w, b = _embed_one(i, conv.weight, k), conv.bias
        if k == 1:  # a plain GEMM over the voxels (hipBLASLt): pre-activation + shift as glue
            x = _operand(x) if pro is None else _preact(x, pro)
            if self.mask == "A":
                x = _shift(x, i)
            return pointwise(x, w, b)
        pa = pb = None
        if self.mask == "A":
            x = _shift(_operand(x) if pro is None else _preact(x, pro), i)
        elif pro is not None:
            pa, pb = pro
        return CausalConvFn.apply(_operand(x), w, b, pa, pb, k, _tap_mask(i, k, self.width_conv.weight.shape[-1]))

    def forward(self, stack):
        return torch.stack(self.run(to_list(stack)))


def to_list(stack):
    if isinstance(stack, (list, tuple)):
        return [cl(s) for s in stack]
    return [cl(stack[i]) for i in range(3)]


class ExpandRFConv(nn.Module):
    """layers.py:225-248"""

    def __init__(self, in_channels):
        super().__init__()
        self.depth_conv = nn.Conv3d(in_channels=in_channels, out_channels=in_channels * 2, kernel_size=1)
        self.height_conv = nn.Conv3d(in_channels=in_channels, out_channels=in_channels, kernel_size=1)

    def run(self, stack):
        d, h, w = stack
        # on lane 0 (the lanes only ever synchronise with lane 0: side-to-side waits inside a
        # captured multi-stream backward crash hipStreamEndCapture on this ROCm)
        with _lane(0):
            h = _take(0, 1, h)
            w = _take(0, 2, w)
            dc = pointwise(_operand(d), self.depth_conv.weight, self.depth_conv.bias)
            dch, dcw = torch.chunk(dc, 2, dim=1)
            hc = pointwise(_operand(h), self.height_conv.weight, self.height_conv.bias)
            h2 = cl(h + dch)
            w2 = cl(w + hc + dcw)
        return [d, _take(1, 0, h2), _take(2, 0, w2)]

    def forward(self, stack):
        return torch.stack(self.run(to_list(stack)))


def _dropout3d(stack, mod):
    if mod is None or not mod.training or mod.p == 0:
        return stack
    return [cl(F.dropout3d(s, mod.p, True)) for s in stack]


class PreActFixupCausalResBlock(nn.Module):
    """layers.py:338-497"""

    def __init__(self, in_channels, out_channels, kernel_size, mask="B", condition_dim=0, condition_kernel_size=1,
                 activation=nn.ELU, dropout_prob=0.5, bottleneck_divisor=4, concat_activation=False, aux=False,
                 *args, **kwargs):
        super().__init__()
        if concat_activation:
            # the reference cannot run this variant either: ExpandRFConv(branch_channels * 2)
            # (pixel_model/layers.py:399) receives branch_conv1's branch_channels outputs (:370-377,
            # :432), so its forward raises "expected input ... to have 2B channels, but got B"
            raise NotImplementedError("concat_activation: the reference's forward fails on it (ExpandRFConv "
                                      "channel mismatch, pixel_model/layers.py:399,432)")
        self.bias1a, self.bias1b, self.bias2a, self.bias2b, self.bias3a, self.bias3b, self.bias4 = (
            nn.Parameter(torch.zeros(1)) for _ in range(7))
        self.scale = nn.Parameter(torch.ones(1))
        groups = 1
        branch_channels = max(max(in_channels, out_channels) // bottleneck_divisor, groups)
        self.branch_conv1 = CausalConv3dAdd(in_channels=in_channels * groups, out_channels=branch_channels,
                                            kernel_size=1, mask=mask, bias=False, groups=groups)
        self.branch_conv2 = CausalConv3dAdd(in_channels=branch_channels * groups, out_channels=branch_channels,
                                            kernel_size=kernel_size, mask="B", bias=False, groups=groups)
        self.branch_conv3 = CausalConv3dAdd(in_channels=branch_channels * groups, out_channels=out_channels,
                                            kernel_size=1, mask="B", bias=False, groups=groups)
        self.expand_rf = ExpandRFConv(branch_channels * groups)
        self.skip_conv = CausalConv3dAdd(in_channels=in_channels, out_channels=out_channels, kernel_size=1,
                                         mask=mask, bias=True) if (in_channels != out_channels or mask == "A") else None
        self.condition = nn.Conv3d(in_channels=condition_dim, out_channels=branch_channels,
                                   kernel_size=condition_kernel_size, padding=condition_kernel_size // 2,
                                   bias=True) if condition_dim > 0 else None
        self.aux = CausalConv3dAdd(in_channels=branch_channels, out_channels=branch_channels, kernel_size=1,
                                   bias=True) if aux else None
        self.activation = activation()
        self.dropout = nn.Dropout3d(dropout_prob) if dropout_prob > 0 else None

    def run(self, stack, aux=None):
        """each stream on its lane; the streams meet in expand_rf"""
        out = self.branch_conv1.run(stack, pro=(self.bias1a, self.bias1b))
        out = self.expand_rf.run(out)
        res = []
        for i in range(3):
            with _lane(i):
                o = out[i]
                if aux is not None:
                    assert self.aux is not None
                    o = cl(o + self.aux.run_one(i, cl(F.elu(aux[i]))))
                o = self.branch_conv2.run_one(i, o, pro=(self.bias2a, self.bias2b))
                o = _dropout3d([o], self.dropout)[0]
                o = self.branch_conv3.run_one(i, o, pro=(self.bias3a, self.bias3b))
                s = stack[i] if self.skip_conv is None else self.skip_conv.run_one(i, stack[i])
                # o * scale + bias4 + skip: fp32 (the 1-element fp32 parameters promote, as in the reference)
                if _fused_glue():
                    res.append(ScaleBiasResFn.apply(o, self.scale, self.bias4, s))
                else:
                    res.append(cl(o * self.scale + self.bias4 + s))
        return res

    def forward(self, stack, aux=None, condition=None, condition_cache=None):
        if condition is not None or condition_cache is not None:
            raise NotImplementedError("conditioning (use_conditioning) is not implemented")
        return torch.stack(self.run(to_list(stack), None if aux is None else to_list(aux)))

    @torch.no_grad()
    def initialize_weights(self, num_layers):
        """layers.py:469-497 (same init calls in the same order)"""
        getter = attrgetter("depth_conv.weight", "height_conv.weight", "width_conv.weight")
        for weight in getter(self.branch_conv1):
            torch.nn.init.normal_(weight, mean=0,
                                  std=np.sqrt(2 / (weight.shape[0] * np.prod(weight.shape[2:]))) * num_layers ** (-0.5))
        for weight in getter(self.branch_conv2):
            torch.nn.init.kaiming_normal_(weight)
        for weight in getter(self.branch_conv3):
            torch.nn.init.constant_(weight, val=0)
        if self.skip_conv is not None:
            for weight in getter(self.skip_conv):
                torch.nn.init.xavier_normal_(weight)
            for bias in attrgetter("depth_conv.bias", "height_conv.bias", "width_conv.bias")(self.skip_conv):
                torch.nn.init.constant_(tensor=bias, val=0)


# ============================================================================================ attention
class CausalAttentionFn(torch.autograd.Function):
    """One stream's causal attention (attention.hip): q, k [b][n][nh * dk], v [b][n][nh * dv].
    train: None (eval) or (dropout p, device int64 seed tensor of this forward): the reference's
    training-mode logits (layers.py:633-637) -- dropout, then every zero logit -> -1e3 -- with the
    drop mask a hash of the seed that the backward recomputes."""

    @staticmethod
    def forward(ctx, q, k, v, nh, train=None):
        b, ck = q.shape[:2]
        n = math.prod(q.shape[2:])
        cv = v.shape[1]
        dk, dv = ck // nh, cv // nh
        scale = float(dk) ** -0.5
        q, k, v = (t.contiguous(memory_format=CL) for t in (q, k, v))
        out = torch.empty_like(v, memory_format=CL)
        lse = torch.empty((b, nh, n), dtype=torch.float32, device=q.device)
        tr, seed = _attn_train(train)
        L.call("vq3d_causal_attn_fwd_ex", L.dtype_code(q), b, n, nh, dk, dv, scale, L.ptr(q), L.ptr(k), L.ptr(v),
               None if tr is None else ctypes.byref(tr), L.ptr(out), L.ptr(lse), L.stream())
        ctx.dims = (b, n, nh, dk, dv, scale)
        ctx.train = None if train is None else (train[0], seed)
        ctx.save_for_backward(q, k, v, out, lse)
        return out

    @staticmethod
    def backward(ctx, g):
        q, k, v, out, lse = ctx.saved_tensors
        b, n, nh, dk, dv, scale = ctx.dims
        g = cl(g)
        gq, gk, gv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        nws = int(L.query("vq3d_causal_attn_workspace_bytes", b, n, nh))
        ws = torch.empty(max(nws, 4), dtype=torch.uint8, device=q.device)
        tr, _ = _attn_train(ctx.train)
        L.call("vq3d_causal_attn_bwd_ex", L.dtype_code(q), b, n, nh, dk, dv, scale, L.ptr(q), L.ptr(k), L.ptr(v),
               None if tr is None else ctypes.byref(tr), L.ptr(out), L.ptr(g), L.ptr(lse), L.ptr(ws),
               ctypes_size(nws), L.ptr(gq), L.ptr(gk), L.ptr(gv), L.stream())
        return gq, gk, gv, None, None


def _attn_train(train):
    """(vq3d_attn_train struct or None, the seed tensor kept alive)"""
    if train is None:
        return None, None
    p, seed = train
    return L.AttnTrain(dropout_p=float(p), seed=None if seed is None else ctypes.c_void_p(seed.data_ptr())), seed


def ctypes_size(n):
    import ctypes
    return ctypes.c_size_t(int(n))


class CausalAttention(nn.Module):
    """layers.py:613-647.  Parameter names as the reference's forward: the caller
    (CausalAttentionPixelBlock, layers.py:694) passes its projected queries as `keys` and its keys
    as `queries`, and the logits are `queries`^T `keys` -- reproduced exactly."""

    def __init__(self, dropout_prob=0.5, num_heads=8):
        super().__init__()
        self.num_heads = num_heads
        self.dropout = nn.Dropout(dropout_prob)

    def _seeds(self, device):
        """one fresh device seed per stream and forward: a device counter advanced by a device add,
        so a captured HIP graph draws new dropout masks on every replay"""
        if getattr(self, "_seed", None) is None or self._seed.device != device:
            base = int(torch.randint(0, 2 ** 62, (1,)).item())
            self._seed = torch.tensor([base], dtype=torch.int64, device=device)
        seeds = self._seed * 3 + torch.arange(3, dtype=torch.int64, device=device)
        self._seed.add_(1)
        return [seeds[i:i + 1] for i in range(3)]

    def run(self, keys, queries, values):
        """stream i on its lane (the training seeds are drawn on lane 0)"""
        nh = self.num_heads
        assert values[0].shape[1] % nh == 0 and keys[0].shape[1] % nh == 0
        train = [None] * 3
        if self.dropout.training:
            p = float(self.dropout.p)
            with _lane(0):
                seeds = self._seeds(keys[0].device) if p > 0 else [None] * 3
            train = [(p, sd) for sd in seeds]
        out = []
        for i, (q, k, v) in enumerate(zip(queries, keys, values)):
            with _lane(i):
                if train[i] is not None and train[i][1] is not None:
                    _take(i, 0, train[i][1])
                out.append(CausalAttentionFn.apply(cl(q), cl(k), cl(v), nh, train[i]))
        return out

    def forward(self, keys, queries, values, attn_mask=None):
        return torch.stack(self.run(to_list(keys), to_list(queries), to_list(values)))


class CausalAttentionPixelBlock(nn.Module):
    """layers.py:650-703 (attn_mask: the kernels implement the tril mask the reference generates)."""

    def __init__(self, in_channels, bottleneck_divisor, num_layers, causal_conv, num_heads=8,
                 attention_dropout_prob=0.5):
        super().__init__()
        branch_channels = in_channels // bottleneck_divisor
        self.key_value_proj = CausalConv3dAdd(in_channels=(in_channels * 2 + 3), out_channels=(branch_channels * 2),
                                              kernel_size=1)
        self.query_proj = CausalConv3dAdd(in_channels=(in_channels + 3), out_channels=branch_channels, kernel_size=1)
        self.causal_layers = nn.ModuleList([causal_conv() for _ in range(num_layers)])
        self.causal_attention = CausalAttention(dropout_prob=attention_dropout_prob, num_heads=num_heads)
        self.out_proj = causal_conv(aux=True)

    def run(self, stack, bg):
        out = stack
        for layer in self.causal_layers:
            out = layer.run(out)
        keys, values, queries = [], [], []
        for i in range(3):
            with _lane(i):
                kv = self.key_value_proj.run_one(i, cl(torch.cat([stack[i], out[i], bg[i]], dim=1)))
                k, v = torch.chunk(kv, 2, dim=1)
                keys.append(k)
                values.append(v)
                queries.append(self.query_proj.run_one(i, cl(torch.cat([out[i], bg[i]], dim=1))))
        att = self.causal_attention.run(queries, keys, values)
        return self.out_proj.run(out, aux=att)

    def forward(self, stack, background, attn_mask=None, condition=None, condition_cache=None):
        if condition is not None or condition_cache is not None:
            raise NotImplementedError("conditioning (use_conditioning) is not implemented")
        return torch.stack(self.run(to_list(stack), to_list(background)))


# ============================================================================================ model
def background_list(b, dims, dtype, device):
    """_generate_background (pixelsnail.py:283-293) per stream: the (d, h, w) linspace grids."""
    d, h, w = dims
    g = torch.cat([
        torch.linspace(-1, 1, d, device=device).view(1, 1, -1, 1, 1).expand(b, 1, d, h, w),
        torch.linspace(-1, 1, h, device=device).view(1, 1, 1, -1, 1).expand(b, 1, d, h, w),
        torch.linspace(-1, 1, w, device=device).view(1, 1, 1, 1, -1).expand(b, 1, d, h, w),
    ], dim=1).to(dtype)
    g = cl(g)
    return [g, g, g]


class PixelSNAIL(nn.Module):
    """pixel_model/pixelsnail.py:27-320 (module tree, argument parsing, init and loss of the
    reference; mixup as train_helpers.py:20-63.  Conditioning is not implemented: the published prior
    runs disable it (train_pixelsnail_*.job: --use-conditioning False) and the reference's own
    conditioned forward passes the condition tensor as `condition_cache` (layers.py:692), whose
    `.popleft()` (layers.py:446) fails, so there is no working reference behaviour to match)."""

    def __init__(self, args, compute_dtype="bf16"):
        super().__init__()
        self._parse_input_args(args)
        self.compute_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(compute_dtype, torch.float32)
        self.parse_input = nn.Conv3d(in_channels=self.input_dim, out_channels=self.model_dim, kernel_size=1)
        condition_dim = self.model_dim if self.use_conditioning else 0
        self.embed_condition = nn.Conv3d(in_channels=self.condition_dim, out_channels=condition_dim,
                                         kernel_size=1) if self.use_conditioning else None
        causal_conv = partial(PreActFixupCausalResBlock, in_channels=self.model_dim, out_channels=self.model_dim,
                              kernel_size=self.kernel_size, dropout_prob=self.causal_dropout_prob,
                              condition_dim=condition_dim, condition_kernel_size=1,
                              bottleneck_divisor=self.bottleneck_divisor)
        self.to_causal = causal_conv(mask="A")
        self.layers = nn.ModuleList([
            CausalAttentionPixelBlock(in_channels=self.model_dim, bottleneck_divisor=self.bottleneck_divisor,
                                      causal_conv=partial(causal_conv, mask="B"),
                                      num_layers=self.num_layers_per_block,
                                      attention_dropout_prob=self.attention_dropout_prob)
            for _ in range(self.num_blocks)])
        self.parse_output = nn.Conv3d(in_channels=self.model_dim, out_channels=self.input_dim, kernel_size=1)
        num_layers = self.num_blocks * self.num_layers_per_block + 1
        self.apply(lambda layer: layer.initialize_weights(num_layers=num_layers)
                   if isinstance(layer, PreActFixupCausalResBlock) else None)

    def _parse_input_args(self, args: Namespace):
        args.use_gated_block = False
        self.input_dim, self.condition_dim = args.num_embeddings
        if not args.use_conditioning:
            self.condition_dim = 0
        for name in ("model_dim", "kernel_size", "num_layers_per_block", "num_blocks", "causal_dropout_prob",
                     "attention_dropout_prob", "bottleneck_divisor", "use_conditioning", "mixup_alpha"):
            setattr(self, name, getattr(args, name))
        if self.use_conditioning:
            raise NotImplementedError("conditioning (use_conditioning) is not implemented")
        if args.metric != "cross_entropy":
            raise ValueError
        self.lr = args.lr

    @classmethod
    def add_model_specific_args(cls, parent_parser):
        """pixelsnail.py:193-217"""
        from .utils import booltype
        parser = ArgumentParser(parents=[parent_parser], add_help=False)
        parser.add_argument("--model-dim", default=32, type=int)
        parser.add_argument("--kernel-size", default=3, type=int)
        parser.add_argument("--num-layers-per-block", default=5, type=int)
        parser.add_argument("--num-blocks", default=5, type=int)
        parser.add_argument("--causal-dropout-prob", default=0.5, type=float)
        parser.add_argument("--attention-dropout-prob", default=0.5, type=float, help="Set to 0 to disable dropout.")
        parser.add_argument("--bottleneck-divisor", default=4, type=int, help="Set to 1 to disable bottlenecking")
        parser.add_argument("--use-conditioning", default=False, type=booltype)
        parser.add_argument("--mixup-alpha", default=0, type=float)
        parser.add_argument("--use-mixup-batch-hack", default=False, type=booltype)
        parser.add_argument("--metric", choices=["cross_entropy"])
        parser.add_argument("--lr", default=1e-5, type=float)
        return parser

    def configure_optimizers(self):
        return torch.optim.Adam(self.parameters(), lr=self.lr, amsgrad=True)

    def logits(self, onehot):
        """forward (pixelsnail.py:301-320) of a one-hot (b, K, d, h, w) input; fp32 logits."""
        b = onehot.shape[0]
        dims = tuple(onehot.shape[2:])
        _compute[0] = self.compute_dtype
        x = cl(onehot.to(self.compute_dtype))
        # the GEMM weights of this forward: one cast of the flat parameter buffer (if there is one)
        _shadow[0] = None
        if self.compute_dtype != torch.float32:
            from .flat import flat_of
            fl = flat_of(self.parse_input.weight)
            if fl is not None:
                fl.refresh_shadow(self.compute_dtype)
                _shadow[0] = (fl, self.compute_dtype)
        x = cl(pointwise(x, self.parse_input.weight, self.parse_input.bias))
        bg = background_list(b, dims, self.compute_dtype, x.device)
        lanes = None
        if _lanes_on[0] and self.compute_dtype != torch.float32 and x.is_cuda:
            # (the lane streams exist before any capture: created on the first eager forward)
            aux = [ops.aux_stream(x.device, "psnail_lane1"), ops.aux_stream(x.device, "psnail_lane2")]
            if _lanes_on[0] is True or torch.cuda.is_current_stream_capturing():
                lanes = [torch.cuda.current_stream()] + aux
        _LANES[0] = lanes
        if lanes is not None:
            shared = [p for p in self.parameters() if p.numel() == 1]
            _LSTATE[0] = _LaneGrads(shared, lanes, x.device)
        try:
            xs = [x] + [_take(i, 0, x, bg[0])[0] for i in (1, 2)]
            stack = self.to_causal.run(xs)
            for layer in self.layers:
                stack = layer.run(stack, bg)
            stack = [stack[0]] + [_take(0, i, stack[i]) for i in (1, 2)]
        finally:
            _LANES[0] = None
            _LSTATE[0] = None
        s = _operand(stack[0] + stack[1] + stack[2])
        return pointwise(s, self.parse_output.weight, self.parse_output.bias).float()

    def forward(self, data, background=None, attn_mask=None, condition=None, condition_cache=None):
        if condition is not None or condition_cache is not None:
            raise NotImplementedError("conditioning (use_conditioning) is not implemented")
        return self.logits(data)

    def cross_entropy(self, batch, batch_idx=0, metrics=None, mode="train"):
        """pixelsnail.py:112-161 without conditioning: mean cross-entropy of the logits over every
        code position (with mixup in training when mixup_alpha != 0), plus the log dict's
        bits_per_dim."""
        codes = batch[0].squeeze(1)
        onehot = F.one_hot(codes, num_classes=self.input_dim).permute(0, 4, 1, 2, 3).float()
        mix = mixup_draw(codes.shape[0], self.mixup_alpha) if (self.mixup_alpha != 0 and mode == "train") else None
        return self.cross_entropy_onehot(onehot, codes, mix)

    def cross_entropy_onehot(self, onehot, codes, mix=None):
        """the loss from a prepared one-hot input (F.one_hot validates its input on the host, which
        a captured HIP graph cannot do).  mix = (lam, index) from mixup_draw: the input is
        lam x + (1 - lam) x[index] and the loss lam CE(y) + (1 - lam) CE(y[index]), averaged
        (train_helpers.py:20-63)."""
        if mix is None:
            logits = self.logits(onehot)
            unreduced = F.cross_entropy(logits, codes, reduction="none")
        else:
            lam, index = mix  # lam a Python float as in the reference (no host-to-device copy: capturable)
            x = onehot.float()
            if torch.equal(index, torch.arange(index.numel())):  # host check (batch 1: always)
                xi, ci = x, codes
            else:
                idx = index.to(x.device)
                xi, ci = x[idx], codes[idx]
            logits = self.logits(lam * x + (1 - lam) * xi)
            unreduced = (lam * F.cross_entropy(logits, codes, reduction="none")
                         + (1 - lam) * F.cross_entropy(logits, ci, reduction="none"))
        loss = unreduced.mean()
        return loss, {"bits_per_dim": loss.detach() / np.log(2)}

    def training_step(self, batch, batch_idx):
        return self.cross_entropy(batch, batch_idx, mode="train")[0]


def sattolo_cycle(n):
    """train_helpers.py:23-37: a random cyclic permutation of range(n) (Sattolo's algorithm on
    Python's global random), so no sample is mixed with itself when n > 1"""
    out = np.arange(n)
    i = n
    while i > 1:
        i -= 1
        j = randrange(i)
        out[j], out[i] = out[i], out[j]
    return out


def mixup_draw(batch_size, alpha):
    """mixup_data's random draws (train_helpers.py:39-47): lam ~ Beta(alpha, alpha) from numpy's
    global generator, then the Sattolo cycle -- the same global RNGs in the same order as the
    reference, so a seeded run draws the same lam / index"""
    lam = float(np.random.beta(alpha, alpha))
    return lam, torch.as_tensor(sattolo_cycle(batch_size))


def default_args(**kw):
    """the reference's argparse defaults (pixelsnail.py:197-216) as a Namespace."""
    a = Namespace(num_embeddings=[512, 0], model_dim=32, kernel_size=3, num_layers_per_block=5, num_blocks=5,
                  causal_dropout_prob=0.5, attention_dropout_prob=0.5, bottleneck_divisor=4, use_conditioning=False,
                  mixup_alpha=0.0, use_mixup_batch_hack=False, metric="cross_entropy", lr=1e-5)
    for k, v in kw.items():
        setattr(a, k, v)
    return a
