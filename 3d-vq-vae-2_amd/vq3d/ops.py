"""Tensor-level wrappers over the libvq3d C-ABI.

Activations are torch tensors with the reference's logical shape (B, C, H, W, D) stored
channels-last (torch.channels_last_3d == physical [B][H][W][D][C]), fp32 or bf16.
Every call enqueues on the current torch stream; nothing here synchronises the host.
"""
import ctypes

import torch

from . import _lib as L

CL = torch.channels_last_3d


def new_act(b, c, h, w, d, dtype, device):
    return torch.empty((b, c, h, w, d), dtype=dtype, device=device, memory_format=CL)


def as_cl(x):
    """Return x in channels-last layout (no copy when already there; C == 1 is both)."""
    if x.is_contiguous(memory_format=CL):
        return x
    if x.shape[1] == 1 and x.is_contiguous():
        return x
    raise L.Vq3dError("vq3d activations must be channels-last (torch.channels_last_3d); "
                      "convert once at the model boundary")


def _p(t):
    return None if t is None else t.data_ptr()


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------------------------------------ conv
class ConvGeom:
    """Geometry of one nn.Conv3d call (kernel, stride, pad, padding mode)."""
    __slots__ = ("k", "s", "p", "circular")

    def __init__(self, k, s=1, p=0, circular=False):
        self.k, self.s, self.p, self.circular = int(k), int(s), int(p), bool(circular)

    def out(self, n):
        return (n + 2 * self.p - self.k) // self.s + 1

    def key(self):
        return (self.k, self.s, self.p, self.circular)


_desc_cache = {}


def conv_desc(dtype, b, cin, cin2, cout, h, w, d, geom, pro_kind, taps=0):
    key = (dtype, b, cin, cin2, cout, h, w, d, geom.key(), pro_kind, taps)
    r = _desc_cache.get(key)
    if r is None:
        oh, ow, od = geom.out(h), geom.out(w), geom.out(d)
        desc = L.ConvDesc(dtype=L.dtype_code(dtype), batch=b, cin=cin, cin2=cin2, cout=cout, in_h=h, in_w=w,
                          in_d=d, out_h=oh, out_w=ow, out_d=od, kernel=geom.k, stride=geom.s, pad=geom.p,
                          pad_mode=L.PAD_CIRCULAR if geom.circular else L.PAD_ZEROS, pro_kind=pro_kind,
                          tap_mask=taps)
        r = (desc, (oh, ow, od))
        _desc_cache[key] = r
    return r


def pro_kind_of(pro):
    """pro = None | (a,) | (a, b): none / x + a / elu(x + a) + b (device scalar tensors)."""
    if pro is None:
        return L.PRO_NONE, None, None
    if len(pro) == 1:
        return L.PRO_ADD, pro[0], None
    return L.PRO_ELU_ADD, pro[0], pro[1]


def _act(act):
    """act = None | 'elu' | (a, b) -> (kind, a, b): none / elu(v) / elu(v + a) + b."""
    if act is None:
        return L.ACT_NONE, None, None
    if act == "elu":
        return L.ACT_ELU, None, None
    return L.ACT_ELU_AFFINE, act[0], act[1]


def conv_fwd(x, w, geom, pro=None, x2=None, scale=None, bias=None, cbias=None, residual=None,
             residual_up2=False, act=None, out=None, taps=0):
    """taps: vq3d_conv_desc.tap_mask (0 = dense; else the weight taps that may be nonzero)"""
    x = as_cl(x)
    b, cin, h, wd, d = x.shape
    cin2 = 0 if x2 is None else x2.shape[1]
    cout = w.shape[0]
    kind, pa, pb = pro_kind_of(pro)
    desc, (oh, ow, od) = conv_desc(x.dtype, b, cin, cin2, cout, h, wd, d, geom, kind, taps)
    if w.shape[1] != cin + cin2 or w.shape[2] != geom.k:
        raise L.Vq3dError(f"weight {tuple(w.shape)} does not match conv ({cin}+{cin2} -> {cout}, k={geom.k})")
    y = out if out is not None else new_act(b, cout, oh, ow, od, x.dtype, x.device)
    if residual is not None:
        rs = (b, cout, oh // 2, ow // 2, od // 2) if residual_up2 else (b, cout, oh, ow, od)
        if tuple(residual.shape) != rs or residual.dtype != x.dtype:
            raise L.Vq3dError(f"residual {tuple(residual.shape)} does not match {rs}")
        as_cl(residual)
    ak, aa, ab = _act(act)
    epi = L.ConvEpilogue(scale=_p(scale), bias=_p(bias), cbias=_p(cbias), residual=_p(residual),
                         residual_up2=int(residual_up2), act=ak, act_a=_p(aa), act_b=_p(ab))
    ws, wsb = _ws(desc, L.PASS_FWD, x.device)
    L.call("vq3d_conv3d_fwd", ctypes.byref(desc), L.ptr(x), _p(x2), L.ptr(w), _p(pa), _p(pb),
           ctypes.byref(epi), L.ptr(y), _p(ws), wsb, L.stream())
    return y


_ws_cache = {}


def conv_workspace_bytes(desc, pass_):
    """Scratch bytes one conv launch needs (vq3d_conv3d_workspace_size), cached per descriptor."""
    key = (bytes(desc), pass_)
    r = _ws_cache.get(key)
    if r is None:
        r = _ws_cache[key] = int(L.query("vq3d_conv3d_workspace_size", ctypes.byref(desc), pass_))
    return r


def _ws(desc, pass_, device):
    n = conv_workspace_bytes(desc, pass_)
    return (workspace(n, device), n) if n else (None, 0)


def _depi(aux, aux_b, addend):
    """dgrad epilogue: aux with aux_b=None -> derivative of the conv's own prologue (aux = its
    input before the prologue); with aux_b -> aux is an activated tensor elu(z) + aux_b."""
    return L.DgradEpilogue(aux=_p(aux), aux_kind=0 if aux_b is None else 1, aux_b=_p(aux_b), addend=_p(addend))


def conv_bwd(g, x, w, geom, pro=None, x2=None, gscale=None, aux=None, aux_b=None, addend=None, want_gx=True,
             dw=None, dscale=None, dbias=None, dcbias=None, dpro_pre=None, dpro_post=None, escale=None, taps=0):
    """Backward of conv_fwd: returns (gx, gx2); parameter gradients are ACCUMULATED (fp32
    atomics) into the given buffers (dw: weight, dscale/dbias: epilogue scalars, dcbias: conv
    bias, dpro_pre/dpro_post: prologue scalars (+b / +a of elu(x+a)+b, or a of x+a)); with a tap
    mask the weight-gradient entries of the clear taps may be left unwritten."""
    x = as_cl(x)
    b, cin, h, wd, d = x.shape
    cin2 = 0 if x2 is None else x2.shape[1]
    kind, pa, pb = pro_kind_of(pro)
    desc, _ = conv_desc(x.dtype, b, cin, cin2, w.shape[0], h, wd, d, geom, kind, taps)
    s = L.stream()
    gx = gx2 = None
    if want_gx or dpro_pre is not None or dpro_post is not None:
        gx = new_act(b, cin, h, wd, d, x.dtype, x.device)
        gx2 = None if x2 is None else new_act(b, cin2, h, wd, d, x.dtype, x.device)
        epi = _depi(aux, aux_b, addend)
        ws, wsb = _ws(desc, L.PASS_BWD_DATA, x.device)
        L.call("vq3d_conv3d_bwd_data", ctypes.byref(desc), L.ptr(g), _p(gscale), L.ptr(w), _p(pa),
               ctypes.byref(epi), L.ptr(gx), _p(gx2), _p(dpro_pre), _p(dpro_post), _p(ws), wsb, s)
    if dw is None and dscale is None and dbias is None and dcbias is None:
        return gx, gx2
    if _concurrent:
        # the weight gradient only reads x and g: run it on the side stream, overlapped with the
        # backward-data chain on the main stream (joined before the optimizer, join_side())
        main = torch.cuda.current_stream()
        side = _side_stream(x.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            ws, wsb = _ws(desc, L.PASS_BWD_WEIGHT, x.device)
            L.call("vq3d_conv3d_bwd_weight", ctypes.byref(desc), L.ptr(x), _p(x2), L.ptr(g), _p(pa), _p(pb),
                   L.ptr(w), _p(escale), _p(dw), _p(dscale), _p(dbias), _p(dcbias), _p(ws), wsb, L.stream())
        for t in (x, x2, g):
            if t is not None:
                t.record_stream(side)
        return gx, gx2
    ws, wsb = _ws(desc, L.PASS_BWD_WEIGHT, x.device)
    L.call("vq3d_conv3d_bwd_weight", ctypes.byref(desc), L.ptr(x), _p(x2), L.ptr(g), _p(pa), _p(pb), L.ptr(w),
           _p(escale), _p(dw), _p(dscale), _p(dbias), _p(dcbias), _p(ws), wsb, s)
    return gx, gx2


# ------------------------------------------------------------------------------------------------ kernel timing
_ktimer = [None]


class KernelTimer:
    """HIP-event timing of ONE engine kernel's launches inside a real (eager) training step.

    While active (``with KernelTimer("k_pm_bwd2") as t: step()``), the run-level wrappers below issue
    the selected kernel as a launch of its own (the multi-kernel entry points are split into their
    stages, which is numerically identical) and bracket each launch with HIP events on the stream it
    is launched on.  ``avg_us()`` is then the kernel's average duration with the step's real data
    and neighbours -- what bench.py reports as the dominant kernel's live launch time.  Kinds:
    k_pm_fwd, k_pm_bwd2, k_pm_w2grad, k_pm_w13grad (chained 18-channel runs), k_col_fwd<C_B>,
    k_col_bwd<C_B> (few-channel column blocks, e.g. "k_col_bwd<4_2"), k_stackm_fwd, k_stackm_bwd."""

    def __init__(self, kind):
        self.kind = kind
        self.events = []

    def __enter__(self):
        _ktimer[0] = self
        return self

    def __exit__(self, *exc):
        _ktimer[0] = None
        return False

    def wants(self, kind):
        return kind == self.kind

    def run(self, fn):
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        self.events.append((e0, e1))

    def avg_us(self):
        if not self.events:
            return None
        self.events[-1][1].synchronize()
        return 1e3 * sum(a.elapsed_time(b) for a, b in self.events) / len(self.events)


def _timed(kind, fn):
    """fn() bracketed by HIP events when the active KernelTimer selects `kind`."""
    t = _ktimer[0]
    if t is not None and t.wants(kind() if callable(kind) else kind):
        t.run(fn)
    else:
        fn()


def _small_kind(which, b, c, nb, h, w, d):
    """timer kind of a few-channel block launch: the column kernels (plan 2) or the brick kernels"""
    col = int(L.query("vq3d_preact_small_plan", b, c, nb, h, w, d)) == 2
    return f"k_{'col' if col else 'small'}_{which}<{c}_{nb}"


def timing(kind):
    """True when a KernelTimer for `kind` is active (the caller then issues that kernel alone)."""
    t = _ktimer[0]
    return t is not None and t.wants(kind)


# ------------------------------------------------------------------------------------------------ streams
_concurrent = False
_side = {}


def set_concurrent_wgrad(enabled=True):
    """Run every conv weight gradient on a per-device side stream, overlapped with the
    backward-data chain (the two only share read-only inputs and write disjoint gradient
    entries).  join_side() must precede any read of the gradients (the optimizer and the
    gradient all-reduce call it)."""
    global _concurrent
    _concurrent = bool(enabled)


def _side_stream(device):
    s = _side.get(device.index)
    if s is None:
        s = _side[device.index] = torch.cuda.Stream(device=device)
    return s


_levels = {}
_overlap = [True]


def set_overlap_levels(enabled=True):
    """Run the decoder's top-level chain (its post-quantize blocks and up block, which need only
    the top code) on a second stream beside the encoder's lower levels (VQVAE.forward); autograd
    runs their backward on that stream too."""
    _overlap[0] = bool(enabled)


def overlap_levels():
    return _overlap[0]


def level_stream(device):
    s = _levels.get(device.index)
    if s is None:
        s = _levels[device.index] = torch.cuda.Stream(device=device)
    return s


_aux = {}


def aux_stream(device, key):
    """a named per-device stream (PixelSNAIL's per-stack-stream lanes), created once"""
    k = (device.index, key)
    s = _aux.get(k)
    if s is None:
        s = _aux[k] = torch.cuda.Stream(device=device)
    return s


def side_streams():
    """Every stream besides the current one that may hold work of the step: the weight-gradient
    side streams and the level streams (the aux streams are joined by their users: PixelSNAIL's
    lanes through its forward's end and autograd's cross-stream gradient hand-offs)."""
    return list(_side.values()) + list(_levels.values())


def join_side():
    """Current stream waits for all work issued on the weight-gradient side streams and the
    level streams (the optimizer and the gradient all-reduce call it before reading gradients)."""
    if _side or _levels:
        cur = torch.cuda.current_stream()
        for s in side_streams():
            cur.wait_stream(s)


# ------------------------------------------------------------------------------------------------ upsample
def upsample2x(x, pro=None):
    x = as_cl(x)
    b, c, h, w, d = x.shape
    kind, pa, pb = pro_kind_of(pro)
    y = new_act(b, c, 2 * h, 2 * w, 2 * d, x.dtype, x.device)
    L.call("vq3d_upsample2x_fwd", L.dtype_code(x), b, c, h, w, d, L.ptr(x), kind, _p(pa), _p(pb), L.ptr(y),
           L.stream())
    return y


def upsample2x_bwd(gy, src_shape, pro=None, aux=None, aux_b=None, addend=None, dpro_pre=None, dpro_post=None):
    b, c, h, w, d = src_shape
    kind, pa, _ = pro_kind_of(pro)
    gx = new_act(b, c, h, w, d, gy.dtype, gy.device)
    epi = _depi(aux, aux_b, addend)
    L.call("vq3d_upsample2x_bwd", L.dtype_code(gy), b, c, h, w, d, L.ptr(gy), kind, _p(pa), ctypes.byref(epi),
           L.ptr(gx), _p(dpro_pre), _p(dpro_post), L.stream())
    return gx


# ------------------------------------------------------------------------------------------------ tiny PreAct block
_tiny = [True]


def set_tiny_blocks(enabled):
    """Route eligible PreAct blocks on tiny grids through the one-workgroup block kernels."""
    _tiny[0] = bool(enabled)


def tiny_blocks_enabled():
    return _tiny[0]


def preact_tiny_supported(x_shape, branch):
    b, c, h, w, d = x_shape
    return bool(L.query("vq3d_preact_tiny_supported", b, c, branch, h, w, d))


def _preact_params(blk):
    return L.PreactParams(*[_p(getattr(blk, n)) for n in ("bias1a", "bias1b", "bias2a", "bias2b", "bias3a",
                                                            "bias3b", "scale", "bias4")])


def preact_tiny_fwd(x, blk):
    """Whole PreActFixupResBlock ('same', no skip) in one kernel on a tiny grid (vq3d.h)."""
    x = as_cl(x)
    b, c, h, w, d = x.shape
    w1, w2, w3 = blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    out = torch.empty_like(x, memory_format=CL)
    nb = w1.shape[0]
    saved = torch.empty(L.query("vq3d_preact_tiny_saved_floats", b, nb, h, w, d), dtype=torch.float32,
                        device=x.device)
    prm = _preact_params(blk)
    L.call("vq3d_preact_tiny_fwd", L.dtype_code(x), b, c, nb, h, w, d, L.ptr(x), L.ptr(w1), L.ptr(w2),
           L.ptr(w3), ctypes.byref(prm), L.ptr(out), L.ptr(saved), L.stream())
    return out, saved


def preact_tiny_bwd(g, x, saved, blk, grads):
    """gx of preact_tiny_fwd; grads: dict name -> fp32 buffer (+=), names as in L.PreactGrads."""
    b, c, h, w, d = x.shape
    w1, w2, w3 = blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    nb = w1.shape[0]
    gx = torch.empty_like(x, memory_format=CL)
    ws = torch.empty(L.query("vq3d_preact_tiny_workspace_floats", b, nb, h, w, d), dtype=torch.float32,
                     device=x.device)
    prm = _preact_params(blk)
    gr = L.PreactGrads(*[_p(grads.get(n)) for n, _ in L.PreactGrads._fields_])
    L.call("vq3d_preact_tiny_bwd", L.dtype_code(x), b, c, nb, h, w, d, L.ptr(x), L.ptr(g), L.ptr(w1),
           L.ptr(w2), L.ptr(w3), ctypes.byref(prm), ctypes.byref(gr), L.ptr(saved), L.ptr(ws), L.ptr(gx),
           L.stream())
    return gx


_mid = [True]


_batched_wgrad = True


def set_batched_wgrad(enabled):
    """Mid-level (18-channel) and wide (72-channel) runs: the weight gradients of all blocks as one
    launch per kind after the data chain (vq3d_preact_mid_wgrad_run / vq3d_preact_wide_wgrad_run,
    the default) or per block between the data kernels."""
    global _batched_wgrad
    _batched_wgrad = bool(enabled)


def batched_wgrad():
    return _batched_wgrad


def concurrent_wgrad():
    return _concurrent


def set_mid_blocks(enabled):
    """Route eligible bf16 PreAct blocks of the 18-channel level through the fused forward."""
    _mid[0] = bool(enabled)


def preact_mid_supported(x, branch):
    b, c, h, w, d = x.shape
    return _mid[0] and bool(L.query("vq3d_preact_mid_supported", L.dtype_code(x), b, c, branch, h, w, d))


def preact_mid_fwd(x, blk, stages=None, bufs=None, save=True):
    """Fused PreAct block forward (vq3d.h): returns out, t2, t3 (bf16 channels-last); save=False
    (no backward follows): t3 is not written (None).  stages / bufs: measurement only
    (vq3d_preact_mid_fwd_stages, preallocated outputs)."""
    x = as_cl(x)
    b, c, h, w, d = x.shape
    w1, w2, w3 = blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    nb = w1.shape[0]
    if bufs is None:
        out = torch.empty_like(x, memory_format=CL)
        t2 = new_act(b, nb, h, w, d, x.dtype, x.device)
        t3 = new_act(b, nb, h, w, d, x.dtype, x.device) if save else None
    else:
        out, t2, t3 = bufs
    prm = _preact_params(blk)
    args = (L.dtype_code(x), b, c, nb, h, w, d, L.ptr(x), L.ptr(w1), L.ptr(w2), L.ptr(w3), ctypes.byref(prm),
            L.ptr(out), L.ptr(t2), _p(t3), L.stream())
    if stages is None:
        L.call("vq3d_preact_mid_fwd", *args)
    else:
        L.call("vq3d_preact_mid_fwd_stages", int(stages), *args)
    return out, t2, t3


def preact_mid_bwd(g, x, t2, t3, blk, grads, stages=None, bufs=None):
    """gx of preact_mid_fwd; grads: dict name -> fp32 buffer (+=, all required), names as in
    L.PreactGrads.  stages / bufs: measurement only (vq3d_preact_mid_bwd_stages, preallocated
    gx and workspace)."""
    b, c, h, w, d = x.shape
    w1, w2, w3 = blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    nb = w1.shape[0]
    if bufs is None:
        gx = torch.empty_like(x, memory_format=CL)
        ws = workspace(L.query("vq3d_preact_mid_workspace_bytes", b, h, w, d), x.device)
    else:
        gx, ws = bufs
    prm = _preact_params(blk)
    gr = L.PreactGrads(*[_p(grads.get(n)) for n, _ in L.PreactGrads._fields_])
    args = (L.dtype_code(x), b, c, nb, h, w, d, L.ptr(g), L.ptr(x), L.ptr(t2), L.ptr(t3), L.ptr(w1), L.ptr(w2),
            L.ptr(w3), ctypes.byref(prm), ctypes.byref(gr), L.ptr(ws), ctypes.c_size_t(ws.numel()), L.ptr(gx))
    if stages is not None:
        L.call("vq3d_preact_mid_bwd_stages", int(stages), *args, L.stream())
    elif _concurrent:
        # data stages (gz3, gx; gz1 to the workspace) on the main stream, the weight gradient and
        # the fixed-order reduction on the side stream (they read g / x / t2 / t3 / workspace only)
        L.call("vq3d_preact_mid_bwd_stages", 3, *args, L.stream())
        main = torch.cuda.current_stream()
        side = _side_stream(x.device)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            L.call("vq3d_preact_mid_bwd_stages", 28, *args, L.stream())
        for t in (g, x, t2, t3, ws):
            t.record_stream(side)
    else:
        L.call("vq3d_preact_mid_bwd", *args, L.stream())
    return gx


def preact_mid_run_fwd(x, blocks, save=True):
    """A RUN of fused mid-level blocks, chained (vq3d_preact_mid_fwd_chain): the first block's t2
    stage, then one tile launch per block that also writes the next block's t2 from its out while
    the tile is in LDS.  Returns out and, per block, (x_i, t2_i, t3_i) (t3_i None when save=False:
    no backward follows)."""
    x = as_cl(x)
    b, c, h, w, d = x.shape
    nb = blocks[0].branch_conv1.weight.shape[0]
    dc = L.dtype_code(x)
    b0 = blocks[0]
    t2 = new_act(b, nb, h, w, d, x.dtype, x.device)
    out = torch.empty_like(x, memory_format=CL)
    prm = _preact_params(b0)
    L.call("vq3d_preact_mid_fwd_stages", 1, dc, b, c, nb, h, w, d, L.ptr(x), L.ptr(b0.branch_conv1.weight),
           L.ptr(b0.branch_conv2.weight), L.ptr(b0.branch_conv3.weight), ctypes.byref(prm), L.ptr(out), L.ptr(t2),
           None, L.stream())
    saved = []
    for i, blk in enumerate(blocks):
        nxt = blocks[i + 1] if i + 1 < len(blocks) else None
        if i:
            out = torch.empty_like(x, memory_format=CL)
        t3 = new_act(b, nb, h, w, d, x.dtype, x.device) if save else None
        t2n = new_act(b, nb, h, w, d, x.dtype, x.device) if nxt is not None else None
        prm = _preact_params(blk)
        prmn = _preact_params(nxt) if nxt is not None else None
        fargs = (dc, b, c, nb, h, w, d, L.ptr(x), L.ptr(blk.branch_conv2.weight), L.ptr(blk.branch_conv3.weight),
                 ctypes.byref(prm), L.ptr(t2), L.ptr(out), _p(t3),
                 None if nxt is None else L.ptr(nxt.branch_conv1.weight),
                 None if prmn is None else ctypes.byref(prmn), _p(t2n), L.stream())
        # k_pm_fwd<..., true> (the chained tile kernel) is the launch of every block but the last
        _timed("k_pm_fwd" if nxt is not None else "", lambda a=fargs: L.call("vq3d_preact_mid_fwd_chain", *a))
        if save:
            saved.append((x, t2, t3))
        x, t2 = out, t2n
    return x, saved


def preact_mid_run_bwd(g, plan, saved, on_done=None):
    """Backward of preact_mid_run_fwd (vq3d_preact_mid_bwd_chain): per block, in reverse, the data
    tile kernel also computes the PREVIOUS block's pointwise gz3 stage from its gx, and the weight
    gradient kernels follow (on the side stream in concurrent weight-gradient mode); every block's
    workspace is a slice of one run buffer, so the fixed-order reductions of all blocks run as ONE
    launch at the end (vq3d_preact_mid_reduce_run, plan's device tables).  Returns gx of the run's
    input; on_done() runs once the reduction is enqueued."""
    blocks = plan.blocks
    g = g if g.is_contiguous(memory_format=CL) else g.contiguous(memory_format=CL)
    b, c, h, w, d = g.shape
    nb = blocks[0].branch_conv1.weight.shape[0]
    dc = L.dtype_code(g)
    nws = int(L.query("vq3d_preact_mid_workspace_bytes", b, h, w, d))
    stride = (nws + 255) // 256 * 256
    run_ws = workspace(stride * len(blocks), g.device)
    base = run_ws.data_ptr()
    ptab, gtab = plan.tables(g.device)
    run_g = []  # batched weight gradients: every block's incoming gradient, kept for the run launch
    for i in reversed(range(len(blocks))):
        blk = blocks[i]
        x, t2, t3 = saved[i]
        gx = torch.empty_like(x, memory_format=CL)
        prm = _preact_params(blk)
        gr = L.PreactGrads(*[ctypes.c_void_p(int(gp)) for gp in plan.grad_ptrs(i)])
        if i:
            prev = blocks[i - 1]
            prmp = _preact_params(prev)
            chain = (L.ptr(saved[i - 1][2]), L.ptr(prev.branch_conv3.weight), ctypes.byref(prmp),
                     ctypes.c_void_p(base + (i - 1) * stride), ctypes.c_size_t(nws))
        else:
            chain = (None, None, None, None, ctypes.c_size_t(0))
        first = 1 if i == len(blocks) - 1 else 0
        args = (dc, b, c, nb, h, w, d, L.ptr(g), L.ptr(x), L.ptr(t2), L.ptr(t3), L.ptr(blk.branch_conv1.weight),
                L.ptr(blk.branch_conv2.weight), L.ptr(blk.branch_conv3.weight), ctypes.byref(prm), ctypes.byref(gr),
                ctypes.c_void_p(base + i * stride), ctypes.c_size_t(nws), L.ptr(gx))
        if _concurrent:
            L.call("vq3d_preact_mid_bwd_chain", first | 2, *args, *chain, L.stream())
            _on_side(g.device, lambda a=args: L.call("vq3d_preact_mid_bwd_stages", 12, *a, L.stream()),
                     g, x, t2, t3)
        elif timing("k_pm_bwd2") or timing("k_pm_w2grad") or timing("k_pm_w13grad"):
            # the same stages as one launch each (k_pm_bwd2<..., true> = the chained data tile of
            # every block but the first / last, whose calls also carry the pointwise stage)
            _timed("k_pm_bwd2" if (i and not first) else "",
                   lambda a=args, ch=chain: L.call("vq3d_preact_mid_bwd_chain", first | 2, *a, *ch, L.stream()))
            _timed("k_pm_w2grad", lambda a=args: L.call("vq3d_preact_mid_bwd_stages", 4, *a, L.stream()))
            _timed("k_pm_w13grad", lambda a=args: L.call("vq3d_preact_mid_bwd_stages", 8, *a, L.stream()))
        elif _batched_wgrad:
            # the data stage only; the run's weight gradients follow as one launch per kind
            L.call("vq3d_preact_mid_bwd_chain", first | 2, *args, *chain, L.stream())
            run_g.append(g)
        else:
            L.call("vq3d_preact_mid_bwd_chain", first | 14, *args, *chain, L.stream())
        g = gx
    if run_g:
        n = len(blocks)
        arr = ctypes.c_void_p * n
        run_g.reverse()  # run_g[i]: block i's incoming gradient
        L.call("vq3d_preact_mid_wgrad_run", dc, n, b, h, w, d, arr(*[s_[1].data_ptr() for s_ in saved]),
               arr(*[s_[2].data_ptr() for s_ in saved]), arr(*[s_[0].data_ptr() for s_ in saved]),
               arr(*[t.data_ptr() for t in run_g]), L.ptr(ptab), ctypes.c_void_p(base), ctypes.c_size_t(stride),
               L.stream())
    red = (len(blocks), b, h, w, d, ctypes.c_void_p(base), ctypes.c_size_t(stride), L.ptr(gtab), L.ptr(ptab))
    if _concurrent:
        _on_side(g.device, lambda: L.call("vq3d_preact_mid_reduce_run", *red, L.stream()), run_ws, ptab, gtab)
    else:
        L.call("vq3d_preact_mid_reduce_run", *red, L.stream())
    if on_done is not None:
        on_done()
    return g


def _on_side(device, fn, *keep):
    """Run fn() on the device's side stream after the work already queued on the current one;
    `keep` tensors stay allocated until the side stream is done with them."""
    main = torch.cuda.current_stream()
    side = _side_stream(device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        fn()
    for t in keep:
        if t is not None:
            t.record_stream(side)


_small = [True, True]


def set_small_blocks(enabled, fused_backward=True):
    """Route eligible bf16 few-channel PreAct blocks ((C, branch) = (2, 1), (4, 2), (8, 4))
    through the fused block kernels (preact_small.hip); fused_backward=False keeps the fused
    forward but runs the per-conv backward from its saved t2 / t3."""
    _small[0] = bool(enabled)
    _small[1] = bool(fused_backward)


# the brick kernels' fused backward up to this many voxels (measured, bench 3L pub: 23.6 vs ~100
# us per (8, 4) block at 32x32x8); beyond it their per-brick weight-gradient partials are
# LDS-bound and, where the column kernels (preact_col.hip, D % 16 == 0) do not apply, the
# per-conv backward wins
_SMALL_BWD_MAX_VOX = 1 << 19


def small_backward_fused(x):
    b, c, h, w, d = x.shape
    if not _small[1]:
        return False
    nb = c // 2
    if int(L.query("vq3d_preact_small_plan", b, c, nb, h, w, d)) == 2:  # column kernels
        return True
    return b * h * w * d <= _SMALL_BWD_MAX_VOX


def preact_small_supported(x, branch):
    b, c, h, w, d = x.shape
    return _small[0] and bool(L.query("vq3d_preact_small_supported", L.dtype_code(x), b, c, branch, h, w, d))


_fp32_stream = [True]


def set_fp32_stream(enabled=True):
    """Carry the residual stream of a RUN of fused blocks in fp32 between its blocks (conv operands
    stay bf16), as the reference's autocast blocks return fp32 (layers.py:187-193); off: bf16."""
    _fp32_stream[0] = bool(enabled)


def fp32_stream():
    return _fp32_stream[0]


def _fmt16(x):
    """The 16-bit format of a few-channel run (t2 / t3 and every conv operand): its input's, or
    bf16 when the input is already fp32."""
    return x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.bfloat16


def preact_small_fwd(x, blk, save=True, out_dtype=None, fmt=None):
    """Fused few-channel PreAct block forward (vq3d.h): returns out, t2, t3 (channels-last; t2 / t3
    in the 16-bit format fmt (default: x's), out in out_dtype, default x's: the residual stream is
    16-bit or fp32 per tensor); save=False (no backward follows): t2 / t3 are not written (None)."""
    x = as_cl(x)
    b, c, h, w, d = x.shape
    fmt = fmt or _fmt16(x)
    w1, w2, w3 = blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    nb = w1.shape[0]
    out = torch.empty_like(x, memory_format=CL, dtype=out_dtype or x.dtype)
    t2 = new_act(b, nb, h, w, d, fmt, x.device) if save else None
    t3 = new_act(b, nb, h, w, d, fmt, x.device) if save else None
    prm = _preact_params(blk)
    _timed(lambda: _small_kind("fwd", b, c, nb, h, w, d), lambda: L.call(
        "vq3d_preact_small_fwd_io", L.dtype_code(fmt), L.dtype_code(x), L.dtype_code(out), b, c, nb, h, w, d,
        L.ptr(x), L.ptr(w1), L.ptr(w2), L.ptr(w3), ctypes.byref(prm), L.ptr(out), _p(t2), _p(t3), L.stream()))
    return out, t2, t3


_chain = [True]


def set_small_chain(enabled=True):
    """Chain the column-kernel runs' forward (vq3d_preact_small_fwd_chain): each block's t2 formed
    once per voxel in the previous block's epilogue instead of on every brick's halo."""
    _chain[0] = bool(enabled)


def small_chain_ok(x, nblocks):
    b, c, h, w, d = x.shape
    return (_chain[0] and nblocks > 1 and
            int(L.query("vq3d_preact_small_plan", b, c, c // 2, h, w, d)) == 2)


def preact_small_run_fwd(x, blocks, save, out_dtypes):
    """Forward of a chained run of column-kernel blocks: per block one launch that reads its t2 from
    the previous launch and writes the next block's.  out_dtypes[i]: block i's output storage.
    Returns (out, [(x_i, t2_i, t3_i)] if save else [])."""
    x = as_cl(x)
    b, c, h, w, d = x.shape
    fmt = _fmt16(x)
    nb = blocks[0].branch_conv1.weight.shape[0]
    n = len(blocks)
    saved = []
    t2 = new_act(b, nb, h, w, d, fmt, x.device)
    prms = [_preact_params(blk) for blk in blocks]
    for i, blk in enumerate(blocks):
        out = torch.empty_like(x, memory_format=CL, dtype=out_dtypes[i])
        t3 = new_act(b, nb, h, w, d, fmt, x.device) if save else None
        t2n = new_act(b, nb, h, w, d, fmt, x.device) if i + 1 < n else None
        mode = (1 if i else 0) | (2 if i + 1 < n else 0)
        nxt = blocks[i + 1] if i + 1 < n else None
        args = (mode, L.dtype_code(fmt), L.dtype_code(x), L.dtype_code(out), b, c, nb, h, w, d, L.ptr(x),
                L.ptr(t2) if i else None, L.ptr(blk.branch_conv1.weight), L.ptr(blk.branch_conv2.weight),
                L.ptr(blk.branch_conv3.weight), ctypes.byref(prms[i]), L.ptr(out), L.ptr(t2), _p(t3),
                _p(nxt.branch_conv1.weight) if nxt is not None else None,
                ctypes.byref(prms[i + 1]) if nxt is not None else None, _p(t2n), L.stream())
        _timed(lambda: _small_kind("fwd", b, c, nb, h, w, d),
               lambda a=args: L.call("vq3d_preact_small_fwd_chain", *a))
        if save:
            saved.append((x, t2, t3))
        x, t2 = out, t2n
    return x, saved


def preact_small_bwd(g, x, t2, t3, blk, grads):
    """gx of preact_small_fwd; grads: dict name -> fp32 buffer (+=), names as in L.PreactGrads."""
    b, c, h, w, d = x.shape
    w1, w2, w3 = blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    nb = w1.shape[0]
    gx = torch.empty_like(x, memory_format=CL)
    nbytes = L.query("vq3d_preact_small_workspace_bytes", b, c, nb, h, w, d)
    ws = workspace(nbytes, x.device)
    prm = _preact_params(blk)
    gr = L.PreactGrads(*[_p(grads.get(n)) for n, _ in L.PreactGrads._fields_])
    args = (L.dtype_code(x), b, c, nb, h, w, d, L.ptr(g), L.ptr(x), L.ptr(t2), L.ptr(t3), L.ptr(w1), L.ptr(w2),
            L.ptr(w3), ctypes.byref(prm), ctypes.byref(gr), L.ptr(ws), ctypes.c_size_t(ws.numel()), L.ptr(gx))
    L.call("vq3d_preact_small_bwd", *args, L.stream())
    return gx


def preact_small_run_bwd(g, plan, saved, on_done=None):
    """Backward of a run of fused few-channel blocks: per block, in reverse, the fused data /
    partial-sum kernel into its slice of one run workspace, then the fixed-order reductions of every
    block as one launch pair (vq3d_preact_small_reduce_run, plan's device tables).  Each block's g
    has its out's storage and its gx its input's (the fp32 stream inside the run).  (A backward
    chained like the forward -- each launch forming the previous block's gz3 in its epilogue --
    was measured slower: the epilogue's extra registers cost more than the halo math it saves.)
    Returns gx of the run's input."""
    blocks = plan.blocks
    g = g if g.is_contiguous(memory_format=CL) else g.contiguous(memory_format=CL)
    b, c, h, w, d = g.shape
    nb = blocks[0].branch_conv1.weight.shape[0]
    fmt = saved[0][1].dtype
    nws = int(L.query("vq3d_preact_small_workspace_bytes", b, c, nb, h, w, d))
    stride = (nws + 255) // 256 * 256
    run_ws = workspace(stride * len(blocks), g.device)
    base = run_ws.data_ptr()
    ptab, gtab = plan.tables(g.device)
    run_g = []  # batched weight gradients: every block's incoming gradient, kept for the run launch
    for i in reversed(range(len(blocks))):
        blk = blocks[i]
        x, t2, t3 = saved[i]
        gx = torch.empty_like(x, memory_format=CL)
        prm = _preact_params(blk)
        gr = L.PreactGrads(*[ctypes.c_void_p(int(gp)) for gp in plan.grad_ptrs(i)])
        sargs = (L.dtype_code(fmt), L.dtype_code(x), L.dtype_code(g), b, c, nb, h, w, d, L.ptr(g), L.ptr(x),
                 L.ptr(t2), L.ptr(t3), L.ptr(blk.branch_conv1.weight), L.ptr(blk.branch_conv2.weight),
                 L.ptr(blk.branch_conv3.weight), ctypes.byref(prm), ctypes.byref(gr),
                 ctypes.c_void_p(base + i * stride), ctypes.c_size_t(nws), L.ptr(gx), L.stream())
        _timed(lambda: _small_kind("bwd", b, c, nb, h, w, d),
               lambda a=sargs: L.call("vq3d_preact_small_bwd_stages_io", 1, *a))
        g = gx
    L.call("vq3d_preact_small_reduce_run", len(blocks), b, c, nb, h, w, d, ctypes.c_void_p(base),
           ctypes.c_size_t(stride), L.ptr(gtab), L.ptr(ptab), L.stream())
    if on_done is not None:
        on_done()
    return g


# ------------------------------------------------------------------------------------------------ wide blocks
_wide = [True]


def set_wide_blocks(enabled):
    """Route runs of bf16 72-channel / branch-36 PreAct blocks through preact_wide.hip."""
    _wide[0] = bool(enabled)


def preact_wide_supported(x, branch):
    b, c, h, w, d = x.shape
    return (_wide[0] and x.dtype in (torch.bfloat16, torch.float16)
            and bool(L.query("vq3d_preact_wide_supported", b, c, branch, h, w, d)))


def preact_wide_pack(ptab, nblocks, c, nb, device, dtype=torch.bfloat16):
    """Packed 16-bit (dtype) fragment images of a run's weights (one per block, consecutive)."""
    per = int(L.query("vq3d_preact_wide_image_bytes", c, nb))
    img = torch.empty(nblocks * per, dtype=torch.uint8, device=device)
    L.call("vq3d_preact_wide_pack", L.dtype_code(dtype), nblocks, c, nb, L.ptr(ptab), L.ptr(img), L.stream())
    return img, per


def preact_wide_fwd(x32, img_ptr, blk, save=True, dtype=torch.bfloat16):
    """One block on the fp32 residual stream: returns out (fp32), t2, t3 (16-bit dtype, the
    fragment image's format), channels-last; save=False (no backward follows): t2 / t3 are not
    written (None)."""
    b, c, h, w, d = x32.shape
    nb = blk.branch_conv1.weight.shape[0]
    out = torch.empty_like(x32, memory_format=CL)
    t2 = new_act(b, nb, h, w, d, dtype, x32.device) if save else None
    t3 = new_act(b, nb, h, w, d, dtype, x32.device) if save else None
    prm = _preact_params(blk)
    L.call("vq3d_preact_wide_fwd", L.dtype_code(dtype), b, c, nb, h, w, d, L.ptr(x32), ctypes.c_void_p(img_ptr), ctypes.byref(prm),
           L.ptr(out), _p(t2), _p(t3), L.stream())
    return out, t2, t3


def preact_wide_bwd(g32, x32, t2, t3, img_ptr, blk, grads, ws_ptr=None, reduce=True, weights=True):
    """gx (fp32) of preact_wide_fwd; the parameter gradients (grads: name -> fp32 buffer, +=) on
    the side stream when concurrent weight gradients are on.  ws_ptr: the block's slice of a run
    workspace (else one is allocated); reduce=False leaves the fixed-order reduction to the
    caller's vq3d_preact_wide_reduce_run; weights=False also leaves the weight-gradient stage to
    the caller's vq3d_preact_wide_wgrad_run (preact_wide_wgrad_run)."""
    b, c, h, w, d = x32.shape
    nb = blk.branch_conv1.weight.shape[0]
    gx = torch.empty_like(x32, memory_format=CL)
    nws = int(L.query("vq3d_preact_wide_workspace_bytes", b, h, w, d))
    ws = None
    if ws_ptr is None:
        ws = torch.empty(nws, dtype=torch.uint8, device=x32.device)
        ws_ptr = ws.data_ptr()
    wsp = ctypes.c_void_p(ws_ptr)
    prm = _preact_params(blk)
    dc = L.dtype_code(t2)
    L.call("vq3d_preact_wide_bwd_data", dc, b, c, nb, h, w, d, L.ptr(g32), L.ptr(x32), L.ptr(t2), L.ptr(t3),
           ctypes.c_void_p(img_ptr), ctypes.byref(prm), wsp, ctypes.c_size_t(nws), L.ptr(gx), L.stream())
    if not weights:
        return gx
    gr = L.PreactGrads(*[_p(grads.get(n)) for n, _ in L.PreactGrads._fields_])
    args = (1 | (2 if reduce else 0), dc, b, c, nb, h, w, d, L.ptr(g32), L.ptr(x32), L.ptr(t2), L.ptr(t3),
            ctypes.byref(prm), ctypes.byref(gr), wsp, ctypes.c_size_t(nws))
    if _concurrent:
        _on_side(x32.device, lambda: L.call("vq3d_preact_wide_bwd_weight_stages", *args, L.stream()),
                 g32, x32, t2, t3, ws)
    else:
        L.call("vq3d_preact_wide_bwd_weight_stages", *args, L.stream())
    return gx


def preact_wide_run_workspace(plan, shape, device):
    """One workspace for a run of wide blocks: (buffer, base address, per-block stride)."""
    b, c, h, w, d = shape
    nws = int(L.query("vq3d_preact_wide_workspace_bytes", b, h, w, d))
    stride = (nws + 255) // 256 * 256
    buf = workspace(stride * len(plan.blocks), device)
    return buf, buf.data_ptr(), stride


def preact_wide_wgrad_run(plan, shape, run_ws, stride, gs, xs, t2s, t3s):
    """Every block's weight-gradient partial rows of a wide run, one launch (after the data chain;
    per-block lists: incoming gradient, input, saved t2 / t3)."""
    b, c, h, w, d = shape
    n = len(plan.blocks)
    ptab, _ = plan.tables(run_ws.device)
    arr = ctypes.c_void_p * n
    L.call("vq3d_preact_wide_wgrad_run", L.dtype_code(t2s[0]), n, b, h, w, d, arr(*[t.data_ptr() for t in gs]),
           arr(*[t.data_ptr() for t in xs]), arr(*[t.data_ptr() for t in t2s]), arr(*[t.data_ptr() for t in t3s]),
           L.ptr(ptab), L.ptr(run_ws), ctypes.c_size_t(stride), L.stream())


def preact_wide_reduce_run(plan, shape, run_ws, stride):
    """The fixed-order gradient reductions of every block of a wide run, one launch."""
    b, c, h, w, d = shape
    ptab, gtab = plan.tables(run_ws.device)
    args = (len(plan.blocks), b, h, w, d, L.ptr(run_ws), ctypes.c_size_t(stride), L.ptr(gtab), L.ptr(ptab))
    if _concurrent:
        _on_side(run_ws.device, lambda: L.call("vq3d_preact_wide_reduce_run", *args, L.stream()), run_ws, ptab, gtab)
    else:
        L.call("vq3d_preact_wide_reduce_run", *args, L.stream())


# ------------------------------------------------------------------------------------------------ misc
def cast(x, dtype):
    if x.dtype == dtype:
        return x
    y = torch.empty_like(x, dtype=dtype)
    L.call("vq3d_cast", L.dtype_code(x), L.ptr(x), L.dtype_code(dtype), L.ptr(y), x.numel(), L.stream())
    return y


def zero_(t):
    L.call("vq3d_zero", L.ptr(t), t.numel() * t.element_size(), L.stream())
    return t


def copy_(dst, src):
    assert dst.numel() == src.numel() and dst.dtype == src.dtype
    L.call("vq3d_copy", L.ptr(dst), L.ptr(src), src.numel() * src.element_size(), L.stream())
    return dst


def scale_(t, a):
    L.call("vq3d_scale", L.ptr(t), float(a), t.numel(), L.stream())
    return t
