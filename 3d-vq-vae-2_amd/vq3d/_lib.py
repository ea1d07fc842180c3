"""ctypes binding of libvq3d.so (C-ABI declared in include/vq3d.h).

The library is REQUIRED: importing an op without it, or calling it on a non-GPU tensor,
raises.  There is no CPU / PyTorch fallback anywhere in the product path.
"""
import ctypes
import os

import torch

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("VQ3D_LIB", os.path.join(_PKG_ROOT, "lib", "libvq3d.so"))

F32, BF16, F16 = 0, 1, 2
PAD_ZEROS, PAD_CIRCULAR = 0, 1
PRO_NONE, PRO_ADD, PRO_ELU_ADD = 0, 1, 2
PASS_FWD, PASS_BWD_DATA, PASS_BWD_WEIGHT = 0, 1, 2

c_int, c_i64, c_size, c_float, c_void = ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t, ctypes.c_float, ctypes.c_void_p
P = ctypes.c_void_p


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("dtype", "batch", "cin", "cin2", "cout", "in_h", "in_w", "in_d",
                                     "out_h", "out_w", "out_d", "kernel", "stride", "pad", "pad_mode",
                                     "pro_kind")] + [("tap_mask", ctypes.c_uint32)]


ACT_NONE, ACT_ELU, ACT_ELU_AFFINE = 0, 1, 2


class ConvEpilogue(ctypes.Structure):
    _fields_ = [("scale", P), ("bias", P), ("cbias", P), ("residual", P), ("residual_up2", c_int),
                ("act", c_int), ("act_a", P), ("act_b", P)]


class PreactParams(ctypes.Structure):
    _fields_ = [(n, P) for n in ("bias1a", "bias1b", "bias2a", "bias2b", "bias3a", "bias3b", "scale", "bias4")]


class PreactGrads(ctypes.Structure):
    _fields_ = [(n, P) for n in ("dw1", "dw2", "dw3", "dbias1a", "dbias1b", "dbias2a", "dbias2b", "dbias3a",
                                 "dbias3b", "dscale", "dbias4")]


class AttnTrain(ctypes.Structure):
    _fields_ = [("dropout_p", ctypes.c_double), ("seed", P)]


class DgradEpilogue(ctypes.Structure):
    _fields_ = [("aux", P), ("aux_kind", c_int), ("aux_b", P), ("addend", P)]


_SIGS = {
    "vq3d_conv3d_workspace_size": (c_size, [P, c_int]),
    "vq3d_conv3d_fwd": (c_int, [P, P, P, P, P, P, P, P, P, c_size, P]),
    "vq3d_conv3d_bwd_data": (c_int, [P, P, P, P, P, P, P, P, P, P, P, c_size, P]),
    "vq3d_conv3d_bwd_weight": (c_int, [P, P, P, P, P, P, P, P, P, P, P, P, P, c_size, P]),
    "vq3d_upsample2x_fwd": (c_int, [c_int] * 6 + [P, c_int, P, P, P, P]),
    "vq3d_upsample2x_bwd": (c_int, [c_int] * 6 + [P, c_int, P, P, P, P, P, P]),
    "vq3d_preact_tiny_supported": (c_int, [c_int] * 6),
    "vq3d_preact_tiny_saved_floats": (c_size, [c_int] * 5),
    "vq3d_preact_tiny_workspace_floats": (c_size, [c_int] * 5),
    "vq3d_preact_tiny_fwd": (c_int, [c_int] * 7 + [P, P, P, P, P, P, P, P]),
    "vq3d_preact_tiny_bwd": (c_int, [c_int] * 7 + [P, P, P, P, P, P, P, P, P, P, P]),
    "vq3d_preact_mid_supported": (c_int, [c_int] * 7),
    "vq3d_preact_mid_fwd": (c_int, [c_int] * 7 + [P] * 9),
    "vq3d_preact_mid_workspace_bytes": (c_size, [c_int] * 4),
    "vq3d_preact_mid_bwd": (c_int, [c_int] * 7 + [P] * 10 + [c_size, P, P]),
    "vq3d_preact_mid_fwd_stages": (c_int, [c_int] * 8 + [P] * 9),
    "vq3d_preact_mid_bwd_stages": (c_int, [c_int] * 8 + [P] * 10 + [c_size, P, P]),
    "vq3d_preact_mid_fwd_chain": (c_int, [c_int] * 7 + [P] * 11),
    "vq3d_preact_mid_bwd_chain": (c_int, [c_int] * 8 + [P] * 10 + [c_size, P] + [P] * 4 + [c_size, P]),
    "vq3d_preact_mid_reduce_run": (c_int, [c_int] * 5 + [P, c_size, P, P, P]),
    "vq3d_preact_mid_wgrad_run": (c_int, [c_int] * 6 + [P, P, P, P, P, P, c_size, P]),
    "vq3d_preact_stack_supported": (c_int, [c_int] * 6),
    "vq3d_preact_stack_saved_floats": (c_size, [c_int] * 7),
    "vq3d_preact_stack_fwd": (c_int, [c_int] * 8 + [P] * 5),
    "vq3d_preact_stack_bwd": (c_int, [c_int] * 8 + [P] * 6),
    "vq3d_preact_stack_bwd_workspace_bytes": (c_size, [c_int] * 7),
    "vq3d_preact_stack_bwd_ws": (c_int, [c_int] * 8 + [P] * 6 + [c_size, P]),
    "vq3d_preact_wide_supported": (c_int, [c_int] * 6),
    "vq3d_preact_wide_image_bytes": (c_size, [c_int] * 2),
    "vq3d_preact_wide_pack": (c_int, [c_int] * 4 + [P] * 3),
    "vq3d_preact_wide_fwd": (c_int, [c_int] * 7 + [P] * 7),
    "vq3d_preact_wide_workspace_bytes": (c_size, [c_int] * 4),
    "vq3d_preact_wide_bwd_data": (c_int, [c_int] * 7 + [P] * 7 + [c_size, P, P]),
    "vq3d_preact_wide_bwd_weight": (c_int, [c_int] * 7 + [P] * 7 + [c_size, P]),
    "vq3d_preact_wide_bwd_weight_stages": (c_int, [c_int] * 8 + [P] * 7 + [c_size, P]),
    "vq3d_preact_wide_reduce_run": (c_int, [c_int] * 5 + [P, c_size, P, P, P]),
    "vq3d_preact_wide_wgrad_run": (c_int, [c_int] * 6 + [P, P, P, P, P, P, c_size, P]),
    "vq3d_preact_small_supported": (c_int, [c_int] * 7),
    "vq3d_preact_small_workspace_bytes": (c_size, [c_int] * 6),
    "vq3d_preact_small_plan": (c_int, [c_int] * 6),
    "vq3d_preact_small_fwd": (c_int, [c_int] * 7 + [P] * 9),
    "vq3d_preact_small_bwd": (c_int, [c_int] * 7 + [P] * 10 + [c_size, P, P]),
    "vq3d_preact_small_bwd_stages": (c_int, [c_int] * 8 + [P] * 10 + [c_size, P, P]),
    "vq3d_preact_small_reduce_run": (c_int, [c_int] * 7 + [P, c_size, P, P, P]),
    "vq3d_preact_small_fwd_io": (c_int, [c_int] * 9 + [P] * 9),
    "vq3d_preact_small_bwd_stages_io": (c_int, [c_int] * 10 + [P] * 10 + [c_size, P, P]),
    "vq3d_preact_small_fwd_chain": (c_int, [c_int] * 10 + [P] * 13),
    "vq3d_vq_workspace_size": (c_size, [c_i64, c_int, c_int]),
    "vq3d_vq_nearest": (c_int, [c_int, P, c_i64, c_int, P, c_int, P, c_int, P, P, P, P]),
    "vq3d_vq_commit_loss": (c_int, [P, c_float, P, P]),
    "vq3d_vq_bwd": (c_int, [c_int, P, c_i64, c_int, P, P, c_int, P, P, c_float, P, P]),
    "vq3d_vq_ema_stats": (c_int, [c_int, P, c_i64, c_int, P, c_int, P, P, P, P]),
    "vq3d_vq_ema_update": (c_int, [P, P, P, P, P, c_int, c_int, c_float, c_float, P]),
    "vq3d_vq_moments": (c_int, [c_int, P, c_i64, c_int, P, P, P, P]),
    "vq3d_vq_init_apply": (c_int, [P, P, P, P, P, P, c_int, c_int, c_float, c_float, P]),
    "vq3d_parse_input_fwd": (c_int, [c_int, c_i64, c_int, P, P, P, P, P]),
    "vq3d_parse_input_workspace_bytes": (c_size, [c_i64, c_int]),
    "vq3d_parse_input_bwd": (c_int, [c_int, c_i64, c_int, P, P, P, P, P, c_size, P]),
    "vq3d_recon_loss_workspace_size": (c_size, [c_int] * 4),
    "vq3d_recon_loss_fwd": (c_int, [c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P]),
    "vq3d_recon_loss_bwd": (c_int, [c_int, P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P]),
    "vq3d_cylinder_count": (c_i64, [c_int, c_int]),
    "vq3d_evonorm_workspace_size": (c_size, [c_int, c_i64]),
    "vq3d_evonorm_fwd": (c_int, [c_int, P, c_int, c_i64, P, P, P, P, P, P, P]),
    "vq3d_evonorm_bwd": (c_int, [c_int, P, P, c_int, c_i64, P, P, P, P, P, P, P, P, P]),
    "vq3d_adam_amsgrad": (c_int, [P, P, P, P, P, c_i64, c_float, c_float, c_float, c_float, c_i64, P]),
    "vq3d_adam_amsgrad_dev": (c_int, [P, P, P, P, P, c_i64, c_float, c_float, c_float, c_float, P, P, P]),
    "vq3d_grad_unscale": (c_int, [P, c_i64, P, P, P]),
    "vq3d_loss_scale_update": (c_int, [P, P, P, c_float, c_float, c_int, P]),
    "vq3d_cast": (c_int, [c_int, P, c_int, P, c_i64, P]),
    "vq3d_zero": (c_int, [P, c_size, P]),
    "vq3d_copy": (c_int, [P, P, c_size, P]),
    "vq3d_poison_lds": (c_int, [P]),
    "vq3d_scale": (c_int, [P, c_float, c_i64, P]),
    "vq3d_preact_act_fwd": (c_int, [c_int, c_int, c_i64, P, P, P, P, P]),
    "vq3d_preact_act_bwd": (c_int, [c_int, c_int, c_i64, P, P, P, P, P, P, P]),
    "vq3d_scale_bias_res_fwd": (c_int, [c_int, c_i64, P, P, P, P, P, P]),
    "vq3d_scale_bias_res_bwd": (c_int, [c_int, c_i64, P, P, P, P, P, P, P]),
    "vq3d_rows_gemm": (c_int, [c_int, c_i64, c_int, c_int, P, c_i64, P, c_i64, c_int, P, P, c_i64, P]),
    "vq3d_rows_wgrad_workspace_bytes": (c_size, [c_i64, c_int, c_int]),
    "vq3d_rows_wgrad": (c_int, [c_int, c_i64, c_int, c_int, P, c_i64, P, c_i64, P, P, P, c_size, P]),
    "vq3d_causal_attn_supported": (c_int, [c_int] * 3),
    "vq3d_causal_attn_workspace_bytes": (c_size, [c_int] * 3),
    "vq3d_causal_attn_fwd": (c_int, [c_int] * 6 + [c_float] + [P] * 6),
    "vq3d_causal_attn_bwd": (c_int, [c_int] * 6 + [c_float] + [P] * 7 + [c_size] + [P] * 4),
    "vq3d_causal_attn_fwd_ex": (c_int, [c_int] * 6 + [c_float] + [P] * 7),
    "vq3d_causal_attn_bwd_ex": (c_int, [c_int] * 6 + [c_float] + [P] * 8 + [c_size] + [P] * 4),
    "vq3d_elu_bwd_from_output": (c_int, [c_int, P, P, P, c_i64, P]),
    "vq3d_last_error": (ctypes.c_char_p, []),
    "vq3d_version": (ctypes.c_char_p, []),
}

_lib = None


def load():
    """Load libvq3d.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libvq3d.so not found at {LIB_PATH}: run `make -C 3d-vq-vae-2_amd` "
                               "(or __graft_entry__.build()); the HIP path has no fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def declared_symbols():
    return sorted(_SIGS)


class Vq3dError(RuntimeError):
    pass


_fns = {}


def _fn(name):
    f = _fns.get(name)
    if f is None:
        f = _fns[name] = getattr(load(), name)
    return f


def call(name, *args):
    rc = _fn(name)(*args)
    if rc != 0:
        raise Vq3dError(f"{name}: {load().vq3d_last_error().decode()}")
    return rc


def query(name, *args):
    return _fn(name)(*args)


def stream():
    """The current torch (HIP) stream of the current device, as the raw handle (an int: ctypes
    passes it for a void * argument): every launch goes there (graph-capture safe)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise Vq3dError("vq3d ops take GPU tensors only (no CPU path)")
    return t.data_ptr()


def dtype_code(t_or_dtype):
    dt = t_or_dtype.dtype if isinstance(t_or_dtype, torch.Tensor) else t_or_dtype
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float16:
        return F16
    raise Vq3dError(f"unsupported activation dtype {dt}")
