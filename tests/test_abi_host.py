"""CPU: the C-ABI library loads and exports every declared symbol; host-side logic
(descriptor validation, workspace sizing, cylinder count, module API / state_dict layout,
argument parsing) — no GPU compute is called here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import torch

from conftest import ROOT, golden

HEADER = os.path.join(ROOT, "include", "vq3d.h")


def header_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(vq3d_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from vq3d import _lib as L
    lib = L.load()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s
    # the python binding declares exactly the header's entry points
    assert sorted(L.declared_symbols()) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (vq3d_\w+)", out))
    assert exported == set(syms)
    assert b"gfx950" in lib.vq3d_version()


def test_conv_descriptor_validation_and_workspace():
    from vq3d import _lib as L
    from vq3d import ops
    desc, out = ops.conv_desc(torch.float32, 1, 9, 0, 9, 128, 128, 32, ops.ConvGeom(3, 1, 1, True), 2)
    assert out == (128, 128, 32)
    desc, out = ops.conv_desc(torch.bfloat16, 1, 4, 0, 4, 512, 512, 128, ops.ConvGeom(4, 2, 1, True), 2)
    assert out == (256, 256, 64)
    bad = L.ConvDesc(dtype=0, batch=1, cin=4, cin2=0, cout=4, in_h=8, in_w=8, in_d=8, out_h=9, out_w=8, out_d=8,
                     kernel=3, stride=1, pad=1, pad_mode=1, pro_kind=0)
    rc = L.load().vq3d_conv3d_fwd(ctypes.byref(bad), None, None, None, None, None, None, None, None, 0, None)
    assert rc < 0 and b"output size" in L.load().vq3d_last_error()
    # a null pointer is refused before any launch
    good = L.ConvDesc(dtype=0, batch=1, cin=4, cin2=0, cout=4, in_h=8, in_w=8, in_d=8, out_h=8, out_w=8, out_d=8,
                      kernel=3, stride=1, pad=1, pad_mode=1, pro_kind=0)
    rc = L.load().vq3d_conv3d_fwd(ctypes.byref(good), None, None, None, None, None, None, None, None, 0, None)
    assert rc < 0 and b"null" in L.load().vq3d_last_error()
    # workspace sizes (host-only planning): the 1x1 weight gradient keeps per-workgroup partials,
    # the k^3 MFMA engine its packed bf16 weight fragments
    d3 = L.ConvDesc(dtype=1, batch=1, cin=9, cin2=0, cout=9, in_h=128, in_w=128, in_d=32, out_h=128, out_w=128,
                    out_d=32, kernel=3, stride=1, pad=1, pad_mode=1, pro_kind=2)
    assert L.query("vq3d_conv3d_workspace_size", ctypes.byref(d3), L.PASS_FWD) > 0
    assert L.query("vq3d_conv3d_workspace_size", ctypes.byref(d3), L.PASS_BWD_DATA) > 0
    d1 = L.ConvDesc(dtype=1, batch=1, cin=18, cin2=0, cout=9, in_h=128, in_w=128, in_d=32, out_h=128, out_w=128,
                    out_d=32, kernel=1, stride=1, pad=0, pad_mode=0, pro_kind=2)
    assert L.query("vq3d_conv3d_workspace_size", ctypes.byref(d1), L.PASS_BWD_WEIGHT) >= 9 * 19 * 4
    d3.dtype = 0  # fp32 k^3 runs on the VALU engine: no scratch
    assert L.query("vq3d_conv3d_workspace_size", ctypes.byref(d3), L.PASS_FWD) == 0


def test_cylinder_count_matches_reference_mask():
    from vq3d import _lib as L
    from vq3d.utils import cylinder_xy_mask
    d = golden("loss")
    assert L.query("vq3d_cylinder_count", 512, 512) == 205859
    assert int(np.unpackbits(d["mask512"]).sum()) == 205859
    assert L.query("vq3d_cylinder_count", 12, 10) == int(d["mask12x10"].sum())
    assert np.array_equal(cylinder_xy_mask((12, 10)).numpy(), d["mask12x10"])


def test_ops_refuse_cpu_tensors():
    from vq3d import _lib as L
    from vq3d import ops
    x = torch.zeros((1, 4, 4, 4, 4)).contiguous(memory_format=torch.channels_last_3d)
    w = torch.zeros((4, 4, 1, 1, 1))
    try:
        ops.conv_fwd(x, w, ops.ConvGeom(1))
    except L.Vq3dError as e:
        assert "GPU" in str(e)
    else:
        raise AssertionError("CPU tensor accepted")


def test_module_api_state_dict_and_init_match_reference():
    import vq3d
    for name, kw in [("model_2l_dflt_32", dict(n_bottleneck_blocks=2)),
                     ("model_2l_blocks_32", dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=1,
                                                 n_post_quantization_blocks=1, n_post_upscale_blocks=1,
                                                 n_post_downscale_blocks=1, num_embeddings=[64, 32])),
                     ("model_2l_regular_32", dict(n_bottleneck_blocks=2, block_type="regular",
                                                  base_network_channels=2)),
                     ("model_2l_evonorm_32", dict(n_bottleneck_blocks=2, block_type="evonorm"))]:
        d = golden(name)
        torch.manual_seed(0)
        m = vq3d.VQVAE(vq3d.default_args(**kw))
        g = torch.Generator().manual_seed(1)
        with torch.no_grad():
            for _, p in sorted(m.named_parameters()):
                p.add_(0.02 * torch.randn(p.shape, generator=g))
        sd = m.state_dict()
        ref = {k[5:]: d[k] for k in d.files if k.startswith("init/")}
        assert set(sd) == set(ref), name
        for k, v in ref.items():
            assert tuple(sd[k].shape) == v.shape and sd[k].dtype == torch.from_numpy(v).dtype, (name, k)
            assert np.array_equal(sd[k].numpy(), v), (name, k)


def test_argparse_defaults_mirror_reference():
    import vq3d
    a = vq3d.default_args()
    assert (a.input_channels, a.base_network_channels, a.n_bottleneck_blocks, a.n_downscales_per_bottleneck) == \
        (1, 4, 3, 2)
    assert a.num_embeddings == [256] and a.block_type == "pre-activation" and a.extract_center_cylinder is True
    assert a.metric == "huber" and a.base_lr == 1e-5
    m = vq3d.VQVAE(vq3d.default_args(n_bottleneck_blocks=2))
    assert sum(p.numel() for p in m.parameters()) == 166281
    assert m.num_layers == 2 + 2 * 4 + 1


def test_library_operators_registered():
    """vq3d.library registers every hot-path operator with a typed schema (no GPU needed)."""
    import torch

    from vq3d import library as lb
    for name in lb.OPS:
        schema = str(getattr(torch.ops.vq3d, name).default._schema)
        assert schema.startswith(f"vq3d::{name}("), schema
    assert "Tensor(a" in str(torch.ops.vq3d.conv3d_backward.default._schema)  # gradient buffers are mutated
