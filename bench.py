#!/usr/bin/env python3
"""Throughput of the 3D VQ-VAE-2 training step (enc + VQ + dec, fwd + bwd + Adam) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3l_pub] [--eager] [--encode-only]

N > 1 runs one process per GPU (RCCL); each rank trains on its own synthetic 512x512x128 volume
(weak scaling: batch 1 per GPU, BASELINE.json configs[2]).  Started bare (`python bench.py --gpus
N`), the script launches its own N ranks -- `python -m torch.distributed.run --nproc-per-node N
bench.py ...` as a child process, before anything imports torch or touches a GPU (vq3d/launch.py,
the reference's gpus=-1 / accelerator='ddp', vqvae/train.py:25-27) -- forwards rank 0's JSON line
and exits with the child's code; under an existing torchrun (WORLD_SIZE set) it is that rank.
Rank 0 prints ONE JSON line.  Default workload = the BASELINE metric's configuration:
3-layer VQ-VAE with the reference's published block counts (50 pre-q / 50 post-q / 3 post-up /
2 post-down, K = 128/256/512, slurm-jobs/train_vqvae_3d.job:76-86), bf16 activations.
--config 2l_pub is BASELINE configs[1] (256x256x128, batch 2); --encode-only is configs[3]
(eval encode + codebook search per volume, the extract_embeddings.py path).

The line carries:
  roofline       the dominant kernel of the step -- the top kernel of the step's own rocprofv3
                 kernel-time ranking (profiles/rNN_step_top.json of the newest round, tools/step_profile.py) that has
                 a probe below -- launched alone on resident inputs and timed with HIP events on
                 its stream; achieved = algorithmic bytes / average launch time; traffic = PMC HBM
                 bytes per launch (profiles/rNN_pmc_<kernel>.json, tools/gpu_traffic.sh) when collected
  roofline_top   the same for the top probe-able kernels of the ranking
  step_conv_roofline_frac  the per-layer conv roofline of the whole step (SURVEY.md 8(d):
                 5.55 ms per 3L-pub volume) / the measured step time
  cpu_baseline   the CPU oracle (oracle/vqvae_cpu.py) on this host: warm-up + median of 3 steps
                 on a bounded sample volume, scaled by voxel count
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (model kwargs, volume (H, W, D), batch per GPU, conv-roofline ms per volume)
    "3l_pub": (dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
                    n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512]),
               (512, 512, 128), 1, 5.55),
    "3l_dflt": (dict(n_bottleneck_blocks=3, num_embeddings=[256]), (512, 512, 128), 1, 1.97),
    "2l_pub": (dict(n_bottleneck_blocks=2, n_pre_quantization_blocks=150, n_post_quantization_blocks=150,
                    n_post_upscale_blocks=5, n_post_downscale_blocks=5, num_embeddings=[128, 256]),
               (256, 256, 128), 2, 2.52),
    "2l_dflt": (dict(n_bottleneck_blocks=2, num_embeddings=[256]), (256, 256, 128), 2, 0.49),
}
ENC_ROOF_MS = {"3l_pub": 0.42, "3l_dflt": 0.27}  # encoder-only fwd roofline per volume
ENC_BYTES = {"3l_pub": 3.39e9, "3l_dflt": 2.19e9}
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFS = 2500.0  # dense bf16
ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # newest first: committed profiles of the most recent round win
STEP_TOP = next((p for p in (os.path.join(ROOT, "profiles", f"{r}_step_top.json") for r in ROUNDS)
                 if os.path.exists(p)), os.path.join(ROOT, "profiles", "r02_step_top.json"))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="3l_pub", choices=sorted(CONFIGS))
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"],
                   help="activation / matrix-core format: bf16 (BASELINE's), fp16 (the reference's AMP, with dynamic "
                        "loss scaling) or fp32")
    p.add_argument("--size", type=int, nargs=3, default=None, help="override the volume H W D")
    p.add_argument("--encode-only", action="store_true", help="eval encode + codebook search (configs[3])")
    p.add_argument("--encode-batch", type=int, default=1,
                   help="--encode-only: volumes per encode call (codes are per volume whatever the batch)")
    p.add_argument("--prior", action="store_true",
                   help="PixelSNAIL mid-level prior training step (configs[4]) instead of the VQ-VAE step")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-roofline", action="store_true")
    p.add_argument("--profile-steps", action="store_true", help="print per-step times to stderr")
    p.add_argument("--concurrent-wgrad", action="store_true",
                   help="run weight gradients on a side stream, overlapped with backward-data (measured "
                        "0.3 ms/step slower than serial on the 3L-pub step now that the big blocks are fused)")
    p.add_argument("--no-overlap-levels", action="store_true",
                   help="run the decoder's top-level chain on the main stream (default: on the level stream, "
                        "beside the encoder's lower levels)")
    p.add_argument("--no-small-chain", action="store_true",
                   help="unchained column-kernel runs (each block forms its t2 / gz3 on its bricks' halos)")
    p.add_argument("--eager", action="store_true",
                   help="launch every kernel from Python each step instead of replaying a captured HIP graph")
    p.add_argument("--no-dist-graph", action="store_true", help="N > 1: never capture the collectives")
    p.add_argument("--cpu-plumbing", action="store_true",
                   help="tests only: exercise the rank launch / barrier / max-over-ranks / JSON plumbing on CPU "
                        "ranks over gloo with a stand-in step (one all-reduce of a gradient-sized buffer); no model")
    p.add_argument("--binding", default="ctypes", choices=["ctypes", "library"],
                   help="library: the layers call the registered torch.ops.vq3d.* operators (vq3d.library) "
                        "instead of the ctypes autograd Functions (same kernels)")
    return p.parse_args()


# ---------------------------------------------------------------------------------------------- kernel probes
def _mid_block(dev, seed=7):
    import torch

    from vq3d import layers as VL
    from vq3d.flat import FlatParams
    torch.manual_seed(seed)
    blk = VL.PreActFixupResBlock(18, 18, mode="same").to(dev)
    FlatParams(blk.parameters(), dev)
    with torch.no_grad():
        for p in blk.parameters():
            p.normal_(0, 0.2)
    g = torch.Generator(device=dev).manual_seed(seed)
    shape = (1, 18, 128, 128, 32)
    x = (torch.randn(shape, device=dev, generator=g) * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last_3d)
    gy = (torch.randn(shape, device=dev, generator=g) * 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last_3d)
    return blk, x, gy


def probe_mid(dev, kind):
    """Kernels of the fused 18-channel / branch-9 block at 128x128x32 (the decoder's 50 bottom-level
    post-quantize blocks), launched alone through vq3d_preact_mid_*_stages."""
    import torch

    from vq3d import _lib as L
    from vq3d import ops
    blk, x, gy = _mid_block(dev)
    nv = 128 * 128 * 32
    out, t2, t3 = ops.preact_mid_fwd(x, blk)
    grads = {n: p.grad for n, p in (("dw1", blk.branch_conv1.weight), ("dw2", blk.branch_conv2.weight),
                                    ("dw3", blk.branch_conv3.weight), ("dbias1a", blk.bias1a),
                                    ("dbias1b", blk.bias1b), ("dbias2a", blk.bias2a), ("dbias2b", blk.bias2b),
                                    ("dbias3a", blk.bias3a), ("dbias3b", blk.bias3b), ("dscale", blk.scale),
                                    ("dbias4", blk.bias4))}
    gx = torch.empty_like(x)
    ws = ops.workspace(L.query("vq3d_preact_mid_workspace_bytes", 1, 128, 128, 32), dev)
    ops.preact_mid_bwd(gy, x, t2, t3, blk, grads, bufs=(gx, ws))
    wb = (18 * 9 * 2 + 9 * 9 * 27) * 4
    fl_pw, fl_k3 = 2.0 * nv * 18 * 9, 2.0 * nv * 9 * 9 * 27
    # the step runs 49 of a run's 50 blocks through the CHAINED tile kernels (vq3d.h *_chain): the
    # probes launch those, with the same block standing in as its own neighbour
    import ctypes
    dc, w1, w2, w3 = L.dtype_code(x), blk.branch_conv1.weight, blk.branch_conv2.weight, blk.branch_conv3.weight
    prm = ops._preact_params(blk)
    t2n = torch.empty_like(t2)
    nws = L.query("vq3d_preact_mid_workspace_bytes", 1, 128, 128, 32)
    wsp = ops.workspace(nws, dev)
    gr = L.PreactGrads(*[ops._p(grads.get(n)) for n, _ in L.PreactGrads._fields_])

    def fwd_chain():
        L.call("vq3d_preact_mid_fwd_chain", dc, 1, 18, 9, 128, 128, 32, L.ptr(x), L.ptr(w2), L.ptr(w3),
               ctypes.byref(prm), L.ptr(t2), L.ptr(out), L.ptr(t3), L.ptr(w1), ctypes.byref(prm), L.ptr(t2n),
               L.stream())

    def bwd_chain():
        L.call("vq3d_preact_mid_bwd_chain", 2, dc, 1, 18, 9, 128, 128, 32, L.ptr(gy), L.ptr(x), L.ptr(t2),
               L.ptr(t3), L.ptr(w1), L.ptr(w2), L.ptr(w3), ctypes.byref(prm), ctypes.byref(gr), L.ptr(ws),
               ctypes.c_size_t(nws), L.ptr(gx), L.ptr(t3), L.ptr(w3), ctypes.byref(prm), L.ptr(wsp),
               ctypes.c_size_t(nws), L.stream())
    if kind == "k_pm_fwd":  # reads t2 9 (halo) + x 18, writes t3 9 + out 18 + the next block's t2 9
        return (fwd_chain, nv * 63 * 2 + wb, fl_k3 + 2 * fl_pw,
                "k_pm_fwd (chained): fused 18-ch block t3 + out (3x3x3 9->9 + 1x1 9->18 + residual) + next "
                "block's t2 (1x1 18->9) @128x128x32 bf16")
    if kind == "k_pm_t2":
        return (lambda: ops.preact_mid_fwd(x, blk, stages=1, bufs=(out, t2, t3)), nv * 27 * 2 + wb, fl_pw,
                "k_pm_t2: fused 18-ch block t2 (1x1 18->9 + elu) @128x128x32 bf16")
    if kind == "k_pm_bwd2":  # reads gz3 9 + t2 9 + x 18 + g 18 + prev t3 9, writes gx 18 + gz1 9 + prev gz3 9
        return (bwd_chain, nv * 99 * 2 + wb, fl_k3 + 2 * fl_pw,
                "k_pm_bwd2 (chained): fused 18-ch block backward data tile (dgrad 3x3x3 + 1x1 dgrad) + previous "
                "block's gz3 (1x1 18->9 dgrad) @128x128x32")
    if kind == "k_pm_w2grad":  # reads gz3 9 + t2 9 (halo re-reads are L2 traffic), writes partials
        return (lambda: ops.preact_mid_bwd(gy, x, t2, t3, blk, grads, stages=4, bufs=(gx, ws)), nv * 18 * 2 + wb,
                fl_k3, "k_pm_w2grad: fused 18-ch block 3x3x3 9->9 weight gradient @128x128x32")
    if kind == "k_pm_w13grad":  # reads gz1 9 + t3 9 + x 18 + g 18
        return (lambda: ops.preact_mid_bwd(gy, x, t2, t3, blk, grads, stages=8, bufs=(gx, ws)), nv * 54 * 2 + wb,
                2 * fl_pw, "k_pm_w13grad: fused 18-ch block 1x1 weight gradients (W1, W3) @128x128x32")
    if kind == "k_pm_bwd1":  # reads g 18 + t3 9, writes gz3 9
        return (lambda: ops.preact_mid_bwd(gy, x, t2, t3, blk, grads, stages=1, bufs=(gx, ws)), nv * 36 * 2 + wb,
                2 * fl_pw, "k_pm_bwd1: fused 18-ch block backward pointwise (gz3 + W3 grad) @128x128x32")
    raise KeyError(kind)


def probe_stack(dev, kind):
    """The fused run of 50 top-level blocks (8x8x2, 32 channels, branch 16, bf16) through
    vq3d_preact_stack_fwd (one launch) / vq3d_preact_stack_bwd_ws (chain + weight-gradient launch)."""
    import torch

    from vq3d import _lib as L
    from vq3d import layers as VL
    from vq3d.flat import FlatParams
    from vq3d.functional import StackPlan
    torch.manual_seed(3)
    nblk, c, nb, shp = 50, 32, 16, (8, 8, 2)
    stack = VL.BlockStack(*[VL.PreActFixupResBlock(c, c, mode="same") for _ in range(nblk)]).to(dev)
    FlatParams(stack.parameters(), dev)
    with torch.no_grad():
        for p in stack.parameters():
            p.normal_(0, 0.05)
    cl = torch.channels_last_3d
    x = torch.randn((1, c) + shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    gy = torch.randn((1, c) + shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    out, gx = torch.empty_like(x), torch.empty_like(x)
    plan = StackPlan(list(stack))
    ptab, gtab = plan.tables(dev)
    dims = (L.dtype_code(x), nblk, 1, c, nb) + shp
    saved = torch.empty(L.query("vq3d_preact_stack_saved_floats", *dims[1:]), dtype=torch.float32, device=dev)

    def fwd():
        L.call("vq3d_preact_stack_fwd", *dims, L.ptr(x), L.ptr(ptab), L.ptr(out), L.ptr(saved), L.stream())

    nws = L.query("vq3d_preact_stack_bwd_workspace_bytes", *dims[1:])
    ws = torch.empty(max(nws, 256), dtype=torch.uint8, device=dev)

    def bwd():
        L.call("vq3d_preact_stack_bwd_ws", *dims, L.ptr(gy), L.ptr(ptab), L.ptr(gtab), L.ptr(saved), L.ptr(gx),
               L.ptr(ws), ws.numel(), L.stream())
    fwd()
    nv = 128
    wbytes = nblk * (c * nb * 2 + nb * nb * 27 + 8) * 4
    # the residual stream and saved branch tensors stay in the kernel's LDS / L2; HBM sees the
    # weights, the saved-tensor round trip (fp32) and the bf16 input / output
    sv = saved.numel() * 4
    flops = nblk * 2.0 * nv * (c * nb * 2 + nb * nb * 27)
    if kind == "k_stackr_fwd":
        return fwd, wbytes + sv + 2 * nv * c * 2, flops, \
            "k_stackr_fwd: 50 fused top-level blocks (8x8x2, 32 ch) forward, one launch"
    if kind == "k_stackr_bwd":
        return bwd, 2 * wbytes + sv + 2 * nv * c * 2, 2 * flops, \
            "k_stackr_bwd: 50 fused top-level blocks (8x8x2, 32 ch) backward: the gradient-stream chain (one " \
            "workgroup) + the weight gradients (one workgroup per block)"
    raise KeyError(kind)


def probe_col(dev, kind):
    """The few-channel column block kernels (preact_col.hip) at their production shapes: (4, 2) at
    512x512x128 (decoder post-upscale blocks), (8, 4) at 256x256x64, (2, 1) at 128x128x32."""
    import torch

    from vq3d import _lib as L
    from vq3d import layers as VL
    from vq3d import ops
    from vq3d.flat import FlatParams
    c = {"4_2": 4, "8_4": 8, "2_1": 2}[kind.split("<")[-1]] if "<" in kind else 4
    shp = {4: (512, 512, 128), 8: (256, 256, 64), 2: (128, 128, 32)}[c]
    if kind.startswith("k_small"):  # the brick kernels: (8, 4) at the 32x32x8 pre-quantize level
        shp = (32, 32, 8)
    torch.manual_seed(5)
    blk = VL.PreActFixupResBlock(c, c, mode="same").to(dev)
    FlatParams(blk.parameters(), dev)
    with torch.no_grad():
        for p in blk.parameters():
            p.normal_(0, 0.2)
    cl = torch.channels_last_3d
    x = torch.randn((1, c) + shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    gy = torch.randn((1, c) + shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    out, t2, t3 = ops.preact_small_fwd(x, blk)
    grads = {n: p.grad for n, p in (("dw1", blk.branch_conv1.weight), ("dw2", blk.branch_conv2.weight),
                                    ("dw3", blk.branch_conv3.weight), ("dbias1a", blk.bias1a),
                                    ("dbias1b", blk.bias1b), ("dbias2a", blk.bias2a), ("dbias2b", blk.bias2b),
                                    ("dbias3a", blk.bias3a), ("dbias3b", blk.bias3b), ("dscale", blk.scale),
                                    ("dbias4", blk.bias4))}
    nv = shp[0] * shp[1] * shp[2]
    nb = c // 2
    fl = 2.0 * nv * (c * nb * 2 + nb * nb * 27)
    kn = kind.split("_")[1]
    if kind.startswith(("k_col_fwd", "k_small_fwd")):  # reads x c, writes out c + t2 nb + t3 nb
        return (lambda: ops.preact_small_fwd(x, blk), nv * (2 * c + 2 * nb) * 2, fl,
                f"k_{kn}_fwd<{c},{nb}>: fused few-channel block forward @{shp[0]}x{shp[1]}x{shp[2]}")
    # reads g c + x c + t2 nb + t3 nb, writes gx c (+ per-brick partial rows)
    return (lambda: ops.preact_small_bwd(gy, x, t2, t3, blk, grads), nv * (3 * c + 2 * nb) * 2, 2 * fl,
            f"k_{kn}_bwd<{c},{nb}>: fused few-channel block backward + reduction @{shp[0]}x{shp[1]}x{shp[2]}")


def probe_wgrad(dev, kind):
    """The generic k^3 weight-gradient engine (conv_mfma.inc k_wgrad_mfma) on the unfused
    (16, 8)-block branch conv of the 128x128x32 level: 8 -> 8, 3x3x3 circular, bf16."""
    import torch

    from vq3d import ops
    cl = torch.channels_last_3d
    shp = (1, 8, 128, 128, 32)
    x = torch.randn(shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    g = torch.randn(shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn((8, 8, 3, 3, 3), device=dev)
    dw = torch.zeros_like(w)
    nv = 128 * 128 * 32
    geom = ops.ConvGeom(3, 1, 1, True)
    return (lambda: ops.conv_bwd(g, x, w, geom, want_gx=False, dw=dw), nv * 16 * 2, 2.0 * nv * 27 * 64,
            "k_wgrad_mfma<8,1,4>: 3x3x3 8->8 circular weight gradient @128x128x32 bf16")


def probe_pw(dev, kind):
    """Full-resolution 1x1x1 convs of the published model's first down / last up block (512x512x128,
    bf16): k_pw_rows 4 -> 4 with the PreAct prologue elu(x + a) + b and the next conv's ELU_AFFINE
    epilogue (down block conv1), k_pw2 4 -> 4 with scale / bias and the half-grid skip upsampled
    on the fly as residual (up block conv3)."""
    import torch

    from vq3d import ops
    cl = torch.channels_last_3d
    shp = (1, 4, 512, 512, 128)
    x = torch.randn(shp, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn((4, 4, 1, 1, 1), device=dev) * 0.3
    sc = [torch.full((1,), v, device=dev) for v in (0.1, 0.2, 0.3, 0.4)]
    y = torch.empty_like(x)
    nv = 512 * 512 * 128
    g1 = ops.ConvGeom(1)
    if kind.startswith("k_pw_rows"):
        return (lambda: ops.conv_fwd(x, w, g1, pro=(sc[0], sc[1]), act=(sc[2], sc[3]), out=y), nv * 8 * 2,
                2.0 * nv * 16, "k_pw_rows<4,4>: 1x1 4->4 + prologue + ELU_AFFINE epilogue @512x512x128")
    res = torch.randn((1, 4, 256, 256, 64), device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    return (lambda: ops.conv_fwd(x, w, g1, scale=sc[0], bias=sc[1], residual=res, residual_up2=True, out=y),
            nv * 8 * 2 + nv // 8 * 4 * 2, 2.0 * nv * 16,
            "k_pw2<4>: 1x1 4->4 + scale / bias + upsampled half-grid residual @512x512x128")


def probe_s2(dev, kind):
    """Stride-2 backward-data (conv_s2.hip) of the first down block's branch conv2: 4x4x4 stride 2
    circular 4 -> 4, g on 256x256x64, gx on 512x512x128 with the activated-aux derivative."""
    import torch

    from vq3d import ops
    cl = torch.channels_last_3d
    x = torch.randn((1, 4, 512, 512, 128), device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    g = torch.randn((1, 4, 256, 256, 64), device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn((4, 4, 4, 4, 4), device=dev) * 0.2
    b = torch.full((1,), 0.1, device=dev)
    dpre, dpost = torch.zeros(1, device=dev), torch.zeros(1, device=dev)
    nv = 512 * 512 * 128
    geom = ops.ConvGeom(4, 2, 1, True)
    return (lambda: ops.conv_bwd(g, x, w, geom, aux=x, aux_b=b, dpro_pre=dpre, dpro_post=dpost),
            nv * 4 * 2 * 2 + nv // 8 * 4 * 2, 2.0 * nv * 8 * 16,
            "k_dgrad_s2<4,4>: 4x4x4 stride-2 4->4 backward-data + activated-aux derivative @512x512x128")


def probe_wgrad_s2(dev, kind):
    """The generic k^3 weight-gradient engine on a down block's branch conv2: 4x4x4 stride 2
    circular 9 -> 9 from 256x256x64 to 128x128x32, bf16."""
    import torch

    from vq3d import ops
    cl = torch.channels_last_3d
    x = torch.randn((1, 9, 256, 256, 64), device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    g = torch.randn((1, 9, 128, 128, 32), device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn((9, 9, 4, 4, 4), device=dev)
    dw = torch.zeros_like(w)
    nv = 128 * 128 * 32
    geom = ops.ConvGeom(4, 2, 1, True)
    return (lambda: ops.conv_bwd(g, x, w, geom, want_gx=False, dw=dw), (nv * 8 + nv) * 9 * 2, 2.0 * nv * 64 * 81,
            "k_wgrad_mfma<16,1,14>: 4x4x4 stride-2 9->9 circular weight gradient 256^2x64 -> 128^2x32 bf16")


PROBES = {
    "k_wgrad_mfma<16_1_14": probe_wgrad_s2,
    "k_dgrad_s2<4_4": probe_s2,
    "k_pw_rows<4_4": probe_pw, "k_pw2<4": probe_pw,
    "k_wgrad_mfma<8_1_4": probe_wgrad,
    "k_col_bwd<4_2": probe_col, "k_col_fwd<4_2": probe_col, "k_col_bwd<8_4": probe_col, "k_col_fwd<8_4": probe_col,
    "k_col_bwd<2_1": probe_col, "k_col_fwd<2_1": probe_col, "k_small_bwd<8_4": probe_col, "k_small_fwd<8_4": probe_col,
    "k_pm_bwd2": probe_mid, "k_pm_w2grad": probe_mid, "k_pm_w13grad": probe_mid, "k_pm_fwd": probe_mid, "k_pm_bwd1": probe_mid, "k_pm_t2": probe_mid,
    "k_stackr_bwd": probe_stack, "k_stackr_fwd": probe_stack,
}


# probes whose kernels are bounded by a chain of dependent phases on one workgroup, not by HBM
# (no HBM roofline applies: a few MB per launch).  Their bound is the compute waves' instruction
# issue: 4 compute waves, one per SIMD, each issuing ~490 (forward) / ~550 (backward) instructions
# per block (tools/probes/loop_mix.py), a VALU instruction per 4 cycles -> a floor of ~0.9 us per
# block; measured ~1.7 / 2.3 us per block (profiles/r06_stack_phase_probe.txt, PMC in
# profiles/r06_stack_pmc.txt: VALU busy ~45 % of the chain, the rest dependent MFMA / LDS latency)
LATENCY_BOUND = {k: "one workgroup walks the 50-block top-level run (8x8x2 voxels, 32 channels) with one barrier per "
                    "block: bounded by its compute waves' instruction issue (~0.9 us per block floor at one VALU "
                    "instruction per 4 cycles per SIMD), not by HBM"
                 for k in ("k_stackr_bwd", "k_stackr_fwd")}


def probe_for(name):
    n = name.replace(", ", "_")
    for k in PROBES:
        if "<" in k:  # shape-keyed probes: k_col_bwd<4_2 matches "k_col_bwd<4, 2>"
            if k + ">" in n:
                return k
            continue
        if k + "<" in name or name.endswith(k) or (k + " ") in name or k == name.split("::")[-1].split("<")[0]:
            return k
    return None


def timed_launch(dev, launch, iters=20):
    """Average launch time: `iters` back-to-back launches captured in a HIP graph, HIP events
    on the replay stream (no host gaps)."""
    import torch
    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            for _ in range(iters):
                launch()
    graph.replay()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    graph.replay()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / 1e3 / iters


def roofline_of(dev, kind, step_entry=None, live_us=None):
    """Roofline of one engine kernel.  Its launch time is taken, in order of preference, from
    (1) the committed rocprofv3 kernel trace of the bench step (profiles/rNN_step_top.json, the
        same tree: `tools/gpu_steps.sh TAG prof` writes it from this command's step) average,
    (2) `live_us`: HIP events around each of its launches inside one more (eager) training step of
        this run (vq3d.ops.KernelTimer, on the stream the kernel is launched on; the events keep
        neighbouring launches from overlapping, so it reads a few % above the trace),
    (3) the isolated probe (the kernel alone on resident inputs of its production shape, 20 launches
        captured in a HIP graph).
    All three are reported (trace_avg_us, live_avg_us, avg_launch_us_isolated / frac_isolated) so
    they can be checked against each other."""
    launch, algo, flops, desc = PROBES[kind](dev, kind)
    t_iso = timed_launch(dev, launch)
    t_trace = step_entry["avg_us"] * 1e-6 if step_entry else None
    if t_trace:
        t, src = t_trace, f"rocprofv3 kernel trace of the bench step ({os.path.relpath(STEP_TOP, ROOT)})"
    elif live_us:
        t, src = live_us * 1e-6, "live: HIP events around each launch inside an eager training step of this run"
    else:
        t, src = t_iso, "isolated probe (HIP-graph replay of 20 launches)"
    achieved = algo / t / 1e9
    traffic = None
    for rnd in ROUNDS:
        pmc = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{kind}.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
            break
    r = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
         "traffic": traffic, "kernel": desc, "avg_launch_us": t * 1e6, "time_source": src,
         "algorithmic_bytes": algo, "tflops": flops / t / 1e12, "mfma_frac_of_peak": flops / t / 1e12 / MFMA_PEAK_TFS,
         "avg_launch_us_isolated": t_iso * 1e6, "frac_isolated": algo / t_iso / 1e9 / HBM_PEAK_GBS}
    if t_trace:
        r["trace_avg_us"] = t_trace * 1e6
        r["frac_trace"] = algo / t_trace / 1e9 / HBM_PEAK_GBS
    if live_us:
        r["live_avg_us"] = live_us
        r["frac_live"] = algo / (live_us * 1e-6) / 1e9 / HBM_PEAK_GBS
    if step_entry:
        r["step_share"] = {"launches_per_step": step_entry["launches"], "us_per_step": step_entry["total_us"],
                           "trace_avg_us": step_entry["avg_us"]}
    return r


def rooflines(dev, live=None, top=5):
    """(dominant, top list, unprobed) from the committed step ranking (by total us per step).
    The dominant kernel is the first ranked kernel with a probe; `unprobed` lists the kernels ranked
    ABOVE it (more us per step) that have no probe.  live(kind) -> in-step average launch us."""
    ranking = []
    if os.path.exists(STEP_TOP):
        ranking = json.load(open(STEP_TOP)).get("by_name", [])
    out, unprobed, latency = [], [], []
    for e in ranking:
        k = probe_for(e["kernel"])
        if k is None:
            if not out:
                unprobed.append({"kernel": e["kernel"], "us_per_step": e["total_us"], "launches": e["launches"]})
            continue
        if k in LATENCY_BOUND:
            # one workgroup walking a 50-block chain: no HBM roofline applies (a few MB per launch,
            # ~0.1 % of HBM); listed with its step share, never as an HBM fraction
            latency.append({"kernel": e["kernel"], "us_per_step": e["total_us"], "launches": e["launches"],
                            "avg_launch_us": e.get("avg_us"), "bound": "latency", "note": LATENCY_BOUND[k]})
            continue
        if any(r.get("probe") == k for r in out):
            continue
        r = roofline_of(dev, k, e, live(k) if (live is not None and not out) else None)
        r["probe"] = k
        out.append(r)
        if len(out) >= top:
            break
    if not out:
        r = roofline_of(dev, "k_pm_bwd2", None, live("k_pm_bwd2") if live is not None else None)
        r["probe"] = "k_pm_bwd2"
        out.append(r)
    return out[0], out, unprobed, latency


# ---------------------------------------------------------------------------------------------- distributed
def host_cores():
    """CPU cores this process may actually use: the affinity mask (what `nproc` prints), capped by
    the cgroup CPU quota when one is set (a GPU box grants a share of a larger machine; nproc
    there counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


# ---------------------------------------------------------------------------------------------- CPU baseline
def cpu_baseline(mkw, size, encode_only=False, sample=(256, 256, 64), reps=3):
    """The CPU oracle (oracle/vqvae_cpu.py, fp32 torch-CPU restatement of the reference step) on
    this host: one warm-up, then the median of `reps` steps of the same model on a sample volume
    with `frac` of the voxels, scaled to volumes/s of the full volume."""
    import torch

    from oracle import vqvae_cpu as O
    # the CPU restatement on all of the host's cores (nproc)
    threads = host_cores()
    torch.set_num_threads(threads)
    import vq3d
    cfg = O.Config(**{k: v for k, v in mkw.items()})
    torch.manual_seed(0)
    ref = vq3d.VQVAE(vq3d.default_args(**mkw))
    sd = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    x = torch.rand((1, 1) + tuple(sample), generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5
    st = {}
    if encode_only:
        def once():
            with torch.no_grad():
                O.encode(cfg, sd, x, train=False)
        for k in [k for k in sd if k.endswith("first_pass")]:
            sd[k].zero_()
    else:
        def once():
            O.train_step(cfg, sd, st, x, [sample[2]], 1e-4)
    once()  # warm-up (first-pass codebook init)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        once()
        ts.append(time.perf_counter() - t0)
    dt = statistics.median(ts)
    frac = (sample[0] * sample[1] * sample[2]) / float(size[0] * size[1] * size[2])
    what = "eval encode" if encode_only else "train step"
    return {"value": frac / dt, "unit": "volumes/s", "cores": threads, "kind": "port",
            "sample": f"oracle {what} (fp32 torch-CPU, same model) on a {sample[0]}x{sample[1]}x{sample[2]} volume "
                      f"= {frac:.4g} of the {size[0]}x{size[1]}x{size[2]} voxels: warm-up + median of {reps} "
                      f"({', '.join(f'{t:.2f}' for t in ts)} s), scaled by voxel count"}


# ---------------------------------------------------------------------------------------------- main
def capture(step, warmup):
    """Capture one call of step() as a HIP graph (after an allocator warm-up on the capture
    stream); returns (graph, static result)."""
    import torch
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step(warmup)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        res = step(warmup + 1)
    torch.cuda.synchronize()
    return graph, res


# PixelSNAIL mid-level prior (BASELINE configs[4]; slurm-jobs/train_pixelsnail_mid_downscaled.job:76-90):
# codes of the 3-layer published model's middle level at 512^2 x 128 (32 x 32 x 8, K = 256),
# model-dim 256, 8 blocks x 5 layers, causal dropout 0.2, attention dropout 0, batch 1
PRIOR = dict(dims=(32, 32, 8), num_embeddings=[256, 0], model_dim=256, num_blocks=8, num_layers_per_block=5,
             causal_dropout_prob=0.2, attention_dropout_prob=0.0, bottleneck_divisor=4, lr=5e-5, mixup_alpha=0.2)


def prior_cpu_baseline(sample=(8, 8, 8), reps=2):
    """oracle/pixelsnail_cpu.py: forward + backward of the same prior (dropout 0) on a bounded
    sample of positions, scaled linearly by position count (the attention's n^2 term makes the
    real CPU cost at 8,192 positions higher: the scaled number flatters the CPU)."""
    import torch

    from oracle import pixelsnail_cpu as O
    from vq3d import pixelsnail as PS
    torch.set_num_threads(host_cores())
    kw = {k: v for k, v in PRIOR.items() if k != "dims"}
    torch.manual_seed(0)
    m = PS.PixelSNAIL(PS.default_args(**kw), compute_dtype="fp32")
    P = {n: p.detach().clone().requires_grad_(True) for n, p in m.named_parameters()}
    data = torch.randint(0, kw["num_embeddings"][0], (1, 1) + sample)
    ts = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        loss, _ = O.loss(P, data, kw["num_embeddings"][0], kw["num_blocks"], kw["num_layers_per_block"])  # no mixup
        loss.backward()
        ts.append(time.perf_counter() - t0)
    t = statistics.median(ts[1:])
    scale = (PRIOR["dims"][0] * PRIOR["dims"][1] * PRIOR["dims"][2]) / (sample[0] * sample[1] * sample[2])
    return {"value": 1.0 / (t * scale), "unit": "samples/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle fwd+bwd (no optimizer) of the same prior on {sample[0]}x{sample[1]}x{sample[2]} codes, "
                      f"median of {reps} after a warm-up ({t:.2f} s), scaled x{scale:.0f} by position count"}


def prior_main(a):
    import torch

    from vq3d import pixelsnail as PS
    from vq3d.flat import FlatParams
    from vq3d.optim import FusedAdam
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    kw = {k: v for k, v in PRIOR.items() if k != "dims"}
    dims = PRIOR["dims"]
    model = PS.PixelSNAIL(PS.default_args(**kw), compute_dtype=a.dtype).to(dev)
    flat = FlatParams(model.parameters(), dev)
    opt = FusedAdam(model.parameters(), flat, lr=kw["lr"], amsgrad=True)
    model.train()
    g = torch.Generator().manual_seed(1)
    data = torch.randint(0, kw["num_embeddings"][0], (1, 1) + dims, generator=g).to(dev)
    codes = data.squeeze(1)
    onehot = torch.nn.functional.one_hot(codes, kw["num_embeddings"][0]).permute(0, 4, 1, 2, 3).contiguous()

    def step(i):
        opt.zero_grad()
        # mixup (--mixup-alpha 0.2 of the published job): the blend and the two-target loss run in the
        # step; lam / index are host draws (train_helpers.py:39-47), fixed in a captured graph
        loss, _ = model.cross_entropy_onehot(onehot.float(), codes, PS.mixup_draw(1, kw["mixup_alpha"]))
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    print("[bench] prior warm-up done", file=sys.stderr, flush=True)
    graph = None
    if not a.eager and a.warmup >= 2:
        graph, static = capture(step, a.warmup)
        print("[bench] prior step captured", file=sys.stderr, flush=True)

        def step(i):  # noqa: F811
            graph.replay()
            return static
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        res = step(a.warmup + i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms = 1000.0 * elapsed / a.steps
    # the attention kernels alone (forward + backward of one stream at the step's shape), HIP
    # events on the launching stream: flops = causal pairs x (fwd 2 (dk + dv) + bwd 2 (2 dk + 2 dv))
    n, c, nh = dims[0] * dims[1] * dims[2], kw["model_dim"] // kw["bottleneck_divisor"], 8
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    q, k, v = (torch.randn((1, c) + dims, device=dev).to(dtype).contiguous(memory_format=torch.channels_last_3d)
               .requires_grad_(True) for _ in range(3))
    gy = torch.randn((1, c) + dims, device=dev).to(dtype).contiguous(memory_format=torch.channels_last_3d)
    for _ in range(3):
        PS.CausalAttentionFn.apply(q, k, v, nh).backward(gy)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    reps = 10
    e0.record(st)
    for _ in range(reps):
        y = PS.CausalAttentionFn.apply(q, k, v, nh)
    e1.record(st)
    for _ in range(reps):
        y.backward(gy, retain_graph=True)
    e2.record(st)
    e2.synchronize()
    tf, tb = e0.elapsed_time(e1) / reps, e1.elapsed_time(e2) / reps
    d = c // nh
    pairs = nh * n * (n + 1) / 2
    res_line = {
        "metric": f"samples/sec (PixelSNAIL prior train step) on {dims[0]}x{dims[1]}x{dims[2]} codes",
        "value": 1000.0 / ms, "unit": "samples/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
        "data": "synthetic codes (uniform over K = 256), reference init weights, seed 0",
        "launch": "hip_graph" if graph is not None else "eager",
        "config": {"workload": "pixelsnail_mid_prior_train_step", "codes": list(dims), "num_embeddings": 256,
                   "model_dim": kw["model_dim"], "blocks_x_layers": [kw["num_blocks"], kw["num_layers_per_block"]],
                   "batch_per_gpu": 1, "global_batch": 1, "parallelism": "dp1", "final_loss": float(res.detach()),
                   "mixup_alpha": kw["mixup_alpha"]},
        "attention_kernel": {"positions": n, "heads": nh, "head_dim": d, "fwd_ms": tf, "bwd_ms": tb,
                             "fwd_tflops": pairs * 4 * d / (tf * 1e-3) / 1e12,
                             "bwd_tflops": pairs * 8 * d / (tb * 1e-3) / 1e12,
                             "note": "matrix-core kernels (16-bit, head dim 8), fp32 online softmax; per stream and block (24 per step)"},
    }
    if not a.no_cpu_baseline:
        print("[bench] prior CPU baseline", file=sys.stderr, flush=True)
        res_line["cpu_baseline"] = prior_cpu_baseline()
    print(json.dumps(res_line), flush=True)


def _launcher():
    """vq3d/launch.py loaded by path: standard library only, so the decision to start ranks is
    taken before the vq3d package (and torch) is imported."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("vq3d_launch", os.path.join(ROOT, "3d-vq-vae-2_amd", "vq3d",
                                                                                "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def timed_steps(step, a, world, dev):
    """The timed region of the contract: barrier + device sync, exactly a.steps steps, barrier +
    device sync; returns (max elapsed seconds over the ranks, last result, per-step seconds)."""
    import torch
    import torch.distributed as dist

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    per, res = [], None
    for i in range(a.steps):
        ts = time.perf_counter()
        res = step(a.warmup + i)
        if a.profile_steps:
            sync()
            per.append(time.perf_counter() - ts)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    return elapsed, res, per


def plumbing_main(a):
    """--cpu-plumbing (tests only): the same launch, timing and reporting path on CPU ranks over
    gloo, with one all-reduce of a 3L-pub-gradient-sized fp32 buffer standing in for the step."""
    import torch
    import torch.distributed as dist

    from vq3d import parallel
    rank, world, _, dev = parallel.init_from_env(backend="gloo")
    if dev.type != "cpu":
        dev = torch.device("cpu")
    buf = torch.full((1 << 16,), float(rank + 1))

    def step(i):
        if world > 1:
            dist.all_reduce(buf)
            buf.div_(world)
        return buf
    for i in range(a.warmup):
        step(i)
    elapsed, res, _ = timed_steps(step, a, world, dev)
    ok = abs(float(res[0]) - (world + 1) / 2.0) < 1e-6
    if rank == 0:
        print(json.dumps({"metric": "launcher plumbing self-test (no model)", "value": world * a.steps / elapsed,
                          "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": 1000.0 * elapsed / a.steps, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "fp32", "data": "stand-in all-reduce on CPU ranks (gloo)",
                          "allreduce_ok": ok,
                          "config": {"workload": "cpu_plumbing", "global_batch": world,
                                     "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("stand-in all-reduce returned the wrong average")


def main():
    a = parse()
    launch = _launcher()
    if a.gpus > 1 and not launch.is_rank_process():
        # bare `bench.py --gpus N`: start the N ranks as a child process (no GPU touched here)
        raise SystemExit(launch.run_ranks(a.gpus, os.path.abspath(__file__), sys.argv[1:], json_only_stdout=True))
    if a.cpu_plumbing:
        return plumbing_main(a)
    if a.prior:
        return prior_main(a)
    import torch
    import torch.distributed as dist

    import vq3d
    from vq3d import ops, parallel
    from vq3d.utils import synthetic_volume

    rank, world, local, dev = parallel.init_from_env()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    mkw, size, batch, roof_ms = CONFIGS[a.config]
    if a.size:
        size = tuple(a.size)
    torch.manual_seed(0)
    ops.set_concurrent_wgrad(a.concurrent_wgrad)
    ops.set_overlap_levels(not a.no_overlap_levels)
    ops.set_small_chain(not a.no_small_chain)
    args = vq3d.default_args(compute_dtype=a.dtype, base_lr=1e-4 * world, **mkw)
    model = vq3d.VQVAE(args).to(dev)
    if a.binding != "ctypes":
        from vq3d import functional as Fn
        Fn.set_binding(a.binding)
    if a.encode_only:
        batch = a.encode_batch
    # this rank's synthetic volumes, resident in HBM before timing
    idx = parallel.shard_indices(0, rank, world, batch)
    x = torch.cat([synthetic_volume((1, 1) + size, i) for i in idx]).to(dev)
    nvs = torch.full((batch,), size[2], dtype=torch.int64, device=dev)
    allreduce = None
    if a.encode_only:
        from vq3d.extract import extract_samples
        model.eval()
        for q in model.encoder.quantize:  # a trained checkpoint's codebooks (no first-pass init in eval)
            q.first_pass.zero_()
            q.first_pass_host = False

        def step(i):
            with torch.no_grad():
                return next(extract_samples(model, [x]))[0]
    else:
        from vq3d.optim import GradScaler
        model.train()
        opt = model.configure_optimizers()
        allreduce = parallel.GradientAllReduce(model)
        # fp16: the reference's native AMP loss scaling (device-resident, captured with the step)
        scaler = GradScaler(dev, enabled=a.dtype == "fp16")

        def step(i):
            opt.zero_grad()
            loss = model.training_step((x, nvs), i)
            scaler.scale(loss).backward()
            allreduce()
            scaler.step(opt)
            scaler.update()
            return loss

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    # Capture one whole step (training: forward, loss, backward, gradient all-reduce, Adam) as a
    # HIP graph after the eager warm-up (the Quantizer's first-pass init happened there) and
    # replay it per step: no Python / launch overhead on the timed path; every replay runs the
    # full step on the resident input; Adam's step count lives on the device.  N > 1: the RCCL
    # collectives are captured too once a probe capture of the same pattern replayed correctly on
    # every rank; otherwise the ranks run eagerly.
    eager_step = step
    graph = None
    use_graph = not a.eager and a.warmup >= 2
    graph_why = "--eager" if a.eager else ("--warmup < 2" if a.warmup < 2 else "whole step captured")
    if use_graph and world > 1:
        # gloo (the one-GPU rank rehearsal) has no graph-capturable collectives: eager there
        if a.no_dist_graph:
            use_graph, graph_why = False, "--no-dist-graph"
        elif dist.get_backend() != "nccl":
            use_graph, graph_why = False, f"backend {dist.get_backend()}: no graph-capturable collectives"
        else:
            why = []
            use_graph = parallel.graph_collectives_ok(dev, why)
            graph_why = ("RCCL capture probe replayed correctly on every rank: collectives captured with the step"
                         if use_graph else "RCCL capture probe failed, eager steps: " + "; ".join(why))
    if use_graph:
        graph, static = capture(step, a.warmup)

        def step(i):  # noqa: F811
            graph.replay()
            return static
    elapsed, res, per = timed_steps(step, a, world, dev)
    if a.profile_steps and rank == 0:
        print("per-step s:", [round(v, 4) for v in per], file=sys.stderr)
    vols = world * batch * a.steps
    ms = 1000.0 * elapsed / a.steps
    if a.encode_only:
        metric = f"volumes/sec (encode+VQ, eval, codes extraction) at {size[0]}x{size[1]}x{size[2]}"
        workload = f"vqvae_{a.config}_encode_extract"
    else:
        metric = f"volumes/sec (enc+VQ+dec fwd+bwd) at {size[0]}x{size[1]}x{size[2]}"
        workload = f"vqvae_{a.config}_train_step"
    res_line = {
        "metric": metric,
        "value": vols / elapsed,
        "unit": "volumes/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": a.dtype,
        "data": "synthetic (torch.rand*4.5-0.5 volumes, reference init weights, seed 0)",
        "launch": "hip_graph" if graph is not None else "eager",
        "launch_reason": graph_why,
        "binding": a.binding,
        "config": {"workload": workload, "volume": list(size), "batch_per_gpu": batch, "global_batch": batch * world,
                   "parallelism": f"dp{world}" if not a.encode_only else f"replicas{world}"},
    }
    if not a.encode_only:
        res_line["config"]["final_loss"] = float(res.detach())
        res_line["step_conv_roofline_frac"] = roof_ms * batch / ms
        res_line["step_conv_roofline"] = {"ms_per_volume": roof_ms, "source": "SURVEY.md 8(d) per-layer conv "
                                          "roofline (bf16 bytes per layer / 8 TB/s, FLOPs / 2.5 PF)"}
    elif a.config in ENC_ROOF_MS:
        # per-volume roofline / bytes times the volumes one step encodes (--encode-batch)
        res_line["step_conv_roofline_frac"] = ENC_ROOF_MS[a.config] * batch / ms
        res_line["encoder_traffic_frac"] = ENC_BYTES[a.config] * batch / (ms / 1e3) / 1e9 / HBM_PEAK_GBS
    if rank == 0 and not a.no_roofline:
        def live(kind):
            """the kernel's average launch time inside one more (eager, untimed) step of this run"""
            if a.encode_only or world > 1:
                return None
            with ops.KernelTimer(kind) as kt:
                eager_step(a.warmup + a.steps)
            torch.cuda.synchronize()
            return kt.avg_us()
        dom, top, unprobed, latency = rooflines(dev, live)
        res_line["roofline"] = dom
        res_line["roofline_top"] = [{k: r[k] for k in ("probe", "frac", "achieved", "avg_launch_us", "time_source",
                                                       "frac_isolated", "tflops", "mfma_frac_of_peak", "traffic")
                                     if k in r} |
                                    ({"us_per_step": r["step_share"]["us_per_step"]} if "step_share" in r else {})
                                    for r in top]
        if unprobed:
            res_line["unprobed_above_dominant"] = unprobed
        if latency:
            res_line["latency_bound"] = latency
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res_line["cpu_baseline"] = cpu_baseline(mkw, size, encode_only=a.encode_only)
    if rank == 0:
        print(json.dumps(res_line), flush=True)
    if allreduce is not None:
        allreduce.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
