#!/usr/bin/env python3
"""Precision study (CPU, test infrastructure): how much of the bf16 path's code-index mismatch
against the fp32 reference is the residual-stream storage and how much the bf16 rounding of the
conv OPERANDS, on the published 3-layer model (50 / 50 / 3 / 2 blocks, K = 128 / 256 / 512) at
256 x 256 x 128 with the perturbed weights and volume of tests/test_gpu_bf16_model.py.

The fp32 CPU oracle (oracle/vqvae_cpu.py, pinned to the reference by the golden tests) is run
with rounding hooks:
  * operands: every conv's input and weight rounded to bf16 (or fp16, the reference's own AMP
    dtype), fp32 accumulation -- what the matrix cores see;
  * stream: each residual block's output rounded to bf16 or kept fp32 -- everywhere, or only
    inside the fused runs of the product path (fp32 between the blocks of a run of few-channel /
    18 / 72-channel / tiny-grid blocks, the encoder's pre-quantize runs handing fp32 z to the
    Quantizer, bf16 at every other block boundary).
Printed: the per-level code match (bottom / mid / top) against the unrounded oracle and the
decoded volume's relative MSE.  Output committed as profiles/r03_precision_study.txt.

    python tests/precision_study.py [H W D]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "3d-vq-vae-2_amd"))
from oracle import vqvae_cpu as O  # noqa: E402

import vq3d  # noqa: E402

PUB3 = dict(n_bottleneck_blocks=3, n_pre_quantization_blocks=50, n_post_quantization_blocks=50,
            n_post_upscale_blocks=3, n_post_downscale_blocks=2, num_embeddings=[128, 256, 512])
FUSED = {2, 4, 8, 18, 72}  # channel counts of the fused run engines (and 32 on tiny grids)


def setup(size):
    torch.manual_seed(0)
    m = vq3d.VQVAE(vq3d.default_args(compute_dtype="fp32", base_lr=1e-4, **PUB3))
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for _, p in sorted(m.named_parameters()):
            p.add_(0.02 * torch.randn(p.shape, generator=g))
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    x = torch.rand((1, 1) + size, generator=torch.Generator().manual_seed(1234)) * 4.5 - 0.5
    return sd, x


def run(sd0, x, op_dt=None, stream="fp32", pre_q_fp32=True):
    """stream: 'fp32' (every block output kept), 'bf16' (every block output rounded), 'runs' (kept
    only inside the product's fused runs), 'enc_runs' (only inside the encoder's fused runs)"""
    conv0, seq0, blk0 = O.conv, O._seq, O.BLOCKS["pre-activation"]

    def conv(t, w, *a, **k):
        if op_dt is None:
            return conv0(t, w, *a, **k)
        return conv0(t.to(op_dt).float(), w.to(op_dt).float(), *a, **k)

    def keep(prefix, specs, j, t):
        if stream == "fp32":
            return True
        if stream == "bf16" or (stream == "enc_runs" and not prefix.startswith("encoder.")):
            return False
        ci, co, mode = specs[j]
        fused = mode == "same" and ci == co and (ci in FUSED or (ci == 32 and t[0, 0].numel() <= 256))
        nxt = j + 1 < len(specs) and specs[j + 1] == specs[j]
        return fused and (nxt or (pre_q_fp32 and prefix.startswith("encoder.pre_quantize.")))

    def seq(sd, prefix, t, specs, block):
        for j, (ci, co, mode) in enumerate(specs):
            y = blk0(sd, f"{prefix}{j}.", t, ci, co, mode)
            t = y if keep(prefix, specs, j, t) else y.to(torch.bfloat16).float()
        return t

    def blk(sd, p, t, *a):  # blocks outside a sequence (pre_q): their output leaves as bf16
        y = blk0(sd, p, t, *a)
        return y if stream == "fp32" else y.to(torch.bfloat16).float()

    O.conv, O._seq, O.BLOCKS["pre-activation"] = conv, seq, blk
    try:
        sd = {k: v.clone() for k, v in sd0.items()}
        with torch.no_grad():
            dec, (_, _, idx) = O.forward(O.Config(**PUB3), sd, x, True)
    finally:
        O.conv, O._seq, O.BLOCKS["pre-activation"] = conv0, seq0, blk0
    return idx, dec


def main():
    size = tuple(int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (256, 256, 128)
    torch.set_num_threads(os.cpu_count() or 1)
    sd, x = setup(size)
    t0 = time.time()
    ref, dref = run(sd, x)
    print(f"3-layer published model, {size}, perturbed weights (seed 1), volume seed 1234; fp32 oracle "
          f"forward {time.time() - t0:.1f} s")
    cases = [("bf16 operands, bf16 stream everywhere (round-2 product)", dict(op_dt=torch.bfloat16, stream="bf16")),
             ("bf16 operands, fp32 stream inside the fused runs (round-3 product)",
              dict(op_dt=torch.bfloat16, stream="runs")),
             ("bf16 operands, fp32 stream inside the encoder's fused runs only",
              dict(op_dt=torch.bfloat16, stream="enc_runs")),
             ("bf16 operands, fp32 stream everywhere", dict(op_dt=torch.bfloat16, stream="fp32")),
             ("fp16 operands, fp32 stream everywhere (the reference's AMP)", dict(op_dt=torch.float16, stream="fp32"))]
    for name, kw in cases:
        idx, dec = run(sd, x, **kw)
        match = [float((a == b).float().mean()) for a, b in zip(idx, ref)]
        rm = float(((dec.double() - dref.double()) ** 2).sum() / (dref.double() ** 2).sum())
        print(f"{name:72s} code match bottom / mid / top {100 * match[0]:6.2f} / {100 * match[1]:6.2f} / "
              f"{100 * match[2]:6.2f} %   decoded rel-MSE {rm:.2e}")


if __name__ == "__main__":
    main()
