"""GPU: no kernel of the training step may depend on LDS it did not write.

Every libvq3d launch of one full training step of the published 3-layer model at the bench size
(512 x 512 x 128, bf16) is preceded by vq3d_poison_lds, which fills the LDS of every CU with
all-ones words (NaN as bf16 and fp32).  A kernel that reads LDS it never wrote -- even only to
multiply it by a zero weight, as the mid engine's chained t2 stage once did -- then yields NaN
or different values.  The loss and the codes of every level must be bit-identical to the same
step without poisoning (the forward is deterministic); the gradient buffer must be finite and
equal up to the summation order of the few weight-gradient kernels that accumulate with fp32
atomics (1e-4 of its largest entry; a stale-LDS read shows up as NaN or O(1) errors)."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _step(gpu, poison):
    sys.path.insert(0, ROOT)
    import bench
    import vq3d
    from vq3d import _lib as L
    from vq3d.utils import synthetic_volume
    mkw, size, batch = bench.CONFIGS["3l_pub"][:3]
    torch.manual_seed(0)
    model = vq3d.VQVAE(vq3d.default_args(compute_dtype="bf16", base_lr=1e-4, **mkw)).to(gpu)
    model.train()
    x = synthetic_volume((1, 1) + size, 0).to(gpu)
    nvs = torch.full((1,), size[2], dtype=torch.int64, device=gpu)
    call = L.call

    def poisoned(name, *args):
        call("vq3d_poison_lds", L.stream())
        return call(name, *args)
    if poison:
        L.call = poisoned
    try:
        model.flat.zero_grad()
        cap = {}
        fwd = model.forward

        def capture(data):
            cap["r"] = fwd(data)
            return cap["r"]
        model.forward = capture
        loss = model.training_step((x, nvs), 0)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        L.call = call
    codes = [c.clone() for c in cap["r"][1][2]]
    return float(loss.detach()), codes, model.flat.grad.clone()


def test_training_step_ignores_stale_lds(gpu):
    l0, c0, g0 = _step(gpu, poison=False)
    l1, c1, g1 = _step(gpu, poison=True)
    assert torch.isfinite(g1).all(), "NaN / inf gradients with poisoned LDS"
    assert l1 == l0, (l0, l1)
    for a, b in zip(c0, c1):
        assert torch.equal(a, b)
    err = float((g1 - g0).abs().max())
    assert err <= 1e-4 * float(g0.abs().max()), err
