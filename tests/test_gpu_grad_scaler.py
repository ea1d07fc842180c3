"""GPU: the fp16 path's dynamic loss scaling (vq3d.optim.GradScaler, torch.cuda.amp.GradScaler
semantics as PL 1.2.10's native AMP uses them for the reference's precision=16,
vqvae/train.py:32) on its non-finite path: a flagged step leaves parameters, Adam state and
the step count untouched and halves the scale; `growth_interval` clean steps double it; the
state survives a state_dict round trip through a weights-only checkpoint file."""
import io

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(gpu, growth_interval=3):
    from vq3d.flat import FlatParams
    from vq3d.optim import FusedAdam, GradScaler
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s)) for s in ((7, 5), (33,), (4, 4, 3))]
    flat = FlatParams(ps, gpu)
    opt = FusedAdam(ps, flat, lr=1e-2, amsgrad=True)
    sc = GradScaler(gpu, init_scale=2.0 ** 10, growth_interval=growth_interval)
    return flat, opt, sc


def _state(flat, opt):
    return [t.detach().clone() for t in (flat.data, opt.m, opt.v, opt.vmax, opt.step_t)]


def _fill_grad(flat, scale, seed):
    g = torch.Generator(device=flat.grad.device).manual_seed(seed)
    flat.grad.copy_(torch.randn(flat.grad.shape, generator=g, device=flat.grad.device) * scale)


def test_flagged_step_is_skipped_and_scale_backs_off(gpu):
    flat, opt, sc = _setup(gpu)
    s0 = sc.get_scale()
    _fill_grad(flat, s0, 1)
    before = _state(flat, opt)
    sc.step(opt)
    sc.update()
    torch.cuda.synchronize()
    assert int(opt.step_t) == 1 and float(sc.found_inf) == 0.0
    assert not torch.equal(flat.data, before[0])  # a clean step updates
    assert sc.get_scale() == s0 and int(sc.tracker) == 1
    # inject a non-finite gradient value
    _fill_grad(flat, s0, 2)
    flat.grad[5] = float("inf")
    flat.grad[17] = float("nan")
    before = _state(flat, opt)
    sc.step(opt)
    sc.update()
    torch.cuda.synchronize()
    after = _state(flat, opt)
    for a, b in zip(before, after):
        assert torch.equal(a, b), "a flagged step must leave params / m / v / vmax / step count unchanged"
    assert sc.get_scale() == s0 * 0.5 and int(sc.tracker) == 0


def test_growth_after_interval_of_clean_steps(gpu):
    flat, opt, sc = _setup(gpu, growth_interval=3)
    s0 = sc.get_scale()
    for i in range(2):
        _fill_grad(flat, s0, 10 + i)
        sc.step(opt)
        sc.update()
    torch.cuda.synchronize()
    assert sc.get_scale() == s0 and int(sc.tracker) == 2
    _fill_grad(flat, s0, 20)
    sc.step(opt)
    sc.update()
    torch.cuda.synchronize()
    assert sc.get_scale() == 2 * s0 and int(sc.tracker) == 0
    assert int(opt.step_t) == 3


def test_unscaled_update_matches_unit_scale(gpu):
    """The update from a gradient scaled by S equals the update from the unscaled gradient."""
    flat_a, opt_a, sc = _setup(gpu)
    flat_b, opt_b, _ = _setup(gpu)
    s = sc.get_scale()
    _fill_grad(flat_a, s, 3)
    _fill_grad(flat_b, 1.0, 3)
    sc.step(opt_a)
    sc.update()
    opt_b.step()
    torch.cuda.synchronize()
    assert torch.allclose(flat_a.data, flat_b.data, rtol=1e-6, atol=1e-7)


def test_scaler_state_roundtrip(gpu):
    from vq3d.optim import GradScaler
    flat, opt, sc = _setup(gpu)
    _fill_grad(flat, 1.0, 4)
    flat.grad[0] = float("inf")
    sc.step(opt)
    sc.update()
    _fill_grad(flat, 1.0, 5)
    sc.step(opt)
    sc.update()
    sd = sc.state_dict()
    assert set(sd) == {"scale", "growth_factor", "backoff_factor", "growth_interval", "_growth_tracker"}
    buf = io.BytesIO()
    torch.save({"native_amp_scaling_state": sd}, buf)
    buf.seek(0)
    back = torch.load(buf, weights_only=True)["native_amp_scaling_state"]
    sc2 = GradScaler(gpu, init_scale=1.0, growth_interval=99)
    sc2.load_state_dict(back)
    assert sc2.get_scale() == sc.get_scale() == 2.0 ** 9
    assert int(sc2.tracker) == int(sc.tracker) == 1 and sc2.growth_interval == 3
