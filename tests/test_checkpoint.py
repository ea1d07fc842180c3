"""PL 1.2-layout checkpoints: what the reference's Trainer writes and
`VQVAE.load_from_checkpoint` reads (train.py:56, extract_embeddings.py:45)."""
import numpy as np
import pytest
import torch

from conftest import golden

KEYS = {"epoch", "global_step", "pytorch-lightning_version", "state_dict", "callbacks", "optimizer_states",
        "lr_schedulers", "hparams_name", "hyper_parameters"}


def _model(**kw):
    import vq3d
    torch.manual_seed(0)
    return vq3d.VQVAE(vq3d.default_args(n_bottleneck_blocks=2, n_pre_quantization_blocks=1,
                                        num_embeddings=[64, 32], **kw))


def test_checkpoint_layout_and_roundtrip(tmp_path):
    import vq3d
    from vq3d.checkpoint import load_checkpoint, save_checkpoint
    m = _model()
    # an Adam(amsgrad) state in torch's own layout, as the reference's optimizer holds it
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, amsgrad=True)
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    path = str(tmp_path / "last.ckpt")
    save_checkpoint(path, m, opt, epoch=3, global_step=120)
    ck = load_checkpoint(path)
    assert set(ck) == KEYS
    assert ck["hparams_name"] == "kwargs" and ck["epoch"] == 3 and ck["global_step"] == 120
    assert ck["hyper_parameters"]["args"].n_pre_quantization_blocks == 1
    sd = m.state_dict()
    assert list(ck["state_dict"]) == list(sd)
    for k, v in sd.items():
        assert ck["state_dict"][k].dtype == v.dtype and torch.equal(ck["state_dict"][k], v), k
    st = ck["optimizer_states"][0]
    assert st["param_groups"][0]["amsgrad"] and len(st["state"]) == len(list(m.parameters()))
    m2 = vq3d.VQVAE.load_from_checkpoint(path)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, sd[k]), k
    assert m2.num_embeddings == [64, 32] and m2.n_pre_quantization_blocks == 1
    # keyword overrides replace fields of the saved args (PL passes them to __init__)
    m3 = vq3d.VQVAE.load_from_checkpoint(path, compute_dtype="fp32")
    assert m3.compute_dtype == torch.float32


def test_loads_reference_state_dict_and_pl_callbacks(tmp_path):
    """A checkpoint shaped like the reference Trainer's: reference parameters (golden state
    after one step, incl. Quantizer buffers with first_pass = 0), hyper_parameters as the
    reference's args Namespace (Trainer fields included), a ModelCheckpoint-keyed callbacks
    entry; loads with the weights-only unpickler and restores every tensor bit for bit."""
    import vq3d
    from vq3d.checkpoint import PL_VERSION, _SAFE
    d = golden("encode_2l_blocks_32")
    sd = {k[6:]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith("state/")}
    args = vq3d.default_args(n_bottleneck_blocks=2, n_pre_quantization_blocks=1, n_post_quantization_blocks=1,
                             n_post_upscale_blocks=1, n_post_downscale_blocks=1, num_embeddings=[64, 32])
    del args.compute_dtype  # the reference's args have no such field
    args.gpus, args.precision, args.max_epochs = 1, 16, 1000  # Trainer.add_argparse_args fields
    from pathlib import Path
    args.dataset_path = Path("/data")  # train.py:22 parses it with type=Path
    args.num_workers, args.rescale_input = 5, None  # train.py:20-21
    mc = next(c for c, q in (x for x in _SAFE if isinstance(x, tuple)) if q.endswith("ModelCheckpoint"))
    ck = {"epoch": 0, "global_step": 1, "pytorch-lightning_version": PL_VERSION, "state_dict": sd,
          "callbacks": {mc: {"monitor": "val_recon_loss", "best_model_score": torch.tensor(0.5)}},
          "optimizer_states": [], "lr_schedulers": [], "native_amp_scaling_state": {"scale": 65536.0},
          "hparams_name": "kwargs", "hyper_parameters": {"args": args}}
    path = str(tmp_path / "ref.ckpt")
    # write it as the reference's process would (PL importable there): the callback class is a
    # global of pytorch_lightning.callbacks.model_checkpoint; removed again before loading
    import sys
    import types
    names = ["pytorch_lightning", "pytorch_lightning.callbacks", "pytorch_lightning.callbacks.model_checkpoint"]
    saved = {n: sys.modules.get(n) for n in names}
    try:
        for n in names:
            sys.modules[n] = types.ModuleType(n)
        sys.modules[names[-1]].ModelCheckpoint = mc
        torch.save(ck, path)
    finally:
        for n, v in saved.items():
            if v is None:
                sys.modules.pop(n, None)
            else:
                sys.modules[n] = v
    m = vq3d.VQVAE.load_from_checkpoint(path)
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k]), k
    assert m.compute_dtype == torch.bfloat16
    assert m.hparams["args"].dataset_path == Path("/data")
    q = m.encoder.quantize[0]
    assert not q.first_pass_host and int(q.first_pass) == 0


def test_refuses_arbitrary_pickles(tmp_path):
    from vq3d.checkpoint import load_checkpoint

    class Evil:
        def __reduce__(self):
            return (print, ("executed",))
    path = str(tmp_path / "evil.ckpt")
    torch.save({"state_dict": {}, "x": Evil()}, path)
    with pytest.raises(Exception):
        load_checkpoint(path)


@pytest.mark.gpu
def test_gpu_fused_adam_state_resumes(gpu, tmp_path):
    """Train 2 steps; vs train 1, checkpoint, reload into a fresh model + FusedAdam, train 1:
    the same parameters (the optimizer state crosses the checkpoint in torch Adam's layout)."""
    import vq3d
    from vq3d.checkpoint import load_checkpoint, save_checkpoint
    x = [(torch.rand((1, 1, 32, 32, 32), generator=torch.Generator().manual_seed(40 + i)) * 4.5 - 0.5).to(gpu)
         for i in range(2)]
    nvs = torch.tensor([32], device=gpu)

    def step(m, opt, i):
        opt.zero_grad()
        m.training_step((x[i], nvs), i).backward()
        opt.step()
    a = _model(compute_dtype="fp32").to(gpu)
    oa = a.configure_optimizers()
    step(a, oa, 0)
    path = str(tmp_path / "mid.ckpt")
    save_checkpoint(path, a, oa, global_step=1)
    step(a, oa, 1)
    b = vq3d.VQVAE.load_from_checkpoint(path, map_location=gpu)
    ob = b.configure_optimizers()
    ob.load_state_dict(load_checkpoint(path)["optimizer_states"][0])
    assert ob.step_count == 1
    step(b, ob, 1)
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        assert torch.allclose(va.float(), vb.float(), rtol=1e-5, atol=1e-6), k
