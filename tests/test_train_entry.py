"""The training entry (vq3d/train.py, mirroring the reference's vqvae/train.py:14-59).

CPU: argument composition and the reference's defaults (train.py:17-40), seed_everything(42),
and the ModelCheckpoint(save_top_k=1, save_last=True) bookkeeping on PL-layout checkpoints.
GPU: two training steps over synthetic NRRD scans through the CT datamodule, then
--resume_from_checkpoint continuing from the saved step with identical restored state."""
import os

import numpy as np
import pytest
import torch

from test_data import _write


def test_parse_arguments_matches_reference_defaults(tmp_path):
    from vq3d import train
    a = train.parse_arguments([str(tmp_path), "--batch-size", "1", "--num-embeddings", "128", "256", "512",
                               "--n-pre-quantization-blocks", "50"])
    assert a.dataset_path == tmp_path and a.batch_size == 1
    assert a.gpus == "-1" and a.accelerator == "ddp" and a.benchmark is True and a.precision == 16
    assert a.num_sanity_val_steps == 0 and a.log_every_n_steps == 50 and a.val_check_interval == 0.5
    assert a.max_epochs == int(1e5) and a.weights_summary == "full" and a.flush_logs_every_n_steps == 100
    assert a.num_embeddings == [128, 256, 512] and a.n_pre_quantization_blocks == 50
    assert a.block_type == "pre-activation" and a.base_lr == 1e-5 and a.rescale_input is None


def test_seed_everything_is_reproducible():
    from vq3d import train
    train.seed_everything(42)
    a = (np.random.rand(), torch.rand(3))
    train.seed_everything(42)
    b = (np.random.rand(), torch.rand(3))
    assert a[0] == b[0] and torch.equal(a[1], b[1]) and os.environ["PL_GLOBAL_SEED"] == "42"


def test_checkpointer_keeps_best_and_last(tmp_path):
    import vq3d
    from vq3d import train
    from vq3d.checkpoint import load_checkpoint
    m = vq3d.VQVAE(vq3d.default_args(n_bottleneck_blocks=2))
    ck = train.Checkpointer(tmp_path)
    ck(m, None, 0, 10, 0.5)
    ck(m, None, 0, 20, 0.7)   # worse: best stays at step 10
    ck(m, None, 1, 30, 0.3)   # better: replaces the old best file
    files = sorted(p.name for p in tmp_path.iterdir())
    assert files == ["epoch=1-step=30.ckpt", "last.ckpt"]
    last = load_checkpoint(str(tmp_path / "last.ckpt"))
    # PL 1.2.10 dump_checkpoint: global_step + 1, epoch + 1 (max_steps not reached)
    assert last["global_step"] == 31 and last["epoch"] == 2
    assert last["callbacks"]["ModelCheckpoint"]["best_model_score"] == 0.3
    ck(m, None, 1, 40, None, max_steps=40)   # max_steps reached: the epoch is not advanced
    last = load_checkpoint(str(tmp_path / "last.ckpt"))
    assert last["global_step"] == 41 and last["epoch"] == 1


def test_pl_counter_convention_round_trip():
    """A checkpoint the reference's PL 1.2.10 Trainer wrote mid-epoch 5 at global_step 99 holds
    epoch 6 / global_step 100 and resumes at epoch 6, step 100 -- here as in PL -- and a
    checkpoint written here resumes in PL at the same place."""
    from argparse import Namespace

    from vq3d import train
    ep, gs = train.pl_checkpoint_counters(5, 99)
    assert (ep, gs) == (6, 100)
    pl_dict = {"epoch": 6, "global_step": 100, "pytorch-lightning_version": "1.2.10", "state_dict": {},
               "callbacks": {}, "optimizer_states": [], "lr_schedulers": [], "hparams_name": "kwargs",
               "hyper_parameters": {"args": Namespace()}}
    assert train.resume_counters(pl_dict) == (6, 100)
    assert train.pl_checkpoint_counters(3, 7, max_steps=7) == (3, 8)
    assert train.pl_checkpoint_counters(3, 6, max_steps=7) == (4, 7)


class _SmallCT:
    """CTDataModule over 32 x 32 scans (its default size filter is the reference's 512 x 512)."""

    def __init__(self, path):
        self.path, self.batch_size, self.num_workers = path, 1, 0

    def setup(self, stage=None):
        from torch.utils.data import Subset

        from vq3d import data as D
        ds = D.CTScanDataset(str(self.path), transform=D.CTTransform(128), size=(32, 32, None),
                             spacing=(0.976, 0.976, 3))
        self.train_dataset, self.val_dataset = Subset(ds, [0, 1]), Subset(ds, [2])


@pytest.mark.gpu
def test_train_two_steps_then_resume(gpu, tmp_path):
    from vq3d import train
    from vq3d.checkpoint import load_checkpoint
    rng = np.random.default_rng(0)
    for i, d in enumerate((20, 40, 24)):
        _write(str(tmp_path / f"scan{i}.nrrd"), rng.integers(-1500, 3000, size=(32, 32, d)).astype(np.int16))
    root = tmp_path / "run"
    base = [str(tmp_path), "--batch-size", "1", "--n-bottleneck-blocks", "2", "--default_root_dir", str(root),
            "--val_check_interval", "1.0", "--log_every_n_steps", "1"]
    model, opt, hist, ck = train.main(train.parse_arguments(base + ["--max_steps", "2"]), datamodule=_SmallCT(tmp_path))
    assert [s for s, _ in hist] == [1, 2] and all(np.isfinite(v) for _, v in hist)
    last = root / "checkpoints" / "last.ckpt"
    saved = load_checkpoint(str(last))
    # PL 1.2.10 counters: global_step = steps done, epoch advanced (resume starts the next epoch)
    assert saved["global_step"] == 2 and saved["epoch"] == 1
    assert ck.best_path and os.path.exists(ck.best_path)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    for k, v in saved["state_dict"].items():
        assert torch.equal(v, sd[k]), k
    m2, opt2, hist2, _ = train.main(train.parse_arguments(base + ["--max_steps", "3", "--resume_from_checkpoint",
                                                                   str(last)]), datamodule=_SmallCT(tmp_path))
    assert [s for s, _ in hist2] == [3]
    st0 = saved["optimizer_states"][0]["state"]
    assert {int(float(v["step"])) for v in st0.values()} == {2}, {float(v["step"]) for v in st0.values()}
    r_st = load_checkpoint(str(last))["optimizer_states"][0]["state"]
    assert opt2.step_count == 3, (opt2.step_count, {float(v["step"]) for v in r_st.values()})
    resumed = load_checkpoint(str(last))
    assert resumed["global_step"] == 3 and resumed["epoch"] == 2


@pytest.mark.gpu
def test_step_graph_replay_matches_eager(gpu):
    """vq3d.graph.StepGraph (what vq3d.train and bench.py run): two eager warm-up steps, the step
    captured once as a HIP graph, then replays with new inputs copied into its static buffers --
    the losses and the trained weights follow the eager run (only fp32-atomic summation order in
    some weight-gradient engines may differ)."""
    import vq3d
    from vq3d.graph import StepGraph

    def run(graph):
        torch.manual_seed(0)
        m = vq3d.VQVAE(vq3d.default_args(n_bottleneck_blocks=2, compute_dtype="bf16", base_lr=1e-3)).to(gpu)
        m.train()
        opt = m.configure_optimizers()

        def step(x, nvs):
            opt.zero_grad()
            loss = m.training_step((x, nvs), 0)
            loss.backward()
            opt.step()
            return loss
        runner = StepGraph(step, warmup=2, enabled=graph)
        losses = []
        for i in range(5):
            x = (torch.rand((1, 1, 32, 32, 32), generator=torch.Generator().manual_seed(10 + i)) * 4.5 - 0.5).to(gpu)
            nvs = torch.tensor([32 - i], device=gpu)
            losses.append(float(runner(x, nvs)))
        torch.cuda.synchronize()
        return losses, m.flat.data.clone(), runner
    le, we, _ = run(False)
    lg, wg, r = run(True)
    assert len(r.graphs) == 1
    assert np.allclose(le, lg, rtol=2e-3), (le, lg)
    assert float((we - wg).abs().max()) <= 1e-3 * float(we.abs().max())


class _SmallCTWorkers(_SmallCT):
    """The same scans through a DataLoader with worker processes and a pin-memory thread that keep
    prefetching while the training thread captures its step graph."""

    def __init__(self, path):
        super().__init__(path)
        self.num_workers = 2


@pytest.mark.gpu
def test_train_graph_capture_with_prefetching_loader(gpu, tmp_path):
    """vq3d.train with --hip-graph 1 (the default) captures the step on step 3 while the loader's
    workers and pin-memory thread are still prefetching; 6 steps must equal --hip-graph 0 (only
    fp32-atomic summation order in some weight-gradient engines may differ)."""
    from vq3d import train
    rng = np.random.default_rng(1)
    for i, d in enumerate((20, 40, 24)):
        _write(str(tmp_path / f"scan{i}.nrrd"), rng.integers(-1500, 3000, size=(32, 32, d)).astype(np.int16))

    def run(hip_graph):
        base = [str(tmp_path), "--batch-size", "1", "--n-bottleneck-blocks", "2",
                "--default_root_dir", str(tmp_path / f"run{hip_graph}"), "--val_check_interval", "1.0",
                "--log_every_n_steps", "1", "--max_steps", "6", "--hip-graph", str(hip_graph)]
        model, _, hist, _ = train.main(train.parse_arguments(base), datamodule=_SmallCTWorkers(tmp_path))
        torch.cuda.synchronize()
        return [v for _, v in hist], model.flat.data.clone()
    le, we = run(0)
    lg, wg = run(1)
    assert len(le) == len(lg) == 6 and all(np.isfinite(le + lg))
    assert np.allclose(le, lg, rtol=2e-3), (le, lg)
    assert float((we - wg).abs().max()) <= 1e-3 * float(we.abs().max())
