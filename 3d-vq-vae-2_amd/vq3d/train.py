"""Training entry mirroring the reference's vqvae/train.py:14-59 on the vq3d path.

    python -m vq3d.train DATASET [--batch-size 1] [model flags of VQVAE.add_model_specific_args]
                         [--max_epochs N] [--max_steps N] [--default_root_dir DIR]
                         [--resume_from_checkpoint last.ckpt]

--gpus follows the reference (train.py:25-27: gpus=-1, accelerator='ddp'): -1 = every visible GPU,
N = N GPUs.  With more than one, the command starts its own ranks -- `python -m
torch.distributed.run --nproc-per-node N -m vq3d.train ...` as a child process (vq3d/launch.py),
before this process touches a GPU -- and exits with its code; started by an existing torchrun
(WORLD_SIZE set) it is simply that rank.

What the reference gets from PyTorch-Lightning 1.2.10 (Trainer.from_argparse_args +
ModelCheckpoint), restated here without that dependency:
  * argument composition: Trainer flags (the subset the reference's jobs set), then
    VQVAE.add_model_specific_args, then the script's own --rescale-input / --batch-size /
    dataset_path, with the reference's set_defaults (train.py:25-40);
  * seed_everything(42) (train.py:50): Python, numpy and torch RNGs;
  * CTDataModule(path, batch_size, num_workers=5, rescale_input) (train.py:52);
  * 'ddp': one process per GPU, DistributedSampler sharding, the bucketed RCCL gradient average
    of vq3d.parallel (overlapped with backward) and the Quantizers' fused EMA all-reduce;
  * validation every val_check_interval of an epoch (val_recon_loss_mean, eval mode);
  * ModelCheckpoint(save_top_k=1, save_last=True, monitor='val_recon_loss_mean') (train.py:56):
    last.ckpt after every validation, the best one as epoch=E-step=S.ckpt (PL 1.2 layout,
    vq3d.checkpoint);
  * --resume_from_checkpoint restores weights, codebooks, Adam state, epoch and global step with
    PL 1.2.10's counter convention (pl_checkpoint_counters / resume_counters), so a checkpoint
    written by the reference resumes here at the epoch PL would resume it at, and vice versa;
    last.ckpt is also written when training stops (max_steps / max_epochs).
precision=16 is recorded; the path computes in the --compute-dtype format: bf16 (default) or fp16 with
the reference's AMP loss scaling (optim.GradScaler, its state saved as native_amp_scaling_state).
"""
import os
import random
from argparse import ArgumentParser, Namespace
from pathlib import Path

import numpy as np
import torch

from . import parallel
from .checkpoint import load_checkpoint, save_checkpoint
from .data import CTDataModule
from .graph import StepGraph
from .model import VQVAE
from .optim import GradScaler


def add_trainer_args(parser):
    """The Trainer flags the reference's jobs use (pl.Trainer.add_argparse_args, train.py:17)."""
    parser.add_argument("--gpus", type=str, default=None)
    parser.add_argument("--accelerator", type=str, default=None)
    parser.add_argument("--benchmark", type=bool, default=False)
    parser.add_argument("--num_sanity_val_steps", type=int, default=2)
    parser.add_argument("--precision", type=int, default=32)
    parser.add_argument("--log_every_n_steps", type=int, default=50)
    parser.add_argument("--val_check_interval", type=float, default=1.0)
    parser.add_argument("--flush_logs_every_n_steps", type=int, default=100)
    parser.add_argument("--weights_summary", type=str, default="top")
    parser.add_argument("--max_epochs", type=int, default=1000)
    parser.add_argument("--max_steps", type=int, default=None)
    parser.add_argument("--default_root_dir", type=str, default=os.getcwd())
    parser.add_argument("--resume_from_checkpoint", type=str, default=None)
    parser.add_argument("--num_nodes", type=int, default=1)
    parser.add_argument("--hip-graph", dest="hip_graph", type=int, default=1,
                        help="replay each training step as a captured HIP graph (1) or launch eagerly (0)")
    return parser


def build_parser():
    parser = ArgumentParser()
    parser = add_trainer_args(parser)
    parser = VQVAE.add_model_specific_args(parser)
    parser.add_argument('--rescale-input', type=int, nargs='+')
    parser.add_argument("--batch-size", type=int)
    parser.add_argument("dataset_path", type=Path)
    parser.set_defaults(gpus="-1", accelerator='ddp', benchmark=True, num_sanity_val_steps=0, precision=16,
                        log_every_n_steps=50, val_check_interval=0.5, flush_logs_every_n_steps=100,
                        weights_summary='full', max_epochs=int(1e5))
    return parser


def parse_arguments(argv=None):
    args = build_parser().parse_args(argv)
    if isinstance(args.num_embeddings, int):
        args.num_embeddings = [args.num_embeddings]
    return args


def seed_everything(seed=42):
    """pl.trainer.seed_everything (train.py:50)."""
    os.environ["PL_GLOBAL_SEED"] = str(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    return seed


def pl_checkpoint_counters(epoch, pl_global_step, max_steps=None):
    """(epoch, global_step) as PL 1.2.10's CheckpointConnector.dump_checkpoint writes them while the
    trainer is at `epoch` with its global_step counter at `pl_global_step` (the 0-based index of the
    batch being finished: PL increments its counter only after the batch's validation /
    checkpoint callbacks): global_step + 1, and epoch + 1 unless max_steps was reached.  On
    restore PL sets current_epoch = ckpt['epoch'] and global_step = ckpt['global_step']
    (resume_counters), so a checkpoint written mid-epoch resumes at the next epoch boundary."""
    reached = max_steps is not None and max_steps <= pl_global_step
    return (int(epoch) if reached else int(epoch) + 1), int(pl_global_step) + 1


def resume_counters(ck):
    """(first epoch, global step) a run resumed from checkpoint dict `ck` continues with (PL 1.2.10
    restore_training_state): the saved values as they are."""
    return int(ck["epoch"]), int(ck["global_step"])


class Checkpointer:
    """ModelCheckpoint(save_top_k=1, save_last=True, monitor='val_recon_loss_mean'): the best
    checkpoint as epoch=E-step=S.ckpt with PL's counters at save time (E = current epoch, S = the
    trainer's global_step before its increment), last.ckpt always; the counters inside follow
    pl_checkpoint_counters."""

    def __init__(self, dirpath, monitor="val_recon_loss_mean"):
        self.dirpath = Path(dirpath)
        self.monitor = monitor
        self.best_score = None
        self.best_path = None

    def state(self):
        return {"monitor": self.monitor, "best_model_score": self.best_score, "best_model_path": self.best_path,
                "dirpath": str(self.dirpath)}

    def __call__(self, model, opt, epoch, pl_global_step, score, max_steps=None, scaler=None):
        self.dirpath.mkdir(parents=True, exist_ok=True)
        ep, gs = pl_checkpoint_counters(epoch, pl_global_step, max_steps)
        if score is not None and (self.best_score is None or score < self.best_score):
            old = self.best_path
            self.best_score = float(score)
            self.best_path = str(self.dirpath / f"epoch={epoch}-step={pl_global_step}.ckpt")
            save_checkpoint(self.best_path, model, opt, epoch=ep, global_step=gs,
                            callbacks={"ModelCheckpoint": self.state()}, scaler=scaler)
            if old and old != self.best_path and os.path.exists(old):
                os.remove(old)
        save_checkpoint(str(self.dirpath / "last.ckpt"), model, opt, epoch=ep, global_step=gs,
                        callbacks={"ModelCheckpoint": self.state()}, scaler=scaler)


def _to_device(batch, dev):
    x, nvs = batch
    return x.to(dev, non_blocking=True).float(), torch.as_tensor(nvs).to(dev)


def validate(model, loader, dev):
    model.eval()
    tot, n = 0.0, 0
    with torch.no_grad():
        for batch in loader:
            x, nvs = _to_device(batch, dev)
            model.validation_step((x, nvs), n)
            tot += float(model.logged["val_recon_loss_mean"])
            n += 1
    model.train()
    if torch.distributed.is_initialized():
        t = torch.tensor([tot, float(n)], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t)
        tot, n = float(t[0]), int(t[1])
    return tot / n if n else None


def main(args: Namespace, datamodule=None):
    """train.py:47-59."""
    rank, world, _, dev = parallel.init_from_env()
    if dev.type != "cuda":
        raise RuntimeError("vq3d.train runs the HIP path: a GPU is required")
    seed_everything(42)
    if datamodule is None:
        datamodule = CTDataModule(path=args.dataset_path, batch_size=args.batch_size, num_workers=5,
                                  rescale_input=args.rescale_input)
    datamodule.setup()
    model = VQVAE(args).to(dev)
    model.train()
    opt = model.configure_optimizers()
    # --compute-dtype fp16 trains like the reference's precision=16: PL native AMP's loss scaling
    scaler = GradScaler(dev, enabled=model.compute_dtype == torch.float16)
    ckpt = Checkpointer(Path(args.default_root_dir) / "checkpoints")
    epoch0, step = 0, 0
    if args.resume_from_checkpoint:
        ck = load_checkpoint(args.resume_from_checkpoint)
        model.load_state_dict(ck["state_dict"])
        if ck.get("optimizer_states"):
            opt.load_state_dict(ck["optimizer_states"][0])
        scaler.load_state_dict(ck.get("native_amp_scaling_state"))
        epoch0, step = resume_counters(ck)
        st = ck.get("callbacks", {}).get("ModelCheckpoint") or {}
        ckpt.best_score, ckpt.best_path = st.get("best_model_score"), st.get("best_model_path")
    # built after any resume, so the replicas start from the restored (identical) state
    reducer = parallel.GradientAllReduce(model)
    try:
        return _fit(args, model, opt, reducer, ckpt, datamodule, rank, world, dev, epoch0, step, scaler)
    finally:
        reducer.close()


def _fit(args, model, opt, reducer, ckpt, datamodule, rank, world, dev, epoch0, step, scaler):
    train_ds, val_ds = datamodule.train_dataset, datamodule.val_dataset
    sampler = (torch.utils.data.distributed.DistributedSampler(train_ds, world, rank, shuffle=True, seed=42,
                                                               drop_last=True) if world > 1 else None)
    # persistent workers: the worker processes are forked once, before the step graph is captured,
    # not again at every epoch from a process whose GPU work (and pin-memory thread) is in flight
    # (an epoch-boundary re-fork after capture was seen to hang the next host-to-device copy)
    persist = datamodule.num_workers > 0
    loader = torch.utils.data.DataLoader(train_ds, batch_size=datamodule.batch_size, shuffle=sampler is None,
                                         sampler=sampler, num_workers=datamodule.num_workers, pin_memory=True,
                                         drop_last=True, persistent_workers=persist)
    vsampler = (torch.utils.data.distributed.DistributedSampler(val_ds, world, rank, shuffle=False)
                if world > 1 else None)
    vloader = torch.utils.data.DataLoader(val_ds, batch_size=datamodule.batch_size, shuffle=False, sampler=vsampler,
                                          num_workers=datamodule.num_workers, pin_memory=True, drop_last=True,
                                          persistent_workers=persist)
    n_batches = len(loader)

    def train_step(x, nvs):
        opt.zero_grad()
        loss = model.training_step((x, nvs), 0)
        scaler.scale(loss).backward()
        reducer()
        scaler.step(opt)
        scaler.update()
        return loss
    # the whole step as a HIP graph per input shape (single rank, or ranks whose RCCL collectives
    # replay correctly inside a graph: parallel.graph_collectives_ok)
    use_graph = bool(getattr(args, "hip_graph", 1)) and (
        world == 1 or (torch.distributed.get_backend() == "nccl" and parallel.graph_collectives_ok(dev)))
    runner = StepGraph(train_step, warmup=2, enabled=use_graph)
    val_every = max(1, int(n_batches * args.val_check_interval)) if args.val_check_interval <= 1 else \
        int(args.val_check_interval)
    history = []
    epoch = epoch0
    for epoch in range(epoch0, args.max_epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        for i, batch in enumerate(loader):
            x, nvs = _to_device(batch, dev)
            loss = runner(x, nvs)
            step += 1
            if step % args.log_every_n_steps == 0 or step == 1:
                history.append((step, float(loss.detach())))
                if rank == 0:
                    print(f"epoch {epoch} step {step} loss {history[-1][1]:.6f}", flush=True)
            if (i + 1) % val_every == 0 or (i + 1) == n_batches:
                score = validate(model, vloader, dev) if len(val_ds) else None
                if rank == 0:  # PL's global_step is still this batch's 0-based index here
                    ckpt(model, opt, epoch, step - 1, score, args.max_steps, scaler)
            if args.max_steps is not None and step >= args.max_steps:
                break
        if args.max_steps is not None and step >= args.max_steps:
            break
    if rank == 0 and step > 0:  # training ended (max_steps / max_epochs): last.ckpt holds the final state
        ckpt(model, opt, epoch, step - 1, None, args.max_steps, scaler)
    return model, opt, history, ckpt


def launch_ranks(args, argv):
    """The 'ddp' self-launch (train.py:25-27): the exit code of the N ranks this command started
    when --gpus asks for more than one GPU and this process is not already a rank, else None."""
    from . import launch
    if launch.is_rank_process() or args.accelerator not in (None, "ddp"):
        return None
    n = launch.resolve_gpus(args.gpus)
    if n <= 1:
        return None
    env = dict(os.environ)
    pkg = str(Path(__file__).resolve().parent.parent)  # the ranks import vq3d from the same tree
    env["PYTHONPATH"] = pkg + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return launch.run_ranks(n, "vq3d.train", list(argv), module=True, env=env)


def cli(argv=None):
    import sys
    argv = sys.argv[1:] if argv is None else argv
    args = parse_arguments(argv)
    rc = launch_ranks(args, argv)
    if rc is not None:
        return rc
    main(args)
    return 0


if __name__ == '__main__':
    raise SystemExit(cli())
