"""PyTorch-Lightning-shaped `.ckpt` save / load.

The reference saves checkpoints through the PL 1.2.10 Trainer (train.py:56, ModelCheckpoint)
and reloads them with `VQVAE.load_from_checkpoint(path)` (extract_embeddings.py:45,
decode_embeddings.py:23).  PL is a third-party dependency absent from this image
(environment.yml pins pytorch-lightning 1.2.10); its checkpoint is a torch.save'd dict:

    epoch, global_step, pytorch-lightning_version, state_dict, callbacks, optimizer_states,
    lr_schedulers, [native_amp_scaling_state], hparams_name, hyper_parameters

with `hyper_parameters = {"args": Namespace}` and `hparams_name = "kwargs"` because the
reference calls `self.save_hyperparameters()` inside `__init__(self, args)` (model.py:38-42):
PL collects the init arguments by name and `load_from_checkpoint` calls `cls(**hyper_parameters)`.
`state_dict` keys / shapes / dtypes are the reference's (model.state_dict()), and
`optimizer_states[0]` is torch Adam's per-parameter layout (FusedAdam.state_dict), so a
checkpoint written here loads in the reference and vice versa.

Loading never unpickles arbitrary objects: `torch.load(weights_only=True)` with an allowlist
of `argparse.Namespace`, the `pathlib` path classes (train.py:22 stores `dataset_path` as a
Path) and inert stand-ins for the PL callback classes whose *types* key the
`callbacks` entry of a Trainer checkpoint.
"""
import pathlib
from argparse import Namespace

import torch

PL_VERSION = "1.2.10"  # the reference's pinned pytorch-lightning (environment.yml)
_PL_CALLBACKS = ("pytorch_lightning.callbacks.model_checkpoint.ModelCheckpoint",
                 "pytorch_lightning.callbacks.early_stopping.EarlyStopping",
                 "pytorch_lightning.callbacks.lr_monitor.LearningRateMonitor")


def _stub(qualname):
    return type(qualname.rsplit(".", 1)[1], (), {"__module__": qualname.rsplit(".", 1)[0]})


# the reference's train.py parses `dataset_path` with type=Path (train.py:22), so every Namespace it
# saves holds a pathlib object
_PATHS = [pathlib.PosixPath, pathlib.PurePosixPath, pathlib.WindowsPath, pathlib.PureWindowsPath]
_SAFE = [Namespace] + _PATHS + [(_stub(q), q) for q in _PL_CALLBACKS]


def save_checkpoint(path, model, optimizer=None, epoch: int = 0, global_step: int = 0, callbacks=None, scaler=None):
    """Write a PL 1.2-layout checkpoint of `model` (and its optimizer's state) to `path`; with an
    enabled loss scaler (the fp16 path) also its state as PL's native AMP plugin stores it."""
    ck = {
        "epoch": int(epoch),
        "global_step": int(global_step),
        "pytorch-lightning_version": PL_VERSION,
        "state_dict": {k: v.detach().cpu().clone() for k, v in model.state_dict().items()},
        "callbacks": dict(callbacks or {}),
        "optimizer_states": [] if optimizer is None else [_cpu(
            optimizer if isinstance(optimizer, dict) else optimizer.state_dict())],
        "lr_schedulers": [],
        "hparams_name": "kwargs",
        "hyper_parameters": {"args": Namespace(**vars(model.hparams["args"]))},
    }
    if scaler is not None and scaler.enabled:
        ck["native_amp_scaling_state"] = scaler.state_dict()
    torch.save(ck, path)


def _cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu().clone()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def load_checkpoint(path, map_location="cpu"):
    """The checkpoint dict, loaded with the weights-only unpickler (see module doc)."""
    with torch.serialization.safe_globals(_SAFE):
        return torch.load(path, map_location=map_location, weights_only=True)


def model_args(ck) -> Namespace:
    """The VQVAE constructor's `args` from a checkpoint's hyper_parameters."""
    hp = ck["hyper_parameters"]
    name = ck.get("hparams_name", "kwargs")
    if name != "kwargs":  # hyper-parameters saved under the init argument's own name
        hp = {name: hp}
    args = hp["args"]
    return args if isinstance(args, Namespace) else Namespace(**dict(args))


def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True, **overrides):
    """`LightningModule.load_from_checkpoint`: rebuild `cls(args)` from the saved
    hyper-parameters (keyword overrides replace fields of args), then load the state_dict."""
    ck = load_checkpoint(checkpoint_path, map_location="cpu")
    args = model_args(ck)
    for k, v in overrides.items():
        setattr(args, k, v)
    model = cls(args)
    model.load_state_dict(ck["state_dict"], strict=strict)
    if map_location is not None:
        model = model.to(map_location)
    return model
