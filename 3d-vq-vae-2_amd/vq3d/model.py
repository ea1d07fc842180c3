"""VQVAE with the reference's module API and checkpoint layout (reference vqvae/model.py),
running every op of the training step on libvq3d kernels.

Differences a reference user sees: the class is a plain nn.Module with the LightningModule
methods the reference uses (training_step, configure_optimizers, add_model_specific_args, log
hooks); call .to('cuda') (or .cuda()) before use: that moves the parameters into one flat
fp32 buffer (flat.py).  Activations run in `compute_dtype` (bf16 by default on the GPU,
`--compute-dtype fp32` for exact-arithmetic parity runs); the Quantizer is always fp32
(layers.py:685-687) and parameters are fp32 masters.
"""
from argparse import ArgumentParser, Namespace
from typing import Tuple

import torch
from torch import nn

from . import functional as Fn
from . import ops
from . import parallel
from .flat import FlatParams
from .layers import Decoder, Encoder2, EvonormResBlock, FixupResBlock, PreActFixupResBlock
from .optim import FusedAdam
from .utils import booltype

DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


class VQVAE(nn.Module):
    # first in line is the default
    supported_metrics = ("huber",)

    def __init__(self, args: Namespace):
        super().__init__()
        self.save_hyperparameters(args)
        self._parse_input_args(args)
        self.encoder = Encoder2(
            in_channels=self.input_channels,
            base_network_channels=self.base_network_channels,
            n_enc=self.n_bottleneck_blocks,
            n_down_per_enc=self.n_blocks_per_bottleneck,
            n_pre_q_blocks=self.n_pre_quantization_blocks,
            n_post_downscale_blocks=self.n_post_downscale_blocks,
            n_post_upscale_blocks=self.n_post_upscale_blocks,
            num_embeddings=self.num_embeddings,
            resblock=self.resblock,
        )
        self.decoder = Decoder(
            out_channels=self.output_channels,
            base_network_channels=self.base_network_channels,
            n_enc=self.n_bottleneck_blocks,
            n_up_per_enc=self.n_blocks_per_bottleneck,
            n_post_q_blocks=self.n_post_quantization_blocks,
            n_post_upscale_blocks=self.n_post_upscale_blocks,
            resblock=self.resblock,
        )

        def init_fixupresblock(layer):
            if isinstance(layer, (FixupResBlock, PreActFixupResBlock)):
                layer.initialize_weights(num_layers=self.num_layers)
        self.apply(init_fixupresblock)
        self.flat = None
        self.logged = {}
        self.set_compute_dtype(DTYPES[getattr(args, "compute_dtype", "bf16")])

    # ------------------------------------------------------------------ Lightning-shaped hooks
    def save_hyperparameters(self, args):
        self.hparams = {"args": args}

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True, **overrides):
        """LightningModule.load_from_checkpoint (used by extract_embeddings.py:45,
        decode_embeddings.py:23) over a PL 1.2-layout .ckpt; see vq3d/checkpoint.py."""
        from .checkpoint import load_from_checkpoint
        return load_from_checkpoint(cls, checkpoint_path, map_location=map_location, strict=strict, **overrides)

    def log(self, name, value, **kwargs):
        self.logged[name] = value.detach() if torch.is_tensor(value) else value

    def log_dict(self, d, **kwargs):
        for k, v in d.items():
            self.log(k, v)

    # ------------------------------------------------------------------ device / dtype
    def set_compute_dtype(self, dtype):
        self.compute_dtype = dtype
        self.encoder.compute_dtype = dtype
        return self

    def _apply(self, fn, recurse=True):
        r = super()._apply(fn, recurse)
        p = next(self.parameters())
        if p.is_cuda and (self.flat is None or not self.flat.owns(p) or self.flat.device != p.device):
            self.flat = FlatParams(self.parameters(), p.device)
        return r

    def zero_grad(self, set_to_none: bool = False):
        if self.flat is not None:
            self.flat.zero_grad()
        else:
            super().zero_grad(set_to_none)

    # ------------------------------------------------------------------ model
    def forward(self, data):
        if torch.is_grad_enabled():
            parallel.step_begin()
        pre, hook = {"k": 0}, None
        levels = len(self.decoder.up)
        if ops.overlap_levels() and data.is_cuda and levels > 1:
            # Each decoder level chain above the bottom (layers.py:511-514: proj(cat[q_l, out]),
            # post-quantize blocks, up block) needs only its own code and the chain above it, so it
            # starts on the level stream as soon as that level's Quantizer is done, beside the
            # encoder's lower levels (layers.py:583-586).  Same launches, same arithmetic.
            def hook(quantization):
                i = pre["k"]
                if i >= levels - 1:  # the bottom chain needs the last code: nothing left to overlap
                    return
                s = ops.level_stream(data.device)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    pre["out"] = self.decoder.level_chain(i, quantization[1], pre.get("out"))
                pre["k"] = i + 1
        commitment_loss, quantizations, encoding_idx = zip(*self.encoder(data, on_quantized=hook))
        decoded = self.decoder(quantizations, pre=(pre["out"], ops.level_stream(data.device), pre["k"])
                               if pre["k"] else None)
        return decoded, (commitment_loss, quantizations, encoding_idx)

    def encode(self, data):
        return self.encoder(data)

    def decode(self, quantizations):
        return self.decoder(quantizations)

    def configure_optimizers(self):
        if self.flat is None:
            raise RuntimeError("move the model to the GPU (model.cuda()) before configure_optimizers()")
        return FusedAdam(self.parameters(), self.flat, lr=self.lr, amsgrad=True)

    def training_step(self, batch, batch_idx):
        return self.shared_step(batch, batch_idx, mode='train')

    def validation_step(self, batch, batch_idx):
        return self.shared_step(batch, batch_idx, mode='val')

    def shared_step(self, batch, batch_idx, mode='train'):
        assert mode in ('train', 'val')
        loss, log_dict = self.recon_loss_f(batch, batch_idx)
        self.log_dict({f'{mode}_{key}': val for key, val in log_dict.items()}, logger=True)
        return loss

    def loc_metric(self, batch, batch_idx) -> Tuple[torch.Tensor, dict]:
        """elu -> pad-slice mask -> centre cylinder -> smooth-L1 mean + sum(commitment),
        one fused kernel pair (model.py:115-160)."""
        x, num_valid_slices = batch
        loc, (commitment_loss, *_) = self(x)
        if x.dtype != torch.float32:
            raise TypeError("the target volume must be fp32 (the reference normalises it to [-0.5, 4])")
        if not torch.is_tensor(num_valid_slices):
            num_valid_slices = torch.as_tensor(num_valid_slices)
        nvs = num_valid_slices.to(device=x.device, dtype=torch.int64)
        loss, recon = Fn.recon_loss(loc, x, nvs, bool(self.pre_loss_f), *commitment_loss)
        log_dict = {'recon_loss_mean': recon}
        log_dict.update({f'commitment_loss_{i}': c for i, c in enumerate(commitment_loss)})
        self.log('recon loss', recon, prog_bar=True, logger=False)
        return loss, log_dict

    def huber(self, batch, batch_idx, **pre_loss_f_metrics):
        return self.loc_metric(batch, batch_idx)

    def _parse_input_args(self, args: Namespace):
        """model.py:165-210"""
        assert args.metric in self.supported_metrics
        if args.metric == 'huber':
            self.recon_loss_f = self.huber
        self.metric = args.metric
        self.lr = args.base_lr
        self.input_channels = args.input_channels
        self.output_channels = args.input_channels
        self.base_network_channels = args.base_network_channels
        self.n_bottleneck_blocks = args.n_bottleneck_blocks
        self.n_blocks_per_bottleneck = args.n_downscales_per_bottleneck
        self.n_pre_quantization_blocks = args.n_pre_quantization_blocks
        self.n_post_quantization_blocks = args.n_post_quantization_blocks
        self.n_post_upscale_blocks = args.n_post_upscale_blocks
        self.n_post_downscale_blocks = args.n_post_downscale_blocks
        assert len(args.num_embeddings) in (1, args.n_bottleneck_blocks)
        if len(args.num_embeddings) == 1:
            self.num_embeddings = [args.num_embeddings[0] for _ in range(args.n_bottleneck_blocks)]
        else:
            self.num_embeddings = args.num_embeddings
        resblocks = {'regular': FixupResBlock, 'pre-activation': PreActFixupResBlock, 'evonorm': EvonormResBlock}
        self.resblock = resblocks[args.block_type]
        n_down = args.n_bottleneck_blocks * args.n_downscales_per_bottleneck
        self.num_layers = (
            2 + 2 * n_down + args.n_pre_quantization_blocks + args.n_post_quantization_blocks
            + args.n_post_downscale_blocks * n_down + args.n_post_upscale_blocks * n_down + 1
        )
        self.pre_loss_f = bool(args.extract_center_cylinder)

    @classmethod
    def add_model_specific_args(cls, parent_parser):
        """model.py:213-246 (+ --compute-dtype)."""
        parser = ArgumentParser(parents=[parent_parser], add_help=False)
        parser.add_argument('--input-channels', type=int, default=1)
        parser.add_argument('--base-network_channels', type=int, default=4)
        parser.add_argument('--n-bottleneck-blocks', type=int, default=3)
        parser.add_argument('--n-downscales-per-bottleneck', type=int, default=2)
        parser.add_argument('--n-pre-quantization-blocks', type=int, default=0)
        parser.add_argument('--n-post-quantization-blocks', type=int, default=0)
        parser.add_argument('--n-post-upscale-blocks', type=int, default=0)
        parser.add_argument('--n-post-downscale-blocks', type=int, default=0)
        parser.add_argument('--num-embeddings', type=int, default=256, nargs='+',
                            help=("Can be either a single int or multiple."
                                  " If multiple, number of args should be equal to n-bottleneck-blocks"))
        parser.add_argument('--block-type', type=str, default='pre-activation',
                            choices=['regular', 'pre-activation', 'evonorm'])
        parser.add_argument('--extract-center-cylinder', type=booltype, default=True)
        parser.add_argument('--metric', choices=cls.supported_metrics, default=cls.supported_metrics[0])
        parser.add_argument('--base_lr', default=1e-5, type=float)
        parser.add_argument('--n-mix', default=2)
        parser.add_argument('--compute-dtype', choices=sorted(DTYPES), default='bf16',
                            help="activation storage dtype of the conv path (Quantizer is always fp32)")
        return parser


def default_args(**kw):
    """Namespace with the reference CLI defaults (model.py:220-244), overridable."""
    p = VQVAE.add_model_specific_args(ArgumentParser(add_help=False))
    a = p.parse_args([])
    if isinstance(a.num_embeddings, int):
        a.num_embeddings = [a.num_embeddings]
    for k, v in kw.items():
        setattr(a, k, v)
    return a
