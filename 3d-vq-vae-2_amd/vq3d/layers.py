"""Network modules with the reference's constructor signatures, attribute names and
state_dict layout (reference vqvae/layers.py), running on libvq3d kernels.

Modules are built in the reference's order with the same nn.Conv3d parameter containers, so
torch.manual_seed(s) + construction reproduces the reference's initial weights exactly.
Forward passes take channels-last GPU tensors (ops.py) and go through functional.py.
"""
from itertools import chain
from typing import List

import numpy as np
import torch
from torch import nn

from . import _lib as L
from . import functional as Fn
from .evonorm import EvoNorm3DS0
from . import ops
from .ops import ConvGeom
from .parallel import sum_allreduce


# ============================================================================================ conv containers
class Conv3d(nn.Conv3d):
    """nn.Conv3d parameter container whose forward runs the libvq3d conv (optionally over the
    channel concatenation of two inputs: proj(torch.cat([a, b], 1)) == proj(a, b))."""

    def _spec(self):
        spec = getattr(self, "_vq3d_spec", None)
        if spec is None:
            k, s, p = self.kernel_size[0], self.stride[0], self.padding[0]
            geom = ConvGeom(k, s, p, circular=self.padding_mode == "circular")
            spec = Fn.ConvSpec(self.weight, geom, cbias=self.bias)
            self._vq3d_spec = spec
        return spec

    def forward(self, x, x2=None):
        return Fn.conv(x, self._spec(), x2=x2)


class ResizeConv3D(Conv3d):
    """Trilinear x2 upsample then conv (layers.py:591-597)."""

    def __init__(self, *conv_args, **conv_kwargs):
        super().__init__(*conv_args, **conv_kwargs)
        self.upsample = nn.Upsample(mode='trilinear', scale_factor=2, align_corners=False)

    def forward(self, x, x2=None):
        assert x2 is None
        return Fn.conv(Fn.upsample(x), self._spec())


def _mode_conv(mode):
    if mode == 'down':
        return Conv3d, 4, 2, 1
    if mode in ('same', 'out'):
        return Conv3d, 3, 1, 1
    return ResizeConv3D, 3, 1, 1


# ============================================================================================ residual blocks
class PreActFixupResBlock(nn.Module):
    """layers.py:102-216 — the published block type; circular padding; fused kernels."""

    def __init__(self, in_channels, out_channels, mode, activation=nn.ELU, bottleneck_divisor=2):
        super().__init__()
        padding_mode = 'circular'
        assert mode in ("down", "same", "up", "out")
        self.mode = mode
        self.in_channels, self.out_channels = in_channels, out_channels
        branch_channels = max(max(in_channels, out_channels) // bottleneck_divisor, 1)
        self.activation = activation()
        if not isinstance(self.activation, nn.ELU) or self.activation.alpha != 1.0:
            raise NotImplementedError("the fused PreAct kernels implement ELU(alpha=1) only (reference default)")
        self.bias1a, self.bias1b, self.bias2a, self.bias2b, self.bias3a, self.bias3b, self.bias4 = (
            nn.Parameter(torch.zeros(1)) for _ in range(7)
        )
        self.scale = nn.Parameter(torch.ones(1))
        conv, kernel_size, stride, padding = _mode_conv(mode)
        self.branch_conv1 = Conv3d(in_channels, branch_channels, kernel_size=1, stride=1, padding=0, bias=False)
        self.branch_conv2 = conv(branch_channels, branch_channels, kernel_size=kernel_size, stride=stride,
                                 padding=padding, bias=False, padding_mode=padding_mode)
        self.branch_conv3 = Conv3d(branch_channels, out_channels, kernel_size=1, stride=1, padding=0, bias=False)
        if not (mode in ("same", "out") and in_channels == out_channels):
            self.bias1c, self.bias1d = (nn.Parameter(torch.zeros(1)) for _ in range(2))
            self.skip_conv = conv(in_channels, out_channels, kernel_size=(1 if mode != 'down' else 2),
                                  stride=(1 if mode != 'down' else 2), padding=0, bias=False)
        else:
            self.skip_conv = None

    @property
    def _fn_params(self):
        # the Parameter objects in kernel order, cached (parameters keep their identity: .to() and
        # load_state_dict write .data in place); a re-assigned attribute drops the cache (__setattr__)
        ps = self.__dict__.get("_fn_params_cache")
        if ps is None:
            ps = [self.bias1a, self.bias1b, self.bias2a, self.bias2b, self.bias3a, self.bias3b, self.bias4,
                  self.scale, self.branch_conv1.weight, self.branch_conv2.weight, self.branch_conv3.weight]
            if self.skip_conv is not None:
                ps += [self.bias1c, self.bias1d, self.skip_conv.weight]
            self.__dict__["_fn_params_cache"] = ps
        return ps

    def __setattr__(self, name, value):
        self.__dict__.pop("_fn_params_cache", None)
        super().__setattr__(name, value)

    def forward(self, input: torch.Tensor):
        return Fn.preact_block(input, self)

    @torch.no_grad()
    def initialize_weights(self, num_layers):
        """Fixup init (layers.py:197-216)."""
        weight = self.branch_conv1.weight
        nn.init.normal_(weight, mean=0,
                        std=np.sqrt(2 / (weight.shape[0] * np.prod(weight.shape[2:]))) * num_layers ** (-0.5))
        nn.init.kaiming_normal_(self.branch_conv2.weight)
        nn.init.constant_(self.branch_conv3.weight, val=0)
        if self.skip_conv is not None:
            nn.init.xavier_normal_(self.skip_conv.weight)


class FixupResBlock(nn.Module):
    """layers.py:219-303 ('regular'): zero padding, post-activation."""

    def __init__(self, in_channels, out_channels, mode, activation=nn.ELU):
        super().__init__()
        assert mode in ("down", "same", "up", "out")
        self.mode = mode
        branch_channels = out_channels
        self.activation = activation()
        self.bias1a, self.bias1b, self.bias2a, self.bias2b = (nn.Parameter(torch.zeros(1)) for _ in range(4))
        self.scale = nn.Parameter(torch.ones(1))
        conv, kernel_size, stride, padding = _mode_conv(mode)
        self.branch_conv1 = conv(in_channels, branch_channels, kernel_size=kernel_size, stride=stride,
                                 padding=padding, bias=False)
        self.skip_conv = conv(in_channels, out_channels, kernel_size=(1 if mode != 'down' else 2),
                              stride=(1 if mode != 'down' else 2), padding=0, bias=True)
        self.branch_conv2 = Conv3d(branch_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self._specs = None

    def _build_specs(self):
        _, k, s, p = _mode_conv(self.mode)
        ks = 2 if self.mode == 'down' else 1
        self._specs = (
            Fn.ConvSpec(self.branch_conv1.weight, ConvGeom(k, s, p), pro=(self.bias1a,)),
            Fn.ConvSpec(self.branch_conv2.weight, ConvGeom(3, 1, 1), pro=(self.bias1b, self.bias2a),
                        scale=self.scale, bias=self.bias2b, post_elu=self.mode != 'out'),
            Fn.ConvSpec(self.skip_conv.weight, ConvGeom(ks, ks, 0), cbias=self.skip_conv.bias),
        )

    def forward(self, input):
        if self._specs is None:
            self._build_specs()
        s1, s2, sk = self._specs
        # up mode: upsample(x + b1a) == upsample(x) + b1a (trilinear weights sum to 1)
        x = Fn.upsample(input) if self.mode == 'up' else input
        h = Fn.conv(x, s1)
        skip = Fn.conv(x, sk)
        return Fn.conv(h, s2, residual=skip)

    def initialize_weights(self, num_layers):
        weight = self.branch_conv1.weight
        nn.init.normal_(weight, mean=0,
                        std=np.sqrt(2 / (weight.shape[0] * np.prod(weight.shape[2:]))) * num_layers ** (-0.5))
        nn.init.constant_(tensor=self.branch_conv2.weight, val=0)
        nn.init.kaiming_normal_(self.skip_conv.weight)
        nn.init.constant_(tensor=self.skip_conv.bias, val=0)


class EvonormResBlock(nn.Module):
    """layers.py:14-99: EvoNorm-S0 pre-normalised bottleneck block, zero padding, conv biases
    (batch 1 only, like the reference)."""

    def __init__(self, in_channels, out_channels, mode, bottleneck_divisor=4):
        super().__init__()
        assert mode in ("down", "same", "up", "out")
        if mode == 'out':
            mode = 'same'
        self.mode = mode
        branch_channels = max(max(in_channels, out_channels) // bottleneck_divisor, 1)
        conv, kernel_size, stride, padding = _mode_conv(mode)
        self.evonorm_1 = EvoNorm3DS0(in_channels)
        self.branch_conv1 = Conv3d(in_channels, branch_channels, kernel_size=1, stride=1, padding=0)
        self.evonorm_2 = EvoNorm3DS0(branch_channels)
        self.branch_conv2 = conv(branch_channels, branch_channels, kernel_size=kernel_size, stride=stride,
                                 padding=padding)
        self.evonorm_3 = EvoNorm3DS0(branch_channels)
        self.branch_conv3 = Conv3d(branch_channels, out_channels, kernel_size=1, stride=1, padding=0)
        self.skip_conv = conv(in_channels, out_channels, kernel_size=(1 if mode != 'down' else 2),
                              stride=(1 if mode != 'down' else 2), padding=0,
                              ) if not (mode in ("same", "out") and in_channels == out_channels) else None
        self.initialize_weights()
        self._specs = None

    def _build_specs(self):
        _, k, s, p = _mode_conv(self.mode)
        ks = 2 if self.mode == 'down' else 1
        self._specs = (
            Fn.ConvSpec(self.branch_conv1.weight, ConvGeom(1), cbias=self.branch_conv1.bias),
            Fn.ConvSpec(self.branch_conv2.weight, ConvGeom(k, s, p), cbias=self.branch_conv2.bias),
            Fn.ConvSpec(self.branch_conv3.weight, ConvGeom(1), cbias=self.branch_conv3.bias),
            None if self.skip_conv is None else
            Fn.ConvSpec(self.skip_conv.weight, ConvGeom(ks, ks, 0), cbias=self.skip_conv.bias),
        )

    def forward(self, input: torch.Tensor):
        if self._specs is None:
            self._build_specs()
        s1, s2, s3, sk = self._specs
        up = self.mode == 'up'
        out = Fn.conv(self.evonorm_1(input), s1)
        t = self.evonorm_2(out)
        if up:
            t = Fn.upsample(t)
        out = Fn.conv(t, s2)
        if sk is None:
            res = input
        else:
            res = Fn.conv(Fn.upsample(input) if up else input, sk)
        return Fn.conv(self.evonorm_3(out), s3, residual=res)

    @torch.no_grad()
    def initialize_weights(self):
        for weight in (self.branch_conv1.weight, self.branch_conv2.weight, self.branch_conv3.weight):
            nn.init.kaiming_normal_(weight)
        if self.skip_conv is not None:
            nn.init.xavier_normal_(self.skip_conv.weight)
            nn.init.zeros_(self.skip_conv.bias)


# ============================================================================================ stacks
class BlockStack(nn.Sequential):
    """nn.Sequential (same children, same state_dict keys) whose forward runs every maximal run of
    identical PreActFixupResBlocks ('same', no skip) fused: >= 2 blocks on a tiny grid as ONE stack
    (Fn.PreActStackFn: one launch forward, one backward), a run of 72-channel / branch-36 blocks
    through Fn.PreActWideFn (preact_wide.hip), a run of 18-channel / branch-9 blocks chained through
    Fn.PreActMidRunFn (preact_mid.hip), a run of few-channel blocks through Fn.PreActSmallRunFn
    (one reduction for the whole run); everything else runs module by module."""

    out_fp32 = False  # set where the consumer takes an fp32 tensor (the encoder's Quantizers)
    small_runs_only = False  # Down / UpBlock: only few-channel runs fused (their fp32 stream)

    def forward(self, x):
        mods = list(self)
        i = 0
        while i < len(mods):
            j = i
            if Fn.stack_eligible(mods[i]):
                c, nb = mods[i].in_channels, mods[i].branch_conv1.weight.shape[0]
                while (j + 1 < len(mods) and Fn.stack_eligible(mods[j + 1]) and mods[j + 1].in_channels == c
                       and mods[j + 1].branch_conv1.weight.shape[0] == nb):
                    j += 1
            fn = None
            if self.small_runs_only:
                if j > i and Fn.small_run_eligible(x, mods[i]):
                    fn = Fn.PreActSmallRunFn
            elif Fn.stack_eligible(mods[i]):
                if j > i and self._stack_ok(x, mods[i]):
                    fn = Fn.PreActStackFn
                elif Fn.wide_eligible(x, mods[i]):
                    fn = Fn.PreActWideFn
                elif j > i and Fn.mid_run_eligible(x, mods[i]):
                    fn = Fn.PreActMidRunFn
                elif j > i and Fn.small_run_eligible(x, mods[i]):
                    fn = Fn.PreActSmallRunFn
            if fn is not None:
                run = tuple(mods[i:j + 1])
                plan = self._plans.get((i, j)) if hasattr(self, "_plans") else None
                if plan is None or plan.blocks != list(run):
                    if not hasattr(self, "_plans"):
                        self._plans = {}
                    plan = self._plans[(i, j)] = Fn.StackPlan(run)
                # the stack's last run hands an fp32 stream on when the consumer takes it
                plan.out_dtype = torch.float32 if (self.out_fp32 and j == len(mods) - 1 and
                                                   fn is Fn.PreActSmallRunFn and ops.fp32_stream()) else None
                x = Fn.preact_run(fn, x, plan)
                i = j + 1
            else:
                x = mods[i](x)
                i += 1
        return x

    @staticmethod
    def _stack_ok(x, blk):
        if not (x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16)):
            return False
        b, c, h, w, d = x.shape
        return c == blk.in_channels and bool(L.query("vq3d_preact_stack_supported", b, c,
                                                      blk.branch_conv1.weight.shape[0], h, w, d))


class DownBlock(nn.Module):
    """layers.py:306-324."""

    def __init__(self, in_channels, n_down=2, resblock=FixupResBlock, n_post_downscale_blocks=0):
        super().__init__()
        # a BlockStack (an nn.Sequential: same state_dict keys) so the post-downscale blocks run as
        # one fused run where an engine takes them
        self.layers = BlockStack(*chain.from_iterable(
            (resblock(in_channels * 2 ** i, in_channels * 2 ** (i + 1), mode='down'),
             *(resblock(in_channels * 2 ** (i + 1), in_channels * 2 ** (i + 1), mode='same')
               for _ in range(n_post_downscale_blocks)))
            for i in range(n_down)
        ))
        self.layers.small_runs_only = True

    def forward(self, data):
        return self.layers(data)


class UpBlock(nn.Module):
    """layers.py:327-354."""

    def __init__(self, in_channels, out_channels, aux_channels=0, n_up=2, mode='encoder', resblock=FixupResBlock,
                 n_post_upscale_blocks=0):
        super().__init__()
        assert mode in ('encoder', 'decoder')
        self.layers = BlockStack(*chain.from_iterable((
            (resblock(in_channels if i == n_up - 1 else out_channels * (2 ** (i + 1)), out_channels * (2 ** i),
                      mode='up'),
             *(resblock(out_channels * (2 ** i), out_channels * (2 ** i), mode='same')
               for _ in range(n_post_upscale_blocks)))
            for i in range(n_up - 1, -1, -1)
        )))
        self.layers.small_runs_only = True

    def forward(self, data):
        return self.layers(data)


class PreQuantizationConditioning(nn.Module):
    """layers.py:357-387; proj(cat[data, up(aux)]) runs as one two-input 1x1 conv."""

    def __init__(self, in_channels, out_channels, n_up=2, resblock=FixupResBlock, n_post_upscale_blocks=0):
        super().__init__()
        self.has_aux = in_channels - out_channels * 8 != 0
        if self.has_aux:
            self.upsample = UpBlock(out_channels * 2 ** n_up, out_channels, n_up=n_up, resblock=resblock,
                                    n_post_upscale_blocks=n_post_upscale_blocks)
            self.proj = Conv3d(in_channels, in_channels, kernel_size=1)
        self.pre_q = resblock(in_channels, out_channels, mode='same')

    def forward(self, data, auxilary=None):
        assert self.has_aux is (auxilary is not None)
        if self.has_aux:
            data = self.proj(data, self.upsample(auxilary))
        return self.pre_q(data)


class Encoder2(nn.Module):
    """layers.py:519-588 (the encoder the model uses)."""

    def __init__(self, in_channels, base_network_channels, num_embeddings: List[int], n_enc=3, n_down_per_enc=2,
                 n_pre_q_blocks=0, n_post_upscale_blocks=0, n_post_downscale_blocks=0, resblock=FixupResBlock):
        super().__init__()
        self.parse_input = Conv3d(in_channels, base_network_channels, kernel_size=1)
        before_channels = base_network_channels
        self.down, self.pre_quantize, self.pre_quantize_cond, self.quantize = (nn.ModuleList() for _ in range(4))
        for i in range(n_enc):
            after_channels = before_channels * 2 ** n_down_per_enc
            self.down.append(DownBlock(before_channels, n_down_per_enc, resblock=resblock,
                                       n_post_downscale_blocks=n_post_downscale_blocks))
            assert after_channels % 8 == 0
            embedding_dim = after_channels // 8
            self.pre_quantize_cond.append(PreQuantizationConditioning(
                in_channels=after_channels + (embedding_dim if i != n_enc - 1 else 0), out_channels=embedding_dim,
                n_up=n_down_per_enc, resblock=resblock, n_post_upscale_blocks=n_post_upscale_blocks))
            self.pre_quantize.append(BlockStack(
                *(resblock(embedding_dim, embedding_dim, mode='same') for _ in range(n_pre_q_blocks))))
            self.pre_quantize[-1].out_fp32 = True  # z goes to the fp32 Quantizer (layers.py:685-687)
            self.quantize.append(Quantizer(num_embeddings=num_embeddings[i], embedding_dim=embedding_dim,
                                           commitment_cost=0.1))
            before_channels = after_channels
        self.compute_dtype = torch.float32

    def forward(self, data, on_quantized=None):
        """on_quantized(quantization): called after each level's Quantizer, top level first (the
        model uses it to start the decoder's top-level chain early, VQVAE.forward)."""
        if Fn.parse_input_fused(data, self.parse_input, self.compute_dtype):
            # the fp32 volume straight into the 16-bit activation (never rounded to bf16 itself)
            down = Fn.parse_input(data, self.parse_input.weight, self.parse_input.bias, self.compute_dtype)
        else:
            if data.dtype != self.compute_dtype:
                data = ops.cast(data, self.compute_dtype)
            down = self.parse_input(data)
        downsampled = []
        for downblock in self.down:
            down = downblock(down)
            downsampled.append(down)
        aux = None
        quantizations = []
        for q in self.quantize:
            q.zst_dtype = self.compute_dtype
        stats = self._ema_slots(data.device) if self.training else None
        try:
            for down, pre_quantize, pre_quantize_cond, quantize in reversed(
                    list(zip(downsampled, self.pre_quantize, self.pre_quantize_cond, self.quantize))):
                quantization = quantize(pre_quantize(pre_quantize_cond(down, aux)))
                quantizations.append(quantization)
                _, aux, *_ = quantization
                if on_quantized is not None:
                    on_quantized(quantization)
        finally:
            for q in self.quantize:
                q.ema_slot = None
        if stats is not None:
            # the reference all-reduces counts and dw inside each level's forward (C1 / C2,
            # layers.py:645-647: six latency-bound calls on the critical path); every level's
            # codes are final before any EMA update matters (the updated codebooks are first
            # read by the next step), so one SUM all-reduce of all levels' statistics follows
            sum_allreduce(stats)
            off = 0
            for q in self.quantize:
                n = q.num_embeddings * (q.embedding_dim + 1)
                if q.training:
                    Fn.ema_update(q, stats[off:off + n])
                off += n
        return reversed(quantizations)

    def _ema_slots(self, device):
        sizes = [q.num_embeddings * (q.embedding_dim + 1) for q in self.quantize]
        stats = torch.empty(sum(sizes), dtype=torch.float32, device=device)
        off = 0
        for q, n in zip(self.quantize, sizes):
            q.ema_slot = stats[off:off + n] if q.training else None
            off += n
        return stats


class Decoder(nn.Module):
    """layers.py:463-517."""

    def __init__(self, out_channels, base_network_channels, n_enc=3, n_up_per_enc=2, n_post_q_blocks=0,
                 n_post_upscale_blocks=0, resblock=FixupResBlock):
        super().__init__()
        self.up = nn.ModuleList()
        self.proj = nn.ModuleList()
        after_channels = base_network_channels
        for i in range(n_enc):
            before_channels = after_channels * 2 ** n_up_per_enc
            assert before_channels % 8 == 0
            embedding_dim = before_channels // 8
            in_channels = embedding_dim + (before_channels if i != n_enc - 1 else 0)
            if i != n_enc - 1:
                self.proj.append(Conv3d(in_channels, in_channels, kernel_size=1))
            self.up.append(BlockStack(
                *(resblock(in_channels, in_channels, mode='same') for _ in range(n_post_q_blocks)),
                UpBlock(in_channels=in_channels, out_channels=after_channels, n_up=n_up_per_enc, mode='decoder',
                        resblock=resblock, n_post_upscale_blocks=n_post_upscale_blocks),
            ))
            after_channels = before_channels
        self.out = Conv3d(base_network_channels, out_channels, kernel_size=1)

    def forward(self, quantizations, pre=None):
        """pre: (output of the first k level chains, top first; the stream they were issued on; k)
        when the caller already ran them (VQVAE.forward); the current stream joins it here."""
        k, out = 0, None
        if pre is not None:
            out, stream, k = pre
            torch.cuda.current_stream().wait_stream(stream)
        for i, (quantization, up) in enumerate(reversed(list(zip(quantizations, self.up)))):
            if i < k:
                continue
            out = quantization if i == 0 else self.proj[-i](quantization, out)
            out = up(out)
        return self.out(out)

    def level_chain(self, i, quantization, out):
        """The decoder's i-th level chain, top first (layers.py:511-514): proj(cat[q, out]) for
        i > 0, then the level's post-quantize blocks and up block."""
        out = quantization if i == 0 else self.proj[-i](quantization, out)
        return self.up[-1 - i](out)


# ============================================================================================ quantizer
class Quantizer(nn.Module):
    """EMA vector quantiser (layers.py:602-728).  Buffers embed / embed_avg / cluster_size /
    first_pass as in the reference state_dict; `first_pass` is mirrored on the host so the
    forward never synchronises (the reference's bool(tensor) at layers.py:695 does)."""

    def __init__(self, num_embeddings: int, embedding_dim: int, commitment_cost: float, decay=0.99,
                 laplace_alpha=1e-5):
        super().__init__()
        embed = torch.randn(num_embeddings, embedding_dim)
        self.register_buffer("embed", embed)
        self.register_buffer("embed_avg", embed.clone())
        self.register_buffer("cluster_size", torch.zeros(num_embeddings))
        self.register_buffer("first_pass", torch.as_tensor(1))
        self.first_pass_host = True
        # fp32 [counts (K) | dw (K x D)] slice of the encoder's fused EMA-statistics buffer while
        # Encoder2.forward runs (None: a standalone forward reduces and updates by itself)
        self.ema_slot = None
        self.commitment_cost = commitment_cost
        self.decay = decay
        self.laplace_alpha = laplace_alpha
        self.embedding_dim = embedding_dim
        self.num_embeddings = num_embeddings
        self._register_load_state_dict_pre_hook(self._load_hook)

    def _load_hook(self, state_dict, prefix, *args):
        fp = state_dict.get(prefix + "first_pass")
        if fp is not None:
            self.first_pass_host = bool(int(fp))

    def embed_code(self, embed_idx):
        """F.embedding(idx, embed) (layers.py:633-634)."""
        return self.embed[embed_idx]

    def forward(self, inputs):
        loss, zst, idx = Fn.quantize(inputs, self)
        return loss, zst, idx
