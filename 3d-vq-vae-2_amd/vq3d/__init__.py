"""vq3d — MI355X-native 3D VQ-VAE-2 training path (module API of sara-nl/3D-VQ-VAE-2's
vqvae package; kernels in libvq3d.so, C-ABI in include/vq3d.h)."""
from . import _lib  # noqa: F401
from .layers import (Conv3d, Decoder, DownBlock, Encoder2, EvonormResBlock, FixupResBlock,  # noqa: F401
                     PreActFixupResBlock, PreQuantizationConditioning, Quantizer, ResizeConv3D, UpBlock)
from .evonorm import EvoNorm3DS0  # noqa: F401
from .model import VQVAE, default_args  # noqa: F401

__all__ = ["VQVAE", "default_args", "Encoder2", "Decoder", "PreActFixupResBlock", "FixupResBlock",
           "EvonormResBlock", "Quantizer", "ResizeConv3D", "EvoNorm3DS0", "DownBlock", "UpBlock",
           "PreQuantizationConditioning", "Conv3d"]
