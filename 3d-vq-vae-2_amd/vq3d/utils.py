"""Small host-side helpers mirroring the reference utils the training path uses."""
import numpy as np
import torch


def booltype(inp: str) -> bool:
    """utils/argparse_helpers.py:2-9"""
    if type(inp) is str:
        if inp.lower() == 'true':
            return True
        elif inp.lower() == 'false':
            return False
    raise ValueError(f"input should be either 'True', or 'False', found {inp}")


def cylinder_xy_mask(size):
    """ExtractCenterCylinder.create_cylinder_xy_mask (utils/load_nrrd_dataset.py:288-300);
    the GPU loss kernel evaluates the same disc as (2h-H)^2 + (2w-W)^2 <= min(H,W)^2."""
    x_size, y_size = size
    radius = min(x_size, y_size) / 2
    x, y = np.ogrid[:x_size, :y_size]
    return torch.from_numpy(np.sqrt((x - x_size / 2) ** 2 + (y - y_size / 2) ** 2) <= radius)


def synthetic_volume(shape, index, device=None):
    """Synthetic CT-like volume in the reference's normalised range [-0.5, 4.0]
    (HU clip [-1500, 3000] / 1000 + 1, load_nrrd_dataset.py:73-80); deterministic per index
    (SURVEY.md §8(d))."""
    g = torch.Generator().manual_seed(1234 + int(index))
    x = torch.rand(shape, generator=g) * 4.5 - 0.5
    return x if device is None else x.to(device)
