"""Dense sigma-grid query for mesh extraction (extract_color_mesh.py:114-141).

The reference embeds an N^3 grid chunk by chunk, runs the full fine NeRF with a
zero direction and keeps max(sigma, 0).  Here the sigma-only fused kernel
evaluates the grid with the positional encoding computed in-kernel (sigma does
not depend on the direction, nerf.py:112); marching cubes itself (PyMCubes)
stays a host-side dependency of the caller.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def grid_points(N, x_range, y_range, z_range, device) -> torch.Tensor:
    """The (N^3, 3) grid in the reference's order (np.meshgrid default 'xy'
    indexing, extract_color_mesh.py:119-123)."""
    x = np.linspace(x_range[0], x_range[1], N)
    y = np.linspace(y_range[0], y_range[1], N)
    z = np.linspace(z_range[0], z_range[1], N)
    return torch.tensor(np.stack(np.meshgrid(x, y, z), -1).reshape(-1, 3), dtype=torch.float32,
                        device=device)


@torch.no_grad()
def query_sigma(model, pts: torch.Tensor) -> torch.Tensor:
    """Raw sigma (n,) of ``model`` (a nerf_pl_amd.NeRF) at points (n,3)."""
    packed, _ = model.packed()
    return ops.sigma_points(packed, pts)


@torch.no_grad()
def sigma_grid(model, N=256, x_range=(-1.2, 1.2), y_range=(-1.2, 1.2), z_range=(-1.2, 1.2)):
    """max(sigma, 0) on the N^3 grid, shape (N, N, N) (extract_color_mesh.py:138-139)."""
    dev = model.flat_params().device
    sigma = query_sigma(model, grid_points(N, x_range, y_range, z_range, dev))
    return torch.clamp_min(sigma, 0).reshape(N, N, N)
