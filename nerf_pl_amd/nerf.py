"""``Embedding`` and ``NeRF`` with the reference's constructor signatures and
parameter names (models/nerf.py:4-124), backed by the fused HIP kernels.

* ``NeRF`` keeps the exact submodule layout of the reference
  (``xyz_encoding_{1..8}.0``, ``xyz_encoding_final``, ``dir_encoding.0``,
  ``sigma``, ``rgb.0``), so ``state_dict()`` keys and shapes are identical and
  reference checkpoints load unchanged (``utils/__init__.py:72-76`` strips the
  ``nerf_coarse.``/``nerf_fine.`` prefix).
* Its parameters are views into one flat fp32 buffer in
  ``named_parameters()`` order; the packer gathers from that buffer and the
  weight-gradient kernel writes into a flat gradient of the same order.
* ``forward(x, sigma_only)`` accepts the pre-embedded input exactly like the
  reference (used e.g. by extract_color_mesh.py); ``render_rays`` takes the
  fused path that embeds in-kernel.
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops, packing


class Embedding(nn.Module):
    """x -> (x, sin(2^k x), cos(2^k x), ...), models/nerf.py:4-38 (logscale only)."""

    def __init__(self, in_channels, N_freqs, logscale=True):
        super().__init__()
        if in_channels != 3 or not logscale:
            raise NotImplementedError("nerf_pl_amd: only Embedding(3, F, logscale=True) "
                                      "(the reference's configuration, train.py:34-35)")
        self.N_freqs = N_freqs
        self.in_channels = in_channels
        self.funcs = [torch.sin, torch.cos]
        self.out_channels = in_channels * (len(self.funcs) * N_freqs + 1)
        self.freq_bands = 2 ** torch.linspace(0, N_freqs - 1, N_freqs)

    def forward(self, x):
        shp = x.shape
        out = ops.embed(x.reshape(-1, 3), self.N_freqs)
        return out.view(*shp[:-1], self.out_channels)


class NeRF(nn.Module):
    """models/nerf.py:41-124 (D=8, W=256, 63/27 inputs, skip at layer 4)."""

    def __init__(self, D=8, W=256, in_channels_xyz=63, in_channels_dir=27, skips=[4]):  # noqa: B006
        super().__init__()
        if (D, W, in_channels_xyz, in_channels_dir, list(skips)) != (8, 256, 63, 27, [4]):
            raise NotImplementedError("nerf_pl_amd: the fused kernels implement the reference "
                                      "default NeRF(D=8, W=256, 63, 27, skips=[4])")
        self.D, self.W = D, W
        self.in_channels_xyz, self.in_channels_dir = in_channels_xyz, in_channels_dir
        self.skips = skips
        for i in range(D):
            if i == 0:
                layer = nn.Linear(in_channels_xyz, W)
            elif i in skips:
                layer = nn.Linear(W + in_channels_xyz, W)
            else:
                layer = nn.Linear(W, W)
            setattr(self, f"xyz_encoding_{i + 1}", nn.Sequential(layer, nn.ReLU(True)))
        self.xyz_encoding_final = nn.Linear(W, W)
        self.dir_encoding = nn.Sequential(nn.Linear(W + in_channels_dir, W // 2), nn.ReLU(True))
        self.sigma = nn.Linear(W, 1)
        self.rgb = nn.Sequential(nn.Linear(W // 2, 3), nn.Sigmoid())
        self._flat = None
        self._pack_cache = None

    # -- flat parameter storage ---------------------------------------------
    def ordered_params(self):
        named = dict(self.named_parameters())
        return [named[k] for k in packing.param_shapes()]

    def flat_params(self) -> torch.Tensor:
        """The flat fp32 buffer all parameters view into (re-flattened after
        ``.to()``/``load_state_dict`` replaced their storage)."""
        ps = self.ordered_params()
        flat = self._flat
        ok = flat is not None and flat.device == ps[0].device
        if ok:
            base, off = flat.data_ptr(), 0
            for p in ps:
                if p.data_ptr() != base + 4 * off or p.dtype != torch.float32:
                    ok = False
                    break
                off += p.numel()
        if not ok:
            flat = torch.empty(packing.N_PARAMS, dtype=torch.float32, device=ps[0].device)
            off = 0
            with torch.no_grad():
                for p in ps:
                    n = p.numel()
                    flat[off:off + n].copy_(p.reshape(-1))
                    p.data = flat[off:off + n].view_as(p)
                    off += n
            self._flat = flat
            self._pack_cache = None
        return flat

    def packed(self, backward=False):
        """Fragment-order weights for the fused kernels, re-packed whenever the
        parameters changed (tracked through their version counters)."""
        flat = self.flat_params()
        ver = tuple(p._version for p in self.ordered_params())
        key = (flat.data_ptr(), ver, ops.MATH)
        c = self._pack_cache
        if c is None or c[0] != key:
            c = [key, ops.pack_fwd(flat), None]
            self._pack_cache = c
        if backward and c[2] is None:
            c[2] = ops.pack_bwd(flat)
        return c[1], c[2]

    def forward(self, x, sigma_only=False):
        from .functions import mlp_apply
        return mlp_apply(self, x=x, sigma_only=sigma_only)
