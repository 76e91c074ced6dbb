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
* Any other configuration (``NeRF(D, W, in_xyz, in_dir, skips)``,
  ``Embedding(C, F, logscale)``) is accepted too and runs composably on the
  device: the reference's layer sequence on PyTorch-ROCm GEMMs, with
  ``render_rays``'s sampling and compositing still on the HIP kernels
  (SURVEY.md 8b).  Every caller of the reference uses the defaults.
* Host (CPU) inputs run the same layer sequence on the host
  (nerf_pl_amd.host, BASELINE configs[0]).
"""
from __future__ import annotations

import torch
from torch import nn

from . import ops, packing


class Embedding(nn.Module):
    """x -> (x, sin(f_0 x), cos(f_0 x), ...), models/nerf.py:4-38.  The
    reference configuration (3 channels, log-scale bands) runs on nr_embed;
    others compose the same sequence with torch ops on the device."""

    def __init__(self, in_channels, N_freqs, logscale=True):
        super().__init__()
        self.N_freqs = N_freqs
        self.in_channels = in_channels
        self.logscale = logscale
        self.funcs = [torch.sin, torch.cos]
        self.out_channels = in_channels * (len(self.funcs) * N_freqs + 1)
        if logscale:
            self.freq_bands = 2 ** torch.linspace(0, N_freqs - 1, N_freqs)
        else:
            self.freq_bands = torch.linspace(1, 2 ** (N_freqs - 1), N_freqs)
        self._fused = in_channels == 3 and logscale and N_freqs < 31

    def forward(self, x):
        if self._fused and x.is_cuda:
            shp = x.shape
            out = ops.embed(x.reshape(-1, 3), self.N_freqs)
            return out.view(*shp[:-1], self.out_channels)
        out = [x]
        for freq in self.freq_bands.tolist():
            for func in self.funcs:
                out += [func(freq * x)]
        return torch.cat(out, -1)


class NeRF(nn.Module):
    """models/nerf.py:41-124 (D=8, W=256, 63/27 inputs, skip at layer 4)."""

    def __init__(self, D=8, W=256, in_channels_xyz=63, in_channels_dir=27, skips=[4]):  # noqa: B006
        super().__init__()
        # the fused kernels implement the reference default; others compose
        self._fused = (D, W, in_channels_xyz, in_channels_dir, list(skips)) == (8, 256, 63, 27, [4])
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
        if not self._fused:
            raise RuntimeError("nerf_pl_amd.NeRF: flat/packed parameters exist for the fused "
                               "default configuration only")
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
        if not self._fused or not x.is_cuda:
            # a host input (nerf_pl_amd.host) or a configuration the fused
            # kernels do not implement: the layer sequence
            return self.forward_layers(x, sigma_only)
        from .functions import mlp_apply
        return mlp_apply(self, x=x, sigma_only=sigma_only)

    def forward_layers(self, x, sigma_only=False):
        """nerf.py:83-124 as a sequence of GEMMs on the parameters' device
        (configurations the fused kernels do not implement; host batches)."""
        dev = self.sigma.weight.device
        if x.device != dev:
            raise ValueError(f"nerf_pl_amd.NeRF: input on {x.device}, parameters on {dev}")
        if not sigma_only:
            input_xyz, input_dir = torch.split(x, [self.in_channels_xyz, self.in_channels_dir], -1)
        else:
            input_xyz = x
        xyz_ = input_xyz
        for i in range(self.D):
            if i in self.skips:
                xyz_ = torch.cat([input_xyz, xyz_], -1)
            xyz_ = getattr(self, f"xyz_encoding_{i + 1}")(xyz_)
        sigma = self.sigma(xyz_)
        if sigma_only:
            return sigma
        xyz_encoding_final = self.xyz_encoding_final(xyz_)
        dir_encoding = self.dir_encoding(torch.cat([xyz_encoding_final, input_dir], -1))
        rgb = self.rgb(dir_encoding)
        return torch.cat([rgb, sigma], -1)
