"""nerf_pl_amd -- MI355X-native (gfx950) drop-in for ktiwary2/nerf_pl's
render_rays / sample_pdf / NeRF hot path.

    from nerf_pl_amd import NeRF, Embedding, render_rays
"""
from .nerf import Embedding, NeRF
from .rendering import render_rays, sample_pdf
from .rng import PhiloxRNG, ReplayRNG
from .searchsorted import searchsorted

__all__ = ["Embedding", "NeRF", "render_rays", "sample_pdf", "searchsorted", "PhiloxRNG",
           "ReplayRNG"]
__version__ = "0.1.0"
