"""nerf_pl_amd -- MI355X-native (gfx950) drop-in for ktiwary2/nerf_pl's
render_rays / sample_pdf / NeRF hot path.

    from nerf_pl_amd import NeRF, Embedding, render_rays
"""
import os as _os

# A training step keeps three of our streams busy at once (the caller's, the
# fine pass's, the pipelined step's second main stream) and RCCL adds its own;
# with HIP's default of 4 hardware queues per process two of them share a
# queue and their kernels serialise (measured: the distributed path's two
# backward chains never overlapped, 488k vs 529k rays/s at one RCCL rank;
# DESIGN.md 15).  Raised to 8 when lower (the GPU boxes export HIP's default
# of 4 explicitly) unless NERF_PL_AMD_KEEP_HW_QUEUES=1; takes effect when set
# before the process's first HIP call.
if (_os.environ.get("NERF_PL_AMD_KEEP_HW_QUEUES") != "1"
        and int(_os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8):
    _os.environ["GPU_MAX_HW_QUEUES"] = "8"

from .nerf import Embedding, NeRF  # noqa: E402
from .rendering import render_rays, sample_pdf  # noqa: E402
from .rng import PhiloxRNG, ReplayRNG  # noqa: E402
from .searchsorted import searchsorted  # noqa: E402

__all__ = ["Embedding", "NeRF", "render_rays", "sample_pdf", "searchsorted", "PhiloxRNG",
           "ReplayRNG"]
__version__ = "0.1.0"
