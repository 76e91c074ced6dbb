"""Randomness sources for ``render_rays``.

The reference draws five tensors from the global torch generator per call
(SURVEY.md 8a-RNG): ``rand(B,S)`` [perturb>0] -> ``randn(B,S)`` -> ``rand(B,I)`` ->
``rand_like(B,I)`` -> ``randn(B,S+I)``.

* :class:`PhiloxRNG` (default): nothing is materialised; the kernels draw
  in-register from Philox4x32-10 keyed by a per-call 64-bit seed (taken from
  the torch CPU generator, so ``torch.manual_seed`` makes runs repeatable).
  Distribution-equivalent to the reference, not stream-identical.
* :class:`ReplayRNG`: replays recorded tensors in draw order -- used for
  bit-level parity with the reference (tests/golden).
* :class:`TorchRNG`: draws from the global torch generator exactly as the
  reference does (``torch.rand`` / ``torch.randn`` on the rays' device) -- the
  default of a host batch (nerf_pl_amd.host), which then consumes the same
  numbers as the reference under the same ``torch.manual_seed``.
"""
from __future__ import annotations

import torch

# Philox stream ids of the five draws (csrc kernels use the same numbers)
STREAM_PERTURB, STREAM_NOISE_COARSE, STREAM_U, STREAM_JITTER, STREAM_NOISE_FINE = range(5)


class PhiloxRNG:
    def __init__(self, seed: int | None = None):
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.seed = seed

    def rand(self, shape, device):   # noqa: ARG002 -- drawn in-kernel
        return None

    randn = rand


class ReplayRNG:
    def __init__(self, tensors, seed: int = 0):
        self._queue = list(tensors)
        self._pos = 0
        self.seed = seed

    def _next(self, shape, device):
        t = torch.as_tensor(self._queue[self._pos], dtype=torch.float32)
        self._pos += 1
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"replayed draw #{self._pos} has shape {tuple(t.shape)}, "
                             f"expected {tuple(shape)}")
        return t.to(device).contiguous()

    rand = _next
    randn = _next

    def exhausted(self) -> bool:
        return self._pos == len(self._queue)


class TorchRNG:
    seed = 0

    def rand(self, shape, device):
        return torch.rand(*shape, device=device)

    def randn(self, shape, device):
        return torch.randn(*shape, device=device)
