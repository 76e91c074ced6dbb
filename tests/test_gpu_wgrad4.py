"""The f16x3 weight gradient's LDS-DMA kernel (wgrad.hip wgrad4_kernel, round 5)
against the register-staged one it replaced (wgrad3_kernel, selected with
NR_WGRAD_W4=0 at run time), on the same inputs, in the three ways a training
step launches it: over the gathered sample list (*_active), over buffers saved
by position for the listed samples (*_listed, the deferred save) and over every
sample.  Both split the same fp32 operands into the same f16 pieces and scale
the gradient operand by the same power of two; only the fp32 summation order
differs, so the two agree to ~1e-6 of each tensor's largest entry (bound
written below: 1e-5).  Ragged sizes put the last stage's tail (positions >= m,
zeroed in LDS) inside a workgroup; the larger size splits every task over many
workgroups.  The end-to-end accuracy of either kernel against autograd is
test_gpu_render.py's test_mlp_backward_matches_autograd.
"""
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
RTOL = 1e-5


def _grads(monkeypatch, w4, active, defer, size, zero_frac, seed=5):
    from nerf_pl_amd import NeRF, functions, ops
    from nerf_pl_amd.functions import mlp_apply
    monkeypatch.setattr(ops, "MATH", "f16x3")
    monkeypatch.setattr(functions, "ACTIVE_SAMPLES", active)
    monkeypatch.setattr(functions, "DEFER_SAVE", defer)
    monkeypatch.setenv("NR_WGRAD_W4", "1" if w4 else "0")
    g = torch.Generator().manual_seed(seed)
    n_rays, spr = size
    rays = torch.cat([torch.randn(n_rays, 3, generator=g) * 0.3,
                      torch.nn.functional.normalize(torch.randn(n_rays, 3, generator=g), dim=-1),
                      torch.full((n_rays, 1), 2.0), torch.full((n_rays, 1), 6.0)], 1)
    z = 2 + 4 * torch.rand(n_rays, spr, generator=g)
    gout = torch.randn(n_rays * spr, 4, generator=g)
    gout *= torch.exp2(-20 * torch.rand(n_rays, 1, generator=g)).repeat_interleave(spr, 0)
    gout[torch.rand(n_rays * spr, generator=g) < zero_frac] = 0     # unlisted samples
    net = NeRF()
    net.load_state_dict(O.make_params(7, sigma_bias=0.4))
    net = net.to(DEV)
    out = mlp_apply(net, rays=rays.to(DEV), z=z.to(DEV), spr=spr)
    (out * gout.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().cpu().double() for k, p in net.named_parameters()}


@pytest.mark.parametrize("active,defer", [(True, "none"), (True, "all"), (False, "none")])
@pytest.mark.parametrize("size", [(23, 37), (509, 61)])
def test_wgrad_dma_matches_register_staged(monkeypatch, active, defer, size):
    new = _grads(monkeypatch, True, active, defer, size, zero_frac=0.45)
    old = _grads(monkeypatch, False, active, defer, size, zero_frac=0.45)
    for k, ref in old.items():
        scale = ref.abs().max().item()
        err = (new[k] - ref).abs().max().item()
        assert err <= RTOL * scale + 1e-30, f"{k}: {err:.3g} of {scale:.3g}"
        assert torch.isfinite(new[k]).all(), k


def test_wgrad_dma_empty_list(monkeypatch):
    """No sample with a nonzero output gradient: every launch runs with m = 0
    (clamped, bounds-checked DMAs, nothing multiplied) and writes exact zeros."""
    g = _grads(monkeypatch, True, True, "none", (23, 37), zero_frac=1.1)
    for k, v in g.items():
        assert (v == 0).all(), k


def test_wgrad_dma_at_the_size_limit(monkeypatch):
    """n = 2^21 - 1 (16,513 rays x 127 samples): the largest launch the LDS-DMA
    kernel takes (wgrad_launch falls back at 2^21), where its 256-wide
    gradient segments span exactly 2^31 bytes -- past int's range for the
    buffer resources' record count; gathered list, every tensor against the
    register-staged kernel."""
    new = _grads(monkeypatch, True, True, "none", (16513, 127), zero_frac=0.45, seed=9)
    old = _grads(monkeypatch, False, True, "none", (16513, 127), zero_frac=0.45, seed=9)
    for k, ref in old.items():
        scale = ref.abs().max().item()
        err = (new[k] - ref).abs().max().item()
        assert err <= RTOL * scale + 1e-30, f"{k}: {err:.3g} of {scale:.3g}"
