"""dev: per-tensor gradient deviations of the cfg4 training step (tests/test_gpu_cfg4.py)
for each arithmetic with and without the sample list."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import test_gpu_cfg4 as T
from oracle import nerf_oracle as O
from nerf_pl_amd import ops, functions

torch.set_num_threads(16)
n = 1024
_, _, _, rays, rgbs = T._batch()
rays, rgbs = rays[:n].contiguous(), rgbs[:n]
draws = [d[:n] for d in T._draws(T.B)]
p32, p64 = T._params(grad=True), T._params(torch.float64, grad=True)
c32, c64 = {}, {}
ref = O.render_rays(p32, rays, T.S, False, 1.0, 1.0, T.I, 32768, False, rng=O.ReplayRNG(draws), capture=c32)
ref64 = O.render_rays(p64, rays.double(), T.S, False, 1.0, 1.0, T.I, 32768, False,
                      rng=O.ReplayRNG([d.double() for d in draws]), capture=c64)
z32, z64 = c32["z_fine"].detach().double(), c64["z_fine"].detach()
bad64 = ((z32 - z64).abs().max(1).values > 1e-4 * z64.abs().max(1).values.clamp(min=1)).numpy()
results = {}
for math_ in sys.argv[1:] or ["fp32", "f16x3"]:
    for active in (True, False):
        ops.MATH = math_
        functions.ACTIVE_SAMPLES = active
        models = T._models()
        cap = {}
        res = T._ours(models, rays, draws, cap)
        bad = T._screen(cap, c32, draws) | bad64
        keep = torch.from_numpy(~bad)
        T._loss(res, rgbs, keep).backward()
        results[(math_, active)] = ([[w.grad.detach().cpu().double() for _, w in m.named_parameters()] for m in models], keep)
keep = list(results.values())[0][1]
for p in p32 + p64:
    for v in p.values():
        v.grad = None
T._loss(ref, rgbs, keep).backward()
T._loss(ref64, rgbs, keep).backward()
names = [nm for nm, _ in T._models()[0].named_parameters()]
for (math_, active), (grads, k2) in results.items():
    assert torch.equal(k2, keep)
    worst = []
    for mi, (p, q) in enumerate(zip(p32, p64)):
        for j, name in enumerate(names):
            exp, e64 = p[name].grad.double(), q[name].grad
            got = grads[mi][j]
            scale = exp.norm() + 1e-30
            bound = max(1e-4, ((exp - e64).norm() / scale).item())
            dev = ((got - exp).norm() / scale).item()
            d64 = ((got - e64).norm() / (e64.norm() + 1e-30)).item()
            worst.append((dev / bound, f"m{mi} {name}: dev {dev:.3g} bound {bound:.3g} vs64 {d64:.3g}"))
    worst.sort(reverse=True)
    print(math_, "active" if active else "every-sample", *[w[1] for w in worst[:4]], sep="\n   ")
