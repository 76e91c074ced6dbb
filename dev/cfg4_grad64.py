"""dev: per-tensor distance of the cfg4 step's gradients from float64
(tests/test_gpu_cfg4.py, tests/grad64.py) next to the fp32 oracle's own, per
arithmetic; every evaluation's fine pass at the depths that arithmetic chose
(NR_G64_OWNZ=0: each at its own depths, the round-4 comparison).

    python dev/cfg4_grad64.py [mode...]     modes: f16x3 fp32 bf16x6 f16x3:every
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import grad64  # noqa: E402
import test_gpu_cfg4 as T  # noqa: E402
from nerf_pl_amd import functions, ops  # noqa: E402

torch.set_num_threads(16)
n = 1024
_, _, _, rays, rgbs = T._batch()
rays, rgbs = rays[:n].contiguous(), rgbs[:n]
draws = [d[:n] for d in T._draws(T.B)]
own_z = os.environ.get("NR_G64_OWNZ", "1") == "1"
for mode in sys.argv[1:] or ["f16x3", "fp32"]:
    math_, _, opt = mode.partition(":")
    ops.MATH = math_
    functions.ACTIVE_SAMPLES = opt != "every"
    functions.DEFER_SAVE = "none"
    models = T._models()
    cap = {}
    res = T._ours(models, rays, draws, cap)
    zf = cap["z_fine"].detach().cpu() if own_z else None
    pts = {u: (T._oracle_point(torch.float32, u, rays, draws, zf),
               T._oracle_point(torch.float64, u, rays, draws, zf)) for u in (None, 1, 2)}
    c64 = pts[None][1][2]
    bad = T._kinks(models, rays, cap, c64, draws)
    keep = torch.from_numpy(~bad)
    g32s, g64s = [], []
    for u, ((p32, o32, _), (p64, o64, _)) in pts.items():
        T._loss(o32, rgbs, keep).backward()
        T._loss(o64, rgbs, keep).backward()
        g32s.append({f"m{i}.{k}": v.grad for i, p in enumerate(p32) for k, v in p.items()})
        g64s.append({f"m{i}.{k}": v.grad for i, p in enumerate(p64) for k, v in p.items()})
    g64, f0, floor = g64s[0], grad64.fp32_floor(g32s[:1], g64s[:1]), grad64.fp32_floor(g32s, g64s)
    T._loss(res, rgbs, keep).backward()
    ours = {f"m{i}.{k}": w.grad.detach().cpu().double() for i, m in enumerate(models)
            for k, w in m.named_parameters()}
    rows = []
    for k, e in g64.items():
        d = ((ours[k] - e).norm() / e.norm()).item()
        rows.append((d / max(grad64.ABS_FLOOR, grad64.C * floor[k]), k, d))
    rows.sort(reverse=True)
    print(f"== {mode} ({int(bad.sum())} rays screened; fine pass at {'our' if own_z else 'own'} depths)")
    for r, k, d in rows[:6]:
        print(f"   {k}: {d:.3g} from float64 | fp32 oracle {f0[k]:.3g} (max of 3 points {floor[k]:.3g}) "
              f"| {r:.2f} of the c=2 bound", flush=True)
