"""Ray-generation fixtures from the REFERENCE's own ``get_rays`` and
``get_ndc_rays`` (datasets/ray_utils.py:27-50, :53-93).

Run in the survey/build container only (it reads /root/reference):

    python tests/golden/make_golden_rays.py

``datasets/ray_utils.py`` starts with ``from kornia import create_meshgrid``
and kornia is not installed, so the module cannot be imported whole.  Its
other two functions use torch alone: this script parses the reference file,
takes the ``get_rays`` and ``get_ndc_rays`` definitions as they stand and
executes them (nothing replaces kornia; ``get_ray_directions``, the one
function that needs it, is not run).  Their input directions come from the
restatement ``oracle.rays_oracle.get_ray_directions`` (kornia 0.2.0's
``create_meshgrid(normalized_coordinates=False)``: i = column, j = row, no
+0.5), which the fixtures therefore pin only through what get_rays does with
them.  Output: ``tests/golden/rays/rays.npz`` (plain arrays).
"""
from __future__ import annotations

import ast
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("NERF_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import rays_oracle as RO  # noqa: E402

CASES = [  # (H, W, focal, ndc)
    (17, 23, 21.5, False),
    (32, 24, 555.5555, False),
    (9, 14, 7.25, True),
    (21, 28, 407.0, True),
]


def reference_functions():
    path = os.path.join(REF, "datasets", "ray_utils.py")
    tree = ast.parse(open(path).read(), path)
    keep = [n for n in tree.body
            if isinstance(n, ast.FunctionDef) and n.name in ("get_rays", "get_ndc_rays")]
    assert len(keep) == 2, "reference ray_utils.py changed"
    _vet(keep)
    # no builtins: the two bodies may reach torch and their own arguments only
    ns = {"torch": torch, "__builtins__": {}}
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return ns["get_rays"], ns["get_ndc_rays"]


_ALLOWED_ATTRS = {"T", "norm", "expand", "shape", "view", "stack", "reshape", "unsqueeze"}
# torch functions get_rays / get_ndc_rays call (ray_utils.py:43, :91-92); every
# other torch attribute (torch.load, torch.save, torch.compile, ...) is refused
_ALLOWED_TORCH = {"stack", "norm", "ones_like", "meshgrid", "sum", "cat"}


def _vet(defs):
    """The untrusted reference code is executed only after this check (ADVICE
    r2): plain arithmetic, subscripts and assignments over the function's own
    names, calls only of whitelisted torch.<fn> or tensor methods; no
    decorators, imports, defaults that call, lambdas, comprehensions, loops,
    with-blocks, attribute access to dunders or globals other than torch."""
    ok_nodes = (ast.FunctionDef, ast.arguments, ast.arg, ast.Expr, ast.Constant, ast.Assign,
                ast.Return, ast.Name, ast.Load, ast.Store, ast.BinOp, ast.UnaryOp, ast.Add,
                ast.Sub, ast.Mult, ast.Div, ast.USub, ast.MatMult, ast.Pow, ast.Subscript,
                ast.Slice, ast.Tuple, ast.List, ast.Attribute, ast.Call, ast.keyword, ast.Ellipsis
                if hasattr(ast, "Ellipsis") else ast.Constant)
    for fn in defs:
        assert not fn.decorator_list, "decorated reference function"
        assert all(isinstance(d, ast.Constant) for d in fn.args.defaults), "computed default"
        local = {a.arg for a in fn.args.args}
        for node in ast.walk(fn):
            assert isinstance(node, ok_nodes), f"{fn.name}: {type(node).__name__} not allowed"
            if isinstance(node, ast.Assign):
                for t in node.targets:
                    for n in ast.walk(t):
                        if isinstance(n, ast.Name):
                            local.add(n.id)
            if isinstance(node, ast.Attribute):
                assert not node.attr.startswith("_"), f"{fn.name}: dunder attribute"
                base = node.value
                if isinstance(base, ast.Name) and base.id == "torch":
                    assert node.attr in _ALLOWED_TORCH, f"{fn.name}: torch.{node.attr} not allowed"
                    continue
                assert node.attr in _ALLOWED_ATTRS, f"{fn.name}: .{node.attr} not allowed"
            if isinstance(node, ast.Name) and isinstance(node.ctx, ast.Load):
                assert node.id in local or node.id == "torch", f"{fn.name}: global {node.id}"


def poses(k, ndc):
    from nerf_pl_amd.rays import pose_spherical
    out = []
    for p in range(2):
        if ndc:
            a = 0.1 * (k + p)
            out.append(torch.tensor([[math.cos(a), -math.sin(a), 0.0, 0.05 * (p - k)],
                                     [math.sin(a), math.cos(a), 0.0, 0.03 * (k + 1)],
                                     [0.0, 0.0, 1.0, -0.02 * p]]))
        else:
            out.append(pose_spherical(-170.0 + 97.0 * (k + 2 * p), -25.0 - 11.0 * p, 4.0 + 0.3 * k))
    return torch.stack(out).float()


def main():
    get_rays, get_ndc_rays = reference_functions()
    arrs = {}
    for k, (H, W, f, ndc) in enumerate(CASES):
        P = poses(k, ndc)
        dirs = RO.get_ray_directions(H, W, f)
        os_, ds_ = [], []
        for c2w in P:
            o, d = get_rays(dirs, c2w)
            if ndc:
                o, d = get_ndc_rays(H, W, f, 1.0, o, d)
            os_.append(o)
            ds_.append(d)
        arrs[f"c{k}_poses"] = P.numpy()
        arrs[f"c{k}_dirs"] = dirs.numpy()
        arrs[f"c{k}_rays_o"] = torch.cat(os_).numpy()
        arrs[f"c{k}_rays_d"] = torch.cat(ds_).numpy()
        arrs[f"c{k}_cfg"] = np.array([H, W, f, float(ndc)], np.float64)
    arrs["n_cases"] = np.array(len(CASES))
    os.makedirs(os.path.join(HERE, "rays"), exist_ok=True)
    out = os.path.join(HERE, "rays", "rays.npz")
    np.savez_compressed(out, **arrs)
    print("wrote", out, sum(v.nbytes for v in arrs.values()), "bytes")


if __name__ == "__main__":
    main()
