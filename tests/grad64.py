"""Gradient parity against float64 (test infrastructure).

The parameter gradient of the reference's training step is ill-conditioned in
fp32 (xyz = o + d*z rounded to fp32 meets the 2^9 positional-encoding
frequency; ReLU kinks within an ulp pick a branch by summation order), so an
fp32 oracle on the test host is itself one random sample of an fp32-accurate
evaluation, and its distance from ours moves with the host's BLAS.  The bound
is therefore taken against the float64 oracle, whose result does not depend on
the host, with ONE constant:

    |ours - o64| / |o64|  <=  max(ABS_FLOOR, C * floor)       per tensor,

where ``floor`` is the fp32 oracle's own normwise distance from float64,
measured at the unperturbed parameters and at two points one fp32 ulp away
(every weight moved up or down by one ulp; each against its own float64
evaluation) -- the largest of the three, so one lucky fp32 evaluation cannot
shrink the bound.  ``C`` = 2: our gradient must be at most twice as far from
float64 as an fp32 evaluation of the reference algorithm is.

Every evaluation's fine pass runs at the importance depths our kernels chose
(the oracle's z_fine_override): the reference detaches them
(rendering.py:253-255), so the gradient is that of the fine pass at whichever
depths it ran at, and their continuous dependence on the coarse pass's
rounding -- amplified by the 2^9 encoding frequency -- is a forward matter the
forward parity tests bound.  Rays whose gradient is discontinuous at the
evaluation point leave the loss, each explained: a ReLU kink of the
compositing (relu_kinks).  Screened rays must stay rare."""
import torch

C = 2.0
ABS_FLOOR = 1e-4


def ulp_perturbed(params, seed, dt):
    """every parameter moved by one fp32 ulp up or down (seeded), in dtype dt"""
    out = {}
    g = torch.Generator().manual_seed(seed)
    for k, v in params.items():
        sgn = torch.randint(0, 2, v.shape, generator=g).to(torch.float32) * 2 - 1
        out[k] = (v.float() * (1 + sgn * 2.0 ** -23)).to(dt)
    return out


def relu_kinks(sig_ours, sig64, noise, tol=1e-4):
    """(flipped, explained) per ray: the compositing's relu(sigma + noise)
    (rendering.py:169-176, alphas = 1 - exp(-deltas * relu(sigmas + noise)))
    switched on or off between our sigma and the float64 oracle's at some
    sample -- that sample's d sigma jumps between 0 and a full-size value, a
    discontinuity of the gradient no arithmetic can be blamed for; explained
    when every such sample has |sigma64 + noise| <= tol (a kink, not an error)"""
    x_o = sig_ours.detach().cpu().double() + noise.double()
    x_64 = sig64.detach().cpu().double() + noise.double()
    flip = (x_o > 0) != (x_64 > 0)
    expl = (~flip | (x_64.abs() <= tol)).all(1)
    return flip.any(1).numpy(), expl.numpy()


def fp32_floor(grads32, grads64):
    """per-tensor max over evaluation points of |g32 - g64| / |g64|: grads32 and
    grads64 are lists (one entry per point) of {name: tensor}"""
    floor = {}
    for g32, g64 in zip(grads32, grads64):
        for k, e64 in g64.items():
            e32 = g32[k].double()
            d = ((e32 - e64).norm() / (e64.norm() + 1e-30)).item()
            floor[k] = max(floor.get(k, 0.0), d)
    return floor


def check(ours, g64, floor, label=""):
    """assert every tensor of ``ours`` within the bound of the float64
    gradients ``g64``; prints the five closest to their bound and returns the
    worst (deviation / bound) and its tensor"""
    rows = []
    for k, e64 in g64.items():
        got = ours[k].double()
        dev = ((got - e64).norm() / (e64.norm() + 1e-30)).item()
        bound = max(ABS_FLOOR, C * floor[k])
        rows.append((dev / bound, k, dev, bound))
    rows.sort(reverse=True)
    for r, k, dev, bound in rows[:5]:
        print(f"{label} {k}: {dev:.3g} from float64, bound {bound:.3g} (fp32 floor {floor[k]:.3g}), "
              f"{r:.2f} of it")
    for r, k, dev, bound in rows:
        assert dev <= bound, (f"{label} {k}: {dev:.3g} from the float64 oracle, bound {bound:.3g} "
                              f"(fp32 floor {floor[k]:.3g})")
    return rows[0][0], rows[0][1]
