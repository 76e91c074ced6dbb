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
measured at the unperturbed parameters and at nine points one fp32 ulp away
(every weight moved up or down by one ulp; each against its own float64
evaluation) -- the largest of the ten (FLOOR_POINTS), so one lucky fp32
evaluation cannot shrink the bound.  The float64 evaluations take the fp32
sample positions our kernels see (the oracle's fp32_positions): the floor then
measures the MLP's and the compositing's accumulation, not the fp32 rounding
of xyz = o + d z that the 2^9 encoding frequency turns into ~1e-3 rad.  ``C`` = 2: our gradient must be at most twice as far from
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
# the floor's evaluation points: the unperturbed weights and nine points one
# fp32 ulp away (seeds 1-9).  A heavily cancelled gradient (the coarse
# sigma.bias at cfg4 sums d sigma over 65,536 samples with 80x cancellation,
# and each d sigma is itself a difference, dw_i - R_i) moves by ~1e-3 when
# only the forward's outputs are rounded to fp32 (dev/sigma_bias.py); three
# points sampled that spread too thinly to bound it
FLOOR_POINTS = (None, 1, 2, 3, 4, 5, 6, 7, 8, 9)


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


def fp32_floor(grads32, grads64, spread=None):
    """per-tensor max over evaluation points of |g32 - g64| / |g64|: grads32 and
    grads64 are lists (one entry per point) of {name: tensor}; ``spread``
    (optional dict) receives every point's value per tensor"""
    floor = {}
    for g32, g64 in zip(grads32, grads64):
        for k, e64 in g64.items():
            e32 = g32[k].double()
            d = ((e32 - e64).norm() / (e64.norm() + 1e-30)).item()
            floor[k] = max(floor.get(k, 0.0), d)
            if spread is not None:
                spread.setdefault(k, []).append(d)
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


def mlp_flips(save, n, x64, p64, gmag=None, tol=1e-5, rel=1e-5):
    """(flipped, explained) per sample: a ReLU of the MLP (layers 1-8 and the
    dir layer, nerf.py:104-118) that our training forward switched on or off
    against float64 -- read from the activations the forward saved (h > 0 is
    the mask the backward used) -- is a discontinuity of that sample's
    gradient, like relu_kinks' compositing ReLU: the whole pre-activation
    gradient of that unit jumps between 0 and its full value.  Explained when
    every flipped unit's float64 pre-activation lies within ``tol`` of the
    kink.  The split arithmetic's pre-activations carry ~1e-6 absolute
    rounding where a layer sums terms of |x w| ~ 10-100 (raw xyz up to ~200
    at near/far 1/200 in the first layers' input), so its kink band is wider
    than fp32's: at cfg4 it switches a few of 65,536 coarse samples whose
    pre-activation is within 1e-6 of 0, and each such sample moves a whole
    layer's gradient by ~2.5e-3 of its norm (dev/grad_range.py).

    ``gmag`` (optional, per sample): the magnitude of the sample's output
    gradient (max |d raw|, float64 oracle).  A flip on a sample whose gradient
    is below ``rel`` of the batch's largest moves the parameter gradient by
    less than that fraction (times the layers' gain): such flips are counted
    but not returned as flipped.  Returns (flipped, explained, n_all_flips)."""
    from nerf_pl_amd import ops
    seg = ops.save_segments(save, n)
    xe, de = x64[:, :63], x64[:, 63:]
    flip = torch.zeros(n, dtype=torch.bool)
    expl = torch.ones(n, dtype=torch.bool)

    def note(pre, name, width):
        ours = ops.saved_rows(seg[name], n, width).cpu() > 0
        f = ours != (pre > 0)
        flip.logical_or_(f.any(1))
        expl.logical_and_(~(f & (pre.abs() > tol)).any(1))
        agree = 1 - f.double().mean().item()
        assert agree > 0.99, f"{name}: saved activations disagree with float64 ({agree:.3f})"

    with torch.no_grad():
        h = xe
        for i in range(8):
            if i == 4:
                h = torch.cat([xe, h], -1)
            pre = torch.nn.functional.linear(h, p64[f"xyz_encoding_{i + 1}.0.weight"],
                                             p64[f"xyz_encoding_{i + 1}.0.bias"])
            note(pre, f"h{i + 1}", 256)
            h = torch.relu(pre)
        feat = torch.nn.functional.linear(h, p64["xyz_encoding_final.weight"],
                                          p64["xyz_encoding_final.bias"])
        pre = torch.nn.functional.linear(torch.cat([feat, de], -1), p64["dir_encoding.0.weight"],
                                         p64["dir_encoding.0.bias"])
        note(pre, "hdir", 128)
    n_all = int(flip.sum())
    if gmag is not None:
        gmag = torch.as_tensor(gmag).double().cpu()
        flip &= gmag >= rel * gmag.max()
    return flip.numpy(), expl.numpy(), n_all
