"""Screening of the reference's sample_pdf discontinuity for the GPU parity
tests (test infrastructure): a fine depth may move by a whole bin when its u
lies within an ulp-scale distance of a CDF knot, and every such move must be
explained by that proximity -- a screened ray is never just "rare"."""
import numpy as np
import torch


def _cdf(w):
    """sample_pdf's CDF as the reference forms it (rendering.py:29-33, fp32)."""
    w = torch.as_tensor(w).float()[:, 1:-1] + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    return torch.cat([torch.zeros_like(cdf[:, :1]), cdf], -1)


def pdf_flips(z_fine_ours, ocap, u, thr=1e-5):
    """(moved, explained) rays of a render: a ray's fine depths moved when some
    importance depth of the reference (sample_pdf's z for u[j]) is missing from
    our merged depths; the move is explained when every such u[j] lies within
    ``thr`` of one of the reference's CDF knots (an ulp of CDF difference -- from
    the coarse weights, or from the sum order of the CDF's normalisation --
    puts it in the neighbouring bin, a whole bin away)."""
    zf = z_fine_ours.detach().cpu().numpy()
    zp = ocap["z_pdf"].numpy()
    cdf = _cdf(ocap["weights_coarse"]).double().numpy()
    u = np.asarray(u, np.float64)
    moved = np.zeros(zf.shape[0], bool)
    explained = np.zeros(zf.shape[0], bool)
    for r in range(zf.shape[0]):
        missing = ~np.isin(zp[r], zf[r])
        if missing.any():
            moved[r] = True
            d = np.abs(cdf[r][None, :] - u[r][missing][:, None]).min(1)
            explained[r] = bool((d < thr).all())
    return moved, explained


