"""metrics.py:4-13 on host operands (no GPU): eval.py:143 calls
metrics.psnr(img_gt, img_pred) with a CPU tensor and a numpy image; the
package's mse/psnr take the reference's own expression there (the HIP kernel
serves float32 device tensors, tests/test_gpu_loss.py)."""
import numpy as np
import torch

from nerf_pl_amd.losses import mse, psnr


def test_psnr_of_cpu_tensor_and_numpy_image_is_the_reference_expression():
    g = torch.Generator().manual_seed(3)
    gt = torch.rand(20, 30, 3, generator=g)
    pred = (gt.numpy() * 0.9 + 0.05).astype(np.float32)
    ref = -10 * torch.log10(torch.mean((gt - torch.from_numpy(pred)) ** 2))
    assert torch.equal(psnr(gt, pred), ref)
    assert torch.equal(mse(gt, gt * 0.5), torch.mean((gt - gt * 0.5) ** 2))


def test_masked_and_unreduced_metrics_on_cpu():
    g = torch.Generator().manual_seed(4)
    a, b = torch.rand(64, 3, generator=g), torch.rand(64, 3, generator=g)
    m = torch.rand(64, generator=g) > 0.5
    assert torch.equal(mse(a, b, m), torch.mean(((a - b) ** 2)[m]))
    assert torch.equal(mse(a, b, reduction="none"), (a - b) ** 2)
