"""apply_lens_to_loss on the device (utils.data_utils -> mlvae_masked_mean), every reduction the
reference offers ('mean', 'batchmean', 'batch': ref:src/utils/data_utils.py:93-98), against the
reference's own outputs on the golden inputs (tests/golden/masks.npz, written by importing the
reference: T = 17 / 50 / 500 incl. the 127/500 length_to_mask quirk) and the gradient against the
oracle's autograd (oracle/vae_cpu.apply_lens_to_loss)."""
import os

import numpy as np
import pytest
import torch

from gpu_utils import need_gpu

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("T", [17, 50, 500])
@pytest.mark.parametrize("reduction,key", [("mean", "maskmean_rand"), ("batchmean", "batchmean_rand"),
                                           ("batch", "batch_rand")])
def test_masked_mean_reductions_match_reference(T, reduction, key):
    need_gpu()
    from oracle import vae_cpu as O
    from utils.data_utils import apply_lens_to_loss
    d = np.load(os.path.join(GOLDEN, "masks.npz"))
    r = torch.from_numpy(d[f"T{T}/rand"])
    lens = torch.from_numpy(d[f"T{T}/lens"])
    x = r.cuda().requires_grad_(True)
    out = apply_lens_to_loss(x, lens.cuda(), reduction)
    np.testing.assert_allclose(out.detach().cpu().numpy(), d[f"T{T}/{key}"], rtol=2e-6, atol=1e-7)
    cot = torch.randn(out.shape)
    (out * cot.cuda()).sum().backward()
    xr = r.clone().requires_grad_(True)
    (O.apply_lens_to_loss(xr, lens, reduction) * cot).sum().backward()
    torch.testing.assert_close(x.grad.cpu(), xr.grad, rtol=1e-6, atol=1e-9)
