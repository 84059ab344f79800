"""The oracle's weight normalization (``wn_weight`` / ``wn_grads``) against torch's own
``nn.utils.weight_norm`` (dim 0) forward and autograd, the module TD3_featured.py:33-35 / 68-70
wraps every Linear in -- at widths and scales beyond the golden fixture's (CPU)."""
import warnings

import numpy as np
import pytest

from helpers import orc


@pytest.mark.parametrize("n,k,scale", [(500, 17, 1.0), (400, 500, 0.05), (1, 200, 3.0), (6, 300, 1.0)])
def test_wn_forward_backward_match_torch(n, k, scale):
    import torch
    rs = np.random.RandomState(n * 1000 + k)
    v = (rs.standard_normal((n, k)) * scale).astype(np.float32)
    g = rs.uniform(0.5, 1.5, size=(n, 1)).astype(np.float32)
    x = rs.standard_normal((64, k)).astype(np.float32)
    gz = rs.standard_normal((64, n)).astype(np.float32)
    lin = torch.nn.Linear(k, n, bias=False)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", FutureWarning)
        lin = torch.nn.utils.weight_norm(lin)
    with torch.no_grad():
        lin.weight_g.copy_(torch.from_numpy(g))
        lin.weight_v.copy_(torch.from_numpy(v))
    z = lin(torch.from_numpy(x))
    z.backward(torch.from_numpy(gz))
    w = orc.wn_weight(g, v)
    np.testing.assert_allclose(w, lin.weight.detach().numpy(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(x @ w.T, z.detach().numpy(), rtol=1e-4, atol=1e-5)
    gW = (gz.T @ x).astype(np.float32)
    dg, dv = orc.wn_grads(gW, g, v)
    tg, tv = lin.weight_g.grad.numpy(), lin.weight_v.grad.numpy()
    np.testing.assert_allclose(dg, tg, rtol=1e-4, atol=1e-5 * np.abs(tg).max())
    np.testing.assert_allclose(dv, tv, rtol=1e-4, atol=1e-5 * np.abs(tv).max())
