"""Wide policy / actor heads (action width > 8; Humanoid: 17) stage their weight rows in LDS once per
workgroup (kernels.hip wide_stage, row kernels launched with kWideRows rows per workgroup) instead of
requesting them block by block.  The staged rows are the same values, used in the same order, so the
parameters after Philox steps (critic-only and policy steps) are bit-identical to the block-by-block
path (TD3_WIDE_HEADS=0), for both LayerNorm settings and for widths that leave a ragged last block."""
import numpy as np
import pytest

from helpers import featured_setup_dims
from test_gpu_w4 import _make, _snap

pytestmark = pytest.mark.gpu


def _run(S, on, monkeypatch):
    monkeypatch.setenv("TD3_WIDE_HEADS", on)   # read at each row-kernel launch
    pol, rb = _make(S)
    for _ in range(6):
        pol.train(rb, S["B"])
    pol.sync()
    return _snap(pol)


@pytest.mark.parametrize("sd,ad,norm,B", [(376, 17, "layer", 256), (376, 17, None, 256),
                                          (45, 9, "layer", 128), (60, 24, "layer", 1024)])
def test_wide_heads_bit_identical(sd, ad, norm, B, monkeypatch):
    S = featured_setup_dims(sd, ad, 1.0, norm, B)
    a = _run(S, "1", monkeypatch)
    b = _run(S, "0", monkeypatch)
    for g, (u, v) in enumerate(zip(a, b)):
        assert np.array_equal(u, v), (sd, ad, norm, ("actor", "critic", "actor_target", "critic_target")[g],
                                      int(np.sum(u != v)))
