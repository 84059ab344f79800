"""The float64 host shadow of the replay buffers (td3_amd/my_replay_buffer.py _HostShadow) on CPU:
single and bulk row writes, including a bulk add longer than the ring, land where the reference's
``add`` (my_replay_buffer.py:109-117, restated by oracle.FeaturedBuffer) puts them."""
import numpy as np

from helpers import orc

from td3_amd.my_replay_buffer import _HostShadow


def test_shadow_rows_follow_reference_add():
    sd, ad, cap = 4, 2, 16
    rs = np.random.RandomState(0)
    ref = orc.FeaturedBuffer(sd, ad, cap)
    sh = _HostShadow.zeros({"state": (cap, sd), "action": (cap, ad), "next_state": (cap, sd),
                            "reward": (cap, 1), "not_done": (cap, 1)})
    for n in (1, 5, 1, 37, 3, 16, 2):                   # 37 > cap: the batch wraps twice
        s, a, s2 = rs.standard_normal((n, sd)), rs.standard_normal((n, ad)), rs.standard_normal((n, sd))
        r, d = rs.standard_normal(n), (rs.uniform(size=n) < 0.3).astype(np.float64)
        for i in range(n):
            ref.add(s[i], a[i], s2[i], r[i], d[i])
        if n == 1:
            sh.put((s[0], a[0], s2[0], r[0], 1. - d[0]))
        else:
            sh.put_batch((s, a, s2, r, 1. - d), n)
        assert sh.ptr == ref.ptr
        for k in sh.arrays:
            np.testing.assert_array_equal(sh.arrays[k], getattr(ref, k), err_msg=k)
