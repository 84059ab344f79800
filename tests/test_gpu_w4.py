"""The k-quad weight images (td3.hip Group::P4 / T4, kernels.h GemmProb::wsk) change where the
forward GEMM stages read their weights, not what they read or the order they sum it in: a plan that
reads the images (TD3_W4=1, the default) and one that reads the row-major arena
(TD3_W4=0) give bit-identical parameters -- through Philox steps, a td3_set_params mid-run (the
images go stale and are repacked before the next step) and batch-size changes (plan rebuilds over
every dW kernel that keeps the images: dw_kernel, dw64_kernel, the split-K combine)."""
import numpy as np
import pytest

from helpers import featured_setup, gen

pytestmark = pytest.mark.gpu


class Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def _make(S):
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    hp = dict(S["hp"])
    lr = hp.pop("lr", 1e-4)
    pol = TD3(Box((S["sd"],)), Box((S["ad"],)), max_action=S["ma"], norm=S["norm"], lr=lr, init="none", **hp)
    pol.set_weights(S["actor"], S["critic"])
    rb = ReplayBuffer_featured(Box((S["sd"],)), Box((S["ad"],)), max_size=gen.BUFFER_ROWS, seed=11)
    s, a, s2, r, d = gen.fill_featured_buffer(S["sd"], S["ad"], S["ma"], gen.BUFFER_ROWS, gen.SEED)
    rb.add_batch(s, a, s2, r, d)
    return pol, rb


def _snap(pol):
    return [v.flat().copy() for v in (pol.actor, pol.critic, pol.actor_target, pol.critic_target)]


def _flags(pol):
    import ctypes as C
    from td3_amd import _lib
    f = C.c_int(-1)
    _lib.check(pol._lib.td3_debug_plan_flags(pol._h, C.byref(f)), "td3_debug_plan_flags")
    return f.value


def _run(S, w4, monkeypatch):
    monkeypatch.setenv("TD3_W4", w4)           # read when a step plan is built
    pol, rb = _make(S)
    B = S["B"]
    out = []
    for _ in range(12):
        pol.train(rb, B)
    assert _flags(pol) & 1 == int(w4)          # the plan under test reads the images (or not)
    out.append(_snap(pol))
    rs = np.random.RandomState(7)              # new online and target weights: the images go stale
    nd = lambda d: {k: (v + 0.01 * rs.standard_normal(v.shape)).astype(np.float32) for k, v in d.items()}
    pol.set_weights(nd(pol.actor.numpy_dict()), nd(pol.critic.numpy_dict()),
                    nd(pol.actor_target.numpy_dict()), nd(pol.critic_target.numpy_dict()))
    for _ in range(6):
        pol.train(rb, B)
    out.append(_snap(pol))
    for b in (B // 2, B, 600, 1024, B):        # plan rebuilds: dw_kernel, dw64_kernel, split-K + combine
        for _ in range(3):
            pol.train(rb, b)
        assert _flags(pol) & 1 == int(w4)
    out.append(_snap(pol))
    pol.sync()
    return out


@pytest.mark.parametrize("name", ["hc_layer", "hc_none", "pend_layer", "hum_layer"])
def test_k_quad_images_bit_identical(name, monkeypatch):
    S = featured_setup(name)
    a = _run(S, "1", monkeypatch)
    b = _run(S, "0", monkeypatch)
    for phase, (x, y) in enumerate(zip(a, b)):
        for g, (u, v) in enumerate(zip(x, y)):
            assert np.array_equal(u, v), (name, phase, ("actor", "critic", "actor_target", "critic_target")[g],
                                          int(np.sum(u != v)))


@pytest.mark.parametrize("name,b,shard,buckets", [("hc_layer", 128, "1", "0"), ("hc_layer", 128, "0", "0"),
                                                  ("hum_layer", 1024, "1", "1")])
def test_k_quad_images_data_parallel(name, b, shard, buckets, monkeypatch):
    """Data-parallel plans (two td3_comm_init_local replicas) update P / T with the flat optimizer
    behind the exchange and repack the images in a stage of their own (push_w4_pack): the sharded and
    the all-reduce schedules, and Humanoid's overlapped two-bucket critic, bit-identical to the
    row-major plans over free-running Philox steps and a mid-run set_weights."""
    from td3_amd.data_parallel import local_group, train_local
    S = featured_setup(name)
    monkeypatch.setenv("TD3_DP_SHARD", shard)
    monkeypatch.setenv("TD3_DP_BUCKETS", buckets)
    res = []
    for w4 in ("1", "0"):
        monkeypatch.setenv("TD3_W4", w4)
        pols, rbs = [], []
        for _ in range(2):
            p, rb = _make(S)
            pols.append(p)
            rbs.append(rb)
        local_group(pols)
        snaps = []
        for _ in range(5):
            train_local(pols, rbs, b)
        assert _flags(pols[0]) & 1 == int(w4)
        snaps.append([x for p in pols for x in _snap(p)])
        rs = np.random.RandomState(9)
        nd = lambda d: {k: (v + 0.01 * rs.standard_normal(v.shape)).astype(np.float32) for k, v in d.items()}
        new = [nd(pols[0].actor.numpy_dict()), nd(pols[0].critic.numpy_dict())]
        for p in pols:
            p.set_weights(*new)
        for _ in range(4):
            train_local(pols, rbs, b)
        snaps.append([x for p in pols for x in _snap(p)])
        for p in pols:
            p.sync()
        res.append(snaps)
    for phase, (x, y) in enumerate(zip(*res)):
        for i, (u, v) in enumerate(zip(x, y)):
            assert np.array_equal(u, v), (name, shard, phase, i, int(np.sum(u != v)))
