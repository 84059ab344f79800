"""Ordering of replay-ring writes against training steps in flight, graph re-capture after a
ring is replaced, and Adam hyper-parameters adopted from a checkpoint.

Reference semantics: ``main.py:261`` adds the transition, ``main.py:269`` trains; in the
reference both are synchronous, so a step samples exactly the rows added before it
(``my_replay_buffer.py:109-128``).  Here adds are asynchronous uploads on the ring's stream and
steps are queued on the learner's stream, so the library must keep that order in both
directions: a step waits for the adds before it, and an add waits for the steps before it
(``Ring::read_ev``, replay.h).  The checks are bitwise: a run that queues adds behind steps in
flight must equal the same run synchronised after every call.
"""
import numpy as np
import pytest

from helpers import gen, featured_setup
from test_gpu_parity import Box, _make

pytestmark = pytest.mark.gpu

CAP = 1200


def _rows(sd, ad, n, seed):
    return gen.fill_featured_buffer(sd, ad, 1.0, n, seed)


def _ring_run(serial, use_graph="auto", phases=3, steps=8, add_rows=300):
    """steps x train(256), then add `add_rows` rows (the ring wraps and overwrites records),
    repeated; `serial` synchronises after every call."""
    from td3_amd.TD3_featured import TD3
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    S = featured_setup("hc_layer")
    sd, ad = S["sd"], S["ad"]
    pol = TD3(Box((sd,)), Box((ad,)), max_action=1.0, norm="layer", use_graph=use_graph, init="none")
    pol.set_weights(S["actor"], S["critic"])
    rb = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=CAP, seed=7)
    rb.add_batch(*_rows(sd, ad, 1000, 1))
    for ph in range(phases):
        for _ in range(steps):
            pol.train(rb, 256)
        if serial:
            pol.sync()
        rb.add_batch(*_rows(sd, ad, add_rows, 10 + ph))
        if serial:
            rb.flush()
            pol._lib.rb_sync(rb.handle)
    last = pol.train_step(rb, 256, stats=True)          # synchronises
    return pol, rb, last


@pytest.mark.parametrize("use_graph", ["auto", False])
def test_adds_queue_behind_steps_in_flight(use_graph):
    a, _, la = _ring_run(serial=True, use_graph=use_graph)
    b, _, lb = _ring_run(serial=False, use_graph=use_graph)
    np.testing.assert_array_equal(la["idx"], lb["idx"])
    np.testing.assert_array_equal(la["y"], lb["y"])
    for va, vb in ((a.critic, b.critic), (a.actor, b.actor), (a.critic_target, b.critic_target)):
        np.testing.assert_array_equal(va.flat(), vb.flat())


def test_philox_draws_reproducible_with_adds_between_steps():
    """two identical runs (graph auto, adds between steps, no synchronisation) draw
    the same rows: the draw depends on (seed, step, size) only, never on host/GPU timing."""
    _, _, la = _ring_run(serial=False, steps=5, phases=4, add_rows=90)
    _, _, lb = _ring_run(serial=False, steps=5, phases=4, add_rows=90)
    np.testing.assert_array_equal(la["idx"], lb["idx"])
    np.testing.assert_array_equal(la["noise"], lb["noise"])
    # the last step drew from the whole (full) ring
    assert la["idx"].max() < CAP and la["idx"].min() >= 0


def test_graph_recaptured_after_ring_reload(tmp_path):
    """Captured step graphs bake the ring in; ReplayBuffer.load() replaces the ring (usually at
    the same heap address) with another max_size: the next steps must use the new ring."""
    from td3_amd.my_replay_buffer import ReplayBuffer_featured
    S = featured_setup("hc_layer")
    sd, ad = S["sd"], S["ad"]
    other = ReplayBuffer_featured(Box((sd,)), Box((ad,)), max_size=gen.BUFFER_ROWS // 2 + 37)
    other.add_batch(*_rows(sd, ad, gen.BUFFER_ROWS // 2 + 50, 3))     # wraps
    other.save(str(tmp_path))

    a, rb = _make(S, use_graph=True)
    for _ in range(2):                                   # both step variants captured
        a.train(rb, S["B"])
    rb.load(str(tmp_path))
    for _ in range(3):
        a.train(rb, S["B"])

    b, rb_b = _make(S, use_graph=False)
    for _ in range(2):
        b.train(rb_b, S["B"])
    rb_b2 = ReplayBuffer_featured(Box((sd,)), Box((ad,)), load_folder=str(tmp_path))
    for _ in range(3):
        b.train(rb_b2, S["B"])
    a.sync()
    b.sync()
    for va, vb in ((a.critic, b.critic), (a.actor, b.actor), (a.critic_target, b.critic_target)):
        np.testing.assert_array_equal(va.flat(), vb.flat())


def test_optimizer_lr_adopted_from_checkpoint(tmp_path):
    """torch.optim.Adam.load_state_dict adopts the checkpoint's param_groups: a learner built with
    lr 1e-4 that loads a 3e-4 checkpoint steps exactly like the 3e-4 learner that wrote it."""
    S = featured_setup("hc_layer")
    S3 = dict(S, hp=dict(S["hp"], lr=3e-4))
    src, rb = _make(S3)
    for _ in range(3):
        src.train(rb, S["B"])
    src.save(str(tmp_path))
    dst, _ = _make(S)
    dst.load(str(tmp_path))
    dst.total_it = src.total_it
    for opt in (dst.actor_optimizer, dst.critic_optimizer):
        assert opt.state_dict()["param_groups"][0]["lr"] == pytest.approx(3e-4, rel=0, abs=1e-18)
    rs = np.random.RandomState(9)
    for _ in range(2):                                   # a critic-only and an actor step
        idx = rs.randint(0, gen.BUFFER_ROWS, S["B"])
        noise = rs.standard_normal((S["B"], S["ad"])).astype(np.float32)
        src.train_step(rb, S["B"], indices=idx, noise=noise)
        dst.train_step(rb, S["B"], indices=idx, noise=noise)
    for va, vb in ((src.actor, dst.actor), (src.critic, dst.critic), (src.actor_target, dst.actor_target)):
        np.testing.assert_array_equal(va.flat(), vb.flat())
