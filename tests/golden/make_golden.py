"""Generate golden fixtures by running the REFERENCE implementation on CPU.

TEST INFRASTRUCTURE ONLY.  Run in the build container (where
``/root/reference`` exists); the GPU box never runs this script, it only reads
the committed ``tests/golden/*.npz`` files.

For every config in ``gen.FEATURED_CONFIGS`` / ``gen.PARTICLE_CONFIGS``:

1. build the reference learner (``TD3_featured.TD3`` / ``TD3_particles.TD3``)
   and ``load_state_dict`` the deterministic init of ``gen.init_params`` into
   the online AND target networks (targets are deep copies in the reference,
   ``TD3_featured.py:102,107``);
2. fill the reference replay buffer through its own ``add``
   (``my_replay_buffer.py:109-117``) with ``gen.fill_*_buffer``;
3. call ``policy.train(rb, B)`` ``steps`` times while recording the only two
   RNG draws inside ``train`` (``np.random.randint`` at
   ``my_replay_buffer.py:120`` and ``torch.randn_like`` at
   ``TD3_featured.py:132``), the losses and the Q / target values;
4. after every step store exact samples + (sum, sumsq, max|x|) of every
   parameter, target parameter, Adam moment and gradient.

Usage:  python tests/golden/make_golden.py  [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import contextlib
import io
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen  # noqa: E402


class _Box:
    def __init__(self, shape):
        self.shape = tuple(shape)


def _stub_particle_imports():
    # TD3_particles.py:2,10,11 import pysplishsplash / torchvision / gym at module
    # level; the learner never uses them.
    for name in ("pysplishsplash", "gym", "torchvision", "torchvision.models"):
        if name not in sys.modules:
            sys.modules[name] = types.ModuleType(name)
    sys.modules["torchvision"].models = sys.modules["torchvision.models"]


class _Recorder:
    """Monkey-patches the RNG draws and loss calls inside one ``train`` call."""

    def __init__(self, torch, F):
        self.torch, self.F = torch, F
        self.rec = {}

    @contextlib.contextmanager
    def active(self):
        torch, F = self.torch, self.F
        orig_randint = np.random.randint
        orig_randn_like = torch.randn_like
        orig_mse = F.mse_loss
        self.rec = {"mse": []}

        def randint(*a, **k):
            out = orig_randint(*a, **k)
            self.rec["idx"] = np.asarray(out, dtype=np.int64).copy()
            return out

        def randn_like(x, *a, **k):
            out = orig_randn_like(x, *a, **k)
            self.rec["noise"] = out.detach().cpu().numpy().astype(np.float32).copy()
            return out

        def mse(inp, tgt, *a, **k):
            out = orig_mse(inp, tgt, *a, **k)
            self.rec["mse"].append((inp.detach().numpy().copy(), tgt.detach().numpy().copy(),
                                    float(out.detach())))
            return out

        np.random.randint = randint
        torch.randn_like = randn_like
        F.mse_loss = mse
        try:
            yield self.rec
        finally:
            np.random.randint = orig_randint
            torch.randn_like = orig_randn_like
            F.mse_loss = orig_mse


def _store_module(out, prefix, module, salt_base=0):
    for i, (name, t) in enumerate(module.state_dict().items()):
        st, smp = gen.summarize(t.detach().numpy(), salt=salt_base + i)
        out[f"{prefix}/{name}/stats"] = st
        out[f"{prefix}/{name}/samples"] = smp


def _store_opt(out, prefix, opt, module, salt_base=0):
    names = [n for n, _ in module.named_parameters()]
    params = list(module.parameters())
    for i, (n, p) in enumerate(zip(names, params)):
        st = opt.state[p]
        for key in ("exp_avg", "exp_avg_sq"):
            s, smp = gen.summarize(st[key].numpy(), salt=salt_base + i)
            out[f"{prefix}/{key}/{n}/stats"] = s
            out[f"{prefix}/{key}/{n}/samples"] = smp
        out[f"{prefix}/step"] = np.array(float(st["step"]))


def _store_grads(out, prefix, module, salt_base=0):
    for i, (n, p) in enumerate(module.named_parameters()):
        s, smp = gen.summarize(p.grad.numpy(), salt=salt_base + i)
        out[f"{prefix}/{n}/stats"] = s
        out[f"{prefix}/{n}/samples"] = smp


def _load(module, params):
    import torch
    sd = {k: torch.from_numpy(v.copy()) for k, v in params.items()}
    module.load_state_dict(sd, strict=True)


@contextlib.contextmanager
def _weight_norm_deepcopy(TD3_featured):
    """``TD3.__init__`` deep-copies the online networks into the targets (TD3_featured.py:102,
    107).  With ``norm="weight_normalization"`` this torch refuses: ``weight_norm`` keeps the
    hook-computed ``weight`` as a plain (non-leaf) tensor attribute, and deepcopy only copies
    graph leaves.  For the duration of the constructor the module's ``copy`` is replaced by one
    whose deepcopy leaves that attribute out; the copy's forward pre-hook recomputes it from its
    own ``weight_g`` / ``weight_v`` (torch's weight_norm semantics), so the targets are exact
    copies as the reference intends.  Nothing else of the reference is changed."""
    orig = TD3_featured.copy

    class _Copy:
        @staticmethod
        def deepcopy(m):
            held = [(mod, mod.__dict__.pop("weight")) for mod in m.modules()
                    if "weight_g" in mod._parameters and "weight" in mod.__dict__]
            try:
                return orig.deepcopy(m)
            finally:
                for mod, w in held:
                    mod.__dict__["weight"] = w

    TD3_featured.copy = _Copy
    try:
        yield
    finally:
        TD3_featured.copy = orig


def make_featured(name, cfg, ref_mods, torch, F):
    sd, ad, ma, norm, B, steps, hp = cfg
    TD3_featured, my_rb = ref_mods
    wn = _weight_norm_deepcopy(TD3_featured) if norm == "weight_normalization" else contextlib.nullcontext()
    with contextlib.redirect_stdout(io.StringIO()), wn:   # TD3_featured.py:103 prints params
        pol = TD3_featured.TD3(_Box((sd,)), _Box((ad,)), max_action=ma, norm=norm, **hp)
    ashapes = gen.featured_actor_shapes(sd, ad, norm)
    cshapes = gen.featured_critic_shapes(sd, ad, norm)
    assert [(k, tuple(v.shape)) for k, v in pol.actor.state_dict().items()] == ashapes
    assert [(k, tuple(v.shape)) for k, v in pol.critic.state_dict().items()] == cshapes
    a0 = gen.init_params(ashapes, gen.SEED)
    c0 = gen.init_params(cshapes, gen.SEED + 100)
    for m, p in ((pol.actor, a0), (pol.actor_target, a0), (pol.critic, c0), (pol.critic_target, c0)):
        _load(m, p)

    rb = my_rb.ReplayBuffer_featured(_Box((sd,)), _Box((ad,)), max_size=gen.BUFFER_ROWS)
    s, a, s2, r, d = gen.fill_featured_buffer(sd, ad, ma, gen.BUFFER_ROWS, gen.SEED)
    for i in range(gen.BUFFER_ROWS):
        rb.add(s[i], a[i], s2[i], r[i], d[i])

    out = {"config/dims": np.array([sd, ad, B, steps]), "config/max_action": np.array(ma),
           "config/norm": np.array(norm or ""),
           "buffer/checksum": np.array([rb.state.sum(), rb.action.sum(), rb.next_state.sum(),
                                        rb.reward.sum(), rb.not_done.sum()])}
    rec = _Recorder(torch, F)
    outputs = {}

    def hook(tag):
        def f(_m, _i, o):
            outputs[tag] = o.detach().numpy().copy()
        return f

    pol.actor_target.register_forward_hook(hook("ta_out"))
    pol.actor.register_forward_hook(hook("pi"))
    pol.critic.q1.register_forward_hook(hook("q1_last"))
    np.random.seed(gen.SEED)
    torch.manual_seed(gen.SEED)
    for step in range(1, steps + 1):
        outputs.clear()
        with rec.active() as rc:
            pol.train(rb, B)
        p = f"step{step}"
        out[f"{p}/idx"] = rc["idx"]
        out[f"{p}/noise"] = rc["noise"]
        (q1, y, l1), (q2, y2, l2) = rc["mse"]
        assert np.array_equal(y, y2)
        out[f"{p}/q1"], out[f"{p}/q2"], out[f"{p}/y"] = q1, q2, y
        out[f"{p}/critic_loss"] = np.array(l1 + l2, dtype=np.float64)
        out[f"{p}/critic_loss_parts"] = np.array([l1, l2], dtype=np.float64)
        out[f"{p}/ta_out"] = outputs["ta_out"]
        actor_step = pol.total_it % pol.policy_freq == 0
        out[f"{p}/actor_step"] = np.array(actor_step)
        if actor_step:
            out[f"{p}/pi"] = outputs["pi"]
            out[f"{p}/actor_q1"] = outputs["q1_last"]
            out[f"{p}/actor_loss"] = np.array(-float(outputs["q1_last"].mean()))
            _store_grads(out, f"{p}/grad/actor", pol.actor)
        else:
            _store_grads(out, f"{p}/grad/critic", pol.critic, salt_base=500)
        _store_module(out, f"{p}/actor", pol.actor)
        _store_module(out, f"{p}/actor_target", pol.actor_target)
        _store_module(out, f"{p}/critic", pol.critic, salt_base=500)
        _store_module(out, f"{p}/critic_target", pol.critic_target, salt_base=500)
        _store_opt(out, f"{p}/critic_opt", pol.critic_optimizer, pol.critic, salt_base=500)
        if pol.actor_optimizer.state:
            _store_opt(out, f"{p}/actor_opt", pol.actor_optimizer, pol.actor)
    path = os.path.join(HERE, f"featured_{name}.npz")
    np.savez_compressed(path, **out)
    return path


def make_particles(name, cfg, TD3_particles, my_rb, torch, F):
    Fd, N, D, A, norm, cdq, B, steps = cfg
    obs = (_Box((Fd,)), _Box((N, D)))
    with contextlib.redirect_stdout(io.StringIO()):
        pol = TD3_particles.TD3(obs, _Box((A,)), norm=norm, CDQ=cdq)
    ashapes = gen.particle_actor_shapes(Fd, D, A, norm)
    cshapes = gen.particle_critic_shapes(Fd, D, A, norm, cdq)
    assert [(k, tuple(v.shape)) for k, v in pol.actor.state_dict().items()] == ashapes
    assert [(k, tuple(v.shape)) for k, v in pol.critic.state_dict().items()] == cshapes
    a0 = gen.init_params(ashapes, gen.SEED)
    c0 = gen.init_params(cshapes, gen.SEED + 100)
    for m, p in ((pol.actor, a0), (pol.actor_target, a0), (pol.critic, c0), (pol.critic_target, c0)):
        _load(m, p)
    rb = my_rb.ReplayBuffer_particles(obs, _Box((A,)), max_size=gen.BUFFER_ROWS)
    f, pp, a, f2, pp2, r, d = gen.fill_particle_buffer(Fd, N, D, A, gen.BUFFER_ROWS, gen.SEED)
    for i in range(gen.BUFFER_ROWS):
        rb.add((f[i], pp[i]), a[i], (f2[i], pp2[i]), r[i], d[i])
    out = {"config/dims": np.array([Fd, N, D, A, B, steps, int(cdq)]),
           "config/norm": np.array(norm or ""),
           "buffer/checksum": np.array([rb.state_features.sum(), rb.state_particles.sum(),
                                        rb.action.sum(), rb.next_state_features.sum(),
                                        rb.next_state_particles.sum(), rb.reward.sum(),
                                        rb.not_done.sum()])}
    rec = _Recorder(torch, F)
    outputs = {}

    def hook(tag):
        def f_(_m, _i, o):
            outputs[tag] = o.detach().numpy().copy()
        return f_

    pol.actor_target.register_forward_hook(hook("ta_out"))
    pol.actor.register_forward_hook(hook("pi"))
    pol.critic.q1.register_forward_hook(hook("q1_last"))
    np.random.seed(gen.SEED)
    torch.manual_seed(gen.SEED)
    for step in range(1, steps + 1):
        outputs.clear()
        with rec.active() as rc:
            pol.train(rb, B)
        p = f"step{step}"
        out[f"{p}/idx"] = rc["idx"]
        out[f"{p}/noise"] = rc["noise"]
        out[f"{p}/y"] = rc["mse"][0][1]
        for j, (q, _y, l) in enumerate(rc["mse"]):
            out[f"{p}/q{j + 1}"] = q
        out[f"{p}/critic_loss"] = np.array(sum(m[2] for m in rc["mse"]), dtype=np.float64)
        out[f"{p}/ta_out"] = outputs["ta_out"]
        actor_step = pol.total_it % pol.policy_freq == 0
        out[f"{p}/actor_step"] = np.array(actor_step)
        if actor_step:
            out[f"{p}/pi"] = outputs["pi"]
            out[f"{p}/actor_q1"] = outputs["q1_last"]
            out[f"{p}/actor_loss"] = np.array(-float(outputs["q1_last"].mean()))
            _store_grads(out, f"{p}/grad/actor", pol.actor)
        else:
            _store_grads(out, f"{p}/grad/critic", pol.critic, salt_base=500)
        _store_module(out, f"{p}/actor", pol.actor)
        _store_module(out, f"{p}/actor_target", pol.actor_target)
        _store_module(out, f"{p}/critic", pol.critic, salt_base=500)
        _store_module(out, f"{p}/critic_target", pol.critic_target, salt_base=500)
        _store_opt(out, f"{p}/critic_opt", pol.critic_optimizer, pol.critic, salt_base=500)
        if pol.actor_optimizer.state:
            _store_opt(out, f"{p}/actor_opt", pol.actor_optimizer, pol.actor)
    path = os.path.join(HERE, f"particles_{name}.npz")
    np.savez_compressed(path, **out)
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    import torch
    import torch.nn.functional as F
    torch.set_num_threads(1)           # the oracle's own run-to-run determinism
    import my_replay_buffer
    import TD3_featured
    _stub_particle_imports()
    with contextlib.redirect_stdout(io.StringIO()):
        import TD3_particles
    for name, cfg in gen.FEATURED_CONFIGS.items():
        if args.only and args.only != name:
            continue
        print("wrote", make_featured(name, cfg, (TD3_featured, my_replay_buffer), torch, F))
    for name, cfg in gen.PARTICLE_CONFIGS.items():
        if args.only and args.only != name:
            continue
        print("wrote", make_particles(name, cfg, TD3_particles, my_replay_buffer, torch, F))


if __name__ == "__main__":
    main()
