"""TD3_particles learner with the reference's surface, computing on MI355X through libtd3hip.

Drop-in for ``/root/reference/TD3_particles.py``:

* ``TD3(obs_space, action_space, lr=1e-4, norm=None, CDQ=True, **kwargs)`` (:136-149) where
  ``obs_space`` is the 2-tuple (features Box [F], particles Box [N, D]) and kwargs are the
  TD3_base hyper-parameters (max_action, discount, tau, policy_noise, noise_clip, policy_freq)
* ``train(replay_buffer, batch_size=100)`` (:167-224): particle encoders (conv1 1xD, conv2 1x1,
  mean over particles), lnorm1 on the MLP input, Q heads with one output per action
  dimension, no clamp on the smoothed target action, tanh policy output, CDQ optional
* ``select_action((features, particles))`` (:153-157), ``eval_q(state, action)`` (:159-164)
* the same ``actor`` / ``critic`` / optimizer state_dict views and ``save`` / ``load`` as the
  featured learner (reference key layout, e.g. ``conv1.weight`` [256, 1, 1, D]).

Initial weights are drawn like the reference constructors: Actor, Actor (target, then
overwritten), Critic, Critic (target), each built from the same torch modules in the same
order, so ``torch.manual_seed(s)`` before ``TD3(...)`` gives the reference's initial weights.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np

from . import _lib
from ._lib import check
from .TD3_featured import TD3 as _FeaturedTD3
from .TD3_featured import _AdamView, _ParamView, _torch
from .TD3_base import TD3_base
from .my_replay_buffer import ReplayBuffer_particles, default_device_index

ARCH = (500, 400, 300)      # TD3_particles.py:25 / :76
NUM_FEATURES = 128          # :27


def torch_default_init(F, N, D, A, norm, cdq=True):
    """Initial weights drawn exactly like the reference constructors (global torch RNG)."""
    torch = _torch()
    nn = torch.nn

    def net(inp, out, prefix):
        conv1 = nn.Conv2d(1, NUM_FEATURES * 2, kernel_size=(1, D), stride=1)
        conv2 = nn.Conv1d(NUM_FEATURES * 2, NUM_FEATURES, kernel_size=1, stride=1)
        dims = [inp] + list(ARCH)
        lin = [nn.Linear(dims[i], dims[i + 1]) for i in range(len(ARCH))] + [nn.Linear(ARCH[-1], out)]
        d = OrderedDict()
        d[f"{prefix}conv1.weight"] = conv1.weight.detach().numpy().copy()
        d[f"{prefix}conv1.bias"] = conv1.bias.detach().numpy().copy()
        d[f"{prefix}conv2.weight"] = conv2.weight.detach().numpy().copy()
        d[f"{prefix}conv2.bias"] = conv2.bias.detach().numpy().copy()
        for i, l in enumerate(lin):
            d[f"{prefix}linears.{i}.weight"] = l.weight.detach().numpy().copy()
            d[f"{prefix}linears.{i}.bias"] = l.bias.detach().numpy().copy()
        if norm == "layer":
            d[f"{prefix}lnorm1.weight"] = np.ones(inp, np.float32)
            d[f"{prefix}lnorm1.bias"] = np.zeros(inp, np.float32)
            for i, dim in enumerate(ARCH):
                d[f"{prefix}lnorms.{i}.weight"] = np.ones(dim, np.float32)
                d[f"{prefix}lnorms.{i}.bias"] = np.zeros(dim, np.float32)
        return d

    def critic():
        c = net(NUM_FEATURES + F + A, A, "q1.")
        if cdq:
            c.update(net(NUM_FEATURES + F + A, A, "q2."))
        return c

    actor = net(NUM_FEATURES + F, A, "")
    net(NUM_FEATURES + F, A, "")             # actor_target = Actor(...) then load_state_dict (:139-141)
    crit = critic()
    critic()                                  # critic_target (:144-146)
    return actor, crit


_REF_SHAPES = {"conv1.weight": lambda D: (NUM_FEATURES * 2, 1, 1, D),
               "conv2.weight": lambda D: (NUM_FEATURES, NUM_FEATURES * 2, 1)}


class TD3(_FeaturedTD3):
    """TD3_particles.TD3 (TD3_particles.py:135-224) on the HIP pipeline."""

    def __init__(self, obs_space, action_space, lr=1e-4, norm=None, CDQ=True, device=None, seed=0,
                 use_graph="auto", init="torch", **kwargs):
        TD3_base.__init__(self, **kwargs)
        self._lib = _lib.load()
        if norm not in (None, "layer"):
            raise ValueError(f"norm={norm!r} is not supported (None or 'layer')")
        self.norm = norm
        self.CDQ = bool(CDQ)
        F = int(obs_space[0].shape[0])
        N, D = (int(x) for x in obs_space[1].shape)
        A = int(action_space.shape[0])
        self.feat_dim, self.n_particles, self.particle_dim = F, N, D
        self.state_dim, self.action_dim = F, A
        self._dev = default_device_index() if device is None else int(device)
        torch = _torch()
        self.device = torch.device("cuda", self._dev)
        cfg = _lib.default_config()
        cfg.state_dim, cfg.action_dim = F, A
        for i in range(3):
            cfg.actor_hidden[i] = ARCH[i]
            cfg.critic_hidden[i] = ARCH[i]
        cfg.norm = 1 if norm == "layer" else 0
        cfg.max_action = float(self.max_action)
        cfg.discount, cfg.tau = float(self.discount), float(self.tau)
        cfg.policy_noise, cfg.noise_clip = float(self.policy_noise), float(self.noise_clip)
        cfg.policy_freq = int(self.policy_freq)
        cfg.lr = float(lr)
        cfg.seed = int(seed)
        cfg.device = self._dev
        cfg.use_graph = 2 if use_graph == "auto" else (1 if use_graph else 0)
        cfg.particles = 1
        cfg.n_particles, cfg.particle_dim = N, D
        cfg.cdq = 1 if self.CDQ else 0
        self._cfg = cfg
        h = C.c_void_p()
        check(self._lib.td3_create(C.byref(cfg), C.byref(h)), "td3_create")
        self._h = h
        self._tensors = {g: self._query_tensors(g) for g in (0, 1)}
        self._nparams = {g: int(self._lib.td3_num_params(h, g)) for g in (0, 1)}
        self.actor = _ParamView(self, _lib.TD3_ACTOR, 0)
        self.actor_target = _ParamView(self, _lib.TD3_ACTOR_TARGET, 0)
        self.critic = _ParamView(self, _lib.TD3_CRITIC, 1)
        self.critic_target = _ParamView(self, _lib.TD3_CRITIC_TARGET, 1)
        self.actor_optimizer = _AdamView(self, 0)
        self.critic_optimizer = _AdamView(self, 1)
        if init == "torch":
            a0, c0 = torch_default_init(F, N, D, A, norm, self.CDQ)
            self.set_weights(a0, c0)

    def _query_tensors(self, g):
        out = []
        for name, shape in super()._query_tensors(g):
            base = name.split(".", 1)[1] if name.startswith(("q1.", "q2.")) else name
            if base in _REF_SHAPES:
                shape = _REF_SHAPES[base](self.particle_dim)
            out.append((name, shape))
        return out

    # ------------------------------------------------------------------ reference API
    def _state_arrays(self, states):
        F, N, D = self.feat_dim, self.n_particles, self.particle_dim
        feat = np.ascontiguousarray(np.asarray(states[0], dtype=np.float32).reshape(-1, F))
        part = np.ascontiguousarray(np.asarray(states[1], dtype=np.float32).reshape(-1, N * D))
        return feat, part

    def select_action(self, state):
        """TD3_particles.py:153-157: state = (features, particles) -> tanh action [A]."""
        feat, part = self._state_arrays(state)
        out = np.empty((1, self.action_dim), dtype=np.float32)
        check(self._lib.td3_select_action_particles(self._h, _lib.fptr(feat), _lib.fptr(part),
                                                    _lib.fptr(out), 1), "td3_select_action_particles")
        return out.reshape(-1)

    def select_action_batch(self, states):
        feat, part = self._state_arrays(states)
        n = feat.shape[0]
        out = np.empty((n, self.action_dim), dtype=np.float32)
        check(self._lib.td3_select_action_particles(self._h, _lib.fptr(feat), _lib.fptr(part),
                                                    _lib.fptr(out), n), "td3_select_action_particles")
        return out

    def eval_q(self, state, action):
        """TD3_particles.py:159-164: [Q1 [A], Q2 [A]] (one entry without CDQ)."""
        feat, part = self._state_arrays(state)
        a = np.ascontiguousarray(np.asarray(action, dtype=np.float32).reshape(1, -1))
        q = np.empty((2, self.action_dim), dtype=np.float32)
        check(self._lib.td3_eval_q_particles(self._h, _lib.fptr(feat), _lib.fptr(part), _lib.fptr(a),
                                             _lib.fptr(q), 1), "td3_eval_q_particles")
        return [q[0].copy(), q[1].copy()] if self.CDQ else [q[0].copy()]

    def _actor_learn(self, state_features, state_particles, stats=False):
        """TD3_particles.py:209-224: the delayed policy update on the given states (torch tensors or
        arrays, [B, F] and [B, N, D]), as ``evaluate_model.py:39-49`` calls it outside ``train``:
        -mean Q1(s, pi(s)), the actor's Adam step, Polyak of critic and actor.  ``total_it`` is not
        touched.  Returns None like the reference (``stats=True``: the actor loss)."""
        torch = _torch()
        F, N, D = self.feat_dim, self.n_particles, self.particle_dim
        f = torch.as_tensor(state_features, dtype=torch.float32).to(self.device).reshape(-1, F).contiguous()
        p = torch.as_tensor(state_particles, dtype=torch.float32).to(self.device).reshape(-1, N * D).contiguous()
        if f.shape[0] != p.shape[0]:
            raise ValueError(f"state_features has {f.shape[0]} rows, state_particles {p.shape[0]}")
        loss = C.c_double() if stats else None
        with self._torch_order():
            check(self._lib.td3_actor_learn_particles(self._h, f.data_ptr(), p.data_ptr(), int(f.shape[0]),
                                                      self._stream(), C.byref(loss) if stats else None),
                  "td3_actor_learn_particles")
        return float(loss.value) if stats else None

    def train_step(self, replay_buffer, batch_size=100, indices=None, noise=None, stats=False):
        """``train`` with optional injected sample indices / N(0,1) noise and loss read-back."""
        B, A = int(batch_size), self.action_dim
        st = None
        keep = []
        if stats:
            st = _lib.td3_step_stats()
            keep = [np.empty((B, A), np.float32), np.empty((B, A), np.float32), np.empty((B, A), np.float32),
                    np.empty(B, np.int64), np.empty((B, A), np.float32)]
            st.y, st.q1, st.q2, st.idx, st.noise = (k.ctypes.data for k in keep)
        nz = None
        if noise is not None:
            nz = np.ascontiguousarray(np.asarray(noise, dtype=np.float32).reshape(B, A))
        if isinstance(replay_buffer, ReplayBuffer_particles):
            replay_buffer.flush(self._lib.td3_stream(self._h))   # in the step's stream order
            ix = None
            if indices is not None:
                ix = np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(B))
            check(self._lib.td3_train_step(self._h, replay_buffer.handle, B, self._stream(),
                                           _lib.i64ptr(ix) if ix is not None else None,
                                           _lib.fptr(nz) if nz is not None else None,
                                           C.byref(st) if st is not None else None), "td3_train_step")
        else:
            torch = _torch()
            batch = replay_buffer.sample(B)
            ts = [torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous() for x in batch]
            # the batch was produced on torch's stream; on exit torch's stream waits for the
            # library's, so the blocks freed with `ts` are reused only after the step read them
            # (no record_stream: its free-time event on the library stream could outlive the
            # handle's stream, and a later stream created at the same address made torch's next
            # allocation fail with hipErrorCapturedEvent)
            with self._torch_order():
                check(self._lib.td3_train_step_batch_particles(
                    self._h, *[t.data_ptr() for t in ts], B, self._stream(),
                    _lib.fptr(nz) if nz is not None else None, C.byref(st) if st is not None else None),
                    "td3_train_step_batch_particles")
            keep.append(ts)
        if st is None:
            return None
        out = {"critic_loss": st.critic_loss, "actor_step": bool(st.actor_step),
               "y": keep[0], "q1": keep[1], "q2": keep[2], "idx": keep[3], "noise": keep[4]}
        if st.actor_step:
            out["actor_loss"] = st.actor_loss
        return out
