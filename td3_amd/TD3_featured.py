"""TD3 learner with the reference's surface, computing on MI355X through libtd3hip.

Drop-in for ``/root/reference/TD3_featured.py``:

* ``TD3(obs_space, action_space, max_action=1, lr=1e-4, norm=None, CDQ=True, **kwargs)``
  (:100-110; kwargs = TD3_base hyper-parameters discount / tau / policy_noise /
  noise_clip / policy_freq)
* ``train(replay_buffer, batch_size=100)`` (:123-171) -- one fused HIP step
  (hipGraph replay); a foreign duck-typed buffer is sampled through its own
  ``sample()`` and fed to the same kernels
* ``select_action(state)`` (:113-115), ``eval_q(state, action)`` (:117-121)
* ``actor`` / ``critic`` / ``actor_target`` / ``critic_target`` expose
  ``state_dict()`` / ``load_state_dict()`` with the reference keys; the two
  optimizers expose torch-Adam-format ``state_dict()`` / ``load_state_dict()``;
  ``save`` / ``load`` (TD3_base.py:26-50) therefore interoperate with reference
  checkpoints.

Initial weights: the networks are initialised by constructing the same
``torch.nn.Linear`` / ``LayerNorm`` modules on the CPU in the reference's order
(Actor, then Critic q1, q2), so ``torch.manual_seed(s)`` before ``TD3(...)`` gives
the reference's initial weights; the targets start as exact copies
(``copy.deepcopy`` at :102, :107).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np

from . import _lib
from ._lib import check
from .TD3_base import TD3_base
from .my_replay_buffer import ReplayBuffer_featured, default_device_index

ACTOR_ARCH = (500, 400, 300)   # TD3_featured.py:19
Q_ARCH = (500, 400, 200)       # TD3_featured.py:54


def _torch():
    import torch
    return torch


class _ParamView:
    """state_dict() / load_state_dict() over one parameter group of the C arenas."""

    def __init__(self, owner, which, group):
        self._o, self._which, self._group = owner, which, group

    def names_shapes(self):
        return self._o._tensors[self._group]

    def flat(self):
        n = self._o._nparams[self._group]
        out = np.empty(n, dtype=np.float32)
        check(self._o._lib.td3_get_params(self._o._h, self._which, _lib.fptr(out), n), "td3_get_params")
        return out

    def set_flat(self, flat):
        flat = np.ascontiguousarray(flat, dtype=np.float32)
        n = self._o._nparams[self._group]
        if flat.size != n:
            raise ValueError(f"expected {n} floats, got {flat.size}")
        check(self._o._lib.td3_set_params(self._o._h, self._which, _lib.fptr(flat), n), "td3_set_params")

    def numpy_dict(self):
        flat = self.flat()
        out = OrderedDict()
        o = 0
        for name, shape in self.names_shapes():
            k = int(np.prod(shape))
            out[name] = flat[o:o + k].reshape(shape).copy()
            o += k
        return out

    def state_dict(self):
        torch = _torch()
        return OrderedDict((k, torch.from_numpy(v)) for k, v in self.numpy_dict().items())

    def load_state_dict(self, sd, strict=True):
        parts = []
        for name, shape in self.names_shapes():
            if name not in sd:
                raise KeyError(f"missing key {name!r} in state_dict")
            v = sd[name]
            v = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
            if tuple(v.shape) != tuple(shape):
                raise ValueError(f"{name}: shape {tuple(v.shape)} != {tuple(shape)}")
            parts.append(v.astype(np.float32).reshape(-1))
        if strict:
            extra = set(sd.keys()) - {n for n, _ in self.names_shapes()}
            if extra:
                raise KeyError(f"unexpected keys {sorted(extra)}")
        self.set_flat(np.concatenate(parts))

    def parameters(self):
        return [v for v in self.state_dict().values()]


class _AdamView:
    """torch.optim.Adam-format state_dict over the fused optimizer state."""

    def __init__(self, owner, group):
        self._o, self._group = owner, group
        self._m = _lib.TD3_ACTOR_ADAM_M if group == 0 else _lib.TD3_CRITIC_ADAM_M
        self._v = _lib.TD3_ACTOR_ADAM_V if group == 0 else _lib.TD3_CRITIC_ADAM_V

    def _step(self):
        t, cs, as_ = self._o._counters()
        return as_ if self._group == 0 else cs

    def state_dict(self):
        torch = _torch()
        if getattr(self._o, "_dp_rccl", False):     # sharded moments: a collective gather first
            check(self._o._lib.td3_dp_gather_optimizer_state(self._o._h), "td3_dp_gather_optimizer_state")
        m = _ParamView(self._o, self._m, self._group).numpy_dict()
        v = _ParamView(self._o, self._v, self._group).numpy_dict()
        step = self._step()
        state = {}
        if step > 0:
            for i, k in enumerate(m):
                state[i] = {"step": torch.tensor(float(step)), "exp_avg": torch.from_numpy(m[k]),
                            "exp_avg_sq": torch.from_numpy(v[k])}
        lr, b1, b2, eps = self._o._adam_hparams(self._group)
        group = {"lr": lr, "betas": (b1, b2), "eps": eps, "weight_decay": 0,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False,
                 "differentiable": False, "fused": None, "decoupled_weight_decay": False,
                 "params": list(range(len(m)))}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        names = self._o._tensors[self._group]
        st = sd.get("state", {})
        mv = {0: OrderedDict(), 1: OrderedDict()}
        step = 0
        for i, (name, shape) in enumerate(names):
            s = st.get(i, st.get(str(i)))
            if s is None:
                mv[0][name] = np.zeros(shape, np.float32)
                mv[1][name] = np.zeros(shape, np.float32)
                continue
            mv[0][name] = np.asarray(s["exp_avg"].cpu().numpy() if hasattr(s["exp_avg"], "cpu") else s["exp_avg"])
            mv[1][name] = np.asarray(s["exp_avg_sq"].cpu().numpy() if hasattr(s["exp_avg_sq"], "cpu") else s["exp_avg_sq"])
            step = int(float(s["step"]))
        _ParamView(self._o, self._m, self._group).load_state_dict(mv[0])
        _ParamView(self._o, self._v, self._group).load_state_dict(mv[1])
        t, cs, as_ = self._o._counters()
        if self._group == 0:
            self._o._set_counters(t, cs, step)
        else:
            self._o._set_counters(t, step, as_)
        pg = sd.get("param_groups")
        if pg:
            self._o._adam_from_group(self._group, pg[0])

    def zero_grad(self, set_to_none=True):
        pass


def torch_default_init(sd, ad, norm, actor_arch=ACTOR_ARCH, q_arch=Q_ARCH):
    """Initial weights drawn exactly like the reference constructors (global torch RNG)."""
    torch = _torch()
    nn = torch.nn

    def mlp(inp, arch, out, prefix):
        dims = [inp] + list(arch)
        lin = [nn.Linear(dims[i], dims[i + 1]) for i in range(len(arch))] + [nn.Linear(arch[-1], out)]
        d = OrderedDict()
        for i, l in enumerate(lin):
            if norm == "weight_normalization":
                # torch.nn.utils.weight_norm(Linear) (TD3_featured.py:33-35, 68-70, dim 0): v = W,
                # g = ||W|| per output row; it draws no random numbers
                import warnings
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore", FutureWarning)
                    l = nn.utils.weight_norm(l)
                for k in ("bias", "weight_g", "weight_v"):
                    d[f"{prefix}linears.{i}.{k}"] = getattr(l, k).detach().numpy().copy()
                continue
            d[f"{prefix}linears.{i}.weight"] = l.weight.detach().numpy().copy()
            d[f"{prefix}linears.{i}.bias"] = l.bias.detach().numpy().copy()
        if norm == "layer":
            for i, dim in enumerate(arch):
                d[f"{prefix}lnorms.{i}.weight"] = np.ones(dim, np.float32)
                d[f"{prefix}lnorms.{i}.bias"] = np.zeros(dim, np.float32)
        return d

    actor = mlp(sd, actor_arch, ad, "")
    critic = mlp(sd + ad, q_arch, 1, "q1.")
    critic.update(mlp(sd + ad, q_arch, 1, "q2."))
    return actor, critic


class TD3(TD3_base):
    """TD3_featured.TD3 (TD3_featured.py:99-171) on the HIP pipeline."""

    def __init__(self, obs_space, action_space, max_action=1, lr=1e-4, norm=None, CDQ=True,
                 device=None, seed=0, use_graph="auto", actor_arch=ACTOR_ARCH, q_arch=Q_ARCH,
                 init="torch", **kwargs):
        super().__init__(max_action=max_action, **kwargs)
        self._lib = _lib.load()
        if norm not in (None, "layer", "weight_normalization"):
            raise ValueError(f"norm={norm!r} is not supported (None, 'layer' or 'weight_normalization')")
        self.norm = norm
        self.CDQ = CDQ          # TD3_featured ignores it (always twin critics), :100
        sd, ad = int(obs_space.shape[0]), int(action_space.shape[0])
        self.state_dim, self.action_dim = sd, ad
        self._dev = default_device_index() if device is None else int(device)
        torch = _torch()
        self.device = torch.device("cuda", self._dev)
        cfg = _lib.default_config()
        cfg.state_dim, cfg.action_dim = sd, ad
        for i in range(3):
            cfg.actor_hidden[i] = actor_arch[i]
            cfg.critic_hidden[i] = q_arch[i]
        cfg.norm = {None: 0, "layer": 1, "weight_normalization": 2}[norm]
        cfg.max_action = float(max_action)
        cfg.discount, cfg.tau = float(self.discount), float(self.tau)
        cfg.policy_noise, cfg.noise_clip = float(self.policy_noise), float(self.noise_clip)
        cfg.policy_freq = int(self.policy_freq)
        cfg.lr = float(lr)
        cfg.seed = int(seed)
        cfg.device = self._dev
        cfg.use_graph = 2 if use_graph == "auto" else (1 if use_graph else 0)
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
            a0, c0 = torch_default_init(sd, ad, norm, actor_arch, q_arch)
            self.set_weights(a0, c0)

    # ------------------------------------------------------------------ plumbing
    def _query_tensors(self, g):
        out = []
        name = C.create_string_buffer(128)
        rows, cols = C.c_int64(), C.c_int64()
        for i in range(self._lib.td3_tensor_count(self._h, g)):
            check(self._lib.td3_tensor_info(self._h, g, i, name, 128, C.byref(rows), C.byref(cols)),
                  "td3_tensor_info")
            shape = (rows.value, cols.value) if cols.value else (rows.value,)
            out.append((name.value.decode(), shape))
        return out

    def _counters(self):
        t, c, a = C.c_int64(), C.c_int64(), C.c_int64()
        check(self._lib.td3_get_counters(self._h, C.byref(t), C.byref(c), C.byref(a)), "td3_get_counters")
        return t.value, c.value, a.value

    def _set_counters(self, t, c, a):
        check(self._lib.td3_set_counters(self._h, int(t), int(c), int(a)), "td3_set_counters")

    def _adam_hparams(self, group):
        out = (C.c_double * 4)()
        check(self._lib.td3_get_adam(self._h, group, out), "td3_get_adam")
        return float(out[0]), float(out[1]), float(out[2]), float(out[3])

    def _adam_from_group(self, group, pg):
        """Adopt a checkpoint's param_groups[0] as torch.optim.Adam.load_state_dict does
        (lr / betas / eps); the options the reference never sets must keep torch's defaults."""
        for k, default in (("weight_decay", 0), ("amsgrad", False), ("maximize", False)):
            if pg.get(k, default) != default:
                raise ValueError(f"Adam {k}={pg[k]!r} is not supported (the reference uses the default)")
        lr, b1, b2, eps = self._adam_hparams(group)
        lr = float(pg.get("lr", lr))
        b1, b2 = (float(b) for b in pg.get("betas", (b1, b2)))
        eps = float(pg.get("eps", eps))
        check(self._lib.td3_set_adam(self._h, group, lr, b1, b2, eps), "td3_set_adam")

    def _stream(self):
        return None                      # the learner's own stream

    def _torch_order(self):
        from .my_replay_buffer import _TorchOrder
        return _TorchOrder(self._lib.td3_stream(self._h), self.device)

    @property
    def total_it(self):
        return self._counters()[0]

    @total_it.setter
    def total_it(self, v):
        t, c, a = self._counters()
        self._set_counters(v, c, a)

    def set_weights(self, actor, critic, actor_target=None, critic_target=None):
        """Load numpy/torch state dicts; targets default to copies (TD3_featured.py:102,107)."""
        self.actor.load_state_dict(actor)
        self.critic.load_state_dict(critic)
        self.actor_target.load_state_dict(actor if actor_target is None else actor_target)
        self.critic_target.load_state_dict(critic if critic_target is None else critic_target)

    # ------------------------------------------------------------------ reference API
    def select_action(self, state):
        s = np.ascontiguousarray(np.asarray(state, dtype=np.float32).reshape(1, -1))
        out = np.empty((1, self.action_dim), dtype=np.float32)
        check(self._lib.td3_select_action(self._h, _lib.fptr(s), _lib.fptr(out), 1), "td3_select_action")
        return out.reshape(-1)

    def select_action_batch(self, states):
        s = np.ascontiguousarray(np.asarray(states, dtype=np.float32).reshape(-1, self.state_dim))
        out = np.empty((s.shape[0], self.action_dim), dtype=np.float32)
        check(self._lib.td3_select_action(self._h, _lib.fptr(s), _lib.fptr(out), s.shape[0]),
              "td3_select_action")
        return out

    def eval_q(self, state, action):
        s = np.ascontiguousarray(np.asarray(state, dtype=np.float32).reshape(1, -1))
        a = np.ascontiguousarray(np.asarray(action, dtype=np.float32).reshape(1, -1))
        q = np.empty(2, dtype=np.float32)
        check(self._lib.td3_eval_q(self._h, _lib.fptr(s), _lib.fptr(a), _lib.fptr(q), 1), "td3_eval_q")
        return [q[0:1].copy(), q[1:2].copy()]

    def eval_q_batch(self, states, actions):
        """``eval_q`` over n (state, action) rows at once: (Q1 [n], Q2 [n])."""
        s = np.ascontiguousarray(np.asarray(states, dtype=np.float32).reshape(-1, self.state_dim))
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.float32).reshape(-1, self.action_dim))
        if s.shape[0] != a.shape[0]:
            raise ValueError("states and actions must have the same number of rows")
        n = s.shape[0]
        q = np.empty(2 * n, dtype=np.float32)
        check(self._lib.td3_eval_q(self._h, _lib.fptr(s), _lib.fptr(a), _lib.fptr(q), n), "td3_eval_q")
        return q[:n].copy(), q[n:].copy()

    def train(self, replay_buffer, batch_size=100):
        self.train_step(replay_buffer, batch_size)

    def train_step(self, replay_buffer, batch_size=100, indices=None, noise=None, stats=False):
        """``train`` with optional injected sample indices / N(0,1) noise and loss read-back."""
        B = int(batch_size)
        st = None
        keep = []
        if stats:
            st = _lib.td3_step_stats()
            y = np.empty(B, np.float32)
            q1 = np.empty(B, np.float32)
            q2 = np.empty(B, np.float32)
            idx = np.empty(B, np.int64)
            drawn = np.empty((B, self.action_dim), np.float32)
            keep = [y, q1, q2, idx, drawn]
            st.y, st.q1, st.q2, st.idx = (y.ctypes.data, q1.ctypes.data, q2.ctypes.data, idx.ctypes.data)
            st.noise = drawn.ctypes.data
        nz = None
        if noise is not None:
            nz = np.ascontiguousarray(np.asarray(noise, dtype=np.float32).reshape(B, self.action_dim))
        if isinstance(replay_buffer, ReplayBuffer_featured):
            replay_buffer.flush(self._lib.td3_stream(self._h))   # in the step's stream order
            ix = None
            if indices is not None:
                ix = np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(B))
            check(self._lib.td3_train_step(self._h, replay_buffer.handle, B, self._stream(),
                                           _lib.i64ptr(ix) if ix is not None else None,
                                           _lib.fptr(nz) if nz is not None else None,
                                           C.byref(st) if st is not None else None),
                  "td3_train_step")
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
                check(self._lib.td3_train_step_batch(self._h, *[t.data_ptr() for t in ts], B, self._stream(),
                                                     _lib.fptr(nz) if nz is not None else None,
                                                     C.byref(st) if st is not None else None),
                      "td3_train_step_batch")
            keep.append(ts)
        if st is None:
            return None
        out = {"critic_loss": st.critic_loss, "actor_step": bool(st.actor_step),
               "y": keep[0], "q1": keep[1], "q2": keep[2], "idx": keep[3], "noise": keep[4]}
        if st.actor_step:
            out["actor_loss"] = st.actor_loss
        return out

    def sync(self):
        check(self._lib.td3_sync(self._h), "td3_sync")

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None and _lib.alive():
                self._lib.td3_destroy(self._h)
                self._h = None
        except Exception:
            pass
