"""HBM-resident replay buffers with the reference's Python surface.

Drop-in for ``/root/reference/my_replay_buffer.py``:

* ``ReplayBuffer_featured(obs_space, action_space, max_size=1e6, load_folder=None)``
  (:72-89) with ``add`` (:109-117), ``sample`` (:119-128), ``save`` / ``load``
  (:91-107) and the ``ptr`` / ``size`` / ``max_size`` attributes.
* ``ReplayBuffer_particles`` (:6-69), the same over (features, particles) states.

The storage lives in HBM (``libtd3hip``'s ring, one fp32 record per transition).
``add`` writes the transition straight into a host array of ring records (the fp32
cast the reference makes at ``sample``, :122-127, made once at ``add``: the same
rounding of the same float64 values) and ``flush`` ships the staged records in one
``rb_add_records`` call; ``sample`` / ``TD3.train`` flush first, so a transition
added at step t is samplable at step t exactly as in the reference (main.py:261
before :269).
``sample`` draws indices with a device Philox stream instead of the global numpy
MT19937 (``np.random.randint`` at :120) -- a documented, deliberate difference.

``host_shadow=True`` also keeps the reference's own float64 host arrays (:79-85 / :15-22) of
every row ``add`` / ``add_batch`` / ``load`` received, written by the same numpy row
assignments; ``save`` then writes those, so a reference folder loaded and saved back, or a
run resumed from a build-saved folder, sees the bytes the reference wrote.  Without it ``save``
writes the fp32 ring (float64(float32(x))).  The fp32 ring stays the training copy either way.
"""
from __future__ import annotations

import os
import pickle

import numpy as np

from . import _lib
from ._lib import check

_STAGE_ROWS = 4096


def _torch():
    import torch
    return torch


def default_device_index() -> int:
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("td3_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"]) % torch.cuda.device_count()
    return torch.cuda.current_device()


def _new_stage(buf, rows):
    """Host records staged by ``add`` (zeroed: the record pad stays 0) and their float*."""
    buf._stage = np.zeros((rows, buf.record_floats), dtype=np.float32)
    buf._stage_ptr = _lib.fptr(buf._stage)
    buf._n = 0


def _flush_stage(buf, stream=None):
    """Ship the staged records; ``stream`` (a learner's, from ``TD3.train``) queues them in that
    stream's order, so the step that samples them needs no cross-stream event (replay.h)."""
    n = buf._n
    if n:
        buf._n = 0
        check(buf._lib.rb_add_records(buf._h, buf._stage_ptr, n, stream), "rb_add_records")


class _SafeIntUnpickler(pickle.Unpickler):
    """ptr.pkl / size.pkl hold a pickled int (my_replay_buffer.py:93-95); refuse anything else."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a buffer file")


class _TorchOrder:
    """Orders work on one of the library's non-blocking streams against torch's current stream:
    on entry the library stream waits for torch's (tensors it reads or fills were made there),
    on exit torch's stream waits for the library's (its outputs are then safe to use)."""

    def __init__(self, stream_ptr, device):
        torch = _torch()
        self._torch_s = torch.cuda.current_stream(device)
        self._lib_s = torch.cuda.ExternalStream(int(stream_ptr), device=device)

    def __enter__(self):
        self._lib_s.wait_stream(self._torch_s)
        return self._lib_s

    def __exit__(self, *exc):
        self._torch_s.wait_stream(self._lib_s)
        return False


class _HostShadow:
    """The reference's float64 arrays (``store_np`` order, the reference's shapes), written row
    by row in ring order with the reference's own assignments (my_replay_buffer.py:109-117)."""

    def __init__(self, arrays, ptr=0):
        self.arrays = arrays                       # name -> ndarray, first dim = capacity
        self.cap = next(iter(arrays.values())).shape[0]
        self.ptr = int(ptr) % self.cap
        self.valid = True                          # False once a device-only write happened

    @classmethod
    def zeros(cls, shapes):
        return cls({k: np.zeros(shp) for k, shp in shapes.items()})

    def put(self, values):
        """One transition: ``values`` in store_np order (not_done already 1 - done)."""
        for arr, v in zip(self.arrays.values(), values):
            arr[self.ptr] = v
        self.ptr = (self.ptr + 1) % self.cap

    def put_batch(self, values, n):
        """n transitions (arrays of n rows each), as n consecutive ``put``."""
        skip = max(0, n - self.cap)                # rows a later row of the batch overwrites
        rows = (self.ptr + skip + np.arange(n - skip)) % self.cap
        for arr, v in zip(self.arrays.values(), values):
            arr[rows] = np.asarray(v).reshape((n,) + arr.shape[1:])[skip:]
        self.ptr = (self.ptr + n) % self.cap


def _save_folder(folder, ptr, size, arrays):
    """my_replay_buffer.py:91-99 / :24-32: ptr / size pickled (protocol 4), arrays np.save'd."""
    os.makedirs(folder, exist_ok=True)
    for attrib, v in (("ptr", int(ptr)), ("size", int(size))):
        with open(os.path.join(folder, attrib + ".pkl"), "wb") as f:
            pickle.dump(v, f, protocol=4)
    for attrib, arr in arrays.items():
        with open(os.path.join(folder, attrib + ".pkl"), "wb") as f:
            np.save(f, arr)


def _load_int(path):
    with open(path, "rb") as f:
        v = _SafeIntUnpickler(f).load()
    if not isinstance(v, (int, np.integer)):
        raise ValueError(f"{path}: expected an int, got {type(v)}")
    return int(v)


class ReplayBuffer_featured(object):
    """Flat-observation replay ring (my_replay_buffer.py:72-128) resident in HBM."""

    store_np = ["state", "action", "next_state", "reward", "not_done"]
    store_pkl = ["ptr", "size"]

    def __init__(self, obs_space, action_space, max_size=int(1e6), load_folder=None,
                 device=None, seed=0, host_shadow=False):
        self._lib = _lib.load()
        self.host_shadow = bool(host_shadow)
        self._shadow = None
        self.state_dim = int(obs_space.shape[0])
        self.action_dim = int(action_space.shape[0])
        self._dev = default_device_index() if device is None else int(device)
        torch = _torch()
        self.device = torch.device("cuda", self._dev)
        self.seed = int(seed)
        self._h = None
        self._n = 0
        if load_folder is not None:
            self.load(load_folder)
        else:
            self._create(int(max_size))

    # ------------------------------------------------------------------ plumbing
    def _create(self, max_size):
        import ctypes as C
        if self._h is not None:
            self._lib.rb_destroy(self._h)
            self._h = None
        h = C.c_void_p()
        check(self._lib.rb_create(self.state_dim, self.action_dim, max_size, self._dev,
                                  self.seed, C.byref(h)), "rb_create")
        self._h = h
        self.max_size = max_size
        info = self._info()
        self.record_floats = info.record_floats
        _new_stage(self, _STAGE_ROWS)
        sd, ad = self.state_dim, self.action_dim
        # replay.h record: [ s | a | s' | r | not_done | pad ]
        self._cols = (slice(0, sd), slice(sd, sd + ad), slice(sd + ad, 2 * sd + ad),
                      slice(2 * sd + ad, 2 * sd + ad + 1), slice(2 * sd + ad + 1, 2 * sd + ad + 2))
        self._shadow = _HostShadow.zeros(self._shapes(max_size)) if self.host_shadow else None

    def _shapes(self, n):
        sd, ad = self.state_dim, self.action_dim
        return {"state": (n, sd), "action": (n, ad), "next_state": (n, sd), "reward": (n, 1),
                "not_done": (n, 1)}

    def _info(self):
        info = _lib.rb_info_t()
        check(self._lib.rb_info(self._h, info), "rb_info")
        return info

    @property
    def handle(self):
        return self._h

    @property
    def ptr(self):
        self.flush()
        return int(self._info().ptr)

    @property
    def size(self):
        self.flush()
        return int(self._info().size)

    def _stream(self):
        return None                      # the ring's own stream (see _torch_order)

    def _torch_order(self):
        return _TorchOrder(self._lib.rb_stream(self._h), self.device)

    # ------------------------------------------------------------------ reference API
    def add(self, state, action, next_state, reward, done):
        """my_replay_buffer.py:109-117 (stores not_done = 1 - done): numpy row assignment as the
        reference's, into the staged fp32 record."""
        row = self._stage[self._n]
        cs, ca, cs2, cr, cnd = self._cols
        row[cs] = state
        row[ca] = action
        row[cs2] = next_state
        row[cr] = reward
        row[cnd] = 1. - np.asarray(done, dtype=np.float64)
        if self._shadow is not None:
            self._shadow.put((state, action, next_state, reward, 1. - done))
        self._n += 1
        if self._n == len(self._stage):
            self.flush()

    def add_batch(self, state, action, next_state, reward, done):
        """Bulk add of n transitions (experience_injection.py / hindsight relabel path)."""
        self.flush()
        s = np.ascontiguousarray(state, dtype=np.float64).reshape(-1, self.state_dim)
        n = s.shape[0]
        a = np.ascontiguousarray(action, dtype=np.float64).reshape(n, self.action_dim)
        s2 = np.ascontiguousarray(next_state, dtype=np.float64).reshape(n, self.state_dim)
        r = np.ascontiguousarray(reward, dtype=np.float64).reshape(n)
        d = np.ascontiguousarray(done, dtype=np.float64).reshape(n)
        if self._shadow is not None:
            self._shadow.put_batch((s, a, s2, r, 1. - d), n)
        check(self._lib.rb_add(self._h, _lib.dptr(s), _lib.dptr(a), _lib.dptr(s2), _lib.dptr(r),
                               _lib.dptr(d), n, self._stream()), "rb_add")

    def flush(self, stream=None):
        _flush_stage(self, stream)

    def fill_synthetic(self, n, max_action=1.0, seed=0):
        """Device-side prefill with the SURVEY §8(d) synthetic distribution (bench/tests)."""
        self.flush()
        if self._shadow is not None:
            self._shadow.valid = False           # rows the host never saw: save() writes the ring
        check(self._lib.rb_fill_synthetic(self._h, int(n), float(max_action), int(seed),
                                          self._stream()), "rb_fill_synthetic")

    def sample(self, batch_size, indices=None, return_indices=False):
        """my_replay_buffer.py:119-128: (state, action, next_state, reward, not_done) fp32 on device."""
        torch = _torch()
        self.flush()
        B = int(batch_size)
        dev = self.device
        out = (torch.empty((B, self.state_dim), device=dev, dtype=torch.float32),
               torch.empty((B, self.action_dim), device=dev, dtype=torch.float32),
               torch.empty((B, self.state_dim), device=dev, dtype=torch.float32),
               torch.empty((B, 1), device=dev, dtype=torch.float32),
               torch.empty((B, 1), device=dev, dtype=torch.float32))
        idx_out = torch.empty((B,), device=dev, dtype=torch.int64)
        inj = None
        if indices is not None:
            inj = torch.as_tensor(np.asarray(indices, dtype=np.int64), device=dev)
            if inj.numel() != B:
                raise ValueError("indices must have batch_size entries")
            size = self.size
            if B and (int(inj.min()) < 0 or int(inj.max()) >= max(size, 1)):
                raise IndexError("index out of range of the filled buffer")
        with self._torch_order():
            check(self._lib.rb_sample(self._h, B, *[t.data_ptr() for t in out],
                                      inj.data_ptr() if inj is not None else None,
                                      idx_out.data_ptr(), self._stream()), "rb_sample")
        if return_indices:
            return out, idx_out
        return out

    # ------------------------------------------------------------------ persistence
    def _records(self):
        n = self.max_size
        rec = np.empty((n, self.record_floats), dtype=np.float32)
        check(self._lib.rb_read_records(self._h, 0, n, _lib.fptr(rec)), "rb_read_records")
        return rec

    def _arrays(self):
        rec = self._records()
        sd, ad = self.state_dim, self.action_dim
        return {
            "state": rec[:, :sd].astype(np.float64),
            "action": rec[:, sd:sd + ad].astype(np.float64),
            "next_state": rec[:, sd + ad:2 * sd + ad].astype(np.float64),
            "reward": rec[:, 2 * sd + ad:2 * sd + ad + 1].astype(np.float64),
            "not_done": rec[:, 2 * sd + ad + 1:2 * sd + ad + 2].astype(np.float64),
        }

    def _saved_arrays(self, info):
        sh = self._shadow
        if sh is not None and sh.valid:
            assert sh.ptr == int(info.ptr) % sh.cap, "host shadow out of step with the ring"
            return sh.arrays
        return self._arrays()

    def save(self, folder):
        """my_replay_buffer.py:91-99: ptr/size pickled (protocol 4), arrays via np.save (the float64
        host shadow when kept, else the fp32 ring widened)."""
        self.flush()
        info = self._info()
        _save_folder(folder, info.ptr, info.size, self._saved_arrays(info))

    def load(self, folder):
        """my_replay_buffer.py:101-107 (pickles are read by an int-only unpickler)."""
        self._n = 0                         # rows added before a load are replaced with it
        ptr = _load_int(os.path.join(folder, "ptr.pkl"))
        size = _load_int(os.path.join(folder, "size.pkl"))
        arrs = {}
        for attrib in self.store_np:
            with open(os.path.join(folder, attrib + ".pkl"), "rb") as f:
                arrs[attrib] = np.load(f, allow_pickle=False)
        n = arrs["state"].shape[0]
        self.state_dim = arrs["state"].shape[1]
        self.action_dim = arrs["action"].shape[1]
        self._create(n)
        if self.host_shadow:                     # the loaded arrays themselves, bytes untouched
            self._shadow = _HostShadow(arrs, ptr)
        sd, ad = self.state_dim, self.action_dim
        rec = np.zeros((n, self.record_floats), dtype=np.float32)
        rec[:, :sd] = arrs["state"]
        rec[:, sd:sd + ad] = arrs["action"]
        rec[:, sd + ad:2 * sd + ad] = arrs["next_state"]
        rec[:, 2 * sd + ad] = arrs["reward"].reshape(n)
        rec[:, 2 * sd + ad + 1] = arrs["not_done"].reshape(n)
        check(self._lib.rb_write_records(self._h, 0, n, _lib.fptr(rec), ptr % n, min(size, n)),
              "rb_write_records")

    def __del__(self):
        try:
            if self._h is not None and _lib.alive():
                self._lib.rb_destroy(self._h)
                self._h = None
        except Exception:
            pass


class ReplayBuffer_particles(object):
    """Particle-observation replay ring (my_replay_buffer.py:6-69) resident in HBM.

    ``obs_space`` is the reference's 2-tuple of Boxes: features ``[F]`` and particles
    ``[N, D]`` (TD3_particles.py:29, :37); a state is the tuple ``(features, particles)``.
    One fp32 record per transition holds both states; the learner's encoders read the
    particle blocks in place, so ``TD3.train`` moves no particle bytes for sampling.
    """

    store_np = ["state_features", "state_particles", "action", "next_state_features",
                "next_state_particles", "reward", "not_done"]
    store_pkl = ["ptr", "size"]

    def __init__(self, obs_space, action_space, max_size=int(1e6), load_folder=None,
                 device=None, seed=0, host_shadow=False):
        self._lib = _lib.load()
        self.host_shadow = bool(host_shadow)
        self._shadow = None
        self.feat_dim = int(obs_space[0].shape[0])
        self.n_particles, self.particle_dim = (int(x) for x in obs_space[1].shape)
        self.action_dim = int(action_space.shape[0])
        self._dev = default_device_index() if device is None else int(device)
        torch = _torch()
        self.device = torch.device("cuda", self._dev)
        self.seed = int(seed)
        self._h = None
        self._n = 0
        if load_folder is not None:
            self.load(load_folder)
        else:
            self._create(int(max_size))

    def _create(self, max_size):
        import ctypes as C
        if self._h is not None:
            self._lib.rb_destroy(self._h)
            self._h = None
        h = C.c_void_p()
        check(self._lib.rb_create_particles(self.feat_dim, self.n_particles, self.particle_dim,
                                            self.action_dim, max_size, self._dev, self.seed,
                                            C.byref(h)), "rb_create_particles")
        self._h = h
        self.max_size = max_size
        self.record_floats = self._info().record_floats
        _new_stage(self, max(1, _STAGE_ROWS // 16))
        self._cols = tuple(slice(c, c + w) for c, w in self._offsets().values())
        self._shadow = _HostShadow.zeros(self._shapes(max_size)) if self.host_shadow else None

    def _shapes(self, n):
        F, A, nd = self.feat_dim, self.action_dim, (self.n_particles, self.particle_dim)
        return {"state_features": (n, F), "state_particles": (n, *nd), "action": (n, A),
                "next_state_features": (n, F), "next_state_particles": (n, *nd), "reward": (n, 1),
                "not_done": (n, 1)}

    def _info(self):
        info = _lib.rb_info_t()
        check(self._lib.rb_info(self._h, info), "rb_info")
        return info

    @property
    def handle(self):
        return self._h

    @property
    def ptr(self):
        self.flush()
        return int(self._info().ptr)

    @property
    def size(self):
        self.flush()
        return int(self._info().size)

    def _stream(self):
        return None

    def _torch_order(self):
        return _TorchOrder(self._lib.rb_stream(self._h), self.device)

    def _np(self):
        return self.n_particles * self.particle_dim

    # ------------------------------------------------------------------ reference API
    def add(self, state, action, next_state, reward, done):
        """my_replay_buffer.py:46-56 (state = (features, particles); stores 1 - done)."""
        row = self._stage[self._n]
        cf, cp, ca, cf2, cp2, cr, cnd = self._cols
        nd = (self.n_particles, self.particle_dim)
        row[cf] = state[0]
        row[cp].reshape(nd)[...] = state[1]
        row[ca] = action
        row[cf2] = next_state[0]
        row[cp2].reshape(nd)[...] = next_state[1]
        row[cr] = reward
        row[cnd] = 1. - np.asarray(done, dtype=np.float64)
        if self._shadow is not None:
            self._shadow.put((state[0], state[1], action, next_state[0], next_state[1], reward, 1. - done))
        self._n += 1
        if self._n == len(self._stage):
            self.flush()

    def add_batch(self, feat, part, action, next_feat, next_part, reward, done):
        self.flush()
        F, npd, A = self.feat_dim, self._np(), self.action_dim
        f = np.ascontiguousarray(feat, dtype=np.float64).reshape(-1, F)
        n = f.shape[0]
        arrs = [f, np.ascontiguousarray(part, dtype=np.float64).reshape(n, npd),
                np.ascontiguousarray(action, dtype=np.float64).reshape(n, A),
                np.ascontiguousarray(next_feat, dtype=np.float64).reshape(n, F),
                np.ascontiguousarray(next_part, dtype=np.float64).reshape(n, npd),
                np.ascontiguousarray(reward, dtype=np.float64).reshape(n),
                np.ascontiguousarray(done, dtype=np.float64).reshape(n)]
        if self._shadow is not None:
            self._shadow.put_batch(arrs[:6] + [1. - arrs[6]], n)
        check(self._lib.rb_add_particles(self._h, *[_lib.dptr(x) for x in arrs], n, self._stream()),
              "rb_add_particles")

    def flush(self, stream=None):
        _flush_stage(self, stream)

    def fill_synthetic(self, n, max_action=1.0, seed=0):
        self.flush()
        if self._shadow is not None:
            self._shadow.valid = False
        check(self._lib.rb_fill_synthetic(self._h, int(n), float(max_action), int(seed), self._stream()),
              "rb_fill_synthetic")

    def sample(self, batch_size, indices=None, return_indices=False):
        """my_replay_buffer.py:58-69: the 7 fp32 device tensors."""
        torch = _torch()
        self.flush()
        B = int(batch_size)
        dev = self.device
        N, D, F, A = self.n_particles, self.particle_dim, self.feat_dim, self.action_dim
        out = (torch.empty((B, F), device=dev), torch.empty((B, N, D), device=dev),
               torch.empty((B, A), device=dev), torch.empty((B, F), device=dev),
               torch.empty((B, N, D), device=dev), torch.empty((B, 1), device=dev),
               torch.empty((B, 1), device=dev))
        idx_out = torch.empty((B,), device=dev, dtype=torch.int64)
        inj = None
        if indices is not None:
            inj = torch.as_tensor(np.asarray(indices, dtype=np.int64), device=dev)
            if inj.numel() != B:
                raise ValueError("indices must have batch_size entries")
            size = self.size
            if B and (int(inj.min()) < 0 or int(inj.max()) >= max(size, 1)):
                raise IndexError("index out of range of the filled buffer")
        with self._torch_order():
            check(self._lib.rb_sample_particles(self._h, B, *[t.data_ptr() for t in out],
                                                inj.data_ptr() if inj is not None else None,
                                                idx_out.data_ptr(), self._stream()), "rb_sample_particles")
        if return_indices:
            return out, idx_out
        return out

    # ------------------------------------------------------------------ persistence
    def _offsets(self):
        F, npd, A = self.feat_dim, self._np(), self.action_dim
        o = {}
        c = 0
        for name, w in (("state_features", F), ("state_particles", npd), ("action", A),
                        ("next_state_features", F), ("next_state_particles", npd), ("reward", 1),
                        ("not_done", 1)):
            o[name] = (c, w)
            c += w
        return o

    def save(self, folder):
        """my_replay_buffer.py:24-32 (ptr / size pickled with protocol 4, arrays np.save'd; the
        float64 host shadow when kept)."""
        self.flush()
        info = self._info()
        sh = self._shadow
        if sh is not None and sh.valid:
            assert sh.ptr == int(info.ptr) % sh.cap, "host shadow out of step with the ring"
            _save_folder(folder, info.ptr, info.size, sh.arrays)
            return
        n = self.max_size
        rec = np.empty((n, self.record_floats), dtype=np.float32)
        check(self._lib.rb_read_records(self._h, 0, n, _lib.fptr(rec)), "rb_read_records")
        shapes = self._shapes(n)
        _save_folder(folder, info.ptr, info.size,
                     {name: rec[:, c:c + w].astype(np.float64).reshape(shapes[name])
                      for name, (c, w) in self._offsets().items()})

    def load(self, folder):
        """my_replay_buffer.py:34-44 (int-only unpickler for ptr / size)."""
        self._n = 0                         # rows added before a load are replaced with it
        ptr = _load_int(os.path.join(folder, "ptr.pkl"))
        size = _load_int(os.path.join(folder, "size.pkl"))
        arrs = {}
        for attrib in self.store_np:
            with open(os.path.join(folder, attrib + ".pkl"), "rb") as f:
                arrs[attrib] = np.load(f, allow_pickle=False)
        n = arrs["state_features"].shape[0]
        self.feat_dim = arrs["state_features"].shape[1]
        self.n_particles, self.particle_dim = arrs["state_particles"].shape[1:3]
        self.action_dim = arrs["action"].shape[1]
        self._create(n)
        if self.host_shadow:
            self._shadow = _HostShadow(arrs, ptr)
        rec = np.zeros((n, self.record_floats), dtype=np.float32)
        for name, (c, w) in self._offsets().items():
            rec[:, c:c + w] = arrs[name].reshape(n, w)
        check(self._lib.rb_write_records(self._h, 0, n, _lib.fptr(rec), ptr % n, min(size, n)),
              "rb_write_records")

    def __del__(self):
        try:
            if self._h is not None and _lib.alive():
                self._lib.rb_destroy(self._h)
                self._h = None
        except Exception:
            pass


# The reference's module-level alias used by main.py:204-208.
ReplayBuffer = ReplayBuffer_featured
