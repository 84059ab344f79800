"""Data-parallel TD3: one replay shard and one learner replica per GPU, the
gradients of each optimizer phase all-reduced before Adam.

The reference trains on one device (``TD3_featured.py:123-171``); the losses are batch means
(``F.mse_loss``, ``.mean()``), so the mean of the replicas' shard gradients is the gradient of the
loss over the concatenated global batch, and replicas that start equal stay equal (the all-reduced
sum is bit-identical on every rank).

* ``init_rccl(policy, dist)``: one process per GPU (``torch.distributed.run``); rank 0 makes the
  RCCL unique id, ``torch.distributed`` broadcasts it, ``td3_comm_init`` joins the communicator.
* ``local_group(policies)`` / ``train_local(...)``: the same data-parallel stage lists for n
  replicas inside ONE process on one device (``td3_comm_init_local``), whose all-reduce is a
  fixed-order device sum over the replicas' gradient arenas -- the test seam that exercises the
  product's all-reduce path without a second GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check


def init_rccl(policy, dist):
    """Join the RCCL communicator of the ``torch.distributed`` world (``td3_comm_init``)."""
    import torch
    lib = policy._lib
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.zeros(128, dtype=torch.uint8, device=policy.device)
    if rank == 0:
        uid = (C.c_ubyte * 128)()
        check(lib.td3_comm_unique_id(uid), "td3_comm_unique_id")
        t.copy_(torch.tensor(list(bytes(uid)), dtype=torch.uint8))
    dist.broadcast(t, 0)
    uid = (C.c_ubyte * 128)(*t.cpu().tolist())
    check(lib.td3_comm_init(policy._h, uid, world, rank), "td3_comm_init")
    policy._dp_rccl = True       # optimizer state_dict() gathers the sharded moments (collective)


def local_group(policies):
    """Make ``policies`` (same configuration, one device) the ranks 0..n-1 of one in-process
    data-parallel group.  They then step only through ``train_local``."""
    lib = policies[0]._lib
    hs = (C.c_void_p * len(policies))(*[p._h.value for p in policies])
    check(lib.td3_comm_init_local(hs, len(policies)), "td3_comm_init_local")


def train_local(policies, buffers, batch_size, indices=None, noise=None, stats=False):
    """One ``TD3.train(buffer_k, batch_size)`` of every replica k of a ``local_group``.

    ``indices`` [n, B] / ``noise`` [n, B, ad] replace the Philox draws (parity tests); with
    ``stats`` a list of per-replica dicts (critic loss, actor loss, y, q1, q2) is returned."""
    n = len(policies)
    lib = policies[0]._lib
    B = int(batch_size)
    ad = policies[0].action_dim
    for rb in buffers:                   # staged adds in rank 0's stream order (the steps' stream)
        rb.flush(lib.td3_stream(policies[0]._h))
    hs = (C.c_void_p * n)(*[p._h.value for p in policies])
    rbs = (C.c_void_p * n)(*[rb.handle.value for rb in buffers])
    ix = nz = None
    if indices is not None:
        ix = np.ascontiguousarray(np.asarray(indices, dtype=np.int64).reshape(n, B))
    if noise is not None:
        nz = np.ascontiguousarray(np.asarray(noise, dtype=np.float32).reshape(n, B, ad))
    st = None
    keep = []
    if stats:
        st = (_lib.td3_step_stats * n)()
        nq = ad if hasattr(policies[0], "n_particles") else 1     # particle Q heads: one per action
        for k in range(n):
            arrs = [np.empty((B, nq), np.float32) for _ in range(3)]
            keep.append(arrs)
            st[k].y, st[k].q1, st[k].q2 = (a.ctypes.data for a in arrs)
    check(lib.td3_train_step_local(hs, rbs, n, B, _lib.i64ptr(ix) if ix is not None else None,
                                   _lib.fptr(nz) if nz is not None else None, st), "td3_train_step_local")
    if not stats:
        return None
    out = []
    for k in range(n):
        d = {"critic_loss": st[k].critic_loss, "actor_step": bool(st[k].actor_step),
             "y": keep[k][0], "q1": keep[k][1], "q2": keep[k][2]}
        if st[k].actor_step:
            d["actor_loss"] = st[k].actor_loss
        out.append(d)
    return out
