"""Multi-GPU plumbing: conversation sharding and the one collective.

Every conversation is independent (its context record, its window state, its utterances), so the
path shards by conversation with NO data-path collective: rank r owns the conversations with
``shard_of(conversation_id, world) == r`` and keeps their context in its own HBM.  The only
exchange is a sum of per-infoType finding counts (a few hundred bytes), done with one
``all_reduce`` -- RCCL over xGMI under the ``nccl`` backend, gloo in CPU tests.
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Sequence

import numpy as np


def shard_of(conversation_id, world: int) -> int:
    """Stable conversation -> rank map (hash64 of the id, mod world); ints map densely."""
    if isinstance(conversation_id, (int, np.integer)):
        return int(conversation_id) % world
    h = hashlib.blake2b(str(conversation_id).encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") % world


def shard_rows(conversation_ids: Sequence, rank: int, world: int) -> np.ndarray:
    """Indices of the rows this rank owns (order preserved, so conversation runs stay contiguous)."""
    return np.array([i for i, c in enumerate(conversation_ids) if shard_of(c, world) == rank], dtype=np.int64)


def reduce_histogram(hist: np.ndarray, group=None) -> np.ndarray:
    """Sum per-infoType counts over all ranks (int64; the last slot may carry the span total)."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return hist.astype(np.int64)
    # (world size 1 still issues the collective: the same RCCL code path as N ranks, tests/test_rccl_gpu.py)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.from_numpy(np.ascontiguousarray(hist, dtype=np.int64)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.cpu().numpy()
