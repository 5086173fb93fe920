"""Multi-GPU partitioning of DPF evaluation, one process per GPU.

  keys      : batches of independent keys shard by key range, no collective
              (configs[1], configs[2]; weak scaling in bench.py).
  subtree   : one huge EvalFull splits by top-level subtree: rank r of a
              power-of-two world evaluates prefix r at depth log2(world)
              (configs[3]); its output is the slice at offset r * size/world.
  pir       : each rank holds the DB slice of its subtree and XOR-folds it to
              32 B per query; the partials are all-gathered (RCCL over xGMI,
              gloo on CPU) and XOR-combined on the host, because RCCL has no
              XOR reduction (configs[4]).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def key_range(nkeys: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of nkeys for this rank."""
    return nkeys * rank // world, nkeys * (rank + 1) // world


def subtree_split(world: int, rank: int) -> Tuple[int, int]:
    """(prefix_bits, prefix) of this rank's top-level subtree."""
    if world < 1 or world & (world - 1):
        raise ValueError("world size must be a power of two for a subtree split")
    return world.bit_length() - 1, rank


def db_slice(nrec_total: int, logN: int, world: int, rank: int) -> Tuple[int, int]:
    """Record range [lo, hi) of the DB that rank's subtree covers."""
    pb, p = subtree_split(world, rank)
    size = 1 << (logN - pb)
    lo = min(nrec_total, p * size)
    return lo, min(nrec_total, lo + size)


def xor_fold(parts: np.ndarray) -> np.ndarray:
    """XOR over axis 0 (the per-rank partial answers)."""
    parts = np.asarray(parts, dtype=np.uint8)
    return np.bitwise_xor.reduce(parts, axis=0)


def gather_xor(partial, group=None) -> np.ndarray:
    """All-gather every rank's uint8 partial answer tensor and XOR them.
    RCCL (nccl backend) has no XOR reduction: the partials are gathered into
    one [world, ...] device tensor, XOR-combined on the device (a pairwise
    tree of elementwise XORs over 64-bit words) and copied to the host once.  gloo
    (CPU rehearsals and tests) gathers host tensors and XORs with numpy."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        if partial.is_cuda:
            partial = partial.cpu()
        bufs = [torch.empty_like(partial) for _ in range(world)]
        dist.all_gather(bufs, partial, group=group)
        return xor_fold(np.stack([b.numpy() for b in bufs]))
    part = partial.contiguous()
    out = torch.empty((world,) + tuple(part.shape), dtype=part.dtype, device=part.device)
    dist.all_gather_into_tensor(out, part, group=group)
    return xor_rows(out).cpu().numpy()


def xor_rows(t):
    """XOR of t[0], t[1], ... (a uint8 torch tensor [world, ...]) on t's
    device, 8 bytes per lane when the row length allows, as a pairwise tree:
    ceil(log2(world)) elementwise launches (3 at 8 ranks) instead of
    world - 1."""
    world = t.shape[0]
    flat = t.reshape(world, -1)
    wide = flat.shape[1] % 8 == 0
    if wide:
        flat = flat.view(torch_int64())
    while flat.shape[0] > 1:
        n = flat.shape[0]
        h = n // 2
        top = flat[:h] ^ flat[h:2 * h]
        if n % 2:
            top[0].bitwise_xor_(flat[2 * h])
        flat = top
    acc = flat[0]
    if wide:
        acc = acc.view(t.dtype)
    return acc.view(t.shape[1:])


def torch_int64():
    import torch
    return torch.int64
