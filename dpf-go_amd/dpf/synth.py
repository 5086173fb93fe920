"""Synthetic workloads for tests and bench (SURVEY §8d / BASELINE.md "Inputs").

SplitMix64 with master seed 0x5EED_D9F0.  Stream j starts at state
master + j * 0x9E3779B97F4A7C15 (mod 2^64) and yields splitmix64 outputs.
Key k: s0 = first two draws of stream 2k (little-endian), s1 = first two
draws of stream 2k+1, alpha = third draw of stream 2k mod 2^logN.
"""
from __future__ import annotations

import numpy as np

MASTER_SEED = 0x5EEDD9F0
_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def splitmix_streams(streams: np.ndarray, ndraws: int, master: int = MASTER_SEED) -> np.ndarray:
    """Draws [len(streams), ndraws] uint64 from the given stream ids."""
    with np.errstate(over="ignore"):
        st = np.uint64(master) + np.asarray(streams, dtype=np.uint64) * _GAMMA
        out = np.empty((st.shape[0], ndraws), dtype=np.uint64)
        for d in range(ndraws):
            st = st + _GAMMA
            out[:, d] = _mix(st.copy())
    return out


def key_seeds(nkeys: int, logN: int, first: int = 0, master: int = MASTER_SEED):
    """(alphas[n] uint64, s0[n,16] uint8, s1[n,16] uint8) for keys first..first+n-1."""
    k = np.arange(first, first + nkeys, dtype=np.uint64)
    a = splitmix_streams(2 * k, 3, master)
    b = splitmix_streams(2 * k + np.uint64(1), 2, master)
    s0 = np.ascontiguousarray(a[:, :2]).view(np.uint8).reshape(nkeys, 16)
    s1 = np.ascontiguousarray(b[:, :2]).view(np.uint8).reshape(nkeys, 16)
    mask = np.uint64((1 << logN) - 1) if logN < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    alphas = a[:, 2] & mask
    return alphas, s0.copy(), s1.copy()


def eval_points(nkeys: int, pts_per_key: int, logN: int, master: int = MASTER_SEED + 1) -> np.ndarray:
    """Uniform points in [0, 2^logN), shape [nkeys, pts_per_key] uint64."""
    raw = splitmix_streams(np.arange(nkeys, dtype=np.uint64), pts_per_key, master)
    mask = np.uint64((1 << logN) - 1) if logN < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    return raw & mask


def db_bytes(nbytes: int, master: int = MASTER_SEED + 2) -> np.ndarray:
    """Uniform random DB bytes."""
    nw = (nbytes + 7) // 8
    rows = (nw + 1023) // 1024
    raw = splitmix_streams(np.arange(rows, dtype=np.uint64), 1024, master).reshape(-1)[:nw]
    return raw.view(np.uint8)[:nbytes].copy()
