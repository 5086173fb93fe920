"""ctypes loader for liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of dkales/dpf-go's evaluation path (oracle/dpf_oracle.c).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product (dpf-go_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_init.restype = None
        L.oracle_have_aesni.restype = ctypes.c_int
        L.oracle_key_len.restype = ctypes.c_size_t
        L.oracle_key_len.argtypes = [ctypes.c_uint64]
        L.oracle_out_len.restype = ctypes.c_size_t
        L.oracle_out_len.argtypes = [ctypes.c_uint64]
        L.oracle_expand_key.argtypes = [_u8p, _u8p]
        L.oracle_aes128_encrypt.argtypes = [_u8p, _u8p, _u8p]
        L.oracle_mmo.argtypes = [ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        L.oracle_gen.restype = ctypes.c_int
        L.oracle_gen.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _u8p, _u8p, _u8p, _u8p]
        L.oracle_eval.restype = ctypes.c_int
        L.oracle_eval.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
        L.oracle_evalfull.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint64, _u8p, ctypes.c_int]
        L.oracle_evalfull_batch.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64, _u8p,
                                            ctypes.c_int, ctypes.c_int]
        L.oracle_eval_batch.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_size_t, _u64p, ctypes.c_size_t,
                                        ctypes.c_uint64, _u8p, ctypes.c_int, ctypes.c_int]
        L.oracle_pir_answer.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint64, _u8p, ctypes.c_uint64,
                                        ctypes.c_uint64, _u8p]
        L.oracle_evalfull_mt.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_uint64, _u8p, ctypes.c_int, ctypes.c_int]
        L.oracle_pir_answer_batch.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64, _u8p,
                                              ctypes.c_uint64, ctypes.c_int, _u8p, ctypes.c_int]
        L.oracle_init()
        _lib = L
    return _lib


def _u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


def _p(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def key_len(logN: int) -> int:
    return int(lib().oracle_key_len(logN))


def out_len(logN: int) -> int:
    return int(lib().oracle_out_len(logN))


def have_aesni() -> bool:
    return bool(lib().oracle_have_aesni())


def aes128_encrypt(key: bytes, block: bytes) -> bytes:
    rk = np.zeros(176, np.uint8)
    lib().oracle_expand_key(_p(_u8(key)), _p(rk))
    out = np.zeros(16, np.uint8)
    lib().oracle_aes128_encrypt(_p(rk), _p(out), _p(_u8(block)))
    return out.tobytes()


def mmo(right: bool, block: bytes, aesni: bool = False) -> bytes:
    out = np.zeros(16, np.uint8)
    lib().oracle_mmo(int(right), int(aesni), _p(out), _p(_u8(block)))
    return out.tobytes()


def gen(alpha: int, logN: int, s0: bytes, s1: bytes):
    n = key_len(logN)
    ka = np.zeros(n, np.uint8)
    kb = np.zeros(n, np.uint8)
    rc = lib().oracle_gen(alpha, logN, _p(_u8(s0)), _p(_u8(s1)), _p(ka), _p(kb))
    if rc != 0:
        raise ValueError("dpf: invalid parameters")
    return ka.tobytes(), kb.tobytes()


def eval_(key: bytes, x: int, logN: int, aesni: bool = False) -> int:
    k = _u8(key)
    return int(lib().oracle_eval(_p(k), k.size, x, logN, int(aesni)))


def evalfull(key: bytes, logN: int, aesni: bool = False) -> bytes:
    k = _u8(key)
    out = np.zeros(out_len(logN), np.uint8)
    lib().oracle_evalfull(_p(k), k.size, logN, _p(out), int(aesni))
    return out.tobytes()


def evalfull_mt(key: bytes, logN: int, nthreads: int = 16, aesni: bool = True) -> np.ndarray:
    """EvalFull of one key split over depth-d subtrees on nthreads threads
    (the DFS output is their concatenation in prefix order) -> uint8 array."""
    k = _u8(key)
    out = np.empty(out_len(logN), np.uint8)
    lib().oracle_evalfull_mt(_p(k), k.size, logN, _p(out), nthreads, int(aesni))
    return out


def evalfull_batch(keys: np.ndarray, logN: int, nthreads: int = 1, aesni: bool = True) -> np.ndarray:
    kk = np.ascontiguousarray(keys, dtype=np.uint8)
    n, kl = kk.shape
    out = np.zeros((n, out_len(logN)), np.uint8)
    lib().oracle_evalfull_batch(_p(kk), kl, n, logN, _p(out), nthreads, int(aesni))
    return out


def eval_batch(keys: np.ndarray, xs: np.ndarray, logN: int, nthreads: int = 1, aesni: bool = True) -> np.ndarray:
    kk = np.ascontiguousarray(keys, dtype=np.uint8)
    x = np.ascontiguousarray(xs, dtype=np.uint64)
    n, kl = kk.shape
    p = x.shape[1]
    out = np.zeros((n, p), np.uint8)
    lib().oracle_eval_batch(_p(kk), kl, n, x.ctypes.data_as(_u64p), p, logN, _p(out), nthreads, int(aesni))
    return out


def pir_answer(key: bytes, logN: int, db: np.ndarray, rec_lo: int, nrec: int) -> bytes:
    k = _u8(key)
    d = np.ascontiguousarray(db, dtype=np.uint8)
    ans = np.zeros(32, np.uint8)
    lib().oracle_pir_answer(_p(k), k.size, logN, _p(d), rec_lo, nrec, _p(ans))
    return ans.tobytes()


def pir_answer_batch(keys: np.ndarray, logN: int, db: np.ndarray, nrec: int, nslices: int = 1,
                     nthreads: int = 16) -> np.ndarray:
    """Every key's XOR inner product over the DB, split into nslices equal
    record slices of the domain -> uint8[nkeys, nslices, 32]; the slice
    partials are what an N = nslices PIR rank returns, their XOR the answer."""
    kk = np.ascontiguousarray(keys, dtype=np.uint8)
    n, kl = kk.shape
    d = np.ascontiguousarray(db, dtype=np.uint8).reshape(-1)
    assert d.size >= nrec * 32
    ans = np.zeros((n, nslices, 32), np.uint8)
    lib().oracle_pir_answer_batch(_p(kk), kl, n, logN, _p(d), nrec, nslices, _p(ans), nthreads)
    return ans
