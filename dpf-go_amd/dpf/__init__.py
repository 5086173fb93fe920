"""dpf — Python mirror of dkales/dpf-go's package ``dpf`` over libdpf_hip.so.

Same names, argument meaning and error behaviour as the Go API
(/root/reference/dpf/dpf.go):

    Gen(alpha, logN)   -> (ka, kb)     dpf.go:71   (host; seeds from getrandom)
    Eval(k, x, logN)   -> 0 | 1        dpf.go:171  (gfx950 kernel)
    EvalFull(k, logN)  -> bytes        dpf.go:243  (gfx950 kernel)

Where Go panics, these raise ``DPFPanic`` ("dpf: invalid parameters" for Gen,
dpf.go:72-74).  Batched and device-resident forms are added for the engine.

There is no CPU evaluation path: the HIP library must be built
(``make -C dpf-go_amd``) and a gfx950 device must be visible, otherwise
evaluation raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPF_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libdpf_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "dpf_hip.h")

DPF_OK = 0
DPF_ERR_PARAM = -1
DPF_ERR_KEYLEN = -2
DPF_ERR_NODEV = -3
DPF_ERR_HIP = -4
DPF_ERR_NOMEM = -5
AES_TTABLE = 0
AES_BITSLICED = 1


class DPFPanic(RuntimeError):
    """Raised where the Go reference panics (or the device path fails)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg or f"dpf: error {code}")
        self.code = code


_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_sz = ctypes.c_size_t
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_int = ctypes.c_int
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must cover every function in include/dpf_hip.h
SIGNATURES = {
    "dpf_last_error": (ctypes.c_char_p, []),
    "dpf_key_len": (_sz, [_u32]),
    "dpf_evalfull_len": (_sz, [_u32]),
    "dpf_workspace_size": (_sz, [_sz, _u32]),
    "dpf_gpu_init": (_int, [_int]),
    "dpf_gpu_init_devices": (_int, [ctypes.POINTER(_int), _int]),
    "dpf_gpu_shutdown": (None, []),
    "dpf_gpu_count": (_int, []),
    "dpf_gen_seeded": (_int, [_u64, _u32, _u8p, _u8p, _u8p, _u8p]),
    "dpf_gen": (_int, [_u64, _u32, _u8p, _u8p]),
    "dpf_gen_batch_seeded": (_int, [_u64p, _u32, _u8p, _u8p, _sz, _u8p, _u8p, _int]),
    "dpf_keys_pack": (_int, [ctypes.POINTER(_vp), ctypes.POINTER(_sz), _sz, _sz, _u8p]),
    "dpf_keys_unpack": (_int, [_u8p, _sz, _sz, ctypes.POINTER(_vp)]),
    "dpf_eval": (_int, [_u8p, _sz, _u64, _u32, _u8p]),
    "dpf_evalfull": (_int, [_u8p, _sz, _u32, _u8p]),
    "dpf_evalfull_batch": (_int, [_u8p, _sz, _sz, _u32, _u8p, _int]),
    "dpf_eval_batch": (_int, [_u8p, _sz, _sz, _u64p, _sz, _u32, _u8p, _int]),
    "dpf_evalfull_split": (_int, [_u8p, _sz, _u32, _u8p, _int]),
    "dpf_evalfull_batch_dev": (_int, [_int, _vp, _sz, _sz, _u32, _vp, _vp, _vp]),
    "dpf_evalfull_subtree_dev": (_int, [_int, _vp, _sz, _sz, _u32, _u32, _u64, _vp, _vp, _vp]),
    "dpf_eval_workspace_size": (_sz, [_sz, _sz, _u32]),
    "dpf_eval_frontier_level": (_u32, [_u32, _sz]),
    "dpf_eval_batch_dev": (_int, [_int, _vp, _sz, _sz, _vp, _sz, _u32, _vp, _vp, _sz, _vp]),
    "dpf_expand_keys_dev": (_int, [_int, _vp, _sz, _sz, _u32, _vp, _vp]),
    "dpf_evalfull_expanded_dev": (_int, [_int, _vp, _sz, _u32, _u32, _u64, _vp, _vp]),
    "dpf_forget_workspace": (_int, [_vp]),
    "dpf_set_small_call_path": (_int, [_int]),
    "dpf_get_small_call_path": (_int, []),
    "dpf_small_call_max_logN": (ctypes.c_uint32, []),
    "dpf_set_aes_impl": (_int, [_int]),
    "dpf_get_aes_impl": (_int, []),
    "dpf_set_eval_kernel": (_int, [_int]),
    "dpf_get_eval_kernel": (_int, []),
    "dpf_set_pir_kernel": (_int, [_int]),
    "dpf_get_pir_kernel": (_int, []),
    "dpf_pir_kernel_for": (_int, [_sz, _u32, _u32]),
    "dpf_aes_mmo_dev": (_int, [_int, _int, _int, _vp, _vp, _sz, _u32, _vp]),
    "dpf_xor_fold_workspace_size": (_sz, []),
    "dpf_xor_fold_dev": (_int, [_int, _vp, _sz, _sz, _vp, _u64, _sz, _vp, _vp, _vp]),
    "dpf_pir_workspace_size": (_sz, [_sz, _u32, _u32]),
    "dpf_pir_answer_dev": (_int, [_int, _vp, _sz, _sz, _u32, _u32, _u64, _vp, _u64, _vp, _vp, _vp]),
    "dpf_pir_db_sliced_size": (_sz, [_u64]),
    "dpf_pir_db_slice_dev": (_int, [_int, _vp, _u64, _vp, _vp]),
    "dpf_pir_answer_sliced_dev": (_int, [_int, _vp, _sz, _sz, _u32, _u32, _u64, _vp, _u64, _vp, _vp, _vp]),
    "dpf_xor_fold_sliced_dev": (_int, [_int, _vp, _sz, _sz, _vp, _u64, _vp, _vp, _vp]),
    "dpf_set_fold_limits": (_int, [_u32, _u32]),
    "dpf_pir_db_create": (_int, [_u8p, _u64, _u32, _int, ctypes.POINTER(_vp)]),
    "dpf_pir_answer": (_int, [_vp, _u8p, _sz, _sz, _u8p]),
    "dpf_pir_db_free": (None, [_vp]),
    "dpf_stream_create_cu_masked": (_int, [_int, _u32, _u32, ctypes.POINTER(_vp)]),
    "dpf_stream_destroy": (_int, [_vp]),
}

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load libdpf_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: build it with `make -C dpf-go_amd` (no CPU fallback exists)")
        # One HIP runtime per process: torch ships its own libamdhip64.so
        # (DT_NEEDED "libamdhip64.so"), ours resolves "libamdhip64.so.7".
        # Loading torch first makes both bind to torch's copy, so device
        # pointers and streams handed over from torch are valid here.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != DPF_OK:
        msg = lib().dpf_last_error().decode(errors="replace")
        raise DPFPanic(rc, msg)


def _buf(a: np.ndarray):
    return a.ctypes.data_as(_u8p)


def _as_u8(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def key_len(logN: int) -> int:
    return int(lib().dpf_key_len(logN))


def evalfull_len(logN: int) -> int:
    return int(lib().dpf_evalfull_len(logN))


def workspace_size(nkeys: int, logN: int) -> int:
    return int(lib().dpf_workspace_size(nkeys, logN))


def gpu_init(ngpus: int = 0) -> int:
    rc = lib().dpf_gpu_init(ngpus)
    if rc < 0:
        _check(rc)
    return rc


def gpu_init_devices(ordinals: Sequence[int]) -> int:
    """Open exactly these HIP ordinals (one process per GPU: its own only)."""
    ids = (_int * len(ordinals))(*ordinals)
    rc = lib().dpf_gpu_init_devices(ids, len(ordinals))
    if rc < 0:
        _check(rc)
    return rc


def gpu_shutdown() -> None:
    lib().dpf_gpu_shutdown()


def gpu_count() -> int:
    """Devices the library has open (dpf_gpu_count)."""
    return int(lib().dpf_gpu_count())


# ------------------------------------------------------- key wire format ---
def keys_pack(keys: Sequence[bytes], key_len: Optional[int] = None) -> np.ndarray:
    """[DPFkey, ...] -> uint8[n, key_len], the batch layout of every batched
    entry point (dpf_keys_pack).  Keys are the reference's bytes (dpf.go:7);
    all must have the same length (DPFPanic DPF_ERR_KEYLEN otherwise)."""
    bufs = [_as_u8(k) for k in keys]
    n = len(bufs)
    kl = key_len if key_len is not None else (bufs[0].size if n else 0)
    out = np.empty((n, kl), np.uint8)
    if n == 0:
        return out
    ptrs = (_vp * n)(*[b.ctypes.data for b in bufs])
    lens = (_sz * n)(*[b.size for b in bufs])
    _check(lib().dpf_keys_pack(ptrs, lens, n, kl, _buf(out)))
    return out


def keys_unpack(packed: np.ndarray) -> list:
    """uint8[n, key_len] -> [DPFkey (bytes), ...] (dpf_keys_unpack)."""
    a = np.ascontiguousarray(packed, dtype=np.uint8)
    n, kl = a.shape
    outs = [np.empty(kl, np.uint8) for _ in range(n)]
    if n:
        ptrs = (_vp * n)(*[o.ctypes.data for o in outs])
        _check(lib().dpf_keys_unpack(_buf(a), kl, n, ptrs))
    return [o.tobytes() for o in outs]


# ------------------------------------------------------------------ Gen ---
def gen_seeded(alpha: int, logN: int, s0: bytes, s1: bytes) -> Tuple[bytes, bytes]:
    """Gen with the two crypto/rand seeds (dpf.go:80-81) supplied."""
    if logN > 63 or logN < 0 or alpha < 0 or alpha >= (1 << logN):
        raise DPFPanic(DPF_ERR_PARAM, "dpf: invalid parameters")
    n = key_len(logN)
    ka = np.zeros(n, np.uint8)
    kb = np.zeros(n, np.uint8)
    _check(lib().dpf_gen_seeded(alpha, logN, _buf(_as_u8(s0)), _buf(_as_u8(s1)), _buf(ka), _buf(kb)))
    return ka.tobytes(), kb.tobytes()


def Gen(alpha: int, logN: int) -> Tuple[bytes, bytes]:
    """dpf.go:71 — two key shares for the point function at alpha."""
    if logN > 63 or logN < 0 or alpha < 0 or alpha >= (1 << logN):
        raise DPFPanic(DPF_ERR_PARAM, "dpf: invalid parameters")
    n = key_len(logN)
    ka = np.zeros(n, np.uint8)
    kb = np.zeros(n, np.uint8)
    _check(lib().dpf_gen(alpha, logN, _buf(ka), _buf(kb)))
    return ka.tobytes(), kb.tobytes()


def gen_batch_seeded(alphas: Sequence[int], logN: int, s0s: np.ndarray, s1s: np.ndarray,
                     nthreads: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Batched seeded Gen on host threads -> (ka[n, klen], kb[n, klen])."""
    al = np.ascontiguousarray(alphas, dtype=np.uint64)
    n = al.shape[0]
    s0 = np.ascontiguousarray(s0s, dtype=np.uint8).reshape(n, 16)
    s1 = np.ascontiguousarray(s1s, dtype=np.uint8).reshape(n, 16)
    kl = key_len(logN)
    ka = np.zeros((n, kl), np.uint8)
    kb = np.zeros((n, kl), np.uint8)
    _check(lib().dpf_gen_batch_seeded(al.ctypes.data_as(_u64p), logN, _buf(s0), _buf(s1), n, _buf(ka), _buf(kb),
                                      nthreads))
    return ka, kb


# ----------------------------------------------------------- evaluation ---
def Eval(k: bytes, x: int, logN: int) -> int:
    """dpf.go:171 — the share of f_alpha(x), 0 or 1.  A latency-bound single
    call: the key bytes go to C without a numpy copy."""
    kb = k if isinstance(k, bytes) else _as_u8(k).tobytes()
    out = ctypes.c_uint8(0)
    rc = _eval_fn()(kb, len(kb), x & 0xFFFFFFFFFFFFFFFF, logN, ctypes.byref(out))
    if rc != DPF_OK:
        _check(rc)
    return out.value


_eval_proto = None


def _eval_fn():
    """dpf_eval with a bytes key argument (c_char_p: no copy)."""
    global _eval_proto
    if _eval_proto is None:
        f = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint32,
                             ctypes.POINTER(ctypes.c_uint8))
        _eval_proto = f(("dpf_eval", lib()))
    return _eval_proto


def EvalFull(key: bytes, logN: int, out: Optional[np.ndarray] = None) -> memoryview:
    """dpf.go:243 — the share of f_alpha over the whole domain, packed bits.

    Returns a writable bytes-like view of a fresh buffer (the Go function
    returns a fresh []byte, dpf.go:251): dpf_evalfull writes every byte of it
    once, with no zero fill before and no copy after.  `out` (uint8,
    evalfull_len(logN) bytes, C-contiguous) reuses a caller buffer instead."""
    if logN > 63:   # the reference panics allocating 2^(logN-3) bytes (dpf.go:251)
        raise DPFPanic(DPF_ERR_PARAM, "dpf: logN > 63")
    kk = _as_u8(key)
    n = evalfull_len(logN)
    if out is None:
        out = np.empty(n, np.uint8)
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size == n
    _check(lib().dpf_evalfull(_buf(kk), kk.size, logN, _buf(out)))
    return out.reshape(-1).data


def evalfull_batch(keys: np.ndarray, logN: int, ngpus: int = 0, out: Optional[np.ndarray] = None) -> np.ndarray:
    """keys[n, klen] uint8 -> out[n, evalfull_len(logN)] uint8 (written into `out` when given)."""
    kk = np.ascontiguousarray(keys, dtype=np.uint8)
    n, kl = kk.shape
    if out is None:
        out = np.empty((n, evalfull_len(logN)), np.uint8)
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.shape == (n, evalfull_len(logN))
    _check(lib().dpf_evalfull_batch(_buf(kk), kl, n, logN, _buf(out), ngpus))
    return out


def eval_batch(keys: np.ndarray, xs: np.ndarray, logN: int, ngpus: int = 0,
               out: Optional[np.ndarray] = None) -> np.ndarray:
    """keys[n, klen], xs[n, p] uint64 -> out[n, p] uint8 (0/1), written into `out` when given."""
    kk = np.ascontiguousarray(keys, dtype=np.uint8)
    x = np.ascontiguousarray(xs, dtype=np.uint64)
    n, kl = kk.shape
    p = x.shape[1]
    if out is None:
        out = np.empty((n, p), np.uint8)
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.shape == (n, p)
    _check(lib().dpf_eval_batch(_buf(kk), kl, n, x.ctypes.data_as(_u64p), p, logN, _buf(out), ngpus))
    return out


def evalfull_split(key: bytes, logN: int, ngpus: int, out: Optional[np.ndarray] = None) -> np.ndarray:
    """One EvalFull split by top-level subtree over ngpus devices -> uint8
    array of evalfull_len(logN) bytes (written into `out` when given)."""
    kk = _as_u8(key)
    if out is None:
        out = np.empty(evalfull_len(logN), np.uint8)
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size == evalfull_len(logN)
    _check(lib().dpf_evalfull_split(_buf(kk), kk.size, logN, _buf(out), ngpus))
    return out


# --------------------------------------------- device-resident (torch) ---
def _ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def _stream_handle(stream) -> int:
    return int(stream.cuda_stream) if stream is not None else 0


def evalfull_batch_dev(d_keys, key_len_: int, nkeys: int, logN: int, d_out, d_work, device: int = 0,
                       stream=None) -> None:
    """Enqueue EvalFull of nkeys HBM-resident keys on `stream` (torch stream)."""
    _check(lib().dpf_evalfull_batch_dev(device, _ptr(d_keys), key_len_, nkeys, logN, _ptr(d_out), _ptr(d_work),
                                        _stream_handle(stream)))


def evalfull_subtree_dev(d_keys, key_len_: int, nkeys: int, logN: int, prefix_bits: int, prefix: int, d_out,
                         d_work, device: int = 0, stream=None) -> None:
    _check(lib().dpf_evalfull_subtree_dev(device, _ptr(d_keys), key_len_, nkeys, logN, prefix_bits, prefix,
                                          _ptr(d_out), _ptr(d_work), _stream_handle(stream)))


def eval_workspace_size(nkeys: int, pts_per_key: int, logN: int) -> int:
    return int(lib().dpf_eval_workspace_size(nkeys, pts_per_key, logN))


def eval_frontier_level(logN: int, pts_per_key: int) -> int:
    """Depth of the shared frontier eval_batch_dev uses with a full workspace (0: root walks)."""
    return int(lib().dpf_eval_frontier_level(logN, pts_per_key))


def eval_batch_dev(d_keys, key_len_: int, nkeys: int, d_xs, pts_per_key: int, logN: int, d_out, d_work,
                   device: int = 0, stream=None) -> None:
    """Batched Eval on HBM tensors; d_work's size picks root walks or a shared frontier."""
    nbytes = int(d_work.numel() * d_work.element_size())
    _check(lib().dpf_eval_batch_dev(device, _ptr(d_keys), key_len_, nkeys, _ptr(d_xs), pts_per_key, logN,
                                    _ptr(d_out), _ptr(d_work), nbytes, _stream_handle(stream)))


def expand_keys_dev(d_keys, key_len_: int, nkeys: int, logN: int, d_work, device: int = 0, stream=None) -> None:
    _check(lib().dpf_expand_keys_dev(device, _ptr(d_keys), key_len_, nkeys, logN, _ptr(d_work),
                                     _stream_handle(stream)))


def evalfull_expanded_dev(d_work, nkeys: int, logN: int, d_out, prefix_bits: int = 0, prefix: int = 0,
                          device: int = 0, stream=None) -> None:
    _check(lib().dpf_evalfull_expanded_dev(device, _ptr(d_work), nkeys, logN, prefix_bits, prefix, _ptr(d_out),
                                           _stream_handle(stream)))


def forget_workspace(d_work) -> None:
    """Drop the library's record of what was expanded into d_work (call before freeing it)."""
    _check(lib().dpf_forget_workspace(_ptr(d_work)))


def set_aes_impl(impl) -> int:
    """Select the tree kernels' AES back end ("ttable"/"bitsliced" or 0/1); returns the previous one."""
    if isinstance(impl, str):
        impl = {"ttable": AES_TTABLE, "lds-ttable": AES_TTABLE, "bitsliced": AES_BITSLICED}[impl]
    rc = lib().dpf_set_aes_impl(impl)
    if rc < 0:
        _check(rc)
    return rc


def get_aes_impl() -> int:
    return int(lib().dpf_get_aes_impl())


EVAL_WALK, EVAL_TRIE = 0, 1


def set_eval_kernel(kernel) -> int:
    """Select the batched Eval kernel ("walk"/"trie" or 0/1); returns the previous one."""
    if isinstance(kernel, str):
        kernel = {"walk": EVAL_WALK, "trie": EVAL_TRIE}[kernel]
    rc = lib().dpf_set_eval_kernel(kernel)
    if rc < 0:
        _check(rc)
    return rc


def get_eval_kernel() -> int:
    return int(lib().dpf_get_eval_kernel())


PIR_SPLIT, PIR_FUSED, PIR_FUSED_ANY = 0, 1, 2


def set_pir_kernel(kernel) -> int:
    """Select the sliced PIR kernel ("split"/"fused"/"fused-any" or 0/1/2); returns the previous one."""
    if isinstance(kernel, str):
        kernel = {"split": PIR_SPLIT, "fused": PIR_FUSED, "fused-any": PIR_FUSED_ANY}[kernel]
    rc = lib().dpf_set_pir_kernel(kernel)
    if rc < 0:
        _check(rc)
    return rc


def get_pir_kernel() -> int:
    return int(lib().dpf_get_pir_kernel())


def pir_kernel_for(nkeys: int, logN: int, prefix_bits: int = 0) -> int:
    """PIR_FUSED or PIR_SPLIT: what pir_answer_sliced_dev runs for this shape now."""
    return int(lib().dpf_pir_kernel_for(nkeys, logN, prefix_bits))


SMALL_AUTO, SMALL_GPU, SMALL_HOST = 0, 1, 2


def set_small_call_path(mode) -> int:
    """Route of the single-key Eval/EvalFull ("auto"/"gpu"/"host" or 0/1/2,
    include/dpf_hip.h); returns the previous mode."""
    if isinstance(mode, str):
        mode = {"auto": SMALL_AUTO, "gpu": SMALL_GPU, "host": SMALL_HOST}[mode]
    rc = lib().dpf_set_small_call_path(mode)
    if rc < 0:
        _check(rc)
    return rc


def get_small_call_path() -> int:
    return int(lib().dpf_get_small_call_path())


def small_call_max_logN() -> int:
    return int(lib().dpf_small_call_max_logN())


def aes_mmo_dev(d_in, d_out, nblocks: int, impl: int = AES_TTABLE, right: bool = False, reps: int = 1,
                device: int = 0, stream=None) -> None:
    """aes128MMO iterated `reps` times over nblocks HBM blocks (both back ends)."""
    _check(lib().dpf_aes_mmo_dev(device, impl, 1 if right else 0, _ptr(d_in), _ptr(d_out), nblocks, reps,
                                 _stream_handle(stream)))


# ------------------------------------------------- CU-partitioned streams ---
def stream_create_cu_masked(cu_first: int, cu_count: int, device: int = 0):
    """A torch stream (ExternalStream) whose kernels run only on CUs
    [cu_first, cu_first + cu_count) of `device`; the _dev entry points size
    their grids to those CUs.  Release with stream_destroy()."""
    import torch
    h = _vp()
    _check(lib().dpf_stream_create_cu_masked(device, cu_first, cu_count, ctypes.byref(h)))
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", device))


def stream_destroy(stream) -> None:
    _check(lib().dpf_stream_destroy(_stream_handle(stream)))


# ------------------------------------------------------- streaming fold ---
def xor_fold_workspace_size() -> int:
    return int(lib().dpf_xor_fold_workspace_size())


def xor_fold_dev(d_bits, bits_stride: int, nkeys: int, d_payload, nrec: int, rec_bytes: int, d_ans, d_work,
                 device: int = 0, stream=None) -> None:
    """ans[k] = XOR of payload records i (rec_bytes each) whose bit i is set
    in EvalFull output k, on the device (dpf_xor_fold_dev)."""
    _check(lib().dpf_xor_fold_dev(device, _ptr(d_bits), bits_stride, nkeys, _ptr(d_payload), nrec, rec_bytes,
                                  _ptr(d_ans), _ptr(d_work), _stream_handle(stream)))


# ------------------------------------------------------------------ PIR ---
def pir_workspace_size(nkeys: int, logN: int, prefix_bits: int = 0) -> int:
    return int(lib().dpf_pir_workspace_size(nkeys, logN, prefix_bits))


def pir_answer_dev(d_keys, key_len_: int, nkeys: int, logN: int, d_db, nrec: int, d_ans, d_work,
                   prefix_bits: int = 0, prefix: int = 0, device: int = 0, stream=None) -> None:
    """Server answers (nkeys x 32 B) for the DB slice of subtree (prefix_bits, prefix)."""
    _check(lib().dpf_pir_answer_dev(device, _ptr(d_keys), key_len_, nkeys, logN, prefix_bits, prefix, _ptr(d_db),
                                    nrec, _ptr(d_ans), _ptr(d_work), _stream_handle(stream)))


def pir_db_sliced_size(nrec: int) -> int:
    return int(lib().dpf_pir_db_sliced_size(nrec))


def pir_db_slice_dev(d_db, nrec: int, d_dbs, device: int = 0, stream=None) -> None:
    """Bit-sliced copy of a row-major 32-B-record DB for the MFMA fold (built once per DB)."""
    _check(lib().dpf_pir_db_slice_dev(device, _ptr(d_db), nrec, _ptr(d_dbs), _stream_handle(stream)))


def pir_answer_sliced_dev(d_keys, key_len_: int, nkeys: int, logN: int, d_dbs, nrec: int, d_ans, d_work,
                          prefix_bits: int = 0, prefix: int = 0, device: int = 0, stream=None) -> None:
    """pir_answer_dev over the bit-sliced DB (the matrix-core fold)."""
    _check(lib().dpf_pir_answer_sliced_dev(device, _ptr(d_keys), key_len_, nkeys, logN, prefix_bits, prefix,
                                           _ptr(d_dbs), nrec, _ptr(d_ans), _ptr(d_work), _stream_handle(stream)))


def xor_fold_sliced_dev(d_bits, bits_stride: int, nkeys: int, d_dbs, nrec: int, d_ans, d_work, device: int = 0,
                        stream=None) -> None:
    """xor_fold_dev for 32-B records over the bit-sliced DB (the matrix-core fold)."""
    _check(lib().dpf_xor_fold_sliced_dev(device, _ptr(d_bits), bits_stride, nkeys, _ptr(d_dbs), nrec, _ptr(d_ans),
                                         _ptr(d_work), _stream_handle(stream)))


def set_fold_limits(max_blocks: int = 0, max_sg_per_block: int = 0) -> None:
    """Tuning / test limits of the fold launches (0 = default): workgroups per
    launch, and super-groups (256 records) per matrix-core fold workgroup;
    larger DBs fold in passes (dpf_set_fold_limits).  Answers do not depend
    on them."""
    _check(lib().dpf_set_fold_limits(max_blocks, max_sg_per_block))


class PirDB:
    """A 32-byte-record DB resident in HBM, sharded by top-level subtree over
    ngpus GPUs; answer() returns each key's XOR-inner-product (host XOR of
    the per-GPU partials)."""

    def __init__(self, db: np.ndarray, logN: int, ngpus: int = 1):
        d = np.ascontiguousarray(db, dtype=np.uint8).reshape(-1)
        if d.size % 32:
            raise ValueError("DB size must be a multiple of 32 bytes")
        self.logN = logN
        self.nrec = d.size // 32
        h = _vp()
        _check(lib().dpf_pir_db_create(_buf(d), self.nrec, logN, ngpus, ctypes.byref(h)))
        self._h = h

    def answer(self, keys: np.ndarray) -> np.ndarray:
        kk = np.ascontiguousarray(keys, dtype=np.uint8)
        n, kl = kk.shape
        ans = np.zeros((n, 32), np.uint8)
        _check(lib().dpf_pir_answer(self._h, _buf(kk), kl, n, _buf(ans)))
        return ans

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().dpf_pir_db_free(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
