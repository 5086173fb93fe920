"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle
and the committed golden vectors, bit-exact.  Run on the MI355X box with
`pytest -m gpu`."""
import hashlib
import json
import os

import numpy as np
import pytest

import dpf
from dpf import synth
import oracle

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NT = 16


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    n = dpf.gpu_init(1)
    assert n >= 1
    # The single-key dpf.Eval / dpf.EvalFull calls here are GPU parity checks:
    # pin them to the kernels (auto mode would route small ones to the host
    # path, which tests/test_gpu_small_calls.py covers).
    prev = dpf.set_small_call_path("gpu")
    yield
    dpf.set_small_call_path(prev)


def _bits(a: np.ndarray) -> np.ndarray:
    return np.unpackbits(np.asarray(a, np.uint8), axis=-1, bitorder="little")


def _keys(nk, logN, first=0):
    al, s0, s1 = synth.key_seeds(nk, logN, first=first)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    return al, ka, kb


@pytest.mark.parametrize("logN", list(range(0, 16)) + [17, 20])
def test_evalfull_batch_vs_oracle(logN):
    nk = 24 if logN <= 14 else 6
    al, ka, kb = _keys(nk, logN, first=logN * 100)
    keys = np.concatenate([ka, kb])
    got = dpf.evalfull_batch(keys, logN, ngpus=1)
    want = oracle.evalfull_batch(keys, logN, nthreads=NT)
    assert np.array_equal(got, want)
    x = _bits(got[:nk] ^ got[nk:])[:, : 1 << logN]
    assert (x.sum(axis=1) == 1).all()
    assert all(x[i, int(al[i])] == 1 for i in range(nk))


@pytest.mark.parametrize("logN", [0, 3, 6, 7, 8, 9, 13, 20, 32, 63])
def test_eval_batch_vs_oracle(logN):
    nk, ppk = 16, 96
    _, ka, _ = _keys(nk, logN, first=7000 + logN)
    xs = synth.eval_points(nk, ppk, logN)
    xs[:, 0] = 0
    xs[:, 1] = (1 << logN) - 1 if logN < 64 else 0xFFFFFFFFFFFFFFFF
    got = dpf.eval_batch(ka, xs, logN, ngpus=1)
    want = oracle.eval_batch(ka, xs, logN, nthreads=NT)
    assert np.array_equal(got, want)


def test_golden_vectors_on_gpu():
    cases = json.load(open(os.path.join(GOLD, "dpf_golden.json")))["cases"]
    for c in cases:
        logN = c["logN"]
        ka, kb = bytes.fromhex(c["ka"]), bytes.fromhex(c["kb"])
        fa, fb = dpf.EvalFull(ka, logN), dpf.EvalFull(kb, logN)
        if "full_a" in c:
            assert fa.hex() == c["full_a"] and fb.hex() == c["full_b"]
        else:
            assert hashlib.sha256(fa).hexdigest() == c["full_a_sha256"]
            assert hashlib.sha256(fb).hexdigest() == c["full_b_sha256"]
        for x, ea, eb in zip(c["eval_xs"], c["eval_a"], c["eval_b"]):
            assert dpf.Eval(ka, x, logN) == ea and dpf.Eval(kb, x, logN) == eb


# Restated reference tests (dpf_test.go:32-73) through the GPU path.
def test_reference_tests_on_gpu():
    ka, kb = dpf.Gen(123, 8)
    for i in range(256):
        assert (dpf.Eval(ka, i, 8) ^ dpf.Eval(kb, i, 8)) == (1 if i == 123 else 0)
    for logN, alpha in ((9, 128), (3, 1)):
        ka, kb = dpf.Gen(alpha, logN)
        a = _bits(np.frombuffer(dpf.EvalFull(ka, logN), np.uint8))
        b = _bits(np.frombuffer(dpf.EvalFull(kb, logN), np.uint8))
        x = (a ^ b)[: 1 << logN]
        assert x[alpha] == 1 and x.sum() == 1


def test_eval_consistent_with_evalfull():
    logN = 14
    _, ka, _ = _keys(4, logN, first=31)
    full = dpf.evalfull_batch(ka, logN, ngpus=1)
    xs = np.tile(np.arange(1 << logN, dtype=np.uint64), (4, 1))
    ev = dpf.eval_batch(ka, xs, logN, ngpus=1)
    assert np.array_equal(ev, _bits(full)[:, : 1 << logN])


@pytest.mark.parametrize("logN", [3, 9, 16, 20])
def test_malformed_keys_match_oracle(logN):
    """Arbitrary key bytes exercise the exactness rules: byte
    t-values tested != 0, root LSB not cleared, final CW at len(k)-16."""
    rng = np.random.default_rng(logN)
    kl = dpf.key_len(logN)
    keys = np.frombuffer(rng.bytes(8 * kl), np.uint8).reshape(8, kl).copy()
    keys[0, 16] = 0
    keys[1, 16] = 0xFE
    got = dpf.evalfull_batch(keys, logN, ngpus=1)
    want = oracle.evalfull_batch(keys, logN, nthreads=NT)
    assert np.array_equal(got, want)
    xs = synth.eval_points(8, 64, logN)
    assert np.array_equal(dpf.eval_batch(keys, xs, logN, ngpus=1), oracle.eval_batch(keys, xs, logN, nthreads=NT))


def test_long_keys_use_last_16_bytes():
    logN = 12
    kl = dpf.key_len(logN)
    rng = np.random.default_rng(5)
    keys = np.frombuffer(rng.bytes(4 * (kl + 21)), np.uint8).reshape(4, kl + 21).copy()
    got = dpf.evalfull_batch(keys, logN, ngpus=1)
    want = oracle.evalfull_batch(keys, logN, nthreads=4)
    assert np.array_equal(got, want)


def test_short_key_rejected():
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.EvalFull(bytes(40), 20)
    assert e.value.code == dpf.DPF_ERR_KEYLEN


def test_device_resident_paths_match_host_paths():
    import torch
    dev = torch.device("cuda", 0)
    logN, nk = 16, 40
    _, ka, _ = _keys(nk, logN, first=999)
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
    d_out = torch.zeros(nk * ol, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    dpf.evalfull_batch_dev(d_keys, kl, nk, logN, d_out, d_work, stream=st)
    torch.cuda.synchronize()
    host = dpf.evalfull_batch(ka, logN, ngpus=1)
    assert np.array_equal(d_out.cpu().numpy().reshape(nk, ol), host)
    # expanded two-phase form + subtree slices reassemble the full output
    dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work, stream=st)
    for pb in (1, 3, 9):
        part = ol >> pb
        d_part = torch.zeros(nk * part, dtype=torch.uint8, device=dev)
        for p in range(1 << pb):
            dpf.evalfull_expanded_dev(d_work, nk, logN, d_part, prefix_bits=pb, prefix=p, stream=st)
            torch.cuda.synchronize()
            got = d_part.cpu().numpy().reshape(nk, part)
            assert np.array_equal(got, host[:, p * part:(p + 1) * part]), (pb, p)
    xs = synth.eval_points(nk, 128, logN)
    d_xs = torch.from_numpy(xs.reshape(-1).view(np.int64)).to(dev)
    d_ev = torch.zeros(nk * 128, dtype=torch.uint8, device=dev)
    dpf.eval_batch_dev(d_keys, kl, nk, d_xs, 128, logN, d_ev, d_work, stream=st)
    torch.cuda.synchronize()
    assert np.array_equal(d_ev.cpu().numpy().reshape(nk, 128), oracle.eval_batch(ka, xs, logN, nthreads=NT))


def test_split_single_gpu_matches():
    logN = 18
    _, ka, _ = _keys(1, logN, first=4242)
    full = dpf.EvalFull(ka[0].tobytes(), logN)
    assert dpf.evalfull_split(ka[0].tobytes(), logN, 1).tobytes() == full
    assert full == oracle.evalfull(ka[0].tobytes(), logN, aesni=True)


def test_config2_full_size_point_function_property():
    """BASELINE configs[1] at full size (4096 keys x logN=20): all outputs
    bit-exact vs the oracle on a sample, and for 256 (ka, kb) pairs the XOR
    of shares is exactly the point function."""
    import torch
    logN, nk = 20, 4096
    al, ka, kb = _keys(nk, logN)
    got = dpf.evalfull_batch(ka, logN, ngpus=1)
    idx = np.array([0, 1, 1000, 2047, 4095])
    assert np.array_equal(got[idx], oracle.evalfull_batch(ka[idx], logN, nthreads=NT))
    gb = dpf.evalfull_batch(kb[:256], logN, ngpus=1)
    x = torch.from_numpy(got[:256] ^ gb)
    pop = torch.from_numpy(_bits(x.numpy())).sum(dim=1)
    assert (pop == 1).all()
    b = _bits(x.numpy())
    assert all(b[i, int(al[i])] == 1 for i in range(256))


def test_logN32_single_key_property():
    """BASELINE configs[3] shape on one GPU: EvalFull logN=32 (512 MiB per
    key) of both shares, XOR == point function, checked on the GPU."""
    import torch
    logN = 32
    alpha = 0xC0FFEE12
    _, s0, s1 = synth.key_seeds(1, 64, first=77)
    ka, kb = dpf.gen_seeded(alpha, logN, s0[0].tobytes(), s1[0].tobytes())
    dev = torch.device("cuda", 0)
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(np.frombuffer(ka + kb, np.uint8).copy()).to(dev)
    d_work = torch.empty(dpf.workspace_size(2, logN), dtype=torch.uint8, device=dev)
    d_out = torch.empty(2 * ol, dtype=torch.uint8, device=dev)
    dpf.evalfull_batch_dev(d_keys, kl, 2, logN, d_out, d_work, stream=torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    x = (d_out[:ol] ^ d_out[ol:]).view(torch.int64)
    nz = torch.nonzero(x).flatten()
    assert nz.numel() == 1
    word = int(nz[0])
    val = int(x[word].item()) & 0xFFFFFFFFFFFFFFFF
    assert val & (val - 1) == 0
    assert word * 64 + val.bit_length() - 1 == alpha
    # spot-check the first leaves against the oracle's Eval
    first = d_out[:64].cpu().numpy()
    for q in (0, 1, 200, 511):
        assert ((first[q >> 3] >> (q & 7)) & 1) == oracle.eval_(ka, q, logN, aesni=True)


@pytest.mark.parametrize("logN,nk,ppk", [(13, 8, 256), (14, 5, 1000), (20, 6, 1024), (20, 3, 3000), (32, 4, 512),
                                         (63, 2, 700), (15, 3, 257), (20, 600, 1024), (17, 2100, 128),
                                         (20, 8, 256), (21, 8, 256), (22, 8, 256)])
def test_eval_frontier_path_vs_oracle(logN, nk, ppk):
    """Shared-frontier Eval kernel (taken when a key has >= 256 points).
    (20, 600, 1024) gives the persistent kernel two ragged passes over its
    resident threads; (17, 2100, 128) one partial pass.  The persistent
    kernel stages a pair's key records in LDS when they fit 64 words
    (one 8-word record per level below the frontier level L, + 4 for
    the final CW): at
    ppk = 256, L = 7, so (20, 8, 256) stages 6*8+4 = 52 words and
    (21, 8, 256) 7*8+4 = 60, the largest LDS-staged walk; (22, 8, 256)
    needs 68, the first size past the limit, and takes the scalar-load
    walk, as does (32, 4, 512)."""
    if ppk == 256 and logN in (20, 21, 22):
        assert dpf.eval_frontier_level(logN, ppk) == 7
    _, ka, _ = _keys(nk, logN, first=8000 + logN + ppk)
    xs = synth.eval_points(nk, ppk, logN)
    xs[:, 0] = 0
    xs[:, 1] = (1 << logN) - 1
    xs[:, 2] = xs[:, 3]          # duplicate points
    got = dpf.eval_batch(ka, xs, logN, ngpus=1)
    want = oracle.eval_batch(ka, xs, logN, nthreads=NT)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("logN,nk,ppk", [(10, 5, 7), (20, 1, 1), (9, 3, 33)])
def test_eval_odd_query_counts(logN, nk, ppk):
    """k_eval2 takes queries in pairs: odd totals and pairs that straddle two
    keys (odd points per key) must match the oracle too."""
    _, ka, _ = _keys(nk, logN, first=8100 + logN + ppk)
    xs = synth.eval_points(nk, ppk, logN)
    assert np.array_equal(dpf.eval_batch(ka, xs, logN, ngpus=1), oracle.eval_batch(ka, xs, logN, nthreads=NT))


def test_empty_and_degenerate_inputs():
    """Empty batches are no-ops; invalid splits and undersized workspaces
    fail with an error code instead of touching memory."""
    import torch
    logN = 12
    kl = dpf.key_len(logN)
    none = np.zeros((0, kl), np.uint8)
    assert dpf.evalfull_batch(none, logN, ngpus=1).shape == (0, dpf.evalfull_len(logN))
    assert dpf.eval_batch(none, np.zeros((0, 5), np.uint64), logN, ngpus=1).shape == (0, 5)
    _, ka, kb = _keys(3, logN, first=31337)
    assert dpf.eval_batch(ka, np.zeros((3, 0), np.uint64), logN, ngpus=1).shape == (3, 0)
    _, k20, _ = _keys(1, 20, first=31338)
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.evalfull_split(k20[0].tobytes(), 20, 3)
    assert e.value.code == dpf.DPF_ERR_PARAM
    dev = torch.device("cuda", 0)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_xs = torch.zeros(3 * 4, dtype=torch.int64, device=dev)
    d_out = torch.zeros(3 * 4, dtype=torch.uint8, device=dev)
    tiny = torch.empty(8, dtype=torch.uint8, device=dev)
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.eval_batch_dev(d_keys, kl, 3, d_xs, 4, logN, d_out, tiny, stream=torch.cuda.current_stream(dev))
    assert e.value.code == dpf.DPF_ERR_PARAM
    # a workspace of exactly the key-expansion size takes the plain path
    from dpf import eval_workspace_size
    need = eval_workspace_size(3, 4, logN)
    d_work = torch.empty(need, dtype=torch.uint8, device=dev)
    dpf.eval_batch_dev(d_keys, kl, 3, d_xs, 4, logN, d_out, d_work, stream=torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    want = oracle.eval_batch(ka, np.zeros((3, 4), np.uint64), logN, nthreads=1)
    assert np.array_equal(d_out.cpu().numpy().reshape(3, 4), want)


@pytest.mark.parametrize("logN", [0, 1, 6, 7, 8])
def test_tiny_domains_all_points(logN):
    """Domains below and at the 2^7 leaf block (stop = 0 / 1): every point of
    Eval and EvalFull against the oracle, both shares."""
    al, ka, kb = _keys(9, logN, first=logN * 100)
    xs = np.tile(np.arange(1 << logN, dtype=np.uint64), (9, 1))
    for k in (ka, kb):
        assert np.array_equal(dpf.eval_batch(k, xs, logN, ngpus=1), oracle.eval_batch(k, xs, logN, nthreads=1))
        assert np.array_equal(dpf.evalfull_batch(k, logN, ngpus=1), oracle.evalfull_batch(k, logN, nthreads=1))
    got = dpf.eval_batch(ka, xs, logN, ngpus=1) ^ dpf.eval_batch(kb, xs, logN, ngpus=1)
    assert np.array_equal(got, (xs == al[:, None]).astype(np.uint8))


def test_eval_dev_points_at_8_byte_offset():
    """the persistent Eval kernel loads a pair's two points with
    one 16-byte LDS-DMA, so a d_xs that is only 8-byte aligned (a tensor
    slice xs[1:]) must take the per-pair kernel and give the same answers;
    a d_xs that is not 8-byte aligned is rejected."""
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    logN, nk, ppk = 20, 64, 1024              # persistent shape (frontier, wave-uniform keys)
    _, ka, _ = _keys(nk, logN, first=6060)
    xs = synth.eval_points(nk, ppk, logN, master=0xA11)
    kl = dpf.key_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_xs_big = torch.zeros(nk * ppk + 2, dtype=torch.int64, device=dev)
    d_xs_big[1:1 + nk * ppk] = torch.from_numpy(xs.reshape(-1).view(np.int64)).to(dev)
    d_xs = d_xs_big[1:1 + nk * ppk]
    assert d_xs.data_ptr() % 16 == 8
    d_work = torch.empty(dpf.eval_workspace_size(nk, ppk, logN), dtype=torch.uint8, device=dev)
    d_out = torch.empty(nk * ppk, dtype=torch.uint8, device=dev)
    dpf.eval_batch_dev(d_keys, kl, nk, d_xs, ppk, logN, d_out, d_work, stream=st)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().reshape(nk, ppk), oracle.eval_batch(ka, xs, logN, nthreads=NT))
    raw = torch.zeros(nk * ppk * 8 + 16, dtype=torch.uint8, device=dev)
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.lib()  # noqa: B018
        rc = dpf.lib().dpf_eval_batch_dev(0, d_keys.data_ptr(), kl, nk, raw.data_ptr() + 3, ppk, logN,
                                          d_out.data_ptr(), d_work.data_ptr(), d_work.numel(), st.cuda_stream)
        dpf._check(rc)
    assert e.value.code == dpf.DPF_ERR_PARAM
