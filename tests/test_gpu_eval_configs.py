"""GPU parity for batched Eval at BASELINE configs[2] full size, the Eval
exactness rule for x >= 2^logN (SURVEY §8c rule 5), keys whose final CW
overlaps the last level record, and a denser logN=32 oracle comparison.

Reference: Eval dpf/dpf.go:171-211 (bit (x&127) of the final leaf, :207-209;
path bits logN-1-i, :194), EvalFull :243-262.
"""
import numpy as np
import pytest

import dpf
from dpf import synth
import oracle

pytestmark = pytest.mark.gpu
NT = 16


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dpf.gpu_init(1) >= 1
    prev = dpf.set_small_call_path("gpu")      # single-key calls here check the kernels
    yield
    dpf.set_small_call_path(prev)


def _keys(nk, logN, first=0):
    al, s0, s1 = synth.key_seeds(nk, logN, first=first)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    return al, ka, kb


@pytest.fixture(scope="module")
def cfg2():
    """configs[2]: 2^16 keys x 2^10 uniform points at logN=20, each key's
    alpha planted at a key-dependent position among its points, and the
    oracle's answer to every one of the 2^26 queries of both shares
    (the share-XOR property alone cannot see off-path errors)."""
    logN, nk, ppk = 20, 1 << 16, 1 << 10
    al, ka, kb = _keys(nk, logN, first=1 << 20)
    xs = synth.eval_points(nk, ppk, logN, master=0x5EEDD9F1)
    pos = (np.arange(nk) * 37) % ppk
    xs[np.arange(nk), pos] = al
    want_a = oracle.eval_batch(ka, xs, logN, nthreads=NT)
    want_b = oracle.eval_batch(kb, xs, logN, nthreads=NT)
    return logN, al, ka, kb, xs, pos, want_a, want_b


def _check_cfg2(got_a, got_b, cfg):
    logN, al, ka, kb, xs, pos, want_a, want_b = cfg
    nk = ka.shape[0]
    want_pf = (xs == al[:, None]).astype(np.uint8)
    assert np.array_equal(want_a ^ want_b, want_pf), "oracle shares are not the point function"
    # every query of both shares vs the oracle
    for got, want in ((got_a, want_a), (got_b, want_b)):
        bad = np.argwhere(got != want)
        assert bad.size == 0, f"{bad.shape[0]} answers differ, first at {tuple(bad[0])}"
    assert (got_a[np.arange(nk), pos] ^ got_b[np.arange(nk), pos] == 1).all()


def test_config2_host_path_full_size(cfg2):
    """dpf_eval_batch: 16 pipelined chunks of 4096 keys (two slots reused
    from the 3rd chunk on), every query of both shares vs the oracle."""
    logN, al, ka, kb, xs, pos = cfg2[:6]
    got_a = dpf.eval_batch(ka, xs, logN, ngpus=1)
    got_b = dpf.eval_batch(kb, xs, logN, ngpus=1)
    _check_cfg2(got_a, got_b, cfg2)


def test_config2_device_frontier_full_size(cfg2):
    """dpf_eval_batch_dev with the full workspace (shared HBM frontier, the
    persistent kernel bench.py times), every query of both shares vs the oracle."""
    import torch
    logN, al, ka, kb, xs, pos = cfg2[:6]
    nk, ppk = xs.shape
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    kl = dpf.key_len(logN)
    d_xs = torch.from_numpy(xs.reshape(-1).view(np.int64)).to(dev)
    d_work = torch.empty(dpf.eval_workspace_size(nk, ppk, logN), dtype=torch.uint8, device=dev)
    outs = []
    for k in (ka, kb):
        d_keys = torch.from_numpy(k.reshape(-1)).to(dev)
        d_out = torch.empty(nk * ppk, dtype=torch.uint8, device=dev)
        dpf.eval_batch_dev(d_keys, kl, nk, d_xs, ppk, logN, d_out, d_work, stream=st)
        torch.cuda.synchronize()
        outs.append(d_out.cpu().numpy().reshape(nk, ppk))
    _check_cfg2(outs[0], outs[1], cfg2)


@pytest.mark.parametrize("logN", [0, 3, 6, 8, 20, 32])
def test_eval_points_beyond_domain(logN):
    """Queries with x >= 2^logN: the reference walks bits logN-1..7 of x and
    reads bit x&127 of the final leaf (dpf.go:194,207-209), so high bits are
    ignored by the walk but bits 0..6 always select the leaf bit; logN < 7
    reads any of the 128 leaf bits.  Both the root-walk and the frontier
    kernels (>= 256 points per key) are exercised."""
    rng = np.random.default_rng(100 + logN)
    for ppk in (64, 600):
        nk = 6
        al, ka, kb = _keys(nk, logN, first=50000 + logN * 7 + ppk)
        raw = rng.integers(0, 2 ** 63, size=(nk, ppk), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
        xs = raw.copy()
        if logN < 7:
            xs[:, : ppk // 2] = np.uint64(1 << logN) + (raw[:, : ppk // 2] % np.uint64(128 - (1 << logN)))
        xs[:, 0] = np.uint64(0xFFFFFFFFFFFFFFFF)
        xs[:, 1] = np.uint64(1) << np.uint64(63)
        for k in (ka, kb):
            got = dpf.eval_batch(k, xs, logN, ngpus=1)
            want = oracle.eval_batch(k, xs, logN, nthreads=NT)
            assert np.array_equal(got, want), (logN, ppk)


@pytest.mark.parametrize("logN", [3, 9, 20])
def test_keys_with_overlapping_final_cw(logN):
    """Keys of 17+18*stop .. 33+18*stop-1 bytes: the final CW at len-16
    overlaps the last level record; the reference evaluates them without an
    index panic (dpf.go:206,219), and so must the engine."""
    stop = max(logN - 7, 0)
    rng = np.random.default_rng(logN + 900)
    for kl in sorted({17 + 18 * stop, 17 + 18 * stop + 5, 32 + 18 * stop}):
        keys = np.frombuffer(rng.bytes(4 * kl), np.uint8).reshape(4, kl).copy()
        got = dpf.evalfull_batch(keys, logN, ngpus=1)
        assert np.array_equal(got, oracle.evalfull_batch(keys, logN, nthreads=NT)), kl
        xs = synth.eval_points(4, 300, logN)
        assert np.array_equal(dpf.eval_batch(keys, xs, logN, ngpus=1),
                              oracle.eval_batch(keys, xs, logN, nthreads=NT)), kl
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.EvalFull(bytes(16 + 18 * stop), logN)
    assert e.value.code == dpf.DPF_ERR_KEYLEN


def test_logN32_dense_oracle_sample():
    """configs[3] shape (one key, logN=32, 512 MiB): 2048 points spread over
    the whole domain (every subtree the split path hands a GPU) compared with
    the oracle's Eval, plus the first and last leaf blocks bit for bit."""
    import torch
    logN = 32
    al, ka, _ = _keys(1, logN, first=321)
    key = ka[0].tobytes()
    dev = torch.device("cuda", 0)
    ol = dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1).copy()).to(dev)
    d_work = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=dev)
    d_out = torch.empty(ol, dtype=torch.uint8, device=dev)
    dpf.evalfull_batch_dev(d_keys, len(key), 1, logN, d_out, d_work, stream=torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    rng = np.random.default_rng(32)
    xs = np.concatenate([rng.integers(0, 1 << 32, size=2000, dtype=np.uint64),
                         np.arange(0, 1 << 32, 1 << 27, dtype=np.uint64), [int(al[0])]]).astype(np.uint64)
    idx = torch.from_numpy((xs >> np.uint64(3)).astype(np.int64)).to(dev)
    got_bytes = d_out[idx].cpu().numpy()
    got = (got_bytes >> (xs & np.uint64(7)).astype(np.uint8)) & 1
    want = oracle.eval_batch(ka, xs.reshape(1, -1), logN, nthreads=NT)[0]
    assert np.array_equal(got, want)
    head = d_out[:4096].cpu().numpy()
    tail = d_out[ol - 4096:].cpu().numpy()
    xs_h = np.arange(0, 4096 * 8, dtype=np.uint64)
    xs_t = np.arange((1 << 32) - 4096 * 8, 1 << 32, dtype=np.uint64)
    for blk, xx in ((head, xs_h), (tail, xs_t)):
        w = oracle.eval_batch(ka, xx.reshape(1, -1), logN, nthreads=NT)[0]
        assert np.array_equal(np.unpackbits(blk, bitorder="little"), w)


def _trie_built() -> bool:
    try:
        prev = dpf.set_eval_kernel("trie")
    except dpf.DPFPanic:
        return False
    dpf.set_eval_kernel(prev)
    return True


@pytest.fixture()
def trie_kernel():
    """The trie kernel is in the experimental build only (make -C dpf-go_amd
    experimental; DPF_LIB=dpf-go_amd/lib/variants/libdpf_hip_exp.so)."""
    if not _trie_built():
        with pytest.raises(dpf.DPFPanic):
            dpf.set_eval_kernel("trie")
        assert dpf.get_eval_kernel() == dpf.EVAL_WALK
        pytest.skip("k_eval_trie is in the experimental build only")
    prev = dpf.set_eval_kernel("trie")
    yield
    dpf.set_eval_kernel(prev)


def test_config2_trie_kernel_full_size(cfg2, trie_kernel):
    """configs[2] through the visited-node trie kernel (DPF_EVAL_TRIE):
    every query by the share property, 512 keys against the oracle."""
    logN, al, ka, kb, xs, pos = cfg2[:6]
    assert dpf.get_eval_kernel() == dpf.EVAL_TRIE
    got_a = dpf.eval_batch(ka, xs, logN, ngpus=1)
    got_b = dpf.eval_batch(kb, xs, logN, ngpus=1)
    _check_cfg2(got_a, got_b, cfg2)


@pytest.mark.parametrize("logN,nk,ppk", [(20, 4097, 1024), (16, 9, 1000), (20, 6, 64), (14, 5, 256),
                                         (12, 7, 64), (18, 3, 777)])
def test_trie_kernel_shapes(logN, nk, ppk, trie_kernel):
    """The trie kernel at ragged shapes: a last workgroup with fewer than 4
    keys, non-power-of-two points per key, the shallowest frontier (L = 4),
    duplicate points, x >= 2^logN and every key's alpha among its points;
    equal to the oracle and to the walk kernel."""
    rng = np.random.default_rng(logN * 1000 + ppk)
    al, ka, kb = _keys(nk, logN, first=70000 + nk + ppk)
    xs = synth.eval_points(nk, ppk, logN, master=0x7E1E + ppk)
    xs[:, 1] = al
    xs[:, 2] = xs[:, 3]                                          # duplicates
    xs[:, 4] = al | (np.uint64(1) << np.uint64(40))              # beyond the domain, same leaf bit
    xs[:, 5:9] = (al[:, None] ^ np.uint64(1)) & np.uint64((1 << logN) - 1)   # the alpha leaf block's neighbours
    xs[:, 9] = rng.integers(0, 2 ** 63, size=nk, dtype=np.uint64)
    for k in (ka, kb):
        got = dpf.eval_batch(k, xs, logN, ngpus=1)
        want = oracle.eval_batch(k, xs, logN, nthreads=NT)
        assert np.array_equal(got, want), (logN, nk, ppk)
    dpf.set_eval_kernel("walk")
    assert np.array_equal(dpf.eval_batch(ka, xs, logN, ngpus=1), oracle.eval_batch(ka, xs, logN, nthreads=NT))
