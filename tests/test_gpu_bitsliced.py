"""GPU parity of the byte-sliced (table-free) AES back end against the CPU
oracle and the T-table back end, bit for bit (BASELINE configs[1]: bitsliced
vs LDS T-table).  Reference: aes128MMO dpf/aes_amd64.s:51-82, prg
dpf/dpf.go:59-69, EvalFull :213-262."""
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
    prev = dpf.set_aes_impl("bitsliced")
    yield
    dpf.set_aes_impl(prev)


def _keys(nk, logN, first=0):
    al, s0, s1 = synth.key_seeds(nk, logN, first=first)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    return al, ka, kb


@pytest.mark.parametrize("right", [False, True])
def test_mmo_blocks_vs_oracle_and_ttable(right):
    """aes128MMO on 8192 random blocks (1024 byte-sliced sets), 1 and 5
    iterations, byte-sliced == T-table == oracle (AES-NI restatement)."""
    import torch
    dev = torch.device("cuda", 0)
    n = 8192
    blocks = synth.db_bytes(n * 16, master=0xB10C + right).reshape(n, 16)
    d_in = torch.from_numpy(blocks.reshape(-1).copy()).to(dev)
    outs = {}
    for impl in (dpf.AES_TTABLE, dpf.AES_BITSLICED):
        for reps in (1, 5):
            d_out = torch.zeros_like(d_in)
            dpf.aes_mmo_dev(d_in, d_out, n, impl=impl, right=right, reps=reps)
            torch.cuda.synchronize()
            outs[(impl, reps)] = d_out.cpu().numpy().reshape(n, 16)
    assert np.array_equal(outs[(0, 1)], outs[(1, 1)])
    assert np.array_equal(outs[(0, 5)], outs[(1, 5)])
    for i in list(range(0, n, 257)) + [n - 1]:
        x = blocks[i].tobytes()
        assert outs[(1, 1)][i].tobytes() == oracle.mmo(right, x, aesni=True)
        for _ in range(5):
            x = oracle.mmo(right, x, aesni=True)
        assert outs[(1, 5)][i].tobytes() == x


@pytest.mark.parametrize("logN", [14, 15, 16, 18, 20])
def test_evalfull_bitsliced_vs_oracle(logN):
    nk = 12 if logN < 18 else 5
    al, ka, kb = _keys(nk, logN, first=logN * 31)
    keys = np.concatenate([ka, kb])
    got = dpf.evalfull_batch(keys, logN, ngpus=1)
    assert np.array_equal(got, oracle.evalfull_batch(keys, logN, nthreads=NT))
    x = np.unpackbits(got[:nk] ^ got[nk:], axis=1, bitorder="little")
    assert (x.sum(axis=1) == 1).all() and all(x[i, int(al[i])] for i in range(nk))


@pytest.mark.parametrize("logN", [14, 20])
def test_malformed_and_overlapping_keys_bitsliced(logN):
    """Exactness rules through the byte-sliced path: t bytes
    other than 0/1 (tested != 0), root LSB kept, final CW at len(k)-16,
    over-long and overlapping-final-CW keys."""
    rng = np.random.default_rng(logN + 4242)
    stop = logN - 7
    for kl in (dpf.key_len(logN), dpf.key_len(logN) + 9, 17 + 18 * stop):
        keys = np.frombuffer(rng.bytes(6 * kl), np.uint8).reshape(6, kl).copy()
        keys[0, 16] = 0
        keys[1, 16] = 0xFE
        keys[2, 17 + 16::18][:stop] = 1          # tLCW bytes == 1
        keys[3, 17 + 17::18][:stop] = 0          # tRCW bytes == 0
        got = dpf.evalfull_batch(keys, logN, ngpus=1)
        assert np.array_equal(got, oracle.evalfull_batch(keys, logN, nthreads=NT)), kl


def test_ttable_and_bitsliced_agree_full_config():
    """configs[1] at full size (4096 keys x logN=20) through the device path:
    the two back ends produce identical 512 MiB outputs, and 6 keys match
    the oracle."""
    import torch
    logN, nk = 20, 4096
    _, ka, _ = _keys(nk, logN, first=99)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
    dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work, stream=st)
    outs = []
    for impl in ("ttable", "bitsliced"):
        dpf.set_aes_impl(impl)
        d_out = torch.zeros(nk * ol, dtype=torch.uint8, device=dev)
        dpf.evalfull_expanded_dev(d_work, nk, logN, d_out, stream=st)
        torch.cuda.synchronize()
        outs.append(d_out)
    dpf.set_aes_impl("bitsliced")
    assert torch.equal(outs[0], outs[1])
    idx = np.array([0, 1, 777, 2048, 4094, 4095])
    got = outs[1].view(nk, ol)[torch.from_numpy(idx).to(dev)].cpu().numpy()
    assert np.array_equal(got, oracle.evalfull_batch(ka[idx], logN, nthreads=NT))


def test_subtree_slices_and_split_bitsliced():
    import torch
    logN, nk = 17, 6
    _, ka, _ = _keys(nk, logN, first=1717)
    host = oracle.evalfull_batch(ka, logN, nthreads=NT)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
    dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work, stream=st)
    for pb in (1, 2, 3):
        part = ol >> pb
        d_part = torch.zeros(nk * part, dtype=torch.uint8, device=dev)
        for p in range(1 << pb):
            dpf.evalfull_expanded_dev(d_work, nk, logN, d_part, prefix_bits=pb, prefix=p, stream=st)
            torch.cuda.synchronize()
            assert np.array_equal(d_part.cpu().numpy().reshape(nk, part), host[:, p * part:(p + 1) * part]), (pb, p)
    assert dpf.evalfull_split(ka[0].tobytes(), logN, 1).tobytes() == host[0].tobytes()


@pytest.mark.parametrize("logN,nrec,nk", [(14, 16384, 9), (16, 50000, 70)])
def test_pir_bitsliced_vs_oracle(logN, nrec, nk):
    """PIR answers with the byte-sliced tree producing the selection bits."""
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    _, ka, _ = _keys(nk, logN, first=logN + 5)
    pdb = dpf.PirDB(db, logN, ngpus=1)
    got = pdb.answer(ka)
    pdb.close()
    want = np.stack([np.frombuffer(oracle.pir_answer(ka[i].tobytes(), logN, db, 0, nrec), np.uint8)
                     for i in range(nk)])
    assert np.array_equal(got, want)
