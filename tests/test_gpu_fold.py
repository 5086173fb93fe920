"""GPU parity of the streaming XOR-fold consumer (dpf_xor_fold_dev):
the PIR fold generalised to payload records of any multiple of 32 bytes, over
EvalFull outputs that stay in HBM.  Checked against the XOR inner product of
the CPU oracle's EvalFull bits (oracle/dpf_oracle.c, dpf.go:243-262) with the
same payload, plus the 2-server property at logN=20."""
import numpy as np
import pytest

import dpf
from dpf import synth
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dpf.gpu_init(1) >= 1


def _keys(nk, logN, first=0):
    al, s0, s1 = synth.key_seeds(nk, logN, first=first)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    return al, ka, kb


def _want(full: np.ndarray, payload: np.ndarray, nrec: int) -> np.ndarray:
    """XOR of payload rows i < nrec with bit i (LSB-first) of each EvalFull row set."""
    bits = np.unpackbits(full, axis=1, bitorder="little")[:, :nrec].astype(bool)
    out = np.zeros((full.shape[0], payload.shape[1]), np.uint8)
    for k in range(full.shape[0]):
        sel = payload[bits[k]]
        if sel.shape[0]:
            out[k] = np.bitwise_xor.reduce(sel, axis=0)
    return out


def _fold(full_dev, stride, nk, payload, nrec, rec_bytes):
    import torch
    dev = full_dev.device
    d_pay = torch.from_numpy(np.ascontiguousarray(payload)).to(dev)
    d_ans = torch.full((nk * rec_bytes,), 0xAB, dtype=torch.uint8, device=dev)   # overwritten, not accumulated
    d_work = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
    dpf.xor_fold_dev(full_dev, stride, nk, d_pay, nrec, rec_bytes, d_ans, d_work)
    torch.cuda.synchronize()
    return d_ans.cpu().numpy().reshape(nk, rec_bytes)


# Every branch of the fold plan (pir_kernels.hip plan_fold): the direct kernel
# (<= 16 keys) at 1/2/4/8 columns, Four-Russians with 1/2/4 lane groups per
# table, several DB passes (> 256 keys, or C = 8 beyond 64 keys), widths that
# run column by column (96, 160 B), ragged record counts, nrec = 1 and nrec = 0
# (answers cleared by the first fold launch, or by a memset when there is none).
@pytest.mark.parametrize("logN,nk,rec_bytes,nrec", [
    (7, 3, 32, 128), (10, 5, 64, 1000), (12, 70, 96, 4096), (13, 9, 256, 5000), (14, 64, 32, 16384),
    (11, 16, 128, 2000), (11, 17, 128, 2000), (12, 130, 64, 4000), (12, 300, 32, 4096), (12, 100, 128, 3000),
    (11, 70, 256, 2048), (9, 20, 32, 1), (13, 40, 160, 8000), (10, 1, 32, 777), (10, 4, 64, 0),
])
def test_xor_fold_matches_oracle(logN, nk, rec_bytes, nrec):
    import torch
    _, ka, _ = _keys(nk, logN, first=100 + logN)
    full = oracle.evalfull_batch(ka, logN, nthreads=8)
    stride = dpf.evalfull_len(logN)
    payload = synth.db_bytes(nrec * rec_bytes).reshape(nrec, rec_bytes)
    kl = dpf.key_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).cuda()
    d_full = torch.empty(nk * stride, dtype=torch.uint8, device="cuda")
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
    dpf.evalfull_batch_dev(d_keys, kl, nk, logN, d_full, d_work)    # the output never leaves HBM
    torch.cuda.synchronize()
    got = _fold(d_full, stride, nk, payload, nrec, rec_bytes)
    assert np.array_equal(got, _want(full, payload, nrec))


@pytest.mark.parametrize("nk,nrec", [(64, 1 << 19), (40, (1 << 19) - 1000), (64, (1 << 19) + 4321)])
def test_xor_fold_full_grid_vs_numpy(nk, nrec):
    """A grid of 2 workgroups per CU, where launch_4r splits a CU's chunks
    unevenly between them (DPF_FOLD_SKEW): every record must be folded once.
    Random selection bits, checked against a numpy fold of all keys."""
    import torch
    rng = np.random.default_rng(nk + nrec)
    stride = ((nrec + 127) // 128) * 16
    bits = rng.integers(0, 256, size=(nk, stride), dtype=np.uint8)
    payload = rng.integers(0, 256, size=(nrec, 32), dtype=np.uint8)
    got = _fold(torch.from_numpy(bits.reshape(-1)).cuda(), stride, nk, payload, nrec, 32)
    assert np.array_equal(got, _want(bits, payload, nrec))


def test_xor_fold_two_server_property_logN20():
    """answer(ka) ^ answer(kb) == payload[alpha] for 128-byte records at logN=20."""
    import torch
    logN, nk, rec = 20, 16, 128
    nrec = 1 << logN
    al, ka, kb = _keys(nk, logN, first=7)
    payload = synth.db_bytes(nrec * rec).reshape(nrec, rec)
    stride, kl = dpf.evalfull_len(logN), dpf.key_len(logN)
    outs = []
    for keys in (ka, kb):
        d_keys = torch.from_numpy(keys.reshape(-1)).cuda()
        d_full = torch.empty(nk * stride, dtype=torch.uint8, device="cuda")
        d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
        dpf.evalfull_batch_dev(d_keys, kl, nk, logN, d_full, d_work)
        outs.append(_fold(d_full, stride, nk, payload, nrec, rec))
    x = outs[0] ^ outs[1]
    for k in range(nk):
        assert np.array_equal(x[k], payload[int(al[k])])


def test_xor_fold_equals_pir_answer_for_32_byte_records():
    import torch
    logN, nk = 12, 20
    nrec = 1 << logN
    _, ka, _ = _keys(nk, logN, first=3)
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    pdb = dpf.PirDB(db, logN, ngpus=1)
    want = pdb.answer(ka)
    pdb.close()
    stride, kl = dpf.evalfull_len(logN), dpf.key_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).cuda()
    d_full = torch.empty(nk * stride, dtype=torch.uint8, device="cuda")
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
    dpf.evalfull_batch_dev(d_keys, kl, nk, logN, d_full, d_work)
    assert np.array_equal(_fold(d_full, stride, nk, db, nrec, 32), want)


def test_xor_fold_rejects_bad_shapes():
    import torch
    d = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    w = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device="cuda")
    for stride, nrec, rec in ((16, 128, 48), (24, 8, 32), (16, 129, 32)):
        with pytest.raises(dpf.DPFPanic) as e:
            dpf.xor_fold_dev(d, stride, 1, d, nrec, rec, d, w)
        assert e.value.code == dpf.DPF_ERR_PARAM
    dpf.xor_fold_dev(d, 16, 0, d, 128, 32, d, w)   # no keys: nothing to do


# ---- the matrix-core fold over the bit-sliced DB (dpf_xor_fold_sliced_dev,
# dpf_pir_answer_sliced_dev): every key tile count (1/2/4/8 x 32 keys), more
# than one 256-key pass, ragged record counts (the sliced layout pads the last
# 256-record super-group with zero bits), selection strides that are not a
# multiple of 8 words, and nrec = 0.
@pytest.mark.parametrize("logN,nk,nrec", [
    (7, 1, 128), (9, 3, 300), (12, 33, 4096), (12, 64, 4000), (13, 65, 8192), (13, 128, 8000),
    (12, 129, 4096), (12, 256, 4096), (12, 300, 3001), (8, 5, 1), (10, 7, 0), (16, 64, 65536 - 77),
])
def test_sliced_mfma_fold_matches_oracle(logN, nk, nrec):
    import torch
    dev = torch.device("cuda", 0)
    _, ka, _ = _keys(nk, logN, first=700 + nk)
    full = dpf.evalfull_batch(ka, logN, ngpus=1)
    stride = full.shape[1]
    payload = synth.db_bytes(max(nrec, 1) * 32).reshape(-1, 32)[:nrec]
    d_full = torch.from_numpy(full.reshape(-1)).to(dev)
    d_db = torch.from_numpy(np.ascontiguousarray(payload).reshape(-1)).to(dev) if nrec else \
        torch.zeros(16, dtype=torch.uint8, device=dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs)
    d_ans = torch.full((nk * 32,), 0xAB, dtype=torch.uint8, device=dev)
    d_work = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
    dpf.xor_fold_sliced_dev(d_full, stride, nk, d_dbs, nrec, d_ans, d_work)
    torch.cuda.synchronize()
    got = d_ans.cpu().numpy().reshape(nk, 32)
    assert np.array_equal(got, _want(full, payload.reshape(-1, 32), nrec))
    if nrec:
        assert np.array_equal(got, _fold(d_full, stride, nk, payload, nrec, 32))


def test_sliced_pir_answer_two_server_full_size():
    """configs[4] through the MFMA fold: logN=24, 2^24 x 32 B, B=64 and 256:
    answers equal the LDS fold's and the two servers XOR to DB[alpha]."""
    import torch
    dev = torch.device("cuda", 0)
    logN = 24
    nrec = 1 << logN
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    d_db = torch.from_numpy(db.reshape(-1)).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs)
    kl = dpf.key_len(logN)
    for nk in (64, 256):
        al, ka, kb = _keys(nk, logN, first=9000 + nk)
        d_work = torch.empty(dpf.pir_workspace_size(nk, logN), dtype=torch.uint8, device=dev)
        res = []
        for keys, sliced in ((ka, True), (kb, True), (ka, False)):
            d_keys = torch.from_numpy(keys.reshape(-1)).to(dev)
            d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
            f = dpf.pir_answer_sliced_dev if sliced else dpf.pir_answer_dev
            f(d_keys, kl, nk, logN, d_dbs if sliced else d_db, nrec, d_ans, d_work)
            torch.cuda.synchronize()
            res.append(d_ans.cpu().numpy().reshape(nk, 32))
        assert np.array_equal(res[0], res[2])
        rec = res[0] ^ res[1]
        for i in range(nk):
            assert np.array_equal(rec[i], db[int(al[i])]), (nk, i)


@pytest.fixture
def fold_limits():
    yield dpf.set_fold_limits
    dpf.set_fold_limits(0, 0)


# the MFMA fold's answer bits are parities of fp32 counts, exact
# only while a count stays <= 2^24.  No workgroup folds more than 2^15 super-
# groups (2^23 records); a DB with more than 1024 x 2^15 super-groups folds in
# passes.  Forced small limits (1-7 workgroups of 1-5 super-groups: many
# passes, ragged last passes, several key groups) must all give the answers of
# the default shape and of the LDS fold over the row-major DB.
@pytest.mark.parametrize("max_blocks,max_sg,nk,nrec", [
    (1, 1, 64, 8192), (3, 5, 33, 30000 - 7), (2, 3, 129, 20000), (1, 0, 256, 65536), (7, 2, 1, 9999),
    (5, 4, 300, 12345),
])
def test_sliced_fold_forced_passes(fold_limits, max_blocks, max_sg, nk, nrec):
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(nk * 7 + nrec)
    stride = ((nrec + 7) // 8 + 15) // 16 * 16
    bits = rng.integers(0, 256, (nk, stride), dtype=np.uint8)
    payload = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    d_bits = torch.from_numpy(bits.reshape(-1)).to(dev)
    d_db = torch.from_numpy(payload.reshape(-1)).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs)
    d_work = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)

    def run():
        d_ans = torch.full((nk * 32,), 0xAB, dtype=torch.uint8, device=dev)
        dpf.xor_fold_sliced_dev(d_bits, stride, nk, d_dbs, nrec, d_ans, d_work)
        torch.cuda.synchronize()
        return d_ans.cpu().numpy().reshape(nk, 32)

    base = run()
    fold_limits(max_blocks, max_sg)
    assert np.array_equal(run(), base)
    fold_limits(0, 0)
    assert np.array_equal(base, _fold(d_bits, stride, nk, payload, nrec, 32))
    if nk <= 64:
        assert np.array_equal(base, _want(bits, payload, nrec))


def test_sliced_fold_counts_past_2p24_in_one_workgroup(fold_limits):
    """2^24 + 2^21 records of an all-ones DB under selection words that are
    mostly ones, with one workgroup per launch: a single run would count past
    2^24 (fp32's last exact integer, where a plain fp32 accumulation rounds
    odd partial sums); the launcher splits it into passes of 2^15 super-groups
    and the answer bit must be the parity of the number of selected records."""
    import torch
    dev = torch.device("cuda", 0)
    nk, nrec = 32, (1 << 24) + (1 << 21)
    stride = nrec // 8
    rng = np.random.default_rng(5)
    bits = np.full((nk, stride), 0xFF, np.uint8)
    holes = rng.random((nk, stride)) < 0.125
    bits[holes] = rng.integers(0, 256, int(holes.sum()), dtype=np.uint8)
    d_bits = torch.from_numpy(bits.reshape(-1)).to(dev)
    d_dbs = torch.full((dpf.pir_db_sliced_size(nrec),), 0xFF, dtype=torch.uint8, device=dev)
    d_work = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
    fold_limits(1, 0)
    dpf.xor_fold_sliced_dev(d_bits, stride, nk, d_dbs, nrec, d_ans, d_work)
    torch.cuda.synchronize()
    got = d_ans.cpu().numpy().reshape(nk, 32)
    par = np.unpackbits(bits, axis=1).sum(axis=1) & 1
    want = np.where(par[:, None] == 1, 0xFF, 0).astype(np.uint8) * np.ones((1, 32), np.uint8)
    assert np.array_equal(got, want)


def test_pir_answer_rejects_bad_buffers():
    """null or misaligned device buffers are DPF_ERR_PARAM at the
    C ABI of both PIR answer entry points, not a GPU fault."""
    import torch
    logN, nk = 12, 2
    _, ka, _ = _keys(nk, logN, first=5)
    kl = dpf.key_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to("cuda")
    d = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    w = torch.empty(dpf.pir_workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
    for f in (dpf.pir_answer_dev, dpf.pir_answer_sliced_dev):
        for db, ans, work in ((None, d, w), (d, None, w), (d, d, None), (d[1:], d, w), (d, d[2:], w),
                              (d, d, w[4:])):
            with pytest.raises(dpf.DPFPanic) as e:
                f(d_keys, kl, nk, logN, db, 100, ans, work)
            assert e.value.code == dpf.DPF_ERR_PARAM
