"""GPU parity of the PIR answer fold (BASELINE configs[4]) against the CPU
oracle's XOR inner product over EvalFull bits, plus the 2-server property
answer(ka) ^ answer(kb) == DB[alpha] at full size (logN=24, 512 MiB DB)."""
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


@pytest.mark.parametrize("logN,nrec,nk", [(7, 128, 3), (10, 1000, 5), (12, 4096, 70), (16, 40000, 9), (12, 4000, 200), (13, 8192, 300)])
def test_pir_matches_oracle(logN, nrec, nk):
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    _, ka, _ = _keys(nk, logN, first=logN)
    pdb = dpf.PirDB(db, logN, ngpus=1)
    got = pdb.answer(ka)
    pdb.close()
    want = np.stack([np.frombuffer(oracle.pir_answer(ka[i].tobytes(), logN, db, 0, nrec), np.uint8)
                     for i in range(nk)])
    assert np.array_equal(got, want)


def test_pir_subtree_slices_xor_to_whole():
    import torch
    logN, nk = 14, 6
    nrec = 1 << logN
    dev = torch.device("cuda", 0)
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    _, ka, _ = _keys(nk, logN, first=5)
    kl = dpf.key_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    total = np.zeros((nk, 32), np.uint8)
    pb = 2
    slice_n = nrec >> pb
    for p in range(1 << pb):
        d_db = torch.from_numpy(db[p * slice_n:(p + 1) * slice_n].reshape(-1).copy()).to(dev)
        d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
        d_work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=dev)
        dpf.pir_answer_dev(d_keys, kl, nk, logN, d_db, slice_n, d_ans, d_work, prefix_bits=pb, prefix=p,
                           stream=torch.cuda.current_stream(dev))
        torch.cuda.synchronize()
        part = d_ans.cpu().numpy().reshape(nk, 32)
        want = np.stack([np.frombuffer(oracle.pir_answer(ka[i].tobytes(), logN, db[p * slice_n:], p * slice_n,
                                                         slice_n), np.uint8) for i in range(nk)])
        assert np.array_equal(part, want), p
        total ^= part
    whole = np.stack([np.frombuffer(oracle.pir_answer(ka[i].tobytes(), logN, db, 0, nrec), np.uint8)
                      for i in range(nk)])
    assert np.array_equal(total, whole)


def test_pir_two_server_recovers_record_full_size():
    """configs[4] shape on one GPU: logN=24, 2^24 x 32 B DB, 64 queries."""
    logN, nk = 24, 64
    nrec = 1 << logN
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    al, ka, kb = _keys(nk, logN, first=123)
    pdb = dpf.PirDB(db, logN, ngpus=1)
    a, b = pdb.answer(ka), pdb.answer(kb)
    pdb.close()
    rec = a ^ b
    for i in range(nk):
        assert np.array_equal(rec[i], db[int(al[i])]), i
