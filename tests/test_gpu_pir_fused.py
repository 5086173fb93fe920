"""GPU parity of the sliced PIR answer over subtree slices (the two-launch
product path: tree kernel, then the matrix-core fold) and of the fused PIR
kernel (k_pir_fused: subtree EvalFull and the matrix-core fold in one launch,
DESIGN.md §4.4) against the CPU oracle's XOR inner product over EvalFull bits
(dpf/dpf.go:213-262 for the bits), and the 2-server property at the configs[4]
shape (logN=24, 2^24 x 32 B DB).  The fused kernel is in the experimental
build only (make -C dpf-go_amd experimental; run these tests with
DPF_LIB=dpf-go_amd/lib/variants/libdpf_hip_exp.so): with the product library
its legs are skipped."""
import numpy as np
import pytest

import dpf
from dpf import synth
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dpf.gpu_init(1) >= 1


def _fused_built() -> bool:
    try:
        prev = dpf.set_pir_kernel("fused-any")
    except dpf.DPFPanic:
        return False
    dpf.set_pir_kernel(prev)
    return True


@pytest.fixture
def pir_kernel():
    prev = dpf.get_pir_kernel()
    yield dpf.set_pir_kernel
    dpf.set_pir_kernel(prev)


needs_fused = pytest.mark.skipif("not _fused_built()", reason="k_pir_fused is in the experimental build only")


def _keys(nk, logN, first=0):
    al, s0, s1 = synth.key_seeds(nk, logN, first=first)
    return (al,) + tuple(dpf.gen_batch_seeded(al, logN, s0, s1))


def _answer(ka, logN, db_slice, nrec, pb=0, prefix=0):
    """dpf_pir_answer_sliced_dev over one slice, answers on the host."""
    import torch
    dev = torch.device("cuda", 0)
    nk = ka.shape[0]
    d_keys = torch.from_numpy(ka.reshape(-1).copy()).to(dev)
    d_db = torch.from_numpy(np.ascontiguousarray(db_slice[:nrec]).reshape(-1)).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs, stream=st)
    d_ans = torch.full((nk * 32,), 0xA5, dtype=torch.uint8, device=dev)   # overwritten
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=dev)
    dpf.pir_answer_sliced_dev(d_keys, dpf.key_len(logN), nk, logN, d_dbs, nrec, d_ans, d_work, prefix_bits=pb,
                              prefix=prefix, stream=st)
    torch.cuda.synchronize()
    dpf.forget_workspace(d_work)
    return d_ans.cpu().numpy().reshape(nk, 32)


# (logN, nrec, nkeys, prefix_bits, prefix): one to eight workgroups of 256
# leaf pairs, every producer range and piece split, ragged DBs, partial key
# lanes, and subtree slices.
SHAPES = [
    (16, 1 << 16, 64, 0, 0),
    (16, 50001, 1, 0, 0),
    (17, 1 << 17, 37, 0, 0),
    (17, 60000, 64, 1, 0),
    (18, 1 << 17, 64, 1, 1),
    (19, 100000, 33, 2, 3),
    (20, 1 << 19, 64, 1, 0),
]


@pytest.mark.parametrize("logN,nrec,nk,pb,prefix", SHAPES)
def test_sliced_split_matches_oracle(pir_kernel, logN, nrec, nk, pb, prefix):
    slice_n = 1 << (logN - pb)
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    _, ka, _ = _keys(nk, logN, first=logN + nk)
    want = np.stack([np.frombuffer(oracle.pir_answer(ka[i].tobytes(), logN, db, prefix * slice_n, nrec), np.uint8)
                     for i in range(nk)])
    pir_kernel("split")
    assert np.array_equal(_answer(ka, logN, db, nrec, pb, prefix), want)


@needs_fused
@pytest.mark.parametrize("logN,nrec,nk,pb,prefix", SHAPES)
def test_fused_matches_oracle(pir_kernel, logN, nrec, nk, pb, prefix):
    slice_n = 1 << (logN - pb)
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    _, ka, _ = _keys(nk, logN, first=logN + nk)
    pir_kernel("fused-any")
    got = _answer(ka, logN, db, nrec, pb, prefix)
    want = np.stack([np.frombuffer(oracle.pir_answer(ka[i].tobytes(), logN, db, prefix * slice_n, nrec), np.uint8)
                     for i in range(nk)])
    assert np.array_equal(got, want)


@needs_fused
def test_fused_at_configs4_recovers_records(pir_kernel):
    """configs[4] on one GPU (logN=24, 2^24 x 32 B, 64 keys) through the
    fused kernel: answer(ka) ^ answer(kb) == DB[alpha] and the answers equal
    the two-launch path's (the default)."""
    logN, nk = 24, 64
    nrec = 1 << logN
    assert dpf.get_pir_kernel() == dpf.PIR_SPLIT
    assert dpf.pir_kernel_for(nk, logN) == dpf.PIR_SPLIT
    pir_kernel("fused")
    assert dpf.pir_kernel_for(nk, logN) == dpf.PIR_FUSED
    assert dpf.pir_kernel_for(65, logN) == dpf.PIR_SPLIT
    assert dpf.pir_kernel_for(nk, 20) == dpf.PIR_SPLIT
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    al, ka, kb = _keys(nk, logN, first=321)
    a, b = _answer(ka, logN, db, nrec), _answer(kb, logN, db, nrec)
    rec = a ^ b
    for i in range(nk):
        assert np.array_equal(rec[i], db[int(al[i])]), i
    pir_kernel("split")
    assert np.array_equal(_answer(ka, logN, db, nrec), a)
    # a partial key tile (40 lanes live) through the handle
    pir_kernel("fused")
    pdb = dpf.PirDB(db, logN, ngpus=1)
    got = pdb.answer(ka[:40])
    pdb.close()
    assert np.array_equal(got, a[:40])


def test_pir_kernel_switch(pir_kernel):
    prev = pir_kernel("split")
    assert dpf.get_pir_kernel() == dpf.PIR_SPLIT
    assert pir_kernel(prev) == dpf.PIR_SPLIT
    with pytest.raises(Exception):
        pir_kernel(7)
    if not _fused_built():
        # product build: the fused kernel is refused, and every shape runs split
        with pytest.raises(dpf.DPFPanic) as e:
            pir_kernel("fused")
        assert e.value.code == dpf.DPF_ERR_PARAM
        assert dpf.get_pir_kernel() == dpf.PIR_SPLIT
        assert dpf.pir_kernel_for(64, 24) == dpf.PIR_SPLIT
