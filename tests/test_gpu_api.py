"""GPU checks of the C-ABI's contracts around the kernels (include/dpf_hip.h):
the expanded-key form's shape check, and a process that exits without
dpf_gpu_shutdown (no HIP call from static teardown)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import dpf
from dpf import synth
import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dpf.gpu_init(1) >= 1


def test_expanded_form_checks_nkeys_and_logN():
    import torch
    logN, nk = 12, 8
    al, s0, s1 = synth.key_seeds(nk, logN, first=31)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    kl, olen = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).cuda()
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(nk * olen, dtype=torch.uint8, device="cuda")
    dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work)
    for bad_nk, bad_logN in ((nk // 2, logN), (nk, logN + 1)):
        with pytest.raises(dpf.DPFPanic) as e:
            dpf.evalfull_expanded_dev(d_work, bad_nk, bad_logN, d_out)
        assert e.value.code == dpf.DPF_ERR_PARAM
    dpf.evalfull_expanded_dev(d_work, nk, logN, d_out)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().reshape(nk, olen), oracle.evalfull_batch(ka, logN, nthreads=4))


def test_process_exits_cleanly_without_shutdown():
    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import numpy as np, dpf\n"
        "from dpf import synth\n"
        "assert dpf.gpu_init(1) >= 1\n"
        "al, s0, s1 = synth.key_seeds(4, 14)\n"
        "ka, kb = dpf.gen_batch_seeded(al, 14, s0, s1)\n"
        "full = dpf.evalfull_batch(np.concatenate([ka, kb]), 14, ngpus=1)\n"
        "x = full[:4] ^ full[4:]\n"
        "assert all(np.unpackbits(x[k], bitorder='little').sum() == 1 for k in range(4))\n"
        "print('done')\n"   # no dpf_gpu_shutdown: the registry is left to process exit
    ) % (os.path.join(ROOT, "dpf-go_amd"), os.path.join(ROOT, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("done")


def test_expanded_form_builds_byte_sliced_records_on_first_use():
    """Expanded under the T-table back end (8-word records only), evaluated
    under the byte-sliced one: its records are derived from the expanded
    T-table records (launch_bs_from_ek) on first use, bit-exact."""
    import torch
    logN, nk = 16, 12
    al, s0, s1 = synth.key_seeds(nk, logN, first=88)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    kl, olen = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).cuda()
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
    want = oracle.evalfull_batch(ka, logN, nthreads=4)
    prev = dpf.set_aes_impl("ttable")
    try:
        dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work)
        dpf.set_aes_impl("bitsliced")
        for _ in range(2):    # first use builds the planes, the second reuses them
            d_out = torch.zeros(nk * olen, dtype=torch.uint8, device="cuda")
            dpf.evalfull_expanded_dev(d_work, nk, logN, d_out)
            torch.cuda.synchronize()
            assert np.array_equal(d_out.cpu().numpy().reshape(nk, olen), want)
    finally:
        dpf.set_aes_impl(prev)


def test_workspace_reexpanded_by_another_entry_point_is_not_stale():
    """a workspace registered with byte-sliced planes, then used
    for OTHER keys by dpf_evalfull_subtree_dev under the T-table back end,
    must not be evaluated from the old planes when the caller switches back
    to byte-sliced: the registry follows every entry point.  When the
    one-shot call reads the key bytes directly (no expansion into d_work), the
    record is dropped and the expanded call refuses; when it expands, the
    planes are rebuilt from the new keys.  dpf_forget_workspace drops the
    record (the next expanded call refuses)."""
    import torch
    logN, nk = 16, 8
    kl, olen = dpf.key_len(logN), dpf.evalfull_len(logN)
    al, s0, s1 = synth.key_seeds(nk, logN, first=404)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    al2, s02, s12 = synth.key_seeds(nk, logN, first=505)
    kb, _ = dpf.gen_batch_seeded(al2, logN, s02, s12)
    d_a = torch.from_numpy(ka.reshape(-1)).cuda()
    d_b = torch.from_numpy(kb.reshape(-1)).cuda()
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device="cuda")
    d_out = torch.zeros(nk * olen, dtype=torch.uint8, device="cuda")
    prev = dpf.set_aes_impl("bitsliced")
    try:
        dpf.expand_keys_dev(d_a, kl, nk, logN, d_work)           # planes of keys A
        dpf.evalfull_expanded_dev(d_work, nk, logN, d_out)
        dpf.set_aes_impl("ttable")
        dpf.evalfull_subtree_dev(d_b, kl, nk, logN, 0, 0, d_out, d_work)   # records of keys B only
        dpf.set_aes_impl("bitsliced")
        d_out.zero_()
        try:
            dpf.evalfull_expanded_dev(d_work, nk, logN, d_out)    # planes rebuilt from B, or refused
        except dpf.DPFPanic as e:
            assert e.code == dpf.DPF_ERR_PARAM                      # d_work no longer holds expanded keys
        else:
            torch.cuda.synchronize()
            assert np.array_equal(d_out.cpu().numpy().reshape(nk, olen), oracle.evalfull_batch(kb, logN, nthreads=4))
        dpf.expand_keys_dev(d_b, kl, nk, logN, d_work)
        dpf.forget_workspace(d_work)
        with pytest.raises(dpf.DPFPanic) as e:
            dpf.evalfull_expanded_dev(d_work, nk, logN, d_out)
        assert e.value.code == dpf.DPF_ERR_PARAM
    finally:
        dpf.set_aes_impl(prev)


def test_cu_masked_streams_give_identical_results():
    """dpf_stream_create_cu_masked: kernels on a stream limited to a CU range
    (grids sized to it) give the same bytes as on the whole device; the
    tree and the PIR fold on two disjoint ranges at once agree with the
    oracle; bad ranges are refused."""
    import torch
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.stream_create_cu_masked(0, 0)
    assert e.value.code == dpf.DPF_ERR_PARAM
    with pytest.raises(dpf.DPFPanic) as e:
        dpf.stream_create_cu_masked(ncu - 4, 8)
    assert e.value.code == dpf.DPF_ERR_PARAM
    T = dpf.stream_create_cu_masked(16, ncu - 16)
    F = dpf.stream_create_cu_masked(0, 16)
    try:
        logN, nk = 18, 48
        al, s0, s1 = synth.key_seeds(nk, logN, first=515)
        ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
        kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
        d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
        d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
        bits = torch.full((nk * ol,), 0x5A, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        dpf.evalfull_batch_dev(d_keys, kl, nk, logN, bits, d_work, stream=T)
        T.synchronize()
        want = oracle.evalfull_batch(ka, logN, nthreads=8)
        assert np.array_equal(bits.cpu().numpy().reshape(nk, ol), want)
        nrec = (1 << logN) - 300
        db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
        d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
        dpf.pir_db_slice_dev(torch.from_numpy(db.reshape(-1)).to(dev), nrec, d_dbs, stream=F)
        d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
        fwork = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
        bits2 = torch.empty_like(bits)
        # fold the first bits on F while T evaluates the same keys again
        dpf.xor_fold_sliced_dev(bits, ol, nk, d_dbs, nrec, d_ans, fwork, stream=F)
        dpf.evalfull_batch_dev(d_keys, kl, nk, logN, bits2, d_work, stream=T)
        torch.cuda.synchronize()
        assert torch.equal(bits, bits2)
        want_ans = oracle.pir_answer_batch(ka, logN, db, nrec, nslices=1, nthreads=8)[:, 0, :]
        assert np.array_equal(d_ans.cpu().numpy().reshape(nk, 32), want_ans)
    finally:
        torch.cuda.synchronize()
        dpf.stream_destroy(T)
        dpf.stream_destroy(F)


def test_cu_masked_stream_big_tree_workgroups():
    """The r06 tree geometry on a CU-limited stream: 512 keys at logN 20 on 16
    CUs fill more than a round of 512-thread groups, so the launch takes
    1024-thread workgroups with progress-feedback priority (several rounds
    of them on the 16 CUs).  Every byte against the oracle."""
    import torch
    dev = torch.device("cuda", 0)
    S = dpf.stream_create_cu_masked(0, 16)
    try:
        logN, nk = 20, 512
        al, s0, s1 = synth.key_seeds(nk, logN, first=2626)
        ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
        kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
        d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
        d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
        out = torch.full((nk * ol,), 0x5A, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        dpf.evalfull_batch_dev(d_keys, kl, nk, logN, out, d_work, stream=S)
        S.synchronize()
        want = oracle.evalfull_batch(ka, logN, nthreads=8)
        assert np.array_equal(out.cpu().numpy().reshape(nk, ol), want)
    finally:
        torch.cuda.synchronize()
        dpf.stream_destroy(S)
