"""Per-rank shapes of the 8-GPU runs, on one GPU (VERDICT r03 "make the 8-GPU
run work the first time").

An N-GPU configs[3] / configs[4] rank runs exactly the calls below on its own
device (bench.py wl_split / wl_pir, dpf/shard.py):
  - configs[3]: one logN=32 key, rank r evaluates top-level subtree r at depth
    log2(N) (prefix_bits=3 at N=8); its slice is the 64 MiB at offset r*64 MiB
    of EvalFull's output, because evalFullRecursive visits left before right
    (dpf/dpf.go:239-240), so the slices must reassemble the whole output;
  - configs[4]: rank r holds DB records [r*2^21, (r+1)*2^21) and answers with
    dpf_pir_answer_dev(prefix_bits=3, prefix=r); the 8 partials XOR to the
    whole answer, and two servers' answers XOR to DB[alpha].
The RCCL branch of shard.gather_xor runs here with a world of 1 (RCCL refuses
two ranks on one GPU); its device XOR tree runs at the 8-row shape."""
import os
import socket

import numpy as np
import pytest

import dpf
from dpf import shard, synth
import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert dpf.gpu_init(1) >= 1
    prev = dpf.set_small_call_path("gpu")
    yield
    dpf.set_small_call_path(prev)


def _stream():
    import torch
    return torch.cuda.current_stream(torch.device("cuda", 0))


@pytest.mark.parametrize("aes", ["ttable", "bitsliced"])
def test_config3_eight_prefix3_subtrees_of_one_logN32_key(aes):
    import torch
    logN, pb = 32, 3
    alpha = 0x9E3779B9 & ((1 << logN) - 1)
    _, s0, s1 = synth.key_seeds(1, 64, first=3131)
    ka, kb = dpf.gen_seeded(alpha, logN, s0[0].tobytes(), s1[0].tobytes())
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    part = ol >> pb                       # 64 MiB per rank
    leaves_per_part = (1 << logN) >> pb
    dev = torch.device("cuda", 0)
    prev = dpf.set_aes_impl(aes)
    try:
        d_ka = torch.from_numpy(np.frombuffer(ka, np.uint8).copy()).to(dev)
        d_kb = torch.from_numpy(np.frombuffer(kb, np.uint8).copy()).to(dev)
        # The whole output on one GPU (the reference's leaf order).
        d_work = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=dev)
        d_full = torch.empty(ol, dtype=torch.uint8, device=dev)
        dpf.evalfull_batch_dev(d_ka, kl, 1, logN, d_full, d_work, stream=_stream())
        # Rank r's two call forms: the one-shot subtree entry point, and the
        # expanded form bench.py's split rank times (expand once, evaluate its prefix).
        d_wa = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=dev)
        d_wb = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=dev)
        dpf.expand_keys_dev(d_kb, kl, 1, logN, d_wb, stream=_stream())
        sa = torch.empty(part, dtype=torch.uint8, device=dev)
        sb = torch.empty(part, dtype=torch.uint8, device=dev)
        rng = np.random.default_rng(7)
        ones = []
        for r in range(1 << pb):
            dpf.evalfull_subtree_dev(d_ka, kl, 1, logN, pb, r, sa, d_wa, stream=_stream())
            dpf.evalfull_expanded_dev(d_wb, 1, logN, sb, prefix_bits=pb, prefix=r, stream=_stream())
            torch.cuda.synchronize()
            assert torch.equal(sa, d_full[r * part:(r + 1) * part]), f"slice {r} differs from the whole output"
            x = (sa ^ sb).view(torch.int64)
            nz = torch.nonzero(x).flatten()
            base = r * leaves_per_part
            if base <= alpha < base + leaves_per_part:
                assert nz.numel() == 1
                w = int(nz[0])
                v = int(x[w].item()) & 0xFFFFFFFFFFFFFFFF
                assert v & (v - 1) == 0 and base + w * 64 + v.bit_length() - 1 == alpha
                ones.append(r)
            else:
                assert nz.numel() == 0, f"slice {r}: share XOR not zero"
            # first and last leaf blocks (128 points each) and random points vs the oracle's Eval
            head = sa[:16].cpu().numpy()
            tail = sa[part - 16:].cpu().numpy()
            for q in range(0, 128, 3):
                assert ((head[q >> 3] >> (q & 7)) & 1) == oracle.eval_(ka, base + q, logN, aesni=True)
                g = leaves_per_part - 128 + q
                assert ((tail[q >> 3] >> (q & 7)) & 1) == oracle.eval_(ka, base + g, logN, aesni=True)
            pts = rng.integers(0, leaves_per_part, 48)
            idx = torch.from_numpy((pts >> 3).astype(np.int64)).to(dev)
            bytes_ = sb[idx].cpu().numpy()
            for p, b in zip(pts, bytes_):
                assert ((int(b) >> (int(p) & 7)) & 1) == oracle.eval_(kb, base + int(p), logN, aesni=True)
        assert ones == [alpha >> (logN - pb)]
    finally:
        dpf.set_aes_impl(prev)


def test_config4_eight_db_slices_logN24(cfg4):
    """configs[4] per rank at N=8 over the row-major DB (dpf_pir_answer_dev),
    all 8 ranks in turn on one GPU, B=64: every key's partial of both
    servers vs the oracle's slice partial."""
    import torch
    logN, pb, nk = 24, 3, 64
    nrec, db, al, ka, kb = cfg4["nrec"], cfg4["db"], cfg4["al"], cfg4["ka"], cfg4["kb"]
    kl = dpf.key_len(logN)
    dev = torch.device("cuda", 0)
    d_ka = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_kb = torch.from_numpy(kb.reshape(-1)).to(dev)
    d_db = cfg4["d_db"]
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
    # the 1-GPU answer over the whole DB
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, 0), dtype=torch.uint8, device=dev)
    dpf.pir_answer_dev(d_ka, kl, nk, logN, d_db, nrec, d_ans, d_work, stream=_stream())
    torch.cuda.synchronize()
    whole_a = d_ans.cpu().numpy().reshape(nk, 32)
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=dev)
    acc_a = np.zeros((nk, 32), np.uint8)
    acc_b = np.zeros((nk, 32), np.uint8)
    for r in range(1 << pb):
        lo, hi = shard.db_slice(nrec, logN, 1 << pb, r)
        d_slice = d_db[lo * 32:hi * 32]
        parts = []
        for d_k in (d_ka, d_kb):
            dpf.pir_answer_dev(d_k, kl, nk, logN, d_slice, hi - lo, d_ans, d_work, prefix_bits=pb, prefix=r,
                               stream=_stream())
            torch.cuda.synchronize()
            parts.append(d_ans.cpu().numpy().reshape(nk, 32).copy())
        for j, share in enumerate(("a", "b")):
            want = cfg4["oracle_" + share][:, r, :]
            bad = np.argwhere(parts[j] != want)
            assert bad.size == 0, (share, r, f"first differing key {bad[0][0]}" if bad.size else "")
        acc_a ^= parts[0]
        acc_b ^= parts[1]
    assert np.array_equal(acc_a, whole_a)
    rec = acc_a ^ acc_b
    for i in range(nk):
        assert np.array_equal(rec[i], db[int(al[i])]), i


@pytest.fixture(scope="module")
def cfg4():
    """configs[4]'s inputs (logN=24, 2^24 x 32 B synthetic DB, B=64 keys of
    bench.py's seed) and the 1-GPU answers of the product path: the matrix-core
    fold over the whole bit-sliced DB (prefix_bits=0)."""
    import torch
    logN, nk = 24, 64
    nrec = 1 << logN
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    dev = torch.device("cuda", 0)
    d_db = torch.from_numpy(db.reshape(-1)).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs, stream=_stream())
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, 0), dtype=torch.uint8, device=dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
    whole = []
    for k in (ka, kb):
        d_k = torch.from_numpy(k.reshape(-1)).to(dev)
        dpf.pir_answer_sliced_dev(d_k, dpf.key_len(logN), nk, logN, d_dbs, nrec, d_ans, d_work, stream=_stream())
        torch.cuda.synchronize()
        whole.append(d_ans.cpu().numpy().reshape(nk, 32).copy())
    dpf.forget_workspace(d_work)
    del d_dbs, d_work
    # The oracle's partial of every key over each of the 8 rank slices (an
    # N = 2 / 4 rank's partial is the XOR of 4 / 2 consecutive ones).
    ora = {"a": oracle.pir_answer_batch(ka, logN, db, nrec, nslices=8),
           "b": oracle.pir_answer_batch(kb, logN, db, nrec, nslices=8)}
    for j, share in enumerate(("a", "b")):
        want = np.bitwise_xor.reduce(ora[share], axis=1)
        bad = np.argwhere(whole[j] != want)
        assert bad.size == 0, (share, f"1-GPU answer of key {bad[0][0]} differs" if bad.size else "")
    return {"logN": logN, "nk": nk, "nrec": nrec, "db": db, "al": al, "ka": ka, "kb": kb, "d_db": d_db,
            "whole_a": whole[0], "whole_b": whole[1], "oracle_a": ora["a"], "oracle_b": ora["b"]}


@pytest.mark.parametrize("pb", [1, 2, 3])
def test_config4_sliced_product_path_per_rank(cfg4, pb):
    """The N = 2^pb PIR rank's product path, as bench.py --gpus N --workload
    pir runs it (pir_setup / pir_time): rank r bit-slices its DB slice
    [r*2^(24-pb), (r+1)*2^(24-pb)) once (dpf_pir_db_slice_dev on d_db[lo:hi])
    and answers with dpf_pir_answer_sliced_dev(prefix_bits=pb, prefix=r):
    subtree r of every key (dpf/dpf.go:213-241 below the prefix) folded on the
    matrix cores.  The partials XOR to the
    1-GPU sliced answer, and the two servers XOR to DB[alpha].  Every key's
    partial of both servers at every rank against the oracle's partial over
    that slice (dpf.go:243-262 bits)."""
    import torch
    logN, nk, nrec, db = cfg4["logN"], cfg4["nk"], cfg4["nrec"], cfg4["db"]
    ka, kb, d_db = cfg4["ka"], cfg4["kb"], cfg4["d_db"]
    kl = dpf.key_len(logN)
    dev = torch.device("cuda", 0)
    W = 1 << pb
    d_keys = [torch.from_numpy(k.reshape(-1)).to(dev) for k in (ka, kb)]
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
    acc = [np.zeros((nk, 32), np.uint8), np.zeros((nk, 32), np.uint8)]
    for r in range(W):
        pb_r, prefix = shard.subtree_split(W, r)
        assert (pb_r, prefix) == (pb, r)
        lo, hi = shard.db_slice(nrec, logN, W, r)
        assert (lo, hi) == (r << (logN - pb), (r + 1) << (logN - pb))
        d_dbs = torch.empty(dpf.pir_db_sliced_size(hi - lo), dtype=torch.uint8, device=dev)
        dpf.pir_db_slice_dev(d_db[lo * 32:hi * 32], hi - lo, d_dbs, stream=_stream())
        parts = []
        for d_k in d_keys:
            d_ans.fill_(0xA5)                                   # overwritten, not accumulated
            dpf.pir_answer_sliced_dev(d_k, kl, nk, logN, d_dbs, hi - lo, d_ans, d_work, prefix_bits=pb,
                                      prefix=prefix, stream=_stream())
            torch.cuda.synchronize()
            parts.append(d_ans.cpu().numpy().reshape(nk, 32).copy())
        g = 8 // W                                   # oracle slices per rank
        for j, share in enumerate(("a", "b")):
            want = np.bitwise_xor.reduce(cfg4["oracle_" + share][:, r * g:(r + 1) * g, :], axis=1)
            bad = np.argwhere(parts[j] != want)
            assert bad.size == 0, (share, r, f"first differing key {bad[0][0]}" if bad.size else "")
        acc[0] ^= parts[0]
        acc[1] ^= parts[1]
        del d_dbs
    dpf.forget_workspace(d_work)
    assert np.array_equal(acc[0], cfg4["whole_a"])
    assert np.array_equal(acc[1], cfg4["whole_b"])
    rec = acc[0] ^ acc[1]
    for i in range(nk):
        assert np.array_equal(rec[i], db[int(cfg4["al"][i])]), i


def test_config4_pirdb_handle_on_eight_logical_devices():
    """PirDB(db, 24, ngpus=8): the library's own 8-way sharded PIR handle at
    the full configs[4] shape (8 bit-sliced 64 MiB shards, one per logical
    device on this GPU, host XOR of the 8 partials), against the 1-GPU handle
    and the 2-server property.  In a subprocess: the device registry is
    process-wide."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys; sys.path[:0] = [%r, %r]
import numpy as np, dpf, oracle
from dpf import synth
assert dpf.gpu_init_devices([0] * 8) == 8
logN, nk = 24, 64
nrec = 1 << logN
db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
al, s0, s1 = synth.key_seeds(nk, logN, first=8080)
ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
p8 = dpf.PirDB(db, logN, ngpus=8)
a8, b8 = p8.answer(ka), p8.answer(kb)
p8.close()
p1 = dpf.PirDB(db, logN, ngpus=1)
a1 = p1.answer(ka)
p1.close()
assert np.array_equal(a8, a1)
rec = a8 ^ b8
for i in range(nk):
    assert np.array_equal(rec[i], db[int(al[i])]), i
want = oracle.pir_answer_batch(ka, logN, db, nrec, nslices=1)[:, 0, :]
assert np.array_equal(a8, want), np.argwhere(a8 != want)[:1]
dpf.gpu_shutdown()
print("done")
''' % (os.path.join(root, "dpf-go_amd"), os.path.join(root, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().endswith("done")


def test_library_multi_device_entry_points_with_every_opened_device():
    """dpf_evalfull_split and the PIR handle with ngpus = the opened devices
    (1 on a 1-GPU box; the same code shards over 8 on a full node)."""
    n = dpf.gpu_count()
    logN = 22
    al, s0, s1 = synth.key_seeds(2, logN, first=999)
    ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
    out = dpf.evalfull_split(ka[0].tobytes(), logN, n)
    assert out.tobytes() == oracle.evalfull(ka[0].tobytes(), logN, aesni=True)
    lp = 16
    nrec = (1 << lp) - 3                     # ragged last shard
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    a2, t0, t1 = synth.key_seeds(5, lp, first=77)
    qa, qb = dpf.gen_batch_seeded(a2, lp, t0, t1)
    pdb = dpf.PirDB(db, lp, ngpus=n)
    try:
        ga, gb = pdb.answer(qa), pdb.answer(qb)
    finally:
        pdb.close()
    for i in range(5):
        assert ga[i].tobytes() == oracle.pir_answer(qa[i].tobytes(), lp, db, 0, nrec)
        want = db[int(a2[i])] if a2[i] < nrec else np.zeros(32, np.uint8)
        assert np.array_equal(ga[i] ^ gb[i], want)


def test_gather_xor_rccl_branch_and_eight_row_device_xor():
    """shard.gather_xor over a real RCCL process group (world 1 on this box)
    and the device XOR tree at the 8-rank shape [8, 64, 32]."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    rows = rng.integers(0, 256, (8, 64, 32), dtype=np.uint8)
    got = shard.xor_rows(torch.from_numpy(rows).to(dev)).cpu().numpy()
    assert np.array_equal(got, shard.xor_fold(rows))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        part = torch.from_numpy(rows[3]).to(dev)
        ans = shard.gather_xor(part)
        assert np.array_equal(ans, rows[3])
    finally:
        dist.destroy_process_group()


def test_in_library_multi_device_paths_on_eight_logical_devices():
    """The library's own multi-device code (dpf_evalfull_split / _batch /
    dpf_eval_batch over ngpus devices on one host thread each, the PIR handle
    sharded by top-level subtree with the host XOR of the partials) has only
    ever had one device to shard over.  dpf_gpu_init_devices([0] * 8) opens
    the one GPU as 8 logical devices (each its own stream, mutex and
    buffers), so every shard offset, thread and partial XOR of the 8-way paths
    runs here against the oracle.  In a subprocess: the device registry is
    process-wide."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys; sys.path[:0] = [%r, %r]
import numpy as np, dpf, oracle
from dpf import synth
assert dpf.gpu_init_devices([0] * 8) == 8 and dpf.gpu_count() == 8
dpf.set_small_call_path("gpu")
logN = 24
al, s0, s1 = synth.key_seeds(2, logN, first=31)
ka, kb = dpf.gen_batch_seeded(al, logN, s0, s1)
for n in (2, 4, 8):
    out = dpf.evalfull_split(ka[0].tobytes(), logN, n)
    x = out ^ dpf.evalfull_split(kb[0].tobytes(), logN, n)
    bits = np.unpackbits(x, bitorder="little")
    assert bits.sum() == 1 and bits[int(al[0])] == 1, n
full = dpf.evalfull_split(ka[0].tobytes(), logN, 1)
assert np.array_equal(out, full)
for q in (0, 5, (1 << logN) - 1, int(al[0])):
    assert ((int(out[q >> 3]) >> (q & 7)) & 1) == oracle.eval_(ka[0].tobytes(), q, logN, aesni=True)
l2 = 14
a2, t0, t1 = synth.key_seeds(37, l2, first=41)
k2, _ = dpf.gen_batch_seeded(a2, l2, t0, t1)
assert np.array_equal(dpf.evalfull_batch(k2, l2, ngpus=8), oracle.evalfull_batch(k2, l2, nthreads=8))
xs = synth.eval_points(37, 50, l2)
assert np.array_equal(dpf.eval_batch(k2, xs, l2, ngpus=8), oracle.eval_batch(k2, xs, l2, nthreads=8))
lp = 16
nrec = (1 << lp) - 1000
db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
a3, u0, u1 = synth.key_seeds(9, lp, first=51)
qa, qb = dpf.gen_batch_seeded(a3, lp, u0, u1)
pdb = dpf.PirDB(db, lp, ngpus=8)
ga, gb = pdb.answer(qa), pdb.answer(qb)
pdb.close()
for i in range(9):
    assert ga[i].tobytes() == oracle.pir_answer(qa[i].tobytes(), lp, db, 0, nrec)
    want = db[int(a3[i])] if a3[i] < nrec else np.zeros(32, np.uint8)
    assert np.array_equal(ga[i] ^ gb[i], want)
dpf.gpu_shutdown()
print("done")
''' % (os.path.join(root, "dpf-go_amd"), os.path.join(root, "oracle"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().endswith("done")
