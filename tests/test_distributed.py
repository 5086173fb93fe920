"""Multi-process (gloo, world_size 2, 4 and 8, CPU) tests of the multi-GPU partition
logic in dpf/shard.py: subtree-split EvalFull reassembly and the PIR partial
answer gather + host XOR fold.  Per-rank compute uses the CPU oracle here
(test infrastructure); on the GPU box the same logic runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from dpf import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "dpf-go_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist
    import oracle
    from dpf import shard as sh, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        logN = 12
        _, s0, s1 = synth.key_seeds(3, 64, first=9)
        keys = [oracle.gen(a, logN, s0[i].tobytes(), s1[i].tobytes())[0] for i, a in enumerate((5, 1000, 4095))]
        # subtree split: each rank computes its slice of EvalFull, gather, reassemble
        pb, p = sh.subtree_split(world, rank)
        full = [np.frombuffer(oracle.evalfull(k, logN), np.uint8) for k in keys]
        size = len(full[0]) >> pb
        mine = torch.from_numpy(np.stack([f[p * size:(p + 1) * size] for f in full]).copy())
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        joined = np.concatenate([t.numpy() for t in parts], axis=1)
        ok_split = all(np.array_equal(joined[i], full[i]) for i in range(3))
        # PIR: rank folds its DB slice, gather_xor combines
        nrec = 1 << logN
        db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
        lo, hi = sh.db_slice(nrec, logN, world, rank)
        part = np.stack([np.frombuffer(oracle.pir_answer(k, logN, db[lo:hi], lo, hi - lo), np.uint8) for k in keys])
        ans = sh.gather_xor(torch.from_numpy(part.copy()))
        want = np.stack([np.frombuffer(oracle.pir_answer(k, logN, db, 0, nrec), np.uint8) for k in keys])
        q.put((rank, ok_split, bool(np.array_equal(ans, want)), sh.key_range(4096, world, rank)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gloo_split_and_pir(world):
    """The driver's N = 2/4/8 partitions: prefix-log2(N) subtree slices
    reassemble to the whole EvalFull, and the N DB-slice partial answers
    gathered and XORed (shard.gather_xor, the RCCL path's gloo twin) equal the
    whole-DB answer."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] for r in res), "subtree split reassembly failed"
    assert all(r[2] for r in res), "PIR gather+XOR failed"
    assert [r[3] for r in res] == [(r * 4096 // world, (r + 1) * 4096 // world) for r in range(world)]


def test_partition_helpers():
    assert shard.subtree_split(8, 5) == (3, 5)
    assert shard.subtree_split(1, 0) == (0, 0)
    with pytest.raises(ValueError):
        shard.subtree_split(6, 0)
    assert shard.db_slice(1 << 24, 24, 8, 7) == (7 << 21, 8 << 21)
    assert shard.db_slice(1000, 10, 2, 1) == (512, 1000)
    assert [shard.key_range(10, 3, r) for r in range(3)] == [(0, 3), (3, 6), (6, 10)]
    a = np.arange(64, dtype=np.uint8).reshape(2, 32)
    assert np.array_equal(shard.xor_fold(a), a[0] ^ a[1])


def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` outside a launcher starts 2 ranks itself
    (torch.distributed.run as a child) and rank 0 reports n_gpus == 2; the
    dry run goes through the same launch, barrier and max-over-ranks path
    as a real run without touching a device."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    def run(*extra):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                            "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.3", *extra],
                           capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        return json.loads(lines[0])
    d = run()
    assert d["n_gpus"] == 2 and d["dry_run"] and d["local_ranks"] == "2"
    # N > 1 lines keep the CPU baseline (rank 0, after the timed region) ...
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    # ... and report HBM traffic only where a PMC profile measured that
    # per-rank shape: a 2-way PIR/split rank runs half a subtree.
    assert "roofline" in d
    p = run("--workload", "pir")
    assert p["roofline"]["traffic"] is None and "traffic_note" in p["roofline"]
    # ... and every workload line carries its own CPU baseline (queries/s here).
    assert p["cpu_baseline"]["unit"] == "queries/s" and p["cpu_baseline"]["value"] > 0
    # PIR with a fixed batch is strong scaling; --batch queries per GPU is weak.
    assert p["scaling"] == "strong"
    w = run("--workload", "pir", "--pir-per-gpu", "--no-cpu-baseline")
    assert w["scaling"] == "weak"


@pytest.mark.parametrize("workload", ["evalfull", "pir"])
def test_bench_gpus_8_dry_run(workload):
    """The driver's 8-GPU command shape (`bench.py --gpus 8`): 8 ranks through
    the same spawn, barriers and max-over-ranks reduction; rank 0 prints one
    line with n_gpus 8 and the workload's scaling label."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--dry-run", "--workload",
                        workload, "--steps", "3", "--warmup", "1", "--cpu-seconds", "0.3", "--no-cpu-baseline"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["local_ranks"] == "8" and d["workload"] == workload
    assert d["scaling"] == ("weak" if workload == "evalfull" else "strong")


def test_xor_rows_matches_numpy():
    """The device-side combine of the RCCL gather (shard.gather_xor), checked
    on CPU tensors: 8-byte lanes and the byte fallback."""
    import torch
    rng = np.random.default_rng(5)
    for shape in ((8, 64, 32), (2, 5, 3), (1, 16), (3, 8, 4), (7, 2, 8), (5, 9)):
        a = rng.integers(0, 256, shape, dtype=np.uint8)
        got = shard.xor_rows(torch.from_numpy(a)).numpy()
        assert got.shape == a.shape[1:]
        assert np.array_equal(got, shard.xor_fold(a))
