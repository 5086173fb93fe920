"""r06 measurement: the configs[4] PIR step with the tree and the fold of
consecutive batches on two CU-partitioned streams (VERDICT r05 "Next" #2).

Tree of batch i+1 on CUs [k, ncu) while the fold of batch i runs on CUs
[0, k) (dpf_stream_create_cu_masked; mask bits interleave over the XCDs),
double-buffered selection bits.  Baseline: the product one-stream step
(dpf_pir_answer_sliced_dev), timed in the same process, interleaved.

  python tools/r06_pir_cumask.py [--pb 0] [--ks 32,48,64,80,96] [--rounds 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dpf-go_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dpf  # noqa: E402
from dpf import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logN", type=int, default=24)
    ap.add_argument("--nk", type=int, default=64)
    ap.add_argument("--pb", type=int, default=0)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--ks", default="32,48,64,80,96")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--phases", action="store_true", help="also time tree / fold alone on each partition")
    a = ap.parse_args()
    assert dpf.gpu_init(1) >= 1
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    logN, nk, pb = a.logN, a.nk, a.pb
    prefix = 0
    nrec = 1 << (logN - pb)
    kl = dpf.key_len(logN)
    per_key = 16 << (logN - 7 - pb)
    db = synth.db_bytes(nrec * 32)
    d_db = torch.from_numpy(db).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs, stream=torch.cuda.current_stream(dev))
    del d_db
    al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    torch.cuda.synchronize()

    # --- product one-stream step (bench.py pir_time) ---
    main_st = torch.cuda.Stream(dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=dev)
    h1 = [torch.empty(nk * 32, dtype=torch.uint8, pin_memory=True) for _ in range(2)]

    def run_product(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            dpf.pir_answer_sliced_dev(d_keys, kl, nk, logN, d_dbs, nrec, d_ans, d_work, prefix_bits=pb,
                                      prefix=prefix, stream=main_st)
            with torch.cuda.stream(main_st):
                h1[i % 2].copy_(d_ans, non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3, h1[(steps - 1) % 2].clone()

    # --- two-stream pipeline ---
    bits = [torch.empty(nk * per_key, dtype=torch.uint8, device=dev) for _ in range(2)]
    work = [torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev) for _ in range(2)]
    fwork = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
    ans = [torch.empty(nk * 32, dtype=torch.uint8, device=dev) for _ in range(2)]
    h2 = [torch.empty(nk * 32, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    tdone = [torch.cuda.Event() for _ in range(2)]
    fdone = [torch.cuda.Event() for _ in range(2)]

    def run_pipe(T, F, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            s = i % 2
            if i >= 2:
                T.wait_event(fdone[s])
            dpf.evalfull_subtree_dev(d_keys, kl, nk, logN, pb, prefix, bits[s], work[s], stream=T)
            tdone[s].record(T)
            F.wait_event(tdone[s])
            dpf.xor_fold_sliced_dev(bits[s], per_key, nk, d_dbs, nrec, ans[s], fwork, stream=F)
            with torch.cuda.stream(F):
                h2[s].copy_(ans[s], non_blocking=True)
            fdone[s].record(F)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3, h2[(steps - 1) % 2].clone()

    def run_phase(st, which, steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            if which == "tree":
                dpf.evalfull_subtree_dev(d_keys, kl, nk, logN, pb, prefix, bits[0], work[0], stream=st)
            else:
                dpf.xor_fold_sliced_dev(bits[0], per_key, nk, d_dbs, nrec, ans[0], fwork, stream=st)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    # spin up the clock
    t_end = time.time() + 0.6
    while time.time() < t_end:
        run_product(10)
    ks = [int(k) for k in a.ks.split(",") if k]
    streams = {k: (dpf.stream_create_cu_masked(k, ncu - k), dpf.stream_create_cu_masked(0, k)) for k in ks}
    plain = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    res = {"shape": {"logN": logN, "nk": nk, "pb": pb, "nrec": nrec, "ncu": ncu}, "rounds": []}
    for r in range(a.rounds):
        row = {}
        ms, ref = run_product(a.steps)
        row["product"] = round(ms, 4)
        ms, got = run_pipe(plain[0], plain[1], a.steps)
        assert torch.equal(got, ref), "two plain streams: answers differ"
        row["two_streams_unmasked"] = round(ms, 4)
        for k in ks:
            T, F = streams[k]
            ms, got = run_pipe(T, F, a.steps)
            assert torch.equal(got, ref), f"k={k}: answers differ"
            row[f"fold{k}"] = round(ms, 4)
            if a.phases and r == 0:
                row[f"tree_on_{ncu - k}"] = round(run_phase(T, "tree", a.steps), 4)
                row[f"fold_on_{k}"] = round(run_phase(F, "fold", a.steps), 4)
        ms, ref2 = run_product(a.steps)
        row["product_again"] = round(ms, 4)
        if a.phases and r == 0:
            row["tree_all"] = round(run_phase(main_st, "tree", a.steps), 4)
            row["fold_all"] = round(run_phase(main_st, "fold", a.steps), 4)
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res), flush=True)
    torch.cuda.synchronize()
    # Pinned buffers copied on the masked streams record events on those
    # streams when freed (torch's host allocator): free them while the
    # streams still exist.
    del h1, h2, ref, ref2, got
    torch.cuda.synchronize()
    for T, F in streams.values():
        dpf.stream_destroy(T)
        dpf.stream_destroy(F)
    print("streams destroyed", flush=True)
    dpf.gpu_shutdown()
    print("shutdown", flush=True)


if __name__ == "__main__":
    main()
