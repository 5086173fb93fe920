"""r06 measurement: the configs[4] PIR server as a key stream over two
CU-partitioned streams, tree launches decoupled from the 64-query batches.

Why: the tree kernel fills the chip in exactly one round of 16 waves per CU
(64 keys x 2^12 subtrees = 4096 waves at D = 5), so on a CU subset its time
is set by wave quantization (tools/r06_pir_cumask.py: 0.46 ms on any of
128..240 CUs).  Here the tree stream evaluates the key stream in launches of
kt = 16 * C / 64 keys for its C CUs (one exact round), writing selection
bits into a ring of key slots, and the fold stream folds each 64-key batch
once the launches covering its slots are done.  The fold of batch b and the
trees of later keys run side by side on disjoint CUs (mask bits interleave
over the XCDs).

  python tools/r06_pir_stream.py [--ks 48,64,80] [--batches 60]
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
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--ks", default="48,64,80")
    ap.add_argument("--kt", default="", help="keys per tree launch for each k (default 16*(ncu-k)/64)")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    assert dpf.gpu_init(1) >= 1
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    logN, nk = a.logN, a.nk
    nrec = 1 << logN
    kl = dpf.key_len(logN)
    per_key = 16 << (logN - 7)
    db = synth.db_bytes(nrec * 32)
    d_db = torch.from_numpy(db).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs, stream=torch.cuda.current_stream(dev))
    del d_db
    al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    torch.cuda.synchronize()

    main_st = torch.cuda.Stream(dev)
    d_keys1 = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, 0), dtype=torch.uint8, device=dev)
    h1 = [torch.empty(nk * 32, dtype=torch.uint8, pin_memory=True) for _ in range(2)]

    def run_product(batches):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(batches):
            dpf.pir_answer_sliced_dev(d_keys1, kl, nk, logN, d_dbs, nrec, d_ans, d_work, stream=main_st)
            with torch.cuda.stream(main_st):
                h1[i % 2].copy_(d_ans, non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / batches * 1e3, h1[(batches - 1) % 2].clone()

    R = 4 * nk                                              # ring of key slots (4 batches)
    d_ring_keys = torch.from_numpy(np.tile(ka, (R // nk, 1)).reshape(-1)).to(dev)
    ring_bits = torch.empty(R * per_key, dtype=torch.uint8, device=dev)
    work = torch.empty(dpf.workspace_size(R, logN), dtype=torch.uint8, device=dev)
    fwork = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
    ans = [torch.empty(nk * 32, dtype=torch.uint8, device=dev) for _ in range(2)]
    h2 = [torch.empty(nk * 32, dtype=torch.uint8, pin_memory=True) for _ in range(2)]

    def run_stream(T, F, kt, batches):
        """Key g of the stream sits in ring slot g % R.  Tree launch t covers
        keys [kt t, kt (t+1)) (split at the ring's end); batch b = keys
        [nk b, nk (b+1)).  Fold b waits for the launches covering its keys;
        a launch waits for the folds of the batches whose slots it reuses."""
        total = batches * nk
        fold_done = {}
        tree_done = []
        ev_pool = []

        def ev():
            e = ev_pool.pop() if ev_pool else torch.cuda.Event()
            return e
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g_tree = 0                                        # next key the tree stream evaluates
        for b in range(batches):
            need = nk * (b + 1)
            while g_tree < need:                          # issue tree launches up to this batch's last key
                g1 = min(g_tree + kt, total if total > g_tree else g_tree + kt)
                # slots reused: keys g - R for g in [g_tree, g1) belong to batches (g - R) // nk
                lo_b, hi_b = (g_tree - R) // nk, (g1 - 1 - R) // nk
                for ob in range(max(lo_b, 0), hi_b + 1):
                    if ob in fold_done:
                        T.wait_event(fold_done[ob])
                g = g_tree
                while g < g1:                             # split at the ring's end
                    s = g % R
                    n = min(g1 - g, R - s)
                    dpf.evalfull_subtree_dev(d_ring_keys[s * kl:], kl, n, logN, 0, 0, ring_bits[s * per_key:],
                                             work, stream=T)
                    g += n
                e = ev()
                e.record(T)
                tree_done.append((g1, e))
                g_tree = g1
            for g_end, e in tree_done:                    # launches covering [nk b, nk (b+1))
                if g_end > nk * b:
                    F.wait_event(e)
            tree_done = [(g_end, e) for g_end, e in tree_done if g_end > need]
            s = (nk * b) % R
            dpf.xor_fold_sliced_dev(ring_bits[s * per_key:], per_key, nk, d_dbs, nrec, ans[b % 2], fwork, stream=F)
            with torch.cuda.stream(F):
                h2[b % 2].copy_(ans[b % 2], non_blocking=True)
            e = ev()
            e.record(F)
            fold_done[b] = e
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / batches * 1e3, h2[(batches - 1) % 2].clone()

    t_end = time.time() + 0.6
    while time.time() < t_end:
        run_product(10)
    ks = [int(k) for k in a.ks.split(",") if k]
    kts = [int(x) for x in a.kt.split(",")] if a.kt else [16 * (ncu - k) // 64 for k in ks]
    streams = {k: (dpf.stream_create_cu_masked(k, ncu - k), dpf.stream_create_cu_masked(0, k)) for k in ks}
    res = {"shape": {"logN": logN, "nk": nk, "ncu": ncu, "ring": R}, "rounds": []}
    for r in range(a.rounds):
        row = {}
        ms, ref = run_product(a.batches)
        row["product"] = round(ms, 4)
        for k, kt in zip(ks, kts):
            T, F = streams[k]
            ms, got = run_stream(T, F, kt, a.batches)
            assert torch.equal(got, ref), f"k={k}: answers differ"
            row[f"fold{k}_kt{kt}"] = round(ms, 4)
        ms, _ = run_product(a.batches)
        row["product_again"] = round(ms, 4)
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res), flush=True)
    del h1, h2, ref, got
    torch.cuda.synchronize()
    for T, F in streams.values():
        dpf.stream_destroy(T)
        dpf.stream_destroy(F)
    print("done", flush=True)


if __name__ == "__main__":
    main()
