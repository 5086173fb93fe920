#!/usr/bin/env python3
"""api_rates.py — the secondary numbers SURVEY §8d asks for beside bench.py's
device-resident headline, on one MI355X:

  host_api       : the C-ABI host-buffer entry points (dpf_evalfull_batch,
                   dpf_eval_batch, dpf_evalfull_split, dpf_pir_answer),
                   PCIe-inclusive: keys H2D, outputs D2H, synchronous
  single_key     : cfg 1 (one key, logN=20) EvalFull latency, device-resident
                   and through the host API, and Eval of one point
  pir_batch_sweep: PIR logN=24 (cfg 5) at B in {1, 16, 64, 256}, device-resident
  gen            : host Gen throughput (dpf_gen_batch_seeded, all threads)

Prints one JSON object (also written to the path given as argv[1])."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))

import numpy as np  # noqa: E402


def mark(msg):
    print(f"[api_rates] {msg}", file=sys.stderr, flush=True)


def med_time(fn, reps=7, warm=2):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    import torch
    import dpf
    from dpf import synth
    dev = torch.device("cuda", 0)
    dpf.gpu_init(1)
    st = torch.cuda.current_stream(dev)
    res = {"device": torch.cuda.get_device_name(0)}

    mark("host api cfg2")
    # ---- host API, cfg 2: 4096 keys x logN=20 EvalFull -> 512 MiB to host
    logN, nk = 20, 4096
    al, s0, s1 = synth.key_seeds(nk, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    t = med_time(lambda: dpf.evalfull_batch(ka, logN, ngpus=1), reps=5)
    out_b = nk * dpf.evalfull_len(logN)
    res["host_api"] = {"evalfull_batch_cfg2": {"s": t, "points_per_s": nk * (1 << logN) / t,
                                               "D2H_GBs": out_b / t / 1e9, "out": "fresh array per call"}}
    reuse = np.empty((nk, dpf.evalfull_len(logN)), np.uint8)
    t = med_time(lambda: dpf.evalfull_batch(ka, logN, ngpus=1, out=reuse), reps=5)
    res["host_api"]["evalfull_batch_cfg2_reused_out"] = {"s": t, "points_per_s": nk * (1 << logN) / t,
                                                         "D2H_GBs": out_b / t / 1e9}
    mark("cfg3")
    # cfg 3: 2^16 keys x 2^10 points
    ek, ppk = 1 << 16, 1 << 10
    al3, s03, s13 = synth.key_seeds(ek, logN)
    ke, _ = dpf.gen_batch_seeded(al3, logN, s03, s13)
    xs = synth.eval_points(ek, ppk, logN)
    t = med_time(lambda: dpf.eval_batch(ke, xs, logN, ngpus=1), reps=5)
    res["host_api"]["eval_batch_cfg3"] = {"s": t, "queries_per_s": ek * ppk / t}
    mark("cfg4")
    # cfg 4: one key logN=32 -> 512 MiB
    al4, s04, s14 = synth.key_seeds(1, 32, first=777)
    k4, _ = dpf.gen_batch_seeded(al4, 32, s04, s14)
    t = med_time(lambda: dpf.evalfull_split(k4[0].tobytes(), 32, 1), reps=3, warm=1)
    res["host_api"]["evalfull_split_cfg4"] = {"s": t, "points_per_s": (1 << 32) / t, "D2H_GBs": (1 << 29) / t / 1e9}
    reuse4 = np.empty(1 << 29, np.uint8)
    t = med_time(lambda: dpf.evalfull_split(k4[0].tobytes(), 32, 1, out=reuse4), reps=3, warm=1)
    res["host_api"]["evalfull_split_cfg4_reused_out"] = {"s": t, "points_per_s": (1 << 32) / t,
                                                         "D2H_GBs": (1 << 29) / t / 1e9}
    mark("cfg5")
    # cfg 5: PIR through the host handle (DB uploaded once)
    pl, B = 24, 64
    db = synth.db_bytes((1 << pl) * 32)
    alp, s0p, s1p = synth.key_seeds(B, pl, first=4242)
    kp, _ = dpf.gen_batch_seeded(alp, pl, s0p, s1p)
    h = dpf.PirDB(db.reshape(-1, 32), pl, ngpus=1)
    t = med_time(lambda: h.answer(kp), reps=9)
    res["host_api"]["pir_answer_cfg5_B64"] = {"s": t, "queries_per_s": B / t}
    del h

    mark("single key")
    # ---- single key (cfg 1), device-resident and host API
    k1 = ka[:1]
    kl = dpf.key_len(logN)
    d_k = torch.from_numpy(k1.reshape(-1)).to(dev)
    d_w = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=dev)
    d_o = torch.empty(dpf.evalfull_len(logN), dtype=torch.uint8, device=dev)

    def dev1():
        dpf.evalfull_batch_dev(d_k, kl, 1, logN, d_o, d_w, stream=st)
        torch.cuda.synchronize()
    t_dev = med_time(dev1, reps=51, warm=5)
    t_host = med_time(lambda: dpf.EvalFull(k1[0].tobytes(), logN), reps=51, warm=5)
    t_eval = med_time(lambda: dpf.Eval(k1[0].tobytes(), 12345, logN), reps=51, warm=5)
    res["single_key_logN20"] = {"evalfull_device_us": t_dev * 1e6, "evalfull_host_api_us": t_host * 1e6,
                                "eval_one_point_host_api_us": t_eval * 1e6}

    mark("pir sweep")
    # ---- PIR batch sweep (device-resident, like bench.py --workload pir)
    d_db = torch.from_numpy(db).to(dev)
    sweep = {}
    for b in (1, 16, 64, 256):
        alb, s0b, s1b = synth.key_seeds(b, pl, first=4242)
        kb, _ = dpf.gen_batch_seeded(alb, pl, s0b, s1b)
        klp = dpf.key_len(pl)
        d_kb = torch.from_numpy(kb.reshape(-1)).to(dev)
        d_ans = torch.empty(b * 32, dtype=torch.uint8, device=dev)
        d_wk = torch.empty(dpf.pir_workspace_size(b, pl, 0), dtype=torch.uint8, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def run(n):
            for _ in range(n):
                dpf.pir_answer_dev(d_kb, klp, b, pl, d_db, 1 << pl, d_ans, d_wk, stream=st)
        run(3)
        reps = max(5, 640 // b)
        e0.record(st)
        run(reps)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        sweep[str(b)] = {"ms_per_batch": ms, "queries_per_s": b / (ms * 1e-3)}
    res["pir_batch_sweep_logN24"] = sweep

    mark("gen")
    # ---- host Gen throughput (logN=20 and 32)
    gen = {}
    for gl in (20, 32):
        n = 1 << 15
        alg, s0g, s1g = synth.key_seeds(n, gl)
        nt = min(16, os.cpu_count() or 1)
        t = med_time(lambda: dpf.gen_batch_seeded(alg, gl, s0g, s1g, nthreads=nt), reps=3, warm=1)
        t1 = med_time(lambda: dpf.gen_batch_seeded(alg[:2048], gl, s0g[:2048], s1g[:2048], nthreads=1), reps=3, warm=1)
        gen[f"logN{gl}"] = {"key_pairs_per_s": n / t, "threads": nt, "key_pairs_per_s_1thread": 2048 / t1}
    res["gen_host"] = gen

    s = json.dumps(res)
    print(s)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
