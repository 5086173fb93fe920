#!/usr/bin/env python3
"""Single-call latency of the drop-in API (dpf_eval / dpf_evalfull, one key)
through the host small-call path, the GPU path, and the reference-style CPU
restatement (oracle/dpf_oracle.c on AES-NI, one aes128MMO per call, like
dpf.go:171-262), median of N calls per logN.  One JSON object on stdout:
where the host path beats the GPU round trip sets kSmallFullMaxLogN
(dpf_capi.hip)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dpf-go_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import dpf  # noqa: E402
from dpf import synth  # noqa: E402
import oracle  # noqa: E402


def med(f, n):
    f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    assert dpf.gpu_init(1) >= 1
    res = {"evalfull": {}, "eval": {}}
    for logN in (8, 10, 12, 14, 16, 18, 20, 21, 22, 24):
        al, s0, s1 = synth.key_seeds(1, logN, first=3)
        ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
        k = ka[0].tobytes()
        n = 31 if logN <= 20 else 9
        row = {}
        for mode in ("host", "gpu"):
            dpf.set_small_call_path(mode)
            row[mode + "_ms"] = round(med(lambda: dpf.EvalFull(k, logN), n) * 1e3, 4)
        row["ref_style_cpu_ms"] = round(med(lambda: oracle.evalfull(k, logN, aesni=True), min(n, 9)) * 1e3, 4)
        res["evalfull"][str(logN)] = row
        x = int(synth.eval_points(1, 1, logN)[0][0])
        erow = {}
        for mode in ("host", "gpu"):
            dpf.set_small_call_path(mode)
            erow[mode + "_us"] = round(med(lambda: dpf.Eval(k, x, logN), 201) * 1e6, 2)
        erow["ref_style_cpu_us"] = round(med(lambda: oracle.eval_(k, x, logN, aesni=True), 201) * 1e6, 2)
        res["eval"][str(logN)] = erow
    dpf.set_small_call_path("auto")
    res["auto_max_logN"] = dpf.small_call_max_logN()
    res["host_isa"] = os.environ.get("DPF_HOST_ISA", "auto")
    # Largest logN whose host EvalFull beats the GPU round trip (the AUTO
    # threshold this host ISA should have).
    wins = [int(n) for n, r in res["evalfull"].items() if r["host_ms"] < r["gpu_ms"]]
    res["measured_crossover_logN"] = max(wins) if wins else None
    print(json.dumps(res))


if __name__ == "__main__":
    main()
