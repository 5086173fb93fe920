#!/usr/bin/env python3
"""api_diag.py — where the time of a host-buffer EvalFull into a FRESH array
goes (configs[1]: 4096 keys x logN=20 -> 512 MiB): allocation, the call, the
free, and the same call into a pre-touched / reused array.  Measurement only."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))

import numpy as np  # noqa: E402


def rd(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return str(e)


def main():
    import dpf
    from dpf import synth
    dpf.gpu_init(1)
    logN, nk = 20, 4096
    al, s0, s1 = synth.key_seeds(nk, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    shape = (nk, dpf.evalfull_len(logN))
    res = {"thp_enabled": rd("/sys/kernel/mm/transparent_hugepage/enabled"),
           "thp_defrag": rd("/sys/kernel/mm/transparent_hugepage/defrag"),
           "cpu_max": rd("/sys/fs/cgroup/cpu.max"), "fresh": [], "touched": [], "reused": []}
    reuse = np.empty(shape, np.uint8)
    for _ in range(3):
        dpf.evalfull_batch(ka, logN, ngpus=1, out=reuse)
    for _ in range(5):
        t0 = time.perf_counter()
        out = np.empty(shape, np.uint8)
        t1 = time.perf_counter()
        dpf.evalfull_batch(ka, logN, ngpus=1, out=out)
        t2 = time.perf_counter()
        del out
        t3 = time.perf_counter()
        res["fresh"].append({"alloc_ms": (t1 - t0) * 1e3, "call_ms": (t2 - t1) * 1e3, "free_ms": (t3 - t2) * 1e3})
    for _ in range(5):
        out = np.empty(shape, np.uint8)
        t0 = time.perf_counter()
        out.fill(0)
        t1 = time.perf_counter()
        dpf.evalfull_batch(ka, logN, ngpus=1, out=out)
        t2 = time.perf_counter()
        res["touched"].append({"touch_ms": (t1 - t0) * 1e3, "call_ms": (t2 - t1) * 1e3})
        del out
    for _ in range(5):
        t0 = time.perf_counter()
        dpf.evalfull_batch(ka, logN, ngpus=1, out=reuse)
        res["reused"].append({"call_ms": (time.perf_counter() - t0) * 1e3})
    print(json.dumps(res))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
