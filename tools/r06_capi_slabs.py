#!/usr/bin/env python3
"""The drop-in single-key C ABI (dpf_evalfull, host output) at the
reference's own shapes -- BenchmarkEvalFull logN 28 (dpf/dpf_test.go:7-21)
and dpf_main.go's logN 27 -- into a reused and a fresh host buffer, medians
of 31 calls, as bench.py's reference_shapes times it.  Run once per library
(DPF_LIB=...) to compare slab sizes (DPF_SLAB_BYTES builds).
Usage: python tools/r06_capi_slabs.py [tag]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))

import numpy as np  # noqa: E402

import dpf  # noqa: E402


def main() -> None:
    tag = sys.argv[1] if len(sys.argv) > 1 else "product"
    dpf.gpu_init(1)
    L = dpf.lib()
    res = {"lib": tag}
    for logN, alpha in ((28, 0), (27, 123)):
        s0 = np.frombuffer(bytes(range(1, 17)), np.uint8)[None]
        s1 = np.frombuffer(bytes(range(17, 33)), np.uint8)[None]
        ka, _ = dpf.gen_batch_seeded(np.array([alpha], np.uint64), logN, s0, s1)
        kk = ka[0].copy()
        nbytes = dpf.evalfull_len(logN)
        reused = np.empty(nbytes, np.uint8)

        def capi(buf):
            rc = L.dpf_evalfull(dpf._buf(kk), kk.size, logN, dpf._buf(buf))
            assert rc == 0, rc

        def med_ms(f, n=31):
            f()
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                f()
                ts.append(time.perf_counter() - t0)
            return round(float(np.median(ts)) * 1e3, 4)

        res[f"logN{logN}"] = {"reused_ms": med_ms(lambda: capi(reused)),
                              "fresh_ms": med_ms(lambda: capi(np.empty(nbytes, np.uint8)))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
