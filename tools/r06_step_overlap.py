#!/usr/bin/env python3
"""Does a configs[1] launch lose its tail?  Per 4096-key batch, ms:
  one     -- K launches back to back on one stream (bench.py's step);
  two     -- K launches alternating over two streams (own output + workspace
             each), so one batch's last waves can overlap the next's first;
  double  -- K/2 launches of 8192 keys (two batches in one grid).
Each mode after a 0.5 s spin-up; modes interleaved for R rounds.
Usage: python tools/r06_step_overlap.py [rounds] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dpf  # noqa: E402
from dpf import synth  # noqa: E402


def main() -> None:
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    dpf.gpu_init_devices([0])
    dev = torch.device("cuda", 0)
    logN, nk = 20, 4096
    kl, olen = dpf.key_len(logN), dpf.evalfull_len(logN)
    al, s0, s1 = synth.key_seeds(2 * nk, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    outs = [torch.empty(2 * nk * olen, dtype=torch.uint8, device=dev) for _ in range(2)]
    works = [torch.empty(dpf.workspace_size(2 * nk, logN), dtype=torch.uint8, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    main_st = torch.cuda.current_stream(dev)

    def launch(i, n, st):
        dpf.evalfull_batch_dev(d_keys[(i % 2) * nk * kl:], kl, n, logN, outs[i % 2], works[i % 2], device=0,
                               stream=st)

    def run(mode, steps):
        if mode == "one":
            for i in range(steps):
                launch(0, nk, main_st)
        elif mode == "two":
            for i in range(steps):
                launch(i, nk, streams[i % 2])
        else:
            for i in range(steps // 2):
                dpf.evalfull_batch_dev(d_keys, kl, 2 * nk, logN, outs[0], works[0], device=0, stream=main_st)
        torch.cuda.synchronize(dev)

    ref = None
    for r in range(R):
        for mode in ("one", "two", "double"):
            t = time.perf_counter()
            while time.perf_counter() - t < 0.5:
                run(mode, 8)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            run(mode, K)
            ms = (time.perf_counter() - t0) / K * 1e3
            print(f"{r} {mode} {ms:.4f} ms per 4096-key batch = {nk * (1 << logN) / ms * 1e3 / 1e12:.4f} T points/s",
                  flush=True)
    # the three modes write the same bytes for batch 0
    run("one", 1)
    a = outs[0][:nk * olen].clone()
    run("two", 2)
    run("double", 2)
    ref = outs[0][:nk * olen]
    print("batch 0 identical across modes:", bool(torch.equal(a, ref)))


if __name__ == "__main__":
    main()
