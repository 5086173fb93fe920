#!/usr/bin/env python3
"""latency.py — device-resident EvalFull time for small key batches (the
latency-bound regime: one key, logN=20 is BASELINE configs[0]'s shape).
Prints one JSON object {"<logN>/<nkeys>": microseconds}; run it under
different DPF_SUBTREE_DEPTH values to map the per-thread subtree depth."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))


def main():
    import torch
    import dpf
    from dpf import synth
    dev = torch.device("cuda", 0)
    dpf.gpu_init(1)
    st = torch.cuda.current_stream(dev)
    res = {"depth": os.environ.get("DPF_SUBTREE_DEPTH", "auto")}
    for logN, nks in ((20, (1, 4, 16, 64, 256, 1024)), (24, (1, 16, 64)), (28, (1,))):
        for nk in nks:
            al, s0, s1 = synth.key_seeds(nk, logN)
            ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1, nthreads=4)
            kl = dpf.key_len(logN)
            d_k = torch.from_numpy(ka.reshape(-1)).to(dev)
            d_w = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
            d_o = torch.empty(nk * dpf.evalfull_len(logN), dtype=torch.uint8, device=dev)
            dpf.expand_keys_dev(d_k, kl, nk, logN, d_w, stream=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                dpf.evalfull_expanded_dev(d_w, nk, logN, d_o, stream=st)
            reps = 20
            e0.record(st)
            for _ in range(reps):
                dpf.evalfull_expanded_dev(d_w, nk, logN, d_o, stream=st)
            e1.record(st)
            torch.cuda.synchronize()
            res[f"{logN}/{nk}"] = round(e0.elapsed_time(e1) / reps * 1e3, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
