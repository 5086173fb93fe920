#!/usr/bin/env python3
"""AES-128-MMO blocks/s of both back ends through dpf_aes_mmo_dev (the
'AES blocks/sec' half of BASELINE's metric): N blocks resident in HBM, each
iterated `reps` times in registers (out = MMO^reps(in)), timed with HIP
events on the launch stream.  Prints one JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))


def main():
    import torch
    import dpf
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, reps = 1 << 22, 32
    d_in = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device=dev)
    d_out = torch.empty_like(d_in)
    res = {"blocks": n, "reps": reps}
    outs = {}
    for name, impl in (("lds-ttable", dpf.AES_TTABLE), ("bitsliced", dpf.AES_BITSLICED)):
        for _ in range(3):
            dpf.aes_mmo_dev(d_in, d_out, n, impl=impl, reps=reps, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            dpf.aes_mmo_dev(d_in, d_out, n, impl=impl, reps=reps, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        res[name] = {"ms": ms, "G_blocks_per_s": n * reps / (ms * 1e-3) / 1e9}
        outs[name] = d_out.clone()
    res["identical"] = bool(torch.equal(outs["lds-ttable"], outs["bitsliced"]))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
