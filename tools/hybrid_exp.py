#!/usr/bin/env python3
"""Co-scheduling experiment for configs[1]: the byte-sliced tree kernel
(VALU-bound, 1 workgroup/CU via the LDS-padded variant) and the T-table tree
kernel (LDS-bound) on two streams over disjoint key ranges, so both
pipes of every CU are busy.  Sweeps the byte-sliced share; prints JSON.
Usage: DPF_LIB=dpf-go_amd/lib/variants/libdpf_hip_bspad.so tools/hybrid_exp.py"""
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
    logN, nk = 20, 4096
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    al, s0, s1 = synth.key_seeds(nk, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_out = torch.empty(nk * ol, dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ref = None
    res = {}
    for nbs in [0, 1024, 1536, 1792, 2048, 2304, 2560, 4096]:
        ntt = nk - nbs
        wa = torch.empty(dpf.workspace_size(max(nbs, 1), logN), dtype=torch.uint8, device=dev)
        wb = torch.empty(dpf.workspace_size(max(ntt, 1), logN), dtype=torch.uint8, device=dev)
        if nbs:
            dpf.expand_keys_dev(d_keys[: nbs * kl], kl, nbs, logN, wa, stream=sa)
        if ntt:
            dpf.expand_keys_dev(d_keys[nbs * kl:], kl, ntt, logN, wb, stream=sb)
        torch.cuda.synchronize()

        def step():
            e = torch.cuda.Event()
            e.record(torch.cuda.current_stream(dev))
            sa.wait_event(e)
            sb.wait_event(e)
            if nbs:
                dpf.set_aes_impl("bitsliced")
                dpf.evalfull_expanded_dev(wa, nbs, logN, d_out[: nbs * ol], stream=sa)
            if ntt:
                dpf.set_aes_impl("ttable")
                dpf.evalfull_expanded_dev(wb, ntt, logN, d_out[nbs * ol:], stream=sb)
            ea, eb = torch.cuda.Event(), torch.cuda.Event()
            ea.record(sa)
            eb.record(sb)
            torch.cuda.current_stream(dev).wait_event(ea)
            torch.cuda.current_stream(dev).wait_event(eb)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(10):
            step()
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / 10
        h = d_out.view(nk, ol)[::97].clone()
        if ref is None:
            ref = h
        res[nbs] = {"ms": round(ms, 4), "G_blocks_per_s": round(nk * 24574 / (ms * 1e-3) / 1e9, 2),
                    "same_output": bool(torch.equal(ref, h))}
        print(nbs, res[nbs], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
