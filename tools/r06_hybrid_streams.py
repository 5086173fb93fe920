"""r06 measurement (VERDICT r05 "Next" #5): can configs[1] get a second
resource?  The LDS T-table tree kernel leaves VALU issue slots idle; the
byte-sliced back end is VALU-only.  Here configs[1]'s 4096 keys are split
between the two back ends running at the same time:

  - co-resident: two plain streams, T-table on keys [0, n_t), byte-sliced on
    [n_t, 4096) -- the hardware dispatcher mixes their workgroups on CUs;
  - CU-partitioned: the same on two CU-masked streams (dpf_stream_create_
    cu_masked), T-table on CUs [c, 256), byte-sliced on [0, c).

against each back end alone on the whole batch.  Every form is checked to
give the same bytes as the T-table alone.  One JSON line per round.

  python tools/r06_hybrid_streams.py [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dpf-go_amd")]

import torch  # noqa: E402

import dpf  # noqa: E402
from dpf import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    assert dpf.gpu_init(1) >= 1
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    logN, nk = 20, 4096
    al, s0, s1 = synth.key_seeds(nk, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    kl, ol = dpf.key_len(logN), dpf.evalfull_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_out = torch.empty(nk * ol, dtype=torch.uint8, device=dev)
    w = [torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev) for _ in range(2)]
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def launch(impl, k0, k1, st, wi):
        dpf.set_aes_impl(impl)
        dpf.evalfull_batch_dev(d_keys[k0 * kl:], kl, k1 - k0, logN, d_out[k0 * ol:], w[wi], stream=st)

    def timed(fn, steps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def alone(impl):
        return lambda: launch(impl, 0, nk, sA, 0)

    def split(n_t, T, B):
        def f():
            launch("ttable", 0, n_t, T, 0)
            launch("bitsliced", n_t, nk, B, 1)
        return f

    t_end = time.time() + 0.6
    while time.time() < t_end:
        timed(alone("ttable"), 5)
    ref = d_out.clone()
    masked = {c: (dpf.stream_create_cu_masked(c, ncu - c), dpf.stream_create_cu_masked(0, c)) for c in (32, 64)}
    for r in range(a.rounds):
        row = {"ttable_alone": timed(alone("ttable"), a.steps), "bitsliced_alone": timed(alone("bitsliced"), a.steps)}
        for n_t in (3584, 3072, 2048):
            d_out.zero_()
            row[f"coresident_tt{n_t}"] = timed(split(n_t, sA, sB), a.steps)
            assert torch.equal(d_out, ref), n_t
        for c, (T, B) in masked.items():
            n_t = nk * (ncu - c) * 107 // ((ncu - c) * 107 + c * 87) // 64 * 64   # by per-CU rate
            d_out.zero_()
            row[f"cumask_bs{c}cu_tt{n_t}"] = timed(split(n_t, T, B), a.steps)
            assert torch.equal(d_out, ref), c
        row = {k: round(v, 4) for k, v in row.items()}
        print(json.dumps(row), flush=True)
    dpf.set_aes_impl("ttable")
    torch.cuda.synchronize()
    for T, B in masked.values():
        dpf.stream_destroy(T)
        dpf.stream_destroy(B)
    print("done", flush=True)


if __name__ == "__main__":
    main()
