"""r06 microbenchmark (VERDICT r05 "Next" #3): latency of one dependent
AES-128-MMO step on an otherwise idle GPU, T-table (LDS lookups) against the
table-free byte-sliced circuit (VALU only, 8 blocks per lane in registers).

The shared root-to-subtree walk of the small per-rank tree shapes (DESIGN
§4.2) is a chain of dependent MMOs on 64 paths while the CU idles, so what
matters there is the latency of one step, not throughput.  The 64 paths fit
  - T-table: one wave (64 lanes x 2 blocks per lane in k_mmo_tt);
  - byte-sliced: 8 lanes x 8 blocks (k_mmo_bs), or a full wave (512 blocks).
Each shape runs `reps` chained MMOs per block (dpf_aes_mmo_dev); the slope
between two rep counts is the time per dependent step.  One JSON line.

Reference: aes128MMO /root/reference/dpf/aes_amd64.s:50-82; the walk
/root/reference/dpf/dpf.go:183-201 (one MMO per level on the path).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))
import dpf  # noqa: E402
import torch  # noqa: E402

dpf.gpu_init(1)
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
out = {}
shapes = (("ttable_one_wave_64x2", dpf.AES_TTABLE, 128),
          ("bytesliced_8_lanes_x8", dpf.AES_BITSLICED, 64),
          ("bytesliced_one_wave_64x8", dpf.AES_BITSLICED, 512),
          ("ttable_chip", dpf.AES_TTABLE, 256 * 2048),
          ("bytesliced_chip", dpf.AES_BITSLICED, 256 * 4096))
for name, impl, nblocks in shapes:
    d_in = torch.randint(0, 256, (nblocks * 16,), dtype=torch.uint8, device=dev)
    d_out = torch.empty_like(d_in)
    res = {}
    lo, hi = (50, 100) if "chip" in name else (200, 400)
    for reps in (lo, hi):
        for _ in range(3):
            dpf.aes_mmo_dev(d_in, d_out, nblocks, impl=impl, reps=reps, stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            dpf.aes_mmo_dev(d_in, d_out, nblocks, impl=impl, reps=reps, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        res[reps] = e0.elapsed_time(e1) / 10 * 1e3     # us per launch
    per = (res[hi] - res[lo]) / (hi - lo)
    out[name] = {"blocks": nblocks, "us_per_dependent_mmo_step": round(per, 4),
                 "blocks_per_s_G": round(nblocks / (per * 1e-6) / 1e9, 2)}
    print(name, out[name], flush=True)
# bit-exactness of the two back ends on the same input
d_in = torch.randint(0, 256, (512 * 16,), dtype=torch.uint8, device=dev)
a, b = torch.empty_like(d_in), torch.empty_like(d_in)
dpf.aes_mmo_dev(d_in, a, 512, impl=dpf.AES_TTABLE, reps=3, stream=st)
dpf.aes_mmo_dev(d_in, b, 512, impl=dpf.AES_BITSLICED, reps=3, stream=st)
torch.cuda.synchronize()
out["back_ends_identical"] = bool(torch.equal(a, b))
print(json.dumps(out))
