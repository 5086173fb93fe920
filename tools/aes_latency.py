"""Latency of one dependent AES-128-MMO step of the T-table back end on a
lightly loaded GPU (one wave: 64 lanes x 2 blocks, `reps` chained MMOs per
block through dpf_aes_mmo_dev) against the loaded chip (every CU full), to
price the serial root-to-subtree walks of the small per-rank tree shapes
(DESIGN.md §7).  One JSON line."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/dpf-go_amd")
import dpf  # noqa: E402
import torch  # noqa: E402

dpf.gpu_init(1)
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
out = {}
for name, nblocks in (("one_wave", 128), ("one_wg", 1024), ("one_cu_2wg", 2048 * 1), ("chip", 256 * 2048)):
    d_in = torch.randint(0, 256, (nblocks * 16,), dtype=torch.uint8, device=dev)
    d_out = torch.empty_like(d_in)
    res = {}
    for reps in (200, 400):
        for _ in range(3):
            dpf.aes_mmo_dev(d_in, d_out, nblocks, reps=reps, stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            dpf.aes_mmo_dev(d_in, d_out, nblocks, reps=reps, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        res[reps] = e0.elapsed_time(e1) / 10 * 1e3     # us per launch
    per = (res[400] - res[200]) / 200
    out[name] = {"blocks": nblocks, "us_per_dependent_mmo_pair_step": round(per, 4),
                 "blocks_per_s_G": round(nblocks / (per * 1e-6) / 1e9, 2)}
print(json.dumps(out))
