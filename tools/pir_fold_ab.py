"""configs[4] PIR step, matrix-core fold (bit-sliced DB) vs LDS fold (row-major
DB), alternated in one process so clock drift cancels: R rounds of K steps of
each, wall time between synchronizes, plus per-phase kernel times.
Usage: python tools/pir_fold_ab.py [batch] [rounds] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dpf-go_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import dpf  # noqa: E402
from dpf import synth  # noqa: E402


def main():
    nk = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    logN = 24
    nrec = 1 << logN
    dev = torch.device("cuda", 0)
    dpf.gpu_init_devices([0])
    st = torch.cuda.current_stream(dev)
    db = synth.db_bytes(nrec * 32)
    d_db = torch.from_numpy(db).to(dev)
    d_dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
    dpf.pir_db_slice_dev(d_db, nrec, d_dbs, stream=st)
    al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    kl = dpf.key_len(logN)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN), dtype=torch.uint8, device=dev)
    ans = {m: torch.empty(nk * 32, dtype=torch.uint8, device=dev) for m in ("mfma", "lds")}

    def step(m):
        if m == "mfma":
            dpf.pir_answer_sliced_dev(d_keys, kl, nk, logN, d_dbs, nrec, ans[m], d_work, stream=st)
        else:
            dpf.pir_answer_dev(d_keys, kl, nk, logN, d_db, nrec, ans[m], d_work, stream=st)

    t_end = time.perf_counter() + 1.0                     # clock spin-up
    while time.perf_counter() < t_end:
        for m in ("mfma", "lds"):
            step(m)
        torch.cuda.synchronize()
    assert torch.equal(ans["mfma"], ans["lds"])
    res = {"mfma": [], "lds": []}
    for r in range(rounds):
        for m in (("mfma", "lds") if r % 2 == 0 else ("lds", "mfma")):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step(m)
            torch.cuda.synchronize()
            res[m].append((time.perf_counter() - t0) / steps * 1e3)
    for m, v in res.items():
        print(f"{m}: ms/step median {np.median(v):.4f}  all {[round(x, 4) for x in v]}")


if __name__ == "__main__":
    main()
