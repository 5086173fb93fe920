"""Why is the PIR tree slower right after the fold (bench `kernels.back_to_back`:
0.29 vs 0.255 ms alone)?  Times the configs[4] tree (64 keys, logN=24) after
each kind of predecessor: itself, the MFMA fold, an HBM copy of the same size
as the fold's reads, and a spin kernel of the fold's duration.
  python tools/pir_seq.py [reps]"""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))
import numpy as np
import torch
import dpf
from dpf import synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dpf.gpu_init_devices([0])
st = torch.cuda.current_stream(dev)
logN, nk = 24, 64
nrec = 1 << logN
kl, per_key = dpf.key_len(logN), dpf.evalfull_len(logN)
db = torch.from_numpy(synth.db_bytes(nrec * 32)).to(dev)
dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
dpf.pir_db_slice_dev(db, nrec, dbs, device=0, stream=st)
al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
keys = torch.from_numpy(ka.reshape(-1)).to(dev)
bits = torch.empty(nk * per_key, dtype=torch.uint8, device=dev)
work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
fw = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
src = torch.empty(nrec * 32 // 2, dtype=torch.uint8, device=dev)    # 256 MiB read + 256 MiB write
dst = torch.empty_like(src)


def tree():
    dpf.evalfull_subtree_dev(keys, kl, nk, logN, 0, 0, bits, work, device=0, stream=st)


def fold():
    dpf.xor_fold_sliced_dev(bits, per_key, nk, dbs, nrec, ans, fw, device=0, stream=st)


def copy():
    dst.copy_(src)


def spin():
    torch.cuda._sleep(int(os.environ.get("SPIN_CYCLES", "300000")))


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record(st)
    return e


def run(pred, n):
    """n rounds of (pred, tree); returns (pred ms, tree ms) means."""
    es = []
    for _ in range(n):
        a = ev(); pred(); b = ev(); tree(); c = ev()
        es.append((a, b, c))
    torch.cuda.synchronize()
    p = [a.elapsed_time(b) for a, b, c in es]
    t = [b.elapsed_time(c) for a, b, c in es]
    return float(np.mean(p)), float(np.mean(t)), float(np.min(t))


for _ in range(200):                 # clock spin-up
    tree()
torch.cuda.synchronize()
out = {}
for rnd in range(3):
    for name, pred in (("tree", tree), ("fold", fold), ("copy", copy), ("spin", spin)):
        p, t, tmin = run(pred, reps)
        out.setdefault(name, []).append({"pred_ms": round(p, 4), "tree_ms": round(t, 4), "tree_min_ms": round(tmin, 4)})
        print(rnd, name, round(p, 4), round(t, 4), round(tmin, 4), flush=True)
print(json.dumps(out))
