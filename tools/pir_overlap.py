"""Can the PIR tree (LDS/VALU-bound) of batch i+1 overlap the fold
(HBM/MFMA-bound) of batch i?  configs[4] shape (64 keys, logN=24, one GPU):
one stream (tree, fold, tree, fold ...) against two streams with the
selection bits double-buffered (fold(i) waits for tree(i); tree(i+2) waits
for fold(i)).  Prints ms per batch for each.  PB=b: an N = 2^b rank's share
(subtree 0 of depth b and its 2^(logN-b)-record DB slice).
  python tools/pir_overlap.py [batches]"""
import os, sys, json, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))
import numpy as np
import torch
import dpf
from dpf import synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dpf.gpu_init_devices([0])
logN, nk = 24, int(os.environ.get("NK", "64"))
pb = int(os.environ.get("PB", "0"))
nrec = 1 << (logN - pb)
kl, per_key = dpf.key_len(logN), dpf.evalfull_len(logN) >> pb
s0_ = torch.cuda.current_stream(dev)
db = torch.from_numpy(synth.db_bytes(nrec * 32)).to(dev)
dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
dpf.pir_db_slice_dev(db, nrec, dbs, device=0, stream=s0_)
torch.cuda.synchronize()
del db
al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
keys = torch.from_numpy(ka.reshape(-1)).to(dev)
bits = [torch.empty(nk * per_key, dtype=torch.uint8, device=dev) for _ in range(2)]
work = [torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev) for _ in range(2)]
fw = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=dev)
ans = [torch.empty(nk * 32, dtype=torch.uint8, device=dev) for _ in range(2)]
lo_p, hi_p = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, 0)
prio = os.environ.get("FOLD_PRIO", "0") == "1"
sA = torch.cuda.Stream(dev)
sB = torch.cuda.Stream(dev, priority=-1) if prio else torch.cuda.Stream(dev)


def tree(i, st):
    dpf.evalfull_subtree_dev(keys, kl, nk, logN, pb, 0, bits[i % 2], work[i % 2], device=0, stream=st)


def fold(i, st):
    dpf.xor_fold_sliced_dev(bits[i % 2], per_key, nk, dbs, nrec, ans[i % 2], fw, device=0, stream=st)


def seq(m):
    for i in range(m):
        tree(i, sA)
        fold(i, sA)


def pipe(m):
    eT = [torch.cuda.Event() for _ in range(m)]
    eF = [torch.cuda.Event() for _ in range(m)]
    for i in range(m):
        if i >= 2:
            sA.wait_event(eF[i - 2])
        tree(i, sA)
        eT[i].record(sA)
        sB.wait_event(eT[i])
        fold(i, sB)
        eF[i].record(sB)
    sA.wait_stream(sB)


def timeit(fn, m):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(m)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / m * 1e3


for _ in range(3):
    seq(100); pipe(100)
out = {"seq": [], "pipe": []}
for r in range(3):
    out["seq"].append(round(timeit(seq, n), 4))
    out["pipe"].append(round(timeit(pipe, n), 4))
    print(r, out["seq"][-1], out["pipe"][-1], flush=True)
# parity: the pipelined answers equal the sequential ones
seq(2); torch.cuda.synchronize(); a0 = [x.clone() for x in ans]
pipe(2); torch.cuda.synchronize()
out["same_answers"] = all(torch.equal(a, b) for a, b in zip(a0, ans))
out["nk"], out["fold_priority"], out["prefix_bits"] = nk, prio, pb
print(json.dumps(out))
