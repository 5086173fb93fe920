"""Is the PIR step launch-bound at the per-rank shapes?  One step (the
sliced PIR answer: tree, fold, partial XOR; then the 2 KiB answer copy to
pinned host memory) issued eagerly from Python against the same step
captured once in a HIP graph and replayed.  PB=b: an N = 2^b rank's share
(subtree 0 and its DB slice).  Prints ms per step for each and whether the
graph's answers equal the eager ones.
  PB=3 python tools/pir_graph.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))
import torch  # noqa: E402
import dpf  # noqa: E402
from dpf import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dpf.gpu_init_devices([0])
logN, nk = 24, int(os.environ.get("NK", "64"))
pb = int(os.environ.get("PB", "3"))
nrec = 1 << (logN - pb)
kl = dpf.key_len(logN)
st = torch.cuda.Stream(dev)
db = torch.from_numpy(synth.db_bytes(nrec * 32)).to(dev)
dbs = torch.empty(dpf.pir_db_sliced_size(nrec), dtype=torch.uint8, device=dev)
dpf.pir_db_slice_dev(db, nrec, dbs, device=0, stream=st)
torch.cuda.synchronize()
del db
al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
keys = torch.from_numpy(ka.reshape(-1)).to(dev)
ans = torch.empty(nk * 32, dtype=torch.uint8, device=dev)
work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=dev)
host = torch.empty(nk * 32, dtype=torch.uint8, pin_memory=True)


def step(s):
    dpf.pir_answer_sliced_dev(keys, kl, nk, logN, dbs, nrec, ans, work, prefix_bits=pb, prefix=0, device=0, stream=s)
    with torch.cuda.stream(s):
        host.copy_(ans, non_blocking=True)


def eager(m):
    for _ in range(m):
        step(st)


with torch.cuda.stream(st):
    for _ in range(20):
        step(st)                    # lazy library state (occupancy queries, workspace registry) before capture
torch.cuda.synchronize()
want = host.clone()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    step(torch.cuda.current_stream())


def graph(m):
    for _ in range(m):
        g.replay()


def timeit(fn, m):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(m)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / m * 1e3


for _ in range(3):
    eager(200)
    graph(200)
out = {"eager": [], "graph": []}
for r in range(3):
    out["eager"].append(round(timeit(eager, n), 4))
    out["graph"].append(round(timeit(graph, n), 4))
    print(r, out["eager"][-1], out["graph"][-1], flush=True)
host.zero_()
g.replay()
torch.cuda.synchronize()
out["same_answers"] = bool(torch.equal(host, want))
out["prefix_bits"], out["nk"] = pb, nk
print(json.dumps(out))
