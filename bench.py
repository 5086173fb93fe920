#!/usr/bin/env python3
"""bench.py — DPF evaluation throughput on MI355X (driver contract).

A "step" is one batched EvalFull of BASELINE.json configs[1]: 4096 keys x
logN=20 (2^32 leaf points, 100,655,104 AES-128-MMO blocks), keys already
resident in HBM, output left in HBM.  With --gpus N each rank (one process
per GPU, launched by torch.distributed.run) evaluates its own 4096 keys:
weak scaling, no collective on the data path; value = points of all ranks /
max-over-ranks time.

Rank 0 prints ONE JSON line with the metric, a "roofline" object for the
tree kernel (integer VALU bound, timed with HIP events on the launch
stream), and a "cpu_baseline" object (the oracle's reference-faithful C
restatement on AES-NI, timed on a bounded sample on this host).

Other workloads (--workload eval|split|pir) are parity-test / secondary
measurements, reported on separate lines only when asked for.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dpf-go_amd"))

import numpy as np  # noqa: E402

# Per-unit algorithmic figures.
GATES_PER_AES = 22928          # 2-input gate-equivalents per AES-128-MMO block
# Override of the measured v_bitop3_b32 rate (Tops), else profiles/r01_valu_peak.json.
VALU_PEAK_TOPS = float(os.environ.get("DPF_VALU_PEAK_TOPS", "0") or 0) or None
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md (spec)


def stop_of(logN: int) -> int:
    return logN - 7 if logN >= 7 else 0


def aes_full(logN: int) -> int:
    s = stop_of(logN)
    return 3 * (1 << s) - 2 if s > 0 else 1


def load_peaks() -> dict:
    """Measured MI355X rates (tools/valu_peak.hip -> profiles/r01_valu_peak.json)."""
    p = os.path.join(ROOT, "profiles", "r01_valu_peak.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception:
        d = {}
    return {"bitop3_Tops": float(VALU_PEAK_TOPS or d.get("v_bitop3_b32_Tops", 59.7)),
            "lds_lookups_Gs": float(d.get("ds_read_b32_lookup_G_per_s", 16438.3))}


def cpu_baseline(logN: int, target_s: float = 10.0) -> dict:
    """Oracle (reference-faithful C restatement: AES-NI, one block per call,
    DFS, dpf.go:213-262) on this host's cores, over a bounded sample: passes
    over one fixed set of keys until about target_s seconds have elapsed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from dpf import synth
    import dpf

    cores = min(16, os.cpu_count() or 1)
    n = cores * 16
    al, s0, s1 = synth.key_seeds(n, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    oracle.evalfull_batch(ka[:cores], logN, nthreads=cores, aesni=True)   # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        oracle.evalfull_batch(ka, logN, nthreads=cores, aesni=True)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= target_s:
            break
    keys = n * passes
    pts = keys * (1 << logN)
    return {"value": pts / dt, "unit": "points/s", "cores": cores, "kind": "port",
            "aes_blocks_per_s": keys * aes_full(logN) / dt,
            "sample": f"{keys} key-EvalFulls at logN={logN} ({passes} passes over {n} keys, {dt:.1f} s, "
                      f"{cores} threads, AES-NI one block per call; oracle/dpf_oracle.c)"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--logN", type=int, default=20)
    ap.add_argument("--nkeys", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--check", action="store_true", help="verify a sample of outputs against the oracle")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import dpf
    from dpf import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dpf.gpu_init(0)

    logN, nk = args.logN, args.nkeys
    kl = dpf.key_len(logN)
    olen = dpf.evalfull_len(logN)
    # Each rank its own synthetic keys (keys rank*nk ..), generated on the host.
    al, s0, s1 = synth.key_seeds(nk, logN, first=rank * nk)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(dev)
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=dev)
    d_out = torch.empty(nk * olen, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work, device=local, stream=stream)
        dpf.evalfull_expanded_dev(d_work, nk, logN, d_out, device=local, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([t_wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_wall = float(t.item())

    # Tree-kernel-only timing with HIP events on the launch stream.
    dpf.expand_keys_dev(d_keys, kl, nk, logN, d_work, device=local, stream=stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = max(3, min(args.steps, 20))
    ev[0].record(stream)
    for _ in range(reps):
        dpf.evalfull_expanded_dev(d_work, nk, logN, d_out, device=local, stream=stream)
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    k_ms = ev[0].elapsed_time(ev[1]) / reps

    if args.check and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        idx = np.unique(np.linspace(0, nk - 1, 8).astype(int))
        got = d_out.view(nk, olen)[torch.from_numpy(idx).to(dev)].cpu().numpy()
        want = oracle.evalfull_batch(ka[idx], logN, nthreads=8)
        assert np.array_equal(got, want), "bench output differs from oracle"

    pts_per_step = nk * (1 << logN) * world
    aes_per_step = nk * aes_full(logN) * world
    ms_per_step = t_wall / args.steps * 1e3
    value = pts_per_step / (t_wall / args.steps)

    aes_per_launch = nk * aes_full(logN)
    aes_rate = aes_per_launch / (k_ms * 1e-3)
    peaks = load_peaks()
    # PRG roofline: 22,928 two-input gate-equivalents per AES-MMO
    # block; ceiling = measured v_bitop3_b32 lane-op rate x 32 bit-lanes x 2
    # gates per bitop3 (the stricter, bitop3 denominator).
    achieved = aes_rate * GATES_PER_AES / 1e12
    peak = peaks["bitop3_Tops"] * 32 * 2
    bytes_per_launch = nk * olen + nk * (stop_of(logN) + 2) * 32
    roofline = {
        "bound": "valu",
        "achieved": round(achieved, 1),
        "peak": round(peak, 1),
        "unit": "Tgate/s (2-input gate-equivalents; 22,928 per AES-128-MMO block)",
        "frac": round(achieved / peak, 4),
        "traffic": None,
        "kernel": f"k_evalfull<{min(stop_of(logN), 7)},true>",
        "kernel_ms": round(k_ms, 4),
        "aes_blocks_per_s": aes_rate,
        "lds_lookup_frac": round(aes_rate * 160 / (peaks["lds_lookups_Gs"] * 1e9), 4),
        "hbm_write_GBs": round(bytes_per_launch / (k_ms * 1e-3) / 1e9, 1),
        "hbm_frac": round(bytes_per_launch / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
    }
    tr_env = os.environ.get("DPF_TRAFFIC_BYTES")
    if tr_env:
        roofline["traffic"] = float(tr_env)

    if rank == 0:
        line = {
            "metric": "DPF leaf points/sec (EvalFull logN=20, batched keys) + AES blocks/sec",
            "value": value,
            "unit": "points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SplitMix64 seed 0x5EEDD9F0 keys via host Gen)",
            "config": {"workload": f"batched EvalFull, {nk} keys x logN={logN} per GPU (BASELINE configs[1])",
                       "keys_per_gpu": nk, "logN": logN, "aes": "lds-ttable",
                       "parallelism": f"key-shard x{world}"},
            "aes_blocks_per_s": aes_per_step / (t_wall / args.steps),
            "roofline": roofline,
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(logN, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
