#!/usr/bin/env python3
"""bench.py — DPF evaluation throughput on MI355X (driver contract).

Default workload (the headline, BASELINE.json configs[1]): a "step" is one
batched EvalFull of 4096 keys x logN=20 (2^32 leaf points, 100,655,104
AES-128-MMO blocks) with keys already resident in HBM and the output left in
HBM.  With --gpus N each rank (one process per GPU, torch.distributed.run)
evaluates its own 4096 keys: weak scaling, no collective on the data path;
value = points of all ranks / max-over-ranks time.

Rank 0 prints ONE JSON line: the metric, a "roofline" object for the tree
kernel (integer-VALU bound; its time from HIP events recorded on the launch
stream around every k_evalfull of the timed steps), and a "cpu_baseline"
object (the oracle's reference-faithful C restatement on AES-NI, timed on a
bounded sample on this host).

Secondary workloads (--workload), each its own JSON line:
  eval   configs[2]: 2^16 keys x 2^10 random points, logN=20 per GPU (weak)
  split  configs[3]: ONE key, logN=32, split by top-level subtree (strong)
  pir    configs[4]: 2-server PIR answer, logN=24, DB 2^24 x 32 B sharded
         over the GPUs, B queries (--batch), partials all-gathered + host XOR
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
LOOKUPS_PER_AES = 160          # T-table back end: 16 LDS lookups per round x 10 rounds
# Peaks from /opt/skills/guides/MI355X_MICROARCH.md (chip parameters):
#   VALU issue: 256 CU x 4 SIMD-32 x 32 lanes/clk x 2.4 GHz = 78.64 T lane-ops/s;
#   a v_bitop3_b32 lane-op evaluates 32 bit-lanes x up to 2 two-input gates
#   -> 5033 T gate-eq/s, the PRG roofline's denominator;
#   LDS: ds_read_b32 aggregate ~75 TB/s -> 18.75 T 4-byte lookups/s;
#   HBM: 8 TB/s (spec).
GUIDE_VALU_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
GUIDE_GATE_PEAK_T = GUIDE_VALU_TOPS * 32 * 2
GUIDE_LDS_LOOKUPS_T = 75e12 / 4 / 1e12
HBM_PEAK_GBS = 8000.0
METRIC = "DPF leaf points/sec (EvalFull logN=20, batched keys) + AES blocks/sec"


def stop_of(logN: int) -> int:
    return logN - 7 if logN >= 7 else 0


def aes_full(logN: int) -> int:
    s = stop_of(logN)
    return 3 * (1 << s) - 2 if s > 0 else 1


def load_peaks() -> dict:
    """Microbenchmarked MI355X rates (tools/valu_peak.hip ->
    profiles/r03_valu_peak.json: its LDS lookup loop now steps issue
    priority by progress like the tree kernel, 17.17 T lookups/s against
    r01's 16.44); reported beside the guide's peaks."""
    d = {}
    for name in ("r03_valu_peak.json", "r01_valu_peak.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
            break
        except Exception:
            continue
    return {"bitop3_Tops": float(d.get("v_bitop3_b32_Tops", 59.7)),
            "lds_lookups_Gs": float(d.get("ds_read_b32_lookup_G_per_s", 16438.3))}


def prg_roofline(aes_rate: float, kernel: str, k_ms: float, hbm_bytes: float, aes_impl: str = "lds-ttable",
                 workload: str = "evalfull", profiled_shape: bool = True) -> dict:
    """Roofline of the PRG-bound kernels, named by the resource that binds.

    T-table back end (the default): LDS.  Each AES-MMO block is 160
    ds_read_b32 lookups (16 per round x 10), and the lookups, not the VALU,
    bind (the LDS array is ~90% busy, VALU ~54%): achieved =
    lookups/s against the guide's ~75 TB/s of ds_read_b32 = 18.75 T
    lookups/s.  Byte-sliced back end: VALU.  Either way "gate" carries SURVEY
    §8d's headline denominator beside it: 22,928 two-input gate-equivalents
    per block against the guide's VALU issue rate x 32 bit-lanes x 2 gates per
    v_bitop3 (5.03 P gate-eq/s)."""
    peaks = load_peaks()
    gate = aes_rate * GATES_PER_AES / 1e12
    gbs = hbm_bytes / (k_ms * 1e-3) / 1e9
    gate_obj = {"bound": "valu", "achieved": round(gate, 1), "peak": round(GUIDE_GATE_PEAK_T, 1),
                "unit": "Tgate/s (2-input gate-equivalents; 22,928 per AES-128-MMO block)",
                "frac": round(gate / GUIDE_GATE_PEAK_T, 4),
                "peak_source": "MI355X_MICROARCH.md: 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz = 78.64 T lane-op/s x 32 x 2",
                "peak_measured": round(peaks["bitop3_Tops"] * 64, 1),
                "frac_vs_measured": round(gate / (peaks["bitop3_Tops"] * 64), 4)}
    if aes_impl == "lds-ttable":
        lk = aes_rate * LOOKUPS_PER_AES / 1e12
        r = {"bound": "lds", "achieved": round(lk, 3), "peak": GUIDE_LDS_LOOKUPS_T,
             "unit": "T lookups/s (ds_read_b32, 160 per AES-MMO block)",
             "frac": round(lk / GUIDE_LDS_LOOKUPS_T, 4), "traffic": None,
             "peak_source": "MI355X_MICROARCH.md: ds_read_b32 aggregate ~75 TB/s / 4 B",
             "peak_measured": round(peaks["lds_lookups_Gs"] / 1e3, 3),
             "frac_vs_measured": round(lk / (peaks["lds_lookups_Gs"] / 1e3), 4),
             "gate": gate_obj}
    else:
        r = dict(gate_obj)
        r["traffic"] = None
    r.update({"kernel": kernel, "kernel_ms": round(k_ms, 4), "aes_impl": aes_impl, "aes_blocks_per_s": aes_rate,
              "hbm_GBs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)})
    # Measured HBM bytes per launch of this kernel from the committed PMC
    # passes (tools/counters.sh + tools/traffic.py -> profiles/*traffic.json).
    # Multi-kernel steps (eval, pir) sum every dpf kernel of their own PMC
    # run (one launch of each per step).  Only when those passes profiled
    # this per-rank shape (profiled_shape): a split/PIR rank of an N-way
    # split runs a 1/N-size subtree, which no committed profile measured.
    if not profiled_shape:
        r["traffic_note"] = "no PMC profile at this per-rank shape (1/N of the 1-GPU split); traffic not reported"
        return r
    if workload != "evalfull":
        for rnd in ("r06", "r05", "r04", "r03", "r02"):
            name = f"{rnd}_traffic_{workload}.json"
            try:
                with open(os.path.join(ROOT, "profiles", name)) as f:
                    t = json.load(f)
            except Exception:
                continue
            # PIR: the roofline is the tree's (k_evalfull); the fold has its
            # own, and k_slice_db runs once per DB load, not per step.
            ks = sorted(k for k in t if k.startswith("k_") and not k.startswith("k_slice")
                        and (workload != "pir" or not k.startswith(("k_fold", "k_xor"))))
            tot = sum(t[k]["traffic_bytes"] for k in ks)
            r["traffic"] = round(tot)
            r["traffic_over_algorithmic"] = round(tot / hbm_bytes, 3)
            r["traffic_source"] = f"profiles/{name} (sum of {', '.join(ks)})"
            break
        return r
    for name in ("r06_traffic.json", "r05_traffic.json", "r04_traffic.json", "r03_traffic.json", "r02_traffic.json", "r01_traffic.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                t = json.load(f)
        except Exception:
            continue
        # r04 kernel names carry the raw-key flag: k_evalfull<7, true, false, true>.
        hit = kernel if kernel in t else next((k for k in t if k.startswith(kernel.rstrip(">"))), None)
        if hit:
            r["traffic"] = round(t[hit]["traffic_bytes"])
            r["traffic_over_algorithmic"] = round(t[hit]["traffic_bytes"] / hbm_bytes, 3)
            r["traffic_source"] = f"profiles/{name} ({hit})"
            break
    return r


def host_cpus() -> dict:
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota when one is set (the GPU box gives one GPU's job a CPU share)."""
    try:
        mask = len(os.sched_getaffinity(0))
    except Exception:
        mask = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    use = min(mask, quota) if quota else mask
    return {"nproc": os.cpu_count(), "affinity": mask, "cgroup_quota": quota, "model": model, "use": use}


def cpu_baseline(logN: int, target_s: float = 10.0) -> dict:
    """The oracle's reference-faithful C restatement (AES-NI, one aes128MMO
    per call, DFS like evalFullRecursive, dpf.go:213-262) on this host:
      - configs[0]: single-key EvalFull at logN on ONE core (dpf_test.go:7-21
        / dpf_main.go:25-30 shape), repeated for ~15% of target_s;
      - batched: one key per thread at a time over every usable CPU (as
        parallel goroutines would), passes over a fixed key set for the rest."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from dpf import synth
    import dpf

    cpus = host_cpus()
    cores = cpus["use"]
    n = cores * 8
    al, s0, s1 = synth.key_seeds(n, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    # configs[0]: one key, one core
    oracle.evalfull_batch(ka[:1], logN, nthreads=1, aesni=True)
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.evalfull_batch(ka[:1], logN, nthreads=1, aesni=True)
        reps += 1
        dt1 = time.perf_counter() - t0
        if dt1 >= 0.15 * target_s:
            break
    single_ms = dt1 / reps * 1e3
    oracle.evalfull_batch(ka[:cores], logN, nthreads=cores, aesni=True)   # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        oracle.evalfull_batch(ka, logN, nthreads=cores, aesni=True)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= 0.85 * target_s:
            break
    keys = n * passes
    pts = keys * (1 << logN)
    return {"value": pts / dt, "unit": "points/s", "cores": cores, "kind": "port",
            "aes_blocks_per_s": keys * aes_full(logN) / dt,
            "cpu_model": cpus["model"], "nproc": cpus["nproc"], "affinity_cpus": cpus["affinity"],
            "cgroup_cpu_quota": cpus["cgroup_quota"],
            "config0_single_key_1core": {"logN": logN, "ms_per_evalfull": round(single_ms, 3),
                                         "points_per_s": (1 << logN) / (single_ms * 1e-3),
                                         "aes_blocks_per_s": aes_full(logN) / (single_ms * 1e-3),
                                         "reps": reps},
            "sample": f"configs[0]: {reps} single-key EvalFulls at logN={logN} on 1 core ({dt1:.1f} s); "
                      f"batched: {keys} key-EvalFulls ({passes} passes over {n} keys, {dt:.1f} s, "
                      f"{cores} threads, AES-NI one block per call; oracle/dpf_oracle.c)"}


def cpu_baseline_eval(logN: int, nkeys: int, ppk: int, target_s: float = 8.0) -> dict:
    """configs[2] on the host: the oracle's reference-faithful Eval (AES-NI,
    both children per level like dpf.go:171-211) over a bounded sample of
    keys x points, one key's points per thread at a time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from dpf import synth
    import dpf
    cores = host_cpus()["use"]
    nk = min(nkeys, cores * 4)
    al, s0, s1 = synth.key_seeds(nk, logN)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    xs = synth.eval_points(nk, ppk, logN)
    oracle.eval_batch(ka[:1], xs[:1], logN, nthreads=1)
    passes, t0 = 0, time.perf_counter()
    while True:
        oracle.eval_batch(ka, xs, logN, nthreads=cores)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= target_s:
            break
    q = passes * nk * ppk
    return {"value": q / dt, "unit": "queries/s", "cores": cores, "kind": "port",
            "sample": f"{passes} passes over {nk} keys x {ppk} points at logN={logN} ({dt:.1f} s, {cores} "
                      f"threads; oracle/dpf_oracle.c Eval, AES-NI one block per call)"}


def cpu_baseline_pir(logN: int, batch: int, target_s: float = 8.0) -> dict:
    """configs[4] on the host: the oracle's PIR answer (AES-NI EvalFull of
    the key, then a byte-wise XOR fold of the selected 32-B records), one
    query per thread, over a bounded number of queries."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from dpf import synth
    import dpf
    from concurrent.futures import ThreadPoolExecutor
    cores = host_cpus()["use"]
    nrec = 1 << logN
    db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
    al, s0, s1 = synth.key_seeds(max(batch, cores), logN, first=4242)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    keys = [k.tobytes() for k in ka]
    done, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:       # ctypes releases the GIL during each answer
        while True:
            list(ex.map(lambda k: oracle.pir_answer(k, logN, db, 0, nrec), keys[:cores]))
            done += cores
            dt = time.perf_counter() - t0
            if dt >= target_s:
                break
    return {"value": done / dt, "unit": "queries/s", "cores": cores, "kind": "port",
            "sample": f"{done} PIR answers at logN={logN} over a {nrec}-record x 32-B DB ({dt:.1f} s, {cores} "
                      f"threads; oracle/dpf_oracle.c oracle_pir_answer)"}


class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        import dpf
        self.torch, self.dist, self.dpf = torch, dist, dpf
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        # One rank per GPU over RCCL.  When there are more ranks than visible
        # GPUs (a rehearsal on a 1-GPU box) ranks fold onto the devices and
        # the control-plane collectives go over gloo (RCCL refuses two ranks
        # on one GPU).  DPF_BENCH_BACKEND overrides.
        ndev = max(1, torch.cuda.device_count())
        self.folded = self.world > ndev          # a rehearsal, not an N-GPU measurement
        self.backend = os.environ.get("DPF_BENCH_BACKEND", "nccl" if self.world <= ndev else "gloo")
        self.local = int(os.environ.get("LOCAL_RANK", "0")) % ndev
        if self.world > 1:
            torch.cuda.set_device(self.local)
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(self.backend)
        self.dev = torch.device("cuda", self.local)
        torch.cuda.set_device(self.dev)
        dpf.gpu_init_devices([self.local])      # this rank's GPU only: no context on the others
        if args.aes:
            dpf.set_aes_impl(args.aes)
        self.stream = torch.cuda.current_stream(self.dev)

    def timed(self, step, steps, warmup, every=None):
        """Warmup, then `steps` steps between barrier+sync pairs; returns the
        max-over-ranks wall time and the mean kernel time of the event pairs."""
        torch, dist = self.torch, self.dist
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        # Kernel time is sampled: events bracket every n-th step (--event-every,
        # default 10).  A timing event is a barrier packet in the queue; on every
        # step it cost ~8 us/step (0.1431 vs 0.1350 ms at 512 keys, 0.953 vs
        # 0.943 ms at 4096: profiles/r04/events), which the wall clock would
        # then charge to the path.  At least 5 samples per timed region;
        # n=0: no events (kernel_ms NaN).
        if every is None:
            every = self.args.event_every
            every = max(1, min(every, steps // 5)) if every > 0 else 0
        timed_i = [i for i in range(steps) if every > 0 and i % every == 0]
        # Clock spin-up (untimed, before the W warmup steps): an idle MI355X
        # needs a few hundred ms of load to reach its steady-state clock; a
        # 5-step warmup (~6 ms) left configs[1] at 1.174 ms/launch against
        # 1.069 ms after 60 steps (profiles/r02/warmup).  Steady state is what
        # a busy server sees, so every workload first runs its own step for
        # SPINUP_S seconds of wall time.
        # Ranks agree on when to stop (MIN over ranks of "still spinning"):
        # a step may hold a collective (PIR's gather), so every rank must run
        # the same number of spin-up steps.
        t_spin = time.perf_counter()
        more = self.args.spinup > 0
        while more:
            for _ in range(4):
                step(None)
            torch.cuda.synchronize(self.dev)
            more = time.perf_counter() - t_spin < self.args.spinup
            if self.world > 1:
                f = torch.tensor([1.0 if more else 0.0], dtype=torch.float64,
                                 device=self.dev if self.backend == "nccl" else "cpu")
                dist.all_reduce(f, op=dist.ReduceOp.MIN)
                more = float(f.item()) > 0
        for _ in range(warmup):
            step(None)
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for i in range(steps):
            step(evs[i] if every == 1 or i in timed_i else None)
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            dist.barrier()
        t_wall = time.perf_counter() - t0
        if self.world > 1:
            t = torch.tensor([t_wall], dtype=torch.float64,
                             device=self.dev if self.backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t_wall = float(t.item())
        k_ms = (sum(evs[i][0].elapsed_time(evs[i][1]) for i in timed_i) / len(timed_i)) if timed_i else float("nan")
        return t_wall, k_ms

    def line(self, **kw):
        base = {"n_gpus": self.world, "steps": self.args.steps, "warmup": self.args.warmup,
                "spinup_s": self.args.spinup, "event_every": self.args.event_every,
                "higher_is_better": True, "vs_baseline": None, "dtype": "u32"}
        base.update(kw)
        return base


def wl_evalfull(c: Ctx) -> dict:
    """configs[1].  The headline uses the library's AES back end (--aes, or
    the default); the other back end is timed the same way right after and
    reported under "aes_variants" (configs[1]: bitsliced vs LDS T-table)."""
    a, dpf, torch = c.args, c.dpf, c.torch
    from dpf import synth, shard
    logN = a.logN
    W = c.world if c.world > 1 else max(1, a.emulate_world)
    if a.strong:
        # SURVEY 8d's strong-scaling form: a fixed batch of a.nkeys keys split
        # over the ranks by range (no collective).  With --emulate-world W on
        # one GPU: rank 0's share of a W-way split, timed alone.
        lo, hi = shard.key_range(a.nkeys, W, c.rank)
        nk, first = hi - lo, lo
    else:
        nk, first = a.nkeys, c.rank * a.nkeys                        # weak: this rank's own batch
    kl, olen = dpf.key_len(logN), dpf.evalfull_len(logN)
    al, s0, s1 = synth.key_seeds(nk, logN, first=first)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(c.dev)
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=c.dev)
    d_out = torch.empty(nk * olen, dtype=torch.uint8, device=c.dev)

    # One step = one-shot EvalFull of the resident key bytes (dpf_evalfull_batch_dev):
    # the T-table tree kernel reads the key bytes itself where every wave owns a
    # key (no unpack launch); otherwise the keys are unpacked first, inside the step.
    def step(ev):
        if ev:
            ev[0].record(c.stream)
        dpf.evalfull_batch_dev(d_keys, kl, nk, logN, d_out, d_work, device=c.local, stream=c.stream)
        if ev:
            ev[1].record(c.stream)

    names = {dpf.AES_TTABLE: "lds-ttable", dpf.AES_BITSLICED: "bitsliced"}
    main_impl = dpf.get_aes_impl()
    t_wall, k_ms = c.timed(step, a.steps, a.warmup)
    sec = t_wall / a.steps
    aes = nk * aes_full(logN)
    variants = {names[main_impl]: {"ms_per_step": sec * 1e3, "kernel_ms": k_ms,
                                   "aes_blocks_per_s": aes / (k_ms * 1e-3),
                                   "points_per_s": nk * (1 << logN) / sec}}
    if a.check and c.rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        idx = np.unique(np.linspace(0, nk - 1, 8).astype(int))
        got = d_out.view(nk, olen)[torch.from_numpy(idx).to(c.dev)].cpu().numpy()
        assert np.array_equal(got, oracle.evalfull_batch(ka[idx], logN, nthreads=8)), "output differs from oracle"
    if not a.no_variants:
        other = dpf.AES_BITSLICED if main_impl == dpf.AES_TTABLE else dpf.AES_TTABLE
        ref = d_out.view(nk, olen)[:64].clone()
        dpf.set_aes_impl(other)
        t2, k2 = c.timed(step, max(5, a.steps // 2), 3)
        dpf.set_aes_impl(main_impl)
        variants[names[other]] = {"ms_per_step": t2 / max(5, a.steps // 2) * 1e3, "kernel_ms": k2,
                                  "aes_blocks_per_s": aes / (k2 * 1e-3),
                                  "points_per_s": nk * (1 << logN) / (t2 / max(5, a.steps // 2)),
                                  "bit_identical_first_64_keys": bool(torch.equal(ref, d_out.view(nk, olen)[:64]))}
    pipelined = None
    if c.world == 1 and a.pipelined and not a.strong:
        # A server with a queue of batches: consecutive batches on two streams
        # (own output and workspace each), so the last waves of one launch
        # overlap the first of the next.  Reported beside `value`, which stays
        # the one-stream step that the kernel roofline describes.  Opt-in
        # (--pipelined): overlapped launches last longer each, so in the
        # default run they would skew a kernel trace's average for the
        # headline kernel away from the line's roofline.kernel_ms.
        d_out2 = torch.empty_like(d_out)
        d_work2 = torch.empty_like(d_work)
        sts = [c.stream, torch.cuda.Stream(c.dev)]
        flip = [0]

        def step2(ev):
            i = flip[0]
            flip[0] ^= 1
            dpf.evalfull_batch_dev(d_keys, kl, nk, logN, d_out if i == 0 else d_out2, d_work if i == 0 else d_work2,
                                   device=c.local, stream=sts[i])

        tp, _ = c.timed(step2, a.steps, a.warmup, every=0)
        pipelined = {"streams": 2, "ms_per_step": tp / a.steps * 1e3, "points_per_s": nk * (1 << logN) / (tp / a.steps),
                     "note": "batches alternate over two streams; value is the one-stream step"}
        del d_out2, d_work2
    emulated = a.strong and W != c.world
    total = nk if emulated else a.nkeys if a.strong else nk * c.world
    line = c.line(metric=METRIC, value=total * (1 << logN) / sec, unit="points/s",
                  ms_per_step=sec * 1e3, scaling="strong" if a.strong else "weak",
                  data="synthetic (SplitMix64 seed 0x5EEDD9F0 keys via host Gen)",
                  config={"workload": (f"batched EvalFull, {a.nkeys} keys x logN={logN} split over {W} GPU(s)"
                                       + (f" (rank 0's {nk} keys timed on 1 GPU)" if emulated else "")
                                       if a.strong else
                                       f"batched EvalFull, {nk} keys x logN={logN} per GPU") + " (BASELINE configs[1])",
                          "keys_per_gpu": nk, "logN": logN, "aes": names[main_impl],
                          "parallelism": f"key-shard x{c.world}"},
                  aes_blocks_per_s=total * aes_full(logN) / sec)
    if emulated:
        line["emulated_world"] = {"world": W, "keys_per_rank": nk,
                                  "implied_points_per_s": a.nkeys * (1 << logN) / sec,
                                  "note": "if every rank ran rank 0's step time; not an N-GPU measurement"}
    kern = (f"k_evalfull<{min(stop_of(logN), 7)}, true, false>" if main_impl == dpf.AES_TTABLE
            else "k_evalfull<NODES>+k_evalfull_bs<true>")
    line["roofline"] = prg_roofline(aes / (k_ms * 1e-3), kern, k_ms, nk * olen + nk * (stop_of(logN) + 2) * 32,
                                    aes_impl=names[main_impl], profiled_shape=(nk == 4096))
    line["aes_variants"] = variants
    if pipelined:
        line["pipelined"] = pipelined
    if c.world == 1 and not a.no_api:
        line["api"] = api_rates(c, ka, logN)
        line["single_call"] = single_call_latency(c, ka[0].tobytes(), logN)
        c.reference_shapes = reference_shapes_gpu(c)
    return line


# The reference's own timing shapes: BenchmarkEvalFull is one
# EvalFull at logN=28 of a key for alpha=0 (dpf/dpf_test.go:7-21); the CLI
# times Gen(123, 27) then 100 x EvalFull(., 27) (dpf_main.go:25-30).  The GPU
# side runs them through the drop-in single-key API (dpf.EvalFull, a fresh
# output like the Go slice, dpf.go:251) and kernel-resident (one key's
# dpf_evalfull_batch_dev, output left in HBM); the CPU side (finalize) is the
# oracle's reference-style restatement on one core.
REF_SHAPES = {"BenchmarkEvalFull": {"logN": 28, "alpha": 0, "source": "dpf/dpf_test.go:7-21"},
              "dpf_main": {"logN": 27, "alpha": 123, "reps": 100, "source": "dpf_main.go:25-30"}}


def reference_shapes_gpu(c: Ctx) -> dict:
    dpf, torch = c.dpf, c.torch
    out = {}
    for name, sh in REF_SHAPES.items():
        logN = sh["logN"]
        al, s0, s1 = np.array([sh["alpha"]], np.uint64), *[np.frombuffer(bytes(range(i, i + 16)), np.uint8)[None]
                                                           for i in (1, 17)]
        ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
        key = ka[0].tobytes()
        d_key = torch.from_numpy(ka.reshape(-1)).to(c.dev)
        d_work = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=c.dev)
        d_out = torch.empty(dpf.evalfull_len(logN), dtype=torch.uint8, device=c.dev)

        def dev_call():
            dpf.evalfull_batch_dev(d_key, len(key), 1, logN, d_out, d_work, device=c.local, stream=c.stream)
        for _ in range(3):
            dev_call()
        torch.cuda.synchronize(c.dev)
        reps = sh.get("reps", 20)
        t0 = time.perf_counter()
        for _ in range(reps):
            dev_call()
        torch.cuda.synchronize(c.dev)
        dev_ms = (time.perf_counter() - t0) / reps * 1e3
        dpf.EvalFull(key, logN)                                  # warm the host-buffer path
        t0 = time.perf_counter()
        for _ in range(reps):
            dpf.EvalFull(key, logN)
        api_ms = (time.perf_counter() - t0) / reps * 1e3
        # The C ABI itself, as a cgo caller binds it (dpf_evalfull, no Python
        # buffer handling): into one reused host buffer, and into a fresh
        # np.empty per call (first touch of its pages inside the call, like a
        # fresh Go slice, dpf.go:251).  Medians.
        L, kk, nbytes = dpf.lib(), np.frombuffer(key, np.uint8), dpf.evalfull_len(logN)
        reused = np.empty(nbytes, np.uint8)

        def capi(buf):
            rc = L.dpf_evalfull(dpf._buf(kk), kk.size, logN, dpf._buf(buf))
            assert rc == 0, rc

        def med_ms(f, n):
            f()
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                f()
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts)) * 1e3
        capi_reused = med_ms(lambda: capi(reused), 31)
        capi_fresh = med_ms(lambda: capi(np.empty(nbytes, np.uint8)), 31)
        r = {"logN": logN, "alpha": sh["alpha"], "source": sh["source"],
             "gpu_dev_ms_per_evalfull": round(dev_ms, 4),
             "gpu_api_ms_per_evalfull": round(api_ms, 4),
             "capi_reused_ms": round(capi_reused, 4), "capi_fresh_ms": round(capi_fresh, 4),
             "capi_reused_GBps": round(nbytes / (capi_reused * 1e-3) / 1e9, 2),
             "capi_fresh_GBps": round(nbytes / (capi_fresh * 1e-3) / 1e9, 2),
             "gpu_dev_points_per_s": (1 << logN) / (dev_ms * 1e-3),
             "gpu_note": "dev: dpf_evalfull_batch_dev of one key, output left in HBM; api: dpf.EvalFull "
                         "(C ABI dpf_evalfull into a fresh np.empty, returned as a view, incl. its D2H), mean of "
                         "%d calls; capi_*: dpf_evalfull called directly (ctypes), medians of 31, output cut into "
                         ">= 4 subtree slabs so kernel, PCIe copy and host copy overlap" % reps}
        if name == "dpf_main":
            t0 = time.perf_counter()
            k2, _ = dpf.Gen(123, logN)
            for _ in range(reps):
                dpf.EvalFull(k2, logN)
            r["gpu_api_total_s"] = round(time.perf_counter() - t0, 4)
            r["gpu_api_total_note"] = "Gen(123, 27) + 100 x EvalFull(., 27) through the drop-in API, as dpf_main.go"
        out[name] = r
    return out


def reference_shapes_cpu(gpu: dict) -> dict:
    """The same shapes on ONE host core with the oracle's reference-style
    restatement (AES-NI, one aes128MMO per call, DFS: dpf.go:213-262), beside
    the GPU numbers of reference_shapes_gpu."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    out = {}
    for name, sh in REF_SHAPES.items():
        logN = sh["logN"]
        ka, _ = oracle.gen(sh["alpha"], logN, bytes(range(1, 17)), bytes(range(17, 33)))
        r = dict(gpu.get(name, {"logN": logN, "alpha": sh["alpha"], "source": sh["source"]}))
        if name == "dpf_main":
            t0 = time.perf_counter()
            k, _ = oracle.gen(123, logN, bytes(range(1, 17)), bytes(range(17, 33)))
            for _ in range(sh["reps"]):
                oracle.evalfull(k, logN, aesni=True)
            tot = time.perf_counter() - t0
            r["cpu_total_s"] = round(tot, 3)
            r["cpu_ms_per_evalfull"] = round(tot / sh["reps"] * 1e3, 3)
        else:
            oracle.evalfull(ka, logN, aesni=True)
            reps, t0 = 0, time.perf_counter()
            while reps < 3 or time.perf_counter() - t0 < 2.0:
                oracle.evalfull(ka, logN, aesni=True)
                reps += 1
            r["cpu_ms_per_evalfull"] = round((time.perf_counter() - t0) / reps * 1e3, 3)
            r["cpu_reps"] = reps
        r["cpu_cores"] = 1
        r["cpu_kind"] = "port (oracle/dpf_oracle.c, AES-NI one block per call, DFS)"
        if "gpu_dev_ms_per_evalfull" in r:
            r["gpu_dev_speedup_vs_cpu"] = round(r["cpu_ms_per_evalfull"] / r["gpu_dev_ms_per_evalfull"], 1)
            r["gpu_api_speedup_vs_cpu"] = round(r["cpu_ms_per_evalfull"] / r["gpu_api_ms_per_evalfull"], 1)
        out[name] = r
    return out


def single_call_latency(c: Ctx, key: bytes, logN: int) -> dict:
    """The reference's own call shapes, one key (dpf.go:171 Eval, :243
    EvalFull), through the drop-in C ABI: the host small-call path
    (host_eval.cpp, what DPF_SMALL_AUTO picks at this size), the GPU round
    trip, and the reference-style CPU restatement (oracle, one aes128MMO per
    call) for scale.  Medians; latency, not throughput."""
    dpf = c.dpf
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    def med(f, n):
        f()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    x = 12345 % (1 << logN)
    prev = dpf.get_small_call_path()
    out = {"logN": logN, "auto_routes_evalfull_to_host_up_to_logN": dpf.small_call_max_logN()}
    for mode in ("host", "gpu"):
        dpf.set_small_call_path(mode)
        out[f"eval_{mode}_us"] = round(med(lambda: dpf.Eval(key, x, logN), 101) * 1e6, 2)
        out[f"evalfull_{mode}_ms"] = round(med(lambda: dpf.EvalFull(key, logN), 21) * 1e3, 4)
    dpf.set_small_call_path(prev)
    out["eval_ref_style_cpu_us"] = round(med(lambda: oracle.eval_(key, x, logN, aesni=True), 101) * 1e6, 2)
    out["evalfull_ref_style_cpu_ms"] = round(med(lambda: oracle.evalfull(key, logN, aesni=True), 9) * 1e3, 4)
    return out


def api_rates(c: Ctx, ka: np.ndarray, logN: int, reps: int = 5) -> dict:
    """The PCIe-inclusive rate a host caller gets (never `value`): the same
    batch through the host-buffer C ABI dpf_evalfull_batch (keys H2D, output
    D2H into caller memory, synchronous; dpf.go:243-262's EvalFull returns a
    fresh slice).  Two destinations: a FRESH array per call (first touch of
    its pages inside the call; the caller's later free is its own and is
    timed apart) and a REUSED array.  Median of `reps` calls."""
    dpf = c.dpf
    nk = ka.shape[0]
    shape = (nk, dpf.evalfull_len(logN))
    out_b = shape[0] * shape[1]
    reuse = np.empty(shape, np.uint8)
    dpf.evalfull_batch(ka, logN, ngpus=1, out=reuse)
    t_reuse, t_fresh, t_free = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        dpf.evalfull_batch(ka, logN, ngpus=1, out=reuse)
        t_reuse.append(time.perf_counter() - t0)
    for _ in range(reps):
        out = np.empty(shape, np.uint8)
        t0 = time.perf_counter()
        dpf.evalfull_batch(ka, logN, ngpus=1, out=out)
        t1 = time.perf_counter()
        del out
        t_free.append(time.perf_counter() - t1)
        t_fresh.append(t1 - t0)
    med = lambda v: float(np.median(v))  # noqa: E731
    return {"entry": "dpf_evalfull_batch (host buffers, synchronous)", "bytes_out": out_b,
            "reused_out": {"ms": round(med(t_reuse) * 1e3, 3), "points_per_s": nk * (1 << logN) / med(t_reuse),
                           "D2H_GBs": round(out_b / med(t_reuse) / 1e9, 2)},
            "fresh_out": {"ms": round(med(t_fresh) * 1e3, 3), "points_per_s": nk * (1 << logN) / med(t_fresh),
                          "D2H_GBs": round(out_b / med(t_fresh) / 1e9, 2),
                          "caller_free_ms": round(med(t_free) * 1e3, 3)}}


def wl_eval(c: Ctx) -> dict:
    a, dpf, torch = c.args, c.dpf, c.torch
    from dpf import synth
    logN, nk, ppk = a.logN, a.eval_keys, a.eval_points
    kl = dpf.key_len(logN)
    al, s0, s1 = synth.key_seeds(nk, logN, first=c.rank * nk)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    xs = synth.eval_points(nk, ppk, logN, master=0x5EEDD9F1 + c.rank)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(c.dev)
    d_xs = torch.from_numpy(xs.reshape(-1).view(np.int64)).to(c.dev)
    d_work = torch.empty(dpf.eval_workspace_size(nk, ppk, logN), dtype=torch.uint8, device=c.dev)
    d_out = torch.empty(nk * ppk, dtype=torch.uint8, device=c.dev)

    def step(ev):
        if ev:
            ev[0].record(c.stream)
        dpf.eval_batch_dev(d_keys, kl, nk, d_xs, ppk, logN, d_out, d_work, device=c.local, stream=c.stream)
        if ev:
            ev[1].record(c.stream)

    t_wall, k_ms = c.timed(step, a.steps, a.warmup)
    if a.check and c.rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        got = d_out.view(nk, ppk)[:64].cpu().numpy()
        assert np.array_equal(got, oracle.eval_batch(ka[:64], xs[:64], logN, nthreads=8)), "Eval differs"
    sec = t_wall / a.steps
    q = nk * ppk
    aes = q * (stop_of(logN) + 1)                    # algorithmic per-query walks (SURVEY §8a A_eval)
    L = dpf.eval_frontier_level(logN, ppk)
    aes_done = nk * ((1 << (L + 1)) - 2 if L else 0) + q * (stop_of(logN) - L + 1)   # what the kernels compute
    line = c.line(metric="DPF Eval point queries/sec (batched Eval)", value=q * c.world / sec, unit="queries/s",
                  ms_per_step=sec * 1e3, scaling="weak", data="synthetic keys + uniform points",
                  config={"workload": f"batched Eval, {nk} keys x {ppk} points, logN={logN} per GPU "
                                      f"(BASELINE configs[2])", "logN": logN, "parallelism": f"key-shard x{c.world}"},
                  aes_blocks_per_s=aes * c.world / sec,
                  aes_blocks_per_s_executed=aes_done * c.world / sec,
                  aes_blocks_note=(f"aes_blocks_per_s is reference-equivalent: stop+1 = {stop_of(logN) + 1} AES per "
                                   f"query (SURVEY 8d A_eval), more than the kernels run; "
                                   f"aes_blocks_per_s_executed counts the {aes_done / q:.2f} per query they compute "
                                   f"(shared frontier at level {L} + per-query walks)"))
    line["roofline"] = prg_roofline(aes_done / (k_ms * 1e-3), "k_unpack+[k_evalfull<nodes>]+k_eval", k_ms, 
                                    q * 9 + nk * (stop_of(logN) + 2) * 32, workload="eval")
    if L:
        fb = nk * (1 << L) * 17 + q * 17
        line["roofline"]["frontier_bytes"] = fb
        line["roofline"]["frontier_note"] = ("the HBM frontier trades AES for bytes: 17 B per node written once and "
                                             "17 B read per query, not part of the algorithmic 9 B per query")
    line["roofline"]["note"] = (f"achieved counts the AES the kernels compute: a shared frontier at level {L} "
                                f"(2^(L+1)-2 per key) + stop-L+1 per query = {aes_done / q:.2f} per query, against "
                                f"the per-query walk's {stop_of(logN) + 1} (aes_blocks_per_s above)")
    return line


def wl_split(c: Ctx) -> dict:
    a, dpf, torch = c.args, c.dpf, c.torch
    from dpf import synth, shard
    logN = a.split_logN
    kl = dpf.key_len(logN)
    W = c.world if c.world > 1 else max(1, a.emulate_world)
    pb, prefix = shard.subtree_split(W, c.rank)
    al, s0, s1 = synth.key_seeds(1, logN, first=777)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)          # the same key on every rank
    part = dpf.evalfull_len(logN) >> pb
    d_keys = torch.from_numpy(ka.reshape(-1)).to(c.dev)
    d_work = torch.empty(dpf.workspace_size(1, logN), dtype=torch.uint8, device=c.dev)
    d_out = torch.empty(part, dtype=torch.uint8, device=c.dev)

    def step(ev):
        if ev:
            ev[0].record(c.stream)
        dpf.evalfull_subtree_dev(d_keys, kl, 1, logN, pb, prefix, d_out, d_work, device=c.local, stream=c.stream)
        if ev:
            ev[1].record(c.stream)

    t_wall, k_ms = c.timed(step, a.steps, a.warmup)
    if a.check and c.rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        head = d_out[:16].cpu().numpy()
        base = prefix << (logN - pb)
        for q in range(0, 128, 17):
            assert ((head[q >> 3] >> (q & 7)) & 1) == oracle.eval_(ka[0].tobytes(), base + q, logN, aesni=True)
    sec = t_wall / a.steps
    stop = stop_of(logN)
    aes = 3 * (1 << (stop - pb)) - 2 + pb                    # per rank: subtree + prefix walk
    line = c.line(metric="DPF leaf points/sec (single-key EvalFull split by subtree)",
                  value=(1 << logN) / sec, unit="points/s", ms_per_step=sec * 1e3,
                  scaling="strong", data="synthetic key",
                  config={"workload": f"one key EvalFull logN={logN} split over {W} GPU(s)"
                                      + (" (rank 0's share timed on 1 GPU)" if W != c.world else "")
                                      + " (BASELINE configs[3])",
                                                "logN": logN, "parallelism": f"subtree-split x{c.world}"},
                  aes_blocks_per_s=aes * c.world / sec)
    line["roofline"] = prg_roofline(aes / (k_ms * 1e-3), "k_evalfull<7, true, false>", k_ms, part, workload="split",
                                    profiled_shape=(W == 1))
    if c.world == 1 and not a.no_api:
        line["api"] = split_api_rate(c, ka[0].tobytes(), logN)
    return line


def split_api_rate(c: Ctx, key: bytes, logN: int, reps: int = 3) -> dict:
    """configs[3] through the host-buffer C ABI dpf_evalfull_split (key H2D,
    the whole 2^(logN-3)-byte output D2H into caller memory, synchronous):
    what a Go EvalFull caller gets (dpf.go:251 returns the whole slice).
    Into a REUSED caller buffer; median of `reps` calls."""
    dpf = c.dpf
    out = np.empty(dpf.evalfull_len(logN), np.uint8)
    dpf.evalfull_split(key, logN, 1, out=out)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        dpf.evalfull_split(key, logN, 1, out=out)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    return {"entry": "dpf_evalfull_split (host buffer, synchronous, 1 GPU)", "bytes_out": out.nbytes,
            "reused_out": {"ms": round(t * 1e3, 3), "points_per_s": (1 << logN) / t,
                           "D2H_GBs": round(out.nbytes / t / 1e9, 2)}}


def pir_setup(c: Ctx, W: int):
    """This rank's DB slice in HBM (the same synthetic DB on every run), in
    the layout the fold reads: bit-sliced for the matrix-core fold (built
    once on the device, like a server loading its DB; not timed per step),
    row-major for the LDS fold (--pir-fold lds)."""
    from dpf import synth, shard
    torch, dpf = c.torch, c.dpf
    logN = c.args.pir_logN
    nrec = 1 << logN
    lo, hi = shard.db_slice(nrec, logN, W, c.rank)
    db = synth.db_bytes(hi * 32)[lo * 32:]                    # this rank's slice of the synthetic DB
    d_db = torch.from_numpy(db).to(c.dev)
    c.pir_layout = {"fold": c.args.pir_fold}
    if c.args.pir_fold == "mfma":
        d_dbs = torch.empty(dpf.pir_db_sliced_size(hi - lo), dtype=torch.uint8, device=c.dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(c.stream)
        dpf.pir_db_slice_dev(d_db, hi - lo, d_dbs, device=c.local, stream=c.stream)
        ev1.record(c.stream)
        torch.cuda.synchronize(c.dev)
        c.pir_layout.update({"db_layout": "bit-sliced (dpf_pir_db_slice_dev, once per DB load)",
                             "db_slice_ms": round(ev0.elapsed_time(ev1), 3)})
        del d_db
        return d_dbs, lo, hi
    c.pir_layout["db_layout"] = "row-major"
    return d_db, lo, hi


def pir_time(c: Ctx, W: int, d_db, lo: int, hi: int, nk: int, steps: int, warmup: int):
    """Time `steps` PIR steps of nk queries: server answers on this GPU's
    slice (dpf_pir_answer_dev), then the gather + host XOR when world > 1."""
    dpf, torch = c.dpf, c.torch
    from dpf import synth, shard
    logN = c.args.pir_logN
    kl = dpf.key_len(logN)
    pb, prefix = shard.subtree_split(W, c.rank)
    al, s0, s1 = synth.key_seeds(nk, logN, first=4242)       # the same queries on every server GPU
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(c.dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=c.dev)
    d_work = torch.empty(dpf.pir_workspace_size(nk, logN, pb), dtype=torch.uint8, device=c.dev)
    result = {}
    # One server GPU: each step's answers go to pinned host memory (a ring of
    # 2 buffers) by an async copy on the compute stream, so the host does not
    # stall the GPU between batches (a server returns batch i while batch i+1
    # runs); the timed region still ends after the last copy has landed.
    # Several GPUs: the all-gather + XOR of the partial answers is part of
    # every step.
    h_ans = [torch.empty(nk * 32, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    seq = [0]

    def step(ev):
        if ev:
            ev[0].record(c.stream)
        answer = dpf.pir_answer_sliced_dev if c.args.pir_fold == "mfma" else dpf.pir_answer_dev
        answer(d_keys, kl, nk, logN, d_db, hi - lo, d_ans, d_work, prefix_bits=pb, prefix=prefix,
               device=c.local, stream=c.stream)
        if ev:
            ev[1].record(c.stream)
        if c.world > 1:
            result["ans"] = shard.gather_xor(d_ans.view(nk, 32))
        else:
            h = h_ans[seq[0] % 2]
            seq[0] += 1
            with torch.cuda.stream(c.stream):
                h.copy_(d_ans, non_blocking=True)
            result["host"] = h

    t_wall, k_ms = c.timed(step, steps, warmup)
    if c.world == 1:
        result["ans"] = result["host"].view(nk, 32).numpy()     # after timed()'s final synchronize
    return ka, result, t_wall, k_ms


def pir_breakdown(c: Ctx, W: int, d_db, lo: int, hi: int, nk: int, steps: int) -> dict:
    """A PIR step's two phases timed apart with HIP events on the launch
    stream: the tree (key unpack + subtree EvalFull into the selection bits:
    dpf_evalfull_subtree_dev, what dpf_pir_answer_dev runs first) and the XOR
    fold of the DB slice under those bits (dpf_xor_fold_dev: the same
    launch_pir_fold call, its second half)."""
    dpf, torch = c.dpf, c.torch
    from dpf import synth, shard
    logN = c.args.pir_logN
    pb, prefix = shard.subtree_split(W, c.rank)
    kl = dpf.key_len(logN)
    per_key = dpf.evalfull_len(logN) >> pb
    al, s0, s1 = synth.key_seeds(nk, logN, first=4242)
    ka, _ = dpf.gen_batch_seeded(al, logN, s0, s1)
    d_keys = torch.from_numpy(ka.reshape(-1)).to(c.dev)
    d_bits = torch.empty(nk * per_key, dtype=torch.uint8, device=c.dev)
    d_work = torch.empty(dpf.workspace_size(nk, logN), dtype=torch.uint8, device=c.dev)
    d_fw = torch.empty(dpf.xor_fold_workspace_size(), dtype=torch.uint8, device=c.dev)
    d_ans = torch.empty(nk * 32, dtype=torch.uint8, device=c.dev)

    def tree(ev):
        if ev:
            ev[0].record(c.stream)
        dpf.evalfull_subtree_dev(d_keys, kl, nk, logN, pb, prefix, d_bits, d_work, device=c.local, stream=c.stream)
        if ev:
            ev[1].record(c.stream)

    def fold(ev):
        if ev:
            ev[0].record(c.stream)
        if c.args.pir_fold == "mfma":
            dpf.xor_fold_sliced_dev(d_bits, per_key, nk, d_db, hi - lo, d_ans, d_fw, device=c.local, stream=c.stream)
        else:
            dpf.xor_fold_dev(d_bits, per_key, nk, d_db, hi - lo, 32, d_ans, d_fw, device=c.local, stream=c.stream)
        if ev:
            ev[1].record(c.stream)

    _, t_ms = c.timed(tree, steps, 3, every=1)      # kernel times only: events on every step
    _, f_ms = c.timed(fold, steps, 3, every=1)
    # The same two phases back to back, as in a step, with an event between
    # them: each phase's time when it follows the other.
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in evs:
        e[0].record(c.stream)
        tree(None)
        e[1].record(c.stream)
        fold(None)
        e[2].record(c.stream)
    torch.cuda.synchronize(c.dev)
    in_step = {"tree_ms": round(sum(e[0].elapsed_time(e[1]) for e in evs) / steps, 4),
               "fold_ms": round(sum(e[1].elapsed_time(e[2]) for e in evs) / steps, 4)}
    blocks = nk * (3 * (1 << (stop_of(logN) - pb)) - 2)
    fold_bytes = (hi - lo) * 32 + nk * per_key          # DB slice + selection bits, read once
    gbs = fold_bytes / (f_ms * 1e-3) / 1e9
    # Measured HBM bytes of the fold kernels from the committed PMC passes of
    # this exact shape (1 GPU, 64 keys, the fold this run uses).
    traffic, tsrc = None, None
    if W == 1 and nk == 64:
        for rnd in ("r06", "r05", "r04", "r03"):
            name = f"{rnd}_traffic_pir.json"
            try:
                with open(os.path.join(ROOT, "profiles", name)) as f:
                    t = json.load(f)
            except Exception:
                continue
            want = ("k_fold_mfma", "k_fold_sliced") if c.args.pir_fold == "mfma" else ("k_fold4r", "k_fold_direct")
            ks = [k for k in t if k.startswith(want + ("k_xor_parts",))]
            if any(k.startswith(want) for k in ks):
                traffic, tsrc = round(sum(t[k]["traffic_bytes"] for k in ks)), f"profiles/{name} ({', '.join(sorted(ks))})"
                break
    return {"back_to_back": in_step,
            "tree": {"kernel_ms": round(t_ms, 4), "aes_blocks_per_s": blocks / (t_ms * 1e-3),
                     "kernels": "k_evalfull (key bytes read in place; k_unpack first where a wave does not own a key)"},
            "fold": {"kernel_ms": round(f_ms, 4),
                     "kernels": ("k_fold_mfma / k_fold_sliced_direct (bit-sliced DB)" if c.args.pir_fold == "mfma"
                                 else "k_fold_direct / k_fold4r (row-major DB)") + " + k_xor_parts",
                     "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                                  **({"traffic_source": tsrc,
                                      "traffic_over_algorithmic": round(traffic / fold_bytes, 3)} if traffic else {}),
                                  "algorithmic_bytes": fold_bytes,
                                  "note": "DB slice + selection bits read once per batch; the measured streaming-read "
                                          "ceiling of this chip is ~6.17 TB/s (tools/hbm_read.hip)"}}}


def wl_pir(c: Ctx) -> dict:
    a, dpf = c.args, c.dpf
    from dpf import synth
    logN = a.pir_logN
    nrec = 1 << logN
    W = c.world if c.world > 1 else max(1, a.emulate_world)
    # --pir-per-gpu: B queries per server GPU, every GPU folding all B x W of
    # them over its DB slice (weak scaling: per-GPU AES and fold work stay
    # those of one GPU's B-query batch); otherwise B queries in total (strong).
    weak = bool(getattr(a, "pir_per_gpu", False))
    nk = a.batch * W if weak else a.batch
    d_db, lo, hi = pir_setup(c, W)
    ka, result, t_wall, k_ms = pir_time(c, W, d_db, lo, hi, nk, a.steps, a.warmup)
    if a.check and c.rank == 0 and W == c.world:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        full_db = synth.db_bytes(nrec * 32).reshape(nrec, 32)
        for i in range(min(nk, 4)):
            want = oracle.pir_answer(ka[i].tobytes(), logN, full_db, 0, nrec)
            assert result["ans"][i].tobytes() == want, "PIR answer differs from oracle"
    sec = t_wall / a.steps
    pb = (W - 1).bit_length()
    aes = nk * (3 * (1 << (stop_of(logN) - pb)) - 2)
    line = c.line(metric="2-server PIR answered queries/sec per server (EvalFull logN=24 + XOR fold)",
                  value=nk / sec, unit="queries/s", ms_per_step=sec * 1e3, scaling="weak" if weak else "strong",
                  data="synthetic DB (SplitMix64) + keys",
                  config={"workload": f"PIR, DB 2^{logN} x 32 B sharded over {W} GPU(s), batch {nk}"
                                      + (f" ({a.batch} per GPU)" if weak else "")
                                      + f" ({'bitsliced' if dpf.get_aes_impl() else 'lds-ttable'} AES)"
                                      + (" (rank 0's share timed on 1 GPU)" if W != c.world else "")
                                      + " (BASELINE configs[4])", "logN": logN, "batch": nk,
                          "parallelism": f"db-shard x{c.world} + all_gather/XOR"},
                  aes_blocks_per_s=aes * c.world / sec)
    # Which kernel shape the step ran: the fused tree + fold launch
    # (k_pir_fused, dpf_pir_kernel_for) or the tree launch then the fold
    # launch.  The two phases of the two-launch path are timed apart below
    # either way (pir_breakdown).
    fused = a.pir_fold == "mfma" and dpf.pir_kernel_for(nk, logN, pb) == dpf.PIR_FUSED
    kern = pir_breakdown(c, W, d_db, lo, hi, nk, min(a.steps, 20))
    line["kernels"] = kern
    line["pir_kernel"] = "fused" if fused else "split"
    if fused:
        # One launch holds both phases: the roofline is the LDS-bound AES of
        # the tree (lookups/s over the step's kernels: unpack + k_pir_fused +
        # k_xor_parts), and the DB stream it folds on the matrix cores rides
        # under it (its HBM rate beside it, not the bound).
        line["roofline"] = prg_roofline(aes / (k_ms * 1e-3), "k_pir_fused (tree + MFMA fold)", k_ms,
                                        (hi - lo) * 32, workload="pir_fused",
                                        profiled_shape=(W == 1 and nk == 64))
        db_gbs = (hi - lo) * 32 / (k_ms * 1e-3) / 1e9
        line["roofline"]["fold"] = {"bound": "hbm (not binding: under the tree in the same launch)",
                                    "achieved": round(db_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": round(db_gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": (hi - lo) * 32,
                                    "note": "DB slice read once per batch; the selection bits stay in LDS"}
        line["roofline"]["split_path_ms"] = round(kern["tree"]["kernel_ms"] + kern["fold"]["kernel_ms"], 4)
    else:
        line["roofline"] = prg_roofline(aes / (kern["tree"]["kernel_ms"] * 1e-3), "k_evalfull (PIR tree)",
                                        kern["tree"]["kernel_ms"], nk * ((hi - lo) // 8), workload="pir",
                                        profiled_shape=(W == 1 and nk == 64))
        line["roofline"]["fold"] = kern["fold"]["roofline"]
    line["roofline"]["step_kernel_ms"] = round(k_ms, 4)
    line["pir_db"] = c.pir_layout
    if c.world == 1 and not a.no_sweep:
        # B in {1, 16, 64, 256}; the fold reads the DB once per
        # batch up to 256 keys (pir_kernels.hip plan_fold).
        sweep = {}
        for b in (1, 16, 64, 256):
            _, _, tw, km = pir_time(c, W, d_db, lo, hi, b, 20, 3)
            sweep[str(b)] = {"ms_per_step": round(tw / 20 * 1e3, 4), "queries_per_s": b / (tw / 20),
                             "kernel_ms": round(km, 4),
                             "aes_blocks_per_s": b * (3 * (1 << (stop_of(logN) - pb)) - 2) / (km * 1e-3),
                             "db_GBs": round((hi - lo) * 32 / (km * 1e-3) / 1e9, 1)}
        line["batch_sweep"] = sweep
    return line


def sub_workloads(c: Ctx) -> dict:
    """BASELINE configs[2..4] measured in the same process after the
    headline's timed region, each through its own timed loop (barrier +
    synchronize, max over ranks): compact forms of the --workload eval /
    split / pir lines, so the default run (what the driver records) shows all
    four GPU configs.  Their CPU baselines are added by finalize()."""
    a = c.args
    saved = dict(vars(a))
    a.steps, a.warmup = min(a.steps, 20), min(a.warmup, 5)
    a.no_api, a.no_sweep, a.emulate_world = True, True, 1
    out = {}
    # At N > 1 the PIR server is also timed in its weak form (--batch queries
    # per GPU): at N = 1 it is the same run as "pir".
    runs = [("eval", wl_eval, False), ("split", wl_split, False), ("pir", wl_pir, False)]
    if c.world > 1:
        runs.append(("pir_weak", wl_pir, True))
    try:
        for name, fn, per_gpu in runs:
            a.pir_per_gpu = per_gpu
            ln = fn(c)
            keep = {k: ln[k] for k in ("metric", "value", "unit", "ms_per_step", "scaling", "aes_blocks_per_s")}
            keep["steps"] = a.steps
            keep["workload"] = ln["config"]["workload"]
            keep["roofline"] = {k: ln["roofline"][k] for k in ("bound", "achieved", "peak", "unit", "frac",
                                                             "kernel", "kernel_ms", "traffic")
                                if k in ln["roofline"]}
            if "gate" in ln["roofline"]:
                keep["roofline"]["gate_frac"] = ln["roofline"]["gate"]["frac"]
            for k in ("kernels", "pir_db"):
                if k in ln:
                    keep[k] = ln[k]
            out[name] = keep
    finally:
        vars(a).update(saved)
    return out


def spawn_ranks(n: int) -> int:
    """`python bench.py --gpus N` outside a launcher: start N ranks through
    torch.distributed.run as a CHILD process (nothing here has touched a GPU)
    and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def dry_run(args) -> None:
    """The rank/launch/timing skeleton of a real run without a device: gloo
    barrier around a no-op step, max-over-ranks time, one line from rank 0."""
    import torch
    import torch.distributed as dist
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    t = torch.tensor([time.perf_counter() - t0 + rank * 1e-6], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
    if rank == 0:
        # The line skeleton goes through the real policy code: traffic only
        # for a profiled per-rank shape, cpu_baseline on rank 0 at every N.
        wl = args.workload
        same_shape = wl in ("evalfull", "eval") or world == 1
        line = {"dry_run": True, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "max_rank_s": float(t.item()), "local_ranks": os.environ.get("LOCAL_WORLD_SIZE"),
                "workload": wl,
                "scaling": "strong" if wl == "split" or (wl == "pir" and not args.pir_per_gpu) else "weak"}
        line["roofline"] = prg_roofline(1e11, "k_evalfull<7, true, false>", 1.0, 512 << 20, workload=wl,
                                        profiled_shape=same_shape)
        finalize(line, args, world, folded=False)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", choices=["evalfull", "eval", "split", "pir"], default="evalfull")
    ap.add_argument("--logN", type=int, default=20)
    ap.add_argument("--nkeys", type=int, default=4096)
    ap.add_argument("--eval-keys", type=int, default=1 << 16)
    ap.add_argument("--eval-points", type=int, default=1 << 10)
    ap.add_argument("--split-logN", type=int, default=32)
    ap.add_argument("--pir-logN", type=int, default=24)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--pir-fold", choices=["mfma", "lds"], default="mfma",
                    help="pir: XOR fold on the matrix cores over the bit-sliced DB (default) or the LDS fold")
    ap.add_argument("--pir-per-gpu", action="store_true",
                    help="pir: --batch queries per GPU (total batch B x N, weak scaling) instead of B in total")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="split/pir on 1 GPU: time rank 0's share of a W-way split")
    ap.add_argument("--event-every", type=int, default=10,
                    help="record kernel timing events on every n-th timed step (1 = every step, 0 = none)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--aes", choices=["ttable", "bitsliced"], default=None,
                    help="tree-kernel AES back end for the headline (default: the library's)")
    ap.add_argument("--no-variants", action="store_true", help="skip timing the other AES back end")
    ap.add_argument("--pipelined", action="store_true",
                    help="evalfull: also time batches alternating over two streams (reported as 'pipelined')")
    ap.add_argument("--no-api", action="store_true", help="skip the host-buffer (PCIe-inclusive) API rates")
    ap.add_argument("--no-sweep", action="store_true", help="pir: skip the B in {1,16,64,256} batch sweep")
    ap.add_argument("--strong", action="store_true",
                    help="evalfull: split a fixed --nkeys over the ranks (strong scaling) instead of --nkeys per rank")
    ap.add_argument("--no-workloads", action="store_true",
                    help="evalfull: skip the configs[2..4] sub-lines (workloads) of the default run")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--spinup", type=float, default=0.5,
                    help="seconds of untimed steps before the warmup (GPU clock ramp); 0 disables")
    ap.add_argument("--check", action="store_true", help="verify a sample of outputs against the oracle")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/collective plumbing only (gloo, no GPU): what the CPU tests run")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world and world > 1:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    if args.dry_run:
        dry_run(args)
        return
    c = Ctx(args)
    line = {"evalfull": wl_evalfull, "eval": wl_eval, "split": wl_split, "pir": wl_pir}[args.workload](c)
    if args.workload == "evalfull" and not (args.no_workloads or args.strong or args.emulate_world > 1):
        line["workloads"] = sub_workloads(c)
    if c.rank == 0:
        args.ref_gpu = getattr(c, "reference_shapes", {})
        finalize(line, args, c.world, c.folded)
        print(json.dumps(line), flush=True)
    if c.world > 1:
        c.dist.destroy_process_group()


def finalize(line: dict, args, world: int, folded: bool) -> None:
    """Rank 0, after the timed region.  The headline carries the CPU
    baseline at every N (taken after the timed steps, so it cannot perturb
    them).  Ranks folded onto fewer GPUs than ranks are a rehearsal of the
    N-rank plumbing, not an N-GPU number: marked, and no scaling class."""
    if not args.no_cpu_baseline:
        if args.workload == "evalfull":
            line["cpu_baseline"] = cpu_baseline(args.logN, args.cpu_seconds)
            if world == 1 and not args.no_api:
                line["cpu_baseline"]["reference_shapes"] = reference_shapes_cpu(getattr(args, "ref_gpu", {}))
        elif args.workload == "split":
            line["cpu_baseline"] = cpu_baseline(20, min(args.cpu_seconds, 8.0))
            line["cpu_baseline"]["note"] = ("points/s of the batched EvalFull port at logN=20: the per-point "
                                            "rate of a logN=32 EvalFull on the same code")
        elif args.workload == "eval":
            line["cpu_baseline"] = cpu_baseline_eval(args.logN, args.eval_keys, args.eval_points,
                                                     min(args.cpu_seconds, 8.0))
        elif args.workload == "pir":
            line["cpu_baseline"] = cpu_baseline_pir(args.pir_logN, args.batch, min(args.cpu_seconds, 8.0))
        wls = line.get("workloads", {})
        sub_s = min(args.cpu_seconds, 4.0)
        if "eval" in wls:
            wls["eval"]["cpu_baseline"] = cpu_baseline_eval(args.logN, args.eval_keys, args.eval_points, sub_s)
        if "split" in wls:
            wls["split"]["cpu_baseline"] = cpu_baseline(20, sub_s)
            wls["split"]["cpu_baseline"]["note"] = "points/s of the batched EvalFull port at logN=20"
        if "pir" in wls:
            wls["pir"]["cpu_baseline"] = cpu_baseline_pir(args.pir_logN, args.batch, sub_s)
    if folded:
        line["folded_ranks"] = True
        line["scaling"] = None
        line["note"] = f"{world} ranks folded onto fewer GPUs (rehearsal): value is not an {world}-GPU rate"


if __name__ == "__main__":
    main()
