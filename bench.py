"""VBOC boundary OCP solves/sec - triple pendulum, 1..8 MI355X (BASELINE.json metric).

Workloads (--workload):
  dg-loop      (default) one step = the reference's data-generation loop over B problems per GPU:
               `data_generation(v)` of VBOC/triplependulum_vboc.py:19-370 for every problem id, i.e. IC
               sampling, up to 10 horizon-extension solves, the sweep with its twin RK4 steps and the
               verification solves, the save filter - the whole state machine on the device, one problem
               per wave with the wave solver in between (vboc_data_generation, vboc_amd/csrc/dg.h) - then
               X_save in problem order and (N > 1) the RCCL all-gather of every rank's samples that feeds
               the NN fit.  value = OCP solves (all of them) / s; also boundary problems / s.
               The W warmup steps and the K timed steps are each issued as ONE persistent launch over their
               W*B / K*B problems: a launch is bound by throughput plus its single slowest problem (the
               critical problem, reported under loop.tail), which a launch per step would pay K times.
               Default B = 20k (the driver's 5 + 20 steps then cover configs[2]'s 100k states five times).
               The warmup launch (W * B problems; 5 x 20k = 100k = one configs[2] round at the driver's
               command) is timed too and reported as loop.configs2_round: a single round pays its own tail.
  first-solve  one step = the first OCP solve of data_generation for B problems (IC law, straight-line
               guess, N = 100) on the wave solver, inputs resident in HBM, then (N > 1) the all-gather of
               the boundary states x0.  The inputs of `--max-batches` distinct batches (ids of steps
               0 .. max_batches - 1) are built before timing; step s solves batch s mod max_batches.
dg-loop problem ids are a global counter (Philox per id): rank r takes ids [(step * world + r) * B, ... + B), so
per-GPU work is fixed as N grows (weak scaling).
`value` counts OCP solves: for the dg-loop every solve the loop issues (its first, horizon-extension and
verification solves, ~4.4 per problem for the triple - `value_counts` in the line says so), for first-solve
one per problem; loop.boundary_problems_per_s is the per-problem rate.  The two workloads' values are not
comparable with each other.

Output: ONE JSON line on rank 0 (contract in the task statement), with
  roofline     the dominant kernel (k_dg / k_wave: the whole step is one launch): algorithmic FP64 flops of
               the launch by the SURVEY 8(d) convention with the solver's reported iteration counts, over
               its duration (HIP events on the solve stream, vboc_last_kernel_ms), priced against the FP64
               dense peak (78.6 TFLOP/s; the Riccati factorisation runs on v_mfma_f64_16x16x4f64, the rest
               on the FP64 VALU at the same peak).  traffic: memory-side bytes per launch from the committed
               rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE, profiles/*_pmc_<kernel>.json).
  tail         the launch's critical problem (longest single problem on one wave), when the job queue
               drained and when the last problem finished (device real-time clock; dg-loop).
  cpu_baseline the oracle's C restatement (oracle/, test infrastructure) on a bounded sample of the same
               workload on the host's cores, rank 0, N = 1 only.
`run(args, engine_factory)` takes another engine (tests/test_distributed.py runs the N = 2 path on gloo with
the oracle as the engine).

Ranks: launched by torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK in the environment) every process is one
rank.  `python bench.py --gpus N` with no launcher environment starts the N rank processes itself (children of this
process, started before anything here touches the GPU; rank r on GPU r, rendezvous on 127.0.0.1) and exits with
their status - the reference's own fan-out is one command too (`Pool(30).map`, VBOC/triplependulum_vboc.py:399-405).
Every rank checks that the process group's size equals --gpus, and `n_gpus` is the process group's size.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 dense peak, vector and matrix
# SURVEY.md 8(d) algorithmic FLOP convention (triple n=7, m=3; double n=5, m=2; pendulum n=3, m=1)
F_DYN = {3: 6382, 2: 2146, 1: 4 * 14 + 8 * 9 * 4 + 8 * 3 * 4 + 6}
F_IPM = {3: 3513, 2: 1346, 1: int(2 * 9 * 4 + 2 * 3 * 16 + 64 / 3 + 8 * 16)}
C_F = {3: 183, 2: 52, 1: 8}


def _ur5_counts():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "flops.json"))).get("4")
    return (d["C_f"], d["C_fJ"]) if d else (None, None)


# UR5 arm (config 5, n = 8, m = 4): same convention; C_f / C_fJ are the sympy CSE op counts of the
# urdf2casadi-style ABA restatement (oracle/ur5_rbd.py, tools/ur5_flops.py -> tests/golden/flops.json "4")
_UR5_CF, _UR5_CFJ = _ur5_counts()
if _UR5_CF:
    _n, _m = 8, 4
    F_DYN[4] = 4 * _UR5_CFJ + 8 * _n * _n * (_n + _m) + 8 * _n * (_n + _m) + 2 * _n
    F_IPM[4] = int(2 * _n * _n * (_n + _m) + 2 * _n * (_n + _m) ** 2 + (_n + _m) ** 3 / 3 + 8 * (_n + _m) ** 2)
    C_F[4] = _UR5_CF

NAMES = {1: "pendulum", 2: "double pendulum", 3: "triple pendulum", 4: "UR5 arm"}
WORKLOAD = {
    ("dg-loop", 3): "triple-pendulum data_generation loop (VBOC/triplependulum_vboc.py:19-370), {B} problems per GPU "
                    "per step: every OCP solve (horizon extension + verification) and twin step on the device "
                    "(configs[2]; configs[3] at 8 GPUs)",
    ("dg-loop", 2): "double-pendulum data_generation loop (VBOC/doublependulum_vboc.py:19-403), {B} problems per GPU "
                    "per step (configs[1])",
    ("first-solve", 3): "triple-pendulum data_generation first OCP solve, N=100, {B} ICs per GPU per step "
                        "(configs[2]; configs[3] at 8 GPUs)",
    ("first-solve", 2): "double-pendulum data_generation first OCP solve, N=100, {B} ICs per GPU per step (configs[1])",
    ("first-solve", 1): "pendulum data_generation first OCP solve, N=50, {B} ICs per GPU per step",
    ("first-solve", 4): "UR5 (4 revolute joints of ur5.urdf) testing_test first OCP solve, N=100, {B} ICs per GPU "
                        "per step (configs[4]: 100k states; 8 GPUs at N=8)",
}


def pmc_traffic(kernel, problems=None):
    """HBM traffic per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/*_pmc_<kernel>.json, made by tools/pmc_summary.py from FETCH_SIZE / WRITE_SIZE passes of
    this bench command, gfx950-corrected); for the dg-loop (launch sizes differ) the per-problem figure
    scaled to `problems`.  None if there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{kernel}.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    src = os.path.relpath(files[-1], ROOT)
    if problems is not None and "traffic_bytes_per_problem" in d:
        return d["traffic_bytes_per_problem"] * problems / 1e9, src + " (per problem x problems per launch)"
    return d["traffic_bytes_per_launch"] / 1e9, src


def dg_counters():
    """The newest committed driver-shape counter summary of k_dg (profiles/*_k_dg_counters.json, tools/pmc_r04.py over
    the rocprofv3 --pmc passes of tools/gpu_run.sh pmc=...): (summary dict, path) or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_k_dg_counters.json")))
    if not files:
        return None, None
    return json.load(open(files[-1])), os.path.relpath(files[-1], ROOT)


def dg_bound_note(c, src):
    """bound_note of the dg-loop line, computed from the committed counters (verdict r03 item 4)."""
    w, m = c["wave_time_split"], c["memory_side"]
    note = ("'mfma' = the FP64 compute roofline SURVEY.md 8(d) prices the path on (algorithmic FP64 flops); what the "
            f"counters of the driver-shape launch show ({src}): waves {w['issuing']:.0%} issuing (VALU "
            f"{w['issuing_valu']:.0%}, LDS {w['issuing_lds']:.0%}, SALU {w['issuing_salu']:.0%}), "
            f"{w['issue_stalled_dependency_pipe']:.0%} stalled on a dependency or pipe, {w['waiting_s_waitcnt_barrier']:.0%} "
            f"in s_waitcnt; FP64 MFMA busy {c['mfma_busy_share']:.1%}; memory side {m['tb_per_s']:.2f} TB/s "
            f"({m['bytes_per_stage_ipm_iteration'] / 1e3:.1f} KB per stage-IPM-iteration, L2 hit {c['l2_hit_rate']:.0%})")
    ab = c.get("bytes_ab")
    if ab:
        note += "; " + ab["summary"]
    return note


def dg_flops(nq, stats):
    """SURVEY 8(d) FP64 flops of a data-generation launch from its per-problem stats (lib.DG_STATS):
    sum over solves of N*(F_dyn*K_sqp + F_ipm*K_ipm + 8*C_f*K_sqp), plus 4*C_f per twin step."""
    return float(np.sum((F_DYN[nq] + 8 * C_F[nq]) * stats[:, 3] + F_IPM[nq] * stats[:, 4] + 4 * C_F[nq] * stats[:, 1]))


def make_batch(nq, ids, device):
    import torch
    from vboc_amd.ics import data_generation_ics, ur5_ics
    b = ur5_ics(ids) if nq == 4 else data_generation_ics(nq, ids)
    keys = ("N", "x_guess", "u_guess", "p", "lbx", "ubx", "lbu", "ubu", "lbx0", "ubx0", "lbxe", "ubxe")
    return {k: torch.as_tensor(np.ascontiguousarray(b[k]), device=device) for k in keys}


def order_rows(out):
    """X_save in problem order (VBOC/triplependulum_vboc.py:404-405 flattens the results in problem order)
    from the device blocks (one contiguous block per problem, in completion order), on the device."""
    import torch
    cnt = out["row_cnt"].clamp(min=0).to(torch.int64)
    off = out["row_off"]
    tot = int(cnt.sum())
    start = torch.cumsum(cnt, 0) - cnt
    idx = torch.repeat_interleave(off, cnt) + torch.arange(tot, device=cnt.device) - torch.repeat_interleave(start, cnt)
    return out["rows_all"][idx]


class GpuEngine:
    """The product path: libvboc_amd on one GPU (HIP kernels; no CPU fallback)."""

    def __init__(self, nq, args, local):
        import torch
        from vboc_amd import lib
        self.torch, self.lib = torch, lib
        self.device = torch.device("cuda", local)
        torch.cuda.set_device(self.device)
        nmax = 100 + 20 if args.workload == "dg-loop" else 100
        self.solver = lib.Solver(nq, nmax, slots=args.slots, device=local)
        self.solver.set_option("wave_all", 1 if args.mode == "wave" else 0)
        self.solver.set_option("factor_mfma", 1 if args.factor == "mfma" else 0)
        self.solver.set_option("profile_kernels", 1 if args.mode == "lane" else 0)
        self.solver.set_option("dg_spec_early", getattr(args, "spec_early", 0))
        self.solver.set_option("dg_spec_first", getattr(args, "spec_first", 2))
        self.solver.set_option("dg_spec_crit", getattr(args, "spec_crit", 0))
        if getattr(args, "wave_groups", 0):   # resident problems (default: sized to the 256 MiB MALL)
            self.solver.set_option("wave_groups", args.wave_groups)
        self.stream = torch.cuda.current_stream(self.device)
        self.kernel = {("dg-loop", "wave"): f"k_dg<{nq}>", ("first-solve", "wave"): f"k_wave<{nq}>",
                       ("first-solve", "lane"): f"k_qp_factor<{nq}>"}[(args.workload, args.mode)]

    def sync(self):
        self.torch.cuda.synchronize(self.device)

    def first_solve_batch(self, nq, ids):
        return make_batch(nq, ids, self.device)

    def first_solve(self, tb):
        out = self.solver.solve_device(tb, stream=self.stream)
        return dict(x0=out["x"][:, 0, :], status=out["status"], sqp_iter=out["sqp_iter"], qp_iter=out["qp_iter"])

    def dg(self, ids):
        ids_t = self.torch.as_tensor(ids, dtype=self.torch.int64, device=self.device)
        return self.solver.data_generation_device(ids_t, stream=self.stream)

    def kernel_ms(self):
        return self.solver.last_kernel_ms()[0]

    def lane_stats(self):
        return self.solver.kernel_stats()

    def library(self):
        """Which solver build was timed: its path (VBOC_LIB may select a measurement variant) and sha1."""
        path = self.lib.LIB_PATH
        with open(path, "rb") as f:
            digest = hashlib.sha1(f.read()).hexdigest()
        return {"path": os.path.relpath(path, ROOT), "sha1": digest,
                "variant": bool(os.environ.get("VBOC_LIB")),
                "resident_problems": int(self.solver.get_option("last_groups"))}   # of the last launch


def cpu_baseline(nq, workload, B, seconds, threads):
    """Oracle (CPU FP64 restatement, oracle/) on the first problems of the same workload for ~`seconds`:
    first-solve - batches of first solves, one problem per OpenMP thread; dg-loop - the reference's loop at
    full speed: oracle/vboc_dg.c, the C restatement of data_generation (pinned bit for bit to the reference's
    own function), one problem per OpenMP thread with no rounds - as the reference's Pool.map runs it - first
    on 4 problems per thread to size the sample, then on as many as fill the remaining time."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from vboc_amd.ics import data_generation_ics, ur5_ics
    if workload == "dg-loop":
        n, start, solves, t_total = 4 * threads, 0, 0, 0.0
        for _ in range(2):
            t0 = time.time()
            _, st = oracle.data_generation(nq, np.arange(start, start + n), nthreads=threads)
            t_total += time.time() - t0
            solves += st["solves"]
            start += n
            left = seconds - t_total
            if left <= 0.1 * seconds:
                break
            n = max(threads, int(start / t_total * left))
        return solves / t_total, start, solves, t_total
    done, solves, t_total, start = 0, 0, 0.0, 0
    n = max(threads, 8)
    while t_total < seconds and start < B:
        ids = np.arange(start, start + n)
        t0 = time.time()
        b = ur5_ics(ids) if nq == 4 else data_generation_ics(nq, ids)
        oracle.solve_batch(nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                           b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], nthreads=threads)
        solves += n
        t_total += time.time() - t0
        done += n
        start += n
        n = min(4 * n, max(threads, 8) * 64)
    return solves / t_total, done, solves, t_total


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("dg-loop", "first-solve"), default="dg-loop")
    ap.add_argument("--batch", type=int, default=None,
                    help="problems per GPU per step; default 20k for dg-loop (configs[2]'s 100k states every five "
                         "steps), 100k for first-solve")
    ap.add_argument("--nq", type=int, default=3,
                    help="3: triple pendulum (BASELINE metric); 2 / 1: double / pendulum; 4: UR5 arm (configs[4])")
    ap.add_argument("--slots", type=int, default=65536)
    ap.add_argument("--max-batches", type=int, default=4,
                    help="first-solve: distinct input batches held in HBM (steps cycle through them)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--factor", choices=("mfma", "valu"), default="mfma",
                    help="wave solver's Riccati factorisation: FP64 MFMA (default, nq <= 3) or VALU dot-product steps")
    ap.add_argument("--spec-early", type=int, default=0,
                    help="dg-loop: queued speculative restarts go before new problems once this few problems are left "
                         "(0: only once the problem queue is drained)")
    ap.add_argument("--spec-first", type=int, default=2,
                    help="dg-loop: queued speculative restarts go before parked resumes once the new problems run out: "
                         "0 off, 1 on, 2 (default) on for launches of < 128 problems per resident wave (the warmup / "
                         "configs[2] round; DESIGN.md section 14)")
    ap.add_argument("--spec-crit", type=int, default=0,
                    help="dg-loop: 1 = the critical-path rule for speculative restarts (DESIGN.md section 14)")
    ap.add_argument("--mode", choices=("wave", "lane"), default="wave",
                    help="first-solve: wave (one problem per wave, default) or lane (lane-per-problem kernels)")
    ap.add_argument("--wave-groups", type=int, default=0,
                    help="resident problems (persistent workgroups) of the wave solver / data-generation launch "
                         "(0: sized so their hot stage records fit the 256 MiB MALL)")
    ap.add_argument("--progress", type=float, default=0.0,
                    help="print an elapsed-time line to stderr every this many seconds (long runs under a watchdog)")
    ap.add_argument("--engine", default="gpu",
                    help="'gpu' (the product: libvboc_amd) or module:Class of a test engine with GpuEngine's interface "
                         "(CPU tests of the rank launcher only; such a line carries engine = that name)")
    args = ap.parse_args(argv)
    if args.batch is None:
        args.batch = 20_000 if args.workload == "dg-loop" else 100_000
    if args.workload == "dg-loop" and (args.nq not in (2, 3) or args.mode != "wave"):
        ap.error("--workload dg-loop runs the double / triple pendulum on the wave solver")
    return args


def run(args, engine_factory=None):
    """Run the benchmark; returns the JSON line (dict) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    from vboc_amd.dist import gather_boundary_states, gather_samples, shard_ids

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nq, B = args.nq, args.batch
    if engine_factory is None and args.engine != "gpu":
        import importlib
        mod, cls = args.engine.split(":")
        engine_factory = getattr(importlib.import_module(mod), cls)
    engine = (engine_factory or GpuEngine)(nq, args, local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if engine.device.type == "cuda" else "gloo", rank=rank, world_size=world)
        world = dist.get_world_size()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} rank(s) "
                         f"(launch with torch.distributed.run --nproc-per-node {args.gpus}, or without a launcher)")
    dev = engine.device
    beat = _progress(args.progress, rank)
    dgl = args.workload == "dg-loop"

    # first-solve inputs: `max_batches` distinct batches generated and copied to HBM before any timing
    nb = min(args.max_batches, args.warmup + args.steps)
    batches = [] if dgl else [engine.first_solve_batch(nq, shard_ids(s, world, rank, B)) for s in range(nb)]
    rec = dict(solves=0.0, problems=0, rows=0, flops=0.0, kernel_ms=0.0, launches=0, sqp=[], status=[], tail=None,
               stats=None, lane_ms=0.0, lane_launch=0, lane_bytes=0.0)

    def step(s, timed):
        out = engine.first_solve(batches[s % nb])
        if world > 1:
            gather_boundary_states(out["x0"])
        if timed:
            sqp, qpi = out["sqp_iter"].cpu().numpy(), out["qp_iter"].cpu().numpy()
            rec["solves"] += B
            rec["problems"] += B
            rec["flops"] += float(np.sum(100 * (F_DYN[nq] * sqp + F_IPM[nq] * qpi + 2 * 4 * C_F[nq] * sqp)))
            rec["sqp"].append(sqp)
            rec["status"].append(out["status"].cpu().numpy() == 0)
            if args.mode == "lane":
                ms, nl, by = engine.lane_stats()
                rec["lane_ms"] += ms
                rec["lane_launch"] += nl
                rec["lane_bytes"] += by
            else:
                rec["kernel_ms"] += engine.kernel_ms()
                rec["launches"] += 1

    def dg_steps(first, count, timed):
        """`count` consecutive steps as ONE persistent launch over their count * B problems (the launch's
        tail - its slowest problem - is paid once, not once per step), then per step: X_save in problem
        order and (N > 1) the all-gather of every rank's samples."""
        if count == 0:
            return
        ids = np.concatenate([shard_ids(first + k, world, rank, B) for k in range(count)])
        tw = time.perf_counter()
        out = engine.dg(ids)
        if not timed:   # the warmup launch: one round of count * B problems, reported apart (loop.configs2_round)
            engine.sync()
            st = out["stats"].cpu().numpy()
            rec["round"] = dict(problems=int(count * B), wall_s=time.perf_counter() - tw, kernel_ms=engine.kernel_ms(),
                                solves=float(st[:, 0].sum()), stats=st)
        for k in range(count):
            sl = slice(k * B, (k + 1) * B)
            X = order_rows(dict(row_cnt=out["row_cnt"][sl], row_off=out["row_off"][sl], rows_all=out["rows_all"]))
            if world > 1:
                X = gather_samples(X)
            rec["rows"] += X.shape[0] if timed else 0
        if timed:
            st = out["stats"].cpu().numpy()
            rec["solves"] += float(st[:, 0].sum())
            rec["problems"] += count * B
            rec["flops"] += dg_flops(nq, st)
            rec["stats"] = st
            rec["sqp"].append(st[:, 2] / np.maximum(st[:, 0], 1))
            rec["status"].append((out["row_cnt"] >= 0).cpu().numpy())
            rec["kernel_ms"] += engine.kernel_ms()
            rec["launches"] += 1
            rec["spec"] = (int(out.get("spec_solves", 0)), int(out.get("spec_used", 0)))

    if dgl:
        dg_steps(0, args.warmup, False)
    else:
        for s in range(args.warmup):
            step(s, False)
    engine.sync()
    if world > 1:
        dist.barrier()
    engine.sync()
    t0 = time.perf_counter()
    if dgl:
        dg_steps(args.warmup, args.steps, True)
    else:
        for s in range(args.steps):
            step(args.warmup + s, True)
    engine.sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    local_flops, local_solves = rec["flops"], rec["solves"]
    solves, rows = local_solves, rec["rows"]
    if world > 1:
        t = torch.tensor([elapsed, -1.0], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0].item())
        t = torch.tensor([rec["flops"], local_solves], device=dev, dtype=torch.float64)
        dist.all_reduce(t)
        flops, solves = float(t[0].item()), float(t[1].item())   # (gathered rows are already the whole job's)
    else:
        flops = local_flops
    problems = world * args.steps * B
    value = solves / elapsed

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and engine_factory is None:
        threads = len(os.sched_getaffinity(0))
        threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
        v, n, ns, t = cpu_baseline(nq, args.workload, B, args.cpu_seconds, threads)
        what = ("data_generation in C (oracle/vboc_dg.c + vboc_oracle.c), one problem per OpenMP thread" if dgl
                else "first solves on oracle/vboc_oracle.c (OpenMP)")
        cpu = {"value": round(v, 2), "unit": "solves/s", "cores": threads, "kind": "port",
               "sample": f"first {n} problems of the same workload ({ns} OCP solves), {what}, {t:.1f} s"}

    kernel = getattr(engine, "kernel", "k_wave")
    if args.mode == "lane":
        avg_ms = rec["lane_ms"] / max(1, rec["lane_launch"])
        gbs = (rec["lane_bytes"] / max(1, rec["lane_launch"])) / (avg_ms * 1e-3) / 1e9 if rec["lane_launch"] else None
        traffic_gb, src = pmc_traffic("k_qp_factor" if nq == 3 else f"k_qp_factor_nq{nq}")
        roofline = {"bound": "hbm", "achieved": round(gbs, 1) if gbs else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                    "traffic": round(traffic_gb, 4) if traffic_gb else None, "traffic_unit": "GB/launch",
                    "traffic_source": src, "kernel": kernel, "avg_launch_ms": round(avg_ms, 4),
                    "launches": rec["lane_launch"]}
    else:
        pmc_name = ("k_dg" if dgl else "k_wave") + ("" if nq == 3 else f"_nq{nq}")
        traffic_gb, src = pmc_traffic(pmc_name, args.steps * B if dgl else None)
        ctr, ctr_src = dg_counters() if (dgl and nq == 3) else (None, None)
        if ctr is not None and rec["stats"] is not None:
            # bytes per stage-IPM-iteration of the committed driver-shape counters x this launch's stage-IPM-iterations
            traffic_gb = ctr["memory_side"]["bytes_per_stage_ipm_iteration"] * float(rec["stats"][:, 4].sum()) / 1e9
            src = ctr_src + " (bytes per stage-IPM-iteration x this launch's)"
        avg_ms = rec["kernel_ms"] / max(1, rec["launches"])
        per_launch = local_flops / max(1, rec["launches"])
        tf = per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms else None
        roofline = {"bound": "mfma", "achieved": round(tf, 4) if tf else None, "peak": FP64_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(tf / FP64_PEAK_TFLOPS, 5) if tf else None,
                    "traffic": round(traffic_gb, 4) if traffic_gb else None, "traffic_unit": "GB/launch",
                    "traffic_source": src,
                    "bound_note": dg_bound_note(ctr, ctr_src) if ctr is not None else
                                  "'mfma' = the FP64 compute roofline SURVEY.md 8(d) prices the path on; no committed "
                                  "driver-shape counters for this kernel",
                    "pipes": "FP64: Riccati factorisation on v_mfma_f64_16x16x4f64 (factor_mfma), the rest FP64 VALU; "
                             "peak = FP64 dense (vector = matrix on MI355X); latency-bound dependent recursions",
                    "algorithmic": "FP64 flops per launch, SURVEY.md 8(d): sum over solves of "
                                   "N*(F_dyn*K_sqp + F_ipm*K_ipm + 8*C_f*K_sqp)" + (" + 4*C_f per twin step" if dgl else ""),
                    "flops_per_launch": round(per_launch), "kernel": kernel, "avg_launch_ms": round(avg_ms, 3),
                    "launches": rec["launches"]}
    tail = None
    if dgl and rec["stats"] is not None:
        from vboc_amd.lib import DG_CLOCK_HZ
        st = rec["stats"]
        t0s, t1s = st[:, 5], st[:, 6]
        ms = 1e3 / DG_CLOCK_HZ
        tqs = st[:, 9]
        tail = {"critical_problem_ms": round(float((t1s - t0s).max()) * ms, 1),
                "longest_final_run_ms": round(float((t1s - tqs).max()) * ms, 1),
                "mean_problem_ms": round(float((t1s - t0s).mean()) * ms, 2),
                "new_problems_drained_ms": round(float(t0s.max() - t0s.min()) * ms, 1),
                "queue_drained_ms": round(float(st[:, 9].max() - t0s.min()) * ms, 1),
                "last_finish_ms": round(float(t1s.max() - t0s.min()) * ms, 1),
                "note": "last timed launch, device real-time clock from the first problem's start; queue_drained = "
                        "the last job (a new problem or a parked one's resume) taken; a problem's time (critical / mean) "
                        "runs from its first solve to its end and includes the wait of a parked first solve, "
                        "longest_final_run = the longest stretch from a problem's last job start to its end"}
        tail["after_drain_share"] = round(1.0 - tail["queue_drained_ms"] / max(tail["last_finish_ms"], 1e-9), 3)
        tail["stage_ipm_iters"] = float(st[:, 4].sum())   # sum of N x QP iterations over the launch's solves
    sqp = np.concatenate(rec["sqp"]) if rec["sqp"] else np.zeros(1)
    ok = np.concatenate(rec["status"]) if rec["status"] else np.zeros(1)
    if beat is not None:
        beat.set()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return None
    line = {
        "metric": "VBOC boundary OCP solves/sec, triple pendulum, 1/2/4/8 MI355X" if nq == 3 else
                  f"VBOC boundary OCP solves/sec, {NAMES[nq]}, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Philox-seeded ICs by the reference's " +
                ("testing_test law, VBOC/UR5/vboc_multiprocessing_ur5.py)" if nq == 4 else "data_generation law)"),
        "config": {"workload": WORKLOAD[(args.workload, nq)].format(B=B), "problems_per_gpu": B,
                   "horizon_start": 100, "parallelism": f"dp{world}", "mode": args.mode,
                   "allgather": ("samples" if dgl else "x0") if world > 1 else None},
        "roofline": roofline,
        "path_fp64": {"achieved": round(flops / elapsed / 1e12, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(flops / elapsed / 1e12 / FP64_PEAK_TFLOPS, 5)},
        "cpu_baseline": cpu,
        "library": engine.library() if hasattr(engine, "library") else {"engine": args.engine},
        "solver": {"ok_frac": round(float(np.mean(ok)), 4), "sqp_iter_mean": round(float(sqp.mean()), 1),
                   "sqp_iter_max": round(float(sqp.max()), 1)},
    }
    if dgl:
        line["value_counts"] = ("loop solves: every OCP solve the data-generation loop issues (first, horizon-extension "
                                "and verification solves)")
        line["loop"] = {"boundary_problems_per_s": round(problems / elapsed, 2),
                        "solves_per_problem": round(solves / problems, 3),
                        "samples": int(rows), "samples_per_s": round(rows / elapsed, 1), "tail": tail,
                        "speculative_restarts": {"run_by_other_waves": rec.get("spec", (0, 0))[0],
                                                 "used": rec.get("spec", (0, 0))[1],
                                                 "note": "solves of later attempts of failed horizon-extension "
                                                         "chains run ahead on waves the problem queue no longer "
                                                         "feeds; only used ones are in value (as the problem's "
                                                         "own solves)"}}
        rd = rec.get("round")
        if rd is not None and rank == 0:
            from vboc_amd.lib import DG_CLOCK_HZ
            st = rd["stats"]
            ms = 1e3 / DG_CLOCK_HZ
            line["loop"]["configs2_round"] = {
                "problems": rd["problems"], "solves": int(rd["solves"]),
                "solves_per_s": round(rd["solves"] / rd["wall_s"], 2),
                "boundary_problems_per_s": round(rd["problems"] / rd["wall_s"], 2),
                "wall_s": round(rd["wall_s"], 2), "kernel_ms": round(rd["kernel_ms"], 1),
                "critical_problem_ms": round(float((st[:, 6] - st[:, 5]).max()) * ms, 1),
                "queue_drained_ms": round(float(st[:, 9].max() - st[:, 5].min()) * ms, 1),
                "note": "the warmup launch: W x B problems as ONE round (5 x 20k = configs[2]'s 100k states at the "
                        "driver's command), wall time incl. the first launch; rank 0's shard"}
    if world > 1:
        dist.destroy_process_group()
    return line


def _progress(period, rank):
    """A daemon thread printing the elapsed time to stderr every `period` s (0: none); set() the returned event
    to stop it."""
    if not period or period <= 0:
        return None
    stop, t0 = threading.Event(), time.time()

    def beat():
        while not stop.wait(period):
            print(f"bench rank {rank}: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    return stop


def spawn_ranks(argv, n):
    """`bench.py --gpus n` without a launcher: n child processes of this one, rank r on GPU r (LOCAL_RANK), one
    rendezvous on 127.0.0.1 (a free port).  Nothing in this process touches the GPU.  Rank 0 prints the line; a
    failing rank ends the others.  Returns the exit status (the first non-zero one)."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code   # killed by a signal: the shell's convention
                for q in live:        # our own children, by PID
                    q.terminate()
        time.sleep(0.2)
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(argv, args.gpus))
    line = run(args)
    if line is not None:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
