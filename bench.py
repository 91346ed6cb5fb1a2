"""VBOC boundary OCP solves/sec - triple pendulum, 1..8 MI355X (BASELINE.json metric).

One step = one batched solve of B boundary OCPs (the first solve of `data_generation`,
VBOC/triplependulum_vboc.py:32-110: IC law, straight-line guess, N = 100) on each GPU, inputs
already resident in HBM, followed (N > 1) by the RCCL all-gather of the boundary states x0 that
feeds the NN fit (configs[3]).  Problem ids are a global counter (Philox per id), so rank r solves
ids [(step * world + r) * B, ... + B): per-GPU work is fixed as N grows (weak scaling).

Output: ONE JSON line on rank 0 (contract in the task statement), with
  roofline     the dominant kernel.  Default (wave mode) k_wave, the whole solve in one launch per
               step: algorithmic FP64 work of the launch by the SURVEY 8(d) convention / its duration
               (HIP events on the solve stream, vboc_last_kernel_ms); bound "mfma" = the FP64 dense
               peak (78.6 TFLOP/s; vector and matrix are equal on MI355X).  --mode lane: the lane-mode
               dominant kernel k_qp_factor, algorithmic bytes / duration (vboc_kernel_stats), bound "hbm".
               traffic: HBM bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE x2 +
               WRITE_SIZE, profiles/*_pmc_<kernel>.json).
  cpu_baseline the oracle's C restatement (oracle/, test infrastructure) on a bounded sample of the
               same workload on the host's cores, rank 0, N = 1 only.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector peak
# SURVEY.md 8(d) algorithmic FLOP convention (triple n=7, m=3; double n=5, m=2; pendulum n=3, m=1)
F_DYN = {3: 6382, 2: 2146, 1: 4 * 14 + 8 * 9 * 4 + 8 * 3 * 4 + 6}
F_IPM = {3: 3513, 2: 1346, 1: int(2 * 9 * 4 + 2 * 3 * 16 + 64 / 3 + 8 * 16)}
C_F = {3: 183, 2: 52, 1: 8}
# UR5 arm (config 5, n = 8, m = 4): same convention; C_f / C_fJ are the sympy CSE op counts of the
# urdf2casadi-style ABA restatement (oracle/ur5_rbd.py, tools/ur5_flops.py -> tests/golden/flops.json "4")
_UR5_CF, _UR5_CFJ = None, None


def _ur5_counts():
    import json as _j
    d = _j.load(open(os.path.join(ROOT, "tests", "golden", "flops.json"))).get("4")
    return (d["C_f"], d["C_fJ"]) if d else (None, None)


_UR5_CF, _UR5_CFJ = _ur5_counts()
if _UR5_CF:
    _n, _m = 8, 4
    F_DYN[4] = 4 * _UR5_CFJ + 8 * _n * _n * (_n + _m) + 8 * _n * (_n + _m) + 2 * _n
    F_IPM[4] = int(2 * _n * _n * (_n + _m) + 2 * _n * (_n + _m) ** 2 + (_n + _m) ** 3 / 3 + 8 * (_n + _m) ** 2)
    C_F[4] = _UR5_CF


def pmc_traffic(kernel):
    """HBM traffic per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/*_pmc_<kernel>.json, made by tools/pmc_summary.py from FETCH_SIZE / WRITE_SIZE passes of
    this bench command, gfx950-corrected).  None if there is none."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{kernel}.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    return d["traffic_bytes_per_launch"] / 1e9, os.path.relpath(files[-1], ROOT)


def make_batch(nq, ids, device):
    import torch
    from vboc_amd.ics import data_generation_ics, ur5_ics
    b = ur5_ics(ids) if nq == 4 else data_generation_ics(nq, ids)
    keys = ("N", "x_guess", "u_guess", "p", "lbx", "ubx", "lbu", "ubu", "lbx0", "ubx0", "lbxe", "ubxe")
    return {k: torch.as_tensor(np.ascontiguousarray(b[k]), device=device) for k in keys}, b


def cpu_baseline(nq, B, seconds, threads):
    """Oracle (CPU FP64 restatement) on the first problems of the workload for ~`seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from vboc_amd.ics import data_generation_ics, ur5_ics
    done, t_total, n = 0, 0.0, max(threads, 8)
    start = 0
    while t_total < seconds and start < B:
        b = ur5_ics(np.arange(start, start + n)) if nq == 4 else data_generation_ics(nq, np.arange(start, start + n))
        t0 = time.time()
        oracle.solve_batch(nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                           b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], nthreads=threads)
        t_total += time.time() - t0
        done += n
        start += n
        n = min(4 * n, max(threads, 8) * 64)
    return done / t_total, done, t_total


NAMES = {1: "pendulum", 2: "double pendulum", 3: "triple pendulum", 4: "UR5 arm"}
WORKLOAD = {
    3: "triple-pendulum data_generation first OCP solve, N=100, {B} ICs per GPU per step (configs[2]; configs[3] "
       "at 8 GPUs)",
    2: "double-pendulum data_generation first OCP solve, N=100, {B} ICs per GPU per step (configs[1])",
    1: "pendulum data_generation first OCP solve, N=50, {B} ICs per GPU per step",
    4: "UR5 (4 revolute joints of ur5.urdf) testing_test first OCP solve, N=100, {B} ICs per GPU per step "
       "(configs[4]: 100k states; 8 GPUs at N=8)",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=100_000, help="problems per GPU per step (configs[2]: 100k)")
    ap.add_argument("--nq", type=int, default=3,
                    help="3: triple pendulum (BASELINE metric); 2 / 1: double / pendulum; 4: UR5 arm (configs[4])")
    ap.add_argument("--slots", type=int, default=65536)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--factor", choices=("mfma", "valu"), default="mfma",
                    help="wave solver's Riccati factorisation: FP64 MFMA (default, nq <= 3) or VALU dot-product steps")
    ap.add_argument("--mode", choices=("wave", "lane"), default="wave",
                    help="wave: one problem per wave (default); lane: lane-per-problem kernels + wave tail")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from vboc_amd import lib
    nq, B = args.nq, args.batch
    solver = lib.Solver(nq, 100, slots=args.slots, device=local)
    solver.set_option("wave_all", 1 if args.mode == "wave" else 0)
    solver.set_option("factor_mfma", 1 if args.factor == "mfma" else 0)
    solver.set_option("profile_kernels", 1 if args.mode == "lane" else 0)
    stream = torch.cuda.current_stream(device)

    from vboc_amd.dist import gather_boundary_states, shard_ids

    def ids_for(step):
        return shard_ids(step, world, rank, B)

    # inputs for every step generated and copied to HBM before any timing
    batches = [make_batch(nq, ids_for(s), device)[0] for s in range(args.warmup + args.steps)]
    outs = []

    def run_step(tb):
        out = solver.solve_device(tb, stream=stream)
        if world > 1:
            out["gathered"] = gather_boundary_states(out["x"][:, 0, :])
        return out

    for s in range(args.warmup):
        run_step(batches[s])
    torch.cuda.synchronize(device)

    fact_ms, fact_launch, fact_bytes = 0.0, 0, 0.0
    wave_ms, wave_launch = 0.0, 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s in range(args.steps):
        outs.append(run_step(batches[args.warmup + s]))
        if args.mode == "lane":
            ms, nl, by = solver.kernel_stats()
            fact_ms += ms
            fact_launch += nl
            fact_bytes += by
        else:
            ms, _ = solver.last_kernel_ms()
            wave_ms += ms
            wave_launch += 1
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    status = torch.cat([o["status"] for o in outs]).cpu().numpy()
    sqp = torch.cat([o["sqp_iter"] for o in outs]).cpu().numpy()
    qpi = torch.cat([o["qp_iter"] for o in outs]).cpu().numpy()
    # whole-path FP64 work by the SURVEY 8(d) convention, with the solver's reported K_sqp and K_ipm;
    # K_ls counted as 2 merit evaluations per SQP iteration (phi(0) + one trial: a lower bound)
    Nh = 100
    flops = float(np.sum(Nh * (F_DYN[nq] * sqp + F_IPM[nq] * qpi + 2 * 4 * C_F[nq] * sqp)))
    local_flops = flops
    if world > 1:
        ft = torch.tensor([flops], device=device, dtype=torch.float64)
        dist.all_reduce(ft)
        flops = float(ft.item())
    total = world * args.steps * B
    value = total / elapsed
    avg_launch_ms = fact_ms / max(1, fact_launch)
    achieved_gbs = (fact_bytes / max(1, fact_launch)) / (avg_launch_ms * 1e-3) / 1e9 if fact_launch else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = len(os.sched_getaffinity(0))
        threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
        v, n, t = cpu_baseline(nq, B, args.cpu_seconds, threads)
        cpu = {"value": round(v, 2), "unit": "solves/s", "cores": threads, "kind": "port",
               "sample": f"first {n} problems of the same workload (oracle/vboc_oracle.c, OpenMP, {t:.1f} s)"}

    if args.mode == "lane":
        traffic_gb, traffic_src = pmc_traffic("k_qp_factor" if nq == 3 else f"k_qp_factor_nq{nq}")
        roofline = {"bound": "hbm", "achieved": round(achieved_gbs, 1) if achieved_gbs else None,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved_gbs / HBM_PEAK_GBS, 4) if achieved_gbs else None,
                    "traffic": round(traffic_gb, 4) if traffic_gb else None, "traffic_unit": "GB/launch",
                    "traffic_source": traffic_src,
                    "algorithmic_gb_per_launch": round(fact_bytes / max(1, fact_launch) / 1e9, 4),
                    "kernel": f"k_qp_factor<{nq}>", "avg_launch_ms": round(avg_launch_ms, 4),
                    "launches": fact_launch}
    else:
        # PMC passes are per instantiation (profiles/*_pmc_k_wave.json is the triple's k_wave<3>)
        traffic_gb, traffic_src = pmc_traffic("k_wave" if nq == 3 else f"k_wave_nq{nq}")
        avg_ms = wave_ms / max(1, wave_launch)
        per_launch = local_flops / max(1, args.steps)
        wave_tf = per_launch / (avg_ms * 1e-3) / 1e12 if wave_ms else None
        roofline = {"bound": "mfma", "achieved": round(wave_tf, 4) if wave_tf else None,
                    "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(wave_tf / FP64_PEAK_TFLOPS, 5) if wave_tf else None,
                    "traffic": round(traffic_gb, 4) if traffic_gb else None, "traffic_unit": "GB/launch",
                    "traffic_source": traffic_src,
                    "algorithmic": "FP64 flops per launch, SURVEY.md 8(d): N*(F_dyn*K_sqp + F_ipm*K_ipm + 8*C_f*K_sqp)",
                    "flops_per_launch": round(per_launch), "kernel": f"k_wave<{nq}>",
                    "avg_launch_ms": round(avg_ms, 3), "launches": wave_launch}
    if rank == 0:
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
            "config": {"workload": WORKLOAD[nq].format(B=B),
                       "problems_per_gpu": B, "horizon": 100, "parallelism": f"dp{world}", "mode": args.mode,
                       "allgather": world > 1},
            "roofline": roofline,
            "path_fp64": {"achieved": round(flops / elapsed / 1e12, 4), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(flops / elapsed / 1e12 / FP64_PEAK_TFLOPS, 5),
                          "convention": "SURVEY.md 8(d): N*(F_dyn*K_sqp + F_ipm*K_ipm + 8*C_f*K_sqp)"},
            "cpu_baseline": cpu,
            "solver": {"status_ok_frac": round(float(np.mean(status == 0)), 4),
                       "sqp_iter_mean": round(float(sqp.mean()), 1), "sqp_iter_max": int(sqp.max())},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
