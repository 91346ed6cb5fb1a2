"""Summary of k_dg's counters at the driver's launch shape (tools/gpu_run.sh pmc=...: bench.py --steps 20 --warmup 5,
one rocprofv3 --pmc pass per counter group), for the TIMED launch (the largest k_dg dispatch; the warmup launch is
a quarter of its size).  Verdict r03 item 4.

Per launch: the wave-state split (SQ_WAVE_CYCLES = waiting on s_waitcnt + stalled on a dependency/pipe + issuing;
the counters count quad-cycles, ratios only), the instruction mix per stage-IPM-iteration (the launch's sum of
N x QP iterations, from the bench line), memory-side bytes (FETCH_SIZE x 2 + WRITE_SIZE: 128-B lines, calibrated
in round 4 on the product's own window shapes, profiles/r04_fetch_size_calibration.json) per launch, per
stage-IPM-iteration and per second, the L2 hit rate, FP64 MFMA busy share and the effective clock.

usage: python tools/pmc_r04.py <dir with sqa/ sqb/ fetch/ write/ tcc/ mfma/ and bench_*.json> > profiles/r05_k_dg_counters.json
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_dg"


def launch_counters(path):
    """{counter: value} of the largest k_dg dispatch in one pass (by SQ_WAVE_CYCLES / FETCH_SIZE / first counter)."""
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    by = {}
    for r in rows:
        d = by.setdefault(r["Dispatch_Id"], {"_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if not by:
        return {}
    return max(by.values(), key=lambda d: d["_ns"])


def main():
    root = sys.argv[1]
    c, dur = {}, {}
    for p in ("sqa", "sqb", "fetch", "write", "tcc", "mfma"):
        f = glob.glob(os.path.join(root, p, "**", "*counter_collection.csv"), recursive=True)
        if f:
            d = launch_counters(f[0])
            dur[p] = d.pop("_ns", None)
            c.update(d)
    bench = None
    for p in ("sqa", "fetch", "sqb", "write", "tcc", "mfma"):
        f = os.path.join(root, f"bench_{p}.json")
        if os.path.exists(f) and open(f).read().strip():
            bench = json.loads(open(f).read().strip().splitlines()[-1])
            break
    out = {"kernel": "k_dg<3> (timed launch of bench.py --steps 20 --warmup 5)", "launch_ns_per_pass": dur,
           "counters": c}
    sipm = bench["loop"]["tail"].get("stage_ipm_iters") if bench else None
    solves = bench["value"] * bench["ms_per_step"] * bench["steps"] / 1e3 if bench else None
    ns = dur.get("fetch") or dur.get("sqa")
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        out["wave_time_split"] = {
            "waiting_s_waitcnt_barrier": c.get("SQ_WAIT_INST_ANY", 0) / wc,
            "issuing": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            "issuing_valu": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
            "issuing_lds": c.get("SQ_ACTIVE_INST_LDS", 0) / wc,
            "issuing_salu": c.get("SQ_ACTIVE_INST_SCA", 0) / wc,
            "issuing_vmem": c.get("SQ_ACTIVE_INST_VMEM", 0) / wc,
        }
        s = out["wave_time_split"]
        s["issue_stalled_dependency_pipe"] = max(0.0, 1.0 - s["waiting_s_waitcnt_barrier"] - s["issuing"])
    if sipm:
        out["stage_ipm_iters"] = sipm
        out["per_stage_ipm_iteration"] = {k: c[v] / sipm for k, v in
                                          (("valu_insts", "SQ_INSTS_VALU"), ("salu_insts", "SQ_INSTS_SALU"),
                                           ("lds_insts", "SQ_INSTS_LDS"), ("vmem_insts", "SQ_INSTS_VMEM")) if v in c}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fb, wb = 2.0 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        out["memory_side"] = {"fetch_bytes": fb, "write_bytes": wb, "bytes": fb + wb,
                              "correction": "FETCH_SIZE x2 (gfx950; exact 128-B line bytes on the product's window "
                                            "shapes, round-4 calibration), KB -> bytes x1024"}
        if ns:
            out["memory_side"]["tb_per_s"] = (fb + wb) / (ns * 1e-9) / 1e12
        if sipm:
            out["memory_side"]["bytes_per_stage_ipm_iteration"] = (fb + wb) / sipm
        if solves:
            out["memory_side"]["bytes_per_solve"] = (fb + wb) / solves
    if "TCC_HIT_sum" in c:
        out["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in c and dur.get("mfma"):
        out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / (dur["mfma"] * 1e-9) / 1e9
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        # busy cycles summed over the chip's SIMDs (1024) against the kernel's GPU cycles per XCD
        out["mfma_busy_share"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if bench:
        out["bench_value_solves_per_s"] = bench["value"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
