"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Usage: python tools/pmc_summary.py [--max-launch] <fetch_counter_collection.csv> <write_counter_collection.csv>
       <bench_line.json> [kernel-substring] [sq_counter_collection.csv] > profiles/<round>_pmc_<kernel>.json
--max-launch takes the largest launch of the kernel (the driver command's timed launch; its warmup launch is
smaller) instead of the mean over launches.
The optional SQ pass adds the instruction / busy counters of the launch (FP64 MFMA ops, MFMA busy cycles,
VALU and LDS instructions, GRBM_GUI_ACTIVE).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KB) reports half the bytes of wide
coalesced streaming reads, so it is doubled; WRITE_SIZE (KB) is taken as is.  The algorithmic bytes
per launch come from the bench line of the same (warmup 0) run: roofline.achieved x avg_launch_ms.
"""
import csv
import json
import sys


LAUNCH = "mean"   # "max": the largest launch only (the driver command's timed launch beside its warmup launch)


def total(path, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if LAUNCH == "max" and vals:
        return max(vals), 1
    return sum(vals), len(vals)


def main():
    global LAUNCH
    if "--max-launch" in sys.argv:
        sys.argv.remove("--max-launch")
        LAUNCH = "max"
    fetch_csv, write_csv, bench_json = sys.argv[1:4]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "k_qp_factor"
    fs, nf = total(fetch_csv, "FETCH_SIZE", kernel)
    ws, nw = total(write_csv, "WRITE_SIZE", kernel)
    line = json.loads(open(bench_json).read().strip().splitlines()[-1])
    rf = line["roofline"]
    fetch_b = 2.0 * fs * 1024 / nf
    write_b = ws * 1024 / nw
    out = {"kernel": kernel, "launches_fetch_pass": nf, "launches_write_pass": nw,
           "fetch_bytes_per_launch_corrected": fetch_b, "write_bytes_per_launch": write_b,
           "traffic_bytes_per_launch": fetch_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950), KB -> bytes x1024"}
    if rf["unit"] == "GB/s":   # bandwidth roofline: compare with the algorithmic bytes
        alg = rf["achieved"] * 1e9 * rf["avg_launch_ms"] * 1e-3
        out.update(algorithmic_bytes_per_launch=alg, traffic_over_algorithmic=(fetch_b + write_b) / alg)
    else:                      # FP64 roofline: arithmetic intensity against HBM traffic
        if "loop" in line:     # dg-loop: launches differ in size, so the bench scales a per-problem figure
            probs = line["config"]["problems_per_gpu"] * line["steps"]   # the timed launch (--max-launch or warmup 0)
            out.update(problems_per_launch=probs, traffic_bytes_per_problem=(fetch_b + write_b) / probs)
        out.update(flops_per_launch=rf["flops_per_launch"],
                   flop_per_hbm_byte=rf["flops_per_launch"] / (fetch_b + write_b),
                   hbm_gbs_during_launch=(fetch_b + write_b) / (rf["avg_launch_ms"] * 1e-3) / 1e9)
    if len(sys.argv) > 5:
        sq = {}
        for r in csv.DictReader(open(sys.argv[5])):
            if kernel in r["Kernel_Name"]:
                sq[r["Counter_Name"]] = sq.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        out["sq_counters_per_launch"] = sq
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
