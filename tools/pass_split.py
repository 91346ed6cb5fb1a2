"""Per-pass bytes and time of the wave solver's IPM iteration from tools/pass_split.sh output.

For each pass p (a -DVBOC_REPEAT=p build runs it twice, results bit-identical to the product build): the
extra kernel time, memory-side read bytes (FETCH_SIZE x2, the gfx950 correction of MI355X_MICROARCH.md),
written bytes (WRITE_SIZE) over the product build, per stage-IPM-iteration (sum over problems of N x qp_iter).
The base row gives the whole launch per stage-IPM-iteration and its L2 hit rate.
usage: python tools/pass_split.py gpurun_out/<dir> > profiles/<round>_pass_split.json
"""
import csv
import glob
import json
import os
import sys

PASSES = {1: "prep_pred", 2: "factor (MFMA Riccati sweep)", 3: "acl_pass", 4: "vec (predictor)", 5: "fwd (predictor)",
          6: "prep_corr", 7: "vec (corrector)", 8: "fwd (corrector)"}


def counter(d, name, kernel="k_wave"):
    tot, n = 0.0, 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and kernel in r["Kernel_Name"]:
                tot += float(r["Counter_Value"])
                n += 1
    return tot, n


def main():
    d = sys.argv[1]
    rows = {}
    for tf in sorted(glob.glob(os.path.join(d, "time_*.json"))):
        p = int(os.path.basename(tf)[5:-5])
        t = json.loads(open(tf).read().strip().splitlines()[-1])
        fe, nf = counter(os.path.join(d, f"fetch_{p}"), "FETCH_SIZE")
        wr, nw = counter(os.path.join(d, f"write_{p}"), "WRITE_SIZE")
        rows[p] = dict(kernel_ms=t["kernel_ms"], fetch_b=2.0 * fe * 1024, write_b=wr * 1024, digest=t["digest"],
                       sipm=t["stage_ipm_iters"], launches=(nf, nw))
    base = rows[0]
    u = base["sipm"]
    out = {"unit": "per stage-IPM-iteration (sum over problems of N * qp_iter = %d)" % u,
           "workload": "k_wave first solves, triple pendulum, N = 100",
           "correction": "FETCH_SIZE x2 (gfx950), KB -> B",
           "base": {"kernel_ms": round(base["kernel_ms"], 1),
                    "read_B": round(base["fetch_b"] / u, 1), "write_B": round(base["write_b"] / u, 1),
                    "ns": round(base["kernel_ms"] * 1e6 / u, 3)},
           "passes": {}}
    tcc = os.path.join(d, "tcc_0")
    if os.path.isdir(tcc):
        h, _ = counter(tcc, "TCC_HIT_sum")
        m, _ = counter(tcc, "TCC_MISS_sum")
        if h + m:
            out["base"]["l2_hit_rate"] = round(h / (h + m), 4)
    for p, r in sorted(rows.items()):
        if p == 0:
            continue
        out["passes"][PASSES.get(p, str(p))] = {
            "ms": round(r["kernel_ms"] - base["kernel_ms"], 1),
            "time_frac": round((r["kernel_ms"] - base["kernel_ms"]) / base["kernel_ms"], 4),
            "read_B": round((r["fetch_b"] - base["fetch_b"]) / u, 1),
            "write_B": round((r["write_b"] - base["write_b"]) / u, 1),
            "same_results": r["digest"] == base["digest"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
