"""The CPU oracle's converged share on test_ur5_full_batch_properties's 4096 UR5 first solves (ids 10^6 .. +4095,
nlp_solver_max_iter 100), the bar that test holds the GPU solver to (verdict r05 item 7).  Also the status histogram
and the SQP-iteration distribution of the unconverged ones (they are max_iter stops: the truncated budget, not
failures).  Writes the per-problem statuses to tests/golden/ur5_status_4096.json (the GPU test compares problem by
problem).  usage: python tools/ur5_converged_share.py [out.json]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import oracle
    from vboc_amd.ics import ur5_ics
    b = ur5_ics(np.arange(10**6, 10**6 + 4096))
    o = oracle.default_opts(lm=1e-2, max_iter=100)
    t = time.time()
    xo, uo, r = oracle.solve_batch(4, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"], b["ubu"],
                                   b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], opts=o)
    st = np.array(r["status"])
    out = dict(problems=int(st.size), converged_share=float((st == 0).mean()),
               status_hist={int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
               sqp_iter_converged_p50_p99=[float(np.percentile(r["sqp_iter"][st == 0], q)) for q in (50, 99)],
               seconds=time.time() - t, threads=os.cpu_count(), status=st.tolist())
    print(json.dumps({k: v for k, v in out.items() if k != "status"}))
    json.dump({"ids_first": 10**6, "n": 4096, "nlp_solver_max_iter": 100, "levenberg_marquardt": 1e-2,
               "generator": "tools/ur5_converged_share.py (oracle/, CPU)", "status": out.pop("status")},
              open(os.path.join(ROOT, "tests", "golden", "ur5_status_4096.json"), "w"))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
