"""AL labels of the CPU oracle against the LP feasibility of the linearised QP (tests/al_reference.py) on a larger
sample than tests/test_al.py: counts, QP iterations of each class.  usage: python tools/al_lp_pin.py [n] [out.json]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    import oracle
    from al_reference import lp_feasible
    from vboc_amd.al import AlSpec, out_of_bounds, unlabeled_states
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    spec = AlSpec()
    S = unlabeled_states(spec, n, np.random.default_rng(1))
    S = np.array([s for s in S if not out_of_bounds(spec, s)])
    r = oracle.al_solve_batch(spec, S)
    feas = np.array([lp_feasible(spec, s) for s in S])
    lab = r["label"] == 1
    it = r["qp_iter"]
    out = dict(states=int(len(S)), lp_feasible=int(feas.sum()), lp_infeasible=int((~feas).sum()),
               labels_equal=int((lab == feas).sum()), label1_lp_infeasible=int((lab & ~feas).sum()),
               label0_lp_feasible=int((~lab & feas).sum()), status_hist={int(k): int(v) for k, v in
                                                                           zip(*np.unique(r["status"], return_counts=True))},
               qp_iter_feasible_min_p50_max=[int(it[feas].min()), float(np.median(it[feas])), int(it[feas].max())],
               qp_iter_infeasible_min_p50_max=[int(it[~feas].min()), float(np.median(it[~feas])), int(it[~feas].max())],
               qp_iter_max=spec.qp_iter_max, sample="AlSpec unlabeled box, numpy default_rng(1), in-bounds states")
    print(json.dumps(out))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
