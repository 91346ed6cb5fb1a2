"""Per-solve record of the lockstep comparison (tests/lockstep.py) for chosen triple fixture problems: every solve
request both copies issue, with each backend's status, SQP / QP iterations, cost and x_0, so a 'value' parting can
be read solve by solve.  usage (GPU box): python tools/lockstep_probe.py <out.json> <pid> [<pid> ...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


class Recording:
    def __init__(self, inner, log, name):
        self.inner, self.log, self.name = inner, log, name

    def solve(self, b, free_time=False):
        r = self.inner.solve(b, free_time=free_time)
        for k in range(len(r["status"])):
            self.log.append(dict(side=self.name, N=int(b["N"][k]), p=np.asarray(b["p"][k]).tolist(),
                                 status=int(r["status"][k]), sqp=int(r["sqp_iter"][k]), qp=int(r["qp_iter"][k]),
                                 cost=float(r["cost"][k]), x0=np.asarray(r["x"][k, 0]).tolist()))
        return r

    def rk4(self, x, u, T):
        return self.inner.rk4(x, u, T)


def main():
    from lockstep import lockstep
    from oracle_backend import OracleBackend
    from test_drivers import _gens, _golden
    from vboc_amd.drivers import GpuBackend
    cpu = "--cpu" in sys.argv          # dry run of the script with the oracle on both sides
    argv = [a for a in sys.argv[1:] if a != "--cpu"]
    out, pids = argv[0], [int(a) for a in argv[1:]]
    g = _golden(3)
    res = {}
    for pid in pids:
        log = []
        first = OracleBackend(3) if cpu else GpuBackend(3)
        kinds = lockstep(3, _gens(3, "dg", g), [pid], Recording(first, log, "gpu"),
                         Recording(OracleBackend(3), log, "oracle"), nmax=200)
        res[pid] = dict(kind=kinds[pid], solves=log)
        print(pid, kinds[pid], len(log), flush=True)
    json.dump(res, open(out, "w"))


if __name__ == "__main__":
    main()
