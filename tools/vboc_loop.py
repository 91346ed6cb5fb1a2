"""Run the whole VBOC loop on one GPU: held-out set (`testing`), then data generation + NN fit +
RMSE iterations until the time budget is spent (VBOC/triplependulum_vboc.py:372-585), logging the
time split per iteration.  Usage:
  python tools/vboc_loop.py NQ NUM_TEST NUM_PROB STOP_TIME_S OUT_DIR
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vboc_amd.drivers import GpuBackend  # noqa: E402
from vboc_amd.pipeline import make_test_set, vboc_run  # noqa: E402


def main():
    nq, n_test, n_prob, stop, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), sys.argv[5]
    be = GpuBackend(nq)
    t = time.time()
    X_test, st = make_test_set(nq, be, num_prob=n_test, first_id=10**8, out_dir=out)
    t_test = time.time() - t
    print(json.dumps(dict(phase="testing", problems=n_test, rows=int(X_test.shape[0]), seconds=round(t_test, 3),
                          solves=st["solves"], rounds=st["rounds"])), flush=True)
    t = time.time()
    r = vboc_run(nq, be, X_test, stop_time=stop, num_prob=n_prob, out_dir=out,
                 log=lambda m: print(f"[{time.time() - t:8.2f}s] {m}", flush=True))
    print(json.dumps(dict(phase="vboc", iterations=len(r["times"]), rows=int(r["X_save"].shape[0]),
                          times=[round(x, 3) for x in r["times"]], rmse=r["rmse"],
                          fits=r["fits"], solves=[s["solves"] for s in r["stats"]],
                          rk4=[s["rk4"] for s in r["stats"]])), flush=True)


if __name__ == "__main__":
    main()
