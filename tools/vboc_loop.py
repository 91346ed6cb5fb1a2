"""Run the whole VBOC loop on one GPU: held-out set (`testing`), then data generation + NN fit + RMSE iterations
until the time budget or the iteration count is spent (VBOC/triplependulum_vboc.py:372-585), logging the time
split.  With --stream (default) the iterations' data generation is one producer launch running ahead of the fits
(pipeline.StreamedRounds); --no-stream is the reference's synchronous round-by-round structure.
Prints one JSON line per phase; the loop line carries the end-to-end rate: solves of the iterations the loop
consumed over the loop's wall time (the producer's problems past the last consumed iteration are cancelled).
usage: python tools/vboc_loop.py --nq 3 --test 1000 --num-prob 20000 --iters 4 --stop 600 --out /tmp/vboc
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vboc_amd.drivers import GpuBackend  # noqa: E402
from vboc_amd.pipeline import make_test_set, vboc_run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=3)
    ap.add_argument("--test", type=int, default=1000)
    ap.add_argument("--num-prob", type=int, default=1000)
    ap.add_argument("--iters", type=int, default=None, help="VBOC iterations after the first (default: until --stop)")
    ap.add_argument("--stop", type=float, default=300.0)
    ap.add_argument("--stream", action=argparse.BooleanOptionalAction, default=True)
    ap.add_argument("--stream-rounds", type=int, default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    be = GpuBackend(a.nq)
    t = time.time()
    X_test, st = make_test_set(a.nq, be, num_prob=a.test, first_id=10**8, out_dir=a.out)
    t_test = time.time() - t
    print(json.dumps(dict(phase="testing", problems=a.test, rows=int(X_test.shape[0]), seconds=round(t_test, 3),
                          solves=st["solves"], rounds=st["rounds"])), flush=True)
    t = time.time()
    r = vboc_run(a.nq, be, X_test, stop_time=a.stop, num_prob=a.num_prob, max_iterations=a.iters, out_dir=a.out,
                 stream=a.stream, stream_rounds=a.stream_rounds,
                 log=lambda m: print(f"[{time.time() - t:8.2f}s] {m}", flush=True))
    wall = time.time() - t
    solves = sum(s["solves"] for s in r["stats"])
    print(json.dumps(dict(phase="vboc", stream=a.stream, num_prob=a.num_prob, iterations=len(r["times"]),
                          problems=a.num_prob * len(r["stats"]), rows=int(r["X_save"].shape[0]),
                          wall_s=round(wall, 2), solves=solves, end_to_end_solves_per_s=round(solves / wall, 1),
                          boundary_problems_per_s=round(a.num_prob * len(r["stats"]) / wall, 1),
                          times=[round(x, 3) for x in r["times"]], rmse=r["rmse"],
                          fit_iterations=[f["iterations"] for f in r["fits"]],
                          solves_per_iteration=[s["solves"] for s in r["stats"]], producer=r.get("producer"))),
          flush=True)


if __name__ == "__main__":
    main()
