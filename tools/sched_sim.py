"""Makespan of a data-generation launch under different job orders, simulated from measured per-problem stats
(tools/dg_probe.py --save: lib.DG_STATS rows, device real-time clock) - a study of the launch tail (verdict r03
item 5) before changing k_dg's scheduler.

Each problem's measured duration d = t1 - t0 is split into its first solve (share it1 / sqp of the SQP iterations)
and the rest.  G workers (the launch's resident problems) take jobs greedily:
  id        the product: problems in id order, each run to completion
  park      phase A runs every problem's first solve in id order; a problem whose first solve failed
            (first_status != 0, the predictor of long restart chains) continues at once, the others are parked;
            parked problems resume (rest of the state machine) once the id queue is drained
  park_it1  as park, parked problems resumed in decreasing order of their first solve's SQP iterations
  oracle    longest-processing-time-first with the true durations (a bound no online policy reaches)
usage: python tools/sched_sim.py <stats.npy> [groups]
"""
import heapq
import json
import sys

import numpy as np


def simulate(jobs, G):
    """jobs: list of (release_key, duration, follow) processed in list order by G workers; `follow` is a
    duration appended to a second queue (continuations) that workers take only once `jobs` is empty."""
    free = [0.0] * G
    heapq.heapify(free)
    end = 0.0
    cont = []
    for d, follow_now, follow_later in jobs:
        t = heapq.heappop(free)
        t += d + follow_now
        end = max(end, t)
        heapq.heappush(free, t)
        if follow_later is not None:
            cont.append(follow_later)
    return free, end, cont


def run_queue(free, end, items):
    for d in items:
        t = heapq.heappop(free)
        t += d
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def main():
    st = np.load(sys.argv[1])
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 1326
    clk = 100e6
    d = (st[:, 6] - st[:, 5]) / clk
    share = np.clip(st[:, 8] / np.maximum(st[:, 2], 1), 0.0, 1.0)
    d1 = d * share
    rest = d - d1
    failed = st[:, 7] != 0
    out = {"problems": int(len(d)), "groups": G, "sum_s": round(float(d.sum()), 1), "max_s": round(float(d.max()), 2),
           "failed_first": int(failed.sum()),
           "share_of_slowest_100_with_failed_first": float(failed[np.argsort(-d)[:100]].mean())}
    free, end, _ = simulate([(x, 0.0, None) for x in d], G)
    out["id"] = round(end, 2)
    out["bulk_bound"] = round(float(d.sum()) / G, 2)
    jobs = [(d1[i], rest[i] if failed[i] else 0.0, None if failed[i] else rest[i]) for i in range(len(d))]
    free, end, cont = simulate(jobs, G)
    out["park"] = round(run_queue(list(free), end, cont), 2)
    order = np.argsort(-st[:, 8], kind="stable")
    jobs = [(d1[i], rest[i] if failed[i] else 0.0, None) for i in range(len(d))]
    free, end, _ = simulate(jobs, G)
    parked = [rest[i] for i in order if not failed[i]]
    out["park_it1"] = round(run_queue(list(free), end, parked), 2)
    free, end, _ = simulate([(x, 0.0, None) for x in np.sort(d)[::-1]], G)
    out["oracle"] = round(end, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
