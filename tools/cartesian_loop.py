"""The Cartesian double pendulum's main block end to end on one MI355X (pipeline.cartesian_run): test set,
training set through the constrained driver (wave solver with the keep-out circle), NeuralNetRegression fit,
RMSE, artefacts.  usage: python tools/cartesian_loop.py [num_test] [num_train] [out_dir]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from vboc_amd.pipeline import cartesian_run
    nt = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    ntr = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    out = sys.argv[3] if len(sys.argv) > 3 else None
    t = time.time()
    r = cartesian_run(num_test=nt, num_train=ntr, out_dir=out, log=lambda *a: print(*a, flush=True))
    st_test, st_train = r["stats"]
    print(f"test rows {r['X_test'].shape[0]} / {nt}, train rows {r['X_train'].shape[0]} / {ntr}; "
          f"solves {st_test['solves'] + st_train['solves']} in {st_test['rounds'] + st_train['rounds']} rounds; "
          f"total {time.time() - t:.1f} s", flush=True)


if __name__ == "__main__":
    main()
