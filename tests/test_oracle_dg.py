"""The C restatement of the reference's data_generation (oracle/vboc_dg.c - test infrastructure and the
CPU baseline of bench.py's dg-loop leg) against the reference's own function.

tests/golden/driver_{2,3}.json are the return values of `data_generation` AST-extracted from
VBOC/{triple,double}pendulum_vboc.py and run on the CPU oracle (tests/golden/make_driver_golden.py): 256+ problems without failure injection (the triple's
long-tail ids included) and 64 with it (fail_mod 3: restart branches).  The C state machine, one problem per OpenMP thread on the same oracle,
must return the same samples bit for bit (and for the double the same 3-tuples).  A second check runs more
problems, with and without the fixtures' failure injection (restart branches), against the batched Python
driver (vboc_amd.drivers, itself pinned to the same fixtures) on the oracle."""
import json
import os

import numpy as np
import pytest

import oracle
from oracle_backend import OracleBackend

HERE = os.path.dirname(os.path.abspath(__file__))


def _same(nq, got, ref):
    if nq == 3:
        return (got is None and ref is None) or (got is not None and ref is not None and
                                                 np.array_equal(np.asarray(got, float), np.asarray(ref, float)))
    return all(_same(3, a, b) for a, b in zip(got, ref))


@pytest.mark.parametrize("nq", [3, 2])
def test_c_data_generation_matches_reference_fixture(nq):
    g = json.load(open(os.path.join(HERE, "golden", f"driver_{nq}.json")))
    assert len(g["ids"]) >= 256
    for ids, results, fail_mod in ((g["ids"], g["results"], 0), (g["fail_ids"], g["fail_results"], g["fail_mod"])):
        res, st = oracle.data_generation(nq, np.array(ids), N_start=g["N_start"], seed=g["seed"], fail_mod=fail_mod,
                                         nthreads=8)
        assert st["solves"] > len(ids) and st["rk4"] > 0
        bad = [pid for pid, a, b in zip(ids, res, results) if not _same(nq, a, b)]
        assert not bad, (fail_mod, bad)


@pytest.mark.parametrize("nq,fail_mod", [(3, 0), (2, 0), (3, 3), (2, 3)])
def test_c_data_generation_matches_batched_driver(nq, fail_mod):
    """fail_mod 3: the fixtures' failure injection (tests/oracle_backend.py), so the restart branches run."""
    from vboc_amd.drivers import data_generation_batch
    ids = np.arange(200, 216)
    res, st = oracle.data_generation(nq, ids, N_start=40, fail_mod=fail_mod, nthreads=8)
    ref, rst = data_generation_batch(nq, ids, OracleBackend(nq, fail_mod=fail_mod), N_start=40)
    bad = [int(pid) for pid, a, b in zip(ids, res, ref) if not _same(nq, a, b)]
    assert not bad, bad
    assert st["solves"] == rst["solves"] and st["rk4"] == rst["rk4"]
