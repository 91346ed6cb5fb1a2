"""The UR5 arm's kernels (NQ = 4) keep the instructions the GPU suite validated.  k_wave<4> has shown codegen
sensitivity before (a register-allocation change broke the counted ring waits), and the
pendulum-chain changes of rounds 5 and 6 are kept out of it by construction (`WaveLayout::IN_FIRST`, `Coop::Cov`); this
test fails when a source change reaches the arm's code anyway, so that it is re-validated on the GPU
(tests/test_ur5.py) before tests/golden/isa_arm_digest.json is regenerated.  CPU only: the gfx950 code object is
disassembled with the ROCm LLVM tools."""
import json
import os
import sys

import pytest

from vboc_amd import lib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(lib.ROOT, "tools"))


def test_arm_kernels_keep_the_validated_isa():
    import kernel_digest
    if not os.path.exists(os.path.join(kernel_digest.B, "llvm-objdump")):
        pytest.skip("ROCm LLVM tools not present")
    assert os.path.exists(lib.LIB_PATH), "run __graft_entry__.build() first"
    want = json.load(open(os.path.join(HERE, "golden", "isa_arm_digest.json")))["kernels"]
    got = kernel_digest.digests(lib.LIB_PATH, "ILi4E")
    changed = sorted(k for k in want if tuple(want[k]) != tuple(got.get(k, (0, "-"))))
    assert not changed, f"arm kernels changed (re-validate on the GPU): {changed}"
