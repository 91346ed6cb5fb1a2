# Reproducer of the round-2 UR5 merit defect (profiles/r02p_ur5_merit_bisect.log).
# Builds the solver with -DVBOC_MERIT_PARTIAL_EXEC (merit()'s stage trips with the usual `k = t; k <= N; k += 64`
# loop, i.e. the rigid-body RK4 of the last trip under a partial exec mask) and runs the UR5 parity test on that
# build and on the product build.  Expected: the variant fails the SQP-iteration agreement bar (round 2:
# 3 % on ids 300..331, the QP steps identical, the merit line search backtracking more), the product passes.
# usage (CPU): bash tools/ur5_merit_repro.sh build        (on the box via gpurun): bash tools/ur5_merit_repro.sh run <out>
set -o pipefail
cd "$(dirname "$0")/.."
if [ "$1" = "build" ]; then
  bash tools/build_variants.sh "merit_pe:-DVBOC_MERIT_PARTIAL_EXEC"
  exit $?
fi
O=gpurun_out/${2:-ur5_merit}; mkdir -p $O
T="tests/test_ur5.py::test_ur5_parity_with_oracle"
VBOC_LIB=$PWD/vboc_amd/variants/libvboc_amd_merit_pe.so timeout -k 10 300 python -u -m pytest "$T" -v \
  --timeout 240 --timeout-method thread > $O/variant_partial_exec.log 2>&1
echo "variant (partial-exec merit trips): pytest exit $? (1 = the defect reproduced)"
timeout -k 10 300 python -u -m pytest "$T" -v --timeout 240 --timeout-method thread > $O/product.log 2>&1
echo "product (wave-uniform merit trips): pytest exit $?"
