# Round-4 call E (on the box via gpurun): bash tools/gpu_r04e.sh <out-subdir>
#  1. Safe-MPC GPU outputs of the test cases (tools/mpc_probe.py) for analysis against the oracle on the CPU
#  2. the trainer's graph-replay == eager test after the per-fit generator change
#  3. the UR5 k_wave<4> bisect (tools/gpu_r04b.sh) on variants rebuilt from the current source
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04e}; mkdir -p $O
cd $R
timeout -k 10 200 python3 -u tools/mpc_probe.py $O/mpc.npz > $O/mpc_probe.log 2>&1; rc=$?; echo "mpc_probe exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u -m pytest tests/test_learn.py -m gpu -v --timeout 180 --timeout-method thread -k "replay_equals_eager or consecutive" > $O/pytest_learn.log 2>&1
rc=$?; echo "pytest_learn exit $rc"; [ $rc -le 1 ] || exit $rc
bash tools/gpu_r04b.sh ${1:-r04e} sbase sbase_drain wbun wbun_drain
