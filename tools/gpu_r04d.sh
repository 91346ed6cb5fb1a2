# Round-4 call D (on the box via gpurun): bash tools/gpu_r04d.sh <out-subdir>
#  1. GPU tests: Safe MPC (vboc_mpc_solve_batch vs the oracle, closed loop), the busy guard, the trainer
#  2. k_dg at 60k problems: parked first solves on / off; the separate acl_pass build; resident-problem sweep
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04d}; mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest tests/test_safempc.py tests/test_dg_device.py -m gpu -v --timeout 300 --timeout-method thread -k "gpu or refuses" > $O/pytest_a.log 2>&1
rc=$?; echo "pytest_a exit $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest tests/test_learn.py -m gpu -v --timeout 380 --timeout-method thread > $O/pytest_learn.log 2>&1
rc=$?; echo "pytest_learn exit $rc"; [ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 0 --park 1 0 --save $O/stats60k > $O/probe_park.jsonl 2> $O/probe_park.err && cat $O/probe_park.jsonl &&
VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_aclpass.so timeout -k 10 200 python3 $R/tools/dg_probe.py --B 60000 --groups 0 --park 1 > $O/probe_aclpass.jsonl 2> $O/probe_aclpass.err && cat $O/probe_aclpass.jsonl &&
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 880 1760 --park 1 > $O/probe_groups.jsonl 2> $O/probe_groups.err && cat $O/probe_groups.jsonl
