# Round-4 call P: the lockstep classification test after the tolerance fix (bash tools/gpu_r04p.sh <out-subdir>)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04p}; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_drivers.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_drivers.log 2>&1
rc=$?; echo "pytest exit $rc: $(tail -1 $O/pytest_drivers.log)"; [ $rc -le 1 ] || exit $rc
bash $R/tools/gpu_r04q.sh ${1:-r04p}_q
