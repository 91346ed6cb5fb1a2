# Round-4 final check (on the box via gpurun): the whole GPU test suite and smoke() on the final tree.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04t}; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc: $(tail -1 $O/pytest_gpu.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke exit $?"
