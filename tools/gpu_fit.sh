# The NN fit on one GPU: the device-fit tests, per-step times of the native trainer (first fit 500k rows, refit
# 3M rows) and of the PyTorch trainer (eager: its graph mode faulted, profiles/r03f_*), and a kernel-trace profile
# of the native step.  usage (on the box via gpurun): bash tools/gpu_fit.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-fit}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread $R/tests/test_fit_device.py -m gpu > $O/pytest.log 2>&1 && grep -c PASSED $O/pytest.log &&
timeout -k 10 120 python3 -u $R/tools/fit_probe.py --rows 500000 --steps 8192 > $O/native_first.json &&
timeout -k 10 120 python3 -u $R/tools/fit_probe.py --rows 3000000 --steps 8192 --refit > $O/native_refit3m.json &&
timeout -k 10 120 python3 -u $R/tools/fit_probe.py --rows 500000 --steps 2048 --torch --eager > $O/torch_eager_first.json &&
cat $O/*.json &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o fit -- python3 $R/tools/fit_probe.py --rows 500000 --steps 4096 > $O/prof.log 2>&1
