# Round-4 call J (on the box via gpurun): bash tools/gpu_r04j.sh <out-subdir>
#  1. Safe-MPC GPU tests (full SQP at the class's nlp_solver_max_iter 1000)
#  2. k_dg at 60k problems, eager window 0 / 2: the speculation timing stats (taken / wait / lag)
#  3. driver-shape bytes A/B (verdict r03 item 4): bench.py --steps 20 --warmup 5 on the product (A_cl formed inside the
#     factorisation) and on the -DVBOC_ACL_PASS build (the separate pass re-reading A, B, K and writing A_cl), with
#     FETCH_SIZE / WRITE_SIZE passes of the latter (the product's are in r04pmc)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04j}; mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_safempc.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_mpc.log 2>&1
rc=$?; echo "pytest_mpc exit $rc"; [ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 0 --park 1 --window 0 2 --save $O/stats60k > $O/probe_window.jsonl 2> $O/probe_window.err; rc=$?; echo "probe exit $rc"; [ $rc -eq 0 ] || exit $rc
cat $O/probe_window.jsonl
timeout -k 10 360 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_product.json 2> $O/bench_product.err; rc=$?; echo "bench product exit $rc"; [ $rc -eq 0 ] || exit $rc
VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_aclpass.so timeout -k 10 360 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_aclpass.json 2> $O/bench_aclpass.err; rc=$?; echo "bench aclpass exit $rc"; [ $rc -eq 0 ] || exit $rc
for p in fetch write; do
  case $p in fetch) C=FETCH_SIZE;; write) C=WRITE_SIZE;; esac
  VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_aclpass.so timeout -s KILL 360 rocprofv3 --pmc $C --output-format csv -d $O/acl_$p -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_acl_$p.json 2> $O/acl_$p.err
  rc=$?; echo "acl $p exit $rc"; [ $rc -eq 0 ] || exit $rc
done
