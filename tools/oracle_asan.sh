# The CPU restatement (oracle/, test infrastructure) under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
# section 5): builds oracle/libvboc_oracle_asan.so (make asan) and runs the oracle's CPU tests against it, the ASan
# runtime preloaded into the (uninstrumented) interpreter.  CPU container only.
# usage: bash tools/oracle_asan.sh [log]      (default log: profiles/r06_oracle_asan.log)
set -o pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r06_oracle_asan.log}
make -s -C oracle asan || exit 1
export VBOC_ORACLE_LIB=$PWD/oracle/libvboc_oracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
PRE="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)"
{
  echo "# $(date -u +%FT%TZ) oracle tests against $VBOC_ORACLE_LIB (gcc $(gcc -dumpversion), -fsanitize=address,undefined)"
  LD_PRELOAD=$PRE timeout 3000 python -m pytest -q -m "not gpu" -p no:cacheprovider \
    tests/test_golden_dynamics.py tests/test_oracle_solver.py tests/test_oracle_kkt.py tests/test_oracle_dg.py \
    tests/test_drivers.py tests/test_free_time.py tests/test_hjr.py tests/test_cartesian.py tests/test_safempc.py tests/test_al.py \
    -k "not slsqp" 2>&1
  echo "exit $?"
} | tee "$LOG"
