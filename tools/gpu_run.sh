# One parameterised GPU call (on the box via gpurun), replacing round 4's one-off tools/gpu_r04*.sh scripts.
# usage: bash tools/gpu_run.sh <out-subdir> <step> [<step> ...]     steps run in order, each under its own time
# limit, and the call stops at the first failing step (no GPU step after a fault, an abort or a timeout):
#   tests[=<pytest -k expr>]  the GPU suite (or a -k selection of it), parity records to <out>/parity
#   tests_file=<path,...>     GPU test files
#   tests_lib=<name>:<files>[:<-k expr>]  GPU test files (comma-separated) on vboc_amd/ab/libvboc_amd_<name>.so
#                             (VBOC_LIB): the parity suite on a variant build, parity records to <out>/parity_<name>
#   smoke                     __graft_entry__.smoke()
#   bench                     the driver's command (bench.py --steps 20 --warmup 5) -> <out>/bench.json
#   prof                      the same command under rocprofv3 --kernel-trace --stats -> <out>/prof
#   double                    configs[1]: the double pendulum's 10k dg-loop and first-solve lines
#   doubleab                  the same per build (product and every vboc_amd/ab/*.so), same box, no CPU baseline
#   probe=<B>[:<groups,...>]  tools/dg_probe.py over B problems with the product and every vboc_amd/ab/*.so
#                             (same box A/B: kernel time, bulk rate, digest); PROBE_ARGS (env) adds dg_probe options
#   ur5trunc                  tools/ur5_trunc.py (the UR5 parity problems' truncated-solve digests) per build: the
#                             product and every vboc_amd/ab/*.so
#   phases                    every -DVBOC_COOP_PROF build in vboc_amd/prof/: cycles per IPM iteration by phase (and
#                             the split of one pass with -DVBOC_PROF_SPLIT) of 16k triple first solves (tools/gpu_perf.py);
#                             PHASE_COOP=wave1024 (env) runs them on 1 024 resident problems (one wave per SIMD)
#   pmc=<pass,...>            rocprofv3 --pmc passes of bench (sqa sqb fetch write tcc mfma icache), one run per pass
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:?out-subdir}; shift; mkdir -p $O
cd $R
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@"; local rc=$?
  echo "step $name exit $rc"; [ $rc -eq 0 ] || exit $rc
}
for step in "$@"; do
  case $step in
    tests) run tests 1100 env VBOC_PARITY_OUT=$O/parity python -u -m pytest tests -m gpu -x -v --timeout 300 \
             --timeout-method thread > $O/pytest_gpu.log 2>&1;;
    tests=*) run tests 900 env VBOC_PARITY_OUT=$O/parity python -u -m pytest tests -m gpu -x -v --timeout 300 \
               --timeout-method thread -k "${step#tests=}" > $O/pytest_sel.log 2>&1;;
    tests_file=*) run tests_file 900 env VBOC_PARITY_OUT=$O/parity python -u -m pytest $(echo ${step#tests_file=} | tr , ' ') -m gpu \
                    -x -v --timeout 300 --timeout-method thread > $O/pytest_file.log 2>&1;;
    tests_lib=*) spec=${step#tests_lib=}; n=${spec%%:*}; rest=${spec#*:}; files=${rest%%:*}; k=""
                 [ "$rest" != "$files" ] && k=${rest#*:}
                 run "tests_lib $n" 900 env VBOC_LIB=$R/vboc_amd/ab/libvboc_amd_$n.so VBOC_PARITY_OUT=$O/parity_$n \
                   python -u -m pytest $(echo $files | tr , ' ') -m gpu -x -v --timeout 300 --timeout-method thread \
                   ${k:+-k "$k"} > $O/pytest_lib_$n.log 2>&1;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1;;
    bench) run bench 420 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; cat $O/bench.json;;
    prof) (cd /tmp && export TMPDIR=/tmp && run prof 420 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $O/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 \
             > $O/bench_prof.json 2> $O/bench_prof.err) || exit $?;;
    double) run double_dg 200 python bench.py --nq 2 --batch 10000 --steps 1 --warmup 1 > $O/bench_double_dg.json \
              2> $O/bench_double_dg.err &&
            run double_fs 200 python bench.py --workload first-solve --nq 2 --batch 10000 --steps 1 --warmup 1 \
              > $O/bench_double_fs.json 2> $O/bench_double_fs.err;;
    doubleab) for L in $R/vboc_amd/libvboc_amd.so $R/vboc_amd/ab/*.so; do   # configs[1] lines per build, same box
                [ -f "$L" ] || continue
                n=$(basename $L .so)
                run "double fs $n" 300 env VBOC_LIB=$L python bench.py --workload first-solve --nq 2 --batch 10000 --steps 3 \
                  --warmup 1 --no-cpu > $O/double_fs_$n.json 2> $O/double_fs_$n.err &&
                run "double dg $n" 300 env VBOC_LIB=$L python bench.py --nq 2 --batch 10000 --steps 1 --warmup 1 --no-cpu \
                  > $O/double_dg_$n.json 2> $O/double_dg_$n.err
              done;;
    probe=*) spec=${step#probe=}; B=${spec%%:*}; G=0; [ "$spec" != "$B" ] && G=${spec#*:}
             for L in $R/vboc_amd/libvboc_amd.so $R/vboc_amd/ab/*.so; do
               [ -f "$L" ] || continue
               run "probe $(basename $L)" 600 env VBOC_LIB=$L python3 -u tools/dg_probe.py --B $B --groups ${G//,/ } $PROBE_ARGS \
                 >> $O/probe.jsonl 2>> $O/probe.err
             done; cat $O/probe.jsonl;;
    ur5trunc) for L in $R/vboc_amd/libvboc_amd.so $R/vboc_amd/ab/*.so; do   # the UR5 truncated-solve digests per build
                [ -f "$L" ] || continue
                n=$(basename $L .so)
                run "ur5trunc $n" 300 env VBOC_LIB=$L python3 -u tools/ur5_trunc.py $O/trunc_$n > $O/trunc_$n.jsonl \
                  2> $O/trunc_$n.err
              done;;
    phases) for L in $R/vboc_amd/prof/*.so; do   # -DVBOC_COOP_PROF builds (+ -DVBOC_PROF_SPLIT=<pass>)
              n=$(basename $L .so)
              run "phases $n" 300 env VBOC_LIB=$L python3 -u tools/gpu_perf.py 3 16384 0 dg 0 ${PHASE_COOP:-wave} \
                > $O/phases_$n${PHASE_COOP:+_$PHASE_COOP}.log 2>&1
              cat $O/phases_$n${PHASE_COOP:+_$PHASE_COOP}.log
            done;;
    pmc=*) for p in $(echo ${step#pmc=} | tr , ' '); do
             case $p in
               sqa) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES";;
               sqb) C="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM";;
               fetch) C="FETCH_SIZE";;
               write) C="WRITE_SIZE";;
               tcc) C="TCC_HIT_sum TCC_MISS_sum";;
               icache) C="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES";;
               mfma) C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE";;
               *) echo "unknown pmc pass $p"; exit 2;;
             esac
             (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 360 rocprofv3 --pmc $C --output-format csv -d $O/$p -o run \
                -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_$p.json 2> $O/$p.err)
             rc=$?; echo "step pmc $p exit $rc"; [ $rc -eq 0 ] || exit $rc
           done;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo all_steps_ok
