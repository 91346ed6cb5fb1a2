# k_dg counters at the DRIVER's launch shape (bench.py --steps 20 --warmup 5 --no-cpu: one 100k-problem warmup
# launch, one 400k-problem timed launch), one rocprofv3 --pmc pass per counter group (verdict r03 item 4):
#   sqa  wave states (SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, VALU / LDS issue, LDS waits)
#   sqb  instruction mix (SALU, MISC, VMEM issue; VALU / SALU / LDS instructions; LDS bank conflicts)
#   fetch / write / tcc   memory side (FETCH_SIZE x2 = 128-B line bytes, calibrated in round 4), L2 hit rate
#   mfma FP64 MFMA busy cycles / instructions and GRBM_GUI_ACTIVE
# summarised by tools/pmc_r04.py.  usage (on the box via gpurun): bash tools/gpu_r04_pmc.sh <out-subdir> [passes]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04pmc}; mkdir -p $O; shift
PASSES=${@:-sqa sqb fetch write tcc mfma}
cd /tmp && export TMPDIR=/tmp
for p in $PASSES; do
  case $p in
    sqa) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES";;
    sqb) C="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM";;
    fetch) C="FETCH_SIZE";;
    write) C="WRITE_SIZE";;
    tcc) C="TCC_HIT_sum TCC_MISS_sum";;
    mfma) C="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE";;
  esac
  timeout -s KILL 360 rocprofv3 --pmc $C --output-format csv -d $O/$p -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_$p.json 2> $O/$p.err
  rc=$?; echo "$p exit $rc"; [ $rc -eq 0 ] || exit $rc
done
