# SQ wave-state counters of the wave solver (k_wave first solves), separate rocprofv3 --pmc passes (8 SQ each)
# usage (on the box via gpurun): bash tools/gpu_sq.sh <out-subdir> <lib .so> [nq] [B]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-sq}; mkdir -p $O; export VBOC_LIB=$2; NQ=${3:-3}; B=${4:-16384}
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/sqa -o run -- python3 $R/tools/pass_probe.py $NQ $B > $O/sqa.json 2> $O/sqa.err && echo sqa_ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sqb -o run -- python3 $R/tools/pass_probe.py $NQ $B > $O/sqb.json 2> $O/sqb.err && echo sqb_ok
