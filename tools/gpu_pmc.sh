# Memory-side traffic and FP64 MFMA / VALU activity of the bench's dominant kernel: separate rocprofv3 --pmc
# passes (FETCH_SIZE; WRITE_SIZE; SQ instruction / busy counters), each over one timed step with no warmup
# (MI355X_MICROARCH.md HBM section), summarised by tools/pmc_summary.py.
# usage (on the box via gpurun): bash tools/gpu_pmc.sh <out-subdir> [extra bench.py args, e.g. --nq 4 --batch 12500]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmc}; mkdir -p $O; shift; EXTRA="$@"
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --warmup 0 --steps 1 --no-cpu $EXTRA > $O/bench_fetch.json 2> $O/fetch.err && echo fetch_ok &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --warmup 0 --steps 1 --no-cpu $EXTRA > $O/bench_write.json 2> $O/write.err && echo write_ok &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 $R/bench.py --warmup 0 --steps 1 --no-cpu $EXTRA > $O/bench_sq.json 2> $O/sq.err && echo sq_ok
