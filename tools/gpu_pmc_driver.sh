# Memory-side traffic and L2 hit rate of the dg-loop kernel at the DRIVER's launch shape (bench.py --steps 20
# --warmup 5: one 100k-problem warmup launch, one 400k-problem timed launch): separate rocprofv3 --pmc passes
# (FETCH_SIZE; WRITE_SIZE; TCC_HIT_sum + TCC_MISS_sum), summarised for the timed launch by
# tools/pmc_summary.py --max-launch.  usage (on the box via gpurun): bash tools/gpu_pmc_driver.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pmcd}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_fetch.json 2> $O/fetch.err && echo fetch_ok &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_write.json 2> $O/write.err && echo write_ok &&
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_tcc.json 2> $O/tcc.err && echo tcc_ok
