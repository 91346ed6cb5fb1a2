# The VBOC loop end to end on one GPU (tools/vboc_loop.py): configs[2]'s 100k states (5 iterations of 20k) and the
# reference's 1000-problem iterations, each with the streaming producer and with synchronous rounds.
# usage (on the box via gpurun): bash tools/gpu_loop.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-loop}; mkdir -p $O
timeout -k 10 300 python3 -u $R/tools/vboc_loop.py --nq 3 --test 1000 --num-prob 20000 --iters 4 --stop 600 > $O/c2_stream.log 2>&1 && tail -1 $O/c2_stream.log &&
timeout -k 10 300 python3 -u $R/tools/vboc_loop.py --nq 3 --test 1000 --num-prob 20000 --iters 4 --stop 600 --no-stream > $O/c2_sync.log 2>&1 && tail -1 $O/c2_sync.log &&
timeout -k 10 300 python3 -u $R/tools/vboc_loop.py --nq 3 --test 1000 --num-prob 1000 --iters 19 --stop 600 > $O/r1k_stream.log 2>&1 && tail -1 $O/r1k_stream.log &&
timeout -k 10 300 python3 -u $R/tools/vboc_loop.py --nq 3 --test 1000 --num-prob 1000 --iters 19 --stop 600 --no-stream > $O/r1k_sync.log 2>&1 && tail -1 $O/r1k_sync.log
