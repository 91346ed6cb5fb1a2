# Round-4 measurement call A (on the box via gpurun): bash tools/gpu_r04a.sh <out-subdir>
#  1. FETCH_SIZE calibration of the stage-window LDS-DMA shapes (tools/probes/fetch_calib)
#  2. k_dg at 60k problems: resident-problem sweep on the product (A_cl formed in the MFMA factorisation), the
#     128-B-aligned stage-record variant, and the separate acl_pass (round-3 structure; same bits expected)
#  3. SQ wave-state and MFMA counters of k_dg at the driver's launch shape (bench.py --steps 20 --warmup 5)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04a}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib -o run -- $R/tools/probes/fetch_calib > $O/calib.jsonl 2> $O/calib.err && echo calib_ok &&
timeout -k 10 300 python3 $R/tools/dg_probe.py --B 60000 --groups 0 704 1760 --save $O/stats60k > $O/sweep_product.jsonl 2> $O/sweep_product.err && cat $O/sweep_product.jsonl &&
VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_rec256.so timeout -k 10 200 python3 $R/tools/dg_probe.py --B 60000 --groups 0 > $O/sweep_rec256.jsonl 2> $O/sweep_rec256.err && cat $O/sweep_rec256.jsonl &&
VBOC_LIB=$R/vboc_amd/variants/libvboc_amd_aclpass.so timeout -k 10 200 python3 $R/tools/dg_probe.py --B 60000 --groups 0 > $O/sweep_aclpass.jsonl 2> $O/sweep_aclpass.err && cat $O/sweep_aclpass.jsonl &&
timeout -s KILL 330 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --output-format csv -d $O/sqa -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_sqa.json 2> $O/sqa.err && echo sqa_ok &&
timeout -s KILL 330 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/sqb -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --progress 30 > $O/bench_sqb.json 2> $O/sqb.err && echo sqb_ok &&
timeout -k 10 300 python3 -u -m pytest $R/tests/test_learn.py -m gpu -v --timeout 280 --timeout-method thread > $O/pytest_learn.log 2>&1 && echo learn_ok
