# Round-4 call O (on the box via gpurun): do partial-line stores fetch their lines?  tools/probes/write_fill under
# two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE).  usage: bash tools/gpu_r04o.sh <out-subdir>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r04o}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $R/tools/probes/write_fill > $O/write_fill.jsonl 2> $O/fetch.err; rc=$?; echo "fetch exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $R/tools/probes/write_fill > /dev/null 2> $O/write.err; rc=$?; echo "write exit $rc"
cat $O/write_fill.jsonl
