# Per-pass bytes and time of the wave solver's IPM iteration (on the box via gpurun).
# For the product build and each pass-repeat build (vboc_amd/variants/libvboc_amd_rep<p>.so, -DVBOC_REPEAT=p,
# built on the CPU by tools/build_variants.sh): one timed run of tools/pass_probe.py, then separate rocprofv3
# --pmc passes (FETCH_SIZE; WRITE_SIZE; TCC_HIT_sum TCC_MISS_sum), summarised by tools/pass_split.py.
# usage: bash tools/pass_split.sh <out-subdir> [nq] [B] [variant ids...]
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-split}; mkdir -p $O; shift
NQ=${1:-3}; B=${2:-16384}; shift 2; IDS="${@:-0 1 2 3 4 5 6 7 8}"
cd /tmp && export TMPDIR=/tmp
for p in $IDS; do
  if [ "$p" = "0" ]; then L=$R/vboc_amd/libvboc_amd.so; else L=$R/vboc_amd/variants/libvboc_amd_rep$p.so; fi
  export VBOC_LIB=$L
  timeout -k 10 120 python3 $R/tools/pass_probe.py $NQ $B > $O/time_$p.json 2> $O/time_$p.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$p -o run -- python3 $R/tools/pass_probe.py $NQ $B > $O/fetch_$p.json 2> $O/fetch_$p.err || exit 2
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$p -o run -- python3 $R/tools/pass_probe.py $NQ $B > $O/write_$p.json 2> $O/write_$p.err || exit 3
  if [ "$p" = "0" ]; then
    timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc_$p -o run -- python3 $R/tools/pass_probe.py $NQ $B > $O/tcc_$p.json 2> $O/tcc_$p.err || exit 4
  fi
  echo "variant $p done: $(cat $O/time_$p.json)"
done
