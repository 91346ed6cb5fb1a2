set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/groups_r03e; mkdir -p $O
for G in 1024 1408 1792 2048; do
  VBOC_GROUPS=$G timeout -k 10 120 python3 $R/tools/pass_probe.py 3 32768 > $O/g$G.json 2> $O/g$G.err || exit 1
  echo "G=$G $(cat $O/g$G.json)"
done
