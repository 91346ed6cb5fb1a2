#!/bin/bash
# scratch: UR5 wave-solver bisection over build variants (one process per variant)
mkdir -p gpurun_out
out=gpurun_out/ur5_bisect.log
: > $out
true
for v in ${VARIANTS:-o3builtin o3nop o3m0clob o1builtin}; do
  VBOC_LIB=tools/scratch/so/lib_$v.so timeout -k 10 150 python -u tools/scratch/ur5_bisect.py tools/scratch/ref_ur5_96.npz ur5_$v >> $out 2>&1
  rc=$?
  echo "rc $v $rc" >> $out
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
cat $out
