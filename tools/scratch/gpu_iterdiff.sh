#!/bin/bash
mkdir -p gpurun_out; out=gpurun_out/ur5_iterdiff.log; : > $out
for v in ${VARIANTS}; do
  VBOC_LIB=tools/scratch/so/lib_$v.so timeout -k 10 150 python -u tools/scratch/ur5_iterdiff.py $v >> $out 2>&1 || exit 1
done
cat $out
