#!/bin/bash
# Scratch: UR5 first-solve agreement for each experimental build variant
for v in _y2 _y3 _y4; do
  VBOC_LIB=vboc_amd/libvboc_amd$v.so timeout -k 10 120 python -u tools/scratch/ur5_first.py || exit 1
done
