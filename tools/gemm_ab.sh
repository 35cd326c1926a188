#!/bin/bash
# A/B of an env switch on the hand-written GEMMs (square + training shapes): bash tools/gemm_ab.sh VAR "A B"
V=$1; VALS=$2
for v in $VALS; do
  echo "== $V=$v"
  env $V=$v UVA_GEMM_LIB=0 timeout -k 10 200 python -c 'import sys; sys.path.insert(0,"tools"); sys.path.insert(0,"."); import tools_kbench as k; k.square_bench()' 2>&1 | grep square
  env $V=$v timeout -k 10 300 python tools/gemm_gap.py 2>&1 | grep -v amdgpu.ids
done
