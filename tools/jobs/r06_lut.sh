#!/bin/bash
# GELU / GELU' from a bf16-indexed table (abx/libuva_lut.so) vs evaluated: bit-exact tests, then timings
set -o pipefail
cd /root/repo
timeout -k 10 400 python tools/ab_run.py abx/libuva_lut.so -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py -k "fc1 or dgelu or block" 2>&1 | tail -2
for i in 1 2; do
  echo "== default"; timeout -k 10 300 python -u tools/gemm8w_bench.py fused 2>&1 | grep -E "round 1" -A20 | grep -E "nw8\] (fc1|fc2 dX)" || exit 1
  echo "== lut"; timeout -k 10 300 python -u tools/ab_run.py abx/libuva_lut.so tools/gemm8w_bench.py fused 2>&1 | grep -E "round 1" -A20 | grep -E "nw8\] (fc1|fc2 dX)" || exit 1
done
