#!/bin/bash
# EPI 3 row-0 prefetch before the last K-group (abx/libuva_pf3.so) vs row-ahead only (default): tests, timings
set -o pipefail
cd /root/repo
timeout -k 10 400 python tools/ab_run.py abx/libuva_pf3.so -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py -k "dgelu or block" 2>&1 | tail -2
for i in 1 2; do
  echo "== default"; timeout -k 10 300 python -u tools/gemm8w_bench.py fused 2>&1 | grep "dgelu" | grep -v planes || exit 1
  echo "== pf3"; timeout -k 10 300 python -u tools/ab_run.py abx/libuva_pf3.so tools/gemm8w_bench.py fused 2>&1 | grep "dgelu" | grep -v planes || exit 1
done
