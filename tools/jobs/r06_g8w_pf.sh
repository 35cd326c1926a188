#!/bin/bash
# gemm_8w row-input prefetch (default build) vs none (abx/libuva_nopf.so): tests, then alternating timings
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > gpurun_out/r06/t_pf.txt 2>&1; rc=$?; tail -2 gpurun_out/r06/t_pf.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06/t_pf.txt | head; exit 1; }
for i in 1 2; do
  echo "== prefetch (default)"; timeout -k 10 300 python -u tools/gemm8w_bench.py fused 2>&1 | grep -v amdgpu.ids | grep -v planes | grep -v "round 0" || exit 1
  echo "== no prefetch"; timeout -k 10 300 python -u tools/ab_run.py abx/libuva_nopf.so tools/gemm8w_bench.py fused 2>&1 | grep -v amdgpu.ids | grep -v planes || exit 1
done
