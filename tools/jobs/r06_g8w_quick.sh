#!/bin/bash
# gemm_8w change check: bit-exact tests, then the fused timings
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > gpurun_out/r06/t_q.txt 2>&1; rc=$?; tail -2 gpurun_out/r06/t_q.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06/t_q.txt | head; exit 1; }
timeout -k 10 400 python -u tools/gemm8w_bench.py fused > gpurun_out/r06/g8w_q.txt 2>&1 || { tail -20 gpurun_out/r06/g8w_q.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06/g8w_q.txt | grep -v planes
