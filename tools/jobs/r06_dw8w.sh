#!/bin/bash
# dW products on gemm_8w (k-major operands): tests, then timings against gemm_4w / gemm_8ph
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > gpurun_out/r06/t_dw.txt 2>&1; rc=$?; tail -2 gpurun_out/r06/t_dw.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06/t_dw.txt | head; exit 1; }
timeout -k 10 300 python -u tools/dw_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r06/dw_bench.txt
