#!/bin/bash
# two 4-wave workgroups per CU (gemm_8w NW = 4) vs one 8-wave workgroup: bit-exact tests, then timings
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > gpurun_out/r06/t_nw4.txt 2>&1; rc=$?; tail -2 gpurun_out/r06/t_nw4.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r06/t_nw4.txt | head; exit 1; }
timeout -k 10 400 python -u tools/gemm8w_bench.py all > gpurun_out/r06/g8w_nw4.txt 2>&1 || { tail -20 gpurun_out/r06/g8w_nw4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06/g8w_nw4.txt
