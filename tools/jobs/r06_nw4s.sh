#!/bin/bash
# NW = 4 with the grid's second half started later (stagger) vs the 8-wave form: timings only
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 500 python -u tools/gemm8w_bench.py fused > gpurun_out/r06/g8w_nw4s.txt 2>&1 || { tail -20 gpurun_out/r06/g8w_nw4s.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06/g8w_nw4s.txt | grep -E "fc1|dgelu|==" | grep -v planes
