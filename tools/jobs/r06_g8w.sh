#!/bin/bash
# gemm_8w kernel bench (plain + fused Mlp forwards, bit-exactness vs the split route), then the same-box
# r04 / r05 / HEAD A/B (tools/jobs/r06_r04_vs_head.sh)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 240 python -u tools/gemm8w_bench.py all > gpurun_out/r06/g8w_bench.txt 2>&1 || { tail -30 gpurun_out/r06/g8w_bench.txt; exit 1; }
cat gpurun_out/r06/g8w_bench.txt
bash tools/jobs/r06_r04_vs_head.sh
