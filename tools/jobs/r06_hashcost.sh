#!/bin/bash
set -o pipefail
cd /root/repo
for i in 1 2; do
echo "== p=0.1"; timeout -k 10 300 python -u tools/gemm8w_bench.py fused 2>&1 | grep -E "round 1" -A20 | grep -v planes | grep -E "nw8" || exit 1
echo "== p=0"; timeout -k 10 300 python -u tools/gemm8w_bench.py fused_p0 2>&1 | grep -E "round 1" -A20 | grep -v planes | grep -E "nw8" || exit 1
done
