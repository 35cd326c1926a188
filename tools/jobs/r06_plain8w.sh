#!/bin/bash
# bench A/B: remaining plain products on gemm_8w (RT.gemm8w_plain) vs gemm_4w, interleaved twice, same box
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
for i in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python tools/bench_flag.py gemm8w_plain=$v --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/r06/pl.json 2> gpurun_out/r06/pl.err || { tail -20 gpurun_out/r06/pl.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r06/pl.json')); print('gemm8w_plain=$v', d['value'], d['ms_per_step_median'])"
  done
done
