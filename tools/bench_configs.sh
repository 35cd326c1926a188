#!/bin/bash
# BASELINE configs 3-5 at their per-GPU batches (1 GPU), bf16 and fp8 attention for UMI:
#   bash tools/bench_configs.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/r02}
mkdir -p $OUT
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs '' --no-trace "$@" \
    > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "FAIL $name"; tail -5 $OUT/bench_$name.err; exit 1; }
  cat $OUT/bench_$name.json
}
run pusht_joint_b64 --config pusht_joint --batch 64
run libero10_joint_b32 --config libero10_joint --batch 32
run umi_multi_b56_bf16 --config umi_multi --batch 56
run umi_multi_b56_fp8 --config umi_multi --batch 56 --precision fp8_attn
