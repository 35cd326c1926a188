#!/bin/bash
# rocprofv3 kernel stats of the main bench config only (BASELINE configs[1]); per-step figures by
# tools/kstats_per_step.py (divides by the adamw_ema launches = optimizer steps)
set -e
TAG=${1:-r03}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" > $OUT/bench.json 2> $OUT/bench.err
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
echo done
