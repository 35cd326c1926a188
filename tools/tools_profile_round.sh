#!/bin/bash
# Round profile: rocprofv3 kernel-trace/stats of the bench, then two PMC passes (FETCH_SIZE,
# WRITE_SIZE; separate runs, no tracing domains) for tools_traffic.py.  Run from the repo root on
# the GPU box:  bash tools/tools_profile_round.sh <tag>
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --trace-out $OUT/trace_rows.json > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
echo done
