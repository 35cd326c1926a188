#!/bin/bash
# Round-4 end profile: kernel trace + stats of the default bench (main config + PushT joint line), per-grid
# dispatch stats, PMC FETCH_SIZE / WRITE_SIZE passes (separate runs, no tracing domains) -> traffic json,
# and the MFMA-busy PMC pass (tools/pmc_step.sh).  bash tools/profile_r03.sh <tag>
set -e
TAG=${1:-r04_end}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --trace-out $OUT/trace_rows.json > $OUT/bench.json 2> $OUT/bench.err
KT=$(find $OUT/kt -name "run_kernel_trace.csv" | head -1)
KS=$(find $OUT/kt -name "run_kernel_stats.csv" | head -1)
cp $KS $OUT/kernel_stats.csv
python3 tools/kt_by_grid.py $KT $OUT/kernel_stats_by_grid.csv > /dev/null
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --other-configs "" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --other-configs "" > $OUT/pmc_write.log 2>&1
python3 tools/tools_traffic.py $(dirname $(find $OUT/pmc_fetch -name run_counter_collection.csv | head -1)) \
  $(dirname $(find $OUT/pmc_write -name run_counter_collection.csv | head -1)) $OUT/traffic.json
bash tools/pmc_step.sh
cp gpurun_out/pmc_mfma/mfma.json $OUT/mfma_busy.json
rm -rf $OUT/kt $OUT/pmc_fetch $OUT/pmc_write
echo done
