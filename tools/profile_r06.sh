#!/bin/bash
# End-of-round profile (tools only).  All files under profiles/<tag>/ come from THIS run:
#   kernel_stats.csv / kernel_stats_by_grid.csv / trace_rows.json / bench.json : rocprofv3 --kernel-trace --stats
#       of the default bench command (headline + the other-config lines), bench's own HIP-event rows beside it
#   kernel_stats_headline_only.csv / step_gaps.txt : a headline-only traced run (busy / idle per optimizer step)
#   traffic.json : FETCH_SIZE / WRITE_SIZE passes (separate runs, no tracing domains), per traced tag
#   mfma_busy.json : SQ_VALU_MFMA_BUSY_CYCLES pass (tools/pmc_step.sh)
# bash tools/profile_r06.sh <tag>
set -e
set -o pipefail
TAG=${1:-r06_end}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 20 --no-cpu-baseline --trace-out $OUT/trace_rows.json > $OUT/bench.json 2> $OUT/bench.err
KT=$(find $OUT/kt -name "run_kernel_trace.csv" | head -1)
cp $(find $OUT/kt -name "run_kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
python3 tools/kt_by_grid.py $KT $OUT/kernel_stats_by_grid.csv > /dev/null
echo trace_default_ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kth -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" --h2d-steps 0 > $OUT/bench_headline.json 2> $OUT/bench_headline.err
KTH=$(find $OUT/kth -name "run_kernel_trace.csv" | head -1)
cp $(find $OUT/kth -name "run_kernel_stats.csv" | head -1) $OUT/kernel_stats_headline_only.csv
python3 tools/step_gaps.py $KTH > $OUT/step_gaps.txt
echo trace_headline_ok
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --other-configs "" --h2d-steps 0 > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --other-configs "" --h2d-steps 0 > $OUT/pmc_write.log 2>&1
python3 tools/tools_traffic.py $(dirname $(find $OUT/pmc_fetch -name run_counter_collection.csv | head -1)) \
  $(dirname $(find $OUT/pmc_write -name run_counter_collection.csv | head -1)) $OUT/traffic.json
echo traffic_ok
bash tools/pmc_step.sh
cp gpurun_out/pmc_mfma/mfma.json $OUT/mfma_busy.json
rm -rf $OUT/kt $OUT/kth $OUT/pmc_fetch $OUT/pmc_write
echo done
