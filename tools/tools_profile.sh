#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root): kernel trace + stats of the
# bench command, then one PMC pass per TCC counter group (FETCH_SIZE, WRITE_SIZE), as
# MI355X_MICROARCH.md §HBM / §rocprofv3 PMC slots prescribe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof
mkdir -p $OUT
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --trace-out $OUT/trace_rows.json > $OUT/bench_plain.json 2> $OUT/bench_plain.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_ktrace.json 2> $OUT/bench_ktrace.err || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-trace > $OUT/bench_pmc1.json 2> $OUT/bench_pmc1.err || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run -- \
    python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-trace > $OUT/bench_pmc2.json 2> $OUT/bench_pmc2.err || exit $?
echo profile-done
