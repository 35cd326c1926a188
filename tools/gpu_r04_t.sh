# headline-config kernel stats of the current tree (13 steps) for re-ranking
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" --h2d-steps 0 > $O/bench.json 2> $O/bench.err || { echo FAIL; tail -5 $O/bench.err; exit 1; }
KS=$(find $O/kt -name "run_kernel_stats.csv" | head -1); cp $KS $O/kernel_stats.csv
KT=$(find $O/kt -name "run_kernel_trace.csv" | head -1); python3 tools/step_gaps.py $KT > $O/step_gaps.txt 2>&1 || true
rm -rf $O/kt
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'])"
