# kernel trace of the headline step alone (10 timed + 3 warm-up steps): kernel time per step vs wall
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" --h2d-steps 0 --no-trace > $O/bench.json 2> $O/bench.err || { echo PROF_FAIL; tail -20 $O/bench.err; exit 1; }
KT=$(find $O/kt -name "run_kernel_trace.csv" | head -1)
KS=$(find $O/kt -name "run_kernel_stats.csv" | head -1)
cp $KS $O/kernel_stats.csv
python3 tools/kstats_per_step.py $O/kernel_stats.csv 60 > $O/per_step.txt
python3 tools/step_gaps.py $KT > $O/gaps.txt
rm -rf $O/kt
cat $O/bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('bench', d['value'], d['ms_per_step'])"
head -5 $O/per_step.txt; cat $O/gaps.txt
