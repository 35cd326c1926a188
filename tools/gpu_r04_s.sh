# checkpoint bench of the current tree (default driver command) + headline kernel stats under rocprofv3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_ms']); [print(o['config'], o['precision'], o['value']) for o in d['other_configs']]; [print(k) for k in d['top_kernels']]"
