# full GPU check of the current tree: -m gpu suite, smoke, default bench (driver command)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r04m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac']); [print(o['config'], o['precision'], o['value']) for o in d['other_configs']]; print(d['cpu_baseline']['value'])"
