# full GPU suite + smoke + a short bench of the headline config (tools only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error|passed|failed" $O/t.log | head -30; tail -3 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --other-configs "${2-}" --no-cpu-baseline --h2d-steps 0 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac')); [print(v['config'], v['global_batch'], v['value'], v.get('precision')) for v in d.get('other_configs', [])]"
