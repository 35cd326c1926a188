#!/bin/bash
# final tree: full GPU suite (as the driver runs it), smoke, then the driver's bench command timed
set -o pipefail
cd /root/repo
O=gpurun_out/r06final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" $O/t.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
s=$(date +%s)
timeout -k 10 590 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
e=$(date +%s); echo "bench rc=$rc wall=$((e-s)) s" | tee $O/bench_wall.txt
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],[(o['config'],o.get('precision'),o['value']) for o in d['other_configs']]);print(d['roofline'])"
