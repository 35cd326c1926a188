#!/bin/bash
# new fusion tests first, then the full GPU suite + smoke + a short bench + the bf16 per-parameter bound data
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06full}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > $O/t_g8w.log 2>&1; rc=$?
tail -3 $O/t_g8w.log; [ $rc -eq 0 ] || { grep -E "^E |Error" $O/t_g8w.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']]);print([(k['kernel'][:40],k['total_ms_per_step']) for k in d['top_kernels']])"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" $O/t.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u tools/diag_bf16_bounds.py $O/bf16_bounds.json > $O/bounds.log 2>&1 || { echo BOUNDS_FAIL; tail -5 $O/bounds.log; exit 1; }
tail -3 $O/bounds.log
