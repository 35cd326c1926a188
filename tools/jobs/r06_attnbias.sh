#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ab2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_attention_gpu.py tests/test_gemm8w_gpu.py tests/test_workspace_gpu.py tests/test_attention_fp8_gpu.py > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" $O/t.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench',d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']]);print(d['trace_accounting'])"
timeout -k 10 300 python -u tools/bench_flag.py weight_t_prefetch=0 --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 --no-trace > $O/bench_nowt.json 2> $O/bench_nowt.err || { tail -20 $O/bench_nowt.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_nowt.json').read().strip().splitlines()[-1]);print('no wt prefetch',d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']])"
timeout -k 10 300 python -u tools/bench_flag.py attn_bias_grad=0 --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 --no-trace > $O/bench_noab.json 2> $O/bench_noab.err || { tail -20 $O/bench_noab.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_noab.json').read().strip().splitlines()[-1]);print('no attn bias grad',d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']])"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py > $O/tp.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" $O/tp.log | tail -10; exit $rc
