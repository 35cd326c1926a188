# action-head implicit dW: its tests + the parity tests + a short headline bench (tools only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05dw}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_action_head_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error|passed|failed" $O/t.log | head -30; tail -3 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --other-configs "" --no-cpu-baseline --h2d-steps 0 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --other-configs "" --no-cpu-baseline --h2d-steps 0 --config pusht_joint > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -5 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo PROF_OK
