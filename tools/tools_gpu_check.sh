# GPU round-trip: [focused tests] -> full -m gpu suite -> smoke -> bench (+ per-kernel trace rows)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$FOCUS" ]; then
  timeout -k 10 300 python -u -m pytest $FOCUS -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_focus.log 2>&1 || { echo FOCUS_FAIL; tail -40 gpurun_out/pytest_focus.log; exit 1; }
  tail -2 gpurun_out/pytest_focus.log
fi
if [ -n "$KB" ]; then
  timeout -k 10 200 python tools/tools_kbench.py $KB > gpurun_out/kb.log 2>&1 || { echo KB_FAIL; tail -20 gpurun_out/kb.log; exit 1; }
  cat gpurun_out/kb.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --trace-out gpurun_out/trace_rows.json > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
