# focused GPU tests ($FOCUS) then the bench without the extra configs / CPU baseline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $FOCUS -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_t.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/quick_t.log; exit 1; }
tail -1 gpurun_out/quick_t.log
timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline --steps 30 --trace-out gpurun_out/quick_rows.json > gpurun_out/quick_b.json 2>gpurun_out/quick_b.err || { tail -20 gpurun_out/quick_b.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/quick_b.json')); print(d['value'], d['ms_per_step_median'], [(k['kernel'][:40], k['avg_ms'], k['tflops']) for k in d['top_kernels'][:5]])"
