# focused GPU tests + kernels-only vs tuned bench A/B on one box (+ optional MFMA PMC pass: PMC=1)
mkdir -p gpurun_out
FOCUS=${FOCUS:-tests/test_gemm8_gpu.py}
timeout -k 10 300 python -u -m pytest $FOCUS -x -q --timeout 120 --timeout-method thread > gpurun_out/focus.log 2>&1 || { echo FOCUS_FAIL; tail -30 gpurun_out/focus.log; exit 1; }
tail -1 gpurun_out/focus.log
timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline > gpurun_out/bench_k.json 2>gpurun_out/bench_k.err || exit 1
timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline > gpurun_out/bench_t.json 2>gpurun_out/bench_t.err || exit 1
python3 - <<'PY'
import json
for f in ('k', 't'):
    d = json.load(open('gpurun_out/bench_%s.json' % f))
    print(f, d['value'], d['ms_per_step_median'], [(k['kernel'][:40], k['avg_ms'], k['tflops']) for k in d['top_kernels'][:8]])
PY
if [ "${PMC:-0}" = 1 ]; then bash tools/pmc_step.sh; fi
