# halo-conv GN variants: tests, then per-variant kernel timings, then the bench (default build)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_t.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/conv_t.log; exit 1; }
tail -1 gpurun_out/conv_t.log
for v in 0 16; do echo "== GN_VAR=$v"; UVA_CONV_GN_VAR=$v timeout -k 10 120 python tools/tools_kbench.py conv 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline > gpurun_out/bench_c.json 2>gpurun_out/bench_c.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_c.json')); print(d['value'], d['ms_per_step_median'], [(k['kernel'][:40], k['avg_ms'], k['tflops']) for k in d['top_kernels'][:6]])"
