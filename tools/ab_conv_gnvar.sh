# GN halo-conv variant $V (UVA_CONV_GN_VAR): conv tests under it, kernel timings vs the default, bench A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
UVA_CONV_GN_VAR=$V timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_v_t.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/conv_v_t.log; exit 1; }
tail -1 gpurun_out/conv_v_t.log
for v in 0 $V; do echo "== GN_VAR=$v"; UVA_CONV_GN_VAR=$v timeout -k 10 120 python tools/tools_kbench.py conv 2>&1 | grep -v amdgpu.ids | grep -v conv_in || exit 1; done
for v in $V 0; do
UVA_CONV_GN_VAR=$v timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline --steps 30 > gpurun_out/bench_v$v.json 2>gpurun_out/bench_v$v.err || { tail -20 gpurun_out/bench_v$v.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_v$v.json')); print('GN_VAR=$v', d['value'], d['ms_per_step_median'], [(k['kernel'][:40], k['avg_ms'], k['tflops']) for k in d['top_kernels'][:3]])"
done
