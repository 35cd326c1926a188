set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py -x -v --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/ps_t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/ps_t.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_sampler_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ps_t2.log 2>&1 || { tail -20 gpurun_out/ps_t2.log; exit 1; }
tail -2 gpurun_out/ps_t2.log
timeout -k 10 200 python tools/tools_infer_bench.py --batches 1,32 --iters 10 2>&1 | grep -v amdgpu.ids
