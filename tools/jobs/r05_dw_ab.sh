# same-box A/B of the dW products (split-K + reduce): abx/libuva_base.so vs the in-tree build (tools only)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py tests/test_action_head_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/dwab_t.log 2>&1 || { echo TEST_FAIL; grep -E "^E  |FAILED" gpurun_out/dwab_t.log | head; exit 1; }
tail -1 gpurun_out/dwab_t.log
for i in 1 2; do
  echo "== base"; timeout -k 10 120 python tools/ab_run.py abx/libuva_base.so tools/dw_bench.py || exit 1
  echo "== new"; timeout -k 10 120 python tools/dw_bench.py || exit 1
done
