# Block parity against the reference's bf16 run on both GEMM routes (RT.blas_plain 3 / 0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ah
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k block_full_geometry -v --timeout 250 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
grep -E "PASSED|FAILED" $O/t.log; tail -1 $O/t.log
