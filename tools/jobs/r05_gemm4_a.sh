set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error|passed|failed" $O/t.log | head -30; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python -u tools/gemm4_bench.py 2 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
cat $O/bench.log
