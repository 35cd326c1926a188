set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_sk384.so -m pytest tests/test_gemm8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "sk384 $(tail -1 $O/t.log)"
for i in 1 2; do
  for L in new sk384; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py cold 2>&1 | grep "dW" || exit 1
  done
done
