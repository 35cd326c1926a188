# skinny dW split-K cap: parity + timing vs HEAD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_action_head_gpu.py tests/test_gemm8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests $(tail -1 $O/t.log)"
for L in base new; do
  if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
  echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py skinny 2>&1 | grep skinny || exit 1
done
