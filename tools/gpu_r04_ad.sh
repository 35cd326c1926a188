# attention backward without the scaled-dO copy (dropout scale folded into D and the final dK/dQ/dV)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_attention_fp8_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests $(tail -1 $O/t.log)"
for i in 1 2 3; do
  for L in base new; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep "H=12 p=" || exit 1
  done
done
