set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_a8prio.so -m pytest tests/test_attention_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "a8prio $(tail -1 $O/t.log)"
for i in 1 2 3; do
  for L in new a8prio; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep "fp8 quant" || exit 1
  done
done
