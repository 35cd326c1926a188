# dQ kernel variants: 3 workgroups per CU (168 VGPRs), key-half software pipelining, both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
for L in dq3 dq3pipe dqpipe; do
  timeout -k 10 200 python -u tools/ab_run.py abx/libuva_$L.so -m pytest tests/test_attention_gpu.py -x -q --timeout 100 --timeout-method thread > $O/t_$L.log 2>&1 || { echo "TESTS_FAIL $L"; grep -E "^E  |FAILED|Error" $O/t_$L.log | head -20; exit 1; }
  echo "$L $(tail -1 $O/t_$L.log)"
done
for i in 1 2; do
  for L in new dq3 dq3pipe dqpipe; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep -E "H=12 p=" || exit 1
  done
done
