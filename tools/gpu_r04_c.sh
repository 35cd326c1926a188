# attention software-pipelined backward (UVA_ATT_PIPE=1, abx/libuva_attpipe.so): tests + kbench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_attpipe.so -m pytest tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > $O/attpipe_tests.log 2>&1 || { echo ATTPIPE_TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/attpipe_tests.log | head -30; tail -5 $O/attpipe_tests.log; exit 1; }
tail -1 $O/attpipe_tests.log
for i in 1 2; do
  for L in new attpipe; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
