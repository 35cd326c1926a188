# persistent GEMM (in-tree, bias prefetched a K-tile ahead) vs nopersist: parity + 3 interleaved blas rounds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm8_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_new.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t_new.log | head -20; tail -3 $O/t_new.log; exit 1; }
echo "new $(tail -1 $O/t_new.log)"
for i in 1 2 3; do
  for L in nopersist new; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py blas 2>&1 | grep "M=" | sed 's/  dw.*//' || exit 1
  done
done
