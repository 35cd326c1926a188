# GN conv with the whole residual tile prefetched (VAR 320) vs in-tree (VAR 64); shared-exp GELU grad
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_convres.so -m pytest tests/test_conv_halo_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > $O/convres_tests.log 2>&1 || { echo CONVRES_TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/convres_tests.log | head -30; tail -5 $O/convres_tests.log; exit 1; }
tail -1 $O/convres_tests.log
for i in 1 2; do
  for L in new convres; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep -v amdgpu.ids || exit 1
  done
  for L in new ewbase; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py rowk 2>&1 | grep -E "act_" || exit 1
  done
done
