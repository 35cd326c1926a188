# GN conv: 3-deep weight ring (VAR 3136) vs in-tree (1088)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_w3.so -m pytest tests/test_conv_halo_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "w3 $(tail -1 $O/t.log)"
for i in 1 2 3; do
  for L in new w3; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv | grep -v nores || exit 1
  done
done
for L in new w3; do
  if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
  echo "== $L levels"; timeout -k 10 300 $PY tools/tools_kbench.py conv 2>&1 | grep "64x64 Ci256" || exit 1
done
