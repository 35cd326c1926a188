# ILV conv tuning: in-tree (ratio 2, from tap 2) vs ratio 3 / ratio 1 / from tap 3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t_new.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t_new.log | head -20; tail -3 $O/t_new.log; exit 1; }
echo "new $(tail -1 $O/t_new.log)"
for i in 1 2; do
  for L in new r3 r1 t3; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv | grep -v nores || exit 1
  done
done
echo "== new conv levels"; timeout -k 10 300 python tools/tools_kbench.py conv 2>&1 | grep conv3x3 || exit 1
