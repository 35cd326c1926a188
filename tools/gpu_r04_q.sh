# persistent GN conv (UVA_CONV_GN_PT=1) vs in-tree (ILV single-tile): parity, kbench, PMC
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_pt.so -m pytest tests/test_conv_halo_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t_pt.log 2>&1 || { echo "TESTS_FAIL pt"; grep -E "^E  |FAILED|Error" $O/t_pt.log | head -20; tail -3 $O/t_pt.log; exit 1; }
echo "pt $(tail -1 $O/t_pt.log)"
for i in 1 2 3; do
  for L in new pt; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv || exit 1
  done
done
true
true
