# GN conv strip form (UVA_CONV_GN_STRIP): parity on the variant library, then conv kbench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_strip.so -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 100 --timeout-method thread > $O/t_strip.log 2>&1 || { echo "TESTS_FAIL strip"; grep -E "^E  |FAILED|Error" $O/t_strip.log | head -20; tail -3 $O/t_strip.log; exit 1; }
echo "strip $(tail -1 $O/t_strip.log)"
for i in 1 2; do
  for L in new strip; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv || exit 1
  done
done
