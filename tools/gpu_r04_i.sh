# GN conv: unconditional one-tap-ahead weight loads (in-tree) and + late residual rows (VAR 576) vs HEAD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 100 --timeout-method thread > $O/t_new.log 2>&1 || { echo "TESTS_FAIL new"; grep -E "^E  |FAILED|Error" $O/t_new.log | head -20; tail -3 $O/t_new.log; exit 1; }
echo "new $(tail -1 $O/t_new.log)"
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_rlate.so -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 100 --timeout-method thread > $O/t_rlate.log 2>&1 || { echo "TESTS_FAIL rlate"; grep -E "^E  |FAILED|Error" $O/t_rlate.log | head -20; tail -3 $O/t_rlate.log; exit 1; }
echo "rlate $(tail -1 $O/t_rlate.log)"
for i in 1 2; do
  for L in base new rlate; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv || exit 1
  done
done
timeout -k 10 200 python -u -m pytest tests/test_action_head_gpu.py -x -q -s -k mask_flips --timeout 100 --timeout-method thread > $O/t_mask.log 2>&1; echo "mask rc=$?"; grep -E "mask flips|passed|failed|Error" $O/t_mask.log | head
