# kernel survey on the in-tree build: GEMM shapes, attention, square GEMMs, row kernels; mask-flip evidence test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_action_head_gpu.py -x -q -s -k mask_flips --timeout 100 --timeout-method thread > $O/t_mask.log 2>&1; echo "mask rc=$?"; grep -E "mask flips|passed|failed|Error" $O/t_mask.log | head
for m in "" square rowk resgemm; do
  echo "== kbench $m"; timeout -k 10 300 python tools/tools_kbench.py $m 2>&1 | grep -v amdgpu.ids || exit 1
done
