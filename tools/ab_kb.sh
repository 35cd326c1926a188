# same-box A/B: focused tests ($FOCUS) on the in-tree build, then kbench mode $KB on
# abx/libuva_base.so and the in-tree build (twice each, interleaved)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$FOCUS" ]; then
  timeout -k 10 500 python -u -m pytest $FOCUS -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_t.log 2>&1 || { echo TEST_FAIL; grep -E "^E  |FAILED|Error" gpurun_out/ab_t.log | head -30; tail -5 gpurun_out/ab_t.log; exit 1; }
  tail -1 gpurun_out/ab_t.log
fi
for i in 1 2; do
for L in base new; do
  if [ $L = base ]; then PY="python tools/ab_run.py abx/libuva_base.so"; else PY=python; fi
  echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py $KB 2>&1 | grep -v amdgpu.ids || exit 1
done
done
