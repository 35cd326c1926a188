# same-box A/B of the in-tree build against abx/libuva_base.so: focused tests ($FOCUS) on the new build,
# then kbench mode $KB and the bench (short) on both builds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$FOCUS" ]; then
  timeout -k 10 400 python -u -m pytest $FOCUS -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_t.log 2>&1 || { echo TEST_FAIL; tail -30 gpurun_out/ab_t.log; exit 1; }
  tail -1 gpurun_out/ab_t.log
fi
for L in base new; do
  if [ $L = base ]; then PY="python tools/ab_run.py abx/libuva_base.so"; else PY=python; fi
  if [ -n "$KB" ]; then echo "== $L kbench $KB"; timeout -k 10 200 $PY tools/tools_kbench.py $KB 2>&1 | grep -v amdgpu.ids || exit 1; fi
  if [ -n "$PYB" ]; then echo "== $L $PYB"; timeout -k 10 200 $PY $PYB 2>&1 | grep -v amdgpu.ids || exit 1; fi
  [ -n "$NOBENCH" ] && continue
  timeout -k 10 300 $PY bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/ab_$L.json 2>gpurun_out/ab_$L.err || { tail -20 gpurun_out/ab_$L.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$L.json')); print('$L', d['value'], d['ms_per_step_median'])"
done
