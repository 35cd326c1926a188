# same-box bench A/B over builds: in-tree ("new") and each abx/libuva_*.so, interleaved twice
# (python bench.py --steps 30, headline config only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for L in new abx/libuva_*.so; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py $L"; fi
    timeout -k 10 300 $PY bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/abb.json 2>gpurun_out/abb.err || { tail -20 gpurun_out/abb.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/abb.json')); print('$L', d['value'], d['ms_per_step_median'])"
  done
done
