set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in base maskfree base; do
  if [ $L = base ]; then unset UVA_LIB_PATH; else export UVA_LIB_PATH=$PWD/ab/diag_$L.so; fi
  timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/db_$L.json 2>gpurun_out/db_$L.err || { tail -20 gpurun_out/db_$L.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/db_$L.json')); print('$L', d['value'], d['ms_per_step_median'])"
done
