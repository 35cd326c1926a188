set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in off on off on; do
  V=0; [ $L = on ] && V=1
  timeout -k 10 300 python tools/bench_flag.py act_bwd_in_gemm=$V --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || { tail -20 gpurun_out/ab_$L.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$L.json')); print('$L', d['value'], d['ms_per_step_median'], d['final_loss'])"
done
