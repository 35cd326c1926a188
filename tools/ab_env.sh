# same-box bench A/B over one environment variable: ENVVAR=<name> VALS="a b ..." bash tools/ab_env.sh
mkdir -p gpurun_out
for v in $VALS; do
  env $ENVVAR=$v timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { echo BENCH_FAIL $v; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$ENVVAR=$v', d['value'], d['ms_per_step_median'], [(k['kernel'][:34], k['avg_ms']) for k in d['top_kernels'][:6]])"
done
