# same-box bench A/B over one env var, printing the traced rows matching PAT: ENVVAR=.. VALS=".." PAT=".." bash tools/ab_rows.sh
mkdir -p gpurun_out
for v in $VALS; do
  env $ENVVAR=$v timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline --steps 20 --trace-out gpurun_out/rows_$v.json > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { echo BENCH_FAIL $v; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "
import json, re; d=json.load(open('gpurun_out/ab_$v.json')); print('$ENVVAR=$v', d['value'], d['ms_per_step_median'])
for r in json.load(open('gpurun_out/rows_$v.json')):
    if re.search('$PAT', r['kernel']): print('   %7.3f ms x%4.1f %6.0f TF  %s' % (r['avg_ms'], r['launches_per_step'], r['tflops'], r['kernel']))"
done
