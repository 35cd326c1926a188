export TMPDIR=/tmp
mkdir -p gpurun_out/kt
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python3 tools/tools_attn_one.py > gpurun_out/kt/log.txt 2>&1
echo rc=$?
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/kt/run_kernel_stats.csv')):
    if 'attn' in r['Name']: print('%8.1f us  %3s  %s' % (float(r['AverageNs'])/1e3, r['Calls'], r['Name'][:60]))
PY
