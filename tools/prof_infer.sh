# kernel trace of the inference bench (predict_action + sampler, B=1): per-kernel averages
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_infer
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_infer/kt -o run -- \
  python3 tools/tools_infer_bench.py --batches ${BATCHES:-1} --iters 5 > gpurun_out/prof_infer/infer.json 2> gpurun_out/prof_infer/infer.err || { tail -20 gpurun_out/prof_infer/infer.err; exit 1; }
cat gpurun_out/prof_infer/infer.json
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/prof_infer/kt/run_kernel_stats.csv')))
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:90]}")
PY
