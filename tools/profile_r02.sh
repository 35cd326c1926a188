# round-2 profile: kernel trace/stats of the bench + FETCH/WRITE PMC passes + MFMA-busy PMC pass
set -e
export TMPDIR=/tmp
bash tools/tools_profile_round.sh ${1:-r02}
python3 tools/tools_traffic.py gpurun_out/prof_${1:-r02}/pmc_fetch gpurun_out/prof_${1:-r02}/pmc_write gpurun_out/prof_${1:-r02}/traffic.json > /dev/null
bash tools/pmc_step.sh
cp gpurun_out/pmc_mfma/mfma.json gpurun_out/prof_${1:-r02}/mfma_busy.json
python3 -c "
import json; d=json.load(open('gpurun_out/prof_${1:-r02}/bench.json')); print(d['value'], d['roofline'])"
# keep the merge-back under gpurun's 64 MiB cap: drop the raw per-dispatch CSVs (stats, traffic and
# MFMA summaries above are what profiles/ keeps)
python3 tools/kt_by_grid.py gpurun_out/prof_${1:-r02}/kt/run_kernel_trace.csv gpurun_out/prof_${1:-r02}/kernel_stats_by_grid.csv || { ls gpurun_out/prof_${1:-r02}/kt; head -2 gpurun_out/prof_${1:-r02}/kt/*trace*.csv; }
find gpurun_out -name "*.csv" -size +4M -delete
du -sh gpurun_out
