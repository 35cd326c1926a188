# hipBLASLt kernel names / times for the Block products (which tiles the vendor picks)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04k
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04k/prof -o run -- python $GRAFT_REPO_ROOT/tools/tools_kbench.py blas > $GRAFT_REPO_ROOT/gpurun_out/r04k/blas.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; echo rc=$rc; grep "M=" gpurun_out/r04k/blas.log
f=$(find gpurun_out/r04k/prof -name "*kernel_stats.csv" | head -1); echo $f
python - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:30]:
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:230]}")
PY
