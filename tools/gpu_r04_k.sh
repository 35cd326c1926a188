# hipBLASLt kernel names / times for the Block products (which tiles the vendor picks)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/tools_kbench.py blas > $O/blas.log 2>&1
echo rc=$?; grep "M=" $O/blas.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); echo $f
python - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:30]:
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:230]}")
PY
