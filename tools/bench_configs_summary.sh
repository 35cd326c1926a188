# run tools/bench_configs.sh into $1 and print one summary line per config
bash tools/bench_configs.sh $1 > $1.log 2>&1 || { tail -20 $1.log; exit 1; }
python3 - "$1" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], d["value"], d["ms_per_step_median"], d.get("dtype"))
PY
