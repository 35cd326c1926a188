# same-box A/B: attention keep-mask prefetch on the side stream (default) vs inline masks (tools only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05pf
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --other-configs "" --no-cpu-baseline --h2d-steps 0 --no-trace > $O/on$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u tools/bench_flag.py attn_prefetch=0 --steps 20 --warmup 5 --other-configs "" --no-cpu-baseline --h2d-steps 0 --no-trace > $O/off$i.json 2>/dev/null || exit 1
  python3 -c "import json; a=json.load(open('$O/on$i.json')); b=json.load(open('$O/off$i.json')); print('prefetch on', a['value'], a['ms_per_step'], '| off', b['value'], b['ms_per_step'])"
done
