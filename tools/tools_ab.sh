#!/bin/bash
# Same-box A/B of an env switch on the full bench: bash tools/tools_ab.sh VAR "A B" [rounds]
# prints value per run, alternating A, B, A, B ... (box-to-box variance is ~2-5 %, larger than
# most single changes).  Two builds of the library: tools/ab_bench.sh.
VAR=$1; VALS=$2; R=${3:-2}
for r in $(seq $R); do for v in $VALS; do
  tag=$(echo "$v" | tr '/.' '__')
  env $VAR=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-trace > gpurun_out/ab_$tag.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); print('$VAR=$v', d['value'], d['ms_per_step'])"
done; done
