#!/bin/bash
# the driver's bench command, timed (wall budget check with the per-GPU-batch CPU step back on)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
s=$(date +%s)
timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_default.json 2> gpurun_out/r06/bench_default.err; rc=$?
e=$(date +%s); echo "rc=$rc wall=$((e-s)) s"
tail -5 gpurun_out/r06/bench_default.err
python -c "import json;d=json.loads(open('gpurun_out/r06/bench_default.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],[(o['config'],o.get('precision'),o['value']) for o in d['other_configs']]);print(d['cpu_baseline']);print(d['roofline'])"
