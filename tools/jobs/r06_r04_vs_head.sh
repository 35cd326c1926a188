#!/bin/bash
# Same-box A/B: the round-4 tree (abx/r04, d2e9478), the round-5 tree (abx/r05, 7da44fb), each with its own
# libuva_hip.so, and the working tree (+ its mask prefetch at VAE level 0 = the round-5 placement), interleaved.
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06ab
A="--steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 --no-trace"
run() {  # name dir [python-args...]
  local name=$1 dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python -u "$@") > gpurun_out/r06ab/$name.json 2> gpurun_out/r06ab/$name.err || exit 1
  echo "$name: $(python -c "import json,sys;d=json.loads(open('gpurun_out/r06ab/$name.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], [o['value'] for o in d.get('other_configs',[])])")"
}
for i in 1 2; do
  run head_$i . bench.py $A
  run r05_$i abx/r05 bench.py $A
  run r04_$i abx/r04 bench.py $A
  run headL0_$i . -c "import sys; sys.argv=['bench.py']+sys.argv[1:]; import bench; from unified_video_action_amd.runtime import RT; RT.attn_prefetch_level=0; bench.main()" $A
done
