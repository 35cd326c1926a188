#!/bin/bash
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > gpurun_out/r06/t_g8w.txt 2>&1; rc=$?; tail -5 gpurun_out/r06/t_g8w.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/gemm8w_bench.py fused > gpurun_out/r06/g8w_planes.txt 2>&1 || { tail -20 gpurun_out/r06/g8w_planes.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06/g8w_planes.txt
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r06/bench_planes.json 2> gpurun_out/r06/bench_planes.err || { tail -20 gpurun_out/r06/bench_planes.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06/bench_planes.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']]);print([(k['kernel'][:40],k['total_ms_per_step']) for k in d['top_kernels']])"
timeout -k 10 300 python -u tools/bench_flag.py drop_planes=0 --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 --no-trace > gpurun_out/r06/bench_noplanes.json 2> gpurun_out/r06/bench_noplanes.err || { tail -20 gpurun_out/r06/bench_noplanes.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06/bench_noplanes.json').read().strip().splitlines()[-1]);print('no planes', d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']])"
