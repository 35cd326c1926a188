#!/bin/bash
# fused Mlp routes on the 8-wave GEMM: bit-exactness tests, kernel timings, a short bench, the bf16 parity suite
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > gpurun_out/r06/t_g8w.txt 2>&1; rc=$?; tail -15 gpurun_out/r06/t_g8w.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/gemm8w_bench.py fused > gpurun_out/r06/g8w_fused.txt 2>&1 || { tail -20 gpurun_out/r06/g8w_fused.txt; exit 1; }
cat gpurun_out/r06/g8w_fused.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --other-configs pusht_joint:64 --other-steps 15 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r06/bench_fused.json 2> gpurun_out/r06/bench_fused.err || { tail -20 gpurun_out/r06/bench_fused.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06/bench_fused.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],[o['value'] for o in d['other_configs']]);print(json.dumps(d['top_kernels'],indent=0)[:3000]);print(d['roofline']);print(d['trace_accounting'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "bf16 or block" > gpurun_out/r06/t_parity.txt 2>&1; rc=$?; tail -8 gpurun_out/r06/t_parity.txt; exit $rc
