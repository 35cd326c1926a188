set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FOCUS="tests/test_gemm8_gpu.py" bash tools/tools_gpu_check.sh || exit 1
timeout -k 10 300 python tools/bench_flag.py act_bwd_in_gemm=0 --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/ab_off.json 2> gpurun_out/ab_off.err || { tail -20 gpurun_out/ab_off.err; exit 1; }
timeout -k 10 300 python tools/bench_flag.py act_bwd_in_gemm=1 --other-configs "" --no-cpu-baseline --steps 30 --no-trace > gpurun_out/ab_on.json 2> gpurun_out/ab_on.err || { tail -20 gpurun_out/ab_on.err; exit 1; }
for L in off on; do python3 -c "
import json; d=json.load(open('gpurun_out/ab_$L.json')); print('$L', d['value'], d['ms_per_step_median'], d['final_loss'])"; done
