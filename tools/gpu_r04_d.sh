# GEMM residual-ring epilogue + unrolled act_drop_fwd + tap-major im2col: tests, kernel A/B, bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm8_gpu.py tests/test_kernels_gpu.py tests/test_action_head_gpu.py tests/test_torch_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for L in new gemmbase; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py resgemm 2>&1 | grep -v amdgpu.ids || exit 1
  done
  for L in new ewbase; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py rowk 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 400 python -u bench.py --steps 30 --other-configs "" --no-cpu-baseline --h2d-steps 0 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step']); [print(k) for k in d['top_kernels']]"
