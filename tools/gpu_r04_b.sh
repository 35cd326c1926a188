# round 4 second GPU pass: full GPU suite, GN-conv variants (kbench conv0: base / DPP epilogue / +
# pipelined A reads), conv tests on the pipelined build, default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo GPU_TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_convpipe.so -m pytest tests/test_conv_halo_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pipe_tests.log 2>&1 || { echo PIPE_TESTS_FAIL; grep -E "^E  |FAILED|Error" $O/pipe_tests.log | head -30; tail -5 $O/pipe_tests.log; exit 1; }
tail -1 $O/pipe_tests.log
for i in 1 2; do
  for L in base new convpipe; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --config pusht_joint --batch 64 --steps 5 --warmup 2 --other-configs "" --no-cpu-baseline --h2d-steps 0 --trace-out $O/trace_joint.json > $O/bench_joint.json 2> $O/bench_joint.err || { echo JOINT_FAIL; tail -5 $O/bench_joint.err; exit 1; }
