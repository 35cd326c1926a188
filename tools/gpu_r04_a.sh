# round 4 first GPU pass: host CPU quota probe, new sampler / attention parity tests, default bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04a
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > gpurun_out/r04a/host.txt 2>&1
timeout -k 10 500 python -u -m pytest tests/test_sampler_gpu.py tests/test_attention_gpu.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r04a/tests.log 2>&1 || { echo TEST_FAIL; grep -E "^E  |FAILED|Error|mean" gpurun_out/r04a/tests.log | head -40; tail -5 gpurun_out/r04a/tests.log; exit 1; }
tail -3 gpurun_out/r04a/tests.log
grep -E "persistent mean" gpurun_out/r04a/tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r04a/bench.err; exit 1; }
cat gpurun_out/r04a/bench.json
