# which memory copies a bench step issues: kernel + memory-copy trace of 2 steps (no PMC)
export TMPDIR=/tmp
mkdir -p gpurun_out/copies
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/copies -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --other-configs "" --no-trace > gpurun_out/copies/bench.json 2> gpurun_out/copies/bench.err
echo rc=$?
ls gpurun_out/copies
