set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py 2>&1 | tail -15 || exit 1
timeout -k 10 180 python -u tools/gemm4_bench.py dw || exit 1
timeout -k 10 180 python -u tools/gemm4_bench.py 1 || exit 1
