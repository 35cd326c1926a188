set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py tests/test_gemm8_gpu.py 2>&1 | tail -2 || exit 1
timeout -k 10 300 python -u tools/gemm4_bench.py 2 || exit 1
timeout -k 10 300 python -u tools/gemm4_bench.py dw || exit 1
