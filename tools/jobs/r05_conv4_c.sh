set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv4_gpu.py tests/test_conv_halo_gpu.py 2>&1 | tail -4 || exit 1
timeout -k 10 300 python -u tools/conv4_bench.py 256 || exit 1
