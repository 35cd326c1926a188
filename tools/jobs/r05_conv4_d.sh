set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv4_gpu.py 2>&1 | tail -2 || exit 1
echo "== base"; timeout -k 10 120 python -u tools/conv4_quick.py 128 || exit 1
for d in 1 16; do
  echo "== d$d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_c4d$d.so tools/conv4_quick.py 128 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u tools/conv4_bench.py 256 || exit 1
