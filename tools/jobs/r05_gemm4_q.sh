set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_g4sp48.so -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py 2>&1 | tail -2 || exit 1
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_g4sp28.so -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py 2>&1 | tail -2 || exit 1
for i in 1 2; do
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py dwquick || exit 1
timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
for d in sp28 sp48; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py dwquick 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
done
