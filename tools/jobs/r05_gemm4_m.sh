set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_run.py abx/libuva_g4blk.so -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py -k dw 2>&1 | tail -3 || exit 1
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py dwquick || exit 1
for d in blk blkd1; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py dwquick 2>&1 | grep -v amdgpu.ids || exit 1
done
