set -o pipefail
export TMPDIR=/tmp
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py dwquick || exit 1
for d in d1 d2 d8; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py dwquick 2>&1 | grep -v amdgpu.ids || exit 1
done
