set -o pipefail
export TMPDIR=/tmp
for d in d1 d32; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py dwquick 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
