set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
for d in d4 d16; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
done
