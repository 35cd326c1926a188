set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
for d in 1 2 3 4 8 9; do
  echo "== diag $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4d$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 400 bash tools/pmc_kernel.sh g4_fc2fwd gemm_4w tools/gemm4_one.py 768 3072 > $O/pmc_fc2.txt 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_fc2.txt; exit 1; }
cat $O/pmc_fc2.txt
timeout -k 10 400 bash tools/pmc_kernel.sh g4_fc1fwd gemm_4w tools/gemm4_one.py 3072 768 > $O/pmc_fc1.txt 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_fc1.txt; exit 1; }
cat $O/pmc_fc1.txt
