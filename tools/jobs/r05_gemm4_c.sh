set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error|passed|failed" $O/t.log | head -30; exit 1; }
tail -1 $O/t.log
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
for d in 1 4; do
  echo "== diag $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4d$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u tools/gemm4_bench.py 2 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 bash tools/pmc_kernel.sh g4c_fc2fwd gemm_4w tools/gemm4_one.py 768 3072 > $O/pmc_fc2.txt 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_fc2.txt; exit 1; }
cat $O/pmc_fc2.txt
