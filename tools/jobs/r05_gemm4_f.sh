set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_workspace_gpu.py tests/test_conv_halo_gpu.py tests/test_attention_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error|passed|failed" $O/t.log | head -30; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
for d in d1 d2 d4; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 400 bash tools/pmc_kernel.sh g4f_fc1 gemm_4w tools/gemm4_one.py 3072 768 > $O/pmc_fc1.txt 2>&1 || { echo PMC_FAIL; tail -5 $O/pmc_fc1.txt; exit 1; }
cat $O/pmc_fc1.txt
