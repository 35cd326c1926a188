set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm4_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error|passed|failed" $O/t.log | head -30; exit 1; }
tail -1 $O/t.log
echo "== base"; timeout -k 10 120 python -u tools/gemm4_bench.py quick || exit 1
for d in d2 d4; do
  echo "== $d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_g4$d.so tools/gemm4_bench.py quick 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 300 python -u tools/gemm4_bench.py 2 2>&1 | grep -v amdgpu.ids || exit 1
