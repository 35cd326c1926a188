# fp8 quantisation row form vs per-head form (kbench attn), then the Block's epilogue-free products on hipBLASLt (UVA_BLAS_PLAIN bit 1 forward, bit 2 dX) vs gemm_8ph:
# bf16 parity with the route on, then same-box bench A/B (headline config only), interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ae
mkdir -p $O
UVA_BLAS_PLAIN=3 timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_workspace_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests $(tail -1 $O/t.log)"
timeout -k 10 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > $O/t8.log 2>&1 || { echo "FP8_TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t8.log | head -20; tail -3 $O/t8.log; exit 1; }
echo "fp8 tests $(tail -1 $O/t8.log)"
for i in 1 2; do
  for L in base new; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== quant $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep -E "fp8 quant|H=12 p=0.1" || exit 1
  done
done
for i in 1 2; do
  for V in 0 1 2 3; do
    UVA_BLAS_PLAIN=$V timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > $O/b.json 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b.json')); print('blas_plain=$V', d['value'], d['ms_per_step_median'])"
  done
done
