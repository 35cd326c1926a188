# one call for three A/Bs (GPU slots are scarce): (1) hipcc SLP vectorisation off (no v_pk_*_f32
# beside the MFMAs, abx/libuva_noslp.so), (2) the Block's epilogue-free products on hipBLASLt
# (UVA_BLAS_PLAIN=3), (3) the fp8 quantisation pass in its row form (abx/libuva_rows.so = row form)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 400 python tools/ab_run.py abx/libuva_noslp.so -m pytest tests/test_attention_gpu.py tests/test_conv_halo_gpu.py tests/test_gemm8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests(noslp) $(tail -1 $O/t.log)"
UVA_BLAS_PLAIN=3 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 250 --timeout-method thread > $O/tb.log 2>&1 || { echo "BLAS_TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/tb.log | head -20; tail -3 $O/tb.log; exit 1; }
echo "tests(blas) $(tail -1 $O/tb.log)"
timeout -k 10 200 python tools/ab_run.py abx/libuva_rows.so -m pytest tests/test_attention_fp8_gpu.py -x -q --timeout 150 --timeout-method thread > $O/t8.log 2>&1 || { echo "FP8_TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t8.log | head -20; tail -3 $O/t8.log; exit 1; }
echo "tests(fp8 rows) $(tail -1 $O/t8.log)"
for L in new noslp rows; do
  if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
  echo "== attn $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep -E "H=12 p=0.1|fp8 quant" || exit 1
done
for i in 1 2; do
  for L in new noslp; do
    for V in 0 3; do
      if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
      UVA_BLAS_PLAIN=$V timeout -k 10 300 $PY bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > $O/b.json 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/b.json')); print('bench $L blas=$V', d['value'], d['ms_per_step_median'])"
    done
  done
done
