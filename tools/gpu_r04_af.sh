# hipcc SLP vectorisation off (no v_pk_*_f32 beside the MFMAs) for every source / attention only:
# attention, GEMM and GN-conv tests on the no-SLP build, kernel timings and the bench, interleaved
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 500 python tools/ab_run.py abx/libuva_noslp.so -m pytest tests/test_attention_gpu.py tests/test_conv_halo_gpu.py tests/test_gemm8_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests(noslp) $(tail -1 $O/t.log)"
for i in 1 2; do
  for L in new noslp noslpatt; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== attn $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep -E "H=12 p=0.1|fp8 quant" || exit 1
  done
done
for i in 1 2; do
  for L in new noslp; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== conv0 $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | tail -4 || exit 1
  done
done
for i in 1 2; do
  for L in new noslp noslpatt; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    timeout -k 10 300 $PY bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > $O/b.json 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b.json')); print('bench $L', d['value'], d['ms_per_step_median'])"
  done
done
