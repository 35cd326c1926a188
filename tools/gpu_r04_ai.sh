# DiffLoss trunk dX products in bf16 on hipBLASLt (UVA_BLAS_PLAIN bit 4): parity, then bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ai
mkdir -p $O
UVA_BLAS_PLAIN=7 timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests(blas=7) $(tail -1 $O/t.log)"
for i in 1 2; do
  for V in 3 7; do
    UVA_BLAS_PLAIN=$V timeout -k 10 300 python bench.py --other-configs "" --no-cpu-baseline --steps 30 --no-trace > $O/b.json 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b.json')); print('bench blas=$V', d['value'], d['ms_per_step_median'])"
  done
done
