# dX through transposed bf16 weights (RT.dx_wt_layout): tests + bench A/B (UVA_DX_WT=0 / 1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_torch_ops_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo "TESTS_FAIL"; grep -E "^E  |FAILED|Error" $O/t.log | head -20; tail -3 $O/t.log; exit 1; }
echo "tests $(tail -1 $O/t.log)"
for i in 1 2; do
  for V in 0 1; do
    UVA_DX_WT=$V timeout -k 10 400 python -u bench.py --steps 30 --other-configs "" --no-cpu-baseline --h2d-steps 0 > $O/b_${V}_$i.json 2> $O/b_${V}_$i.err || { echo BENCH_FAIL; tail -5 $O/b_${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${V}_$i.json')); print('dx_wt=$V', d['value'], d['ms_per_step'])"
  done
done
