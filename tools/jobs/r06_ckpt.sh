#!/bin/bash
# checkpoint: gemm_8w tests, same-box bench A/B (this tree vs abx/libuva_prev.so), full GPU suite, smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06ckpt}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8w_gpu.py > $O/t_g8w.log 2>&1; rc=$?
tail -2 $O/t_g8w.log; [ $rc -eq 0 ] || { grep -E "^E |Error" $O/t_g8w.log | head -20; exit 1; }
bash tools/ab_bench.sh 2>&1 | tee $O/ab.txt || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
grep -E "^FAILED|passed|failed" $O/t.log | tail -30
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
