# time the B=1 sampler (tools_infer_bench.py) on every abx/diag_*.so build (tools/conv_diag_build.py ps_* variants)
set -o pipefail
export TMPDIR=/tmp
for L in abx/diag_*.so; do
  echo "== $L"
  timeout -k 10 120 python tools/ab_run.py $L tools/tools_infer_bench.py --batches 1 --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
done
