# time the B=1 sampler (tools_infer_bench.py) on every ab/diag_*.so build (tools/conv_diag_build.py ps_* variants)
set -o pipefail
export TMPDIR=/tmp
for L in ab/diag_*.so; do
  echo "== $L"
  UVA_LIB_PATH=$PWD/$L timeout -k 10 120 python tools/tools_infer_bench.py --batches 1 --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
done
