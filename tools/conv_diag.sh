# time the GN conv (kbench conv0) on every abx/diag_*.so build (tools/conv_diag_build.py), same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in abx/diag_*.so; do
  echo "== $L"
  timeout -k 10 120 python tools/ab_run.py $L tools/tools_kbench.py conv0 2>&1 | grep -v amdgpu.ids || exit 1
done
