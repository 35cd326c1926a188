# gemm_8ph raster group size 8 (in-tree) vs 4 / 16: Block products (kbench cold: hot and cold-cache per-call)
set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
  for L in new grp4 grp16; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py cold 2>&1 | grep -E "dx|dW|fwd" || exit 1
  done
done
