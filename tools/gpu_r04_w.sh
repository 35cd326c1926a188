set -o pipefail
export TMPDIR=/tmp
for i in 1 2 3; do
  for L in new noprio; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv || exit 1
  done
done
