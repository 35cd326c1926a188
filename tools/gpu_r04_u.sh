# lockstep diagnostic: odd workgroups start late (attention backward, persistent GN conv)
set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
  for L in new ds20 ds60; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py attn 2>&1 | grep "H=12 p=" || exit 1
  done
  for L in new cds60; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py abx/libuva_$L.so"; fi
    echo "== $L"; timeout -k 10 200 $PY tools/tools_kbench.py conv0 2>&1 | grep nores || exit 1
  done
done
