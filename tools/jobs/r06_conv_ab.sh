#!/bin/bash
# GN conv staging math: packed f32 (default) vs scalar (abx/libuva_scgn.so) vs packed without SLP (noslpconv):
# conv0 timings interleaved twice, then the conv tests on the scalar build
set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r06
for i in 1 2; do
  for L in new abx/libuva_scgn.so abx/libuva_noslpconv.so; do
    if [ $L = new ]; then PY=python; else PY="python tools/ab_run.py $L"; fi
    echo "== $L"; timeout -k 10 120 $PY tools/tools_kbench.py conv0 2>&1 | grep gnconv || exit 1
  done
done
timeout -k 10 400 python tools/ab_run.py abx/libuva_scgn.so -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_halo_gpu.py 2>&1 | tail -2
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_parity_gpu.py -k "toolhang" 2>&1 | tail -3
