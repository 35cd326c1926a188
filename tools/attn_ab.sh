# attention dev loop: correctness tests of the in-tree build, then the attention micro-bench on the
# in-tree build and on abx/libuva_base.so (same box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py ${EXTRA_TESTS} -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_t.log 2>&1
rc=$?
tail -15 gpurun_out/attn_t.log
[ $rc -eq 0 ] || exit 1
for L in new base; do
  if [ $L = base ]; then PY="python tools/ab_run.py abx/libuva_base.so"; else PY=python; fi
  echo "== $L"
  timeout -k 10 120 $PY tools/tools_kbench.py attn 2>&1 | grep -v amdgpu.ids || exit 1
done
