set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attention_fp8_gpu.py tests/test_action_head_gpu.py tests/test_attention_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?
echo "focus rc=$rc"
grep -E "PASSED|FAILED|^E   " gpurun_out/t3.log | head -60 || true
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/tools_kbench.py attn > gpurun_out/kb_attn.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/kb_attn.log
exit $rc
