set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > gpurun_out/attn_t.log 2>&1 || { echo ATTN_TEST_FAIL; tail -30 gpurun_out/attn_t.log; exit 1; }
tail -1 gpurun_out/attn_t.log
for L in ab/libuva_base.so unified_video_action_amd/libuva_hip.so; do echo "== $L"; UVA_LIB_PATH=$PWD/$L timeout -k 10 200 python -u tools/tools_kbench.py attn 2>&1 | grep "attn B" || exit 1; done
for L in unified_video_action_amd/libuva_hip.so ab/diag_gnscalar.so unified_video_action_amd/libuva_hip.so ab/diag_gnscalar.so; do echo "== $L"; UVA_LIB_PATH=$PWD/$L timeout -k 10 200 python -u tools/tools_kbench.py conv 2>&1 | grep "conv3x3 n256 256" || exit 1; done
