set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_prefetch.py tests/test_workspace_gpu.py tests/test_augment.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_focus2.log 2>&1 || { echo FOCUS_FAIL; tail -40 gpurun_out/pytest_focus2.log; exit 1; }
tail -2 gpurun_out/pytest_focus2.log
ENVVAR=UVA_MLP_SPLIT_EPI VALS="1 0 1 0" bash tools/ab_env.sh
