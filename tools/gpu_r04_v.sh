set -o pipefail
export TMPDIR=/tmp
echo "== cold"; timeout -k 10 300 python tools/tools_kbench.py cold 2>&1 | grep -E "dx|dW|fwd" || exit 1
