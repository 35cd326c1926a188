set -o pipefail
export TMPDIR=/tmp
echo "== base"; timeout -k 10 120 python -u tools/conv4_quick.py 128 || exit 1
for d in 1 2 8 16 17 19; do
  echo "== d$d"; timeout -k 10 120 python -u tools/ab_run.py abx/libuva_c4d$d.so tools/conv4_quick.py 128 2>&1 | grep -v amdgpu.ids || exit 1
done
