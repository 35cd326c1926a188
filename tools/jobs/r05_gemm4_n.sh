set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/n
timeout -s KILL 60 rocprofv3 -L > gpurun_out/n/avail.txt 2>&1 || true
for c in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum"; do
  n=$(echo $c | cut -c1-12)
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/n/dw_$n -o pmc -- python tools/gemm4_one.py dw 768 3072 2 > gpurun_out/n/dw_$n.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/n/fwd_$n -o pmc -- python tools/gemm4_one.py 768 3072 2 > gpurun_out/n/fwd_$n.log 2>&1 || exit 1
done
