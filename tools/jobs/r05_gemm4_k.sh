set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/k/hit_dw -o pmc -- python tools/gemm4_one.py dw 768 3072 2 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/k/fetch_dw -o pmc -- python tools/gemm4_one.py dw 768 3072 2 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/k/hit_fwd -o pmc -- python tools/gemm4_one.py 768 3072 2 > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/k/fetch_fwd -o pmc -- python tools/gemm4_one.py 768 3072 2 > /dev/null 2>&1 || exit 1
