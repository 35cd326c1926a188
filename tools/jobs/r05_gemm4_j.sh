set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/j
for sh in "768 3072" "3072 768"; do
  set -- $sh
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/j/kt_$1_$2 -o kt -- python tools/gemm4_one.py dw $1 $2 5 > /dev/null 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/j/pmc_$1_$2 -o pmc -- python tools/gemm4_one.py dw $1 $2 2 > /dev/null 2>&1 || exit 1
done
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/j/pmc_fwd -o pmc -- python tools/gemm4_one.py 768 3072 2 > /dev/null 2>&1 || exit 1
find gpurun_out/j -name "*.csv" | head -20
