# PMC passes (one rocprofv3 run per pass) over a one-shot script; summary filtered by kernel name.
# Usage: bash tools/pmc_kernel.sh <out-name> <kernel-substring> <script.py> [script args]
set -o pipefail
export TMPDIR=/tmp
NAME=$1; KF=$2; shift 2
D=gpurun_out/pmc_$NAME
mkdir -p $D
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $D/p$i -o run -- python3 "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $D/p$i.log; exit 1; }
done
python3 tools/pmc_sum.py $D "$KF"
