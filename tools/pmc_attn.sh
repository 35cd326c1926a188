# PMC passes over tools_attn_one.py (attention fwd+bwd, B32 N1024 H12 p0.1) for the in-tree build
# and abx/libuva_base.so.  Usage: bash tools/pmc_attn.sh [list]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_attn
if [ "$1" = list ]; then
  timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_attn/list.txt 2>&1
  grep -oE "\bSQ_[A-Z0-9_]+" gpurun_out/pmc_attn/list.txt | sort -u > gpurun_out/pmc_attn/sq.txt
  exit 0
fi
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
for L in new base; do
  if [ $L = base ]; then AB="tools/ab_run.py abx/libuva_base.so"; else AB=""; fi
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_attn/${L}_$i -o run -- python3 $AB tools/tools_attn_one.py > gpurun_out/pmc_attn/${L}_$i.log 2>&1 || { echo "pass $L $i failed"; tail -5 gpurun_out/pmc_attn/${L}_$i.log; exit 1; }
  done
done
python3 tools/pmc_attn_sum.py gpurun_out/pmc_attn
