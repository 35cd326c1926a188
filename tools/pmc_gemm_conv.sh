#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, no tracing domains) over the 8192^3 NN GEMM on the
# hand-written 8-phase kernel and the level-0 VAE halo conv: MFMA busy, LDS conflicts, waits.
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_gc}
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/g$i -o run -- python3 tools/tools_gemm_one.py 8192 8192 8192 0 0 3 > $O/g$i.log 2>&1 || { echo "gemm pass $i failed"; tail -3 $O/g$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $O/c$i -o run -- python3 tools/tools_conv_phase.py > $O/c$i.log 2>&1 || { echo "conv pass $i failed"; tail -3 $O/c$i.log; exit 1; }
done
echo done
