#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcci
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU --output-format csv -d gpurun_out/pmcci/a -o run -- python3 tools/tools_convin_pmc.py > gpurun_out/pmcci/a.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR --output-format csv -d gpurun_out/pmcci/b -o run -- python3 tools/tools_convin_pmc.py > gpurun_out/pmcci/b.log 2>&1 || exit 1
echo done
