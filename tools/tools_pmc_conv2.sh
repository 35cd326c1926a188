#!/bin/bash
# LDS bank conflicts of the halo conv (level-0 shape, plain and bias+residual+GN-stats variants)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc2
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcc2 -o run -- python3 tools/tools_conv_phase.py > gpurun_out/pmcc2/log.txt 2>&1
echo rc=$?
