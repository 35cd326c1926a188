#!/bin/bash
# PMC breakdown of the level-0 / level-1 GN convs (tools/tools_kbench.py conv0): wait / issue buckets, LDS
# conflicts, instruction mix, HBM bytes -- one counter group per run, no tracing domains with --pmc
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06/conv_pmc
mkdir -p $O
rocprofv3 -L > $O/counters.txt 2>&1 || true
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/p$N -o run -- python3 tools/tools_kbench.py conv0 > $O/p$N.log 2>&1 || { echo "pass $N failed"; tail -5 $O/p$N.log; exit 1; }; N=$((N+1)); }
N=1
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES
run SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_MFMA_BF16
run FETCH_SIZE
run WRITE_SIZE
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/tools_kbench.py conv0 > $O/kt.log 2>&1 || exit 1
grep -v amdgpu.ids $O/kt.log
python3 tools/pmc_kernels.py conv3x3 $O/p* $O/kt > $O/summary.txt
cat $O/summary.txt
