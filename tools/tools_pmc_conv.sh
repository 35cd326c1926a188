export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcc -o run -- python3 tools/tools_conv_phase.py > gpurun_out/pmcc/log.txt 2>&1
echo rc=$?
