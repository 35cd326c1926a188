# MFMA-utilisation PMC pass over a short bench run (2 timed steps) -> gpurun_out/pmc_mfma/
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_mfma
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/pmc_mfma -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --other-configs "" --no-trace > gpurun_out/pmc_mfma/log.txt 2>&1
rc=$?
echo pmc_rc=$rc
[ $rc -eq 0 ] && python3 tools/pmc_mfma.py gpurun_out/pmc_mfma/run_counter_collection.csv gpurun_out/pmc_mfma/mfma.json
