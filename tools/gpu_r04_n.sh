# PMC breakdown of the level-0 GN conv (with and without the residual epilogue)
set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_kernel.sh conv0res conv3x3_halo tools/tools_conv0_one.py > gpurun_out/pmc_conv0res.txt 2>&1 || { echo FAIL res; tail -5 gpurun_out/pmc_conv0res.txt; exit 1; }
cat gpurun_out/pmc_conv0res.txt
bash tools/pmc_kernel.sh conv0nores conv3x3_halo tools/tools_conv0_one.py nores > gpurun_out/pmc_conv0nores.txt 2>&1 || { echo FAIL nores; tail -5 gpurun_out/pmc_conv0nores.txt; exit 1; }
cat gpurun_out/pmc_conv0nores.txt
