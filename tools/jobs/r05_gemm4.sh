# persistent 4-wave GEMM: GPU tests + kernel benchmark vs gemm_8ph / hipBLASLt (tools only;
# profiles/r05/gemm4_diag.txt).  Diagnostic builds: tools/build_variant.py g4dN gemm4.hip -DUVA_G4_DIAG=N,
# timed with tools/ab_run.py abx/libuva_g4dN.so tools/gemm4_bench.py quick
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4_gpu.py 2>&1 | tail -3 || exit 1
timeout -k 10 300 python -u tools/gemm4_bench.py 2 || exit 1
timeout -k 10 300 python -u tools/gemm4_bench.py dw || exit 1
