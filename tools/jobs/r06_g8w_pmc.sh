#!/bin/bash
# PMC passes over the fused gemm_8w epilogue kernels (one counter group per run, no tracing domains)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r06/g8w_pmc
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 tools/g8w_pmc_one.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p2 -o run -- python3 tools/g8w_pmc_one.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 tools/g8w_pmc_one.py > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/g8w_pmc_one.py > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
O = "gpurun_out/r06/g8w_pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/p*/**/run_counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"][:70], r.get("Dispatch_Id", ""), r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        agg[k][c].append(v)
dur = collections.defaultdict(list)
for f in glob.glob(O + "/kt/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in agg.items():
    if "gemm" not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(k, "| us %.1f" % (sum(dur[k][1:]) / max(1, len(dur[k]) - 1) if dur[k] else -1),
          "| wait_any %.2f wait_inst %.2f active %.2f valu %.2f lds %.2f | mfma_busy/gui %.2f | write MB %.0f fetch MB %.0f" % (
              m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
              m.get("SQ_ACTIVE_INST_VALU", 0) / wc, m.get("SQ_ACTIVE_INST_LDS", 0) / wc,
              m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, m.get("GRBM_GUI_ACTIVE", 1)) / 32,
              m.get("WRITE_SIZE", 0) * 1024 / 1e6, 2 * m.get("FETCH_SIZE", 0) * 1024 / 1e6))
PY
