"""bench.py with one runtime flag overridden (same-box A/B of a fused route):
python tools/bench_flag.py act_bwd_in_gemm=0 [bench.py args...]"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unified_video_action_amd.runtime import RT  # noqa: E402

name, val = sys.argv[1].split("=")
assert hasattr(RT, name), name
setattr(RT, name, bool(int(val)))
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
