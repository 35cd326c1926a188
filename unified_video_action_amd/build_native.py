"""Build libuva_hip.so (gfx950) in-tree from csrc/*.hip with hipcc, and the oracle's
optional C pieces.  Used by __graft_entry__.build(); safe to call repeatedly
(recompiles only sources newer than their object)."""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build_obj")
LIB = os.path.join(HERE, "libuva_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
         "-Wno-unused-result", "-I" + CSRC]
# per-source extras.  gemm8w.hip: no SLP vectorisation -- its fused epilogues (GELU' / GELU / dropout math
# beside the MFMA stream) came out of the SLP pass as packed v_pk_*_f32 with op_sel operand swaps, and the
# GELU-backward form then returned intermittently wrong low halves (one element of a 16-lane row per tile in
# ~half the launches, tools/dbg_dgelu.py; never with the pass off: 16 / 16 launches bit-exact).  The scalar
# form is also the cheaper one beside MFMAs (MI355X_MICROARCH.md: packed f32 VALU is an anti-lever there)
EXTRA = {"gemm8w.hip": ["-fno-slp-vectorize"]}


def _compile(src):
    obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [HIPCC] + FLAGS + EXTRA.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
