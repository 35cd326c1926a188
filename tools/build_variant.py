"""Build an A/B variant of libuva_hip.so into abx/libuva_<name>.so: <file>.hip recompiled with extra
defines, linked with the in-tree objects of every other source (run __graft_entry__.build() first).

    python tools/build_variant.py <name> <file.hip> [-DFOO=1 ...]

Time it on the GPU box with tools/ab_run.py (e.g. tools/ab_kb.sh, tools/ab_bench.sh)."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "unified_video_action_amd")
sys.path.insert(0, ROOT)


def main():
    from unified_video_action_amd import build_native as bn
    name, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    bn.build(verbose=False)
    src = src if os.path.isabs(src) else os.path.join(bn.CSRC, src)
    out_dir = os.path.join(ROOT, "abx")
    os.makedirs(out_dir, exist_ok=True)
    obj = os.path.join(out_dir, f"{name}_{os.path.basename(src).replace('.hip', '.o')}")
    r = subprocess.run([bn.HIPCC] + bn.FLAGS + bn.EXTRA.get(os.path.basename(src), []) + defs + ["-c", src, "-o", obj],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    base = os.path.basename(src).replace(".hip", ".o")
    objs = [o for o in sorted(glob.glob(os.path.join(bn.OBJ, "*.o"))) if os.path.basename(o) != base] + [obj]
    lib = os.path.join(out_dir, f"libuva_{name}.so")
    r = subprocess.run([bn.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs,
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    os.remove(obj)
    print(lib)


if __name__ == "__main__":
    main()
