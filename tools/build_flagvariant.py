"""Build an A/B variant of libuva_hip.so with extra hipcc flags on every source (or on the listed
ones): abx/libuva_<name>.so.

    python tools/build_flagvariant.py <name> "<flags>" [file.hip ...]

Time it on the GPU box with tools/ab_run.py."""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from unified_video_action_amd import build_native as bn
    name, flags, files = sys.argv[1], sys.argv[2].split(), sys.argv[3:]
    bn.build(verbose=False)
    odir = os.path.join(ROOT, "abx", f"obj_{name}")
    os.makedirs(odir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(bn.CSRC, "*.hip")))

    def one(src):
        base = os.path.basename(src).replace(".hip", ".o")
        if files and os.path.basename(src) not in files:
            return os.path.join(bn.OBJ, base)
        obj = os.path.join(odir, base)
        r = subprocess.run([bn.HIPCC] + bn.FLAGS + flags + ["-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        return obj

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, srcs))
    lib = os.path.join(ROOT, "abx", f"libuva_{name}.so")
    r = subprocess.run([bn.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs,
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    for o in glob.glob(os.path.join(odir, "*.o")):
        os.remove(o)
    os.rmdir(odir)
    print(lib)


if __name__ == "__main__":
    main()
