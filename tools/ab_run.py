"""Same-box A/B of two library builds (tools only; the product path never reads an override):

    python tools/ab_run.py <path/to/libuva_other.so> <script.py> [args...]
    python tools/ab_run.py <path/to/libuva_other.so> -m pytest [args...]

binds <lib> through native.lib.use_library() and then runs <script.py> as __main__.  Entry points
that the other build predates stay unbound and are listed on stderr."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    # torch first: it brings its own HIP runtime (libamdhip64), which the library must bind to, as it
    # does on the product path (a library loaded before torch pulls in /opt/rocm's runtime: two
    # runtimes in one process, and the second reports hipErrorNoDevice)
    import torch  # noqa: F401
    from unified_video_action_amd.native.lib import use_library
    use_library(sys.argv[1])
    if sys.argv[2] == "-m":  # python tools/ab_run.py <lib> -m pytest ...
        mod = sys.argv[3]
        sys.argv = [mod] + sys.argv[4:]
        sys.path.insert(0, os.getcwd())
        runpy.run_module(mod, run_name="__main__", alter_sys=True)
    else:
        script = sys.argv[2]
        sys.argv = sys.argv[2:]
        sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
        runpy.run_path(script, run_name="__main__")
