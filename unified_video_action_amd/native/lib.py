"""ctypes binding of libuva_hip.so.  Signatures are parsed from include/uva_hip.h so the
Python side can never drift from the C ABI.  There is NO fallback: if the library is
missing or a symbol is absent, import of the product path fails loudly."""
import ctypes
import os
import re
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ROOT = os.path.dirname(_PKG)
# the product library; nothing in the environment can replace it (A/B runs of another build go
# through tools/ab_run.py, which calls use_library() before the first load)
LIB_PATH = os.path.join(_PKG, "libuva_hip.so")
HEADER = os.path.join(_ROOT, "include", "uva_hip.h")

_CTYPE = {
    "int": ctypes.c_int, "long long": ctypes.c_longlong, "float": ctypes.c_float,
    "unsigned long long": ctypes.c_ulonglong, "hipStream_t": ctypes.c_void_p,
}


def parse_header(path=HEADER):
    """-> {name: (restype, [argtypes])} for every entry point declared in the header."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    out = {}
    for m in re.finditer(r"\b(int|long long)\s+(uva_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        types = []
        for a in [x.strip() for x in args.split(",") if x.strip()]:
            if "*" in a:
                types.append(ctypes.c_void_p)
                continue
            t = re.sub(r"\bconst\b", "", a).strip()
            t = " ".join(t.split()[:-1])  # drop the parameter name
            types.append(_CTYPE[t])
        out[name] = (_CTYPE[ret], types)
    return out


class UvaLib:
    def __init__(self, path=LIB_PATH, allow_missing=False):
        if not os.path.exists(path):
            raise RuntimeError(
                f"libuva_hip.so not found at {path}: run __graft_entry__.build() (hipcc gfx950). "
                "There is no CPU fallback on the product path.")
        self.path = path
        import torch  # noqa: F401  -- torch's HIP runtime first: the library binds to it, not a second copy
        self._lib = ctypes.CDLL(path)
        self.sigs = parse_header()
        self.unbound = []
        for name, (res, args) in self.sigs.items():
            if allow_missing and not hasattr(self._lib, name):
                self.unbound.append(name)  # an older A/B build: calling one of these raises
                continue
            fn = getattr(self._lib, name)  # AttributeError = missing export -> loud
            fn.restype = res
            fn.argtypes = args
            setattr(self, "_" + name, fn)
        if self.unbound:
            print(f"[uva] {path}: {len(self.unbound)} entry points of include/uva_hip.h not exported "
                  f"(older build): {', '.join(self.unbound)}", file=sys.stderr, flush=True)

    def call(self, name, *args):
        rc = getattr(self, "_" + name)(*args)
        if rc != 0:
            raise RuntimeError(f"{name} failed with hipError {rc}")
        return rc

    def query(self, name, *args):
        return getattr(self, "_" + name)(*args)


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = UvaLib()
    return _LIB


def use_library(path):
    """tools only (tools/ab_run.py): bind another build of the library for a same-box A/B run.
    Must run before the first lib() call; entry points the older build lacks stay unbound and are
    listed once on stderr."""
    global _LIB
    if _LIB is not None:
        raise RuntimeError(f"use_library({path}): {_LIB.path} is already loaded")
    _LIB = UvaLib(os.path.abspath(path), allow_missing=True)
    return _LIB
