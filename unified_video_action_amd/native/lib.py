"""ctypes binding of libuva_hip.so.  Signatures are parsed from include/uva_hip.h so the
Python side can never drift from the C ABI.  There is NO fallback: if the library is
missing or a symbol is absent, import of the product path fails loudly."""
import ctypes
import os
import re

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ROOT = os.path.dirname(_PKG)
# UVA_LIB_PATH: an alternative build of this library (same-box A/B of two builds, tools_ab.sh)
LIB_PATH = os.environ.get("UVA_LIB_PATH") or os.path.join(_PKG, "libuva_hip.so")
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
    def __init__(self, path=LIB_PATH):
        if not os.path.exists(path):
            raise RuntimeError(
                f"libuva_hip.so not found at {path}: run __graft_entry__.build() (hipcc gfx950). "
                "There is no CPU fallback on the product path.")
        self._lib = ctypes.CDLL(path)
        self.sigs = parse_header()
        ab = bool(os.environ.get("UVA_LIB_PATH"))
        for name, (res, args) in self.sigs.items():
            if ab and not hasattr(self._lib, name):
                continue  # an older A/B build: entry points it predates stay unbound (calling one raises)
            fn = getattr(self._lib, name)  # AttributeError = missing export -> loud
            fn.restype = res
            fn.argtypes = args
            setattr(self, "_" + name, fn)

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
