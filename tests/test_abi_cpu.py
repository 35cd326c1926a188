"""CPU-side checks of the C-ABI boundary: the library loads and exports every symbol
declared in include/uva_hip.h (no compute: no GPU here)."""
import ctypes
import os

from unified_video_action_amd.native.lib import HEADER, LIB_PATH, parse_header


def test_header_parses_and_library_exports_every_symbol():
    sigs = parse_header(HEADER)
    assert len(sigs) >= 19
    lib = ctypes.CDLL(LIB_PATH)
    missing = [n for n in sigs if not hasattr(lib, n)]
    assert not missing, missing


def test_workspace_queries_are_pure_host():
    from unified_video_action_amd.native.lib import lib
    L = lib()
    assert L.query("uva_layernorm_bwd_workspace", 1000, 768) == 16 * 768 * 2
    assert L.query("uva_colsum_workspace", 1024, 10) == 8 * 10  # one partial row per 128-row slab
