"""Instruction histogram / spill report per kernel of a hipcc -S output (tools only)."""
import re
import sys
from collections import Counter

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
s = open(path).read().split("\n")
starts = [i for i, l in enumerate(s) if re.match(r"^_Z\S+:", l) and pat in l]
for st in starts:
    end = next(i for i in range(st, len(s)) if "s_endpgm" in s[i])
    ins = [l.strip() for l in s[st:end] if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    c = Counter(l.split()[0] for l in ins)
    print(s[st].split(":")[0][:70], len(ins))
    keys = ["v_mfma_f32_16x16x32_bf16", "v_accvgpr_read_b32", "v_accvgpr_write_b32", "v_accvgpr_mov_b32",
            "ds_read_b128", "buffer_load_dwordx4", "scratch_load_dword", "scratch_store_dword",
            "scratch_load_dwordx4", "scratch_store_dwordx4", "s_barrier", "s_waitcnt", "s_nop", "global_store_dwordx4"]
    print("  " + ", ".join(f"{k.replace('v_mfma_f32_16x16x32_bf16','mfma')}={c[k]}" for k in keys if c[k]))
