"""Per-barrier instruction sequence of a kernel in a hipcc -S output: M = MFMA, D = LDS-DMA / buffer load,
r = ds_read, S = global store, w = s_waitcnt, v = other VALU (tools only).
python tools/isa_seq.py file.s <kernel-substring> [first-barrier-index count]"""
import sys

s = open(sys.argv[1]).read().split("\n")
st = [i for i, l in enumerate(s) if l.startswith("_Z") and sys.argv[2] in l.split(":")[0]][0]
end = next(i for i in range(st, len(s)) if "s_endpgm" in s[i])
body = [l for l in s[st:end] if not l.strip().startswith(";")]
idx = [i for i, l in enumerate(body) if "s_barrier" in l] + [len(body)]
k0 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
n = int(sys.argv[4]) if len(sys.argv) > 4 else len(idx) - 1
for k in range(k0, min(k0 + n, len(idx) - 1)):
    seq = []
    for l in body[idx[k]:idx[k + 1]]:
        t = l.strip().split()
        if not t:
            continue
        op = t[0]
        seq.append("M" if op.startswith("v_mfma") else "D" if op.startswith("buffer_load") else
                   "r" if op.startswith("ds_read") else "S" if "store" in op else "w" if op == "s_waitcnt" else
                   "v" if op.startswith("v_") else "")
    print(k, "".join(seq))
