"""Which k does byte j of lane l's 32-byte operand carry in v_mfma_scale_f32_32x32x64_f8f6f4?
A = one-hot probes: lane l's byte j = e4m3(1.0) for a single (l, j), B = an index-coded matrix; the
output row/col pattern names (row, k) of that byte.  Prints the inferred map for A and B."""
import ctypes
import os
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe_mx.so"))
ONE = 0x38  # e4m3 1.0


def run(a_bytes, b_bytes):
    a = torch.tensor(a_bytes, dtype=torch.uint8, device="cuda").contiguous()
    b = torch.tensor(b_bytes, dtype=torch.uint8, device="cuda").contiguous()
    c = torch.zeros(64 * 16, dtype=torch.float32, device="cuda")
    assert lib.probe_mx(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(c.data_ptr())) == 0
    return c.view(64, 16).cpu()


def cd_map(l, i):  # documented 32x32 C/D map: (row, col)
    return (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), l & 31


def main():
    # B operand: ALL ones -> D[row][col] = sum_k A[row][k]: a one-hot A byte lights row r in every col
    ones = [[ONE] * 32 for _ in range(64)]
    amap = {}
    for l in range(64):
        for j in (0, 1, 7, 8, 15, 16, 31):
            a = [[0] * 32 for _ in range(64)]
            a[l][j] = ONE
            d = run(a, ones)
            rows = {cd_map(L, i)[0] for L in range(64) for i in range(16) if d[L, i] != 0}
            amap[(l, j)] = sorted(rows)
    # k index: B one-hot at (lane l, byte j) with A = all ones on row 0 only... use A one-hot on a known
    # (row, k) pair: A byte (l0=0, j) and B byte (l, jb) -> nonzero iff they share k
    kmatch = {}
    for j in range(32):
        for jb in range(32):
            a = [[0] * 32 for _ in range(64)]
            a[0][j] = ONE
            a[32][j] = ONE
            b = [[0] * 32 for _ in range(64)]
            b[0][jb] = ONE
            b[32][jb] = ONE
            d = run(a, b)
            if d.abs().sum() > 0:
                kmatch.setdefault(j, []).append(jb)
    print("A (lane, byte) -> rows:", {k: v for k, v in list(amap.items())[:40]})
    print("A byte j (lanes 0/32) meets B byte jb (lanes 0/32):", kmatch)
    # per-lane k of byte j: A lane 0 byte j vs B lane 0 byte j only (h=0), and lane 32 only (h=1)
    for h in (0, 1):
        same = []
        for j in range(32):
            a = [[0] * 32 for _ in range(64)]
            a[32 * h][j] = ONE
            b = [[0] * 32 for _ in range(64)]
            b[32 * h][j] = ONE
            d = run(a, b)
            same.append(int(d.abs().sum().item() > 0))
        print(f"half {h}: A byte j and B byte j of the same lane half meet:", same)
    for h in (0, 1):
        cross = []
        for j in range(32):
            a = [[0] * 32 for _ in range(64)]
            a[32 * h][j] = ONE
            b = [[0] * 32 for _ in range(64)]
            b[32 * (1 - h)][j] = ONE
            d = run(a, b)
            cross.append(int(d.abs().sum().item() > 0))
        print(f"A half {h} byte j vs B other half byte j:", cross)


if __name__ == "__main__":
    main()
