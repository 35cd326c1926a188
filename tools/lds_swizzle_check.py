"""LDS bank-conflict model of the attention tile images (tools only): extra LDS-array cycles of the
fragment reads of csrc/attention.hip (lds_row_frag: ds_read_b128; lds_tr_frag: ds_read_b64_tr_b16)
under gfx950's lane groups (MI355X_MICROARCH.md 'LDS banking': b128 in 4 x 16 lanes
{0-3,12-15,20-27}, {4-11,16-19,28-31}, +32; b64 / tr in 2 x 32; bank = dword mod 64), for the former
72- and 80-element padded rows and for 128-B rows with the 16-B chunk XOR-ed by (row & 6).

    python tools/lds_swizzle_check.py  ->  layout: (LDS cycles, extra conflict cycles) per tile sweep"""
import collections

B128 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
B128 += [[lane + 32 for lane in g] for g in B128]
B64 = [list(range(32)), list(range(32, 64))]


def cost(groups, addrs):
    tot = extra = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for lane in g:
            for a in addrs[lane]:
                banks[(a // 4) % 64].add(a // 4)
        m = max(len(s) for s in banks.values())
        tot += m
        extra += m - 1
    return tot, extra


def sweep(addr_of):
    """every lds_row_frag (row0 = 0/16/32/48, ks = 0/1) and lds_tr_frag (rowA = 32 ks, col0 = 16 dt)"""
    T = E = 0
    for row0 in range(0, 64, 16):
        for ks in range(2):
            a = {l: [addr_of(row0 + (l & 15), ks * 32 + 8 * (l >> 4)) + 4 * i for i in range(4)] for l in range(64)}
            t, e = cost(B128, a)
            T, E = T + t, E + e
    for ks in range(2):
        for dt in range(4):
            for r0 in (32 * ks, 32 * ks + 16):
                a = {l: [addr_of(r0 + 4 * (l >> 4) + ((l >> 2) & 3), dt * 16 + 4 * (l & 3)) + 4 * i for i in range(2)]
                     for l in range(64)}
                t, e = cost(B64, a)
                T, E = T + t, E + e
    return T, E


def main():
    padded = lambda r, c: (r * 72 + c) * 2  # noqa: E731
    padded80 = lambda r, c: (r * 80 + c) * 2  # noqa: E731
    swz = lambda r, c: r * 128 + ((((c >> 3) ^ (r & 6)) & 7) << 4) + (c & 7) * 2  # noqa: E731
    print("padded rows (AT_LD 72):", sweep(padded))
    print("padded rows (AT_LD 80):", sweep(padded80))
    print("XOR (row & 6) rows    :", sweep(swz))


if __name__ == "__main__":
    main()
