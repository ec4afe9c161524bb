#!/usr/bin/env python3
"""Exhaustive LDS bank check of the F(4,3) x F(4,3) tile's maps (csrc/conv3d_wino44.hip), per
MI355X_MICROARCH.md's LDS table: the V-pass's halo reads as ds_read_b64 (two 32-lane groups,
64 banks) and as the ds_read2_b64 the compiler pairs them into (16-lane groups, 32 banks) --
and, for the record, as the ds_read2_b32 they compiled to while loaded through HIP's float2
struct (32-lane groups, 32 banks: the round-6 PMC's 30 M conflict cycles per launch) -- its
ds_write_b128 / ds_write_b64 of V, and the steps' ds_read_b128 / ds_read_b64 of V, every kh,
x-half, read offset and plane.  Prints the extra cycles per instruction (0 = conflict-free)."""
CB = [1, 1027, 2081, 3107]
RWA, PLANEA = 40, 160
GS, XHS, TRS, TCS = 40, 20, 320, 1284
B128_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]


def conflicts(addrs_by_group, width, banks):
    """extra LDS cycles: per group, the max number of distinct dword addresses on one bank - 1"""
    extra = 0
    for addrs in addrs_by_group:
        per_bank = {}
        for a in set(addrs):
            for k in range(width):
                per_bank.setdefault((a + k) % banks, set()).add(a + k)
        extra += max(len(v) for v in per_bank.values()) - 1
    return extra


def vpass_unit(t):
    g = (t & 3) | (((t >> 3) & 1) << 2)
    c = ((t >> 2) & 1) | (((t >> 4) & 1) << 1)
    return g, c, (t >> 5) & 3, t >> 7


def main():
    worst = 0
    for wave in range(4):
        lanes = range(64 * wave, 64 * wave + 64)
        for pl in range(6):
            for j in range(3):  # the three b64 reads per plane
                addr = {}
                for t in lanes:
                    g, c, r, _ = vpass_unit(t)
                    addr[t % 64] = CB[c] + pl * PLANEA + r * RWA + 3 + 4 * g + 2 * j
                assert all(a % 2 == 0 for a in addr.values()), "b64 alignment"
                e = conflicts([[addr[l] for l in range(0, 32)], [addr[l] for l in range(32, 64)]], 2, 64)
                worst = max(worst, e)
        for m in range(5):  # the V-pass's b128 writes (the fifth: floats 16, 17 + slot padding)
            addr = {}
            for t in lanes:
                g, c, r, xh = vpass_unit(t)
                addr[t % 64] = c * TCS + r * TRS + g * GS + xh * XHS + 4 * m
            e = conflicts([[addr[l] for l in range(8 * k, 8 * k + 8)] for k in range(8)], 4, 32)
            worst = max(worst, e)
    print("V-pass halo reads (ds_read_b64) + V b128 writes: extra cycles", worst)
    w2, w32, wb64 = 0, 0, 0
    for wave in range(4):
        lanes = range(64 * wave, 64 * wave + 64)
        for pl in range(6):
            for j in range(3):
                addr = {}
                for t in lanes:
                    g, c, r, _ = vpass_unit(t)
                    addr[t % 64] = CB[c] + pl * PLANEA + r * RWA + 3 + 4 * g + 2 * j
                w2 = max(w2, conflicts([[addr[l] for l in range(16 * k, 16 * k + 16)] for k in range(4)], 2, 32))
                for k in range(2):  # each dword alone, as ds_read_b32 / one half of ds_read2_b32
                    w32 = max(w32, conflicts([[addr[l] + k for l in range(0, 32)], [addr[l] + k for l in range(32, 64)]], 1, 32))
        addr = {}
        for t in lanes:
            g, c, r, xh = vpass_unit(t)
            addr[t % 64] = c * TCS + r * TRS + g * GS + xh * XHS + 16
        wb64 = max(wb64, conflicts([[addr[l] for l in range(16 * k, 16 * k + 16)] for k in range(4)], 2, 32))
    print("V-pass halo reads as ds_read2_b64: extra cycles", w2)
    print("V-pass halo reads as ds_read_b32 / ds_read2_b32 (the pre-fix code): extra cycles per access", w32)
    print("V-pass V b64 write (the pre-fix tail store): extra cycles", wb64)
    worst = 0
    for xh in range(2):
        for kh in range(3):
            for m in range(5):
                addr = {}
                for l in range(64):
                    ci, p = l >> 4, l & 15
                    addr[l] = ci * TCS + (p // 8 + kh) * TRS + GS * (p % 8) + XHS * xh + 4 * m
                    assert addr[l] % 4 == 0
                worst = max(worst, conflicts([[addr[l] for l in g] for g in B128_GROUPS], 4, 64))
    print("step V reads (ds_read_b128): extra cycles", worst)
    worst = 0
    for xh in range(2):
        for kh in range(3):
            addr = {l: (l >> 4) * TCS + ((l & 15) // 8 + kh) * TRS + GS * ((l & 15) % 8) + XHS * xh + 16 for l in range(64)}
            worst = max(worst, conflicts([[addr[l] for l in range(0, 32)], [addr[l] for l in range(32, 64)]], 2, 64))
    print("step V tail read as ds_read_b64 (pre-fix): extra cycles", worst)
    worst = 0
    for xh in range(2):
        for kh in range(2):  # two kh rows paired into one ds_read2_b64 (16-lane groups, 32 banks)
            addr = {l: (l >> 4) * TCS + ((l & 15) // 8 + kh) * TRS + GS * ((l & 15) % 8) + XHS * xh + 16 for l in range(64)}
            worst = max(worst, 2 * conflicts([[addr[l] for l in range(16 * k, 16 * k + 16)] for k in range(4)], 2, 32))
    print("step V tail reads as ds_read2_b64 (pre-fix, both accesses): extra cycles", worst)


if __name__ == "__main__":
    main()
