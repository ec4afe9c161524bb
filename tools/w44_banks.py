#!/usr/bin/env python3
"""Exhaustive LDS bank check of the F(4,3) x F(4,3) tile's maps (csrc/conv3d_wino44.hip):
the V-pass's ds_read_b64 of the halo (two 32-lane groups, 64 banks), its ds_write_b128 of V
(8 groups of 8 lanes, 32 banks), and the steps' ds_read_b128 of V (4 lane groups of 16 lanes
per MI355X_MICROARCH.md's LDS table, 64 banks) -- every kh, x-half, read offset and plane.
Prints the extra cycles per instruction (0 = conflict-free)."""
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
        for m in range(5):  # the V-pass's writes (4 x b128 + 1 x b64)
            addr = {}
            for t in lanes:
                g, c, r, xh = vpass_unit(t)
                addr[t % 64] = c * TCS + r * TRS + g * GS + xh * XHS + 4 * m
            e = conflicts([[addr[l] for l in range(8 * k, 8 * k + 8)] for k in range(8)], 4, 32)
            worst = max(worst, e)
    print("V-pass halo reads + V writes: extra cycles", worst)
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


if __name__ == "__main__":
    main()
