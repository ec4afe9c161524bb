#!/usr/bin/env python3
"""Exhaustive LDS bank check of the weight-gradient kernel's A / B reads
(csrc/conv3d_grad.hip wgrad_kernel): each is a ds_read_b32, banked in two groups of 32 lanes
on 32 banks (MI355X_MICROARCH.md, LDS).  Prints the worst extra cycles per read for the
strides in use and for the 64-bank strides of rounds 3-5 (0 = conflict-free)."""


def conflicts(groups, banks=32):
    extra = 0
    for addrs in groups:
        per = {}
        for a in set(addrs):
            per.setdefault(a % banks, set()).add(a)
        extra += max(len(v) for v in per.values()) - 1
    return extra


def b_reads(xrs, cis, ks=3, kd=3, ci=4, seg=64, nwave=4):
    tpt, taps = 16 // ci, kd * ks * ks
    worst = 0
    for nt in range((taps + tpt - 1) // tpt):
        offs = []
        for j in range(16):
            tap, c = nt * tpt + j // ci, j % ci
            offs.append(None if tap >= taps else
                        c * cis + ((tap // (ks * ks)) * ks + (tap // ks) % ks) * xrs + tap % ks)
        for wave in range(nwave):
            for q in range(seg // (4 * nwave)):
                lanes = [None if offs[l & 15] is None else offs[l & 15] + 4 * (wave + nwave * q) + (l >> 4)
                         for l in range(64)]
                worst = max(worst, conflicts([[a for a in lanes[:32] if a is not None],
                                              [a for a in lanes[32:] if a is not None]]))
    return worst


def a_reads(grs, seg=64, nwave=4):
    worst = 0
    for wave in range(nwave):
        for q in range(seg // (4 * nwave)):
            lanes = [(l & 15) * grs + 4 * (wave + nwave * q) + (l >> 4) for l in range(64)]
            worst = max(worst, conflicts([lanes[:32], lanes[32:]]))
    return worst


def main():
    print("B reads k=3 (row 70, channel 632):", b_reads(70, 632), " r03-r05 (630):", b_reads(70, 630))
    print("B reads 2D 3x3 (70, 216):", b_reads(70, 216, kd=1), " r03-r05 (210):", b_reads(70, 210, kd=1))
    print("B reads k=1 (channel 66):", b_reads(64, 66, ks=1, kd=1, ci=16), " r03-r05 (68):",
          b_reads(64, 68, ks=1, kd=1, ci=16))
    print("A reads (dz rows 66):", a_reads(66), " r03-r05 (68):", a_reads(68))


if __name__ == "__main__":
    main()
