#!/usr/bin/env python3
"""LDS bank-conflict model of frame_kernel's loop-filter tile accesses (diagnostics).

The loop filter gathers / scatters one byte per lane per instruction (ds_read_u8 / ds_write_b8):
the vertical-edge pass with one lane per pixel ROW (16 luma, 8 U, 8 V rows of the MB), the
horizontal-edge pass with one lane per pixel COLUMN (immediate row offsets, so luma and chroma share
the tile pitch).  A 32-lane group of a wave64 LDS instruction costs one LDS cycle per distinct dword
on its busiest bank (MI355X_MICROARCH.md, LDS: bank = dword mod 32 for 4-byte-and-smaller accesses;
lanes reading the same dword broadcast).  This prints the cost of the 20 gather instructions of each
pass for every ring slot, for the shipped layout (vp8g_device.h: kTP, kLfUV, kCV; two-column
ring) and for the three-column ring of the loop-filter-behind experiment, and, with --search, the
best layouts within the LDS budget of two 4K frames per CU.

Measured (tools/ab_inproc.py, 512 x 4K, one box; profiles/r03_ab_lf_behind.json): round-2 layout
(pitch 40, chroma at 800: vertical pass 3-way) 14.40 ms, chroma at 804 (2-way) 14.26 ms; the
three-column ring at pitch 52 15.58 ms, at pitch 56 / chroma + 4 14.47 ms.  The model ranks bank
conflicts only: pitches that are not a multiple of 8 also split the 8-B luma row accesses (pitch 52
lost 2-3 % whatever its bank score).

  python tools/lds_banks.py [--search]
"""
import argparse

NBANK = 32


def cost(addrs):
    banks = {}
    for a in addrs:
        d = a // 4
        banks.setdefault(d % NBANK, set()).add(d)
    return max(len(s) for s in banks.values())


def passes(P, UV, CV, ring, slot):
    """Per-instruction cycles of the vertical and horizontal gathers (20 each) of one 32-lane half."""
    nslot = (slot - 1) % ring
    v, h = [], []
    for i in range(20):
        av, ah = [], []
        for ln in range(32):
            isy = ln < 16
            cp = (ln >> 3) & 1
            rowp = (4 + ln) * P if isy else UV + (4 + (ln & 7)) * P + cp * CV
            lp = rowp + (nslot * 16 + 12 if isy else nslot * 8 + 4)  # the left neighbour's last 4 px
            mp = rowp + (slot * 16 if isy else slot * 8)
            av.append(lp + i if i < 4 else mp + i - 4)
            colp = slot * 16 + ln if isy else UV + cp * CV + slot * 8 + (ln & 7)
            ah.append(colp + i * P)
        v.append(cost(av))
        h.append(cost(ah))
    return v, h


def report(P, UV, CV, ring=3):
    tot = 0
    for s in range(ring):
        v, h = passes(P, UV, CV, ring, s)
        tot += sum(v) + sum(h)
        print(f"  slot {s}: vertical {''.join(map(str, v))}  horizontal {''.join(map(str, h))}")
    print(f"  cycles per 32-lane group over {ring} slots: {tot} (conflict-free: {ring * 40})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", action="store_true")
    a = ap.parse_args()
    print("shipped: pitch 40, chroma at 804, V at +16, 2-slot ring")
    report(40, 804, 16, 2)
    print("round 2: pitch 40, chroma at 800, V at +16, 2-slot ring")
    report(40, 800, 16, 2)
    print("loop filter one MB behind (be261fe): pitch 56, chroma at 20*56+4, V at +24, 3-slot ring")
    report(56, 20 * 56 + 4, 24)
    print("pitch 52, chroma at 20*52, V at +24, 3-slot ring (first lagged build)")
    report(52, 20 * 52, 24)
    if a.search:
        best = []
        for P in (52, 56):  # 48 B of luma per row; two 4K frames per CU leave ~1830 B of tiles per half
            for UV in range(20 * P, 20 * P + 256, 4):
                for CV in range(24, P - 23, 4):
                    if UV + 12 * P > 1840:
                        continue
                    t = sum(sum(x) for s in range(3) for x in passes(P, UV, CV, 3, s))
                    best.append((t, P, UV, CV))
        for b in sorted(best)[:8]:
            print("cycles %d: pitch %d, chroma at %d, V at +%d" % b)


if __name__ == "__main__":
    main()
