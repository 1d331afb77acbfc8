#!/usr/bin/env python3
"""LDS bank conflicts of k_orient_desc's rBRIEF sample reads (orient_kernels.hip phase C;
ORBextractor.cc:117-157) against the layout of the staged 37x37 blurred neighbourhood: lane L
reads the two points of tests L + 64t (t = 0..3) rotated by a random keypoint angle, as byte
reads; a wave64 byte / dword LDS read issues as two 32-lane groups, bank = (byte address / 4)
mod 32 (MI355X_MICROARCH.md, LDS table), reads of one dword broadcast.  Prints the mean LDS
cycles per 32-lane group read (1.0 = conflict-free) for

  pitch P         row r at byte r * P (today: P = 48)
  xor             dword column d of row r stored at column d ^ h(r) (h: a row hash into the
                  12 dwords a row spans, several hashes)
  rot             a 33-dword pitch with a per-row rotate of the row's dwords by 7 r
  lane order      the best any per-lane order of a lane's 8 reads can do for the slot's angle
                  (a greedy schedule, an upper bound on what such a reorder could reach)
  random          32 uniformly random dwords per group (the balls-in-bins floor of an
                  angle-independent layout)

CPU only.  usage: orient_bank_sim.py [nangles]
"""
import math
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
txt = open(os.path.join(ROOT, "oracle", "orb_pattern.inc")).read()
pairs = re.findall(r"ORBG_PAIR\(\s*(-?\d+),\s*(-?\d+),\s*(-?\d+),\s*(-?\d+)\)", txt)
pat = np.array([int(v) for p in pairs for v in p][-1024:]).reshape(256, 4)  # x0, y0, x1, y1
R = 18


def samples(ang):
    """(8, 64, 2) rotated (row, column) of read k = 2 t + s of lane L, cvRound as the kernel"""
    a, b = np.float32(math.cos(ang)), np.float32(math.sin(ang))
    out = np.zeros((8, 64, 2), np.int64)
    for t in range(4):
        for s in range(2):
            px = pat[64 * t:64 * t + 64, 2 * s].astype(np.float32)
            py = pat[64 * t:64 * t + 64, 2 * s + 1].astype(np.float32)
            ry = np.rint(px * b + py * a).astype(np.int64)
            rx = np.rint(px * a - py * b).astype(np.int64)
            out[2 * t + s, :, 0] = ry + R
            out[2 * t + s, :, 1] = rx + R
    return out


def group_cycles(dw):
    """cycles of one 32-lane group reading dword addresses dw (broadcast of equal dwords)"""
    d = np.unique(dw)
    return np.bincount(d % 32, minlength=32).max()


def cost(addr_fn, angles, sh_rand=True, rng=None):
    tot = n = 0
    for ang in angles:
        sm = samples(ang)
        sh = int(rng.integers(0, 4)) if sh_rand else 0
        for k in range(8):
            dw = addr_fn(sm[k, :, 0], sm[k, :, 1] + sh)
            for g in range(2):
                tot += group_cycles(dw[32 * g:32 * g + 32])
                n += 1
    return tot / n


def pitch(P):
    return lambda r, c: (r * P + c) // 4


def xor_swz(P, h):
    return lambda r, c: r * (P // 4) + ((c // 4) ^ h(r))


def rot33():
    return lambda r, c: r * 33 + ((c // 4 + 7 * r) % 12)


def lane_order(P, angles, rng):
    """greedy per-lane order of the 8 reads of each lane: instruction k takes, per lane, the
    remaining read whose bank is least loaded in that lane's group so far"""
    tot = n = 0
    for ang in angles:
        sm = samples(ang)
        sh = int(rng.integers(0, 4))
        dw = (sm[:, :, 0] * P + sm[:, :, 1] + sh) // 4  # (8, 64)
        for g in range(2):
            left = [list(range(8)) for _ in range(32)]
            for k in range(8):
                load = {}
                for L in rng.permutation(32):
                    best = None
                    for j in left[L]:
                        d = int(dw[j, 32 * g + L])
                        c = 0 if d in load else sum(1 for x in load if x % 32 == d % 32)
                        if best is None or c < best[0]:
                            best = (c, j, d)
                    left[L].remove(best[1])
                    load[best[2]] = 1
                tot += np.bincount(np.array(list(load)) % 32, minlength=32).max()
                n += 1
    return tot / n


def main():
    nang = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rng = np.random.default_rng(1)
    angles = rng.uniform(0, 2 * math.pi, nang)
    print("layout                              cycles / 32-lane read")
    for P in (40, 44, 48, 52, 56, 60, 64, 68, 72, 76, 80):
        print("pitch %-3d                            %.3f" % (P, cost(pitch(P), angles, rng=rng)))
    hashes = {"r % 12": lambda r: r % 12, "(5 r) % 12": lambda r: (5 * r) % 12,
              "(r ^ r >> 2) & 7": lambda r: (r ^ (r >> 2)) & 7, "(3 r) & 7": lambda r: (3 * r) & 7}
    for name, h in hashes.items():
        print("xor, pitch 48, h = %-17s %.3f" % (name, cost(xor_swz(48, h), angles, rng=rng)))
    print("33-dword pitch, rotate 7 r             %.3f" % cost(rot33(), angles, rng=rng))
    print("per-lane read order (greedy), P 48     %.3f" % lane_order(48, angles[:60], rng))
    rnd = np.mean([group_cycles(rng.integers(0, 37 * 12, 32)) for _ in range(20000)])
    print("32 random dwords (balls in bins)       %.3f" % rnd)


if __name__ == "__main__":
    main()
