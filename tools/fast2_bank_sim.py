"""k_fast2 scoring-loop LDS bank conflicts, simulated on the CPU.

Rebuilds the scoring task list of k_fast2 (fast_kernels.hip: the compass pretest at
iniThFAST, one entry per surviving (unit, pixel pair), lane order within each 64-unit
iteration, both-side pairs at the end) for level-0 cells of a synthetic 1241x376 frame, and
counts the LDS cycles of the 21 ds_read_b32 per task (two 32-lane groups per instruction,
bank = dword mod 32, identical addresses broadcast) for several tile row strides and lane
orders.  Prints cycles per group-instruction (1.0 = conflict-free).
"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from orb_slam2_test_amd import synthetic as S

img = S.frame(376, 1241).astype(np.int32)
H, W = img.shape
th = 20
rows = []
# 30-px cells on the level-0 region (border 16-3)
x0s = list(range(13, W - 13 - 30, 30))
y0s = list(range(13, H - 13 - 30, 30))
cells = [(x, y) for y in y0s for x in x0s]


def tasks_of(x0, y0):
    Wc = 36; Hc = 36
    RW, RH = Wc - 6, Hc - 6
    RG = (RW + 3) // 4
    out = []
    nunits = RH * RG
    for u0 in range(0, nunits, 64):
        both = []
        for lane in range(64):
            u = u0 + lane
            if u >= nunits:
                continue
            ry, gg = divmod(u, RG)
            for half in range(2):
                px = x0 + 3 + 4 * gg + 2 * half
                py = y0 + 3 + ry
                res = []
                for i in range(2):
                    x = px + i
                    v = img[py, x]
                    c0, c4, c8, c12 = img[py + 3, x], img[py, x + 3], img[py - 3, x], img[py, x - 3]
                    b = min(max(c0, c8), max(c4, c12)) > v + th
                    d = max(min(c0, c8), min(c4, c12)) < v - th
                    res.append((b, d))
                b = res[0][0] or res[1][0]
                d = res[0][1] or res[1][1]
                if b and d:
                    both.append((ry, gg)); both.append((ry, gg))
                elif b or d:
                    out.append((ry, gg))
        out.extend(both)
    return out


def conflict_cycles(tasks, RS4):
    cyc = 0; ideal = 0
    for j0 in range(0, len(tasks), 32):
        grp = tasks[j0:j0 + 32]
        for r in range(7):
            for k in range(3):
                addrs = set((ry + r) * RS4 + gg + k for ry, gg in grp)
                banks = {}
                for a in addrs:
                    banks[a % 32] = banks.get(a % 32, 0) + 1
                cyc += max(banks.values())
                ideal += 1
    return cyc, ideal


allt = [tasks_of(x, y) for (x, y) in cells[::5]]
print('cells', len(allt), 'tasks/cell', np.mean([len(t) for t in allt]))
for RS4 in [24, 26, 28, 30, 22, 25, 27, 36]:
    c = i = 0
    for t in allt:
        a, b = conflict_cycles(t, RS4)
        c += a; i += b
    print(RS4, 'cycles/instr', round(c / i, 3))


def rr_order(tasks, RS4=24):
    # rank within base bucket, then base: round-robin over the 32 bank classes
    cnt = {}
    keyed = []
    for (ry, gg) in tasks:
        b = (RS4 * ry + gg) % 32
        r = cnt.get(b, 0); cnt[b] = r + 1
        keyed.append((r, b, ry, gg))
    keyed.sort()
    return [(ry, gg) for _, _, ry, gg in keyed]


c = i = 0
for t in allt:
    a, b = conflict_cycles(rr_order(t), 24)
    c += a; i += b
print('rr 24 cycles/instr', round(c / i, 3))

lb = []
for t in allt:
    G = (len(t) + 31) // 32
    cnt = {}
    # distinct addresses only (same unit twice = one address)
    for (ry, gg) in set(t):
        b = (24 * ry + gg) % 32
        cnt[b] = cnt.get(b, 0) + 1
    lb.append((max((v + G - 1) // G for v in cnt.values()), G))
print('lower bound cycles/instr (weighted)', sum(a * g for a, g in lb) / sum(g for a, g in lb))
