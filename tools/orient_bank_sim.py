#!/usr/bin/env python3
"""LDS bank conflicts of k_orient_desc's rBRIEF sample reads (orient_kernels.hip phase C;
ORBextractor.cc:117-157) against the staged neighbourhood's row pitch: lane L reads the two
points of tests L + 64t (t = 0..3) rotated by a random keypoint angle, as byte reads of the
37-row staged tile; a wave64 LDS read issues as two 32-lane halves, 32 banks of 4 bytes,
reads of one dword broadcast.  Prints the mean cycles per half-wave read per pitch.
CPU only.  usage: orient_bank_sim.py
"""
import math
import re

import numpy as np
import os
txt=open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle', 'orb_pattern.inc')).read()
pairs=re.findall(r'ORBG_PAIR\(\s*(-?\d+),\s*(-?\d+),\s*(-?\d+),\s*(-?\d+)\)', txt)
nums=[int(v) for p in pairs for v in p]
pat=np.array(nums[-1024:]).reshape(256,4)   # x0,y0,x1,y1
rng=np.random.default_rng(1)
def cost(P, nang=400, sh_rand=True):
    tot=0; n=0
    for _ in range(nang):
        ang=rng.uniform(0,2*math.pi); a=np.float32(math.cos(ang)); b=np.float32(math.sin(ang))
        sh=rng.integers(0,4) if sh_rand else 0
        cb=18*P+sh+18
        for t in range(4):
            for s in range(2):
                px=pat[64*t:64*t+64, 2*s].astype(np.float32); py=pat[64*t:64*t+64,2*s+1].astype(np.float32)
                ry=np.rint(px*b+py*a).astype(int); rx=np.rint(px*a-py*b).astype(int)
                off=ry*P+rx+cb
                dw=off//4
                for half in range(2):
                    d=np.unique(dw[32*half:32*half+32])
                    banks=d%32
                    tot+=np.bincount(banks,minlength=32).max(); n+=1
    return tot/n
for P in (40,44,48,52,56,60,64,68,72,76,80):
    print(P, round(cost(P),3))
