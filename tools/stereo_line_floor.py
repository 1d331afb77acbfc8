#!/usr/bin/env python3
"""The HBM floor of k_stereo_sad (Frame.cc:740-832): distinct cache lines that the SAD windows
of one synthetic KITTI stereo pair touch (11x11 left patch, 11x21 right strip per match with
a depth, at the keypoint's level, the library's 256-byte level pitch), against the kernel's
algorithmic bytes (bench.py kernel_algo_bytes "stereo_sad").  Any kernel that reads each
touched line once moves at least this ratio: the windows are sparse 11-byte row pieces.
CPU only (oracle for the keypoints and matches).  usage: stereo_line_floor.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam2_test_amd import synthetic as S
from oracle import pyoracle as O
H,W=376,1241
p=O.params(nfeatures=2000)
sp=S.stereo_pair(H,W,seed=S.DEFAULT_SEED+5); L,R=sp[0],sp[1]
el=O.extract(p,L,with_pyramid=True); er=O.extract(p,R,with_pyramid=True)
bf=386.1448
ur,dp=O.stereo_matches(p,el,er,W,H,bf,bf/718.856)
kl=el['kps']; ok=ur>=0
print('kps',len(kl),'with depth',ok.sum())
scale=1.2**np.arange(8)
lw=[len(l[0]) for l in el['pyramid']]
for LINE in (64,128):
  lines=set(); alg=0
  for k,u in zip(kl[ok],ur[ok]):
    o=int(k['octave']); sf=1/scale[o]
    xl=int(round(k['x']*sf)); yl=int(round(k['y']*sf)); xr=int(round(u*sf))
    pitch=((lw[o]+255)//256)*256
    for r in range(yl-5,yl+6):
      for x in (xl-5,xl+5): lines.add((0,o,(r*pitch+x)//LINE))
      for x in (xr-10,xr+10): lines.add((1,o,(r*pitch+x)//LINE))
    alg+=11*11+11*21+12
  print(LINE,'alg KB %.1f distinct-line KB %.1f ratio %.2f'%(alg/1024,len(lines)*LINE/1024,len(lines)*LINE/alg))
