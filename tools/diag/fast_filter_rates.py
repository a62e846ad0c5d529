"""Pass rates of FAST pre-tests on a KITTI-like level-0 frame (numpy, CPU): the compass pair test, 4 of the 8
even ring points, the compass-aligned block of 5 and the exact corner test."""
import sys, numpy as np
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "orb-slam-_amd"), os.path.join(R, "oracle")]
import orbx_synth, orbref
img = orbx_synth.kitti_sequence(1, start=5)[0].astype(np.int32)
H,W = img.shape
ring = [(0,3),(1,3),(2,2),(3,1),(3,0),(3,-1),(2,-2),(1,-3),(0,-3),(-1,-3),(-2,-2),(-3,-1),(-3,0),(-3,1),(-2,2),(-1,3)]
# ring as (dx,dy) order doesn't matter for rates as long as cyclic
c = img[3:H-3,3:W-3]
x = np.stack([img[3+dy:H-3+dy,3+dx:W-3+dx] for dx,dy in ring])
t=7
br = x > c+t; dk = x < c-t
def arc(m, L):
    N=m.shape[0]
    # any cyclic run of length L
    r = np.zeros(m.shape[1:],bool)
    for k in range(N):
        a = np.ones(m.shape[1:],bool)
        for j in range(L): a &= m[(k+j)%N]
        r |= a
    return r
full = arc(br,9)|arc(dk,9)
comp = lambda m: (m[0]&m[4])|(m[4]&m[8])|(m[8]&m[12])|(m[12]&m[0])
cp = comp(br)|comp(dk)
ev = lambda m: arc(m[::2],4)
e8 = ev(br)|ev(dk)
n=c.size
print("pixels",n,"compass",cp.mean(),"even4of8",e8.mean(),"full s>7",full.mean())
t=20
br = x > c+t; dk = x < c-t
print("t20 full", (arc(br,9)|arc(dk,9)).mean(), "compass", (comp(br)|comp(dk)).mean())
t=7
br = x > c+t; dk = x < c-t
def blk(m):
    r = np.zeros(m.shape[1:],bool)
    for P in (0,4,8,12):
        a = np.ones(m.shape[1:],bool)
        for j in range(5): a &= m[(P+j)%16]
        r |= a
    return r
b5 = blk(br)|blk(dk)
print("t7 block5", b5.mean(), "compass&block5", (cp&b5).mean())
# compass then also check block of 3 at P+2 compass? 
