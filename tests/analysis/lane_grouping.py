"""Analysis (test infrastructure, not collected by pytest): would a wave of 64
frames of ONE pixel walk the BVH more coherently than a wave of an 8x8 pixel tile
at one frame?  Node-lane utilization = sum of per-lane node pops / (64 x the
longest lane), per bounce, from the oracle's traversal log (scene 8, seed 1).
Round 1 result: 0.326 (tile) vs 0.345 (frames of one pixel) -- no reason to regroup.
usage: python tests/analysis/lane_grouping.py"""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd")); sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np, pyoracle, rtamd
W,H=1920,1080
sc=rtamd.Scene(8,W,H,seed=1); osc=pyoracle.OracleScene(sc,max_depth=5,spp=4096)
L=pyoracle.lib(); L.oracle_trace_log.restype=ctypes.c_long
L.oracle_trace_log.argtypes=[ctypes.POINTER(pyoracle.OracleSceneDesc)]+[ctypes.c_int]*8+[ctypes.POINTER(ctypes.c_float),ctypes.POINTER(ctypes.c_int32),ctypes.c_long]
def log(x0,x1,y0,y1,frames):
    rf=rtamd.frame_rand_factors(1,0,frames)
    args=(ctypes.byref(osc.desc),W,H,x0,x1,y0,y1,1,frames,rf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    n=L.oracle_trace_log(*args,None,0); buf=np.empty(n,np.int32); L.oracle_trace_log(*args,buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),n)
    out=[];k=0
    while k<n:
        pix,fr,b,m=buf[k:k+4]; out.append((pix,fr,b,m)); k+=4+m
    return out
rng=np.random.default_rng(0)
A=[0,0];B=[0,0]
for _ in range(30):
    tx,ty=int(rng.integers(0,W//8)),int(rng.integers(0,H//8))
    # (a) 8x8 tile, per frame and bounce
    recs=log(tx*8,tx*8+8,ty*8,ty*8+8,4)
    g={}
    for pix,fr,b,m in recs: g.setdefault((fr,b),[]).append(m)
    for (fr,b),ms in g.items():
        A[0]+=sum(ms); A[1]+=64*max(ms)
    # (b) one pixel, 64 frames, per bounce
    px,py=tx*8+3,ty*8+3
    recs=log(px,px+1,py,py+1,64)
    g={}
    for pix,fr,b,m in recs: g.setdefault(b,[]).append(m)
    for b,ms in g.items():
        B[0]+=sum(ms); B[1]+=64*max(ms)
print("8x8 tile same frame: node-lane util %.3f (sum %d / lanes*max %d)"%(A[0]/A[1],A[0],A[1]))
print("1 pixel x 64 frames: node-lane util %.3f (sum %d / lanes*max %d)"%(B[0]/B[1],B[0],B[1]))
