#!/usr/bin/env python3
"""Would a BVH over the C4 pre-cull rows beat the flat pass? Builds approximate boxes of the C4 rows (frozen scene),
a binary median-split tree, and counts, for random bounce rays in the room, the boxes each unbounded ray enters and
the nodes a stackless per-lane traversal tests (mean and slowest lane of each 64-ray wave). CPU only."""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
f=json.load(open(os.path.join(ROOT, 'sail_amd', 'scenes', 'frozen.json')))
sc=f['C4']; n=sc['n']; ob=np.array(sc['objects']).reshape(n,18)
boxes=[]
for i in range(1,n):
    r=ob[i]; t=int(r[0]); p=r[1:4]
    if t==1: lo,hi=r[1:4],r[4:7]
    elif t==2: lo,hi=p-r[4],p+r[4]
    elif t in (4,5): rad,h=r[5],r[4]; lo=p-[rad,0,rad]; hi=p+[rad,h,rad]
    else:
        e=max(abs(r[4:10]).max(),0.5); lo,hi=p-e,p+e
    boxes.append((np.minimum(lo,hi)-1e-3,np.maximum(lo,hi)+1e-3))
B=np.array(boxes)  # (m,2,3)
m=len(B)
# binary BVH by median split on longest axis
nodes=[]  # (lo,hi,leaf_or_-1, left,right)
def build(idx):
    lo=B[idx,0].min(0); hi=B[idx,1].max(0)
    k=len(nodes); nodes.append([lo,hi,-1,-1,-1])
    if len(idx)==1: nodes[k][2]=idx[0]; return k
    c=(B[idx,0]+B[idx,1])/2; ax=np.argmax(hi-lo); o=idx[np.argsort(c[:,ax])]; h=len(o)//2
    l=build(o[:h]); r=build(o[h:]); nodes[k][3]=l; nodes[k][4]=r; return k
build(np.arange(m))
rng=np.random.default_rng(1)
N=64*400
O=rng.uniform(0.2,9.8,(N,3)); O[:,2]=rng.uniform(-0.8,9.8,N)
D=rng.normal(size=(N,3)); D/=np.linalg.norm(D,axis=1,keepdims=True)
inv=1/D
def hit(lo,hi,o,iv):
    t0=(lo-o)*iv; t1=(hi-o)*iv
    tmin=np.minimum(t0,t1).max(-1); tmax=np.maximum(t0,t1).min(-1)
    return (tmin<=tmax)&(tmax>=0)
# flat pass counts
passes=np.zeros(N,int)
for j in range(m): passes+=hit(B[j,0],B[j,1],O,inv)
print('mean padded boxes entered per ray', passes.mean())
visits=np.zeros(N,int)
for r in range(N):
    st=[0]; v=0
    while st:
        k=st.pop(); v+=1
        lo,hi,leaf,l,rr=nodes[k]
        if hit(lo,hi,O[r],inv[r]) and leaf<0: st+= [l,rr]
    visits[r]=v
print('mean node tests per ray', visits.mean(), 'nodes', len(nodes))
w=visits.reshape(-1,64)
print('mean max-over-wave node tests', w.max(1).mean(), 'lane eff', w.mean()/w.max(1).mean())
