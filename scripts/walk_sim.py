#!/usr/bin/env python
"""Request-count simulation of the hash-grid backward walk's fine-level flushes (diagnostics, CPU only): per-slot pending
merge (the kernel) vs a cross-slot merge (a new corner entry matching ANY pending entry of its level group), on
NeuS-like samples (half near a sphere surface) with the SDF batch's 4 taps, 4 samples x 5 points per block.
Prints per level the distinct 64-B line requests of each scheme and their ratio.

    python scripts/walk_sim.py
"""
import numpy as np
rng=np.random.default_rng(0)
R,S=880,64
o=rng.normal(size=(R,3)); o/=np.linalg.norm(o,axis=1,keepdims=True); o*=3
d=-o+0.3*rng.normal(size=(R,3)); d/=np.linalg.norm(d,axis=1,keepdims=True)
# NeuS-like: samples concentrated near the surface |x|=0.5: find t where ray hits sphere r=0.5 approx
b=(o*d).sum(1); c=(o*o).sum(1)-0.25; disc=b*b-c
th=np.where(disc>0,-b-np.sqrt(np.maximum(disc,0)),-b)
t=np.sort(np.concatenate([rng.uniform(1.5,4.5,(R,32)), th[:,None]+rng.normal(scale=0.02,size=(R,32))],1),1)
cen=(o[:,None,:]+t[...,None]*d[:,None,:]).reshape(-1,3).clip(-1,1)
M=cen.shape[0]
delta=2.0/1024/np.sqrt(3)
taps=np.array([[1,-1,-1],[-1,-1,1],[-1,1,-1],[1,1,1]],float)
pts=np.stack([cen]+[cen+delta*k for k in taps],1)  # M,5,3 walk order
P1,P2=2654435761,805459861
T=1<<19
def corners(x,s):
    xh=(x+1)/2*s
    f=np.floor(xh).astype(np.int64); cc=np.ceil(xh).astype(np.int64)
    out=[]
    for cz in (cc,f):
        for (cy,cx) in ((cc,cc),(f,cc),(f,f),(cc,f)):
            pass
    # corner slots q>>1: (xc?) per pr
    idx=[]
    for pr in range(4):
        yc=(pr&1)==0; zc=pr<2
        for xc in (True,False):
            X=(cc if xc else f)[...,0]; Y=(cc if yc else f)[...,1]; Z=(cc if zc else f)[...,2]
            idx.append(((X.astype(np.uint64))^(Y.astype(np.uint64)*np.uint64(P1))^(Z.astype(np.uint64)*np.uint64(P2)))&np.uint64(T-1))
    return np.stack(idx,-1)  # ...,8
CH=4
nb=M//CH
for L in range(8,16):
    s=float(int(16*1.3195079**L))
    idx=corners(pts[:nb*CH].reshape(nb,CH*5,3),s)  # nb, 20, 8
    # current: per-slot pending; flush when change; count requests = distinct lines per (step) among flushing slots (x2 feats same line)
    req_cur=0; req_x=0
    pend=idx[:,0,:].copy()
    for i in range(1,CH*5):
        new=idx[:,i,:]
        ch=new!=pend
        # lines of flushed pendings at this step
        lines=np.where(ch,pend//8,np.uint64(2**62))
        for bidx in range(0,1):
            pass
        ls=np.sort(lines,1); distinct=(np.diff(ls,axis=1)!=0).sum(1)+1 - (ls[:,-1]==2**62)
        req_cur+=distinct.sum()
        pend=np.where(ch,new,pend)
    req_cur+=nb*len(np.unique(pend[0]//8))  # approx final flush: distinct lines per block
    # cross-slot: new idx matching ANY pending in group -> absorbed
    pend=idx[:,0,:].copy()
    for i in range(1,CH*5):
        new=idx[:,i,:]
        match=(new[:,:,None]==pend[:,None,:]).any(2)
        repl=~match
        # slots whose own new is unmatched flush their pending (unless pending equals... ) 
        lines=np.where(repl,pend//8,np.uint64(2**62))
        ls=np.sort(lines,1); distinct=(np.diff(ls,axis=1)!=0).sum(1)+1 - (ls[:,-1]==2**62)
        req_x+=distinct.sum()
        pend=np.where(repl,new,pend)
    req_x+=nb*len(np.unique(pend[0]//8))
    print(L, int(s), 'cur', req_cur, 'cross', req_x, f"{req_x/req_cur:.2f}")
