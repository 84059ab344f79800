#!/usr/bin/env python3
"""Model of the split-K dW unit assignment (td3.hip make_dw_split) at Humanoid C_dw, B = 1024: per
XCD, how long each 64-row block of a dZ / U panel stays live in L2 between its first and last
reader, for the tile-major walk (dwsk_kernel) and the step-major walk (dwsk_sm_kernel).  CPU only."""
# simulate dwsk unit assignment for Humanoid critic C_dw (B=1024): row-step skew within an XCD
import numpy as np
S=16; G=256; wm=6
def layer(N,K): return (-(-N//32)*32, -(-K//32)*32)
nets=[]
for net in range(2):
    dims=[376+17,500,400,200,1]
    for l in range(4):
        Np,Kp=layer(dims[l+1],dims[l]); nets.append((Np,Kp))
tiles=[]; wt=[]
for (Np,Kp) in nets:
    for nt in range(-(-Np//64)):
        for kt in range(-(-Kp//64)):
            tiles.append(('m',nt,kt)); wt.append(2+wm*1//4)
    for j in range(Np//32):
        tiles.append(('v',j,0)); wt.append(1)
units=len(tiles)*S
wtot=sum(w*S for w in wt); cw=-(-wtot//G)
vu=[];pos=0
for u in range(units):
    w=wt[u//S]; v=min(G-1,(2*pos+w)//(2*cw)); vu.append(v); pos+=w
vu=np.array(vu)
print("tiles",len(tiles),"matrix",sum(1 for t in tiles if t[0]=='m'),"units",units,"cw",cw)
def sim(order):
    # per WG: list of (time_start, step) ; compute for each (wg, step) the time when first processed
    first={}  # (xcd, step) -> list of start times
    spread=[]
    for v in range(G):
        us=np.nonzero(vu==v)[0]
        if order=='step': us=sorted(us,key=lambda u:(u%S,u//S))
        t=0
        for u in us:
            s=u%S
            first.setdefault((v//32,s),[]).append(t)
            t+=wt[u//S]
    for k,ts in first.items():
        spread.append(max(ts)-min(ts))
    return np.mean(spread), np.max(spread)
for o in ('tile','step'):
    print(o, "mean/max spread of a step's start times within an XCD (weight units; a step ~ 3):", sim(o))
# J
J=0
for v in range(G):
    us=np.nonzero(vu==v)[0]
    J=max(J,len(set(us//S)))
print("J",J)
# live L2 footprint per XCD: each (panel, step) block of 64 rows x 64 cols x 4 B = 16 KB lives from its
# first to its last read by the XCD's WGs (no reuse across XCDs)
def live(order):
    ev={}  # (xcd, panel_key, step) -> [tmin, tmax]
    tot_reads=0
    for v in range(G):
        us=np.nonzero(vu==v)[0]
        if order=='step': us=sorted(us,key=lambda u:(u%S,u//S))
        t=0
        for u in us:
            ti=u//S; s=u%S; kind,a,b=tiles[ti]
            # problem index
            # recover problem: count tiles per problem
            t1=t+wt[ti]
            if kind=='m':
                p=prob_of[ti]
                for key in (('dz',p,a),('u',p,b)):
                    k=(v//32,key,s); e=ev.setdefault(k,[t,t1]); e[0]=min(e[0],t); e[1]=max(e[1],t1)
                    tot_reads+=1
            t=t1
    # max over time of live blocks per xcd
    res=[]
    for x in range(8):
        iv=[(e[0],e[1]) for k,e in ev.items() if k[0]==x]
        pts=sorted(set([a for a,b in iv]+[b for a,b in iv]))
        mx=0
        for p in pts:
            c=sum(1 for a,b in iv if a<=p<b)
            mx=max(mx,c)
        res.append(mx*16/1024)
    distinct=len(ev)*16/1024
    return res, distinct, tot_reads*16/1024
prob_of=[]
pi=0
for (Np,Kp) in nets:
    n=(-(-Np//64))*(-(-Kp//64))+Np//32
    prob_of+= [pi]*n; pi+=1
for o in ('tile','step'):
    r,d,tr=live(o)
    print(o,"max live MB per XCD",[round(x,2) for x in r],"distinct-per-XCD total MB",round(d,1),"requested MB",round(tr,1))
def live2():
    ev={}
    for v in range(G):
        us=np.nonzero(vu==v)[0]
        mat=[u for u in us if tiles[u//S][0]=='m']; vec=[u for u in us if tiles[u//S][0]=='v']
        mat=sorted(mat,key=lambda u:(u%S,u//S))
        t=0
        for u in mat+vec:
            ti=u//S; s=u%S; kind,a,b=tiles[ti]; t1=t+wt[ti]
            if kind=='m':
                p=prob_of[ti]
                for key in (('dz',p,a),('u',p,b)):
                    k=(v//32,key,s); e=ev.setdefault(k,[t,t1]); e[0]=min(e[0],t); e[1]=max(e[1],t1)
            t=t1
    res=[]
    for x in range(8):
        iv=[(e[0],e[1]) for k,e in ev.items() if k[0]==x]
        pts=sorted(set([a for a,b in iv]))
        res.append(max(sum(1 for a,b in iv if a<=p<b) for p in pts)*16/1024)
    return res
print("matrix step-major, vectors last: max live MB per XCD",[round(x,2) for x in live2()])
# matrix segments per WG
mm=0
for v in range(G):
    us=np.nonzero(vu==v)[0]
    mm=max(mm,len(set(u//S for u in us if tiles[u//S][0]=='m')))
print("max matrix segments per WG",mm)
vv=0
for v in range(G):
    us=np.nonzero(vu==v)[0]
    vv=max(vv,len(set(u//S for u in us if tiles[u//S][0]=='v')))
print("max vector segments per WG",vv)
