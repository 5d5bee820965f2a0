"""CPU model: would the Chamfer's culled per-wave search (Morton-sorted clouds, 64-query waves,
nearest-first tiles, per-query box test against the K-th distance) cut the C = 3 kNN's list
insertions?  Prints the visited fraction of the pairs and the insertions per query, against the
index-order scan's.  DESIGN.md section "kNN" cites the result.

    python tools/knn_cull_sim.py
"""
import numpy as np
rng=np.random.default_rng(0)
N=2048; K=16
def morton(p, bits=4):
    lo=p.min(0); hi=p.max(0); sc=(2**bits-1e-3)/(hi-lo)
    c=np.clip(((p-lo)*sc).astype(int),0,2**bits-1)
    code=np.zeros(len(p),dtype=np.int64)
    for bit in range(bits):
        for ax in range(3): code |= ((c[:,ax]>>bit)&1) << (3*bit+ax)
    return np.argsort(code,kind='stable')
for kind in ["surface","gauss"]:
    if kind=="surface":
        v=rng.standard_normal((N,3)); P=v/np.linalg.norm(v,axis=1,keepdims=True)*[0.4,0.25,0.15]
    else: P=rng.standard_normal((N,3))*0.3
    o=morton(P); S=P[o]
    for TS in (32,64):
        nt=N//TS; tlo=S.reshape(nt,TS,3).min(1); thi=S.reshape(nt,TS,3).max(1)
        visited=0; ins=0; ins_idx=0
        for w in range(N//64):
            Q=S[w*64:(w+1)*64]
            q0=Q.min(0); q1=Q.max(0)
            gap=np.maximum(0,np.maximum(tlo-q1,q0-thi)); lb=(gap**2).sum(1)
            order=np.argsort(lb,kind='stable')
            thr=np.full(64,np.inf); lists=[[] for _ in range(64)]
            g=np.maximum(0,np.maximum(tlo[None]-Q[:,None],Q[:,None]-thi[None])); L=(g**2).sum(-1)
            for j in order:
                if lb[j]>thr.max(): break
                if not (L[:,j]<=thr).any(): continue
                visited+=1
                d=((Q[:,None,:]-S[j*TS:(j+1)*TS][None])**2).sum(-1)
                for l in range(64):
                    for k in range(TS):
                        if d[l,k]<thr[l]:
                            ins+=1; lists[l].append(d[l,k]); lists[l].sort(); lists[l]=lists[l][:K]
                            if len(lists[l])==K: thr[l]=lists[l][-1]
        print(kind,"TS",TS,"visited frac %.3f"%(visited/(nt*(N//64))),"insertions/query %.1f"%(ins/N),flush=True)
    # index order insertion count (original order)
    ins=0
    for qi in range(0,N,8):
        d=((P[qi]-P)**2).sum(-1); lst=[]; thr=np.inf
        for k in range(N):
            if d[k]<thr:
                ins+=1; lst.append(d[k]); lst.sort(); lst=lst[:K]
                if len(lst)==K: thr=lst[-1]
    print(kind,"index-order insertions/query %.1f"%(ins/(N/8)))
