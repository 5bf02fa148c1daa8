import sys, numpy as np, math
sys.path[:0]=['/root/repo','/root/repo/oracle','/root/repo/tests']
import oracle as O, pyref
from lorb_slam_amd import synth
f32=np.float32
def ceilh(d): return int(math.ceil(f32(f32(d)/f32(2))))
def sim(kx,ky,kr,minX,maxX,minY,maxY,N,trace=None,perms=None):
    n=len(kx); kx=np.asarray(kx,f32); ky=np.asarray(ky,f32)
    nini=int(math.floor(float(f32(maxX-minX)/f32(maxY-minY))+0.5)); hx=f32(f32(maxX-minX)/f32(nini)); ht=maxY-minY
    b=[min(int(f32(kx[p]/hx)),nini-1) for p in range(n)]
    perm=[p for bb in range(nini) for p in range(n) if b[p]==bb]
    cur=[]; beg=0
    for bb in range(nini):
        k=sum(1 for p in range(n) if b[p]==bb)
        if k: cur.append(dict(x0=int(f32(hx*f32(bb))),x1=int(f32(hx*f32(bb+1))),y0=0,y1=ht,beg=beg,end=beg+k,cre=bb,pend=0))
        beg+=k
    mode=0
    while True:
        L=len(cur)
        act=[(nd['end']-nd['beg']>=2) if mode==0 else nd['pend'] for nd in cur]
        own=[None]*n
        for i,nd in enumerate(cur):
            for p in range(nd['beg'],nd['end']): own[p]=i
        cls=[-1]*n
        for p in range(n):
            o=own[p]
            if act[o]:
                nd=cur[o]; k=perm[p]
                mx=nd['x0']+ceilh(nd['x1']-nd['x0']); my=nd['y0']+ceilh(nd['y1']-nd['y0'])
                cls[p]=(0 if ky[k]<my else 2) if kx[k]<mx else (1 if ky[k]<my else 3)
        ex=[];run=[0,0,0,0]
        for p in range(n):
            ex.append(list(run))
            if cls[p]>=0: run[cls[p]]+=1
        ex.append(list(run))
        cnt={}; ech={}
        for i,nd in enumerate(cur):
            if act[i]:
                k=[ex[nd['end']][c]-ex[nd['beg']][c] for c in range(4)]; cnt[i]=k; ech[i]=sum(1 for c in k if c>0)
        acts=[i for i in range(L) if act[i]]
        if mode==0: order=acts
        else: order=sorted(acts,key=lambda i:(cur[i]['end']-cur[i]['beg'],cur[i]['cre']),reverse=True)
        rank={i:r for r,i in enumerate(order)}
        cm=len(order)
        if mode==1:
            live=L
            for r,i in enumerate(order):
                live+=ech[i]-1
                if live>=N: cm=r+1; break
        committed=set(order[:cm])
        E=sum(ech[i] for i in order[:cm])
        newperm=list(perm)
        for p in range(n):
            o=own[p]
            if o in committed:
                nd=cur[o];c=cls[p];k=cnt[o]
                newperm[nd['beg']+sum(k[:c])+ex[p][c]-ex[nd['beg']][c]]=perm[p]
        nxt=[None]*(E+ (L-cm))
        sr=0; incl=0
        for i in range(L):
            if i not in committed:
                s=dict(cur[i]); s['pend']=0; nxt[E+sr]=s; sr+=1
        n_pend=0
        for r,i in enumerate(order[:cm]):
            incl+=ech[i]; slot=E-incl; nd=cur[i]; k=cnt[i]; beg=nd['beg']+sum(k)
            mx=nd['x0']+ceilh(nd['x1']-nd['x0']); my=nd['y0']+ceilh(nd['y1']-nd['y0'])
            for c in (3,2,1,0):
                beg-=k[c]
                if k[c]==0: continue
                ch=dict(x0=mx if c&1 else nd['x0'],x1=nd['x1'] if c&1 else mx,y0=my if c&2 else nd['y0'],y1=nd['y1'] if c&2 else my,beg=beg,end=beg+k[c],cre=4*r+c,pend=int(k[c]>1))
                nxt[slot]=ch; slot+=1; n_pend+=k[c]>1
        perm=newperm; newL=len(nxt)
        if perms is not None: perms.append(list(perm))
        if trace is not None:
            row=[L,mode,len(order),cm,E,L-cm,newL,n_pend]
            for q in range(min(16,newL)): row+= [nxt[q]['beg'],nxt[q]['end'],nxt[q]['x0'],nxt[q]['y0']]
            trace.append(row)
        done=newL>=N or newL==L
        if not done and mode==0 and newL+3*n_pend>N: mode=1
        cur=nxt
        if done: break
    out=[]
    for nd in cur:
        best=perm[nd['beg']]
        for q in range(nd['beg']+1,nd['end']):
            if kr[perm[q]]>kr[best]: best=perm[q]
        out.append(best)
    return np.array(out)
if __name__ == "__main__":
    import ctypes as C
    from lorb_slam_amd import _abi as A
    from lorb_slam_amd.runtime import Context, lib
    ctx = Context(0)
    pr = synth.orb_problem(seed=61, n_kps=1); pyr = pr['pyr']
    nd = O.orb_features_per_level(1000)
    buf, P = A.pack_pyramid(pyr); P.data = buf.ctypes.data
    tr = np.zeros(8 * (64 * 72 + 16384), np.int32)
    sf = A.f32(synth.scale_factors())
    rc = lib().lorb_orb_debug_octree(ctx.handle, C.byref(P), A.ptr(A.i32(nd), C.c_int32), A.ptr(sf, C.c_float), 20, 7,
                                     A.ptr(tr, C.c_int32))
    assert rc == 0, lib().lorb_last_error(ctx.handle)
    gperm = tr[8 * 64 * 72:].reshape(8, 16384); tr = tr[:8 * 64 * 72].reshape(8, 64, 72)
    f = O.orb_fast_cells(pyr)
    for l, p in enumerate(pyr):
        b0, b1 = f["cell_off"][f["cell_base"][l] + l], f["cell_off"][f["cell_base"][l + 1] + l]
        kx, ky, kr = f["x"][b0:b1] - 16, f["y"][b0:b1] - 16, f["response"][b0:b1]
        t = []
        ps = []
        sim(kx, ky, kr, 16, p.shape[1] - 16, 16, p.shape[0] - 16, nd[l], t, ps)
        for k, row in enumerate(t):
            g = tr[l, k][:len(row)].tolist()
            print(l, k, "sim", row, "gpu", g, "" if row == g else "<<<")
        break
