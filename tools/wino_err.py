"""f32 error of the Winograd F(2x2x2,3x3x3) conv1 product (numpy f32 emulation of
the transforms and the 4-channel sum) vs float64, beside the sequential f32
direct 108-term sum: measured 4.5e-7 vs 9.9e-7 max on 4000 windows."""
import numpy as np
rng=np.random.default_rng(0)
f=np.float32
G=np.array([[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]],f)
BT=np.array([[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]],f)
AT=np.array([[1,1,1,0],[0,1,-1,-1]],f)
def t3(M, X):  # apply M along each of 3 axes, f32 stepwise
    X=np.einsum('ai,ijk->ajk',M,X).astype(f)
    X=np.einsum('bj,ajk->abk',M,X).astype(f)
    X=np.einsum('ck,abk->abc',M,X).astype(f)
    return X
N=4000
errs=[];errd=[];mags=[]
w=(rng.standard_normal((16,4,3,3,3))/np.sqrt(108)).astype(f)
U=np.stack([np.stack([t3(G,w[co,ci]) for ci in range(4)]) for co in range(16)])  # [16,4,4,4,4]
for t in range(N):
    d=rng.random((4,4,4,4)).astype(f)  # ci, z,y,x
    V=np.stack([t3(BT,d[ci]) for ci in range(4)])  # [4,4,4,4]
    co=t%16
    M=np.zeros((4,4,4),f)
    for ci in range(4):
        M=(M+U[co,ci]*V[ci]).astype(f)
    Y=t3(AT,M)  # 2x2x2
    # f64 direct
    dd=d.astype(np.float64); ww=w[co].astype(np.float64)
    ref=np.zeros((2,2,2))
    for oz in range(2):
        for oy in range(2):
            for ox in range(2):
                ref[oz,oy,ox]=np.sum(dd[:,oz:oz+3,oy:oy+3,ox:ox+3]*ww)
    # f32 direct (sequential)
    dir32=np.zeros((2,2,2),f)
    for oz in range(2):
        for oy in range(2):
            for ox in range(2):
                acc=f(0)
                for v in (d[:,oz:oz+3,oy:oy+3,ox:ox+3]*w[co]).reshape(-1): acc=f(acc+v)
                dir32[oz,oy,ox]=acc
    errs.append(np.abs(Y-ref).max()); errd.append(np.abs(dir32-ref).max())
    mags.append(np.sum(np.abs(dd[:,0:4,0:4,0:4]))*np.abs(ww).max())
errs=np.array(errs);errd=np.array(errd)
print('winograd max err',errs.max(),'p99',np.quantile(errs,.99),'mean',errs.mean())
print('direct   max err',errd.max(),'p99',np.quantile(errd,.99),'mean',errd.mean())
