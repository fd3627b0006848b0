"""How often the runner-up of an FPS step's merge is the next step's winner (numpy, the kernel's
16^3 Morton bucket layout and 512-thread wave assignment, 65 536 uniform points, 4 096 samples).
Measured: 0.851.  Used to price an L2 touch-ahead for the SA1 FPS."""
import numpy as np
rng=np.random.default_rng(2)
N=65536; M=4096; NW=8
x=rng.uniform(-1,1,(N,3)).astype(np.float32)
# bucket layout as the kernel (16^3 Morton, random order inside a cell)
def spread(v):
    r=np.zeros_like(v)
    for b in range(4): r|=((v>>b)&1)<<(3*b)
    return r
lo=x.min(0); hi=x.max(0); c=np.clip(((x-lo)*(16/(hi-lo))).astype(np.int64),0,15)
k=spread(c[:,0])|(spread(c[:,1])<<1)|(spread(c[:,2])<<2)
order=np.lexsort((rng.random(N),k))
wave_of=np.empty(N,np.int64); wave_of[order]=(np.arange(N)//64)%NW
dist=np.full(N,np.inf,np.float32); last=0; hit=0; tot=0
for it in range(1,M):
    q=x[last]; d=((x-q)**2).sum(1).astype(np.float32)
    # prediction made at the merge BEFORE this update: runner-up among wave candidates
    dist=np.minimum(dist,d)
    # merge: per-wave best (max dist, lowest index)
    cands=[]
    for w in range(NW):
        m=np.where(wave_of==w)[0]; j=m[np.argmax(dist[m])]; cands.append((dist[j],-j))
    cands.sort(reverse=True)
    new=-cands[0][1]
    if it>1:
        tot+=1; hit+=(pred==new)
    last=new; pred=-cands[1][1]
print('runner-up prediction hit rate %.3f over %d steps'%(hit/tot,tot))
