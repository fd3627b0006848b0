"""FPS bucket pruning by layout (numpy): active buckets per step (bbox lower bound < bucket max),
buckets with at least one changed member, and changed points per step, for 64-point runs of a 16^3 or
finer Morton order and for runs padded to Morton blocks.  usage: fps_prune_sim.py STEPS LAYOUT...
(m16 m64 oct1 oct2 fo2 fo3)."""
import numpy as np, sys
rng=np.random.default_rng(1)
N=65536; M=int(sys.argv[1]) if len(sys.argv)>1 else 1024
x=rng.uniform(-1,1,(N,3)).astype(np.float32)
def spread(v,bits):
    r=np.zeros_like(v)
    for b in range(bits): r|=((v>>b)&1)<<(3*b)
    return r
def morton(x,g):
    lo=x.min(0); hi=x.max(0)
    c=np.clip(((x-lo)*(g/(hi-lo))).astype(np.int64),0,g-1)
    bits=int(np.log2(g))
    return spread(c[:,0],bits)|(spread(c[:,1],bits)<<1)|(spread(c[:,2],bits)<<2)
def layout(kind):
    if kind=='m16':
        k=morton(x,16); order=np.lexsort((rng.random(N),k))
        return [order[i:i+64] for i in range(0,N,64)]
    if kind in('m64','m128','m256'):
        g=int(kind[1:]); k=morton(x,g); order=np.argsort(k,kind='stable')
        return [order[i:i+64] for i in range(0,N,64)]
    if kind.startswith('oct'):  # pad each level-L block (8^L cells of the 16^3 grid) to whole buckets
        L=int(kind[3:]); k=morton(x,16); order=np.lexsort((rng.random(N),k)); ks=k[order]
        blk=ks>>(3*L); out=[]
        for b in np.unique(blk):
            o=order[blk==b]
            out+= [o[i:i+64] for i in range(0,len(o),64)]
        return out
    if kind.startswith('fo'):  # finer order (64^3 morton) + pad blocks of level L of the 64^3 grid
        L=int(kind[2:]); k=morton(x,64); order=np.argsort(k,kind='stable'); ks=k[order]
        blk=ks>>(3*L); out=[]
        for b in np.unique(blk):
            o=order[blk==b]
            out+= [o[i:i+64] for i in range(0,len(o),64)]
        return out
for kind in sys.argv[2:]:
    B=layout(kind); nb=len(B)
    bmin=np.array([x[b].min(0) for b in B]); bmax=np.array([x[b].max(0) for b in B])
    bid=np.empty(N,np.int64)
    for i,b in enumerate(B): bid[b]=i
    dist=np.full(N,np.inf,np.float32); last=0
    act=0; useful=0; changed=0
    for it in range(1,M):
        q=x[last]
        g=np.maximum(np.maximum(bmin-q,q-bmax),0); lb=(g*g).sum(1)
        bd=np.full(nb,-1.0,np.float32); np.maximum.at(bd,bid,dist)
        a=lb<bd
        d=((x-q)**2).sum(1).astype(np.float32)
        ch=d<dist
        act+=a.sum(); u=np.zeros(nb,bool); u[bid[ch]]=True; useful+=u.sum(); changed+=ch.sum()
        dist=np.minimum(dist,d); last=int(np.argmax(dist))
    print(kind,'buckets',nb,'active/step %.1f useful/step %.1f changed pts/step %.1f'%(act/(M-1),useful/(M-1),changed/(M-1)))
