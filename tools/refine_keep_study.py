"""Refinement with a kept search direction (design tool, CPU): fp32 inner
PCG (A rounded to fp32, the prototype V-cycle of tools/amg_proto.py as the
preconditioner) inside fp64 iterative refinement, each inner solve either
restarted (the library's scheme: p = z) or continuing the previous step's
search direction (p = z + (r.z / r.z_old) p_old, a reliable-update CG).
Prints the iterations of each step and the total to a relative residual of
TARGET (default 1e-10). Round 5, S1 with the library's hierarchy options:
restarted 18 + 24 + 23 = 65, kept 18 + 24 + 27 = 69.

    python tools/refine_keep_study.py CONFIG "sa2=0.66+om=0.7,1.05+sa1a2=0.66+sa1only=1+q0=1+q1=2" [TARGET]

The oracle is test infrastructure; this script is a design tool, never part
of the product path.
"""
import sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
import numpy as np, scipy.sparse as sp
import amg_proto as ap
cfg=sys.argv[1]; spec=sys.argv[2]
A,a2m,f,e,N=ap.system(cfg)
opts=ap.parse(spec.split('+'))
levels=ap.build(A,a2m,e,opts)
A32=A.astype(np.float32).tocsr()
M=lambda r: ap.vcycle(levels,0,r.astype(np.float64),opts).astype(np.float32)
nf=np.linalg.norm(f)
TARGET=float(sys.argv[3]) if len(sys.argv)>3 else 1e-10
def inner(r64, tol, state=None, keep=False):
    """fp32 PCG on A d = r64 from d=0; returns d (fp32), its, state (p, rz)"""
    r=r64.astype(np.float32); d=np.zeros_like(r)
    z=M(r); rz=np.float64(r@z)
    if keep and state is not None:
        p_old, rz_old = state
        p=(z+np.float32(rz/rz_old)*p_old).astype(np.float32)
    else:
        p=z.copy()
    n0=np.linalg.norm(r); its=0
    while True:
        q=A32@p; pq=np.float64(p@q); a=np.float32(rz/pq)
        d+=a*p; r-=a*q; its+=1
        if np.linalg.norm(r)<=tol*n0 or its>500: 
            return d,its,(p.copy(),rz)
        z=M(r); rz2=np.float64(r@z); p=(z+np.float32(rz2/rz)*p).astype(np.float32); rz=rz2
for mode in ('restart','keep'):
    x=np.zeros_like(f); r=f.copy(); tot=0; steps=0; st=None
    while np.linalg.norm(r)>TARGET*nf and steps<8:
        tol=1e-5 if steps==0 else 1e-4
        d,its,st=inner(r,tol,st,keep=(mode=='keep'))
        x+=d; r=f-A@x; tot+=its; steps+=1
        print(' ',mode,'step',steps,'its',its,'rel',np.linalg.norm(r)/nf, flush=True)
    print(cfg,mode,'total its',tot,'steps',steps, flush=True)
