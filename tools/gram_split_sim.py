"""Accuracy of split-precision Gram matrices for the SVD denoiser (gram256s_kernel).

numpy emulation: X^T X from fp16 hi/lo pairs (power-of-two scaled, 3 products), bf16 pairs
(3 / 4 / 6 products) and numpy fp32 BLAS, each accumulated in float64 to isolate the
representation error; top-16 and default-range reconstructions from the float64
eigenvectors of each Gram vs the float64 SVD, relative Frobenius error. CPU only:
    python tools/gram_split_sim.py
"""
import numpy as np
rng=np.random.default_rng(0)
def bf16(x):
    x=np.asarray(x,np.float32); b=x.view(np.uint32).astype(np.uint64)
    b=(b+0x7FFF+((b>>16)&1))&0xFFFF0000
    return b.astype(np.uint32).view(np.float32)
def f16(x): return np.asarray(x,np.float32).astype(np.float16).astype(np.float32)
def gram_split(X,mode):
    X=X.astype(np.float32)
    if mode=="f32": return (X.T@X).astype(np.float64)   # fp32 BLAS
    if mode=="f64": X=X.astype(np.float64); return X.T@X
    if mode.startswith("bf"):
        h=bf16(X); l=bf16(X-h); m3=bf16(X-h-l)
        h,l,m3=[a.astype(np.float64) for a in (h,l,m3)]
        if mode=="bf3": return h.T@h+h.T@l+l.T@h
        if mode=="bf4": return h.T@h+h.T@l+l.T@h+l.T@l
        if mode=="bf6": return h.T@h+h.T@l+l.T@h+l.T@l+h.T@m3+m3.T@h
    if mode=="fp3":
        s=2.0**(14-np.ceil(np.log2(np.abs(X).max())))
        Y=(X*s).astype(np.float32); h=f16(Y); l=f16(Y-h)
        h,l=h.astype(np.float64),l.astype(np.float64)
        return (h.T@h+h.T@l+l.T@h)/s/s
def recon(A,G,lo,hi):
    X=A.astype(np.float64)
    w,V=np.linalg.eigh(G); V=V[:,::-1]
    if hi is None: v=V[:,:1]; return X-X@v@v.T
    v=V[:,lo:hi]; return X@v@v.T
def ref(A,lo,hi):
    u,s,vh=np.linalg.svd(A.astype(np.float64),full_matrices=False)
    if hi is None: lo,hi=1,len(s)
    return (u[:,lo:hi]*s[lo:hi])@vh[lo:hi]
def c3(m=513,n=256,k=16):
    U=np.linalg.qr(rng.standard_normal((m,k)))[0]; V=np.linalg.qr(rng.standard_normal((n,k)))[0]
    s=10*0.8**np.arange(k)
    return ((U*s)@V.T+0.01/m**0.5*rng.standard_normal((m,n))).astype(np.float32)
mats=[("c3",c3()) for _ in range(3)]
# spectrogram-like: positive PSD with wide dynamic range, 3905x256 (X = A^T)
t=np.abs(rng.standard_normal((3905,256)))**2*np.exp(rng.standard_normal((1,256))*3)*1e-9
mats.append(("psd",t.astype(np.float32)))
for name,A in mats:
    for rng_ in [(0,16),(1,None)]:
        R=ref(A,*rng_); nr=np.linalg.norm(R)
        out=[]
        for mode in ["f32","bf3","bf4","bf6","fp3"]:
            G=gram_split(A,mode); out.append(f"{mode} {np.linalg.norm(recon(A,G,*rng_)-R)/nr:.2e}")
        print(name,rng_," | ".join(out))
