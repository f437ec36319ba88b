import numpy as np
NN=8; N=2*NN
x,wt=np.polynomial.legendre.leggauss(NN)
mu=(x+1)/2; w=wt/2; sd=np.sqrt(w/mu)
P=np.array([np.polynomial.legendre.Legendre.basis(l)(mu) for l in range(N)])  # [l][i]
def tour(P_):
    # circle-method rounds
    idx=list(range(P_)); rounds=[]
    for r in range(P_-1):
        rounds.append([(idx[k],idx[P_-1-k]) for k in range(P_//2)])
        idx=[idx[0]]+[idx[-1]]+idx[1:-1]
    return rounds
RND=tour(NN)
def sym_B(ssa,g):
    f=g**N; om=ssa*(1-f)/(1-ssa*f); rf=om/(1-f)
    chi=np.array([g**l for l in range(N+1)]); chi[0]=1
    ap=np.zeros((NN,NN)); lc=np.zeros((NN,NN))
    for l in range(N):
        gl=(2*l+1)*(chi[l]-f)*rf
        M=gl*np.outer(P[l],P[l])
        if l%2==0: ap+=M
        else: lc+=M
    S=np.outer(sd,sd)
    Ap=np.diag(1/mu)-S*ap; Am=np.diag(1/mu)-S*lc
    Lm=np.linalg.cholesky(Am); C=np.linalg.cholesky(Ap)
    return C.T@Lm
def jac(B,maxs=30):
    B=B.copy(); 
    for sweep in range(maxs):
        nrm=(B*B).sum(0); dia=(nrm*nrm).sum(); off=0
        for rnd in RND:
            for p,q in rnd:
                gam=B[:,p]@B[:,q]; off+=gam*gam
                app,aqq=nrm[p],nrm[q]
                if gam*gam<=1e-30*app*aqq: continue
                d=aqq-app; w_=np.sqrt(d*d+4*gam*gam); u=abs(d)+w_; z=1/np.sqrt(2*w_*u)
                c=u*z; s=(-2 if d<0 else 2)*gam*z
                bp=B[:,p].copy(); bq=B[:,q].copy()
                B[:,p]=c*bp-s*bq; B[:,q]=s*bp+c*bq
                nrm[p]=(B[:,p]**2).sum(); nrm[q]=(B[:,q]**2).sum()
        if not off>1e-16*dia: return sweep+1,B
    return maxs,B
rng=np.random.default_rng(1)
nl=64*40
res=[];resp=[]
for t in range(nl):
    ssa=rng.uniform(0,0.99); g=rng.uniform(0,0.85)
    B=sym_B(ssa,g)
    n1,_=jac(B)
    Sym=B.T@B; R=np.linalg.cholesky(Sym).T  # Sym=R^T R
    n2,X=jac(R.T)
    # check eigenvalues
    ev=np.sort((X*X).sum(0)); ev0=np.sort(np.linalg.eigvalsh(Sym))
    assert np.allclose(ev,ev0,rtol=1e-10),(ev,ev0)
    res.append(n1);resp.append(n2)
res=np.array(res);resp=np.array(resp)
print('plain  mean',res.mean(),'wave max mean',res.reshape(-1,64).max(1).mean(), np.bincount(res))
print('precon mean',resp.mean(),'wave max mean',resp.reshape(-1,64).max(1).mean(), np.bincount(resp))
r2=[];r3=[]
rng=np.random.default_rng(1)
for t in range(nl):
    ssa=rng.uniform(0,0.99); g=rng.uniform(0,0.85)
    B=sym_B(ssa,g); Sym=B.T@B; R=np.linalg.cholesky(Sym).T
    R2=np.linalg.cholesky(R@R.T).T
    n,_=jac(R2.T); r2.append(n)
    # reversed order precon
    Rr=np.linalg.cholesky(Sym[::-1,::-1]).T
    n,_=jac(Rr.T); r3.append(n)
r2=np.array(r2); r3=np.array(r3)
print('2xLR mean',r2.mean(),'wave max',r2.reshape(-1,64).max(1).mean(),np.bincount(r2))
print('rev  mean',r3.mean(),'wave max',r3.reshape(-1,64).max(1).mean(),np.bincount(r3))
