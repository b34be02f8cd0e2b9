"""Host check behind DESIGN.md section 6: can the lane kernel drop its stored Riccati gains by
forward shooting (u_i from stationarity, costate carried forward from lambda_0 = p_0)? Compares
the feedback rollout (u = K x + k) with shooting on the same unconstrained LQ (the model of
src/model.cpp:30-59, diagonal Q, R) in fp64; prints the max relative difference of u.
Usage: python tools/shooting_stability.py"""
import numpy as np
def lin(th,v,d,dt):
    L=np.float64(np.float32(0.3302))
    A=np.eye(3); A[0,2]=-v*np.sin(th)*dt; A[1,2]=v*np.cos(th)*dt
    B=np.zeros((3,2)); B[0,0]=np.cos(th)*dt; B[1,0]=np.sin(th)*dt; B[2,0]=np.tan(d)*dt/L; B[2,1]=v/np.cos(d)**2*dt/L
    return A,B
def run(N,q,r,v,d,dt,seed=0):
    rng=np.random.default_rng(seed)
    A,B=lin(0.3,v,d,dt); Q=np.diag(q); R=np.diag(r); ud=np.array([4.5,0.])
    refs=np.cumsum(rng.normal(0,0.05,(N,3)),0)
    # backward
    P=Q.copy(); p=-Q@refs[N-1]; Ks=[];ks=[]
    for i in range(N-1,-1,-1):
        H=R+B.T@P@B; X=B.T@P@A; h=-R@ud+B.T@p
        K=-np.linalg.solve(H,X); k=-np.linalg.solve(H,h)
        Ks.append(K);ks.append(k)
        P=Q+A.T@P@A+X.T@K; p=-Q@refs[i]+A.T@p+X.T@k
    Ks=Ks[::-1];ks=ks[::-1]
    x=np.zeros(3); uK=[]
    for i in range(N):
        u=Ks[i]@x+ks[i]; uK.append(u); x=A@x+B@u
    lam=p.copy(); x=np.zeros(3); uS=[]; Ai=np.linalg.inv(A.T)
    for i in range(N):
        lam=Ai@(lam-Q@(x-refs[i])); u=ud-np.linalg.solve(R,B.T@lam); uS.append(u); x=A@x+B@u
    uK=np.array(uK);uS=np.array(uS)
    term=lam*0  # terminal check
    return np.abs(uK-uS).max()/max(1,np.abs(uK).max())
for N in (20,40,48):
  for (q,r) in (([10,10,0],[0.1,5]),([3,7,2],[0.5,1.5]),([100,100,10],[0.01,0.1])):
    for d in (0.0,0.4):
      for dt in (0.01,0.05,0.1):
        print(N,q,r,d,dt,"%.2e"%run(N,q,r,4.5,d,dt))
