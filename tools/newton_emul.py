"""Diagnostic (CPU): numpy emulation of the k_elements tangency solve
(cone_point + one Newton step, MODEL_SPEC 4.3) for a few elements of the
bench geometry: the |dth| / |dt| sequence of the joint 2-D step and of the
envelope step (lfg_device.hpp tangency_step).  python tools/newton_emul.py"""
import numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle.oracle import Oracle
O=Oracle()
q=0.1037; dphi=0.0392
inc=O.findi(q,dphi); s,c=np.sin(np.radians(inc)),np.cos(np.radians(inc))
xl1=O.xl1(q); cA=2/(1+q); cB=q*cA; mu=q/(1+q)
def pot(x,y,z): return -cA/np.sqrt(x*x+y*y+z*z)-cB/np.sqrt((x-1)**2+y*y+z*z)-(x-mu)**2-y*y
pl1=pot(xl1,0,0); Rs=1-xl1
def cone_point(P,cs,sn,t):
    Px,Py,Pz=P; ex,ey=s*cs,-s*sn
    x,y,z=Px+t*ex,Py+t*ey,Pz+t*c
    r1s=x*x+y*y+z*z; ir1=1/np.sqrt(r1s); ir1s=ir1*ir1
    dx=x-1; r2s=dx*dx+y*y+z*z; ir2=1/np.sqrt(r2s); ir2s=ir2*ir2
    i1=cA*ir1s*ir1; i2=cB*ir2s*ir2; i12=i1+i2; xm=x-mu
    phi=-cA*ir1-cB*ir2-xm*xm-y*y
    gx=i1*x+i2*dx-2*xm; gy=(i12-2)*y; gz=i12*z
    p1=x*ex+y*ey+z*c; p2=p1-ex; q1=x*ey-y*ex; q2=q1-ey
    k1=3*i1*ir1s; k2=3*i2*ir2s; s2=ex*ex+ey*ey
    F2=gx*ex+gy*ey+gz*c; gth=gx*ey-gy*ex
    eHe=i12-k1*p1*p1-k2*p2*p2-2*s2; etHe=-k1*p1*q1-k2*p2*q2
    return phi,gth,F2,eHe,etHe,r2s
def solve(P,th,t,ingress,n=8):
    out=[]
    for it in range(n):
        phi,gth,F2,eHe,etHe,r2s=cone_point(P,np.cos(th),np.sin(th),t)
        F1=phi-pl1; J11=t*gth; J12=F2; J21=t*etHe+gth; J22=eHe
        det=J11*J22-J12*J21
        dth=-(F1*J22-F2*J12)/det; dt=-(J11*F2-J21*F1)/det
        dth=min(max(dth,-0.05),0.05)
        th+=dth; t+=dt; out.append((abs(dth),abs(dt)))
        if max(abs(dth),abs(dt))<=3e-8: break
    return th,t,out
Rcal=None
# Rcal as in setup: sqrt(1-sce^2), sce = s cos(pi dphi)
sce=s*np.cos(np.pi*dphi); Rcal=np.sqrt(1-sce*sce)
def guess(P):
    ux,uy,uz=1-P[0],-P[1],-P[2]; uxy2=ux*ux+uy*uy; uu=uxy2+uz*uz; iuxy=1/np.sqrt(uxy2); uxy=uxy2*iuxy
    cc,sc=ux*iuxy,-uy*iuxy
    ce=(np.sqrt(max(uu-Rcal*Rcal,0))-c*uz)*iuxy/s
    se=np.sqrt(1-ce*ce); thc=np.arctan2(-uy,ux); de=np.arccos(ce)
    ci,si=cc*ce+sc*se, sc*ce-cc*se; co,so=cc*ce-sc*se, sc*ce+cc*se
    return (thc-de, s*(ux*ci-uy*si)+uz*c), (thc+de, s*(ux*co-uy*so)+uz*c)
rwd=0.0187*xl1; rdisc=0.2953*xl1
for name,P in [('wd center',(0,0,0)),('wd limb',(0,rwd,0)),('disc r.1',(0.1*np.cos(1),0.1*np.sin(1),0)),('disc rim',(rdisc*np.cos(2),rdisc*np.sin(2),0)),('disc rim2',(rdisc*np.cos(-0.5),rdisc*np.sin(-0.5),0))]:
    (ti,tti),(to,tto)=guess(P)
    thi,tfi,oi=solve(P,ti,tti,True); tho,tfo,oo=solve(P,to,tto,False)
    print(name,'in: guess err th %.1e t %.1e steps %d'%(abs(ti-thi),abs(tti-tfi),len(oi)),['%.0e/%.0e'%x for x in oi])
    print(name,'out: guess err th %.1e t %.1e steps %d'%(abs(to-tho),abs(tto-tfo),len(oo)),['%.0e/%.0e'%x for x in oo])
print('--- envelope steps')
def solve2(P,th,t,n=8,tol=3e-8):
    out=[]
    for it in range(n):
        phi,gth,F2,eHe,etHe,r2s=cone_point(P,np.cos(th),np.sin(th),t)
        F1=phi-pl1; J11=t*gth; J21=t*etHe+gth; J22=eHe
        dt0=-F2/J22
        F1m=F1-F2*F2/(2*J22)
        # dg/dth at the minimising t: J11 evaluated at t+dt0 ~ J11 + J21*dt0
        dth=-F1m/(J11+J21*dt0)
        dth=min(max(dth,-0.05),0.05)
        dt=dt0-(J21/J22)*dth
        th+=dth; t+=dt; out.append((abs(dth),abs(dt)))
        if max(abs(dth),abs(dt))<=tol: break
    return th,t,out
for name,P in [('wd center',(0,0,0)),('wd limb',(0,rwd,0)),('disc r.1',(0.1*np.cos(1),0.1*np.sin(1),0)),('disc rim',(rdisc*np.cos(2),rdisc*np.sin(2),0)),('disc rim2',(rdisc*np.cos(-0.5),rdisc*np.sin(-0.5),0))]:
    (ti,tti),(to,tto)=guess(P)
    thi,_,oi=solve(P,ti,tti,True,20); tho,_,oo=solve(P,to,tto,False,20)
    a,_,oa=solve2(P,ti,tti); b,_,ob=solve2(P,to,tto)
    print(name,'in steps %d err %.1e'%(len(oa),abs(a-thi)),['%.0e/%.0e'%x for x in oa])
    print(name,'out steps %d err %.1e'%(len(ob),abs(b-tho)),['%.0e/%.0e'%x for x in ob])
