"""Diagnostic (CPU): step-count statistics of the tangency Newton variants
(joint 2-D step vs the envelope step, several stopping rules) on random
geometries, built on tools/newton_emul.py.  python tools/newton_stats.py"""
import numpy as np, sys
exec(open(__file__.replace('newton_stats.py', 'newton_emul.py')).read().split("rwd=0.0187")[0])
rng=np.random.default_rng(0)
def run(scheme, P, th, t, ingress, tolth=3e-8, tolt=3e-8):
    if scheme=='cur':
        for it in range(16):
            phi,gth,F2,eHe,etHe,r2s=cone_point(P,np.cos(th),np.sin(th),t)
            F1=phi-pl1; J11=t*gth; J12=F2; J21=t*etHe+gth; J22=eHe
            det=J11*J22-J12*J21
            dth=-(F1*J22-F2*J12)/det; dt=-(J11*F2-J21*F1)/det
            dth=min(max(dth,-0.05),0.05); th+=dth; t+=dt
            if max(abs(dth),abs(dt))<=3e-8: return th,it+1
    else:
        for it in range(16):
            phi,gth,F2,eHe,etHe,r2s=cone_point(P,np.cos(th),np.sin(th),t)
            F1=phi-pl1; J11=t*gth; J21=t*etHe+gth; J22=eHe
            dt0=-F2/J22; F1m=F1-F2*F2/(2*J22)
            dth=-F1m/(J11+J21*dt0); dth=min(max(dth,-0.05),0.05)
            dt=dt0-(J21/J22)*dth; th+=dth; t+=dt
            if abs(dth)<=tolth and abs(dt)<=tolt: return th,it+1
    return th,99
res={}
for trial in range(6):
    global q,dphi,inc,s,c,xl1,cA,cB,mu,pl1,Rs,Rcal
    q=np.exp(rng.uniform(np.log(0.05),np.log(0.4))); 
    mp=O.findphi(q,90.0); dphi=rng.uniform(0.5,0.95)*mp
    inc=O.findi(q,dphi); s,c=np.sin(np.radians(inc)),np.cos(np.radians(inc))
    xl1=O.xl1(q); cA=2/(1+q); cB=q*cA; mu=q/(1+q); pl1=pot(xl1,0,0); Rs=1-xl1
    sce=s*np.cos(np.pi*dphi); Rcal=np.sqrt(1-sce*sce)
    rwd=rng.uniform(0.01,0.03)*xl1; rdisc=rng.uniform(0.2,0.5)*xl1
    pts=[(r*np.cos(a),r*np.sin(a),0) for r in np.linspace(rwd,rdisc,8) for a in np.linspace(0.06,np.pi-0.06,12)]
    pts+= [(rwd*0.7*np.cos(a)*0+0, rwd*0.7*np.cos(a), rwd*0.7*np.sin(a)) for a in np.linspace(0,np.pi,8)]
    for P in pts:
        try: (ti,tti),(to,tto)=guess(P)
        except Exception: continue
        if not np.isfinite(ti): continue
        for (g,tg,ing) in ((ti,tti,True),(to,tto,False)):
            ref,_=run('cur',P,g,tg,ing)
            ref2,_=run('env',P,g,tg,ing,1e-15,1e-12)
            for key,args in [('cur',('cur',)),('env 3e-8/3e-8',('env',3e-8,3e-8)),('env 3e-8/1e-5',('env',3e-8,1e-5)),('env 1e-6/1e-4',('env',1e-6,1e-4)),('env 1e-7/1e-4',('env',1e-7,1e-4))]:
                th,n=run(args[0],P,g,tg,ing,*args[1:]) if len(args)>1 else run(args[0],P,g,tg,ing)
                res.setdefault(key,[]).append((n,abs(th-ref2)))
for k,v in res.items():
    n=np.array([x[0] for x in v]); e=np.array([x[1] for x in v])
    print('%-16s steps mean %.2f max %d  hist %s  max err %.1e'%(k,n.mean(),n.max(),np.bincount(n)[1:8],e.max()))
