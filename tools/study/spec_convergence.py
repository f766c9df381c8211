"""Convergence of a speculative start (equal metrics) to the true metric vector, in 96-stage groups, on
uniformly random SOFT8 input or BPSK codewords at a given Eb/N0 (tools only; numpy ACS).
Usage: python tools/study/spec_convergence.py <trials> random|<snr dB>"""
import numpy as np, sys
K=7; NS=64
par=lambda v: bin(v).count("1")&1
LAB=np.zeros((NS,2),dtype=np.int64); PRED=np.zeros((NS,2),dtype=np.int64)
for T in range(NS):
    for b in range(2):
        R=((T<<1)|b)&127
        LAB[T,b]=(par(R&0o171)<<1)|par(R&0o133); PRED[T,b]=((T&31)<<1)|b
def step(pm, a, b):
    bm=np.stack([-a-b,-a+b,a-b,a+b],axis=-1)  # (trials,4)
    cand=pm[:,PRED]+np.take_along_axis(bm[:,None,:].repeat(NS,1).reshape(len(a),NS,4), LAB.reshape(1,NS,2).repeat(len(a),0),axis=2)
    return cand.max(axis=2)
rng=np.random.default_rng(1)
trials=int(sys.argv[1]) if len(sys.argv)>1 else 400
kind=sys.argv[2] if len(sys.argv)>2 else "random"
L=96*12
if kind=="random":
    s=rng.integers(-128,128,(trials,L+1000,2))
else:
    # BPSK codeword at 2 dB quantised like the packer (scale 40)
    bits=rng.integers(0,2,(trials,L+1006))
    s=np.zeros((trials,L+1000,2),dtype=np.int64)
    sigma=np.sqrt(1/(2*0.5*10**(float(kind)/10)))
    for i in range(trials):
        reg=0
        for t in range(L+1000):
            reg=((reg>>1)|(int(bits[i,t])<<6))&127
            o0=par(reg&0o171); o1=par(reg&0o133)
            for c,o in enumerate((o0,o1)):
                x=(-1.0 if o else 1.0)+rng.normal()*sigma
                s[i,t,c]=min(127,max(-128,int(round(x*40))))
# true: start 1000 stages earlier from equal metrics; spec: equal metrics at t=1000
pm=np.zeros((trials,NS),dtype=np.int64)
for t in range(1000):
    pm=step(pm,s[:,t,0],s[:,t,1])
spec=np.zeros((trials,NS),dtype=np.int64)
first=np.full(trials,-1)
for t in range(1000,1000+L):
    pm=step(pm,s[:,t,0],s[:,t,1]); spec=step(spec,s[:,t,0],s[:,t,1])
    n=t-1000+1
    if n%96==0:
        eq=((pm-pm[:,:1])==(spec-spec[:,:1])).all(axis=1)
        newly=(first<0)&eq
        first[newly]=n
vals,cnts=np.unique(first,return_counts=True)
print(kind, "first group end (stages) with equal relative vectors:", dict(zip(vals.tolist(),cnts.tolist())))
