# Least-squares fits of the f32 polynomial coefficients of the compat math spec v2
# (oracle/ref_math.h, sail_amd/csrc/sail_math.h); prints max ulp error of each candidate degree.
import numpy as np
from numpy.polynomial import chebyshev as C
def fit(f, lo, hi, deg, n=20000):
    # least squares in the variable u on [lo,hi], Chebyshev nodes, returns power-basis coefficients (ascending)
    k=np.arange(n); u=(lo+hi)/2+(hi-lo)/2*np.cos(np.pi*(k+0.5)/n)
    V=np.vander(u,deg+1,increasing=True)
    w=1/np.maximum(np.abs(f(u)),1e-30)  # relative error weighting
    c,*_=np.linalg.lstsq(V*w[:,None], f(u)*w, rcond=None)
    return c
def f32fma(a,b,c): return np.float32(np.float64(a)*np.float64(b)+np.float64(c))
# atan(t) = t + t^3 * P(t^2) on t in [0,1]  -> P(z) = (atan(sqrt z) - sqrt z)/ z^1.5
for deg in (6,7,8):
    c=fit(lambda z: (np.arctan(np.sqrt(z))-np.sqrt(z))/(z*np.sqrt(z)), 1e-6, 1.0, deg)
    c32=c.astype(np.float32)
    t=np.linspace(0,1,200001).astype(np.float32)[1:]
    z=(t*t).astype(np.float32)
    p=np.full_like(z,c32[-1])
    for ci in c32[-2::-1]: p=np.array([f32fma(a,b,ci) for a,b in zip(p[:0],z[:0])]) if False else (p.astype(np.float64)*z+ci).astype(np.float32)
    r=((t.astype(np.float64)*z)*p + t).astype(np.float32)
    err=np.abs(r.astype(np.float64)-np.arctan(t.astype(np.float64)))/np.spacing(np.arctan(t).astype(np.float32)).astype(np.float64)
    print('atan deg',deg,'max ulp',err.max(), [float(x) for x in c32])
# asin(x) = x + x^3 P(x^2), x in [0,0.5]
for deg in (4,5,6):
    c=fit(lambda z: (np.arcsin(np.sqrt(z))-np.sqrt(z))/(z*np.sqrt(z)), 1e-8, 0.25, deg)
    c32=c.astype(np.float32)
    x=np.linspace(0,0.5,200001).astype(np.float32)[1:]
    z=(x*x).astype(np.float32)
    p=np.full_like(z,c32[-1])
    for ci in c32[-2::-1]: p=(p.astype(np.float64)*z+ci).astype(np.float32)
    r=((x.astype(np.float64)*z)*p + x).astype(np.float32)
    err=np.abs(r.astype(np.float64)-np.arcsin(x.astype(np.float64)))/np.spacing(np.arcsin(x).astype(np.float32)).astype(np.float64)
    print('asin deg',deg,'max ulp',err.max(), [float(v) for v in c32])
# sin(r) = r + r^3 P(r^2), cos(r) = 1 - r^2/2 + r^4 Q(r^2) on |r|<=pi/4
for deg in (2,3,4):
    lim=(np.pi/4)**2
    c=fit(lambda z: (np.sin(np.sqrt(z))-np.sqrt(z))/(z*np.sqrt(z)), 1e-8, lim, deg)
    c32=c.astype(np.float32)
    x=np.linspace(0,np.pi/4,200001).astype(np.float32)[1:]
    z=(x*x).astype(np.float32)
    p=np.full_like(z,c32[-1])
    for ci in c32[-2::-1]: p=(p.astype(np.float64)*z+ci).astype(np.float32)
    r=((x.astype(np.float64)*z)*p + x).astype(np.float32)
    err=np.abs(r.astype(np.float64)-np.sin(x.astype(np.float64)))/np.spacing(np.sin(x).astype(np.float32)).astype(np.float64)
    c2=fit(lambda z: (np.cos(np.sqrt(z))-1+z/2)/(z*z), 1e-6, lim, deg)
    c232=c2.astype(np.float32)
    q=np.full_like(z,c232[-1])
    for ci in c232[-2::-1]: q=(q.astype(np.float64)*z+ci).astype(np.float32)
    zz=(z*z).astype(np.float32)
    rc=(zz.astype(np.float64)*q + (1-z.astype(np.float64)/2)).astype(np.float32)
    errc=np.abs(rc.astype(np.float64)-np.cos(x.astype(np.float64)))/np.spacing(np.cos(x).astype(np.float32)).astype(np.float64)
    print('sin/cos deg',deg,'max ulp',err.max(), errc.max(), [float(v) for v in c32], [float(v) for v in c232])
