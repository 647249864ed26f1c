"""Numpy model of the D1M neighbour lists (cell geometry of csrc/mph_kernels.hip): per sampled
wavefront, the stencil-column window spans and the lane efficiency of column-by-column lockstep vs
ELL lockstep, for the compact-list experiment recorded in DESIGN.md section 4.  CPU only, ~5 min."""
import sys, numpy as np
sys.path.insert(0,'/root/repo')
from particlemethod_fsi_amd import cases
c = cases.get('d1m'); cfg, p = c.build()
x = p.position.copy(); n = len(x)
dx = 0.001; rc = 2.6*dx
lo = np.array(c.lower); hi = np.array(c.upper); W = hi-lo
gc = np.array([int(np.floor(W[d]/(0.5*rc*(1+1e-6)/(2 if d==2 else 1)))) for d in range(3)])
ginv = gc/W
cell = np.minimum(np.floor((x-lo)*ginv).astype(int), gc-1)
key = (cell[:,0]*gc[1]+cell[:,1])*gc[2]+cell[:,2]
order = np.lexsort((np.arange(n), key))
xs = x[order]; ks = key[order]; cs = cell[order]
ncell = gc.prod()
cnt = np.bincount(ks, minlength=ncell); start = np.concatenate([[0],np.cumsum(cnt)])
print('gc',gc,'n',n)
rcm2 = rc*rc*(1+4e-6); cw = 1/ginv
def lane_cols(i):
    u = xs[i]-lo; cx,cy,cz = cs[i]
    res=[]
    for col in range(25):
        dxc, dyc = col//5-2, col%5-2
        def gap(u,c,d,cw):
            g = (c+d)*cw-u if d>0 else (u-(c+d+1)*cw if d<0 else 0.0)
            return max(g,0.0)
        d2 = gap(u[0],cx,dxc,cw[0])**2+gap(u[1],cy,dyc,cw[1])**2
        if d2>rcm2 or not (0<=cx+dxc<gc[0] and 0<=cy+dyc<gc[1]): res.append((0,0,0)); continue
        ra=np.sqrt(rcm2-d2)
        lo_=max(int(np.floor((u[2]-ra)*ginv[2])), cz-2*2); hi_=min(int(np.floor((u[2]+ra)*ginv[2])), cz+2*2)
        lo_=max(lo_,0); hi_=min(hi_,gc[2]-1)
        base=((cx+dxc)*gc[1]+cy+dyc)*gc[2]
        jb,je=start[base+lo_],start[base+hi_+1]
        if je>jb:
            d = xs[jb:je]-xs[i]; acc = ((d*d).sum(1)<=rc*rc).sum() - (1 if jb<=i<je else 0)
        else: acc=0
        res.append((jb,je,acc))
    return res
rng = np.random.default_rng(0)
tiles = rng.choice(n//64, 300, replace=False)
spans=[]; fails=0; eff_col=[]; eff_pair=[]; tot=[]
pairs=[(0,0)]
for t in tiles:
    L=[lane_cols(i) for i in range(t*64,t*64+64)]
    A=np.array(L)  # 64 x 25 x 3
    ok=True; sc=0; mx_sum=0
    for col in range(25):
        jb,je,acc=A[:,col,0],A[:,col,1],A[:,col,2]
        m=je>jb
        if m.any():
            sp=je[m].max()-jb[m].min(); spans.append(sp)
            if sp>192 or (je-jb).max()>48: ok=False
        mx_sum+=acc.max()
    fails+= not ok
    tot_l=A[:,:,2].sum(1)
    eff_col.append(tot_l.mean()/mx_sum)
    eff_pair.append(tot_l.mean()/tot_l.max())
spans=np.array(spans)
print('fail frac',fails/len(tiles),'span mean',spans.mean(),'p90',np.percentile(spans,90),'max',spans.max())
print('efficiency column-lockstep',np.mean(eff_col),' ELL-lockstep',np.mean(eff_pair))
import itertools
As=[np.array([lane_cols(i) for i in range(t*64,t*64+64)]) for t in tiles[:150]]
def eff(groups):
    e=[]
    for A in As:
        acc=A[:,:,2]; tot=acc.sum(1)
        s=sum(acc[:,g].sum(1).max() for g in groups)
        e.append(tot.mean()/s)
    return np.mean(e)
cols=list(range(25))
print('single', eff([[c] for c in cols]))
print('mirror pairs', eff([[c,24-c] for c in range(12)]+[[12]]))
print('rows (same dxc)', eff([[5*a+b for b in range(5)] for a in range(5)]))
print('rows+mirror rows', eff([[5*a+b for b in range(5)]+[5*(4-a)+b for b in range(5)] for a in range(2)]+[[10+b for b in range(5)]]))
print('cols (same dyc)', eff([[5*a+b for a in range(5)] for b in range(5)]))
print('all', eff([cols]))
