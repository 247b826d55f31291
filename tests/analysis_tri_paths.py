"""Which probe path each vertex's count takes (k_tri_light hash sets, k_tri_heavy bitmaps, its hash sets or
the HBM search for out-lists past TH_NU), with the probes on each (analysis, not a test).
The classification restates k_tri_lclass's rule in numpy over analysis_tri_boundary.geometry.
python tests/analysis_tri_paths.py 24 [26]   (s26 needs ~30 GB of host memory and ~8 minutes)
"""
import sys, numpy as np, gc
sys.path.insert(0, str(__import__('pathlib').Path(__file__).resolve().parent))
from analysis_tri_boundary import geometry
s=int(sys.argv[1])
V,u,v,dplus,draw=geometry(s)
del draw; gc.collect()
pre=np.concatenate([[0],np.cumsum(dplus)])
M=len(u)
# suffix length per oriented edge, accumulated per target v (probes of v's items)
suf=(pre[u+1]-np.arange(M)-1).astype(np.int64)
probes_v=np.bincount(v,weights=suf,minlength=V)
del suf; gc.collect()
has=dplus>0
last=np.zeros(V,np.int64); last[has]=v[pre[1:][has]-1]
span=np.where(has,last-np.arange(V),0)
TH_DMAX,TH_HMIN,TH_NU=512,256,4096
BSPAN=(TH_NU//2)*128-32
heavy=(dplus>TH_DMAX)|((dplus>TH_HMIN)&(span<=BSPAN))
bitmap=heavy&(span<=BSPAN)
hashp=heavy&~bitmap&(dplus<=TH_NU)
search=heavy&~bitmap&(dplus>TH_NU)
tot=probes_v.sum()
print(f"s{s}: probes {tot/1e9:.2f}G heavy {probes_v[heavy].sum()/1e9:.2f}G: bitmap {probes_v[bitmap].sum()/1e9:.2f}G hash {probes_v[hashp].sum()/1e9:.2f}G HBM-search {probes_v[search].sum()/1e9:.2f}G; light {probes_v[~heavy].sum()/1e9:.2f}G")
print("heavy vertices",heavy.sum(),"bitmap",bitmap.sum(),"hash",hashp.sum(),"search",search.sum(), "max d+", dplus.max())
