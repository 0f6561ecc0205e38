"""Per-query K5 workload statistics on the seeded D1 corpus (DESIGN.md §4 K5 as measured): tokens,
columns, token entries and (candidate, column) hit pairs per candidate, common columns, segment
lengths per (list, 512-candidate block).  usage: python tools/k5_query_stats.py"""
import sys, time, ctypes, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
import synth
from cfg4_sharing import Desc, arr
t0=time.time()
c=synth.Corpus(n_users=1632803, seed=1, edge_cases=0, threads=16)
d=Desc.from_address(c.desc_ptr()); n,T=d.n_users,d.n_cols
tok_off=arr(d.tok_off,n*T+1,np.int64); tid=arr(d.tok_tid,int(tok_off[-1]),np.int32); tf=arr(d.tok_tf,int(tok_off[-1]),np.int32)
rowlen=np.diff(tok_off).reshape(n,T)
colmask=(rowlen>0)
row_user=np.repeat(np.arange(n*T)//T, np.diff(tok_off)); row_col=np.repeat(np.arange(n*T)%T, np.diff(tok_off))
keep=tf>0
key=(row_col[keep].astype(np.int64)<<32)|tid[keep]
users=row_user[keep]
order=np.argsort(key,kind='stable'); key_s=key[order]; users_s=users[order]
uk,start,cnt=np.unique(key_s,return_index=True,return_counts=True)
print('corpus',time.time()-t0,'tokens',len(key),'lists',len(uk),flush=True)
rng=np.random.default_rng(2)
qs=rng.integers(1,n+1,size=24)
B=512
for qu in qs:
    i=qu-1
    qk=[]
    for t in range(T):
        s,e=tok_off[i*T+t],tok_off[i*T+t+1]
        for x in range(s,e):
            if tf[x]>0: qk.append((t<<32)|int(tid[x]))
    qk=np.unique(np.array(qk,dtype=np.int64))
    pos=np.searchsorted(uk,qk)
    segs=[users_s[start[p]:start[p]+cnt[p]] for p in pos]
    ent=np.concatenate(segs); cols=np.concatenate([np.full(len(s),k>>32) for s,k in zip(segs,qk)])
    E=len(ent)
    qmask=colmask[i]
    common=(colmask & qmask).sum(1)
    hitpair=np.unique(ent.astype(np.int64)*64+cols)
    hits_per_cand=np.bincount(ent,minlength=n)
    blk=ent//B
    # lists per block with >0 entries
    lb=np.unique((np.repeat(np.arange(len(segs)),[len(s) for s in segs]).astype(np.int64)<<22)|blk)
    print(f'q{qu}: toks {len(qk)} cols {qmask.sum()} entries {E} ({E/n:.2f}/cand) hitpairs {len(hitpair)} ({len(hitpair)/n:.2f}/cand) common-cols {common.mean():.2f}/cand maxhits {hits_per_cand.max()} p99hits {np.percentile(hits_per_cand,99):.0f} nonempty(list,blk) {len(lb)} ({len(lb)/(n/B):.1f}/blk, {E/len(lb):.1f} ent/seg) maxlist {max(len(s) for s in segs)}',flush=True)
