"""How wide a fused-histogram window each C5 region needs (CPU analysis).

Regenerates the C5 workload with bench.py's generator on the CPU (torch's CPU
generator: the same distributions, not the same numbers as on the GPU), builds
each contig's exact depth, and reports how many whole-contig regions fall
outside the window the engine places ([body - 648, body + 216)) and how wide a
window their quartile ranks would need.

    python scripts/c5_window_need.py
"""
import sys, time, numpy as np, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from bench import config_contigs, device_workload
t0=time.time()
lengths, weights = config_contigs('c5', 50_000_000, 10_000)
tid, pos, span, counts = device_workload(torch, lengths, weights, 50_000_000, 1, torch.device('cpu'), long_reads=True)
tid=tid.numpy(); pos=pos.numpy(); span=span.numpy()
print('gen', time.time()-t0, flush=True)
nc=len(lengths)
S_mean = span.astype(np.float64).mean()
cb = np.bincount(tid, weights=span.astype(np.float64), minlength=nc)
cnt = np.bincount(tid, minlength=nc)
starts = np.concatenate([[0], np.cumsum(cnt)])
res=[]
for c in range(nc):
    L=int(lengths[c]); a,b=starts[c],starts[c+1]
    d=np.zeros(L+1,np.int64)
    np.add.at(d, pos[a:b], 1); np.add.at(d, pos[a:b]+span[a:b], -1)
    dep=np.cumsum(d[:L]); dep.sort()
    n=L
    qlo=dep[n//4]; qhi=dep[n-n//4-1]; mlo=dep[(n-1)//2]; mhi=dep[n//2]
    body = L - S_mean if L > 2*S_mean else L
    D = cb[c]/body
    res.append((L, cnt[c], D, qlo, mlo, mhi, qhi, dep[0], dep[-1]))
res=np.array(res,dtype=np.float64)
L,N,D,qlo,mlo,mhi,qhi,mn,mx = res.T
base = np.maximum(0, np.round(D) - 648)
fb = (qlo < base) | (qhi >= base+864) | (mlo<base) | (mhi>=base+864)
print('fallbacks current placement:', fb.sum(), 'span needed >864:', ((qhi-qlo)>=864).sum(), 'S_mean', S_mean)
print('fallback need widths:', np.sort(qhi[fb]-qlo[fb])[:50])
w = qhi - qlo
for t in [864, 1024, 1296, 1728, 2048, 3456]:
    print('regions needing a window of at least %d values: %d' % (t, (w >= t).sum()))
