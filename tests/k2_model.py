"""Executable model of K2's decomposition (metacov_amd/csrc/kernels.h,
depth_kernel + ingest_kernel's chunk index + long_count/long_fill kernels), in numpy.

TEST INFRASTRUCTURE: it checks the ALGORITHM (chunks of 16 tiles of 4096
positions, an 8192-slot ring, the max-span halo, long-read end events as a
chunk-relative stream in tile order, per-chunk carries and the halo
tightened to the first crossing read) against the
oracle on the CPU, so that decomposition
bugs show up without a GPU.  Constants must match kernels.h.
"""
import numpy as np
from oracle import coracle
W=4096; TPC_MAX=8; RING=8192; SM=RING-W
GB=18; GMASK=(1<<GB)-1; SCAP=(1<<(32-GB))-1   # K2's read words (kernels.h MC_GPOS 2)


def read_words(gs, span):
    """ingest_kernel's read words: low GB bits of the global start, span
    capped at SCAP above them."""
    return (gs & GMASK) | (np.minimum(span, SCAP).astype(np.int64) << GB)


def decode(word, C0):
    """finish_batch: chunk-relative start (sign-extended GB-bit difference)
    and capped span."""
    d = (int(word) - (C0 & GMASK)) & GMASK
    return (d - (1 << GB) if d >= 1 << (GB - 1) else d), int(word) >> GB


def tiles_per_chunk(G):
    """engine.hip mc_prepare: halve the chunk while it leaves < 2048 chunks."""
    tiles = max(1, (G + W - 1) // W)
    tpc = TPC_MAX
    while tpc // 2 >= RING // W and tpc % 2 == 0 and tiles // tpc < 2048:
        tpc //= 2
    return tpc

def model(lengths, tid, pos, span, origin=0):
    """origin: a multiple of the chunk width added to every global position
    the read words see (as a genome past 2^32 would), the depth unchanged."""
    ext, coff64 = coracle.layout(lengths, tid, pos, span)
    coff=np.zeros(len(ext)+1,np.int64); 
    for i in range(len(ext)): coff[i+1]=coff[i]+ (ext[i]+63)//64*64
    G=coff[-1]; TPC=tiles_per_chunk(G); CW=W*TPC
    nch=max(1,(G+CW-1)//CW); alloc=nch*CW
    gs=coff[tid]+pos; ge=gs+span
    ms=span.max() if len(span) else 0; halo=min(ms,SM)
    long_=span>SM
    # events: chunk-relative end positions, grouped by tile (long_fill_kernel)
    ev={}
    cdiff=np.zeros(nch+1,np.int64)
    for a,b in zip(gs[long_],ge[long_]):
        if b<alloc and b%CW: ev.setdefault(b//CW,[]).append((b//W, b-(b//CW)*CW))
        c0=a//CW+1; c1=(b-1)//CW+1
        if c1>c0: cdiff[c0]+=1; cdiff[c1]-=1
    carry_c=np.cumsum(cdiff)[:nch]
    # chunk index as ingest_kernel builds it in its one pass over the reads:
    # F[m] = first read starting at or after m*BW (a store at the read where
    # m*BW falls between two starts), X[m] = first short read crossing m*BW
    BTPC=4 if TPC>4 and TPC%4==0 else TPC; BW=W*BTPC; S=TPC//BTPC; NB=nch*S
    F=np.full(NB+1,len(gs),np.int64); F[0]=0; Xidx=np.full(NB+1,np.iinfo(np.int64).max,np.int64)
    prev=-1
    for i in range(len(gs)):
        for m in range((prev//BW+1) if prev>=0 else 1, min(gs[i]//BW, NB)+1): F[m]=i
        mb=gs[i]//BW+1
        if 0<span[i]<=SM and mb<NB and ge[i]>mb*BW: Xidx[mb]=min(Xidx[mb],i)
        prev=gs[i]
    def ref_first(C0):
        # the definition it replaces: the first read of the max-span halo that
        # crosses C0 (short reads), else the first read starting at or after C0
        f=np.searchsorted(gs, C0-halo, 'left')
        while f<len(gs) and not (gs[f]>=C0 or (span[f]<=SM and ge[f]>C0)):
            f+=1
        return f
    depth=np.zeros(alloc,np.int64)
    for c in range(nch):
        C0=c*CW
        # ingest_kernel's index (base chunks of BW, a full chunk is S of them):
        # the first short read crossing C0, else the first read starting at or after C0
        b0=c*S
        first=0 if b0==0 else min(Xidx[b0], F[b0])
        assert first==ref_first(C0)
        exact=first
        first&=~3
        ring=np.zeros(RING,np.int64)
        i=first; carry=carry_c[c] if long_.any() else 0
        assert origin % CW == 0
        words=read_words(gs+origin, span)
        stream=[r for _, r in sorted(ev.get(c, []), key=lambda e: e[0])]   # tile order
        k=0
        for t in range(TPC):
            T0=C0+t*W; Tend=T0+W
            while k<len(stream) and stream[k]<(t+1)*W:   # applied while before the tile end
                ring[(C0+stream[k])&(RING-1)]-=1; k+=1
            while i<len(gs) and gs[i]<Tend:
                rs, sp = decode(words[i], C0+origin)
                if i<exact: i+=1; continue          # masked: before the chunk's first read
                assert rs==gs[i]-C0 and sp==min(span[i],SCAP)
                if sp<=SM:
                    s=max(rs,0); e=rs+sp
                    if e>s: ring[(C0+s)&(RING-1)]+=1; ring[(C0+e)&(RING-1)]-=1
                elif rs>=0: ring[(C0+rs)&(RING-1)]+=1
                i+=1
            sl=np.arange(T0,Tend)&(RING-1)
            vals=carry+np.cumsum(ring[sl]); ring[sl]=0
            depth[T0:Tend]=vals; carry=vals[-1]
    return depth, coff, ext
