"""Would decoding the linked 64 KiB blocks of a pyarrow LZ4 frame in
parallel (8x the streams) pay off?  A block decoded without its history
must defer every match reaching before its start, and every later match
whose source overlaps deferred bytes (taint), to a serial fix-up pass.
This replays each block's sequences on the CPU and reports the deferred
fraction (profiles/r2/dec/SUMMARY.md: 47 % for the config-5 val column,
1.4 % for sorted ids, 100 % for text -> not built).

``python tools/lz4_block_split_sim.py``
"""
import numpy as np, pyarrow as pa, struct, sys
sys.path.insert(0,'/root/repo')
from nvme_strom_amd.ops import decompress as D
def blocks_of(f):
    info=D.parse_lz4_frame_header(f); p=info.data_offset; out=[]
    while True:
        bs,=struct.unpack_from("<I",f,p); p+=4
        if bs==0: break
        st=bs>>31; bs&=0x7fffffff
        out.append((st, f[p:p+bs])); p+=bs+(4 if info.block_checksum else 0)
    return out
def seqs(b):
    q=0; e=len(b); res=[]
    while q<e:
        t=b[q];q+=1; lit=t>>4; ml=t&15
        if lit==15:
            while True:
                x=b[q];q+=1;lit+=x
                if x!=255: break
        q+=lit
        if q>=e: res.append((lit,0,0)); break
        off=b[q]|b[q+1]<<8;q+=2
        if ml==15:
            while True:
                x=b[q];q+=1;ml+=x
                if x!=255: break
        res.append((lit,off,ml+4))
    return res
for name, gen in [("val", lambda r: r.integers(0,1_000_000,65536,dtype=np.int64).tobytes()),
                  ("sorted", lambda r: np.cumsum(r.integers(0,4096,65536)).astype(np.int64).tobytes()),
                  ("text", None)]:
    rng=np.random.default_rng(3)
    if gen is None:
        words=[b"select",b"from",b"where",b"gpu",b"hbm",b"nvme",b"strom",b"table",b"index",b"scan"]
        raw=b" ".join(words[i] for i in rng.integers(0,len(words),120000))[:512<<10]
    else:
        raw=gen(rng)
    f=pa.compress(raw,codec="lz4",asbytes=True)
    tot=0; dfr=0; tainted_bytes=0; nblk=0
    for st,b in blocks_of(f)[1:]:
        nblk+=1
        if st: continue
        taint=np.zeros(65536+1024,dtype=bool); op=0
        for lit,off,m in seqs(b):
            op+=lit; tot+=1
            if m:
                s=op-off
                if s<0 or taint[max(s,0):max(s,0)+min(m,off)].any() or (s<0):
                    dfr+=1; taint[op:op+m]=True
                op+=m
        tainted_bytes+=taint[:op].sum()
    print(name, "ratio %.2f"%(len(raw)/len(f)), "blocks", nblk, "seqs", tot, "deferred %.3f"%(dfr/max(tot,1)), "tainted bytes %.3f"%(tainted_bytes/(nblk*65536)))
