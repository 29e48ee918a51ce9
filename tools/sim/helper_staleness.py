"""Estimate for VERDICT r05 item 1(a) (a helper wave preparing the next
compress window's candidates while the walker finishes the current one):
how often the table snapshot a helper would read one window ahead is stale
when the walker gets there.  A plain-Python greedy LZ4 parse (byU16-style
13-bit hash of 5 bytes, acceleration 1) of text-proxy 64 KiB blocks records
its puts; a window's lanes whose hash a put of the previous window changed
would need their candidate re-gathered.  CPU only, no GPU, no reference.

usage: python tools/sim/helper_staleness.py"""
import sys
sys.path.insert(0,'lz4-sgori_amd')
from lz4e_amd import corpus
import numpy as np
def h(buf,p):
    v=int.from_bytes(buf[p:p+8],'little')
    return (((v<<24)&0xFFFFFFFFFFFFFFFF)*889523592379 & 0xFFFFFFFFFFFFFFFF)>>(64-13)
def parse(buf):
    n=len(buf); mflimit=n-12; matchlimit=n-5
    T=[0]*8192
    puts=[]   # (pos) in order
    ip=1; anchor=0
    T[h(buf,0)]=0; puts.append(0)
    events=[]
    while True:
        # search
        step=1; nb=1<<6; fwd=ip
        found=None
        while True:
            p=fwd; step=nb>>6; nb+=1; fwd=p+step
            if fwd>mflimit: return puts
            hh=h(buf,p); c=T[hh]; T[hh]=p; puts.append(p)
            if c+65535>=p and buf[c:c+4]==buf[p:p+4] and c!=p: found=(p,c); break
        p,c=found
        while p>anchor and c>0 and buf[p-1]==buf[c-1]: p-=1;c-=1
        while True:
            ml=4
            while p+ml<matchlimit and buf[p+ml]==buf[c+ml]: ml+=1
            e=p+ml; anchor=e
            if e>mflimit: return puts
            T[h(buf,e-2)]=e-2; puts.append(e-2)
            hh=h(buf,e); c=T[hh]; T[hh]=e; puts.append(e)
            if c+65535>=e and buf[c:c+4]==buf[e:e+4]: p=e; continue
            ip=e+1; break
    return puts
for kind,gen in (("text",lambda s: corpus.text_proxy(65536,s)),):
  for seed in (1,2,3):
    buf=bytes(gen(seed)); puts=parse(buf)
    # windows: cut the put stream at positions crossing multiples of 64 from the walk
    # window w covers positions [B, B+64); staleness: a put during window w (positions in [B,B+64)) to a hash that some position in [B+64,B+128) looks up
    n=len(buf); W=64; stale=0; tot=0; lanes=0
    hs=[h(buf,p) if p+8<=n else -1 for p in range(n)]
    byw={}
    for p in puts: byw.setdefault(p//W,set()).add(hs[p])
    for w in range(0,n//W-2):
        ph=byw.get(w,set())
        nxt=[hs[p] for p in range((w+1)*W,(w+2)*W)]
        k=sum(1 for x in nxt if x in ph)
        tot+=1; stale+= k>0; lanes+=k
    print(kind,seed,'windows',tot,'frac windows with a stale lane %.2f'%(stale/tot),'stale lanes/window %.2f'%(lanes/tot), 'puts/window %.1f'%(len(puts)/tot))
