"""Block structure of the payloads a Beast peer sends (host zlib = Beast's
deflate_stream at L1/L6, memLevel 4, pmd framing): block types, symbols per
block, output bytes per block -- a plain-Python walk of the DEFLATE stream
(RFC 1951), for DESIGN.md 4.1d.  CPU only.
    python scripts/beast_blocks.py
"""
import sys, zlib, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from beast_amd import synth

class BR:
    def __init__(s, b): s.b=b; s.p=0
    def bits(s, n):
        v=0
        for i in range(n):
            byte=s.b[s.p>>3]; v|=((byte>>(s.p&7))&1)<<i; s.p+=1
        return v
def build(lens):
    # canonical decode dict: (len, code) -> sym
    mx=max(lens); bl=[0]*(mx+1)
    for l in lens:
        if l: bl[l]+=1
    code=0; nxt=[0]*(mx+2)
    for b in range(1,mx+1):
        code=(code+bl[b-1])<<1; nxt[b]=code
    d={}
    for sym,l in enumerate(lens):
        if l: d[(l,nxt[l])]=sym; nxt[l]+=1
    return d
def dec(br,d):
    c=0
    for l in range(1,16):
        c=(c<<1)|br.bits(1)
        if (l,c) in d: return d[(l,c)]
    raise ValueError
LB=[3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE=[0]*8+[1]*4+[2]*4+[3]*4+[4]*4+[5]*4+[0]
DB=[1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DE=[0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
FIXL=build([8]*144+[9]*112+[7]*24+[8]*8); FIXD=build([5]*30)
def blocks(p):
    br=BR(p+b'\x00\x00\xff\xff'); out=[]; n=len(p)*8
    while br.p < n:
        start=br.p; fin=br.bits(1); t=br.bits(2)
        if t==0:
            br.p=(br.p+7)&~7; L=br.bits(16); br.bits(16); br.p+=8*L; out.append((start,'S',L,L)); 
        else:
            if t==1: dl,dd=FIXL,FIXD
            else:
                hl=br.bits(5)+257; hd=br.bits(5)+1; hc=br.bits(4)+4
                order=[16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]; cl=[0]*19
                for i in range(hc): cl[order[i]]=br.bits(3)
                cd=build(cl); lens=[]
                while len(lens)<hl+hd:
                    s=dec(br,cd)
                    if s<16: lens.append(s)
                    elif s==16: r=3+br.bits(2); lens+= [lens[-1]]*r
                    elif s==17: lens+=[0]*(3+br.bits(3))
                    else: lens+=[0]*(11+br.bits(7))
                dl=build(lens[:hl]); dd=build(lens[hl:])
            nsym=0; ob=0
            while True:
                s=dec(br,dl); nsym+=1
                if s==256: break
                if s<256: ob+=1
                else:
                    i=s-257; ob+=LB[i]+br.bits(LE[i]); ds=dec(br,dd); br.bits(DE[ds])
            out.append((start,'F' if t==1 else 'D',nsym,ob))
        if fin: break
    return out
for kind,level in (('binary',1),('binary',6),('json',6)):
    raw,off,ln=synth.make_batch(kind,np.full(4,65536,np.uint32),seed=0x5EED0005)
    for i in range(2):
        m=bytes(raw[off[i]:off[i]+ln[i]])
        c=zlib.compressobj(level,zlib.DEFLATED,-15,4); p=c.compress(m)+c.flush(zlib.Z_BLOCK)+c.flush(zlib.Z_SYNC_FLUSH); p=p[:-4]
        bl=blocks(p)
        from collections import Counter
        print(kind,level,len(p), Counter(b[1] for b in bl), 'syms', Counter(b[2] for b in bl if b[1]!='S').most_common(3), 'bytes/blk', np.mean([b[3] for b in bl]))
        print('   first', bl[:6])
