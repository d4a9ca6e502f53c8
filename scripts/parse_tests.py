"""C4-shaped JSON: how the parse's chain-walk candidate tests end (rejected outright / byte run
to extend / short improvement), a sequential restatement of the walk with the level-6 limits
(several candidates per iteration)."""
import sys
sys.path.insert(0,'/root/repo')
from beast_amd import synth
raw, off, ln = synth.make_batch('json', synth.zipf_sizes(4096, 0x5EED0004), seed=0x5EED0004)
tests=0; rej=0; gom=0; impr_short=0
for i in range(len(ln)):
    if ln[i] < 16384: continue
    m = raw[int(off[i]):int(off[i])+int(ln[i])].tobytes()
    for base in range(4096, len(m)-4096, 4096*3):
        w = m[base-2048: base+4096]; wn=len(w)
        head={}; prev=[-1]*wn
        for q in range(wn-3):
            h=((int.from_bytes(w[q:q+4],'little')*0x9E3779B1)&0xffffffff)>>21
            prev[q]=head.get(h,-1); head[h]=q
        # approximate: a find at every 3rd position of the chunk, thr=2, chain 32, good 8 nice 128
        for q in range(2048, wn-3, 3):
            best=2; c=prev[q]; n=32; maxl=min(258, wn-q)
            while c>=0 and n>0:
                n-=1; tests+=1
                if best<maxl and w[c+best]==w[q+best]:
                    k=0
                    while k<8 and q+k<wn and w[c+k]==w[q+k]: k+=1
                    if k==8 and maxl>8:
                        gom+=1
                        l=8
                        while l<maxl and w[c+l]==w[q+l]: l+=1
                        if l>best: best=l
                        if best>=128: break
                    elif k>0:
                        if k>best: best=k; impr_short+=1
                        else: rej+=1
                    else: rej+=1
                else: rej+=1
                c=prev[c]
    if tests>3e5: break
print(f"tests {tests}: rejected w/o extension {rej/tests:.1%}, extension {gom/tests:.1%}, short improvements {impr_short/tests:.1%}")
