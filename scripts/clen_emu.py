import sys
sys.path.insert(0, "/root/repo")
from beast_amd import synth
from oracle import oracle as O
d,_,_ = synth.make_batch("json", [255], seed=1*100+4+255)
p = O.pmd_deflate(bytes(d[:255]), 1, 15, 4) + b"\x00\x00\xff\xff"
bits = int.from_bytes(p, "little")
total = len(p)*8
def get(pos, n): return (bits >> pos) & ((1<<n)-1)
pos = 0
hdr = get(pos,3); pos += 3
print("hdr", hdr)
nlen = get(pos,5)+257; ndist = get(pos+5,5)+1; ncode = get(pos+10,4)+4; pos += 14
order = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
cl = [0]*19
for i in range(ncode): cl[order[i]] = get(pos+3*i,3)
pos += 3*ncode
# canonical codes
codes = {}
code = 0
for L in range(1,8):
    for s in range(19):
        if cl[s] == L: codes[(L, code)] = s; code += 1
    code <<= 1
def rev(c, n): return int(bin(c)[2:].zfill(n)[::-1], 2)
def dec(at):
    for L in range(1,8):
        c = rev(get(at, L), L)
        if (L,c) in codes: return codes[(L,c)], L
    return None, 0
want = nlen + ndist
# serial
have=0; prev=0; cur=pos; lens=[]
while have < want:
    s, cb = dec(cur)
    if s < 16: lens.append(s); cur += cb; have += 1; prev = s
    else:
        xb = {16:2,17:3,18:7}[s]; x = get(cur+cb, xb)
        rep = (3 if s!=18 else 11) + x
        v = prev if s == 16 else 0
        lens += [v]*rep; have += rep; prev = v; cur += cb+xb
print("serial ok", have, want, cur)
# window-parallel emulation
have=0; prevlen=0; p2=pos; lens2=[]
while have < want:
    w = p2
    info=[]
    for lane in range(64):
        s, cb = dec(w+lane)
        xb = 0 if s < 16 else {16:2,17:3,18:7}[s]
        x = get(w+lane+cb, xb)
        step = cb if s < 16 else cb+xb
        info.append((s,cb,xb,x,step))
    J = [lane+info[lane][4] for lane in range(64)]
    R = [(1<<lane) | ((1<<J[lane]) if J[lane] < 64 else 0) for lane in range(64)]
    for k in range(6):
        newR = R[:]; newJ = J[:]
        for o in range(64):
            if J[o] < 64:
                newR[o] = R[o] | R[J[o]]; newJ[o] = J[J[o]]
        R, J = newR, newJ
    chain = R[0]
    members = [o for o in range(64) if (chain>>o)&1]
    hb = have
    stop=False
    for o in members:
        s,cb,xb,x,step = info[o]
        if hb >= want: break
        rep = 1 if s < 16 else (3+x if s==16 else (3 if s==17 else 11)+x)
        if s == 16 and hb == 0: print("err16"); stop=True; break
        if hb + rep > want: print("err over", o, s, hb, rep, want); stop=True; break
        v = s if s < 16 else (prevlen if s == 16 else 0)
        lens2 += [v]*rep; hb += rep; prevlen = v; p2 = w + o + step
    have = hb
    if stop: break
print("parallel", have, lens2 == lens, p2, cur)
