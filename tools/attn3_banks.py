import collections
G128=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32)),
      list(range(32,36))+list(range(44,48))+list(range(52,60)), list(range(36,44))+list(range(48,52))+list(range(60,64))]
H32=[list(range(32)),list(range(32,64))]
def cyc(groups, addr, nbytes):
    tot=0
    for grp in groups:
        cnt=collections.Counter()
        for l in grp:
            a=addr(l)
            for d in range(nbytes//4): cnt[(a//4+d)%64]+=1
        tot+=max(cnt.values())
    return tot
def evaluate(R):
    s=cyc(G128, lambda l: (l&15)*R + 16*(l>>4), 16)           # ideal 4
    t=cyc(H32, lambda l: (l&15)*R + 8*(l>>4), 8)                # tail b64, ideal 2
    o=cyc(H32, lambda l: (4*(l>>4)+((l&15)>>2))*R + 8*(l&3), 8) # tr lo, ideal 2
    o2=cyc(H32, lambda l: (16+4*(l>>4)+((l&15)>>2))*R + 8*(l&3), 8)
    return s,t,o,o2
for DP in (400,208):
    base=6*DP
    res=[]
    for pad in range(0,1025,16):
        R=base+pad
        res.append((sum(evaluate(R)),pad,evaluate(R)))
    res.sort()
    print(DP, res[:6], 'pad16:', evaluate(base+16))
print()
for DB in (1,2,4,8,13,16,25):
    DP=16*DB; NK=DP//32; TAIL=(DP%32)//16
    best=None
    for pad in range(0,1025,16):
        s,t,o,o2=evaluate(6*DP+pad)
        cost=s*2*NK*3+t*2*3*TAIL+(o+o2)*3*DB
        ideal=4*2*NK*3+2*2*3*TAIL+4*3*DB
        if best is None or cost<best[0]: best=(cost,pad,ideal,(s,t,o,o2))
    print(DB, best)
