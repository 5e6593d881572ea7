"""Node-level model of lego_wavesort.h's pipelined heap pops (round 6): levels 0-6 of the heap in
registers, the window below the level-6 path node read when a pop is issued and applied by the next pop
after that pop's register-only top path.  Checked against libstdc++ __sort_heap (restated: __adjust_heap,
__push_heap) on random keys with ties; asserts that no store lands in a pending window before it is
applied and that each pop's value a[len] is current when it is used.   python3 tools/analysis/heap_pipeline_model.py
"""
import random, sys
def lvl(n): return (n+1).bit_length()-1
def adjust(a,hole,ln,v):
    top=hole; second=hole
    while second<(ln-1)//2:
        second=2*(second+1)
        if a[second][0]<a[second-1][0]: second-=1
        a[hole]=a[second]; hole=second
    if (ln&1)==0 and second==(ln-2)//2:
        second=2*(second+1); a[hole]=a[second-1]; hole=second-1
    p=(hole-1)//2
    while hole>top and a[p][0]<v[0]:
        a[hole]=a[p]; hole=p; p=(hole-1)//2
    a[hole]=v
def ref(a):
    a=list(a); n=len(a)
    for p in range((n-2)//2,-1,-1): adjust(a,p,n,a[p])
    heap=list(a)
    for last in range(n-1,0,-1):
        v=a[last]; a[last]=a[0]; adjust(a,0,last,v)
    return heap,a
stats={"pops":0}
def model(heap):
    mem=list(heap); n=len(mem)
    top=mem[:63]; bot=mem[63:127]
    ln=n-1; pend=None
    def anc6(m): l=lvl(m); return ((m+1)>>(l-6))-1
    def subtree(x,hi):
        out=[]; st=[x]
        while st:
            q=st.pop()
            for ch in (2*q+1,2*q+2):
                if ch<=hi: out.append(ch); st.append(ch)
        return out
    def resolve():
        nonlocal pend
        b6,plen,pv,snap=pend; x6=63+b6
        for k,v in snap.items(): assert mem[k]==v, ("window changed before resolution",k)
        lim=(plen-1)//2; s=x6; path=[]
        while s<lim:
            c=2*(s+1)
            if mem[c][0]<mem[c-1][0]: c-=1
            path.append(c); s=c
        if (plen&1)==0 and s==(plen-2)//2: path.append(2*(s+1)-1)
        k=0
        while k<len(path) and not (mem[path[k]][0]<pv[0]): k+=1
        prev=x6
        for c in path[:k]:
            if prev==x6: bot[b6]=mem[c]
            else: mem[prev]=mem[c]
            prev=c
        if prev==x6: bot[b6]=pv
        else: mem[prev]=pv
        pend=None
        return prev
    cv=mem[ln]
    while ln>=255:
        stats["pops"]+=1
        path=[0]; s=0
        for L in range(5):
            c=2*(s+1)
            if top[c][0]<top[c-1][0]: c-=1
            path.append(c); s=c
        x5=s
        vk=cv
        if pend is not None:
            pv=pend[2]; h=resolve()
            if h==ln: vk=pv
        assert vk==mem[ln], "stale value"
        mem[ln]=top[0]
        cv=mem[ln-1]
        TM=[p for p in path[1:] if not (top[p][0]<vk[0])]
        c=2*(x5+1)
        if bot[c-63][0]<bot[c-1-63][0]: c-=1
        b6=c-63
        m6=(x5 in TM) and not (bot[b6][0]<vk[0])
        snap={q:mem[q] for q in subtree(63+b6,ln-1)} if m6 else None
        b6k=bot[b6]
        prev=0
        for p in TM: top[prev]=top[p]; prev=p
        if m6: top[x5]=b6k
        else: top[prev]=vk
        if m6: pend=(b6,ln,vk,snap)
        ln-=1
    if pend is not None:
        pv=pend[2]; h=resolve()
        if h==ln: cv=pv
    mem[:63]=top; mem[63:127]=bot
    assert cv==mem[ln]
    a=mem
    for last in range(ln,0,-1):
        v=a[last]; a[last]=a[0]; adjust(a,0,last,v)
    return a
random.seed(1)
for trial in range(400):
    n=random.choice([255,256,257,300,511,512,513,700,1000,1309,1500,2047,2048])
    d=random.choice([1,2,3,10,100,10**6])
    keys=[(random.randrange(d),i) for i in range(n)]
    heap,out=ref(keys)
    got=model(heap)
    assert got==out,(trial,n,d)
print("ok",stats)
