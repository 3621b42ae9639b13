"""CPU model of the bank-placed R6 claim (dprf_kernels_r6.hip r6_claim_placed, R6_BANK_PLACE, an A/B option measured
slower and off by default): the dual-mask prefix scan over the class bitmap words, the first two queued slots of each
bank residue on lanes b / 32 + b, further slots on the free lanes by the uniform walk.  Checks that every slot the
claim got -- with bits randomly lost to a racing wave -- is placed on exactly one lane and that no more than 64 are
taken, which is what the flow scheduler's termination argument needs."""
import random

import random
def popc(x): return bin(x).count('1')
def claim(words, lost_rng=None):
    """returns (slots taken, LDS cycles of one period read: the largest bank multiplicity of each half)"""
    L=64; W=len(words)
    w=[words[k] if k<W else 0 for k in range(L)]
    s1=[0]*L; s2=[0]*L
    a1=0;a2=0
    for k in range(L):
        a2 = a2 | (a1 & w[k]); a1 = a1 | w[k]; s1[k]=a1; s2[k]=a2
    e1=[0]+s1[:-1]; e2=[0]+s2[:-1]
    r0=[w[k]&~e1[k] for k in range(L)]; r1=[w[k]&e1[k]&~e2[k] for k in range(L)]; ov=[w[k]&e2[k] for k in range(L)]
    room=64-sum(popc(r0[k]|r1[k]) for k in range(L))
    inc=0; tov=[0]*L
    for k in range(L):
        pco=popc(ov[k]); inc+=pco
        if inc<=room: tov[k]=ov[k]
        elif inc-pco<room:
            rest=ov[k]
            for _ in range(room-(inc-pco)):
                tov[k]|=rest&-rest; rest&=rest-1
    take=[(r0[k]|r1[k]|tov[k]) & 0xffffffff for k in range(L)]
    got=[]
    for k in range(L):
        g=take[k]
        if lost_rng:
            for b in range(32):
                if (g>>b)&1 and lost_rng.random()<0.1: g&=~(1<<b)
        got.append(g)
    stage=[None]*64
    g0=[got[k]&r0[k] for k in range(L)]; g1=[got[k]&r1[k] for k in range(L)]; gov=[got[k]&tov[k] for k in range(L)]
    total=sum(popc(g) for g in got)
    for k in range(L):
        b=g0[k]
        while b:
            r=(b&-b).bit_length()-1; assert stage[r] is None; stage[r]=32*k+r; b&=b-1
        b=g1[k]
        while b:
            r=(b&-b).bit_length()-1; assert stage[32+r] is None; stage[32+r]=32*k+r; b&=b-1
    u0=0;u1=0
    for k in range(L): u0|=g0[k]; u1|=g1[k]
    fr=~((u1<<32)|u0) & ((1<<64)-1)
    novt=sum(popc(g) for g in gov)
    jpref=[];acc=0
    for k in range(L): jpref.append(acc); acc+=popc(gov[k])
    rest=list(gov); j=list(jpref)
    for kk in range(novt):
        p=(fr&-fr).bit_length()-1; fr&=fr-1
        for k in range(L):
            if rest[k] and j[k]==kk:
                assert stage[p] is None
                r=(rest[k]&-rest[k]).bit_length()-1; stage[p]=32*k+r; rest[k]&=rest[k]-1; j[k]+=1
    placed=[x for x in stage if x is not None]
    gotids=sorted(32*k+b for k in range(L) for b in range(32) if (got[k]>>b)&1)
    assert sorted(placed)==gotids, (len(placed), len(gotids))
    assert total==len(gotids)<=64
    # conflicts: max multiplicity per half
    cyc=0
    for h in (0,1):
        from collections import Counter
        c=Counter(x%32 for x in stage[32*h:32*h+32] if x is not None)
        cyc+=max(c.values()) if c else 0
    return total,cyc


def test_every_slot_taken_is_placed_once():
    rng = random.Random(5)
    for it in range(1500):
        q = rng.randint(1, 200)
        words = [0] * 34
        for i in rng.sample(range(1088), q):
            words[i // 32] |= 1 << (i % 32)
        total, cyc = claim(words, rng if it % 3 == 0 else None)
        assert total <= 64 and (total > 0 or it % 3 == 0)
        assert cyc <= 2 * total
