# CPU check of k_ppush's index math: simulates its waves over random PK values and
# compares every P(i, l) and its first-minimum key with a brute-force scan; counts each term once.
# simulate k_ppush's index math in Python vs brute-force P with first-min keys
import random, itertools
def run(n, S=8, seed=1):
    rnd = random.Random(seed)
    PK = {}
    for i in range(1, n+1):
        for j in range(i, n+1):
            for k in range(j+2, n+1):
                for l in range(k, n+1):
                    PK[(i,j,k,l)] = rnd.randint(-50, 50)
    def cell(t, a, h, pos):
        m = n - t - 2
        assert 0 <= a <= t and 0 <= h < m and 1 <= pos <= m - h, (t,a,h,pos,m)
        i = pos; j = i + a; k = j + h + 2; l = k + (t - a)
        return PK[(i,j,k,l)]
    brute = {}
    for sg in range(3, n):
        for i in range(1, n - sg + 1):
            best = None
            for jo in range(0, sg):
                for do in range(jo+1, sg):
                    for ko in range(do+1, sg):
                        l = i + sg
                        v = PK[(i, i+jo, i+do+1, i+ko)] + PK[(i+jo+1, i+do, i+ko+1, l)]
                        key = (jo*sg+do)*sg+ko
                        if best is None or (v, key) < best: best = (v, key)
            if best: brute[(sg, i)] = best
    got = {}
    cnt = 0
    for lev in range(0, n-3):
        nmax = min(lev, n-4-lev) + 1
        if nmax <= 0: continue
        ngrp = (n - lev - 3 + 63)//64
        nch = (nmax + S - 1)//S
        mT = n - lev - 2
        for partB in (0, 1):
            for c in range(nch):
                for g in range(ngrp):
                    for outer in range(lev+1):
                        nother = (min(lev-1, n-4-lev) if partB else min(lev, n-4-lev)) + 1
                        o0 = c*S
                        if o0 >= nother: continue
                        ns = min(S, nother - o0)
                        for lane in range(64):
                            bv = [None]*S; bh=[0]*S
                            if not partB:
                                jo = outer; b1 = lev - jo; i = 1 + g*64 + lane
                                if 1 + g*64 > n - (lev+3+o0): break
                                iss = [min(i, n-(lev+3+min(o0+s,o0+ns-1))) for s in range(S)]
                                for h1 in range(0, o0+ns):
                                    va = cell(lev, jo, h1, min(i, mT-h1))
                                    for s in range(S):
                                        if s < ns and h1 <= o0+s:
                                            vb = cell(o0+s, h1, b1, iss[s]+jo+1)
                                            v = va+vb; cnt += (i + lev+3+o0+s <= n)
                                            if bv[s] is None or v < bv[s]: bv[s]=v; bh[s]=h1
                                for s in range(ns):
                                    sg = lev+3+o0+s
                                    if i + sg <= n and bv[s] is not None:
                                        dd = jo+1+bh[s]; ko = dd+1+b1
                                        key = (jo*sg+dd)*sg+ko
                                        got[(sg,i)] = min(got.get((sg,i),(10**9,0)), (bv[s], key))
                            else:
                                a2 = outer; l = lev+4+o0+g*64+lane
                                if lev+4+o0+g*64 > n: break
                                lc = min(l, n)
                                iss = [max(1, lc-(lev+3+min(o0+s,o0+ns-1))) for s in range(S)]
                                for h2 in range(o0+ns-1, -1, -1):
                                    vb = cell(lev, a2, h2, max(1, min(lc-h2-lev-2, mT-h2)))
                                    for s in range(S):
                                        if s < ns and h2 <= o0+s:
                                            va = cell(o0+s, o0+s-h2, a2, iss[s])
                                            v = va+vb; cnt += (l <= n and l-(lev+3+o0+s) >= 1)
                                            if bv[s] is None or v < bv[s]: bv[s]=v; bh[s]=h2
                                for s in range(ns):
                                    sg = lev+3+o0+s; i = l - sg
                                    if l <= n and i >= 1 and bv[s] is not None:
                                        jo = o0+s-bh[s]; dd = jo+1+a2; ko = dd+1+bh[s]
                                        key = (jo*sg+dd)*sg+ko
                                        got[(sg,i)] = min(got.get((sg,i),(10**9,0)), (bv[s], key))
    nterms = sum(1 for sg in range(3,n) for i in range(1,n-sg+1) for jo in range(sg) for do in range(jo+1,sg) for ko in range(do+1,sg))
    assert got == brute, [(k, got.get(k), brute.get(k)) for k in brute if got.get(k)!=brute[k]][:5]
    assert cnt == nterms, (cnt, nterms)
    print(n, S, "ok", len(brute), nterms)
for n, S in [(8,8),(13,2),(17,3),(20,8),(24,4)]:
    run(n, S)
