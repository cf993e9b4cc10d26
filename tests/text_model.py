"""Python model of kSearchTextBatch's chain micro-step (sahara_amd/csrc/search.hip).

Test infrastructure: `chain()` restates, one node at a time and with Python
sets instead of nibble masks, what a lane of the text kernel does per
micro-step — forced-run nodes matching up to RUN symbols, chain nodes walking
up to CHAIN positions of a match chain and checking every error child's forced
run, nodes two errors below their bound keeping only the error children that
outlive their own first step, the stack reserve rule — and `plain()` is the
textbook DFS of policy P0
(docs/semantics.md) against the text. tests/test_text_model.py holds the two
to the same leaf multiset from arbitrary DFS states.
"""
import collections

MS, I_, D_ = 1, 2, 3
RUN = 32    # symbols per micro-step run (kRun in search.hip)
CHAIN = 25  # chain positions per micro-step of a node whose error children are forced (kChain)

def sides(pos, right, lastL, lastR, op):
    if pos == 0: return op, op
    return (lastL, op) if right else (op, lastR)

def plain(P, T, task, sch, edit):
    pi, l, u, dirs = sch
    m = len(pi)
    out = []
    st = [task]
    while st:
        xs, ye, pos, e, lL, lR = st.pop()
        if pos == m:
            out.append((xs, e)); continue
        q = pi[pos]; r = dirs[pos]; side = lR if r else lL
        c = (T[ye] if ye < len(T) else 0) if r else (T[xs-1] if xs > 0 else 0)
        mOK = l[pos] <= e <= u[pos]; misOK = l[pos] <= e+1 <= u[pos]
        delOK = edit and pos > 0 and e+1 <= u[pos] and side != I_
        insOK = edit and misOK and side != D_
        def span1():
            return (xs, ye+1) if r else (xs-1, ye)
        if c != 0:
            a, b = span1()
            if c == P[q]:
                if mOK: st.append((a, b, pos+1, e) + sides(pos, r, lL, lR, MS))
            elif misOK: st.append((a, b, pos+1, e+1) + sides(pos, r, lL, lR, MS))
            if delOK: st.append((a, b, pos, e+1) + sides(pos, r, lL, lR, D_))
        if insOK: st.append((xs, ye, pos+1, e+1) + sides(pos, r, lL, lR, I_))
    return collections.Counter(out)

def tables(sch):
    pi, l, u, dirs = sch
    m = len(pi)
    run = [0]*m; same = [0]*m
    for p in range(m):
        k = 1
        while k < 127 and p+k < m and dirs[p+k] == dirs[p] and u[p+k] == u[p] and l[p+k] <= u[p]: k += 1
        s = 1
        while s < k and l[p+s] == l[p]: s += 1
        run[p], same[p] = k, s
    return run, same

def chain(P, T, task, sch, edit, cap=100, RUN=RUN, CHAIN=CHAIN, PRUNE=True, stats=None):
    pi, l, u, dirs = sch
    m = len(pi)
    run, same = tables(sch)
    out = []
    st = [task]
    while st:
        xs, ye, pos, e, lL, lR = st.pop()
        if stats is not None:
            stats['steps'] = stats.get('steps', 0) + 1
        if pos == m:
            out.append((xs, e)); continue
        q0 = pi[pos]; r0 = dirs[pos]; lb0 = l[pos]; ub0 = u[pos]; run0 = run[pos]; same0 = same[pos]
        side = lR if r0 else lL
        # chain-order sequences
        def pj(j):
            qq = q0 + j if r0 else q0 - j
            # beyond the pattern the kernel reads whatever precedes / follows it in
            # LDS: arbitrary symbols, which the chain logic must never use
            return P[qq] if 0 <= qq < len(P) else (qq * 7 + 3) % 6
        def tj(j):
            tt = ye + j if r0 else xs - 1 - j
            return T[tt] if 0 <= tt < len(T) else 0
        E0 = {j for j in range(RUN) if pj(j) == tj(j)}
        ED = {j for j in range(RUN) if pj(j) == tj(j+1)}
        EI = {j for j in range(RUN) if pj(j+1) == tj(j)}
        TZ = {j for j in range(RUN) if tj(j) != 0}
        forced = e == ub0; kidsF = e + 1 == ub0
        mOK = lb0 <= e <= ub0; misOK = lb0 <= e+1 <= ub0
        B = min(run0, RUN) if forced else (max(1, min(same0, run0-1, CHAIN)) if kidsF else 1)
        L = 0
        if mOK:
            while L < B and L in E0: L += 1
        NN = L+1 if L < B else B
        nodes = set() if forced else set(range(NN))
        Dm = {i for i in nodes if edit and i in TZ}
        if pos == 0 or side == I_: Dm.discard(0)
        Im = set(nodes) if (edit and misOK) else set()
        if side == D_: Im.discard(0)
        Sx = (not forced) and L < B and misOK and (L in TZ) and (L not in E0)
        def run7(S, beyond):
            return {j for j in range(RUN) if all((jj in S) or jj >= beyond for jj in range(j, j+7))}
        if kidsF:
            Dm &= run7(ED, run0)
            Im &= run7(EI, run0 - 1)
            Sx = Sx and ((L+1) in run7(E0, run0))
        elif PRUNE and edit and e + 2 == ub0:
            # a node expanded alone whose error children are chain nodes
            # (kidsF): keep only the children whose subtree survives their own
            # first step (side rules: no I right after D, no D right after I)
            ED2 = {j for j in range(RUN) if pj(j) == tj(j+2)}
            EI2 = {j for j in range(RUN) if pj(j+2) == tj(j)}
            LIM = RUN - 9
            R = run0
            R7 = {}
            def r7(S, beyond, j):
                key = (id(S), beyond)
                if key not in R7: R7[key] = run7(S, beyond)
                return j in R7[key]
            def first_not(S, j):
                while j < RUN and j in S: j += 1
                return j
            if 0 in Dm:   # D child: pattern j vs text j + 1
                LD = first_not(ED, 0)
                if not (LD >= R or LD > LIM or r7(ED, R, LD + 1) or
                        any(r7(ED2, R, j) or (j > 0 and r7(E0, R, j + 1)) for j in range(LD + 1))):
                    Dm.discard(0)
            if 0 in Im:   # I child: pattern x + 1 vs text x
                LI = first_not(EI, 0)
                if not (LI >= R - 1 or LI > LIM or r7(EI, R - 1, LI + 1) or
                        any((x > 0 and r7(E0, R, x + 1)) or r7(EI2, R - 2, x) for x in range(LI + 1))):
                    Im.discard(0)
            if Sx:        # S child at the mismatch L = 0: pattern x vs text x, x >= 1
                LS = first_not(E0, 1)
                if not (LS >= R or LS > LIM or r7(E0, R, LS + 1) or
                        any(r7(ED, R, x) or r7(EI, R - 1, x) for x in range(1, LS + 1))):
                    Sx = False
        contM = L >= B
        n = len(Dm) + len(Im) + (1 if Sx else 0)
        Bc = B
        if n and len(st) + n + (1 if contM else 0) - 1 > 2 * e + 4:
            Bc = 1; Dm &= {0}; Im &= {0}; Sx = Sx and L == 0
            n = len(Dm) + len(Im) + (1 if Sx else 0)
        contM1 = L >= Bc
        if n and len(st) + n + (1 if contM1 else 0) - 1 > cap:
            raise RuntimeError('stack bound violated')
        def ext(k):
            return (xs, ye + k) if r0 else (xs - k, ye)
        def metaAt(i, op, k):
            ml, mr = lL, lR
            if i > 0:
                if pos == 0: ml = mr = MS
                elif r0: mr = MS
                else: ml = MS
            if pos + i == 0: ml = mr = op
            elif r0: mr = op
            else: ml = op
            if k:
                if r0: mr = MS
                else: ml = MS
            return ml, mr
        rl = (lambda i: min(run0 - i, 7)) if kidsF else (lambda i: 0)
        if contM1: st.append(ext(Bc) + (pos + Bc, e) + metaAt(Bc, MS, 0))
        for i in sorted(Dm):
            k = rl(i); st.append(ext(i+1+k) + (pos+i+k, e+1) + metaAt(i, D_, k))
        for i in sorted(Im):
            k = rl(i+1) if i+1 < run0 else 0; st.append(ext(i+k) + (pos+i+1+k, e+1) + metaAt(i, I_, k))
        if Sx:
            k = rl(L+1) if L+1 < run0 else 0; st.append(ext(L+1+k) + (pos+L+1+k, e+1) + metaAt(L, MS, k))
    return collections.Counter(out)
