"""The text kernel's chain micro-step (modelled in tests/text_model.py) yields
the same leaf multiset as the plain P0 DFS against the text, from arbitrary
DFS states, within the 2k + 2 stack bound."""
import random

import pytest

import oracle
from text_model import D_, I_, MS, chain, plain, sides


def states(P, T, sch, edit, limit=300):
    """DFS nodes from every start position (what the FM phase could hand over)."""
    pi, l, u, dirs = sch
    m = len(pi)
    out = []
    for start in range(len(T) + 1):
        st = [(start, start, 0, 0, 0, 0)]
        while st and len(out) < limit:
            node = st.pop()
            xs, ye, pos, e, lL, lR = node
            if ye - xs >= 3:
                out.append(node)
            if pos == m:
                continue
            q, r = pi[pos], dirs[pos]
            side = lR if r else lL
            c = (T[ye] if ye < len(T) else 0) if r else (T[xs - 1] if xs > 0 else 0)
            mOK, misOK = l[pos] <= e <= u[pos], l[pos] <= e + 1 <= u[pos]
            delOK = edit and pos > 0 and e + 1 <= u[pos] and side != I_
            insOK = edit and misOK and side != D_
            a, b = (xs, ye + 1) if r else (xs - 1, ye)
            if c != 0:
                if c == P[q]:
                    if mOK:
                        st.append((a, b, pos + 1, e) + sides(pos, r, lL, lR, MS))
                elif misOK:
                    st.append((a, b, pos + 1, e + 1) + sides(pos, r, lL, lR, MS))
                if delOK:
                    st.append((a, b, pos, e + 1) + sides(pos, r, lL, lR, D_))
            if insOK:
                st.append((xs, ye, pos + 1, e + 1) + sides(pos, r, lL, lR, I_))
    return out


@pytest.mark.parametrize("run,chain_len", [(16, 8), (32, 16), (32, 25)])
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5])
def test_chain_step_equals_plain_dfs(seed, run, chain_len):
    rng = random.Random(seed)
    checked = 0
    for _ in range(60):
        m, k = rng.randint(8, 36), rng.randint(1, 3)
        gen = rng.choice(["h2-k2", "h2-k1", "pigeon", "backtracking", "h2-k3"])
        ham = rng.random() < 0.3
        pi, l, u = oracle.scheme(gen, 0, k, m, hamming=ham)
        s = rng.randrange(len(pi))
        pi, l, u = [int(v) for v in pi[s]], [int(v) for v in l[s]], [int(v) for v in u[s]]
        dirs = [pi[p] > pi[p - 1] if p else (pi[1] > pi[0] if m > 1 else True) for p in range(m)]
        sig = rng.choice([2, 3, 4])  # small alphabets: repeats, many surviving children
        P = [rng.randint(1, sig) for _ in range(m)]
        T = [rng.randint(1, sig) for _ in range(8)] + P[:] + [rng.randint(1, sig) for _ in range(8)]
        for _ in range(rng.randint(0, 3)):
            T[rng.randrange(8, 8 + m)] = rng.randint(1, sig)
        for _ in range(rng.randint(0, 2)):
            j = rng.randrange(8, 8 + m)
            if rng.random() < 0.5:
                del T[j]
            else:
                T.insert(j, rng.randint(1, sig))
        if rng.random() < 0.2:
            T[rng.randrange(len(T))] = 0  # a delimiter
        edit = not ham
        cap = 2 * max(max(u), 1) + 2
        nodes = states(P, T, (pi, l, u, dirs), edit)
        for task in rng.sample(nodes, min(5, len(nodes))):
            assert chain(P, T, task, (pi, l, u, dirs), edit, cap=cap, RUN=run, CHAIN=chain_len) == plain(P, T, task, (pi, l, u, dirs), edit)
            checked += 1
    assert checked > 100


def test_pruning_on_true_reads():
    """h2-k2, m = 100, k = 2: reads with two random edits against their text.
    From every task the FM phase could hand over at depth 16, the pruned step
    (nodes two errors below their bound keep only viable error children) gives
    the plain DFS's leaves, in fewer micro-steps."""
    rng = random.Random(5)
    m, k = 100, 2
    pi, l, u = oracle.scheme("h2-k2", 0, k, m)
    steps = {True: {}, False: {}}
    for _ in range(12):
        T = [rng.randint(1, 4) for _ in range(400)]
        P = T[150:250]
        for _ in range(k):
            j, r = rng.randrange(5, 95), rng.random()
            if r < 0.33:
                P[j] = rng.choice([c for c in (1, 2, 3, 4) if c != P[j]])
            elif r < 0.66:
                del P[j]
                P.append(T[250])
            else:
                P.insert(j, rng.randint(1, 4))
                P.pop()
        for s in range(len(pi)):
            sp, sl, su = [int(v) for v in pi[s]], [int(v) for v in l[s]], [int(v) for v in u[s]]
            dirs = [sp[p] > sp[p - 1] if p else sp[1] > sp[0] for p in range(m)]
            sch = (sp, sl, su, dirs)
            for task in [n for n in states(P, T, sch, True, limit=100000) if n[2] == 16]:
                want = plain(P, T, task, sch, True)
                for prune in (True, False):
                    assert chain(P, T, task, sch, True, cap=6, PRUNE=prune, stats=steps[prune]) == want
    assert steps[True]["steps"] < 0.85 * steps[False]["steps"]
