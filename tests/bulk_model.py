"""The batch engine's bulk formulation of a graph's call schedule, restated in
plain Python (test infrastructure: the CPU model of hge_batch.hip's kb_prep ..
kb_sort, checked against the oracle by tests/test_bulk_model.py).

RunConsensus runs after every call point (node/core.go:179-202).  Once every
event's round and witness flag are known (they depend on the event's ancestry
alone), the per-call work splits into stages that are parallel over calls,
rounds or events, with one short sequential fold per graph:

  prep     R_c (Rounds() after call c's DivideRounds), each event's insertion
           call, the witnesses in insertion order (their arrival calls);
  pairs    DecideFame's decisions for round i at call c (hashgraph.go:598-664),
           a function of the witnesses present at c only (`votes` is rebuilt
           every call), for the rounds i = R_c - 2 - s, s < NS;
  fold     the calls in order: arrivals set the present-witness masks, rounds
           LCR+1 .. R_c-2 take their pair's decisions (a pair outside the NS
           window is decided inline), setLastConsensusRound; every round's
           (decided, famous set) state as intervals of calls;
  theta    per interval, the receive threshold per creator: x is seen by more
           than half of the famous witnesses iff index(x) <= theta
           (hashgraph.go:676-721);
  receive  per event, the first call at which some round above it has a
           decided interval that sees it (the lowest such round at that call),
           and MedianTimestamp (:762-770);
  order    per call, the received events sorted by (rr, cts, S, id)
           (consensus_sorter.go:36-59 with PRN = 0).
"""
import numpy as np

INF = 1 << 60


def coordinates(dag, status):
    """Accepted events in insertion order with LA and FD rows (InitEventCoordinates)."""
    n = int(dag["n"])
    acc = np.nonzero(status >= 0)[0]
    E = len(acc)
    idmap = np.full(len(status), -1, np.int64)
    idmap[acc] = np.arange(E)
    cr = dag["creator"][acc].astype(np.int64)
    ix = dag["index"][acc].astype(np.int64)
    sp = np.array([idmap[s] if s >= 0 else -1 for s in dag["sp"][acc]], np.int64)
    op = np.array([idmap[o] if o >= 0 else -1 for o in dag["op"][acc]], np.int64)
    LA = np.full((E, n), -1, np.int64)
    for x in range(E):
        row = np.full(n, -1, np.int64)
        if sp[x] >= 0:
            row = np.maximum(row, LA[sp[x]])
        if op[x] >= 0:
            row = np.maximum(row, LA[op[x]])
        row[cr[x]] = ix[x]
        LA[x] = row
    chain = [np.nonzero(cr == c)[0] for c in range(n)]
    FD = np.full((E, n), INF, np.int64)
    for d in range(n):
        ch = chain[d]
        for c in range(n):
            col = LA[ch, c] if len(ch) else np.zeros(0, np.int64)
            xs = np.nonzero(cr == c)[0]
            # first chain-d position whose lastAncestor on chain c reaches index(x)
            p = np.searchsorted(col, ix[xs], side="left")
            FD[xs, d] = np.where(p < len(ch), p, INF)
    return dict(n=n, E=E, acc=acc, cr=cr, ix=ix, LA=LA, FD=FD, chain=chain,
                ts=dag["ts"][acc].astype(np.int64), S=dag["S"][acc], ntx=dag["ntx"][acc].astype(np.int64),
                coin=(dag["hash"][acc][:, 16] != 0))


def bulk_replay(dag, call_points, status, rounds, wit, NS=4):
    """The bulk formulation; rounds / wit as the rounds stage leaves them."""
    g = coordinates(dag, status)
    n, E, cr, ix, LA, FD = g["n"], g["E"], g["cr"], g["ix"], g["LA"], g["FD"]
    SM = 2 * n // 3 + 1
    rounds = np.asarray(rounds, np.int64)
    wit = np.asarray(wit, bool)
    accn = np.cumsum(status >= 0)
    ncs = [int(accn[cp - 1]) for cp in call_points]
    K = len(ncs)
    Rmax = int(rounds.max()) + 1 if E else 0
    W = np.full((Rmax + 1, n), -1, np.int64)
    for x in np.nonzero(wit)[0]:
        W[rounds[x], cr[x]] = x

    def see(y, x):
        return LA[y, cr[x]] >= ix[x]

    def ssee(y, w):
        return int((LA[y] >= FD[w]).sum()) >= SM

    seeb = np.zeros((Rmax + 1, n), object)
    ssb = np.zeros((Rmax + 1, n), object)
    for r in range(1, Rmax):
        for c in range(n):
            y = W[r, c]
            if y < 0:
                continue
            a = b = 0
            for d in range(n):
                w = W[r - 1, d]
                if w >= 0:
                    a |= int(see(y, w)) << d
                    b |= int(ssee(y, w)) << d
            seeb[r, c], ssb[r, c] = a, b

    # ---- prep ----
    Rc = []
    xcall = np.full(E, K, np.int64)
    prev = 0
    for c, nc in enumerate(ncs):
        xcall[prev:nc] = c
        prev = nc
        Rc.append(int(rounds[:nc].max()) + 1 if nc else 0)
    n_last = ncs[-1] if K else 0
    arrivals = [(int(xcall[x]), int(rounds[x]), int(cr[x])) for x in range(n_last) if wit[x]]

    # ---- pairs ----
    def fame_pair(i, nc, R):
        pres = [W[i, x] >= 0 and W[i, x] < nc for x in range(n)]
        dec = val = 0
        for x in range(n):
            if not pres[x]:
                continue
            prevv = 0  # vote mask of round j-1's witnesses on x
            fv = 0
            for j in range(i + 1, R):
                diff = j - i
                cur = 0
                ys = [y for y in range(n) if W[j, y] >= 0 and W[j, y] < nc]
                for y in ys:
                    if diff == 1:
                        cur |= int((seeb[j, y] >> x) & 1) << y
                        continue
                    yb = ssb[j, y]
                    yays = bin(yb & prevv).count("1")
                    nays = bin(yb).count("1") - yays
                    v = yays >= nays
                    t = yays if v else nays
                    if diff % n != 0:
                        if t >= SM:
                            fv = 1 if v else 2
                            break
                        cur |= int(v) << y
                    else:
                        cur |= int(v if t >= SM else g["coin"][W[j, y]]) << y
                prevv = cur
            if fv:
                dec |= 1 << x
                val |= int(fv == 1) << x
        return dec, val

    Dp = {}
    for c in range(K):
        for s in range(NS):
            i = Rc[c] - 2 - s
            if i >= 0:
                Dp[(c, s)] = fame_pair(i, ncs[c], Rc[c])
                # round R_c - 2 meets one voting round only (diff = 1): nothing decided,
                # so the kernels never compute s = 0
                assert s > 0 or Dp[(c, s)][0] == 0

    # ---- fold ----
    pres = [0] * (Rmax + 1)
    dfn = [0] * (Rmax + 1)
    vl = [0] * (Rmax + 1)
    ost = [-1] * (Rmax + 1)
    oF = [0] * (Rmax + 1)
    ivl = [[] for _ in range(Rmax + 1)]  # (cs, ce, F)
    LCR, lcr_call, misses = -1, -1, 0
    ap = 0
    for c in range(K):
        touched = set()
        while ap < len(arrivals) and arrivals[ap][0] == c:
            _, r, k = arrivals[ap]
            pres[r] |= 1 << k
            touched.add(r)
            ap += 1
        R = Rc[c]
        newL = -1
        for i in range(LCR + 1, R - 1):
            s = R - 2 - i
            if s < NS:
                dec, v = Dp[(c, s)]
            else:
                dec, v = fame_pair(i, ncs[c], R)
                misses += 1
            dfn[i] |= dec
            vl[i] = (vl[i] & ~dec) | v
            if pres[i] & ~dfn[i] == 0:
                newL = i
            touched.add(i)
        if newL >= 0:
            LCR, lcr_call = newL, c
        for r in touched:
            decided = pres[r] & ~dfn[r] == 0
            key = pres[r] & vl[r] if decided else 0
            if key != oF[r]:
                if ost[r] >= 0:
                    ivl[r].append((ost[r], c, oF[r]))
                ost[r], oF[r] = (c, key) if key else (-1, 0)
    for r in range(Rmax + 1):
        if ost[r] >= 0:
            ivl[r].append((ost[r], K, oF[r]))

    # ---- theta ----
    theta = {}
    for r in range(Rmax + 1):
        for k, (_, _, F) in enumerate(ivl[r]):
            m = bin(F).count("1")
            need = m // 2 + 1
            th = []
            for c in range(n):
                vals = sorted((LA[W[r, d], c] for d in range(n) if (F >> d) & 1), reverse=True)
                th.append(vals[need - 1])
            theta[(r, k)] = th

    # ---- receive + median ----
    rr = np.full(E, -1, np.int64)
    rcall = np.full(E, -1, np.int64)
    cts = np.zeros(E, np.int64)
    for x in range(n_last):
        best_c, best = INF, None
        for i in range(rounds[x] + 1, Rmax):
            for k, (cs, ce, F) in enumerate(ivl[i]):
                if ce <= xcall[x]:
                    continue
                cand = max(cs, xcall[x])
                if cand >= best_c:
                    break
                if ix[x] <= theta[(i, k)][cr[x]]:
                    best_c, best = cand, (i, F)
                    break
        if best is None:
            continue
        i, F = best
        rr[x], rcall[x] = i, best_c
        t = []
        for d in range(n):
            if (F >> d) & 1 and FD[x, d] <= ix[W[i, d]]:
                t.append(g["ts"][g["chain"][d][FD[x, d]]])
        t.sort()
        cts[x] = t[len(t) // 2]

    # ---- order ----
    order, counts = [], []
    for c in range(K):
        xs = [x for x in range(n_last) if rcall[x] == c]
        xs.sort(key=lambda x: (rr[x], cts[x], bytes(g["S"][x]), x))
        order += xs
        counts.append(len(xs))
    fame = np.full((Rc[-1] if K else 0, n), -1, np.int8)
    for r in range(fame.shape[0]):
        for c in range(n):
            if W[r, c] >= 0:
                fame[r, c] = 0 if not (dfn[r] >> c) & 1 else (1 if (vl[r] >> c) & 1 else 2)
    lcre = 0
    if LCR >= 1:
        lcre = int(((rounds[:ncs[lcr_call]]) == LCR - 1).sum())
    und = [x for x in range(n_last) if rr[x] < 0]
    ctx = int(g["ntx"][np.array(order, np.int64)].sum()) if order else 0
    return dict(order=np.array(order, np.int64), counts=np.array(counts, np.int64), rr=rr, cts=cts, fame=fame,
                undetermined=np.array(und, np.int64),
                scalars=np.array([Rc[-1] if K else 0, LCR, lcre, ctx], np.int64),
                stats=dict(misses=misses, max_intervals=max((len(v) for v in ivl), default=0),
                           intervals=sum(len(v) for v in ivl)))
