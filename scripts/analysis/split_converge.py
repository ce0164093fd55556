"""How far a split walker must run past the next walker's start.

Walker p + 1 starts from the time cut at (p + 1) * E / G (hge_frontier_guess),
which is not a row of the true trajectory; after a few rounds its rows equal
true rows.  Walker p must walk past that point for the join to hand over.  For
every p this prints: the first row of walker p + 1 that walker p also holds
(its convergence, in rounds), and how many rows walker p walked past its
stop cut before that row (the overlap the split needs), plus the event id of
the joined row's latest member (the truncation the next walker's tables need).

usage: python scripts/analysis/split_converge.py [N] [E] [G ...]
"""
import json
import os
import sys
import time

import numpy as np

INF = np.iinfo(np.int32).max

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    Gs = [int(g) for g in sys.argv[3:]] or [2, 4, 8]
    dag = random_gossip(n, E, seed=1)
    ev = events_array(dag)
    eng = Engine(n, E)
    eng.prepare(ev, schedule(E, n))
    chains = [np.flatnonzero(dag["creator"] == c) for c in range(n)]
    out = {"n": n, "E": E, "splits": {}}
    for G in Gs:
        eng.split_begin()
        hists, walk_ms = [], []
        for p in range(G):
            start = eng.frontier_guess(p, G)
            stop = eng.frontier_guess(p + 1, G) if p + 1 < G else None
            t0 = time.perf_counter()
            hists.append(eng.frontier_walk(start, stop, 256 if stop is not None else 0))
            walk_ms.append((time.perf_counter() - t0) * 1e3)
        res = []
        for p in range(G - 1):
            rows_p = {hists[p][0][i].tobytes(): i for i in range(len(hists[p][0]))}
            nxt = hists[p + 1][0]
            conv = next((j for j in range(len(nxt)) if nxt[j].tobytes() in rows_p), None)
            cut = (p + 1) * E // G
            # distance of walker p + 1's first rows to the closest row of walker p
            # (L1 over the entries both hold): 0 = on the true trajectory
            X = hists[p][0].astype(np.int64)
            dist = []
            for j in range(min(60, len(nxt))):
                Y = nxt[j].astype(np.int64)
                ok = (X != INF) & (Y != INF)[None, :]
                d = np.where(ok, np.abs(X - Y[None, :]), 0).sum(axis=1) + (~ok).sum(axis=1) * 1000
                dist.append(int(d.min()))
            if conv is None or (nxt[conv] == INF).all():
                res.append({"p": p, "met": False, "rows_p": len(hists[p][0]), "rows_next": len(nxt),
                            "dist": dist})
                continue
            i = rows_p[nxt[conv].tobytes()]
            row = nxt[conv]
            ids = [int(chains[c][row[c]]) for c in range(n) if row[c] < len(chains[c])]
            # first row of walker p whose every member lies at/after the cut
            past = next((k for k in range(len(hists[p][0]))
                         if all(hists[p][0][k][c] >= np.searchsorted(chains[c], cut) for c in range(n))), None)
            res.append({"p": p, "met": True, "conv_rounds_next": conv, "row_in_p": i,
                        "rows_past_stopcut": None if past is None else i - past,
                        "max_member_id_minus_cut": max(ids) - cut, "rows_p": len(hists[p][0]),
                        "rows_next": len(nxt), "dist": dist})
        out["splits"][G] = {"walk_ms": [round(w, 2) for w in walk_ms], "pairs": res}
        print(G, json.dumps(out["splits"][G]), flush=True)
    eng.close()
    if len(sys.argv) > 0:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"split_converge_n{n}_e{E}.json"), "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()
