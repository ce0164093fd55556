"""The committed config-5 digests (tests/golden/make_mc_digests.py) reproduce
from the oracle, and the digest sees every field it claims to cover."""
import json
import os
import sys

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, HERE)

from digest import FIELDS, digest, first_difference  # noqa: E402
from make_mc_digests import OUT, graph_stream, oracle_state  # noqa: E402


def test_mc_digests_reproduce():
    ref = json.load(open(OUT))
    assert ref["graphs"] == 1024 and len(ref["digests"]) == 1024
    for g in (0, 511, 1023):
        st = oracle_state(*graph_stream(g))
        assert digest(st) == ref["digests"][g], g
        assert len(st["order"]) == ref["ordered"][g]
        assert int((st["status"] < 0).sum()) == ref["rejected"][g] > 0


def test_digest_covers_every_field():
    st = oracle_state(*graph_stream(3))
    d0 = digest(st)
    for k, _ in FIELDS:
        mod = {kk: np.array(v, copy=True) for kk, v in st.items()}
        a = mod[k].reshape(-1)
        if k == "cts":  # only ordered events' timestamps count
            a[int(st["order"][0])] += 1
        else:
            a[0] = a[0] + 1 if a[0] < 100 else a[0] - 1
        assert digest(mod) != d0, k
        assert first_difference(mod, st) == k


def test_check_prefix_on_the_bench_golden():
    """parity.check_prefix accepts the N=256 bench golden's own fields and names
    each perturbed one (the golden holds every field: rounds, witnesses, fame,
    round received, timestamps, order, batches)."""
    from parity import check_prefix
    g = np.load(os.path.join(HERE, "bench_n256_e10000000_k256_s1_prefix.npz"))
    assert int(g["prefix"]) >= 200_000 and "rounds" in g.files
    f = {k: np.array(g[k]) for k in ("order", "counts", "rounds", "witness", "rr", "cts", "fame")}
    # a "full run" extends the prefix: more calls, more events, later rounds
    ext = dict(f)
    ext["counts"] = np.concatenate([f["counts"], [5, 7]])
    ext["order"] = np.concatenate([f["order"], [len(f["rounds"]) + 1]])
    ext["rounds"] = np.concatenate([f["rounds"], [99]])
    ext["witness"] = np.concatenate([f["witness"], [1]])
    ext["rr"] = np.concatenate([f["rr"], [100]])
    ext["cts"] = np.concatenate([f["cts"], [0]])
    ext["fame"] = np.concatenate([f["fame"], np.full((3, f["fame"].shape[1]), 1, np.int8)])
    args = ("order", "counts", "rounds", "witness", "rr", "cts", "fame")
    assert check_prefix(g, *[ext[k] for k in args]) == []
    lcr = int(g["scalars"][1])
    for k, idx in (("counts", 3), ("order", 10), ("rounds", 1000), ("witness", 5), ("rr", int(f["order"][7])),
                   ("cts", int(f["order"][9])), ("fame", None)):
        mod = {kk: np.array(v, copy=True) for kk, v in ext.items()}
        if k == "fame":
            r, c = np.argwhere(mod["fame"][:lcr + 1] >= 1)[0]
            mod["fame"][r, c] = 3 - mod["fame"][r, c]
        elif k == "witness":
            mod[k][idx] = 1 - mod[k][idx]
        else:
            mod[k][idx] += 1
        assert check_prefix(g, *[mod[kk] for kk in args]) == [k], k
