"""The host ingest pipeline's crypto: hge_verify_events and
hge_sha256_batch against the pure-Python checkers (hashlib; oracle/p256.py, the
restatement of Go's ecdsa.Verify on P-256), both directions:
  * signatures made by oracle/p256.py verify in the C library;
  * signatures made through OpenSSL (build/libhge_tools.so) verify in the oracle,
    which pins the oracle against an independent implementation;
  * every way Event.Verify fails in the reference fails here: a changed body, a
    changed r or s, r or s outside [1, n-1], a key that is not a curve point, a
    compressed key (elliptic.Unmarshal takes only 0x04 || X || Y).
Host code only: no GPU needed (the library loads without one)."""
import hashlib

import numpy as np
import pytest

from babble_amd import engine, signing
from babble_amd.gossip import random_gossip
from oracle import p256


def test_curve_constants():
    assert p256.on_curve(p256.GX, p256.GY)
    assert p256._affine(p256._mul(p256.N, p256.GX, p256.GY)) is None  # G has order n
    assert p256._affine(p256._mul(p256.N - 1, p256.GX, p256.GY)) == (p256.GX, (-p256.GY) % p256.P)


def test_sha256_batch_matches_hashlib():
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in [0, 1, 55, 56, 63, 64, 65, 1000, 4097]]
    for th in (1, 3):
        out = engine.sha256_batch(data, threads=th)
        for d, h in zip(data, out):
            assert bytes(h) == hashlib.sha256(d).digest()


def _oracle_signed(n, seed=11):
    """n events signed by oracle/p256.py with 4 keys."""
    rng = np.random.default_rng(seed)
    ds = [int.from_bytes(rng.bytes(32), "big") % (p256.N - 1) + 1 for _ in range(4)]
    pubs = [p256.public_key(d) for d in ds]
    bodies, P, S = [], [], []
    for i in range(n):
        body = rng.bytes(int(rng.integers(40, 300)))
        c = i % 4
        k = int.from_bytes(rng.bytes(32), "big") % (p256.N - 1) + 1
        r, s = p256.sign(ds[c], hashlib.sha256(body).digest(), k)
        bodies.append(body)
        P.append(np.frombuffer(pubs[c], np.uint8))
        S.append(np.frombuffer(r.to_bytes(32, "big") + s.to_bytes(32, "big"), np.uint8))
    return bodies, np.array(P), np.array(S)


def test_oracle_signatures_verify_in_engine():
    bodies, pubs, sigs = _oracle_signed(24)
    for th in (1, 4):
        ok, hashes = engine.verify_events(bodies, pubs, sigs, threads=th)
        assert ok.all()
        for b, h in zip(bodies, hashes):
            assert bytes(h) == hashlib.sha256(b).digest()


def test_openssl_signatures_verify_in_oracle():
    dag = random_gossip(4, 40, seed=2)
    pubs, (flat, off), sigs = signing.signed_stream(dag, seed=7, threads=2)
    cre = dag["creator"]
    ok, _ = engine.verify_events((flat, off), pubs[cre], sigs, threads=2)
    assert ok.all()
    for i in range(0, 40, 3):
        assert p256.verify_event(flat[off[i]:off[i + 1]], pubs[cre[i]], sigs[i])
    # the same key set from the same seed, a different one from another seed
    assert np.array_equal(signing.keys(4, 7), pubs)
    assert not np.array_equal(signing.keys(4, 8), pubs)


def test_every_failure_of_event_verify():
    bodies, pubs, sigs = _oracle_signed(12, seed=3)
    bodies = list(bodies)
    pubs, sigs = pubs.copy(), sigs.copy()
    bad = {}
    bodies[1] = bodies[1][:-1] + bytes([bodies[1][-1] ^ 1]); bad[1] = "body"
    sigs[2, 31] ^= 1; bad[2] = "r"
    sigs[3, 63] ^= 1; bad[3] = "s"
    sigs[4, :32] = 0; bad[4] = "r = 0"
    sigs[5, 32:] = np.frombuffer(p256.N.to_bytes(32, "big"), np.uint8); bad[5] = "s = n"
    pubs[6, 64] ^= 1; bad[6] = "key off the curve"
    pubs[7, 0] = 2; bad[7] = "compressed key prefix"
    pubs[8] = pubs[9]; bad[8] = "another creator's key"  # (i % 4 differs: 8 -> key 0, 9 -> key 1)
    ok, _ = engine.verify_events(bodies, pubs, sigs, threads=3)
    for i in range(12):
        want = i not in bad
        assert bool(ok[i]) == want, (i, bad.get(i))
        assert p256.verify_event(bodies[i], pubs[i], sigs[i]) == want, (i, bad.get(i))


def test_verify_rejects_bad_offsets():
    with pytest.raises(engine.HgeError):
        engine.verify_events((np.zeros(8, np.uint8), np.array([0, 5, 3], np.int64)),
                             np.zeros((2, 65), np.uint8), np.zeros((2, 64), np.uint8))
    ok, _ = engine.verify_events([], np.zeros((0, 65), np.uint8), np.zeros((0, 64), np.uint8))
    assert len(ok) == 0
