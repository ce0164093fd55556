"""Pure-Python ECDSA P-256 (TEST INFRASTRUCTURE ONLY: the checker for
hge_verify_events / hge_ingest; nothing in babble_amd/ imports it).

Restates what the reference's signature path calls:
  * crypto.Sign / crypto.Verify -> Go's ecdsa.Sign / ecdsa.Verify on
    elliptic.P256() (/root/reference/crypto/utils.go:36-64);
  * Event.Sign / Event.Verify sign and verify SHA-256 of the body's bytes
    (/root/reference/hashgraph/event.go:131-150);
  * crypto.ToECDSAPub -> elliptic.Unmarshal: 0x04 || X || Y, the point on the
    curve, else no key (utils.go:40-46).
ecdsa.Verify (Go stdlib, the algorithm of SEC 1 v2 §4.1.4): reject r or s
outside [1, n-1]; e = the hash as an integer (P-256 and SHA-256 have the same
bit length, so no truncation); w = s^-1 mod n; (x, y) = (e w) G + (r w) Q;
valid iff that point is not infinity and x mod n == r.  The curve constants are
FIPS 186-4 D.1.2.3; tests check G lies on the curve and has order n.
"""
import hashlib

P = 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF
A = P - 3
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551


def on_curve(x, y):
    return 0 <= x < P and 0 <= y < P and (y * y - (x * x * x + A * x + B)) % P == 0


# Jacobian coordinates (X, Y, Z), infinity = Z == 0
def _dbl(p1):
    X, Y, Z = p1
    if Z == 0 or Y == 0:
        return (0, 1, 0)
    S = 4 * X * Y * Y % P
    M = (3 * X * X + A * pow(Z, 4, P)) % P
    X3 = (M * M - 2 * S) % P
    Y3 = (M * (S - X3) - 8 * pow(Y, 4, P)) % P
    Z3 = 2 * Y * Z % P
    return (X3, Y3, Z3)


def _add(p1, p2):
    if p1[2] == 0:
        return p2
    if p2[2] == 0:
        return p1
    X1, Y1, Z1 = p1
    X2, Y2, Z2 = p2
    Z1Z1, Z2Z2 = Z1 * Z1 % P, Z2 * Z2 % P
    U1, U2 = X1 * Z2Z2 % P, X2 * Z1Z1 % P
    S1, S2 = Y1 * Z2 * Z2Z2 % P, Y2 * Z1 * Z1Z1 % P
    if U1 == U2:
        return _dbl(p1) if S1 == S2 else (0, 1, 0)
    H, R = (U2 - U1) % P, (S2 - S1) % P
    HH = H * H % P
    HHH = H * HH % P
    X3 = (R * R - HHH - 2 * U1 * HH) % P
    Y3 = (R * (U1 * HH - X3) - S1 * HHH) % P
    Z3 = H * Z1 * Z2 % P
    return (X3, Y3, Z3)


def _mul(k, x, y):
    R = (0, 1, 0)
    Q = (x, y, 1)
    while k:
        if k & 1:
            R = _add(R, Q)
        Q = _dbl(Q)
        k >>= 1
    return R


def _affine(p1):
    X, Y, Z = p1
    if Z == 0:
        return None
    zi = pow(Z, P - 2, P)
    return (X * zi * zi % P, Y * zi * zi * zi % P)


def unmarshal(pub):
    """elliptic.Unmarshal: 65-byte uncompressed point on the curve, else None."""
    pub = bytes(pub)
    if len(pub) != 65 or pub[0] != 4:
        return None
    x, y = int.from_bytes(pub[1:33], "big"), int.from_bytes(pub[33:], "big")
    return (x, y) if on_curve(x, y) else None


def public_key(d):
    x, y = _affine(_mul(d, GX, GY))
    return b"\x04" + x.to_bytes(32, "big") + y.to_bytes(32, "big")


def verify(pub, digest, r, s):
    """ecdsa.Verify(pub, digest, r, s) for P-256."""
    Q = unmarshal(pub)
    if Q is None:
        return False
    if not (0 < r < N and 0 < s < N):
        return False
    e = int.from_bytes(bytes(digest), "big")
    w = pow(s, N - 2, N)
    u1, u2 = e * w % N, r * w % N
    X = _affine(_add(_mul(u1, GX, GY), _mul(u2, Q[0], Q[1])))
    if X is None:
        return False
    return X[0] % N == r


def sign(d, digest, k):
    """Textbook ECDSA with the caller's nonce k (tests only)."""
    e = int.from_bytes(bytes(digest), "big")
    x, _ = _affine(_mul(k, GX, GY))
    r = x % N
    s = pow(k, N - 2, N) * (e + r * d) % N
    return r, s


def verify_event(body, pub, sig):
    """Event.Verify: the signature (r || s) over SHA-256 of the body."""
    sig = bytes(sig)
    return verify(pub, hashlib.sha256(bytes(body)).digest(), int.from_bytes(sig[:32], "big"),
                  int.from_bytes(sig[32:], "big"))
