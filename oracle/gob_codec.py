"""TEST INFRASTRUCTURE ONLY (the checker, never the product): a pure-Python
restatement of Go's encoding/gob for the types babble puts on the wire or hashes,
used by tests/test_gob.py to check babble_amd/csrc/hge_gob.cpp.

Reference types: WireEvent / WireBody (hashgraph/event.go:244-259), EventBody
(event.go:26-58, Marshal), SyncResponse (net/commands.go).  The algorithm is the
Go standard library's encoding/gob (absent here); the reference's own tests of
these paths are round trips (event_test.go:34-144, TestMarshallBody,
TestMarshallEvent, TestWireEvent) and hold no golden bytes, so byte-level parity is
unpinned beyond this restatement of the published format.

Written independently of the C++ codec: a generic encoder driven by a small type
schema (ids assigned the way gob's type registry assigns them: a struct when first
seen, before its fields; a slice after its element; first user id 65), and a
generic decoder that reads type definitions and returns nested dicts.
"""

UNIX_TO_GO = 62135596800
T_BOOL, T_INT, T_UINT, T_FLOAT, T_BYTES, T_STRING = 1, 2, 3, 4, 5, 6


def enc_uint(x):
    if x < 128:
        return bytes([x])
    b = x.to_bytes((x.bit_length() + 7) // 8, "big")
    return bytes([256 - len(b)]) + b


def enc_int(i):
    return enc_uint((~i << 1) | 1 if i < 0 else i << 1)


def enc_bytes(b):
    return enc_uint(len(b)) + bytes(b)


def time_gob(ts):
    """time.Time.GobEncode (MarshalBinary, version 1): ts = (unix_sec, nsec, offset_min)."""
    sec, nsec, off = ts
    return (bytes([1]) + (sec + UNIX_TO_GO).to_bytes(8, "big", signed=True) + nsec.to_bytes(4, "big", signed=True)
            + off.to_bytes(2, "big", signed=True))


def bigint_gob(v):
    """big.Int.GobEncode: (version 1 << 1 | sign), then the magnitude big-endian."""
    mag = abs(v).to_bytes((abs(v).bit_length() + 7) // 8, "big")
    return bytes([2 | (1 if v < 0 else 0)]) + mag


# ---- schema: ("struct", name, [(field, type)]), ("slice", name, elem), ("gob", name, encode_fn),
# or a predefined id (T_INT, T_BYTES, T_STRING)
TIME = ("gob", "Time", time_gob)
INT = ("gob", "Int", bigint_gob)
WIREBODY = ("struct", "WireBody", [("Transactions", ("slice", "[][]uint8", T_BYTES)), ("SelfParentIndex", T_INT),
                                   ("OtherParentCreatorID", T_INT), ("OtherParentIndex", T_INT),
                                   ("CreatorID", T_INT), ("Timestamp", TIME), ("Index", T_INT)])
WIREEVENT = ("struct", "WireEvent", [("Body", WIREBODY), ("R", INT), ("S", INT)])
EVENTBODY = ("struct", "EventBody", [("Transactions", ("slice", "[][]uint8", T_BYTES)),
                                     ("Parents", ("slice", "[]string", T_STRING)), ("Creator", T_BYTES),
                                     ("Timestamp", TIME), ("Index", T_INT)])
SYNCRESPONSE = ("struct", "SyncResponse", [("From", T_STRING), ("Head", T_STRING),
                                           ("Events", ("slice", "[]hashgraph.WireEvent", WIREEVENT))])


class Encoder:
    """One gob.Encoder: type ids from a process-wide counter, definitions sent once."""

    def __init__(self, first_id=65):
        self.next = first_id
        self.ids = {}    # schema key -> id
        self.sent = set()
        self.out = bytearray()

    @staticmethod
    def key(t):
        return t if isinstance(t, int) else (t[0], t[1])

    def tid(self, t):
        """gob's registry: struct id at first sight (then its fields), slice after its element."""
        if isinstance(t, int):
            return t
        k = self.key(t)
        if k in self.ids:
            return self.ids[k]
        if t[0] == "struct":
            self.ids[k] = self.next
            self.next += 1
            for _, ft in t[2]:
                self.tid(ft)
        elif t[0] == "slice":
            e = self.tid(t[2])
            if k not in self.ids:
                self.ids[k] = self.next
                self.next += 1
            del e
        else:
            self.ids[k] = self.next
            self.next += 1
        return self.ids[k]

    def message(self, payload):
        self.out += enc_uint(len(payload)) + payload

    @staticmethod
    def common(name, i):
        return enc_uint(1) + enc_bytes(name.encode()) + enc_uint(1) + enc_int(i) + enc_uint(0)

    def send_type(self, t):
        """the definition of t (if not sent yet), then its components in field order"""
        if isinstance(t, int) or self.key(t) in self.sent:
            return
        i = self.tid(t)
        self.sent.add(self.key(t))
        if t[0] == "struct":
            fields = enc_uint(len(t[2])) + b"".join(
                enc_uint(1) + enc_bytes(f.encode()) + enc_uint(1) + enc_int(self.tid(ft)) + enc_uint(0)
                for f, ft in t[2])
            body = enc_uint(3) + enc_uint(1) + self.common(t[1], i) + enc_uint(1) + fields + enc_uint(0) + enc_uint(0)
        elif t[0] == "slice":
            body = (enc_uint(2) + enc_uint(1) + self.common(t[1], i) + enc_uint(1) + enc_int(self.tid(t[2]))
                    + enc_uint(0) + enc_uint(0))
        else:  # GobEncoderT: wireType field 4
            body = enc_uint(5) + enc_uint(1) + self.common(t[1], i) + enc_uint(0) + enc_uint(0)
        self.message(enc_int(-i) + body)
        if t[0] == "struct":
            for _, ft in t[2]:
                self.send_type(ft)
        elif t[0] == "slice":
            self.send_type(t[2])

    def value(self, t, v):
        """the encoding of v (non-zero checked by the caller for struct fields)"""
        if t == T_INT:
            return enc_int(v)
        if t in (T_BYTES,):
            return enc_bytes(v)
        if t == T_STRING:
            return enc_bytes(v.encode())
        if t[0] == "gob":
            return enc_bytes(t[2](v))
        if t[0] == "slice":
            return enc_uint(len(v)) + b"".join(self.value(t[2], x) for x in v)
        out, last = b"", -1
        for k, (f, ft) in enumerate(t[2]):
            x = v.get(f)
            if isinstance(ft, tuple) and ft[0] == "struct":
                x = x or {}  # nested structs always go
            elif isinstance(ft, tuple) and ft[0] == "gob":
                if x is None:  # nil pointer / zero Time
                    continue
            elif x is None or x == 0 or len(x if not isinstance(x, int) else [1]) == 0:
                continue  # zero int, empty string, bytes or slice
            out += enc_uint(k - last) + self.value(ft, x)
            last = k
        return out + enc_uint(0)

    def encode(self, t, v):
        self.send_type(t)
        self.message(enc_int(self.tid(t)) + self.value(t, v))


# ---- decoding (generic)
class _R:
    def __init__(self, b):
        self.b, self.p = b, 0

    def u(self):
        c = self.b[self.p]
        self.p += 1
        if c < 128:
            return c
        k = 256 - c
        x = int.from_bytes(self.b[self.p:self.p + k], "big")
        self.p += k
        return x

    def i(self):
        x = self.u()
        return ~(x >> 1) if x & 1 else x >> 1

    def raw(self):
        n = self.u()
        v = bytes(self.b[self.p:self.p + n])
        self.p += n
        return v


def decode(stream):
    """[(type name, value)] of every top-level value; structs as dicts by field name,
    Time as (unix_sec, nsec, offset_min), Int as int."""
    types, out, r0 = {}, [], _R(stream)
    while r0.p < len(stream):
        n = r0.u()
        r = _R(stream[r0.p:r0.p + n])
        r0.p += n
        tid = r.i()
        if tid < 0:
            types[-tid] = _wiretype(r)
            continue
        if types.get(tid, ("",))[0] != "struct":
            assert r.u() == 0
        out.append((types[tid][1] if tid in types else tid, _value(r, tid, types)))
    return out


def _common(r):
    name, i, f = "", 0, -1
    while True:
        d = r.u()
        if d == 0:
            return name, i
        f += d
        if f == 0:
            name = r.raw().decode()
        else:
            i = r.i()


def _wiretype(r):
    f = r.u() - 1
    g, name, fields, elem = -1, "", [], 0
    while True:
        d = r.u()
        if d == 0:
            break
        g += d
        if g == 0:
            name, _ = _common(r)
        elif f == 2:
            fields = [_common(r) for _ in range(r.u())]
        else:
            elem = r.i()
    assert r.u() == 0
    kind = {1: "slice", 2: "struct", 4: "gob"}[f]
    return (kind, name, fields if kind == "struct" else elem)


def _value(r, tid, types):
    if tid == T_INT:
        return r.i()
    if tid in (T_BOOL, T_UINT, T_FLOAT):
        return r.u()
    if tid == T_BYTES:
        return r.raw()
    if tid == T_STRING:
        return r.raw().decode()
    kind, name, spec = types[tid]
    if kind == "gob":
        b = r.raw()
        if name == "Time":
            return (int.from_bytes(b[1:9], "big", signed=True) - UNIX_TO_GO, int.from_bytes(b[9:13], "big", signed=True),
                    int.from_bytes(b[13:15], "big", signed=True))
        v = int.from_bytes(b[1:], "big")
        return -v if b[0] & 1 else v
    if kind == "slice":
        return [_value(r, spec, types) for _ in range(r.u())]
    out, f = {}, -1
    while True:
        d = r.u()
        if d == 0:
            return out
        f += d
        fname, ftid = spec[f]
        out[fname] = _value(r, ftid, types)


def wire_event_value(e):
    """the WireEvent value (field dict) of a gob_encode_wire_events-style dict"""
    body = {"Transactions": e.get("transactions", []), "SelfParentIndex": e.get("self_parent_index", 0),
            "OtherParentCreatorID": e.get("other_parent_creator_id", 0),
            "OtherParentIndex": e.get("other_parent_index", 0), "CreatorID": e.get("creator_id", 0),
            "Timestamp": e.get("timestamp"), "Index": e.get("index", 0)}
    return {"Body": body, "R": e.get("r"), "S": e.get("s")}
