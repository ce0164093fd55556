"""babble's wire / hashing format: the gob codec of hge_gob.cpp
against an independent Python restatement (oracle/gob_codec.py) and the format's
published integer / string encodings.  The reference's own tests of these paths
are round trips (hashgraph/event_test.go:34-144: TestMarshallBody,
TestMarshallEvent, TestWireEvent); it holds no golden gob bytes, so byte-level
parity with a Go process is unpinned beyond this restatement.  Host-only code:
runs on the CPU."""
import random

import pytest

from oracle import gob_codec as g


def _event(rng, k):
    txs = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))) for _ in range(rng.randrange(0, 4))]
    return {"self_parent_index": rng.choice([-1, 0, k, 70000]), "other_parent_creator_id": rng.choice([-1, 0, 3, 255]),
            "other_parent_index": rng.choice([-1, 0, 12, 1 << 40]), "creator_id": rng.randrange(0, 300),
            "index": rng.choice([0, 1, k, 123456]),
            "timestamp": rng.choice([None, (1500000000 + k, rng.randrange(10 ** 9), -1), (-5, 999, 120),
                                     (1 << 33, 0, 0)]),
            "r": rng.choice([None, 0, 1, rng.getrandbits(256), rng.getrandbits(200)]),
            "s": rng.choice([None, 7, rng.getrandbits(256)]),
            "transactions": txs}


def _norm(e):
    """the fields a round trip must give back (absent = zero)"""
    out = {f: e.get(f, 0) for f in ("self_parent_index", "other_parent_creator_id", "other_parent_index",
                                    "creator_id", "index")}
    out.update(timestamp=e.get("timestamp"), r=e.get("r"), s=e.get("s"), transactions=list(e.get("transactions", [])))
    return out


def test_published_primitive_encodings():
    # encoding/gob: unsigned < 128 in one byte, else -(byte count) then big-endian bytes;
    # signed i -> unsigned (i << 1) or (~i << 1) | 1; strings and []byte: length + bytes
    assert g.enc_uint(0) == b"\x00" and g.enc_uint(7) == b"\x07" and g.enc_uint(127) == b"\x7f"
    assert g.enc_uint(128) == b"\xff\x80" and g.enc_uint(256) == b"\xfe\x01\x00"
    assert g.enc_int(0) == b"\x00" and g.enc_int(1) == b"\x02" and g.enc_int(-1) == b"\x01"
    assert g.enc_int(-129) == b"\xfe\x01\x01"
    assert g.enc_int(-65) == b"\xff\x81"  # the first user type's definition id
    assert g.enc_bytes(b"abc") == b"\x03abc"
    # time.Time.GobEncode version 1 (15 bytes), big.Int.GobEncode (2 | sign, magnitude)
    assert g.time_gob((0, 0, -1)) == b"\x01" + (62135596800).to_bytes(8, "big") + b"\x00" * 4 + b"\xff\xff"
    assert g.bigint_gob(0) == b"\x02" and g.bigint_gob(258) == b"\x02\x01\x02" and g.bigint_gob(-1) == b"\x03\x01"


@pytest.mark.parametrize("first_id", [65, 100])
def test_wire_events_bytes_equal_the_restatement(first_id):
    from babble_amd.engine import gob_encode_wire_events
    rng = random.Random(first_id)
    evs = [_event(rng, k) for k in range(40)]
    enc = g.Encoder(first_id)
    for e in evs:
        enc.encode(g.WIREEVENT, g.wire_event_value(e))
    assert gob_encode_wire_events(evs, first_id) == bytes(enc.out)


def test_wire_events_round_trip():
    """TestMarshallEvent / TestWireEvent's round trip, over random events and the edge
    values (no transactions, empty ones, -1 parents, nil and zero signatures, zero time)."""
    from babble_amd.engine import gob_decode_wire_events, gob_encode_wire_events
    rng = random.Random(7)
    evs = [_event(rng, k) for k in range(200)] + [{}]
    b = gob_encode_wire_events(evs)
    assert [_norm(e) for e in gob_decode_wire_events(b)] == [_norm(e) for e in evs]
    # the independent decoder reads the C++ stream the same way
    got = g.decode(b)
    assert [name for name, _ in got] == ["WireEvent"] * len(evs)
    for (_, v), e in zip(got, evs):
        body = v["Body"]
        assert body.get("Transactions", []) == list(e.get("transactions", []))
        assert body.get("Index", 0) == e.get("index", 0) and v.get("R") == e.get("r") and v.get("S") == e.get("s")
        assert body.get("Timestamp") == e.get("timestamp")
    assert gob_encode_wire_events([]) == b""


def test_sync_response_events_decode():
    """A SyncResponse (net/commands.go) as a babble node sends it: type ids of another
    process history, the events nested in a slice field; the decoder follows the
    stream's own type definitions."""
    from babble_amd.engine import gob_decode_wire_events
    rng = random.Random(11)
    evs = [_event(rng, k) for k in range(25)]
    enc = g.Encoder(80)
    enc.encode(g.SYNCRESPONSE, {"From": "127.0.0.1:1337", "Head": "0xABCD",
                                "Events": [g.wire_event_value(e) for e in evs]})
    enc.encode(g.SYNCRESPONSE, {"From": "peer", "Head": "", "Events": []})
    assert [_norm(e) for e in gob_decode_wire_events(bytes(enc.out))] == [_norm(e) for e in evs]


def test_event_body_bytes_and_round_trip():
    """EventBody.Marshal (the bytes Sign / Verify hash): equal to the restatement,
    and TestMarshallBody's round trip through the independent decoder."""
    from babble_amd.engine import gob_encode_event_body
    body = {"Transactions": [b"abc", b"def"], "Parents": ["0xAAAA", "0x0123"], "Creator": b"public key",
            "Timestamp": (1507000000, 123456789, 60), "Index": 9}
    enc = g.Encoder(65)
    enc.encode(g.EVENTBODY, body)
    b = gob_encode_event_body(body["Transactions"], body["Parents"], body["Creator"], body["Timestamp"],
                              body["Index"])
    assert b == bytes(enc.out)
    [(name, v)] = g.decode(b)
    assert name == "EventBody" and v == body
    # the zero fields are omitted, as gob omits them
    empty = gob_encode_event_body([], [], b"", None, 0)
    [(_, v)] = g.decode(empty)
    assert v == {}


def test_malformed_streams_are_refused():
    from babble_amd.engine import HgeError, gob_decode_wire_events, gob_encode_wire_events
    b = gob_encode_wire_events([{"index": 5, "transactions": [b"x" * 50]}])
    for cut in (1, len(b) // 2, len(b) - 1):
        with pytest.raises(HgeError):
            gob_decode_wire_events(b[:cut])
    with pytest.raises(HgeError):
        gob_decode_wire_events(b"\x05\xff\x81\x03\x01\x99")
