// hge_gob.cpp — babble's wire and hashing format: Go's encoding/gob
// for the types the reference puts on the wire or hashes, host-only.
//
//   WireEvent / WireBody   hashgraph/event.go:244-259   (Core.Sync's payload: SyncResponse.Events,
//                                                        net/commands.go, framed by net_transport.go:297-395)
//   EventBody              hashgraph/event.go:44-66      (Marshal: the bytes Sign/Verify hash)
//
// The algorithm is encoding/gob's published format (the Go standard library of the
// reference's 2017 toolchain; the package is absent here), restated:
//   * a stream is a sequence of messages: uint byte count, then int type id; a
//     negative id defines type -id (a wireType value follows), a positive one
//     carries a value of that type;
//   * uint: < 128 one byte, else a byte holding -(byte length) then big-endian bytes;
//     int i: uint (i << 1) for i >= 0, (~i << 1) | 1 for i < 0;
//     string / []byte: uint length + bytes;
//   * struct: (uint field-number delta, value) for every field that is not zero
//     (zero ints, empty strings and slices, nil pointers and zero GobEncoders are
//     omitted; nested structs always go), then delta 0;
//   * slice: uint count then the elements (zero elements included);
//   * GobEncoder values (time.Time, *big.Int): uint length + their GobEncode bytes:
//     Time: version 1, seconds since year 1 (int64 BE), nanoseconds (int32 BE), zone
//     offset in minutes (int16 BE, -1 = UTC); Int: (1 << 1 | sign) then the
//     magnitude big-endian;
//   * type definitions precede the first value of a type on an encoder, outer type
//     first, then its components in field order; ids: a struct takes the next id
//     when it is first seen, before its fields; a slice after its element; the
//     first user id in a process is 65.
// Type ids are process-global in Go, so bytes depend on which types a process used
// first: the encoder takes the first id as a parameter (65: a fresh process whose
// first gob type is this one).  The decoder reads any ids: it follows the type
// definitions in the stream and matches fields by name, as gob does.
// Parity: the reference's own tests for this path are round trips
// (TestMarshallBody, TestMarshallEvent, TestWireEvent: event_test.go:34-144); no
// golden bytes exist in the reference, so byte-level parity is unpinned beyond
// the format restated here (tests/test_gob.py: round trips, the spec's integer
// and string encodings, an independent Python codec).
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/hge.h"

namespace {

// ------------------------------------------------------------------ encoding
struct Buf {
  std::vector<uint8_t> b;
  void u(uint64_t x) {
    if (x < 128) {
      b.push_back((uint8_t)x);
      return;
    }
    uint8_t t[8];
    int k = 0;
    while (x) {
      t[k++] = (uint8_t)(x & 0xFF);
      x >>= 8;
    }
    b.push_back((uint8_t)(256 - k));
    for (int i = k - 1; i >= 0; i--) b.push_back(t[i]);
  }
  void i(int64_t v) { u(v < 0 ? ((uint64_t)(~v) << 1) | 1 : (uint64_t)v << 1); }
  void bytes(const uint8_t* p, size_t n) {
    u(n);
    b.insert(b.end(), p, p + n);
  }
  void str(const std::string& s) { bytes((const uint8_t*)s.data(), s.size()); }
};

// one message: uint length + payload
void message(std::vector<uint8_t>& out, const Buf& m) {
  Buf l;
  l.u(m.b.size());
  out.insert(out.end(), l.b.begin(), l.b.end());
  out.insert(out.end(), m.b.begin(), m.b.end());
}

// struct encoder state: field deltas
struct Fields {
  Buf& b;
  int last = -1;
  explicit Fields(Buf& bb) : b(bb) {}
  void at(int f) {
    b.u((uint64_t)(f - last));
    last = f;
  }
  void end() { b.u(0); }
};

// wireType definitions (wireType{ArrayT 0, SliceT 1, StructT 2, MapT 3, GobEncoderT 4})
void def_struct(std::vector<uint8_t>& out, int id, const char* name,
                const std::vector<std::pair<std::string, int>>& fields) {
  Buf m;
  m.i(-id);
  Fields wt(m);
  wt.at(2);  // StructT
  {
    Fields st(m);
    st.at(0);  // CommonType
    {
      Fields ct(m);
      ct.at(0);
      m.str(name);
      ct.at(1);
      m.i(id);
      ct.end();
    }
    st.at(1);  // Field []*fieldType
    m.u(fields.size());
    for (const auto& f : fields) {
      Fields ft(m);
      ft.at(0);
      m.str(f.first);
      ft.at(1);
      m.i(f.second);
      ft.end();
    }
    st.end();
  }
  wt.end();
  message(out, m);
}
void def_slice(std::vector<uint8_t>& out, int id, const char* name, int elem) {
  Buf m;
  m.i(-id);
  Fields wt(m);
  wt.at(1);  // SliceT
  {
    Fields sl(m);
    sl.at(0);
    {
      Fields ct(m);
      ct.at(0);
      m.str(name);
      ct.at(1);
      m.i(id);
      ct.end();
    }
    sl.at(1);
    m.i(elem);
    sl.end();
  }
  wt.end();
  message(out, m);
}
void def_gobenc(std::vector<uint8_t>& out, int id, const char* name) {
  Buf m;
  m.i(-id);
  Fields wt(m);
  wt.at(4);  // GobEncoderT
  {
    Fields ge(m);
    ge.at(0);
    {
      Fields ct(m);
      ct.at(0);
      m.str(name);
      ct.at(1);
      m.i(id);
      ct.end();
    }
    ge.end();
  }
  wt.end();
  message(out, m);
}

constexpr int T_INT = 2, T_STRING = 6, T_BYTES = 5;
constexpr int64_t UNIX_TO_GO = 62135596800LL;  // seconds from year 1 to 1970

std::vector<uint8_t> time_bytes(int64_t unix_sec, int32_t nsec, int16_t offset_min) {
  const int64_t s = unix_sec + UNIX_TO_GO;
  std::vector<uint8_t> t = {1};
  for (int k = 7; k >= 0; k--) t.push_back((uint8_t)((uint64_t)s >> (8 * k)));
  for (int k = 3; k >= 0; k--) t.push_back((uint8_t)((uint32_t)nsec >> (8 * k)));
  t.push_back((uint8_t)((uint16_t)offset_min >> 8));
  t.push_back((uint8_t)((uint16_t)offset_min));
  return t;
}
std::vector<uint8_t> bigint_bytes(const uint8_t* mag, int len) {
  int a = 0;
  while (a < len && mag[a] == 0) a++;  // minimal magnitude
  std::vector<uint8_t> v = {2};      // version 1 << 1, non-negative
  v.insert(v.end(), mag + a, mag + len);
  return v;
}

void put_time(Fields& f, Buf& m, int field, const hge_gob_time& t) {
  if (!t.set) return;  // the zero Time is omitted
  f.at(field);
  const std::vector<uint8_t> tb = time_bytes(t.unix_sec, t.nsec, t.offset_min);
  m.bytes(tb.data(), tb.size());
}

void put_txs(Fields& f, Buf& m, int field, const uint8_t* tx, const int64_t* tx_off, int64_t first, int32_t count) {
  if (count <= 0) return;
  f.at(field);
  m.u((uint64_t)count);
  for (int32_t k = 0; k < count; k++) {
    const int64_t a = tx_off[first + k], b = tx_off[first + k + 1];
    m.bytes(tx + a, (size_t)(b - a));
  }
}

// ------------------------------------------------------------------ decoding
struct Reader {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  uint64_t u() {
    if (pos >= n) return fail();
    const uint8_t c = p[pos++];
    if (c < 128) return c;
    const int k = 256 - c;
    if (k > 8 || pos + k > n) return fail();
    uint64_t x = 0;
    for (int q = 0; q < k; q++) x = (x << 8) | p[pos++];
    return x;
  }
  int64_t i() {
    const uint64_t x = u();
    return (x & 1) ? ~(int64_t)(x >> 1) : (int64_t)(x >> 1);
  }
  bool take(size_t len, const uint8_t** out) {
    if (!ok || pos + len > n) {
      ok = false;
      return false;
    }
    *out = p + pos;
    pos += len;
    return true;
  }
  std::string str() {
    const size_t len = (size_t)u();
    const uint8_t* q = nullptr;
    if (!take(len, &q)) return std::string();
    return std::string((const char*)q, len);
  }
  uint64_t fail() {
    ok = false;
    return 0;
  }
};

enum Kind { K_STRUCT, K_SLICE, K_GOBENC, K_MAP, K_ARRAY };
struct TypeDef {
  Kind kind = K_STRUCT;
  std::string name;
  std::vector<std::pair<std::string, int>> fields;  // struct
  int elem = 0, key = 0;                            // slice / map / array
  int64_t len = 0;                                  // array
};

struct Decoder {
  std::map<int, TypeDef> types;
  // outputs
  hge_wire_event* ev;
  int64_t cap_ev, n_ev = 0;
  uint8_t* txb;
  int64_t cap_b, n_b = 0;
  int64_t* tx_off;
  int64_t cap_tx, n_tx = 0;
  bool overflow = false;

  // CommonType {Name, Id}
  void common(Reader& r, std::string& name, int& id) {
    for (int f = -1;;) {
      const int64_t d = (int64_t)r.u();
      if (!r.ok || d == 0) return;
      f += (int)d;
      if (f == 0) name = r.str();
      else if (f == 1) id = (int)r.i();
      else { r.fail(); return; }
    }
  }
  // a wireType value
  bool wiretype(Reader& r, int id) {
    TypeDef t;
    int kind = -1;
    for (int f = -1;;) {
      const int64_t d = (int64_t)r.u();
      if (!r.ok) return false;
      if (d == 0) break;
      f += (int)d;
      kind = f;
      int cid = 0;
      for (int g = -1;;) {  // the pointed-to type struct
        const int64_t e = (int64_t)r.u();
        if (!r.ok) return false;
        if (e == 0) break;
        g += (int)e;
        if (g == 0) {
          common(r, t.name, cid);
        } else if (f == 2 && g == 1) {  // structType.Field
          const uint64_t nf = r.u();
          for (uint64_t k = 0; k < nf && r.ok; k++) {
            std::string fname;
            int fid = 0;
            common(r, fname, fid);  // fieldType has the same shape {Name, Id}
            t.fields.push_back({fname, fid});
          }
        } else if ((f == 1 || f == 0) && g == 1) {  // sliceType.Elem / arrayType.Elem
          t.elem = (int)r.i();
        } else if (f == 0 && g == 2) {  // arrayType.Len
          t.len = r.i();
        } else if (f == 3 && g == 1) {
          t.key = (int)r.i();
        } else if (f == 3 && g == 2) {
          t.elem = (int)r.i();
        } else {
          return false;
        }
      }
    }
    switch (kind) {
      case 0: t.kind = K_ARRAY; break;
      case 1: t.kind = K_SLICE; break;
      case 2: t.kind = K_STRUCT; break;
      case 3: t.kind = K_MAP; break;
      case 4: case 5: case 6: t.kind = K_GOBENC; break;
      default: return false;
    }
    types[id] = t;
    return true;
  }

  // skip or capture one value of type id; `out` (a WireEvent under construction)
  // gets the fields it knows by name
  struct Capture {
    hge_wire_event* w = nullptr;
    std::vector<std::vector<uint8_t>>* txs = nullptr;
  };
  bool value(Reader& r, int id, const std::string& fname, Capture cap, int depth) {
    if (depth > 16) return false;
    switch (id) {
      case 1: case 3: {  // bool, uint
        const uint64_t x = r.u();
        (void)x;
        return r.ok;
      }
      case T_INT: {
        const int64_t x = r.i();
        if (cap.w) {
          if (fname == "SelfParentIndex") cap.w->self_parent_index = x;
          else if (fname == "OtherParentCreatorID") cap.w->other_parent_creator_id = x;
          else if (fname == "OtherParentIndex") cap.w->other_parent_index = x;
          else if (fname == "CreatorID") cap.w->creator_id = x;
          else if (fname == "Index") cap.w->index = x;
        }
        return r.ok;
      }
      case 4: {  // float: a uint
        r.u();
        return r.ok;
      }
      case T_BYTES: case T_STRING: {
        const size_t len = (size_t)r.u();
        const uint8_t* q = nullptr;
        if (!r.take(len, &q)) return false;
        if (cap.txs && id == T_BYTES) cap.txs->emplace_back(q, q + len);
        return true;
      }
      default: break;
    }
    auto it = types.find(id);
    if (it == types.end()) return false;
    const TypeDef& t = it->second;
    if (t.kind == K_GOBENC) {
      const size_t len = (size_t)r.u();
      const uint8_t* q = nullptr;
      if (!r.take(len, &q)) return false;
      if (cap.w && t.name == "Time" && fname == "Timestamp" && len >= 15 && q[0] >= 1) {
        int64_t s = 0;
        for (int k = 1; k <= 8; k++) s = (s << 8) | q[k];
        uint32_t ns = 0;
        for (int k = 9; k <= 12; k++) ns = (ns << 8) | q[k];
        cap.w->timestamp.set = 1;
        cap.w->timestamp.unix_sec = s - UNIX_TO_GO;
        cap.w->timestamp.nsec = (int32_t)ns;
        cap.w->timestamp.offset_min = (int16_t)(((uint16_t)q[13] << 8) | q[14]);
      } else if (cap.w && t.name == "Int" && (fname == "R" || fname == "S") && len >= 1) {
        uint8_t* dst = fname == "R" ? cap.w->r : cap.w->s;
        const size_t m = len - 1;
        if (m > 32 || (q[0] & 1)) return false;  // P-256 signature halves are < 2^256, >= 0
        memset(dst, 0, 32);
        memcpy(dst + 32 - m, q + 1, m);
        (fname == "R" ? cap.w->r_set : cap.w->s_set) = 1;
      }
      return true;
    }
    if (t.kind == K_SLICE || t.kind == K_ARRAY) {
      const uint64_t cnt = r.u();
      if (!r.ok || cnt > r.n) return false;
      Capture sub;
      if (cap.w && fname == "Transactions") sub.txs = cap.txs;
      for (uint64_t k = 0; k < cnt; k++)
        if (!value(r, t.elem, fname, sub, depth + 1)) return false;
      return true;
    }
    if (t.kind == K_MAP) {
      const uint64_t cnt = r.u();
      if (!r.ok || cnt > r.n) return false;
      for (uint64_t k = 0; k < cnt; k++)
        if (!value(r, t.key, "", Capture(), depth + 1) || !value(r, t.elem, "", Capture(), depth + 1)) return false;
      return true;
    }
    // struct: a WireEvent is captured (its Body's fields land in the same record)
    hge_wire_event we;
    std::vector<std::vector<uint8_t>> txs;
    Capture mine = cap;
    const bool is_event = t.name == "WireEvent";
    if (is_event) {
      memset(&we, 0, sizeof(we));
      mine.w = &we;
      mine.txs = &txs;
    }
    for (int f = -1;;) {
      const int64_t d = (int64_t)r.u();
      if (!r.ok) return false;
      if (d == 0) break;
      f += (int)d;
      if (f < 0 || f >= (int)t.fields.size()) return false;
      if (!value(r, t.fields[(size_t)f].second, t.fields[(size_t)f].first, mine, depth + 1)) return false;
    }
    if (is_event) emit(we, txs);
    return true;
  }
  void emit(hge_wire_event& we, const std::vector<std::vector<uint8_t>>& txs) {
    int64_t nb = 0;
    for (const auto& x : txs) nb += (int64_t)x.size();
    if (n_ev >= cap_ev || n_tx + (int64_t)txs.size() > cap_tx || n_b + nb > cap_b) {
      overflow = true;
      n_ev++;
      n_tx += (int64_t)txs.size();
      n_b += nb;
      return;
    }
    we.tx_first = n_tx;
    we.tx_count = (int32_t)txs.size();
    for (const auto& x : txs) {
      if (tx_off) tx_off[n_tx] = n_b;
      if (!x.empty()) memcpy(txb + n_b, x.data(), x.size());
      n_b += (int64_t)x.size();
      n_tx++;
    }
    if (tx_off) tx_off[n_tx] = n_b;
    ev[n_ev++] = we;
  }
};

}  // namespace

extern "C" {

int hge_gob_encode_wire_events(const hge_wire_event* ev, int64_t n, const uint8_t* tx, const int64_t* tx_off,
                               int32_t first_type_id, uint8_t* out, int64_t cap, int64_t* n_out) {
  if (!n_out || n < 0 || (n > 0 && !ev) || first_type_id < 65) return HGE_ERR_ARG;
  std::vector<uint8_t> s;
  // ids as a fresh encoding of WireEvent assigns them: WireEvent, WireBody, [][]uint8, Time, Int
  const int tWE = first_type_id, tWB = tWE + 1, tTX = tWE + 2, tTime = tWE + 3, tInt = tWE + 4;
  if (n > 0) {
    def_struct(s, tWE, "WireEvent", {{"Body", tWB}, {"R", tInt}, {"S", tInt}});
    def_struct(s, tWB, "WireBody",
               {{"Transactions", tTX}, {"SelfParentIndex", T_INT}, {"OtherParentCreatorID", T_INT},
                {"OtherParentIndex", T_INT}, {"CreatorID", T_INT}, {"Timestamp", tTime}, {"Index", T_INT}});
    def_slice(s, tTX, "[][]uint8", T_BYTES);
    def_gobenc(s, tTime, "Time");
    def_gobenc(s, tInt, "Int");
  }
  for (int64_t k = 0; k < n; k++) {
    const hge_wire_event& e = ev[k];
    if (e.tx_count > 0 && (!tx || !tx_off)) return HGE_ERR_ARG;
    Buf m;
    m.i(tWE);
    Fields we(m);
    we.at(0);  // Body (a struct: always sent)
    {
      Fields b(m);
      put_txs(b, m, 0, tx, tx_off, e.tx_first, e.tx_count);
      const int64_t iv[4] = {e.self_parent_index, e.other_parent_creator_id, e.other_parent_index, e.creator_id};
      for (int q = 0; q < 4; q++)
        if (iv[q] != 0) {
          b.at(1 + q);
          m.i(iv[q]);
        }
      put_time(b, m, 5, e.timestamp);
      if (e.index != 0) {
        b.at(6);
        m.i(e.index);
      }
      b.end();
    }
    if (e.r_set) {
      we.at(1);
      const std::vector<uint8_t> v = bigint_bytes(e.r, 32);
      m.bytes(v.data(), v.size());
    }
    if (e.s_set) {
      we.at(2);
      const std::vector<uint8_t> v = bigint_bytes(e.s, 32);
      m.bytes(v.data(), v.size());
    }
    we.end();
    message(s, m);
  }
  *n_out = (int64_t)s.size();
  if ((int64_t)s.size() > cap || (!out && !s.empty())) return cap == 0 && !out ? HGE_OK : HGE_ERR_ARG;
  if (!s.empty()) memcpy(out, s.data(), s.size());
  return HGE_OK;
}

int hge_gob_decode_wire_events(const uint8_t* buf, int64_t len, hge_wire_event* ev, int64_t cap_ev, uint8_t* tx,
                               int64_t cap_bytes, int64_t* tx_off, int64_t cap_tx, int64_t* n_ev, int64_t* n_tx,
                               int64_t* n_bytes) {
  if (!n_ev || !n_tx || !n_bytes || len < 0 || (len > 0 && !buf)) return HGE_ERR_ARG;
  Decoder d;
  d.ev = ev;
  d.cap_ev = ev ? cap_ev : 0;
  d.txb = tx;
  d.cap_b = tx ? cap_bytes : 0;
  d.tx_off = tx_off;
  d.cap_tx = tx_off ? cap_tx - 1 : 0;
  if (tx_off && cap_tx > 0) tx_off[0] = 0;
  Reader top{buf, (size_t)len};
  while (top.ok && top.pos < top.n) {
    const size_t mlen = (size_t)top.u();
    const uint8_t* q = nullptr;
    if (!top.take(mlen, &q)) return HGE_ERR_ARG;
    Reader r{q, mlen};
    const int64_t id = r.i();
    if (!r.ok) return HGE_ERR_ARG;
    if (id < 0) {
      if (!d.wiretype(r, (int)-id)) return HGE_ERR_ARG;
      continue;
    }
    // a top-level value; a non-struct one starts with a 0 delta (gob's singleton field)
    auto it = d.types.find((int)id);
    const bool is_struct = it != d.types.end() && it->second.kind == K_STRUCT;
    if (!is_struct && r.u() != 0) return HGE_ERR_ARG;
    if (!d.value(r, (int)id, "", Decoder::Capture(), 0)) return HGE_ERR_ARG;
  }
  if (!top.ok) return HGE_ERR_ARG;
  *n_ev = d.n_ev;
  *n_tx = d.n_tx;
  *n_bytes = d.n_b;
  return d.overflow ? HGE_ERR_NOT_FOUND : HGE_OK;
}

int hge_gob_encode_event_body(const hge_gob_body* body, const uint8_t* tx, const int64_t* tx_off,
                              const uint8_t* parents, const int64_t* parent_off, int32_t first_type_id,
                              uint8_t* out, int64_t cap, int64_t* n_out) {
  if (!body || !n_out || first_type_id < 65) return HGE_ERR_ARG;
  // EventBody, [][]uint8, []string, Time (fresh ids in field order; Creator is []uint8 = id 5)
  const int tEB = first_type_id, tTX = tEB + 1, tPS = tEB + 2, tTime = tEB + 3;
  std::vector<uint8_t> s;
  def_struct(s, tEB, "EventBody",
             {{"Transactions", tTX}, {"Parents", tPS}, {"Creator", T_BYTES}, {"Timestamp", tTime}, {"Index", T_INT}});
  def_slice(s, tTX, "[][]uint8", T_BYTES);
  def_slice(s, tPS, "[]string", T_STRING);
  def_gobenc(s, tTime, "Time");
  Buf m;
  m.i(tEB);
  Fields b(m);
  if (body->tx_count > 0 && (!tx || !tx_off)) return HGE_ERR_ARG;
  put_txs(b, m, 0, tx, tx_off, 0, body->tx_count);
  if (body->n_parents > 0) {
    if (!parents || !parent_off) return HGE_ERR_ARG;
    b.at(1);
    m.u((uint64_t)body->n_parents);
    for (int32_t k = 0; k < body->n_parents; k++)
      m.bytes(parents + parent_off[k], (size_t)(parent_off[k + 1] - parent_off[k]));
  }
  if (body->creator_len > 0) {
    b.at(2);
    m.bytes(body->creator, (size_t)body->creator_len);
  }
  put_time(b, m, 3, body->timestamp);
  if (body->index != 0) {
    b.at(4);
    m.i(body->index);
  }
  b.end();
  message(s, m);
  *n_out = (int64_t)s.size();
  if ((int64_t)s.size() > cap || !out) return out ? HGE_ERR_ARG : HGE_OK;
  memcpy(out, s.data(), s.size());
  return HGE_OK;
}

}  // extern "C"
