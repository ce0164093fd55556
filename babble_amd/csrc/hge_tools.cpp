// hge_tools.cpp — synthetic signed streams for tests and the bench (not the
// product path; build/libhge_tools.so).  The counterpart of what a babble node
// does before InsertEvent: every participant has an ECDSA P-256 key
// (crypto.GenerateECDSAKey, crypto/utils.go:36-38) and signs SHA-256 of each
// event body (Event.Sign, hashgraph/event.go:131-138).  Keys are derived from a
// seed so runs are reproducible; signatures use OpenSSL's random nonces, as Go's
// ecdsa.Sign does (rand.Reader).
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// private key i = SHA-256("hge-key" || seed || i) reduced into [1, n-1]
EC_KEY* derive_key(uint64_t seed, int32_t i) {
  uint8_t msg[7 + 8 + 4], d[32];
  memcpy(msg, "hge-key", 7);
  memcpy(msg + 7, &seed, 8);
  memcpy(msg + 15, &i, 4);
  SHA256(msg, sizeof msg, d);
  EC_KEY* key = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
  const EC_GROUP* g = EC_KEY_get0_group(key);
  BIGNUM* order = BN_new();
  EC_GROUP_get_order(g, order, nullptr);
  BIGNUM* k = BN_bin2bn(d, 32, nullptr);
  BN_CTX* ctx = BN_CTX_new();
  BN_sub_word(order, 1);
  BN_mod(k, k, order, ctx);
  BN_add_word(k, 1);
  EC_POINT* pub = EC_POINT_new(g);
  EC_POINT_mul(g, pub, k, nullptr, nullptr, ctx);
  EC_KEY_set_private_key(key, k);
  EC_KEY_set_public_key(key, pub);
  EC_POINT_free(pub);
  BN_free(k);
  BN_free(order);
  BN_CTX_free(ctx);
  return key;
}

}  // namespace

extern "C" {

// pubs_out: n x 65 bytes (uncompressed points, crypto.FromECDSAPub)
int hgt_keys(int32_t n, uint64_t seed, uint8_t* pubs_out) {
  for (int32_t i = 0; i < n; i++) {
    EC_KEY* key = derive_key(seed, i);
    EC_POINT_point2oct(EC_KEY_get0_group(key), EC_KEY_get0_public_key(key), POINT_CONVERSION_UNCOMPRESSED,
                       pubs_out + 65 * (size_t)i, 65, nullptr);
    EC_KEY_free(key);
  }
  return 0;
}

// sigs_out: m x 64 bytes (r || s, big-endian) over SHA-256 of each body, signed by
// key creator[i]; returns 0, or -1 on a bad argument
int hgt_sign(int64_t m, const uint8_t* bodies, const int64_t* off, const int32_t* creator, int32_t nkeys,
             uint64_t seed, int32_t threads, uint8_t* sigs_out) {
  if (m < 0 || nkeys <= 0) return -1;
  threads = std::max(1, std::min<int32_t>(threads, 64));
  std::atomic<int64_t> next{0};
  std::atomic<int> bad{0};
  auto work = [&] {
    // every thread signs with keys of its own (no shared EC_KEY state)
    std::vector<EC_KEY*> keys(nkeys);
    for (int32_t i = 0; i < nkeys; i++) keys[i] = derive_key(seed, i);
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= m) break;
      const int32_t c = creator[i];
      if (c < 0 || c >= nkeys) {
        bad = 1;
        continue;
      }
      uint8_t h[32];
      SHA256(bodies + off[i], (size_t)(off[i + 1] - off[i]), h);
      ECDSA_SIG* s = ECDSA_do_sign(h, 32, keys[c]);
      const BIGNUM *r, *ss;
      ECDSA_SIG_get0(s, &r, &ss);
      BN_bn2binpad(r, sigs_out + 64 * i, 32);
      BN_bn2binpad(ss, sigs_out + 64 * i + 32, 32);
      ECDSA_SIG_free(s);
    }
    for (auto* k : keys) EC_KEY_free(k);
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < threads; t++) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  return bad ? -1 : 0;
}

}  // extern "C"
