// hge_ingest.cpp — the host half of InsertEvent: batched
// signature verification and hashing on host cores, overlapped with the device.
//
// Reference front half (mpitid/babble):
//   * EventBody.Hash = SHA-256 of the body's gob bytes (hashgraph/event.go:44-66);
//   * Event.Verify: the creator key is Body.Creator, an uncompressed P-256 point
//     (crypto.ToECDSAPub, crypto/utils.go:40-46), and the signature (R, S) must
//     verify over the body hash (crypto.Verify -> ecdsa.Verify, event.go:140-150);
//   * InsertEvent refuses an event whose signature fails ("Invalid signature",
//     hashgraph.go:330-336) before FromParentsLatest.
// The consensus engine never needs the bytes again: it takes hge_event records.
//
// hge_verify_events is pure host code (OpenSSL libcrypto: SHA-256 and ECDSA
// P-256 verification), thread-safe and independent of any engine handle.
// hge_ingest drives a stream through one engine the way node/core.go:179-202
// does -- insert a batch, run consensus -- while a worker pool verifies the next
// batch: the host crypto and the device consensus overlap.
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <openssl/sha.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/hge.h"

namespace {

// EC_KEY per distinct creator key, per thread (verification only reads it)
struct KeyCache {
  std::unordered_map<std::string, EC_KEY*> m;
  const EC_GROUP* grp = nullptr;
  ~KeyCache() {
    for (auto& kv : m)
      if (kv.second) EC_KEY_free(kv.second);
  }
  EC_KEY* get(const uint8_t* pub) {
    std::string k((const char*)pub, 65);
    auto it = m.find(k);
    if (it != m.end()) return it->second;
    EC_KEY* key = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
    EC_POINT* pt = key ? EC_POINT_new(EC_KEY_get0_group(key)) : nullptr;
    // elliptic.Unmarshal (Go): 0x04 || X || Y with the point on the curve, else no key
    bool ok = pt && pub[0] == 0x04 &&
              EC_POINT_oct2point(EC_KEY_get0_group(key), pt, pub, 65, nullptr) == 1 &&
              EC_KEY_set_public_key(key, pt) == 1;
    if (pt) EC_POINT_free(pt);
    if (!ok && key) {
      EC_KEY_free(key);
      key = nullptr;
    }
    m.emplace(std::move(k), key);
    return key;
  }
};

int verify_one(KeyCache& kc, const uint8_t* body, size_t len, const uint8_t* pub, const uint8_t* sig,
               uint8_t* hash) {
  SHA256(body, len, hash);
  EC_KEY* key = kc.get(pub);
  if (!key) return 0;
  // ecdsa.Verify: r, s must lie in [1, n-1]; OpenSSL checks the same
  BIGNUM* r = BN_bin2bn(sig, 32, nullptr);
  BIGNUM* s = BN_bin2bn(sig + 32, 32, nullptr);
  ECDSA_SIG* es = ECDSA_SIG_new();
  if (!r || !s || !es) {
    BN_free(r);
    BN_free(s);
    ECDSA_SIG_free(es);
    return 0;
  }
  ECDSA_SIG_set0(es, r, s);
  const int v = ECDSA_do_verify(hash, 32, es, key);
  ECDSA_SIG_free(es);
  return v == 1 ? 1 : 0;
}

// a fixed pool of workers; run(n, f) calls f(worker, i) for i in [0, n) and returns
// when every call is done (the caller's thread takes part)
class Pool {
 public:
  explicit Pool(int nthreads) : caches_(std::max(1, nthreads)) {
    for (int w = 1; w < (int)caches_.size(); w++) workers_.emplace_back([this, w] { loop(w); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return (int)caches_.size(); }
  KeyCache& cache(int w) { return caches_[w]; }
  // start a job without waiting (wait() joins it)
  void start(int64_t n, std::function<void(int, int64_t)> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = std::move(f);
      n_ = n;
      next_.store(0);
      pending_ = (int)workers_.size();
      gen_++;
    }
    cv_.notify_all();
  }
  void wait() {
    work(0);
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return pending_ == 0; });
  }
  void run(int64_t n, std::function<void(int, int64_t)> f) {
    start(n, std::move(f));
    wait();
  }

 private:
  void work(int w) {
    // small pieces: a consensus-call batch is only K events (16-256); spread it over every worker
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(64, n_ / (4 * (int64_t)caches_.size())));
    for (;;) {
      const int64_t i0 = next_.fetch_add(chunk);
      if (i0 >= n_) break;
      const int64_t i1 = std::min(n_, i0 + chunk);
      for (int64_t i = i0; i < i1; i++) job_(w, i);
    }
  }
  void loop(int w) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work(w);
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<KeyCache> caches_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::function<void(int, int64_t)> job_;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  int pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

int clamp_threads(int32_t threads) {
  if (threads <= 0) threads = (int32_t)std::max(1u, std::thread::hardware_concurrency());
  return std::min<int32_t>(threads, 256);
}

}  // namespace

extern "C" {

int hge_verify_events(int64_t n, const uint8_t* bodies, const int64_t* body_off, const uint8_t* pubs,
                      const uint8_t* sigs, int32_t threads, uint8_t* body_hash_out, int32_t* ok_out) {
  if (n < 0 || (n > 0 && (!bodies || !body_off || !pubs || !sigs || !ok_out))) return HGE_ERR_ARG;
  if (n == 0) return HGE_OK;
  for (int64_t i = 0; i < n; i++)
    if (body_off[i + 1] < body_off[i]) return HGE_ERR_ARG;
  Pool pool(clamp_threads(threads));
  pool.run(n, [&](int w, int64_t i) {
    uint8_t h[32];
    ok_out[i] = verify_one(pool.cache(w), bodies + body_off[i], (size_t)(body_off[i + 1] - body_off[i]),
                           pubs + 65 * i, sigs + 64 * i, h);
    if (body_hash_out) memcpy(body_hash_out + 32 * i, h, 32);
  });
  return HGE_OK;
}

int hge_sha256_batch(int64_t n, const uint8_t* data, const int64_t* off, int32_t threads, uint8_t* out) {
  if (n < 0 || (n > 0 && (!data || !off || !out))) return HGE_ERR_ARG;
  if (n == 0) return HGE_OK;
  for (int64_t i = 0; i < n; i++)
    if (off[i + 1] < off[i]) return HGE_ERR_ARG;
  Pool pool(clamp_threads(threads));
  pool.run(n, [&](int, int64_t i) { SHA256(data + off[i], (size_t)(off[i + 1] - off[i]), out + 32 * i); });
  return HGE_OK;
}

int hge_ingest(hge_engine* h, const hge_event* ev, int64_t n, const uint8_t* bodies, const int64_t* body_off,
               const uint8_t* keys, const uint8_t* sigs, int64_t k, int32_t threads, int32_t* status_out,
               int64_t* n_accepted, double* times_out) {
  if (!h || n < 0 || k <= 0 || (n > 0 && (!ev || !bodies || !body_off || !keys || !sigs))) return HGE_ERR_ARG;
  const int N = hge_participants(h);
  for (int64_t i = 0; i < n; i++)
    if (body_off[i + 1] < body_off[i]) return HGE_ERR_ARG;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  double verify_ms = 0, device_ms = 0, wait_ms = 0;
  if (n_accepted) *n_accepted = 0;
  Pool pool(clamp_threads(threads));
  std::vector<int32_t> ok(std::max<int64_t>(n, 1));
  const int64_t nb = (n + k - 1) / k;
  auto verify_batch = [&](int64_t b) {
    const int64_t lo = b * k, hi = std::min(n, lo + k);
    return [&, lo, hi](int w, int64_t i) {
      uint8_t hb[32];
      const int64_t e = lo + i;
      if (e >= hi) return;
      const int c = ev[e].creator;
      // no key for this id: let admission refuse it ("Could not find fake creator id")
      ok[e] = (c < 0 || c >= N) ? 1
                                : verify_one(pool.cache(w), bodies + body_off[e],
                                             (size_t)(body_off[e + 1] - body_off[e]), keys + 65 * (size_t)c,
                                             sigs + 64 * e, hb);
    };
  };
  auto tv = clk::now();
  if (nb > 0) pool.run(std::min(k, n), verify_batch(0));
  verify_ms += std::chrono::duration<double, std::milli>(clk::now() - tv).count();
  int64_t acc = 0;
  int rc = HGE_OK;
  for (int64_t b = 0; b < nb && rc == HGE_OK; b++) {
    const int64_t lo = b * k, hi = std::min(n, lo + k);
    // the next batch's signatures on the workers while this one goes through the device
    const bool more = b + 1 < nb;
    if (more) pool.start(std::min(k, n - hi), verify_batch(b + 1));
    int64_t m = lo;
    while (m < hi && ok[m]) m++;  // InsertEvent stops at the first invalid signature
    const auto td = clk::now();
    int64_t got = 0;
    if (m > lo) rc = hge_insert_events(h, ev + lo, m - lo, status_out ? status_out + lo : nullptr, &got);
    acc += got;
    if (rc == HGE_OK) rc = hge_run_consensus(h, nullptr, 0, nullptr);
    device_ms += std::chrono::duration<double, std::milli>(clk::now() - td).count();
    if (rc == HGE_OK && m < hi) {
      if (status_out) status_out[m] = HGE_ERR_SIGNATURE;
      rc = HGE_ERR_SIGNATURE;
    }
    if (more) {
      const auto tw = clk::now();
      pool.wait();  // the caller's thread helps finish the next batch
      wait_ms += std::chrono::duration<double, std::milli>(clk::now() - tw).count();
    }
  }
  if (n_accepted) *n_accepted = acc;
  if (times_out) {
    times_out[0] = verify_ms + wait_ms;  // host time spent on verification not hidden behind the device
    times_out[1] = device_ms;            // insert + consensus calls
    times_out[2] = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  }
  return rc;
}

}  // extern "C"
