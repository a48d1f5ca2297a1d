// Host-side packing of a caller's batch into the compact layout (bh_cbatch)
// inside library-owned page-locked staging: the per-batch work a Go
// BatchVerify would otherwise do itself on one goroutine --
// key de-duplication, a u32 key index per record, and the copy of every
// signature and message out of the caller's (pageable, scattered) buffers.
// measured end to end by bench.py host_path_e2e.
//
// Two passes over the records, both on a pool of worker threads:
//   plan: the lengths only -- byte offsets of every (chunk, thread) block;
//   fill: per record its lengths, its key and its signature / message bytes.
//      With de-duplication a lock-free open-addressing table over the keys
//      hands out key ids (first claimant copies the key; ids come in
//      per-thread blocks, so the key array has a few zero-filled holes);
//      without it (a batch of mostly distinct keys: config 5) each record's
//      key is copied in record order. The bytes stream chunk by chunk; a
//      chunk's bytes are contiguous in the output, so the caller starts its
//      H2D copy while the workers fill the next one (on_chunk).
// Whether to de-duplicate is decided from a strided sample of the keys (the
// distinct count a uniform draw from D keys would show); a table that fills
// anyway is rebuilt at its largest size, so the result never depends on the
// estimate. Key ids are assigned in claim order: any assignment verifies the
// same (record i has key keys[key_idx[i]]).
//
// Pure host code (no HIP): tests/native/hostsim.cpp compiles it for the
// CPU tests (tests/test_pack.py).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>
#ifdef __linux__
#include <sched.h>
#endif
#if defined(__SSE2__)
#include <emmintrin.h>
#endif

namespace bh {
namespace pack {

// ---- worker pool -------------------------------------------------------------
// Persistent threads; run(fn) calls fn(t) for t in [0, threads) on the workers
// and returns when all are done. One job at a time (callers serialise).
class Pool {
 public:
  explicit Pool(int threads) : n_(std::max(1, threads)) {
    for (int t = 0; t < n_; t++) th_.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      quit_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  int threads() const { return n_; }
  // start fn on every worker; wait() joins
  void start(std::function<void(int)> fn) {
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = std::move(fn);
      left_ = n_;
      gen_++;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return left_ == 0; });
  }
  void run(std::function<void(int)> fn) {
    start(std::move(fn));
    wait();
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void(int)> fn;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (quit_) return;
        fn = fn_;
      }
      fn(t);
      std::lock_guard<std::mutex> g(mu_);
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::function<void(int)> fn_;
  uint64_t gen_ = 0;
  int left_ = 0;
  bool quit_ = false;
};

// ---- key hashing / de-duplication ----------------------------------------------
inline uint64_t load64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

// 64-bit mix of the key: X's first 8 bytes and Y's first 8 (a valid key's
// coordinates are uniformly spread, and Y separates the two points of one X).
// Equal keys always collide; keys crafted to share these bytes only lengthen
// probe runs -- past the probe limit the table is rebuilt and then dedup is
// dropped, so the packed batch stays exact whatever the keys (every match is
// confirmed on all 64 bytes).
inline uint64_t key_hash(const uint8_t* k) {
  uint64_t h = (load64(k) ^ 0x9E3779B97F4A7C15ull) * 0xff51afd7ed558ccdull;
  h = (h ^ (h >> 29) ^ load64(k + 32)) * 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 32);
}

// Distinct keys a uniform draw from D keys shows in s samples: D (1 - e^(-s/D)).
// Inverse by bisection; d_s == s (no repeat seen): infinity (returned as 0).
inline double estimate_distinct(size_t s, size_t d_s) {
  if (d_s >= s) return 0.0;
  double lo = (double)d_s, hi = 1e15;
  for (int it = 0; it < 200; it++) {
    const double mid = 0.5 * (lo + hi);
    if (mid * -std::expm1(-(double)s / mid) < (double)d_s) lo = mid;
    else hi = mid;
  }
  return hi;
}

constexpr uint32_t kBusy = 0xFFFFFFFFu;

// Lock-free insert-or-find. slots: cap (power of two) u64 words, 0 = empty,
// else tag (hash high word | 1) << 32 | key id (kBusy while the claimant
// copies its key). keys: the dense key array (64 B per id) the compares read,
// in ordinary cached memory; keys_out: its copy in the upload staging, only
// written (page-locked host memory reads back uncached). Returns the key's
// id, or kBusy when the table is full / the id range exhausted / probing
// exceeds max_probe (the caller rebuilds larger).
// Ids come from per-thread blocks of kIdBlock taken from `next`, so threads
// inserting at once do not contend on one counter; a block's unused tail is a
// hole in the key array (zero-filled, referenced by no record).
constexpr uint32_t kIdBlock = 64;
struct IdBlock {
  uint32_t next = 0, end = 0, size = kIdBlock;
};
inline uint32_t insert_key(std::atomic<uint64_t>* slots, uint64_t cap, std::atomic<uint32_t>* next,
                           uint32_t max_ids, uint8_t* keys, uint8_t* keys_out,
                           const uint8_t* key, uint64_t h, IdBlock* blk) {
  const uint64_t tag = ((h >> 32) | 1u) << 32;
  uint64_t p = h & (cap - 1);
  for (uint64_t probe = 0; probe < cap && probe < 4096; probe++, p = (p + 1) & (cap - 1)) {
    uint64_t v = slots[p].load(std::memory_order_acquire);
    if (v == 0) {
      uint64_t want = tag | kBusy;
      if (slots[p].compare_exchange_strong(v, want, std::memory_order_acq_rel)) {
        if (blk->next == blk->end) {
          blk->next = next->fetch_add(blk->size, std::memory_order_relaxed);
          blk->end = blk->next + blk->size;
        }
        const uint32_t id = blk->next++;
        if (id >= max_ids) {
          slots[p].store(tag | (kBusy - 1), std::memory_order_release);  // never matches a key
          return kBusy;
        }
        std::memcpy(keys + (size_t)id * 64, key, 64);
        std::memcpy(keys_out + (size_t)id * 64, key, 64);
        slots[p].store(tag | id, std::memory_order_release);
        return id;
      }
      // lost the race: v holds the winner's word
    }
    if ((v & 0xFFFFFFFF00000000ull) != tag) continue;
    uint32_t id = (uint32_t)v;
    while (id == kBusy) {  // the claimant is copying its key
      std::this_thread::yield();
      id = (uint32_t)slots[p].load(std::memory_order_acquire);
    }
    if (id < max_ids && std::memcmp(keys + (size_t)id * 64, key, 64) == 0) return id;
  }
  return kBusy;
}

// ---- streaming writer ------------------------------------------------------------
// Pass B's output is written once and read only by the DMA engine: records are
// gathered into a small cache-resident buffer and flushed to the destination
// with non-temporal 16-byte stores, so the destination lines are not first
// read into the cache (a normal store's read-for-ownership would add the
// whole output to the memory traffic again). The head up to 16-byte alignment
// and the final tail go through ordinary stores; fence() before the H2D.
class StreamWriter {
 public:
  explicit StreamWriter(uint8_t* dst) : dst_(dst) {}
  void put(const uint8_t* p, size_t len) {
    if (n_ + len > kBuf) flush(false);
    if (len > kBuf) {  // (not a record size this path sees; kept exact anyway)
      flush(true);
      std::memcpy(dst_, p, len);
      dst_ += len;
      return;
    }
    std::memcpy(buf_ + n_, p, len);
    n_ += len;
  }
  void finish() { flush(true); }
  static void fence() {
#if defined(__SSE2__)
    _mm_sfence();
#endif
  }

 private:
  void flush(bool all) {
    size_t k = 0;
#if defined(__SSE2__)
    const size_t head = std::min<size_t>((16 - ((uintptr_t)dst_ & 15)) & 15, n_);
    if (head) std::memcpy(dst_, buf_, head);
    k = head;
    for (; k + 16 <= n_; k += 16)
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst_ + k),
                       _mm_loadu_si128(reinterpret_cast<const __m128i*>(buf_ + k)));
#endif
    if (all) {
      std::memcpy(dst_ + k, buf_ + k, n_ - k);
      k = n_;
    }
    dst_ += k;
    std::memmove(buf_, buf_ + k, n_ - k);
    n_ -= k;
  }
  static constexpr size_t kBuf = 8192;
  uint8_t* dst_;
  size_t n_ = 0;
  alignas(64) uint8_t buf_[kBuf];
};

// ---- the packer ---------------------------------------------------------------
struct Out {
  uint8_t* keys = nullptr;      // >= m * 64 bytes
  uint32_t* key_idx = nullptr;  // m (written when Result::dedup)
  uint32_t* sig_len = nullptr;  // m
  uint32_t* msg_len = nullptr;  // m
};

struct Result {
  size_t nkeys = 0;
  bool dedup = false;          // key_idx written (keys[key_idx[i]] is record i's key);
                               // else keys hold one key per record
  bool fixed_msg = false;      // every message msg_stride bytes: msg_len not needed
  uint32_t msg_stride = 0;
  uint64_t sig_bytes = 0, msg_bytes = 0;
  int nchunks = 1;
  std::vector<uint64_t> sig_chunk, msg_chunk;  // nchunks + 1 byte offsets
  double est_distinct = 0;     // sample estimate (0: no repeat seen)
  int rebuilds = 0;            // table rebuilt at full size (estimate too low)
  bool dedup_dropped = false;  // rebuilt table overflowed too: identity indices
  double plan_ms = 0, fill_ms = 0;
};

// plan(): the dedup decision from a strided sample, then one pass over the
// lengths -- per (chunk, thread) block byte sums, their prefix offsets, the
// totals and the chunk bounds (the caller sizes its staging from these).
// fill(): ONE pass per record -- lengths, key (dedup probe or copy), and the
// signature / message bytes streamed to their final offsets -- so the dedup's
// table misses overlap the bandwidth-bound copy instead of adding to it;
// after chunk c is complete on every thread, on_chunk(c) runs on the calling
// thread (the H2D of its bytes) while the workers fill chunk c + 1.
// Src: key(i), sig(i), sig_len(i), msg(i), msg_len(i) for i in [lo, lo + m).
class Packer {
 public:
  explicit Packer(int threads) : pool_(threads) {}
  int threads() const { return pool_.threads(); }

  template <class Src>
  void plan(const Src& src, size_t lo, size_t m, Result* r, int force = -1) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    *r = Result{};
    lo_ = lo;
    m_ = m;
    bool dedup = false;
    double est = 0;
    if (force >= 0) {
      dedup = force == 1 && m > 0;
    } else if (m >= 64) {
      const size_t s = std::min<size_t>(m, 8192);
      std::vector<uint64_t> hs(s);
      for (size_t k = 0; k < s; k++) hs[k] = key_hash(src.key(lo + (k * m) / s));
      std::sort(hs.begin(), hs.end());
      const size_t ds = (size_t)(std::unique(hs.begin(), hs.end()) - hs.begin());
      est = estimate_distinct(s, ds);
      dedup = est > 0 && est * 2 <= (double)m;  // >= 2 uses per key on average
    } else {
      dedup = m > 1;
    }
    r->est_distinct = est;
    r->dedup = dedup;
    // chunks: ~16 MB of bytes each (from a sample of lengths), 1..16
    const int T = pool_.threads();
    uint64_t sample = 0;
    const size_t ns = std::min<size_t>(m, 1024);
    for (size_t k = 0; k < ns; k++) {
      const size_t i = lo + (k * m) / std::max<size_t>(ns, 1);
      sample += src.sig_len(i) + src.msg_len(i);
    }
    const double est_bytes = ns ? (double)sample * m / ns : 0.0;
    int K = (int)std::max(1.0, std::min(16.0, est_bytes / (16u << 20)));
    if (const char* e = getenv("BH_PACK_CHUNKS")) K = std::max(1, std::min(64, atoi(e)));
    r->nchunks = K;
    T_ = T;
    const size_t B = (size_t)K * T;
    boff_s_.assign(B + 1, 0);
    boff_m_.assign(B + 1, 0);
    len_min_.assign(T, UINT32_MAX);
    len_max_.assign(T, 0);
    pool_.run([&](int t) {
      uint32_t mn = UINT32_MAX, mx = 0;
      for (int c = 0; c < K; c++) {
        const size_t blk = (size_t)c * T + t;
        size_t a, b;
        brange(blk, &a, &b);
        uint64_t ss = 0, ms = 0;
        for (size_t i = a; i < b; i++) {
          const uint32_t ml = src.msg_len(i);
          ss += src.sig_len(i);
          ms += ml;
          mn = std::min(mn, ml);
          mx = std::max(mx, ml);
        }
        boff_s_[blk + 1] = ss;
        boff_m_[blk + 1] = ms;
      }
      len_min_[t] = mn;
      len_max_[t] = mx;
    });
    for (size_t k = 0; k < B; k++) {
      boff_s_[k + 1] += boff_s_[k];
      boff_m_[k + 1] += boff_m_[k];
    }
    r->sig_bytes = boff_s_[B];
    r->msg_bytes = boff_m_[B];
    r->sig_chunk.assign(K + 1, 0);
    r->msg_chunk.assign(K + 1, 0);
    for (int c = 0; c <= K; c++) {
      r->sig_chunk[c] = boff_s_[(size_t)c * T];
      r->msg_chunk[c] = boff_m_[(size_t)c * T];
    }
    uint32_t mn = UINT32_MAX, mx = 0;
    for (int t = 0; t < T; t++) {
      mn = std::min(mn, len_min_[t]);
      mx = std::max(mx, len_max_[t]);
    }
    r->fixed_msg = m > 0 && mn == mx;
    r->msg_stride = r->fixed_msg ? mn : 0;
    r->plan_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  }

  template <class Src>
  void fill(const Src& src, const Out& out, uint8_t* sig, uint8_t* msg, Result* r,
            const std::function<void(int)>& on_chunk) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const int T = T_, K = r->nchunks;
    const size_t lo = lo_, m = m_;
    bool dedup = r->dedup;
    if (dedup) size_table(r->est_distinct == 0, r->est_distinct);
    std::vector<std::atomic<int>> done(K);
    for (auto& x : done) x.store(0);
    pool_.start([&](int t) {
      IdBlock blk;  // small tables: small blocks, so holes never fill the id range
      blk.size = full_table_ ? 1u
                             : (uint32_t)std::max<uint64_t>(
                                   1, std::min<uint64_t>(kIdBlock, max_ids_ / (8 * T)));
      for (int c = 0; c < K; c++) {
        const size_t b0 = (size_t)c * T + t;
        size_t a, b;
        brange(b0, &a, &b);
        StreamWriter ws(sig + boff_s_[b0]), wm(msg + boff_m_[b0]);
        for (size_t g0 = a; g0 < b; g0 += kGroup) {
          const int cnt = (int)std::min<size_t>(kGroup, b - g0);
          if (dedup) keys_group(src, out, g0, cnt, &blk);
          for (int j = 0; j < cnt; j++) {
            const size_t i = g0 + j;
            const uint32_t sl = src.sig_len(i), ml = src.msg_len(i);
            out.sig_len[i - lo] = sl;
            out.msg_len[i - lo] = ml;
            if (!dedup) std::memcpy(out.keys + (i - lo) * 64, src.key(i), 64);
            if (sl) ws.put(src.sig(i), sl);
            if (ml) wm.put(src.msg(i), ml);
          }
        }
        ws.finish();
        wm.finish();
        StreamWriter::fence();  // the chunk's streamed bytes are globally visible
        if (done[c].fetch_add(1, std::memory_order_acq_rel) + 1 == T) {
          std::lock_guard<std::mutex> g(chunk_mu_);
          chunk_cv_.notify_all();
        }
      }
      if (dedup) zero_holes(out, blk);
    });
    // the calling thread SLEEPS until each chunk is complete: a spinning
    // caller on top of the workers overran the 16-CPU cgroup quota and the
    // CFS throttle stalled whole batches
    for (int c = 0; c < K; c++) {
      {
        std::unique_lock<std::mutex> g(chunk_mu_);
        chunk_cv_.wait(g, [&] { return done[c].load(std::memory_order_acquire) >= T; });
      }
      if (on_chunk) on_chunk(c);
    }
    pool_.wait();
    if (dedup && overflow_.load()) {  // the estimate was low: the keys once more, full size
      r->rebuilds++;
      size_table(true, 0);
      keys_only(src, out);
      if (overflow_.load()) {  // (cannot happen: cap >= 2 m) identity indices, never a wrong key
        r->dedup_dropped = true;
        pool_.run([&](int t) {
          const size_t a = lo + (m * (size_t)t) / T, b = lo + (m * (size_t)(t + 1)) / T;
          for (size_t i = a; i < b; i++) {
            std::memcpy(out.keys + (i - lo) * 64, src.key(i), 64);
            out.key_idx[i - lo] = (uint32_t)(i - lo);
          }
        });
      }
    }
    r->nkeys = !dedup ? m : r->dedup_dropped ? m : std::min<size_t>(next_id_.load(), max_ids_);
    r->fill_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  }

 private:
  static constexpr int kGroup = 16;

  void brange(size_t blk, size_t* a, size_t* b) const {
    const size_t T = (size_t)T_, K = blk_k();
    const size_t c = blk / T, t = blk % T;
    const size_t ca = (m_ * c) / K, cb = (m_ * (c + 1)) / K;
    *a = lo_ + ca + ((cb - ca) * t) / T;
    *b = lo_ + ca + ((cb - ca) * (t + 1)) / T;
  }
  size_t blk_k() const { return (boff_s_.size() - 1) / (size_t)T_; }

  void size_table(bool full, double est) {
    full_table_ = full;
    const size_t m = m_;
    if (full) {
      cap_ = 1024;
      while (cap_ < 2 * (uint64_t)m) cap_ <<= 1;
    } else {
      const double want = std::max(4.0 * est, 4096.0);
      cap_ = 1024;
      while ((double)cap_ < want && cap_ < 2 * (uint64_t)m) cap_ <<= 1;
      while (cap_ < 2 * (uint64_t)std::min<size_t>(m, 512)) cap_ <<= 1;
    }
    max_ids_ = (uint32_t)std::min<uint64_t>(cap_ / 2, m);
    if (table_.size() < cap_) table_ = std::vector<std::atomic<uint64_t>>(cap_);
    if (kcache_.size() < (size_t)max_ids_ * 64) kcache_.resize((size_t)max_ids_ * 64);
    pool_.run([&](int t) {  // clear in parallel (the table can be 2 m words)
      const uint64_t a = cap_ * t / pool_.threads(), b = cap_ * (t + 1) / pool_.threads();
      for (uint64_t k = a; k < b; k++) table_[k].store(0, std::memory_order_relaxed);
    });
    next_id_.store(0);
    overflow_.store(false);
  }

  // the keys of records [g0, g0 + cnt): hashes and table slots first, then
  // the candidate keys, then the compares -- a group's random table and key
  // reads overlap instead of costing a miss each in turn
  template <class Src>
  void keys_group(const Src& src, const Out& out, size_t g0, int cnt, IdBlock* blk) {
    if (overflow_.load(std::memory_order_relaxed)) return;
    std::atomic<uint64_t>* tab = table_.data();
    uint8_t* kc = kcache_.data();
    const uint64_t mask = cap_ - 1;
    const uint8_t* kp[kGroup];
    uint64_t hh[kGroup];
    uint32_t cand[kGroup];
    for (int j = 0; j < cnt; j++) {
      kp[j] = src.key(g0 + j);
      hh[j] = key_hash(kp[j]);
      __builtin_prefetch(&tab[hh[j] & mask]);
    }
    for (int j = 0; j < cnt; j++) {
      const uint64_t v = tab[hh[j] & mask].load(std::memory_order_acquire);
      const uint32_t id = (uint32_t)v;
      cand[j] = kBusy;
      if ((v >> 32) == ((hh[j] >> 32) | 1u) && id < max_ids_) {
        cand[j] = id;
        __builtin_prefetch(kc + (size_t)id * 64);
      }
    }
    for (int j = 0; j < cnt; j++) {
      uint32_t id = cand[j];
      if (id == kBusy || std::memcmp(kc + (size_t)id * 64, kp[j], 64) != 0)
        id = insert_key(tab, cap_, &next_id_, max_ids_, kc, out.keys, kp[j], hh[j], blk);
      if (id == kBusy) {
        overflow_.store(true, std::memory_order_relaxed);
        return;
      }
      out.key_idx[g0 + j - lo_] = id;
    }
  }

  void zero_holes(const Out& out, const IdBlock& blk) {
    for (uint32_t id = blk.next; id < blk.end && id < max_ids_; id++)
      std::memset(out.keys + (size_t)id * 64, 0, 64);
  }

  // the dedup alone over every record (after a table overflow)
  template <class Src>
  void keys_only(const Src& src, const Out& out) {
    const int T = pool_.threads();
    pool_.run([&](int t) {
      IdBlock blk;
      blk.size = 1;
      const size_t a = lo_ + (m_ * (size_t)t) / T, b = lo_ + (m_ * (size_t)(t + 1)) / T;
      for (size_t g0 = a; g0 < b && !overflow_.load(std::memory_order_relaxed); g0 += kGroup)
        keys_group(src, out, g0, (int)std::min<size_t>(kGroup, b - g0), &blk);
    });
  }

  Pool pool_;
  std::mutex chunk_mu_;
  std::condition_variable chunk_cv_;
  int T_ = 1;
  size_t lo_ = 0, m_ = 0;
  std::vector<uint32_t> len_min_, len_max_;
  std::vector<uint64_t> boff_s_, boff_m_;
  std::vector<std::atomic<uint64_t>> table_;
  std::vector<uint8_t> kcache_;  // the dedup's key copies (cached memory)
  uint64_t cap_ = 0;
  uint32_t max_ids_ = 0;
  bool full_table_ = false;
  std::atomic<uint32_t> next_id_{0};
  std::atomic<bool> overflow_{false};
};

// Worker threads: BH_PACK_THREADS, else the CPUs this process may run on
// (affinity, and the cgroup v2 quota when there is one) less one for the
// calling thread (it streams the chunks' copies meanwhile), at most 15.
inline int default_threads() {
  if (const char* e = getenv("BH_PACK_THREADS")) return std::max(1, std::min(64, atoi(e)));
  long n = (long)std::thread::hardware_concurrency();
#ifdef __linux__
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
#endif
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const long quota = std::atol(q) / period;
      if (quota > 0) n = std::min(n, quota);
    }
    std::fclose(f);
  }
  return (int)std::max(1L, std::min(15L, n - 1));
}

}  // namespace pack
}  // namespace bh
