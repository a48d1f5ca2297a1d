// HIP kernels for gfx950 (MI355X): batched ECDSA verification.
//
// Launch structure per batch (one stream; see seq() below and bdls_hip.cpp):
//   k_prep        1 lane/record   parse / checks / SHA-256 / Montgomery inputs
//   k_inv         1 lane/chunk    batched s^-1 mod n, u1, u2
//   k_key_insert / k_key_count / k_key_plan / k_split
//                 1 lane/record   dedup public keys, pick keys used >= kMinUses
//                                 times, route records to the two paths
//   k_ktab_build  1 lane/key      per-key fixed-base table (65 x 8 points)
//   k_keycomb     1 lane/record   u2 Q by table additions (no doublings) + u1 G
//   k_ladder      1 lane/record   u2 Q by Booth-5 ladder + u1 G (unique keys)
//   k_bitmap      1 lane/record   validity bitmap from the reason bytes
// plus k_gtab_build once per device at bh_init (fixed-base comb table for G).
#include "verify.h"

using namespace bh;

namespace {

template <class P, class N, class C, class IN>
__global__ __launch_bounds__(256) void k_prep(IN in, Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  stage_prep<P, N, C>(in, w, i);
}

template <class N>
__global__ __launch_bounds__(256) void k_inv(Work w, uint32_t n, uint32_t chunk) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = (uint64_t)c * chunk;
  if (lo >= n) return;
  const uint64_t hi = lo + chunk < n ? lo + chunk : n;
  stage_inv<N>(w, (uint32_t)lo, (uint32_t)hi);
}

// ---- key dedup / plan ------------------------------------------------------
__global__ __launch_bounds__(256) void k_key_insert(Work w, Plan pl, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if ((w.st[i] & 0x7fu) != R_OK) {
    pl.rec_slot[i] = kNone;
    return;
  }
  const uint64_t h = key_hash(w, i);
  const uint32_t mask = pl.hc - 1;
  uint32_t p = (uint32_t)h & mask;
  for (uint32_t probe = 0; probe < pl.hc; probe++) {
    const unsigned long long cur =
        atomicCAS((unsigned long long*)&pl.slot_hash[p], 0ull, (unsigned long long)h);
    if (cur == 0ull || cur == h) {
      atomicMin(&pl.slot_rep[p], i);
      pl.rec_slot[i] = p;
      return;
    }
    p = (p + 1) & mask;
  }
  pl.rec_slot[i] = kNone;  // table full (cannot happen: hc >= 2 n)
}

// Full-key check against the slot's representative (fingerprint collisions
// fall back to the ladder), then count.
__global__ __launch_bounds__(256) void k_key_count(Work w, Plan pl, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pl.rec_slot[i];
  if (p == kNone) return;
  const uint32_t rep = pl.slot_rep[p];
  if (rep == i || same_key(w, i, rep)) {
    atomicAdd(&pl.slot_cnt[p], 1u);
  } else {
    pl.rec_slot[i] = kNone;
  }
}

__global__ __launch_bounds__(256) void k_key_plan(Plan pl, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || n < kKeyTableMinBatch) return;
  const uint32_t p = pl.rec_slot[i];
  if (p == kNone || pl.slot_rep[p] != i || pl.slot_cnt[p] < kMinUses) return;
  const uint32_t t = atomicAdd(&pl.counters[2], 1u);
  if (t < pl.max_tables) {
    pl.slot_tab[p] = t;
    pl.tab_rec[t] = i;
  }
}

// Route every record: failed prep -> reason now; key table -> comb list;
// otherwise -> ladder list.
__global__ __launch_bounds__(256) void k_split(Work w, Plan pl, uint32_t n,
                                               uint8_t* __restrict__ reason) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t st = w.st[i] & 0x7fu;
  if (st != R_OK) {
    reason[i] = st;
    return;
  }
  const uint32_t p = pl.rec_slot[i];
  const uint32_t t = (p == kNone) ? kNone : pl.slot_tab[p];
  if (t != kNone) pl.comb_list[atomicAdd(&pl.counters[0], 1u)] = i;
  else pl.ladder_list[atomicAdd(&pl.counters[1], 1u)] = i;
}

template <class P>
__global__ __launch_bounds__(64) void k_ktab_build(Work w, Plan pl) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nt = min(pl.counters[2], pl.max_tables);
  if (t >= nt) return;
  ktab_build<P>(pl.tables + (size_t)t * kKTabWords, w, pl.tab_rec[t]);
}

template <class P>
__global__ __launch_bounds__(256) void k_keycomb(Work w, Plan pl, const uint32_t* __restrict__ gtab,
                                                 uint8_t* __restrict__ reason) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cnt = pl.counters[0];
  if (j >= cnt) return;
  const uint32_t i = pl.comb_list[j];
  const uint32_t t = pl.slot_tab[pl.rec_slot[i]];
  const bool ok = stage_keycomb<P>(w, gtab, i, pl.tables + (size_t)t * kKTabWords);
  reason[i] = ok ? R_OK : R_MATH;
}

// Variable-base path over the ladder list; the Q-table scratch slot is the
// list position, so whole waves past the list length exit.
template <class P>
__global__ __launch_bounds__(256) void k_ladder(Work w, Plan pl, const uint32_t* __restrict__ gtab,
                                                uint8_t* __restrict__ reason) {
  const uint32_t j0 = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cnt = pl.counters[1];
  if ((j0 & ~63u) >= cnt) return;
  const bool active = j0 < cnt;
  const uint32_t j = active ? j0 : cnt - 1;
  const uint32_t i = pl.ladder_list[j];
  const bool ok = stage_ladder<P>(w, gtab, i, j0 >> 6, threadIdx.x & 63u);
  if (active) reason[i] = ok ? R_OK : R_MATH;
}

__global__ __launch_bounds__(256) void k_bitmap(const uint8_t* __restrict__ reason, uint32_t n,
                                                uint64_t* __restrict__ bitmap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((i & ~63u) >= n) return;
  const bool ok = i < n && reason[i] == R_OK;
  const uint64_t m = __ballot(ok);
  if ((threadIdx.x & 63u) == 0) bitmap[i >> 6] = m;
}

// G comb table (see verify.h gtab_entry): one lane per entry.
template <class P>
__global__ __launch_bounds__(64) void k_gtab_build(uint32_t* gtab) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (uint32_t)(kCombWindows * kCombEntries)) return;
  gtab_entry<P>(t, gtab + (size_t)t * kGEntry);
}

}  // namespace

// ---------------------------------------------------------------------------
// Launchers (C++ linkage, used by bdls_hip.cpp)
namespace bh {

hipError_t launch_gtab_build(int curve, uint32_t* gtab, hipStream_t s) {
  const int nt = kCombWindows * kCombEntries;
  if (curve == 0)
    hipLaunchKernelGGL((k_gtab_build<F30_p256>), dim3((nt + 63) / 64), dim3(64), 0, s,
                       gtab);
  else
    hipLaunchKernelGGL((k_gtab_build<F30_k1>), dim3((nt + 63) / 64), dim3(64), 0, s, gtab);
  return hipGetLastError();
}

// Full launch sequence. ev (optional, 6 events) brackets: prep | inv | plan
// (dedup + split) | key tables | key comb | ladder+bitmap.
template <class P, class N, class C, class IN>
static hipError_t seq(const IN& in, const Work& w, const Plan& pl, const uint32_t* gtab,
                      uint32_t n, uint32_t chunk, uint64_t* bitmap, uint8_t* reason, hipStream_t s,
                      hipEvent_t* ev) {
  const dim3 blk(256);
  const dim3 grd((n + 255) / 256);
  const uint32_t nchunks = (n + chunk - 1) / chunk;
  const dim3 grc((nchunks + 255) / 256);
  hipError_t e;
#define REC(k)                                                 \
  if (ev) {                                                    \
    if ((e = hipEventRecord(ev[k], s)) != hipSuccess) return e; \
  }
  if ((e = hipMemsetAsync(pl.slot_hash, 0, (size_t)pl.hc * 8, s))) return e;
  if ((e = hipMemsetAsync(pl.slot_rep, 0xff, (size_t)pl.hc * 4, s))) return e;
  if ((e = hipMemsetAsync(pl.slot_cnt, 0, (size_t)pl.hc * 4, s))) return e;
  if ((e = hipMemsetAsync(pl.slot_tab, 0xff, (size_t)pl.hc * 4, s))) return e;
  if ((e = hipMemsetAsync(pl.counters, 0, 16, s))) return e;
  REC(0);
  hipLaunchKernelGGL((k_prep<P, N, C, IN>), grd, blk, 0, s, in, w, n);
  REC(1);
  hipLaunchKernelGGL((k_inv<N>), grc, blk, 0, s, w, n, chunk);
  REC(2);
  hipLaunchKernelGGL(k_key_insert, grd, blk, 0, s, w, pl, n);
  hipLaunchKernelGGL(k_key_count, grd, blk, 0, s, w, pl, n);
  hipLaunchKernelGGL(k_key_plan, grd, blk, 0, s, pl, n);
  hipLaunchKernelGGL(k_split, grd, blk, 0, s, w, pl, n, reason);
  REC(3);
  const uint32_t mt = pl.max_tables ? pl.max_tables : 1;
  hipLaunchKernelGGL((k_ktab_build<P>), dim3((mt + 63) / 64), dim3(64), 0, s, w, pl);
  REC(4);
  hipLaunchKernelGGL((k_keycomb<P>), grd, blk, 0, s, w, pl, gtab, reason);
  REC(5);
  hipLaunchKernelGGL((k_ladder<P>), grd, blk, 0, s, w, pl, gtab, reason);
  hipLaunchKernelGGL(k_bitmap, grd, blk, 0, s, reason, n, bitmap);
  REC(6);
#undef REC
  return hipGetLastError();
}

hipError_t launch_verify(int curve, const BatchIn& in, const Work& w, const Plan& pl,
                         const uint32_t* gtab, uint32_t n, uint32_t chunk, uint64_t* bitmap,
                         uint8_t* reason, hipStream_t s, hipEvent_t* ev) {
  // Fabric / BCCSP records: P-256 only (the low-S table of bccsp/utils covers
  // the NIST curves; secp256k1 never reaches bccsp/sw).
  if (curve != 0) return hipErrorInvalidValue;
  return seq<F30_p256, Fn_p256, Cv_p256>(in, w, pl, gtab, n, chunk, bitmap, reason, s, ev);
}

hipError_t launch_verify_bdls(int curve, const BdlsIn& in, const Work& w, const Plan& pl,
                              const uint32_t* gtab, uint32_t n, uint32_t chunk, uint64_t* bitmap,
                              uint8_t* reason, hipStream_t s, hipEvent_t* ev) {
  if (curve == 0)
    return seq<F30_p256, Fn_p256, Cv_p256>(in, w, pl, gtab, n, chunk, bitmap, reason, s, ev);
  return seq<F30_k1, Fn_k1, Cv_k1>(in, w, pl, gtab, n, chunk, bitmap, reason, s, ev);
}

}  // namespace bh
