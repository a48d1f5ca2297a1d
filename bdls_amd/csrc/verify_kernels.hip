// HIP kernels for gfx950 (MI355X): batched ECDSA verification.
//
// Launch structure per batch (one stream; see seq() below and bdls_hip.cpp):
//   k_prep        1 lane/record   parse / checks / SHA-256 / Montgomery inputs
//   k_inv         1 lane/chunk    batched s^-1 mod n (safegcd), u1, u2
//   k_key_insert / k_key_count / k_key_plan / k_split
//                 1 lane/record   registry lookup, dedup of the other keys,
//                                 per-batch tables for keys used >= min_uses
//                                 times, route records to the two paths
//   k_ktab_ladder 1-2 lanes/key + 1 lane/record
//                                 key-table builds and, in the same grid, the
//                                 variable-base ladder for records without a
//                                 table (independent work: the ladder fills
//                                 the issue slots the latency-bound builds
//                                 leave idle)
//   k_reg_publish 1 lane/build    make new registry tables visible
//   k_keycomb     1 lane/record   u2 Q by table additions (no doublings) + u1 G
//   k_keycomb_wide<L>  L lanes/record, for batches far below chip size
//   k_bitmap      1 lane/record   validity bitmap from the reason bytes
// Small batches whose digests the device computes (BDLS BLAKE2b, fused
// SHA-256 / SHA3) hash on a second stream (k_bdls_hash / k_digest) and split
// the record work around the join: k_ladder2_q / k_ladder1_q and
// k_keycomb_wide_q (u2 Q) before it, k_ladder2_g and k_keycomb_wide_g (u1 G,
// butterfly, x check) after it.
// plus k_gtab_build once per device at bh_init (fixed-base comb table for G)
// and k_reg_prep / k_reg_status for bh_keys_register.
#include <algorithm>
#include <type_traits>

#include <hipcub/hipcub.hpp>

#include "verify.h"

using namespace bh;

namespace {

template <class P, class N, class C, class IN, int HK, bool DEFER = false>
__global__ __launch_bounds__(256) void k_prep(IN in, Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if constexpr (std::is_same_v<IN, BatchIn>) stage_prep<P, N, C, HK, DEFER>(in, w, i);
  else stage_prep<P, N, C>(in, w, i);
}

// The key half of prep (LaunchOpts::records_ready passes).
template <class P, class C>
__global__ __launch_bounds__(256) void k_prep_keys(BatchIn in, Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  stage_prep_key<P, C>(in, w, i);
}

// e of every record (k_prep<..., DEFER>): the fused digests of a small batch
// on the second stream, beside prep / inverse / plan / the u2 Q work.
template <class C, int HK>
__global__ __launch_bounds__(256) void k_digest(BatchIn in, Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t e[8];
  digest_e<C, HK>(in, i, e);
  st8(w.e, i, w.ns, e);
}

// Fused SHA-256 digests of a small batch, kDigG lanes per record (round 5).
// A small batch's digest kernel is a few dozen waves, one per SIMD, each
// issue-bound on the longest message of its 64 records (a config-3 creator
// message is 65 blocks) -- on the latency path's critical path. The rounds are
// a serial chain, but the message schedule of block j depends on block j
// only: lane l of a record's group expands block base + l (W + K, 64 words)
// into its LDS slot, then the whole group runs the rounds of blocks base ..
// base + kDigG - 1 from the slots (every lane the same chain; lane 0 stores
// e). Per kDigG blocks a wave issues one schedule and kDigG round chains
// instead of kDigG of each: ~1.7x fewer instructions at 16 lanes.
constexpr uint32_t kDigG = 16, kDigBlock = 128, kDigSlot = 68;  // slot: 64 words + pad (b128)
template <class C>
__global__ __launch_bounds__(kDigBlock) void k_digest_grp(BatchIn in, Work w, uint32_t n) {
  __shared__ uint4 s_wk[kDigBlock * kDigSlot / 4];
  const uint32_t gid = blockIdx.x * kDigBlock + threadIdx.x;
  const uint32_t i = gid / kDigG, l = gid % kDigG;
  if (i >= n) return;  // whole groups (kDigG divides the wave)
  const uint32_t mlen = in.msg_len[i];
  const uint32_t mlen2 = in.msg2_len ? in.msg2_len[i] : 0u;
  const uint8_t* m1 = in.msg + in.msg_off[i];
  const uint8_t* m2 = mlen2 ? in.msg + in.msg2_off[i] : m1;
  const uint64_t len = (uint64_t)mlen + mlen2;
  const uint64_t total = ((len + 9 + 63) / 64) * 64;
  const uint32_t nblk = (uint32_t)(total / 64);
  uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
  uint4* mine = s_wk + threadIdx.x * (kDigSlot / 4);
  const uint4* grp = s_wk + (threadIdx.x - l) * (kDigSlot / 4);
  for (uint32_t base = 0; base < nblk; base += kDigG) {
    if (base + l < nblk) {
      uint32_t wv[16], wk[64];
      sha256_load_block(wv, m1, mlen2 ? mlen : len, m2, len, total, (uint64_t)(base + l) * 64u);
      sha256_sched_wk(wk, wv);
#pragma unroll
      for (int q = 0; q < 16; q++) mine[q] = uint4{wk[4 * q], wk[4 * q + 1], wk[4 * q + 2], wk[4 * q + 3]};
    }
    // the group's slots, written by its other lanes of this wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t cnt = nblk - base < kDigG ? nblk - base : kDigG;
    for (uint32_t q = 0; q < cnt; q++) {
      uint32_t wk[64];
      const uint4* s = grp + q * (kDigSlot / 4);
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint4 v = s[k];
        wk[4 * k] = v.x; wk[4 * k + 1] = v.y; wk[4 * k + 2] = v.z; wk[4 * k + 3] = v.w;
      }
      sha256_rounds_wk(h, wk);
    }
    // every lane's reads of this round of slots precede the next writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (l != 0) return;
  uint32_t e[8], nn[8], t[8];
#pragma unroll
  for (int k = 0; k < 8; k++) e[k] = h[7 - k];
  load_const8(nn, C::n);
  if (!sub8(t, e, nn)) copy8(e, t);  // as digest_e: e < 2^256 < 2n
  st8(w.e, i, w.ns, e);
}

// Fabric records pick the digest source per batch (SHA3 family or not); BDLS
// records always hash with BLAKE2b.
template <class P, class N, class C>
void launch_prep(const BatchIn& in, const Work& w, uint32_t n, dim3 grd, dim3 blk,
                 hipStream_t s) {
  if (in.flags & BHF_HASH_SHA3_256)
    hipLaunchKernelGGL((k_prep<P, N, C, BatchIn, HK_SHA3_256>), grd, blk, 0, s, in, w, n);
  else
    hipLaunchKernelGGL((k_prep<P, N, C, BatchIn, HK_GIVEN_OR_SHA256>), grd, blk, 0, s, in, w, n);
}
// ---- BDLS SignedProto.Hash, 4 lanes per record -----------------------------
// A BLAKE2b round is 4 independent column G's, then 4 independent diagonal
// G's. Lane c of a quad runs column c and diagonal c, holding v[c], v[4+c],
// v[8+c], v[12+c]; between the halves rows 1..3 rotate across the quad by DPP
// quad_perm (full-rate VALU moves, no LDS traffic). The 128-byte block is
// staged in LDS (lane c writes words 8c..8c+7) and each lane reads the four
// message words its G's take per round. Same digest as bdls_signed_proto_hash
// (blake2b.h), ~3x shorter per-record critical path: the serial chain of a
// lock/decide message (67 embedded proofs, ~100 blocks) dominated a round.
struct B2Quad {
  uint32_t k[4][12];  // lane c, round r: sigma[r][2c], [2c+1], [8+2c], [9+2c]
};
constexpr B2Quad make_b2quad() {
  B2Quad q{};
  for (int c = 0; c < 4; c++)
    for (int r = 0; r < 12; r++)
      q.k[c][r] = (uint32_t)B2Sigma::s[r][2 * c] | ((uint32_t)B2Sigma::s[r][2 * c + 1] << 8) |
                  ((uint32_t)B2Sigma::s[r][8 + 2 * c] << 16) |
                  ((uint32_t)B2Sigma::s[r][9 + 2 * c] << 24);
  return q;
}
constexpr B2Quad kB2Quad = make_b2quad();
constexpr int kQRot1 = 0x39;  // quad_perm [1,2,3,0]: lane c reads lane c+1
constexpr int kQRot2 = 0x4E;  // [2,3,0,1]
constexpr int kQRot3 = 0x93;  // [3,0,1,2]

// (mov_dpp: no `old` operand -- a quad permutation reads a valid lane for
// every lane, and update_dpp's old = 0 cost a v_mov of 0 into every DPP
// destination first, 12 per round; round 6, hipcc -S of k_bdls_hash)
template <int CTRL>
__device__ __forceinline__ uint64_t qperm(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xf, 0xf, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xf, 0xf,
                                                         true);
  return ((uint64_t)hi << 32) | lo;
}

// 64-bit rotation right by N as two v_alignbit_b32 (the shift / or form the
// compiler picks for 24 and 63 costs ~4 more instructions per G)
template <int N>
__device__ __forceinline__ uint64_t b2_rotr(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rl, rh;
  if constexpr (N == 32) {
    rl = hi;
    rh = lo;
  } else if constexpr (N < 32) {
    rl = __builtin_amdgcn_alignbit(hi, lo, N);
    rh = __builtin_amdgcn_alignbit(lo, hi, N);
  } else {
    rl = __builtin_amdgcn_alignbit(lo, hi, N - 32);
    rh = __builtin_amdgcn_alignbit(hi, lo, N - 32);
  }
  return ((uint64_t)rh << 32) | rl;
}

__device__ __forceinline__ void b2_gq(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d,
                                      uint64_t x, uint64_t y) {
  a = a + b + x;
  d = b2_rotr<32>(d ^ a);
  c = c + d;
  b = b2_rotr<24>(b ^ c);
  a = a + b + y;
  d = b2_rotr<16>(d ^ a);
  c = c + d;
  b = b2_rotr<63>(b ^ c);
}

template <class C>
__global__ __launch_bounds__(256) void k_bdls_hash(BdlsIn in, Work w, uint32_t n) {
  __shared__ uint64_t lds_blk[64][16];  // one 128-byte block per quad
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = gid >> 2, c = gid & 3u;
  if (i >= n) return;  // whole quads exit together
  uint64_t* B = lds_blk[threadIdx.x >> 2];
  const uint8_t* xy = in.xy + (size_t)i * 64;
  const uint8_t* msg = in.msg + in.msg_off[i];
  const uint32_t mlen = in.msg_len[i];
  uint32_t sidx[12];
#pragma unroll
  for (int r = 0; r < 12; r++)
    sidx[r] = c == 0 ? kB2Quad.k[0][r]
              : c == 1 ? kB2Quad.k[1][r]
              : c == 2 ? kB2Quad.k[2][r]
                       : kB2Quad.k[3][r];
  const uint64_t iv_a = kB2IV[c], iv_b = kB2IV[4 + c];
  uint64_t h_a = iv_a ^ (c == 0 ? 0x01010000ull ^ 32ull : 0ull), h_b = iv_b;  // h[c], h[4+c]
  const uint64_t total = kBdlsHeader + (uint64_t)mlen;
  for (uint64_t pos = 0;; pos += 128) {
    const bool last = total - pos <= 128;
    uint32_t wv[8];  // stream words pos/4 + 8c .. + 7
    if (pos == 0 && c < 3) {
      uint32_t hx[8], hy[8];
      load_le_words<8>(hx, xy);
      load_le_words<8>(hy, xy + 32);
      if (c == 0) {
        wv[0] = 0x534c4442u;  // "BDLS_CONSENSUS_SIGNATURE", little-endian words
        wv[1] = 0x4e4f435fu;
        wv[2] = 0x534e4553u;
        wv[3] = 0x535f5355u;
        wv[4] = 0x414e4749u;
        wv[5] = 0x45525554u;
        wv[6] = in.version[i];
        wv[7] = hx[0];
      } else if (c == 1) {
#pragma unroll
        for (int k = 0; k < 7; k++) wv[k] = hx[k + 1];
        wv[7] = hy[0];
      } else {
#pragma unroll
        for (int k = 0; k < 7; k++) wv[k] = hy[k + 1];
        wv[7] = mlen;
      }
    } else {
      const uint32_t q = (uint32_t)(pos + 32u * c - kBdlsHeader);  // message byte offset
      if (!last) {
        load_le_words<8>(wv, msg + q);
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) wv[k] = b2_tail_word(msg, mlen, q + 4u * k);
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; k++) B[4 * c + k] = (uint64_t)wv[2 * k] | ((uint64_t)wv[2 * k + 1] << 32);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // all 48 message words this lane's G's take, issued back to back (one LDS
    // latency per block instead of one per half-round)
    uint64_t mx[12][4];
#pragma unroll
    for (int r = 0; r < 12; r++) {
      const uint32_t sx = sidx[r];
      mx[r][0] = B[sx & 0xffu];
      mx[r][1] = B[(sx >> 8) & 0xffu];
      mx[r][2] = B[(sx >> 16) & 0xffu];
      mx[r][3] = B[sx >> 24];
    }
    uint64_t a = h_a, b = h_b, cc = iv_a, d = iv_b;
    if (c == 0) d ^= last ? total : pos + 128;  // v[12] ^= t
    if (c == 2 && last) d = ~d;                  // v[14] = ~v[14]
#pragma unroll
    for (int r = 0; r < 12; r++) {
      b2_gq(a, b, cc, d, mx[r][0], mx[r][1]);
      b = qperm<kQRot1>(b);
      cc = qperm<kQRot2>(cc);
      d = qperm<kQRot3>(d);
      b2_gq(a, b, cc, d, mx[r][2], mx[r][3]);
      b = qperm<kQRot3>(b);
      cc = qperm<kQRot2>(cc);
      d = qperm<kQRot1>(d);
    }
    h_a ^= a ^ cc;
    h_b ^= b ^ d;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (last) break;
  }
  // digest = h[0..3] little-endian; e = big-endian integer (limb 7 = bytes 0..3)
  const uint64_t h1 = qperm<kQRot1>(h_a), h2 = qperm<kQRot2>(h_a), h3 = qperm<kQRot3>(h_a);
  if (c != 0) return;
  const uint64_t hh[4] = {h_a, h1, h2, h3};
  uint32_t e[8], nn[8], t[8];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    e[7 - 2 * k] = bswap32((uint32_t)hh[k]);
    e[6 - 2 * k] = bswap32((uint32_t)(hh[k] >> 32));
  }
  load_const8(nn, C::n);
  if (!sub8(t, e, nn)) copy8(e, t);
  st8(w.e, i, w.ns, e);
}


template <class N, bool U1>
__global__ __launch_bounds__(256) void k_inv(Work w, uint32_t n, uint32_t lanes) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= lanes) return;
  stage_inv<N, U1>(w, c, lanes, n);
}

// ---- key lookup / dedup / plan ----------------------------------------------
// Registry hit -> rec_tab; otherwise insert the fingerprint into the batch's
// dedup table (smallest record index becomes the slot's representative).
__global__ __launch_bounds__(256) void k_key_insert(Work w, Plan pl, KeyReg g, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pl.rec_tab[i] = kNone;
  if ((w.st[i] & 0x7fu) != R_OK) {
    pl.rec_slot[i] = kNone;
    return;
  }
  const uint64_t h = key_hash(w, i);
  const uint32_t t = reg_lookup(g, w, i, h);
  if (t != kNone) {
    pl.rec_tab[i] = t;
    pl.rec_slot[i] = kNone;
    return;
  }
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
// fall back to the ladder), then count. Keys compare as their 64 input bytes
// X || Y: prep admitted only coordinates < p, so equal bytes <=> equal point,
// and the representative's key is one contiguous 64-byte read instead of 18
// scattered limb-major words. A16: the key array is 16-byte aligned.
template <bool A16>
__global__ __launch_bounds__(256) void k_key_count(Work w, Plan pl, const uint8_t* __restrict__ pub,
                                                   uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = pl.rec_slot[i];
  if (p == kNone) return;
  const uint32_t rep = pl.slot_rep[p];
  bool same = rep == i;
  if (!same) {
    uint32_t d = 0;
    if constexpr (A16) {
      const uint4* a = reinterpret_cast<const uint4*>(pub + (size_t)i * 64);
      const uint4* b = reinterpret_cast<const uint4*>(pub + (size_t)rep * 64);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint4 x = a[k], y = b[k];
        d |= (x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w);
      }
    } else {
      for (int k = 0; k < 64; k++) d |= pub[(size_t)i * 64 + k] ^ pub[(size_t)rep * 64 + k];
    }
    same = d == 0;
  }
  if (same) {
    atomicAdd(&pl.slot_cnt[p], 1u);
  } else {
    pl.rec_slot[i] = kNone;
  }
}

// One table build per representative whose key is used >= min_uses times (in
// batches of >= min_batch records). keep: the table goes to the registry
// while it has room, else to the batch. reg_only: registry or nothing
// (bh_keys_register).
__global__ __launch_bounds__(256) void k_key_plan(Work w, Plan pl, KeyReg g, uint32_t n,
                                                  uint32_t min_uses, uint32_t min_batch,
                                                  uint32_t keep, uint32_t reg_only) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || n < min_batch) return;
  const uint32_t p = pl.rec_slot[i];
  if (p == kNone || pl.slot_rep[p] != i || pl.slot_cnt[p] < min_uses) return;
  uint32_t id = kNone;
  if (keep && g.cap) {
    const uint32_t r = atomicAdd(g.count, 1u);
    if (r < g.cap) {
      id = r;
      reg_key_store(g, r, w, i);
    }
  }
  if (id == kNone && reg_only) return;
  const uint32_t job = atomicAdd(&pl.counters[2], 1u);
  if (job >= pl.max_tables) return;  // registry slot (if any) stays unpublished
  if (id == kNone) id = kLocal | job;
  pl.slot_tab[p] = id;
  pl.tab_rec[job] = i;
  pl.tab_dst[job] = id;
}

// Route every record: failed prep -> reason now; key table -> comb list;
// otherwise -> ladder list. List slots come from one atomic per 1024-thread
// block and list: same-address atomics serialise in L2, so a per-wave (let
// alone per-record) atomic costs more than the rest of the routing.
constexpr uint32_t kSplitBlock = 1024;
__global__ __launch_bounds__(kSplitBlock) void k_split(Work w, Plan pl, uint32_t n,
                                                       uint8_t* __restrict__ reason) {
  __shared__ uint32_t wave_cnt[2][kSplitBlock / 64];
  __shared__ uint32_t block_base[2];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  int list = -1;  // 0 comb, 1 ladder, -1 none
  if (i < n) {
    const uint8_t st = w.st[i] & 0x7fu;
    if (st != R_OK) {
      reason[i] = st;
    } else {
      uint32_t t = pl.rec_tab[i];
      if (t == kNone) {
        const uint32_t p = pl.rec_slot[i];
        if (p != kNone) t = pl.slot_tab[p];
        pl.rec_tab[i] = t;
      }
      list = t != kNone ? 0 : 1;
    }
  }
  const uint64_t m0 = __ballot(list == 0), m1 = __ballot(list == 1);
  if (lane == 0) {
    wave_cnt[0][wv] = (uint32_t)__popcll(m0);
    wave_cnt[1][wv] = (uint32_t)__popcll(m1);
  }
  __syncthreads();
  if (threadIdx.x < 2) {  // exclusive prefix over the block's waves, one atomic per list
    uint32_t sum = 0;
    for (uint32_t k = 0; k < kSplitBlock / 64; k++) {
      const uint32_t c = wave_cnt[threadIdx.x][k];
      wave_cnt[threadIdx.x][k] = sum;
      sum += c;
    }
    block_base[threadIdx.x] = sum ? atomicAdd(&pl.counters[threadIdx.x], sum) : 0u;
  }
  __syncthreads();
  if (list < 0) return;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const uint64_t m = list == 0 ? m0 : m1;
  const uint32_t slot = block_base[list] + wave_cnt[list][wv] + (uint32_t)__popcll(m & below);
  if (list == 0) pl.comb_list[slot] = i;
  else pl.ladder_list[slot] = i;
}

// Blocks [0, tab_blocks) build key tables (one lane per table, verify.h
// ktab_build), the next lad_blocks run the ladder list (waves past the list
// length exit whole; the Q-table scratch slot is the list position), the last
// gp_blocks compute the u1 G half of the key-comb list (verify.h stage_gpart)
// while the builds run: one build wave per SIMD leaves issue slots free.
constexpr uint32_t kBuildPerBlock = 256;
template <class P>
__device__ __forceinline__ void ktab_ladder_body(const Work& w, const Plan& pl, const KeyReg& g,
                                                 const uint32_t* __restrict__ gtab,
                                                 uint8_t* __restrict__ reason, uint32_t tab_blocks,
                                                 uint32_t lad_blocks, uint32_t ll) {
  if (blockIdx.x >= tab_blocks + lad_blocks) {
    const uint32_t j = (blockIdx.x - tab_blocks - lad_blocks) * blockDim.x + threadIdx.x;
    if (j < pl.counters[0]) stage_gpart<P>(w, gtab, pl.comb_order[j], j);
    return;
  }
  if (blockIdx.x < tab_blocks) {
    const uint32_t nt = min(pl.counters[2], pl.max_tables);
    const uint32_t base = blockIdx.x * kBuildPerBlock;
    const uint32_t t = base + threadIdx.x;
    if (t < nt) {
      // per-batch tables of one-lane-per-record batches are Lim-Lee combs,
      // small batches' 4-bit windows; registry slots get both forms (verify.h
      // reg_build: the comb + affine windows)
      const uint32_t id = pl.tab_dst[t];
      uint32_t* tab = const_cast<uint32_t*>(tab_ptr(pl, g, id));
      if (!(id & kLocal)) return;  // a registry slot: k_reg_win builds all of it
      if (ll) lltab_build<P>(tab, w, pl.tab_rec[t]);
      else ktab_build<P>(tab, w, pl.tab_rec[t]);
    }
    return;
  }
  const uint32_t j0 = (blockIdx.x - tab_blocks) * blockDim.x + threadIdx.x;
  const uint32_t cnt = pl.counters[1];
  if ((j0 & ~63u) >= cnt) return;
  const bool active = j0 < cnt;
  const uint32_t j = active ? j0 : cnt - 1;
  const uint32_t i = pl.ladder_list[j];
  const bool ok = stage_ladder_fold<P>(w, gtab, i, j0 >> 6, threadIdx.x & 63u);
  if (active) reason[i] = ok ? R_OK : R_MATH;
}

// BH_WAVE_TIMES (experiment builds only, tools/build_exp.sh): every wave of
// k_ktab_ladder records its role (0 table build, 1 ladder, 2 u1 G), CU and
// start / end on the constant-rate wall clock, read back by bh_wave_times.
#ifdef BH_WAVE_TIMES
constexpr uint32_t kWaveTimes = 65536;
__device__ unsigned long long g_wave_t[kWaveTimes * 4];
#endif

// BH_KTAB_WAVES (default 0 = the compiler's choice): occupancy floor for
// k_ktab_ladder, waves per SIMD. Round 6 found the kernel at 132 VGPRs (3
// waves per SIMD; config 5's ladder -6 %) and the cause in BH_ZFILTER; with
// the filter off it is back at 116 (4 waves). A floor of 4 on the 132-VGPR
// code spilled 344 VGPRs to scratch, so it stays a switch, not a default.
#ifndef BH_KTAB_WAVES
#define BH_KTAB_WAVES 0
#endif
#if BH_KTAB_WAVES > 0
#define BH_KTAB_ATTR __attribute__((amdgpu_waves_per_eu(BH_KTAB_WAVES)))
#else
#define BH_KTAB_ATTR
#endif
template <class P>
__global__ __launch_bounds__(256) BH_KTAB_ATTR
void k_ktab_ladder(Work w, Plan pl, KeyReg g,
                                                     const uint32_t* __restrict__ gtab,
                                                     uint8_t* __restrict__ reason,
                                                     uint32_t tab_blocks,
                                                     uint32_t lad_blocks, uint32_t ll) {
#ifdef BH_WAVE_TIMES
  const unsigned long long t0 = wall_clock64();
#endif
  ktab_ladder_body<P>(w, pl, g, gtab, reason, tab_blocks, lad_blocks, ll);
#ifdef BH_WAVE_TIMES
  const unsigned long long t1 = wall_clock64();
  const uint32_t wid = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
  if ((threadIdx.x & 63u) == 0u && wid < kWaveTimes) {
    const uint32_t role = blockIdx.x < tab_blocks ? 0u : blockIdx.x < tab_blocks + lad_blocks ? 1u : 2u;
    g_wave_t[4 * wid] = t0;
    g_wave_t[4 * wid + 1] = t1;
    g_wave_t[4 * wid + 2] = role;
    g_wave_t[4 * wid + 3] = (unsigned long long)__smid();
  }
#endif
}

#ifdef BH_WAVE_TIMES
extern "C" int bh_wave_times(unsigned long long* out, int clear) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (clear) {
    static unsigned long long zero[kWaveTimes * 4];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wave_t), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), sizeof(g_wave_t)) == hipSuccess ? 0 : -1;
}
#endif

// Butterfly over groups of L adjacent lanes: every lane ends with the group's
// sum (L partial sums of one record).
template <class P, int L>
__device__ __forceinline__ void group_sum(J30& C, bool& c_inf) {
  for (int off = 1; off < L; off <<= 1) {
    J30 T;
#pragma unroll
    for (int q = 0; q < 9; q++) {
      T.X[q] = __shfl_xor(C.X[q], off, 64);
      T.Y[q] = __shfl_xor(C.Y[q], off, 64);
      T.Z[q] = __shfl_xor(C.Z[q], off, 64);
    }
    const bool t_inf = __shfl_xor((int)c_inf, off, 64) != 0;
    j_acc<P>(C, c_inf, T, t_inf);
  }
}

// secp256k1 ladder on 2 lanes per record (small, latency-bound batches), split
// around the digests: lane pair (2j, 2j+1) of k_ladder2_q runs the k1 Q / k2
// phi(Q) halves of the GLV split (no u1 needed) while the digests are hashed
// on the second stream; k_ladder2_g adds the G-comb windows of u1 = e w
// afterwards. Each lane owns a Q-table slot (2 per record for batches this
// small); partial sums live in the gpart scratch (slot gid, stride pstride).
template <class P>
__global__ __launch_bounds__(256) void k_ladder2_q(Work w, Plan pl, uint32_t pstride) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j0 = gid >> 1, part = gid & 1u;
  const uint32_t cnt = pl.counters[1];
  if ((j0 & ~31u) >= cnt) return;
  const uint32_t i = pl.ladder_list[j0 < cnt ? j0 : cnt - 1];
  J30 C;
  bool c_inf;
  q_ladder_glv<P>(C, c_inf, w, i, gid >> 6, threadIdx.x & 63u, 1u << part);
  part_store(w, gid, pstride, C, c_inf);
}

// P-256 (no endomorphism): the whole u2 Q Booth ladder on one lane per
// record, before the join; partial sum in slot 2 j (k_ladder2_g, PARTS = 1).
template <class P>
__global__ __launch_bounds__(256) void k_ladder1_q(Work w, Plan pl, uint32_t pstride) {
  const uint32_t j0 = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cnt = pl.counters[1];
  if ((j0 & ~63u) >= cnt) return;
  const uint32_t i = pl.ladder_list[j0 < cnt ? j0 : cnt - 1];
  J30 C;
  bool c_inf;
  q_ladder<P>(C, c_inf, w, i, j0 >> 6, threadIdx.x & 63u);
  part_store(w, 2 * j0, pstride, C, c_inf);
}

// 8 lanes per record: lanes l < PARTS start from the u2 Q partial sums (the
// two GLV halves, or P-256's single ladder), every lane adds the G-comb
// windows l, l + 8, ... of u1 = e w (computed per lane), then a 3-level
// butterfly; lane 0 checks. (One lane: 26 serial mixed additions.)
constexpr int kLadGLanes = 8;
template <class P, class N, int PARTS>
__global__ __launch_bounds__(256) void k_ladder2_g(Work w, Plan pl,
                                                   const uint32_t* __restrict__ gtab,
                                                   uint8_t* __restrict__ reason,
                                                   uint32_t pstride) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j0 = gid / kLadGLanes, l = gid % kLadGLanes;
  const uint32_t cnt = pl.counters[1];
  if (j0 >= cnt) return;  // whole groups exit together
  const uint32_t i = pl.ladder_list[j0];
  J30 C;
  bool c_inf = true;
  if (l < PARTS) {
    part_load(w, 2 * j0 + l, pstride, C, c_inf);
  } else {
    f_const(C.X, P::r1);
    f_const(C.Y, P::r1);
    f_const(C.Z, P::r1);
  }
  uint32_t u1[8];
  calc_u1<N>(u1, w, i);
  g_comb_part<P, kLadGLanes>(C, c_inf, gtab, u1, l);
  group_sum<P, kLadGLanes>(C, c_inf);
  if (l == 0) reason[i] = finish_check<P>(w, i, C, c_inf, C, true) ? R_OK : R_MATH;
}

// The registry slots of this pass (round 5), one workgroup per table: the
// first lane of the third wave builds the comb (verify.h lltab_build) while
// lane 0 walks the bases 16^win Q (four doublings each) into LDS; then lane
// win builds window win (verify.h reg_window) with its raw points and Z
// products in its own LDS column. A registration's critical path is the
// comb build plus one window, not the comb and 65 windows end to end
// (~16.8k F_p ops on one lane).
constexpr uint32_t kRegWinBlock = 192;  // lanes 0 .. kKWin - 1: windows; lane 128: the comb
static_assert(kKWin <= 128, "one lane per window, the comb in the third wave");
struct RegLdsRaw {
  uint32_t* pts;  // [point j][word k][lane]: 27 words per point
  uint32_t* zs;   // [j][k][lane]: 9 words per product
  uint32_t lane;
  __device__ void store(uint32_t j, const J30& P) {
#pragma unroll
    for (int k = 0; k < 9; k++) {
      pts[((j * 27u) + k) * kKWin + lane] = P.X[k];
      pts[((j * 27u) + 9u + k) * kKWin + lane] = P.Y[k];
      pts[((j * 27u) + 18u + k) * kKWin + lane] = P.Z[k];
    }
  }
  __device__ void load(J30& P, uint32_t j) const {
#pragma unroll
    for (int k = 0; k < 9; k++) {
      P.X[k] = pts[((j * 27u) + k) * kKWin + lane];
      P.Y[k] = pts[((j * 27u) + 9u + k) * kKWin + lane];
      P.Z[k] = pts[((j * 27u) + 18u + k) * kKWin + lane];
    }
  }
  __device__ void store_z(uint32_t j, const uint32_t z[9]) {
#pragma unroll
    for (int k = 0; k < 9; k++) zs[(j * 9u + k) * kKWin + lane] = z[k];
  }
  __device__ void load_z(uint32_t z[9], uint32_t j) const {
#pragma unroll
    for (int k = 0; k < 9; k++) z[k] = zs[(j * 9u + k) * kKWin + lane];
  }
};
template <class P>
__global__ __launch_bounds__(kRegWinBlock) void k_reg_win(Work w, Plan pl, KeyReg g) {
  __shared__ uint32_t s_base[kKWin * 27];
  __shared__ uint32_t s_pts[kKEnt * 27 * kKWin];
  __shared__ uint32_t s_zs[kKEnt * 9 * kKWin];
  // the comb build's scratch at the slot's offsets (the entries' words unused):
  // LDS instead of the slot's global scratch, whose round trips (~1 us each on a
  // lone wave) made the build ~2.5x slower than its arithmetic
  __shared__ __attribute__((aligned(16))) uint32_t s_comb[kLLPre + 12u * kLLEnt];
  const uint32_t t = blockIdx.x;
  const uint32_t nt = min(pl.counters[2], pl.max_tables);
  if (t >= nt) return;  // the whole workgroup
  const uint32_t id = pl.tab_dst[t];
  if (id & kLocal) return;  // a per-batch table: no windows
  uint32_t* tab = const_cast<uint32_t*>(tab_ptr(pl, g, id));
  const uint32_t lane = threadIdx.x;
  // The record index is workgroup-uniform, so the compiler would run a lone
  // lane's build on the SALU (scalar 32-bit multiplies: ~3x slower than the
  // VALU's v_mad_u64_u32, measured in tools/lat_chain.hip); an empty asm with
  // a VGPR operand makes it a per-lane value and keeps the work on the VALU.
  uint32_t rec = pl.tab_rec[t];
  asm volatile("" : "+v"(rec));
  if (lane == 128u) reg_build_comb<P>(tab, w, rec, s_comb);
  if (lane == 0) {
    J30 B;
    ld9(B.X, w.qx, rec, w.ns);
    ld9(B.Y, w.qy, rec, w.ns);
    f_const(B.Z, P::r1);
#pragma unroll
    for (int k = 0; k < 9; k++) asm volatile("" : "+v"(B.Z[k]));
#pragma unroll 1
    for (uint32_t win = 0; win < (uint32_t)kKWin; win++) {
#pragma unroll
      for (int k = 0; k < 9; k++) {
        s_base[win * 27u + k] = B.X[k];
        s_base[win * 27u + 9u + k] = B.Y[k];
        s_base[win * 27u + 18u + k] = B.Z[k];
      }
      if (win + 1u < (uint32_t)kKWin) {
#pragma unroll 1
        for (int d = 0; d < kKW; d++) j_dbl<P>(B, B);
      }
    }
  }
  __syncthreads();
  if (lane >= (uint32_t)kKWin) return;
  J30 B;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    B.X[k] = s_base[lane * 27u + k];
    B.Y[k] = s_base[lane * 27u + 9u + k];
    B.Z[k] = s_base[lane * 27u + 18u + k];
  }
  RegLdsRaw raw{s_pts, s_zs, lane};
  reg_window<P>(tab, lane, B, raw);
}

template <class P>
static void launch_reg_win(const Work& w, const Plan& pl, const KeyReg& g, hipStream_t s) {
  if (pl.max_tables)
    hipLaunchKernelGGL((k_reg_win<P>), dim3(pl.max_tables), dim3(kRegWinBlock), 0, s, w, pl, g);
}

// Publish registry tables built in this batch (after the builds completed).
__global__ __launch_bounds__(256) void k_reg_publish(Work w, Plan pl, KeyReg g) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nt = min(pl.counters[2], pl.max_tables);
  if (t >= nt) return;
  const uint32_t id = pl.tab_dst[t];
  if (id & kLocal) return;
  const uint64_t h = key_hash(w, pl.tab_rec[t]);
  const uint32_t mask = g.hc - 1;
  uint32_t p = (uint32_t)h & mask;
  for (uint32_t probe = 0; probe < g.hc; probe++) {
    if (atomicCAS((unsigned long long*)&g.slot_hash[p], 0ull, (unsigned long long)h) == 0ull) {
      g.slot_tab[p] = id;
      return;
    }
    p = (p + 1) & mask;
  }
}

// BH_KEYCOMB_WAVES: optional occupancy target for k_keycomb (waves per SIMD;
// the register budget follows from it). Unset = the compiler's choice.
#ifdef BH_KEYCOMB_WAVES
#define BH_KEYCOMB_ATTR __attribute__((amdgpu_waves_per_eu(BH_KEYCOMB_WAVES, BH_KEYCOMB_WAVES)))
#else
#define BH_KEYCOMB_ATTR
#endif
// BH_KEYCOMB_LDS (default 1): with comb tables, each 256-record workgroup
// first copies the tables its records use -- the list is grouped by table, so
// they are the runs of equal ids, ~17 at 16 records per key -- into LDS
// (kLdsTabs slots of 64 x 72 B = 78 KB: two workgroups per CU, the occupancy
// the registers allow anyway), then reads every Horner step's entry from
// there. Each table is then fetched from L2 / HBM once per workgroup instead
// of once per Horner step of every wave that uses it, whose working set
// (~5 MB per XCD) overflowed the 4 MB L2. Runs beyond the slots read their
// table in global memory.
#ifndef BH_KEYCOMB_LDS
#define BH_KEYCOMB_LDS 1
#endif
// BH_LDS_TABS: slots per workgroup (default 17 at 7 teeth: 78 KB, two
// workgroups per CU)
#ifndef BH_LDS_TABS
#define BH_LDS_TABS ((17u * 64u) / kLLEnt)
#endif
constexpr uint32_t kLdsTabs = BH_LDS_TABS;  // 78 KB of slots: 17 at 7 teeth, 8 at 8
constexpr uint32_t kLdsTabWords = kLLEnt * kLLLds;
template <class P>
__global__ __launch_bounds__(256) BH_KEYCOMB_ATTR void k_keycomb(Work w, Plan pl, KeyReg g,
                                                 const uint32_t* __restrict__ gtab,
                                                 uint8_t* __restrict__ reason, uint32_t ll) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t cnt = pl.counters[0];
  if (!BH_KEYCOMB_LDS || !ll) {  // uniform over the grid
    if (j >= cnt) return;
    const uint32_t i = pl.comb_order[j];
    const uint32_t id = pl.rec_tab[i];
    const bool ok = ll ? stage_keycomb_fold<P>(w, i, tab_ptr(pl, g, id), kLLAff, g2_of(gtab))
                       : stage_keycomb_q<P>(w, i, j, tab_ptr(pl, g, id), false, 0u,
                                            !(id & kLocal));  // registry: affine windows
    reason[i] = ok ? R_OK : R_MATH;
    return;
  }
  if (blockIdx.x * blockDim.x >= cnt) return;  // the whole workgroup: no barrier skipped
  __shared__ uint32_t s_tab[kLdsTabs * kLdsTabWords];
  __shared__ const uint32_t* s_src[kLdsTabs];
  __shared__ uint32_t s_id[256];
  __shared__ uint32_t s_wsum[4];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const bool have = j < cnt;
  uint32_t i = 0, id = kNone;
  if (have) {
    i = pl.comb_order[j];
    id = pl.rec_tab[i];
  }
  // every table of a one-lane comb batch has a comb (per-batch tables are
  // combs, registry slots carry one at offset 0): all are staged by runs
  const bool lcl = have && id != kNone;
  s_id[t] = lcl ? id : kNone;
  __syncthreads();
  // runs of equal ids -> slots: inclusive count of run starts up to this lane
  const bool start = lcl && (t == 0u || s_id[t - 1u] != id);
  const uint64_t m = __ballot(start);
  uint32_t slot = (uint32_t)__popcll(m & (lane == 63u ? ~0ull : ((2ull << lane) - 1ull)));
  if (lane == 0u) s_wsum[wv] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t runs = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4u; q++) {
    const uint32_t c = s_wsum[q];
    if (q < wv) slot += c;
    runs += c;
  }
  slot -= 1u;  // meaningful for lcl lanes (>= 1 start at or before them)
  if (start && slot < kLdsTabs) s_src[slot] = tab_ptr(pl, g, id);
  __syncthreads();
  const uint32_t nst = runs < kLdsTabs ? runs : kLdsTabs;
  for (uint32_t e = t; e < nst * kLLEnt; e += 256u) {  // one entry per lane: 5 x 16 B in, 9 x 8 B out
    const W4* s = reinterpret_cast<const W4*>(s_src[e / kLLEnt] + (e % kLLEnt) * kLLAff);
    const W4 a = s[0], b = s[1], c = s[2], d = s[3], f = s[4];
    W2* o = reinterpret_cast<W2*>(s_tab + e * kLLLds);
    o[0] = W2{a.x, a.y}; o[1] = W2{a.z, a.w}; o[2] = W2{b.x, b.y};
    o[3] = W2{b.z, b.w}; o[4] = W2{c.x, c.y}; o[5] = W2{c.z, c.w};
    o[6] = W2{d.x, d.y}; o[7] = W2{d.z, d.w}; o[8] = W2{f.x, f.y};
  }
  __syncthreads();
  if (!have) return;
  const bool in_lds = lcl && slot < kLdsTabs;
  const uint32_t* tab = in_lds ? s_tab + slot * kLdsTabWords : tab_ptr(pl, g, id);
  // the key's comb (per-batch or registry slot) with u1 G folded into the
  // Horner (round 5, verify.h q_llcomb_g)
  const bool ok = stage_keycomb_fold<P>(w, i, tab, in_lds ? kLLLds : kLLAff, g2_of(gtab));
  reason[i] = ok ? R_OK : R_MATH;
}

// L lanes per record (a group of L adjacent lanes of one wave): partial sums
// over interleaved windows, butterfly over the group, lane 0 checks.
template <class P, int L>
__global__ __launch_bounds__(256) void k_keycomb_wide(Work w, Plan pl, KeyReg g,
                                                      const uint32_t* __restrict__ gtab,
                                                      uint8_t* __restrict__ reason) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = gid / L, l = gid % L;
  const uint32_t cnt = pl.counters[0];
  if (j >= cnt) return;  // whole groups exit together
  const uint32_t i = pl.comb_order[j];
  const uint32_t id = pl.rec_tab[i];
  J30 C;
  bool c_inf;
  // registry slots: their affine windows (mixed additions)
  keycomb_part<P, L>(C, c_inf, w, gtab, i, tab_ptr(pl, g, id), l, !(id & kLocal));
  group_sum<P, L>(C, c_inf);
  if (l == 0) reason[i] = finish_check<P>(w, i, C, c_inf, C, true) ? R_OK : R_MATH;
}

// k_keycomb_wide split around the BDLS digests like k_ladder2_q / _g: the key
// table windows first, the u1 G windows once u1 = e w exists. Partial-sum slot
// pbase + gid.
template <class P, int L>
__global__ __launch_bounds__(256) void k_keycomb_wide_q(Work w, Plan pl, KeyReg g,
                                                        uint32_t pbase, uint32_t pstride) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = gid / L, l = gid % L;
  const uint32_t cnt = pl.counters[0];
  if (j >= cnt) return;
  const uint32_t i = pl.comb_order[j];
  const uint32_t id = pl.rec_tab[i];
  J30 C;
  bool c_inf;
  keycomb_q_part<P, L>(C, c_inf, w, i, tab_ptr(pl, g, id), l, !(id & kLocal));
  part_store(w, pbase + gid, pstride, C, c_inf);
}

template <class P, class N, int L>
__global__ __launch_bounds__(256) void k_keycomb_wide_g(Work w, Plan pl,
                                                        const uint32_t* __restrict__ gtab,
                                                        uint8_t* __restrict__ reason,
                                                        uint32_t pbase, uint32_t pstride) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = gid / L, l = gid % L;
  const uint32_t cnt = pl.counters[0];
  if (j >= cnt) return;
  const uint32_t i = pl.comb_order[j];
  J30 C;
  bool c_inf;
  part_load(w, pbase + gid, pstride, C, c_inf);
  uint32_t u1[8];
  calc_u1<N>(u1, w, i);
  g_comb_part<P, L>(C, c_inf, gtab, u1, l);
  group_sum<P, L>(C, c_inf);
  if (l == 0) reason[i] = finish_check<P>(w, i, C, c_inf, C, true) ? R_OK : R_MATH;
}

__global__ __launch_bounds__(256) void k_bitmap(const uint8_t* __restrict__ reason, uint32_t n,
                                                uint64_t* __restrict__ bitmap) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((i & ~63u) >= n) return;
  const bool ok = i < n && reason[i] == R_OK;
  const uint64_t m = __ballot(ok);
  if ((threadIdx.x & 63u) == 0) bitmap[i >> 6] = m;
}

// ---- latency path: two launches for a small batch (bh_csp_verify_p256's
// coalesced batches, small host batches). 32 lanes per record (round 3: 3 key
// windows + 1 G window + a 5-level butterfly per lane, ~140 F_p ops of chain
// against ~166 at 16 lanes). k_small: lane 0 runs prep and the record's own
// inverse (variable-time safegcd: no batch inversion, no plan, no dedup) and
// looks the key up in the registry; a registered key's record is finished by
// the group (key-table and G-comb windows over 32 lanes,
// butterfly, lane 0 checks); an unregistered one is marked for k_small_lad
// (lane 0 runs the Booth ladder while the group adds the G-comb windows) --
// a separate kernel so that neither carries the other's registers. Same
// stage functions (verify.h) as the batch path: bit-identical results.
constexpr int kSmallL = 32;
constexpr uint8_t kSmallLadder = 0xfeu;  // reason placeholder: k_small_lad's record
template <class P, class N, class CV, int HK>
__global__ __launch_bounds__(256) void k_small(BatchIn in, Work w, KeyReg g,
                                               const uint32_t* __restrict__ gtab, uint32_t n,
                                               uint8_t* __restrict__ reason) {
  __shared__ uint32_t tab_of[256 / kSmallL];
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = gid / kSmallL, l = gid % kSmallL, grp = threadIdx.x / kSmallL;
  const bool act = j < n;
  if (act && l == 0) {
    stage_prep<P, N, CV, HK>(in, w, j);
    uint32_t t = kNone;
    if ((w.st[j] & 0x7fu) == R_OK) {
      stage_inv<N, true, true>(w, j, n, n);  // this record alone (variable-time): u1, u2
      t = reg_lookup(g, w, j, key_hash(w, j));
    }
    tab_of[grp] = t;
  }
  __syncthreads();  // w (global) and tab_of (LDS) visible to the group
  if (!act) return;  // whole groups (and whole waves past n) leave together
  const uint8_t st = w.st[j] & 0x7fu;
  const uint32_t t = tab_of[grp];
  if (st != R_OK || t == kNone) {
    if (l == 0) reason[j] = st != R_OK ? st : kSmallLadder;
    return;
  }
  J30 C;
  bool c_inf;
  keycomb_part<P, kSmallL>(C, c_inf, w, gtab, j, g.tables + (size_t)t * kKTabWords, l, true);
  group_sum<P, kSmallL>(C, c_inf);
  if (l == 0) reason[j] = finish_check<P>(w, j, C, c_inf, C, true) ? R_OK : R_MATH;
}

template <class P>
__global__ __launch_bounds__(256) void k_small_lad(Work w, const uint32_t* __restrict__ gtab,
                                                   uint32_t n, uint8_t* __restrict__ reason) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t j = gid / kSmallL, l = gid % kSmallL;
  if (j >= n || reason[j] != kSmallLadder) return;  // whole groups leave together
  J30 C;
  bool c_inf = true;
  f_const(C.X, P::r1);
  f_const(C.Y, P::r1);
  f_const(C.Z, P::r1);
  if (l == 0) q_ladder<P>(C, c_inf, w, j, j >> 6, j & 63u);  // Q-table slot = record
  uint32_t u1[8];
  ld8(u1, w.e, j, w.ns);
  g_comb_part<P, kSmallL>(C, c_inf, gtab, u1, l);
  group_sum<P, kSmallL>(C, c_inf);
  if (l == 0) reason[j] = finish_check<P>(w, j, C, c_inf, C, true) ? R_OK : R_MATH;
}

// G tables (verify.h gtab_entry, gtab2_base, gtab2_entry): one lane per
// entry -- the 13-bit comb and the folded tables' base points, then (a second
// launch) the folded group / single-column entries from those base points.
template <class P>
__global__ __launch_bounds__(64) void k_gtab_build(uint32_t* gtab) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr uint32_t nc = (uint32_t)(kCombWindows * kCombEntries);
  if (t < nc) gtab_entry<P>(t, gtab + (size_t)t * kGEntry);
  else if (t < nc + kGBase) gtab2_base<P>(t - nc, gtab + kGCombWords);
}
template <class P>
__global__ __launch_bounds__(64) void k_gtab2_build(uint32_t* gtab) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < kG2Ent + kG1Ent) gtab2_entry<P>(t, gtab + kGCombWords);
}

// bh_keys_register: keys only (X || Y per record) -> Work.qx / qy / st.
template <class P, class C>
__global__ __launch_bounds__(256) void k_reg_prep(const uint8_t* __restrict__ pub, Work w,
                                                  uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t qx[9], qy[9];
  const bool ok = key_import<P, C>(pub + (size_t)i * 64, qx, qy);
  if (!ok) {
    f_const(qx, P::gx_m);
    f_const(qy, P::gy_m);
  }
  st9(w.qx, i, w.ns, qx);
  st9(w.qy, i, w.ns, qy);
  w.st[i] = ok ? R_OK : R_BAD_KEY;
}

// Per key: 0 = in the registry (new or already), R_BAD_KEY, or kRegFull.
__global__ __launch_bounds__(256) void k_reg_status(Work w, Plan pl, uint32_t n,
                                                    uint8_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if ((w.st[i] & 0x7fu) != R_OK) {
    status[i] = R_BAD_KEY;
    return;
  }
  uint32_t t = pl.rec_tab[i];
  if (t == kNone && pl.rec_slot[i] != kNone) t = pl.slot_tab[pl.rec_slot[i]];
  status[i] = (t != kNone && !(t & kLocal)) ? 0 : 0xffu;
}

}  // namespace

// ---------------------------------------------------------------------------
// Launchers (C++ linkage, used by bdls_hip.cpp)
namespace bh {

// ---- compact host batches (bh_verify_compact): expansion on the device ----
// pub[i] = keys[key_idx[i]] (64 B), and the u64 offsets as exclusive prefix
// sums of the u32 lengths (or i * stride with a fixed message length), so the
// verify passes read an ordinary bh_batch. Runs on the compute stream after
// the upload; key indices were range-checked on the host.
__global__ __launch_bounds__(256) void k_expand_keys(const uint8_t* __restrict__ keys,
                                                     const uint32_t* __restrict__ idx,
                                                     uint8_t* __restrict__ pub, uint32_t m) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint4* src = reinterpret_cast<const uint4*>(keys + (size_t)idx[i] * 64);
  uint4* dst = reinterpret_cast<uint4*>(pub + (size_t)i * 64);
  const uint4 a = src[0], b = src[1], c = src[2], d = src[3];
  dst[0] = a;
  dst[1] = b;
  dst[2] = c;
  dst[3] = d;
}

__global__ __launch_bounds__(256) void k_stride_offsets(uint64_t* __restrict__ off,
                                                        uint32_t* __restrict__ len,
                                                        uint32_t stride, uint32_t m) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  off[i] = (uint64_t)i * stride;
  len[i] = stride;
}

struct ToU64 {
  __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};

size_t expand_temp_bytes(uint32_t m) {
  size_t t = 0;
  hipcub::TransformInputIterator<uint64_t, ToU64, const uint32_t*> it(nullptr, ToU64());
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, t, it, (uint64_t*)nullptr, (int)m) != hipSuccess)
    return 0;
  return t;
}

hipError_t launch_expand(const uint8_t* keys, const uint32_t* key_idx, uint8_t* pub,
                         const uint32_t* sig_len, uint64_t* sig_off, const uint32_t* msg_len,
                         uint64_t* msg_off, uint32_t* msg_len_out, uint32_t stride, void* temp,
                         size_t temp_bytes, uint32_t m, hipStream_t s) {
  if (!m) return hipSuccess;
  const dim3 grd((m + 255) / 256), blk(256);
  if (key_idx) hipLaunchKernelGGL(k_expand_keys, grd, blk, 0, s, keys, key_idx, pub, m);
  hipError_t e;
  size_t t = temp_bytes;
  hipcub::TransformInputIterator<uint64_t, ToU64, const uint32_t*> sl(sig_len, ToU64());
  if ((e = hipcub::DeviceScan::ExclusiveSum(temp, t, sl, sig_off, (int)m, s))) return e;
  if (msg_len) {
    t = temp_bytes;
    hipcub::TransformInputIterator<uint64_t, ToU64, const uint32_t*> ml(msg_len, ToU64());
    if ((e = hipcub::DeviceScan::ExclusiveSum(temp, t, ml, msg_off, (int)m, s))) return e;
  } else {
    hipLaunchKernelGGL(k_stride_offsets, grd, blk, 0, s, msg_off, msg_len_out, stride, m);
  }
  return hipGetLastError();
}

// Results to page-locked host memory by the compute stream's own kernel: a
// device-to-host copy engine command that waits on a pass holds every later
// command of its engine ring, uploads of the next batches included
// (bdls_hip.cpp enqueue_part). Both pointers 16-byte aligned.
__global__ __launch_bounds__(256) void k_result_out(const uint4* __restrict__ src,
                                                    uint4* __restrict__ dst, size_t n16,
                                                    const uint8_t* __restrict__ src_b,
                                                    uint8_t* __restrict__ dst_b, size_t nb) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t k = i; k < n16; k += stride) dst[k] = src[k];
  for (size_t k = n16 * 16 + i; k < nb; k += stride) dst_b[k] = src_b[k];
}

hipError_t launch_result_out(const void* src, void* host_dst, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  const size_t n16 = bytes / 16;
  const uint32_t blocks = (uint32_t)std::min<size_t>(1024, (n16 + 255) / 256 + 1);
  hipLaunchKernelGGL(k_result_out, dim3(blocks), dim3(256), 0, s, (const uint4*)src,
                     (uint4*)host_dst, n16, (const uint8_t*)src, (uint8_t*)host_dst, bytes);
  return hipGetLastError();
}

hipError_t launch_gtab_build(int curve, uint32_t* gtab, hipStream_t s) {
  const int nt = kCombWindows * kCombEntries + (int)kGBase, nt2 = (int)(kG2Ent + kG1Ent);
  if (curve == 0) {
    hipLaunchKernelGGL((k_gtab_build<F30_p256>), dim3((nt + 63) / 64), dim3(64), 0, s, gtab);
    hipLaunchKernelGGL((k_gtab2_build<F30_p256>), dim3((nt2 + 63) / 64), dim3(64), 0, s, gtab);
  } else {
    hipLaunchKernelGGL((k_gtab_build<F30_k1>), dim3((nt + 63) / 64), dim3(64), 0, s, gtab);
    hipLaunchKernelGGL((k_gtab2_build<F30_k1>), dim3((nt2 + 63) / 64), dim3(64), 0, s, gtab);
  }
  return hipGetLastError();
}

static const uint8_t* key_bytes(const BatchIn& in) { return in.pub; }
static const uint8_t* key_bytes(const BdlsIn& in) { return in.xy; }

static void launch_key_count(const Work& w, const Plan& pl, const uint8_t* pub, uint32_t n,
                             dim3 grd, dim3 blk, hipStream_t s) {
  if (((uintptr_t)pub & 15u) == 0)
    hipLaunchKernelGGL(k_key_count<true>, grd, blk, 0, s, w, pl, pub, n);
  else
    hipLaunchKernelGGL(k_key_count<false>, grd, blk, 0, s, w, pl, pub, n);
}

// The dedup table's reset (slot_hash 0, slot_rep / slot_tab kNone, slot_cnt 0,
// the counters 0) in ONE launch: 16-byte stores, a grid-stride loop over the
// hc / 4 quads (hc is a power of two >= 256) -- instead of five memset
// kernels, each with its own launch gap (round 4).
__global__ __launch_bounds__(256) void k_plan_reset(Plan pl) {
  const uint32_t nq = pl.hc / 4u;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += stride) {
    const uint4 z = make_uint4(0u, 0u, 0u, 0u), f = make_uint4(kNone, kNone, kNone, kNone);
    reinterpret_cast<uint4*>(pl.slot_hash)[2u * q] = z;
    reinterpret_cast<uint4*>(pl.slot_hash)[2u * q + 1u] = z;
    reinterpret_cast<uint4*>(pl.slot_rep)[q] = f;
    reinterpret_cast<uint4*>(pl.slot_cnt)[q] = z;
    reinterpret_cast<uint4*>(pl.slot_tab)[q] = f;
  }
  if (blockIdx.x == 0 && threadIdx.x < 4) pl.counters[threadIdx.x] = 0u;
}

static hipError_t plan_reset(const Plan& pl, hipStream_t s) {
  // (carve_work takes every plan array at a 256-byte boundary, hc >= 256)
  const uint32_t nq = pl.hc / 4u;
  hipLaunchKernelGGL(k_plan_reset, dim3(std::min<uint32_t>((nq + 255) / 256, 2048)), dim3(256),
                     0, s, pl);
  return hipGetLastError();
}

// Group the comb list by table id so the (on average 16) records of one key
// sit in adjacent lanes of one wave: their table reads then hit the same L2
// lines instead of streaming the 58 KB table once per record. Order within a
// key does not matter (one record per lane), so this is a counting sort over
// the compacted ids (k_comb_keys' mapping): histogram, exclusive scan,
// scatter -- three passes instead of a radix / merge sort's ten. Wide table-id
// ranges (a registry above 2^16 tables) fall back to the radix sort. Runs on
// plan buffers that are dead once k_split has routed every record: slot_hash
// holds the scan temp, slot_cnt / slot_rep the histogram and offsets (or the
// sort keys), and rec_slot receives the grouped list -- so after this call
// rec_slot no longer holds slots, and the list is published as
// Plan::comb_order (every later kernel reads that, never rec_slot).
constexpr uint32_t kSortMin = 65536;
constexpr uint32_t kCountSortBits = 16;  // histogram of 2^(bits+1) ids

__device__ __forceinline__ uint32_t comb_key(uint32_t t, uint32_t bits) {
  return (t & kLocal) ? ((1u << bits) | (t & ~kLocal)) : t;
}

__global__ __launch_bounds__(256) void k_comb_hist(Plan pl, uint32_t bits,
                                                   uint32_t* __restrict__ hist) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= pl.counters[0]) return;
  atomicAdd(&hist[comb_key(pl.rec_tab[pl.comb_list[j]], bits)], 1u);
}

__global__ __launch_bounds__(256) void k_comb_scatter(Plan pl, uint32_t bits,
                                                      uint32_t* __restrict__ offs,
                                                      uint32_t* __restrict__ out) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= pl.counters[0]) return;
  const uint32_t i = pl.comb_list[j];
  out[atomicAdd(&offs[comb_key(pl.rec_tab[i], bits)], 1u)] = i;
}

// Radix-sort fallback keys: table ids compacted to `bits` + 2 bits so the sort
// runs only the passes it needs (registry id < 2^bits as is, kLocal | job as
// 2^bits | job); entries past the list length get 2^(bits+1) and sort last.
__global__ __launch_bounds__(256) void k_comb_keys(Plan pl, uint32_t n, uint32_t bits,
                                                   uint32_t* __restrict__ keys) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t cnt = pl.counters[0];
  if (j < cnt) {
    keys[j] = comb_key(pl.rec_tab[pl.comb_list[j]], bits);
  } else {
    keys[j] = 2u << bits;
    pl.comb_list[j] = 0;
  }
}

static hipError_t comb_sort(const Plan& pl, const KeyReg& g, uint32_t n, hipStream_t s,
                            Plan* out) {
  *out = pl;
  if (n < kSortMin) return hipSuccess;
  uint32_t bits = 16;
  while ((1ull << bits) < (uint64_t)g.cap) bits++;
  const uint32_t hsize = 2u << bits;
  hipError_t e;
  if (bits <= kCountSortBits && hsize <= pl.hc) {
    size_t temp = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, temp, pl.slot_cnt, pl.slot_rep,
                                              (int)hsize, s)))
      return e;
    if (temp > (size_t)pl.hc * 8) return hipSuccess;  // keep the unsorted list
    if ((e = hipMemsetAsync(pl.slot_cnt, 0, (size_t)hsize * 4, s))) return e;
    const dim3 grd((n + 255) / 256), blk(256);
    hipLaunchKernelGGL(k_comb_hist, grd, blk, 0, s, pl, bits, pl.slot_cnt);
    if ((e = hipcub::DeviceScan::ExclusiveSum(pl.slot_hash, temp, pl.slot_cnt, pl.slot_rep,
                                              (int)hsize, s)))
      return e;
    hipLaunchKernelGGL(k_comb_scatter, grd, blk, 0, s, pl, bits, pl.slot_rep, pl.rec_slot);
  } else {
    const int end_bit = (int)bits + 2;
    size_t temp = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp, pl.slot_rep, pl.slot_cnt,
                                                pl.comb_list, pl.rec_slot, (int)n, 0, end_bit,
                                                s)))
      return e;
    if (temp > (size_t)pl.hc * 8) return hipSuccess;  // keep the unsorted list
    hipLaunchKernelGGL(k_comb_keys, dim3((n + 255) / 256), dim3(256), 0, s, pl, n, bits,
                       pl.slot_rep);
    if ((e = hipcub::DeviceRadixSort::SortPairs(pl.slot_hash, temp, pl.slot_rep, pl.slot_cnt,
                                                pl.comb_list, pl.rec_slot, (int)n, 0, end_bit,
                                                s)))
      return e;
  }
  out->comb_order = pl.rec_slot;
  out->rec_slot = nullptr;  // consumed: holds the grouped list now
  return hipSuccess;
}


// BH_DIGEST_GRP=0: the one-lane-per-record k_digest for fused SHA-256 (A/B)
static bool digest_grp() {
  static const bool on = [] {
    const char* e = getenv("BH_DIGEST_GRP");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

// Full launch sequence. ev (optional, 7 events) brackets: prep | inv | plan
// (lookup + dedup + split) | key tables + ladder | publish | key comb + bitmap.
// BDLS batches hash their SignedProtos on the second stream (o.aux): forked
// after the plan reset, joined before the first kernel that needs u1. Small
// (wide) BDLS batches, and small Fabric batches with fused hashing, run the u2 Q
// halves of the ladder and key comb before the join and only the u1 G halves
// after it (the digests of long lock / decide messages, or of a block's 4 KB
// creator payloads, are serial chains as long as prep + inverse + plan).
template <class P, class N, class C, class IN>
static hipError_t seq(const IN& in, const Work& w, const Plan& pl, const KeyReg& g,
                      const uint32_t* gtab, uint32_t n, const LaunchOpts& o, uint64_t* bitmap,
                      uint8_t* reason, hipStream_t s, hipEvent_t* ev) {
  constexpr bool kBdls = std::is_same_v<IN, BdlsIn>;
  const dim3 blk(256);
  const dim3 grd((n + 255) / 256);
  // the multi-lane kernels of small batches: o.wide_block threads per
  // workgroup (64: one wave each, spread over CUs)
  const uint32_t wb = o.wide_block ? o.wide_block : 256u;
  const dim3 wblk(wb);
  auto wgrd = [&](uint32_t lanes) { return dim3((lanes + wb - 1) / wb); };
  const uint32_t nlanes = (n + o.inv_chunk - 1) / o.inv_chunk;  // records per lane ~ inv_chunk
  const dim3 grc((nlanes + 255) / 256);
  bool fused = false;  // Fabric records whose digest the device computes
  if constexpr (!kBdls) fused = (in.flags & (BHF_HASH_SHA256 | BHF_HASH_SHA3_256)) != 0;
  const bool split = (kBdls || fused) && o.wide > 1;
  // partial-sum slots (verify.h gpart_slots): ladder pairs, then key-comb groups
  const uint32_t pstride = (uint32_t)gpart_slots(w.ns), pbase = 2u * w.ns;
  hipError_t e;
#define REC(k)                                                 \
  if (ev) {                                                    \
    if ((e = hipEventRecord(ev[k], s)) != hipSuccess) return e; \
  }
  // Host batches whose keys arrived first (records_ready): the key half --
  // key import, plan, table builds -- runs while the signatures and messages
  // are still uploading; the records' half after the event. One-lane comb
  // batches without registry writes or stage timing; otherwise wait up front.
  if (o.records_ready) {
    const bool ll1 = o.ll_tables && o.wide <= 1;
    if (kBdls || split || !ll1 || o.keep || ev) {
      if ((e = hipStreamWaitEvent(s, (hipEvent_t)o.records_ready, 0))) return e;
    } else if constexpr (!kBdls) {
      if ((e = plan_reset(pl, s))) return e;
      hipLaunchKernelGGL((k_prep_keys<P, C>), grd, blk, 0, s, in, w, n);
      hipLaunchKernelGGL(k_key_insert, grd, blk, 0, s, w, pl, g, n);
      launch_key_count(w, pl, key_bytes(in), n, grd, blk, s);
      hipLaunchKernelGGL(k_key_plan, grd, blk, 0, s, w, pl, g, n, o.min_uses, o.min_batch, 0u,
                         0u);
      const uint32_t tb = (pl.max_tables + kBuildPerBlock - 1) / kBuildPerBlock;
      if (o.ev_build_wait && (e = hipStreamWaitEvent(s, (hipEvent_t)o.ev_build_wait, 0)))
        return e;
      hipLaunchKernelGGL((k_ktab_ladder<P>), dim3(tb), blk, 0, s, w, pl, g, gtab, reason, tb, 0u,
                         1u);
      if (o.ev_build_done && (e = hipEventRecord((hipEvent_t)o.ev_build_done, s))) return e;
      if ((e = hipStreamWaitEvent(s, (hipEvent_t)o.records_ready, 0))) return e;
      launch_prep<P, N, C>(in, w, n, grd, blk, s);
      hipLaunchKernelGGL((k_inv<N, true>), grc, blk, 0, s, w, n, nlanes);
      hipLaunchKernelGGL(k_split, dim3((n + kSplitBlock - 1) / kSplitBlock), dim3(kSplitBlock), 0,
                         s, w, pl, n, reason);
      Plan plk;
      if ((e = comb_sort(pl, g, n, s, &plk))) return e;
      // the ladder records alone (no table blocks)
      hipLaunchKernelGGL((k_ktab_ladder<P>), grd, blk, 0, s, w, plk, g, gtab, reason, 0u, grd.x,
                         1u);
      hipLaunchKernelGGL((k_keycomb<P>), grd, blk, 0, s, w, plk, g, gtab, reason, 1u);
      hipLaunchKernelGGL(k_bitmap, grd, blk, 0, s, reason, n, bitmap);
      return hipGetLastError();
    }
  }
  // digests: on the second stream when there is one (forked here, joined
  // before the first kernel that needs u1), else first on this stream. The
  // fork and the digest launch come before the plan reset (round 6): on a
  // latency call the digest chain is the critical path, and every host
  // launch ahead of it delays it by the launch's API time.
  bool joined = true;
  hipStream_t hs = s;
  if ((kBdls || split) && o.aux) {
    hs = (hipStream_t)o.aux;
    if ((e = hipEventRecord((hipEvent_t)o.ev_fork, s))) return e;
    if ((e = hipStreamWaitEvent(hs, (hipEvent_t)o.ev_fork, 0))) return e;
    joined = false;
  }
  if constexpr (kBdls) {
    hipLaunchKernelGGL((k_bdls_hash<C>), dim3((n * 4 + 255) / 256), blk, 0, hs, in, w, n);
    if (!joined && (e = hipEventRecord((hipEvent_t)o.ev_join, hs))) return e;
  } else if (split) {
    if (in.flags & BHF_HASH_SHA3_256) {
      hipLaunchKernelGGL((k_digest<C, HK_SHA3_256>), grd, blk, 0, hs, in, w, n);
    } else if ((in.flags & BHF_HASH_SHA256) && digest_grp()) {
      hipLaunchKernelGGL((k_digest_grp<C>), dim3((n * kDigG + kDigBlock - 1) / kDigBlock),
                         dim3(kDigBlock), 0, hs, in, w, n);
    } else {
      hipLaunchKernelGGL((k_digest<C, HK_GIVEN_OR_SHA256>), grd, blk, 0, hs, in, w, n);
    }
    if (!joined && (e = hipEventRecord((hipEvent_t)o.ev_join, hs))) return e;
  }
  if ((e = plan_reset(pl, s))) return e;
  REC(0);
  if constexpr (kBdls) {
    hipLaunchKernelGGL((k_prep<P, N, C, BdlsIn, 0>), grd, blk, 0, s, in, w, n);
  } else if (split) {
    if (in.flags & BHF_HASH_SHA3_256)
      hipLaunchKernelGGL((k_prep<P, N, C, BatchIn, HK_SHA3_256, true>), grd, blk, 0, s, in, w, n);
    else
      hipLaunchKernelGGL((k_prep<P, N, C, BatchIn, HK_GIVEN_OR_SHA256, true>), grd, blk, 0, s, in,
                         w, n);
  } else {
    launch_prep<P, N, C>(in, w, n, grd, blk, s);
  }
  REC(1);
  auto join = [&]() -> hipError_t {
    if (joined) return hipSuccess;
    joined = true;
    return hipStreamWaitEvent(s, (hipEvent_t)o.ev_join, 0);
  };
  if (split) {
    hipLaunchKernelGGL((k_inv<N, false>), grc, blk, 0, s, w, n, nlanes);
  } else {
    if ((e = join())) return e;
    hipLaunchKernelGGL((k_inv<N, true>), grc, blk, 0, s, w, n, nlanes);
  }
  REC(2);
  hipLaunchKernelGGL(k_key_insert, grd, blk, 0, s, w, pl, g, n);
  launch_key_count(w, pl, key_bytes(in), n, grd, blk, s);
  hipLaunchKernelGGL(k_key_plan, grd, blk, 0, s, w, pl, g, n, o.min_uses, o.min_batch,
                     o.keep ? 1u : 0u, 0u);
  hipLaunchKernelGGL(k_split, dim3((n + kSplitBlock - 1) / kSplitBlock), dim3(kSplitBlock), 0, s,
                     w, pl, n, reason);
  Plan plc;
  if (o.wide <= 1) {
    if ((e = comb_sort(pl, g, n, s, &plc))) return e;
  } else {
    plc = pl;
  }
  REC(3);
  const uint32_t tab_blocks = (pl.max_tables + kBuildPerBlock - 1) / kBuildPerBlock;
  // Lim-Lee comb tables for the one-lane key comb (o.wide == 1)
  const uint32_t ll = (o.ll_tables && o.wide <= 1) ? 1u : 0u;
  // u1 G of the key-comb list: folded into k_keycomb's Horner with comb tables
  // (round 5); with windowed tables (BH_LL=0) inside k_ktab_ladder beside the
  // builds, stored by list position (a separate kernel on the aux stream, 146
  // VGPRs, did not run faster: profiles/r04/v14)
  const uint32_t gp_blocks = (o.wide <= 1 && !ll) ? grd.x : 0u;
  // from here on only plc (rec_slot consumed by the sort)
  if (split) {
    // key tables (no u1), then the u2 Q halves; u1 G after the join
    hipLaunchKernelGGL((k_ktab_ladder<P>), dim3(tab_blocks), blk, 0, s, w, plc, g, gtab, reason,
                       tab_blocks, 0u, 0u);
    if (o.keep) launch_reg_win<P>(w, plc, g, s);  // the new registry slots' windows
    if constexpr (!P::a_is_minus3)
      hipLaunchKernelGGL((k_ladder2_q<P>), wgrd(2 * n), wblk, 0, s, w, plc,
                         pstride);
    else
      hipLaunchKernelGGL((k_ladder1_q<P>), wgrd(n), wblk, 0, s, w, plc, pstride);
    if (o.wide == 16)
      hipLaunchKernelGGL((k_keycomb_wide_q<P, 16>), wgrd(n * 16), wblk, 0, s, w, plc,
                         g, pbase, pstride);
    else
      hipLaunchKernelGGL((k_keycomb_wide_q<P, 4>), wgrd(n * 4), wblk, 0, s, w, plc, g,
                         pbase, pstride);
    REC(4);
    if (o.keep)
      hipLaunchKernelGGL(k_reg_publish, dim3((pl.max_tables + 255) / 256), blk, 0, s, w, plc, g);
    if ((e = join())) return e;
    hipLaunchKernelGGL((k_ladder2_g<P, N, P::a_is_minus3 ? 1 : 2>),
                       wgrd(kLadGLanes * n), wblk, 0, s, w, plc, gtab, reason,
                       pstride);
    REC(5);
    if (o.wide == 16)
      hipLaunchKernelGGL((k_keycomb_wide_g<P, N, 16>), wgrd(n * 16), wblk, 0, s, w,
                         plc, gtab, reason, pbase, pstride);
    else
      hipLaunchKernelGGL((k_keycomb_wide_g<P, N, 4>), wgrd(n * 4), wblk, 0, s, w,
                         plc, gtab, reason, pbase, pstride);
    hipLaunchKernelGGL(k_bitmap, grd, blk, 0, s, reason, n, bitmap);
    REC(6);
    return hipGetLastError();
  }
  // (small secp256k1 batches are BDLS, hence split: the 2-lane GLV ladder)
  if (o.ev_build_wait && (e = hipStreamWaitEvent(s, (hipEvent_t)o.ev_build_wait, 0))) return e;
  hipLaunchKernelGGL((k_ktab_ladder<P>), dim3(tab_blocks + grd.x + gp_blocks), blk, 0, s, w, plc,
                     g, gtab, reason, tab_blocks, grd.x, ll);
  if (o.keep) launch_reg_win<P>(w, plc, g, s);  // the new registry slots' windows
  if (o.ev_build_done && (e = hipEventRecord((hipEvent_t)o.ev_build_done, s))) return e;
  REC(4);
  if (o.keep)
    hipLaunchKernelGGL(k_reg_publish, dim3((pl.max_tables + 255) / 256), blk, 0, s, w, plc, g);
  REC(5);
  switch (o.wide) {
    case 4:
      hipLaunchKernelGGL((k_keycomb_wide<P, 4>), wgrd(n * 4), wblk, 0, s, w, plc, g,
                         gtab, reason);
      break;
    case 16:
      hipLaunchKernelGGL((k_keycomb_wide<P, 16>), wgrd(n * 16), wblk, 0, s, w, plc,
                         g, gtab, reason);
      break;
    default:
      hipLaunchKernelGGL((k_keycomb<P>), grd, blk, 0, s, w, plc, g, gtab, reason, ll);
  }
  hipLaunchKernelGGL(k_bitmap, grd, blk, 0, s, reason, n, bitmap);
  REC(6);
#undef REC
  return hipGetLastError();
}

hipError_t launch_verify(int curve, const BatchIn& in, const Work& w, const Plan& pl,
                         const KeyReg& g, const uint32_t* gtab, uint32_t n, const LaunchOpts& o,
                         uint64_t* bitmap, uint8_t* reason, hipStream_t s, hipEvent_t* ev) {
  // Fabric / BCCSP records: P-256 only (the low-S table of bccsp/utils covers
  // the NIST curves; secp256k1 never reaches bccsp/sw).
  if (curve != 0) return hipErrorInvalidValue;
  return seq<F30_p256, Fn_p256, Cv_p256>(in, w, pl, g, gtab, n, o, bitmap, reason, s, ev);
}

hipError_t launch_verify_bdls(int curve, const BdlsIn& in, const Work& w, const Plan& pl,
                              const KeyReg& g, const uint32_t* gtab, uint32_t n,
                              const LaunchOpts& o, uint64_t* bitmap, uint8_t* reason,
                              hipStream_t s, hipEvent_t* ev) {
  if (curve == 0)
    return seq<F30_p256, Fn_p256, Cv_p256>(in, w, pl, g, gtab, n, o, bitmap, reason, s, ev);
  return seq<F30_k1, Fn_k1, Cv_k1>(in, w, pl, g, gtab, n, o, bitmap, reason, s, ev);
}

// The latency path (k_small): P-256 Fabric / BCCSP records only; reasons only
// (the host forms the bitmap).
// bs: threads per workgroup (64 = one wave per workgroup, so a latency-bound
// batch of a few waves spreads over CUs instead of sharing one CU's SIMDs).
hipError_t launch_small(int curve, const BatchIn& in, const Work& w, const KeyReg& g,
                        const uint32_t* gtab, uint32_t n, uint8_t* reason, hipStream_t s,
                        uint32_t bs) {
  if (curve != 0 || !n) return n ? hipErrorInvalidValue : hipSuccess;
  const dim3 grd((n * kSmallL + bs - 1) / bs), blk(bs);
  if (in.flags & BHF_HASH_SHA3_256)
    hipLaunchKernelGGL((k_small<F30_p256, Fn_p256, Cv_p256, HK_SHA3_256>), grd, blk, 0, s, in, w,
                       g, gtab, n, reason);
  else
    hipLaunchKernelGGL((k_small<F30_p256, Fn_p256, Cv_p256, HK_GIVEN_OR_SHA256>), grd, blk, 0, s,
                       in, w, g, gtab, n, reason);
  hipLaunchKernelGGL((k_small_lad<F30_p256>), grd, blk, 0, s, w, gtab, n, reason);
  return hipGetLastError();
}

// bh_keys_register: import, dedup against the registry and within the call,
// build a registry table per new key, publish, per-key status.
template <class P, class C>
static hipError_t reg_seq(const uint8_t* pub, const Work& w, const Plan& pl, const KeyReg& g,
                          uint32_t n, uint8_t* status, hipStream_t s) {
  const dim3 blk(256);
  const dim3 grd((n + 255) / 256);
  hipError_t e;
  if ((e = plan_reset(pl, s))) return e;
  hipLaunchKernelGGL((k_reg_prep<P, C>), grd, blk, 0, s, pub, w, n);
  hipLaunchKernelGGL(k_key_insert, grd, blk, 0, s, w, pl, g, n);
  launch_key_count(w, pl, pub, n, grd, blk, s);
  hipLaunchKernelGGL(k_key_plan, grd, blk, 0, s, w, pl, g, n, 1u, 0u, 1u, 1u);
  const uint32_t tab_blocks = (pl.max_tables + kBuildPerBlock - 1) / kBuildPerBlock;
  hipLaunchKernelGGL((k_ktab_ladder<P>), dim3(tab_blocks), blk, 0, s, w, pl, g,
                     (const uint32_t*)nullptr, (uint8_t*)nullptr, tab_blocks, 0u, 0u);
  launch_reg_win<P>(w, pl, g, s);
  hipLaunchKernelGGL(k_reg_publish, dim3((pl.max_tables + 255) / 256), blk, 0, s, w, pl, g);
  hipLaunchKernelGGL(k_reg_status, grd, blk, 0, s, w, pl, n, status);
  return hipGetLastError();
}

hipError_t launch_register(int curve, const uint8_t* pub, const Work& w, const Plan& pl,
                           const KeyReg& g, uint32_t n, uint8_t* status, hipStream_t s) {
  if (curve == 0) return reg_seq<F30_p256, Cv_p256>(pub, w, pl, g, n, status, s);
  return reg_seq<F30_k1, Cv_k1>(pub, w, pl, g, n, status, s);
}

}  // namespace bh
