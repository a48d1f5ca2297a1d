// HIP kernels for gfx950 (MI355X): batched ECDSA verification.
//
// Launch structure per batch (one stream, see bdls_hip.cpp):
//   k_prep   <<<ceil(n/256), 256>>>   parse / checks / SHA-256 / Montgomery inputs
//   k_inv    <<<ceil(chunks/256),256>>> batched s^-1 mod n, u1, u2
//   k_ladder <<<ceil(n/256), 256>>>   u1 G + u2 Q, x check, bitmap word per wave
// plus k_gtab_build once per device at bh_init (fixed-base comb table for G).
#include "verify.h"

using namespace bh;

namespace {

template <class P, class N, class C>
__global__ __launch_bounds__(256) void k_prep(BatchIn in, Work w, uint32_t n) {
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

template <class P>
__global__ __launch_bounds__(256) void k_ladder(Work w, const uint32_t* __restrict__ gtab,
                                                uint32_t n, uint64_t* __restrict__ bitmap,
                                                uint8_t* __restrict__ reason) {
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = i0 >> 6;
  // Waves wholly past n exit: the per-wave Q-table scratch exists only for
  // ceil(n/64) waves (wave-uniform branch).
  if ((i0 & ~63u) >= n) return;
  // Inside the last wave every lane runs (lanes past n recompute record n-1
  // into their own scratch slots) so the ballot below sees the whole wave.
  const bool active = i0 < n;
  const uint32_t i = active ? i0 : (n - 1);
  const uint8_t st = w.st[i];
  const bool pre_ok = (st & 0x7fu) == R_OK;
  bool ok = stage_ladder<P>(w, gtab, i, wave, lane);
  ok = ok && pre_ok && active;
  const uint64_t m = __ballot(ok);
  if (lane == 0) bitmap[wave] = m;
  if (active) reason[i] = pre_ok ? (ok ? R_OK : R_MATH) : (uint8_t)(st & 0x7fu);
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

hipError_t launch_verify(int curve, const BatchIn& in, const Work& w, const uint32_t* gtab,
                         uint32_t n, uint32_t chunk, uint64_t* bitmap, uint8_t* reason,
                         hipStream_t s) {
  const dim3 blk(256);
  const dim3 grd((n + 255) / 256);
  const uint32_t nchunks = (n + chunk - 1) / chunk;
  const dim3 grc((nchunks + 255) / 256);
  if (curve == 0) {
    hipLaunchKernelGGL((k_prep<F30_p256, Fn_p256, Cv_p256>), grd, blk, 0, s, in, w, n);
    hipLaunchKernelGGL((k_inv<Fn_p256>), grc, blk, 0, s, w, n, chunk);
    hipLaunchKernelGGL((k_ladder<F30_p256>), grd, blk, 0, s, w, gtab, n, bitmap,
                       reason);
  } else {
    hipLaunchKernelGGL((k_prep<F30_k1, Fn_k1, Cv_k1>), grd, blk, 0, s, in, w, n);
    hipLaunchKernelGGL((k_inv<Fn_k1>), grc, blk, 0, s, w, n, chunk);
    hipLaunchKernelGGL((k_ladder<F30_k1>), grd, blk, 0, s, w, gtab, n, bitmap,
                       reason);
  }
  return hipGetLastError();
}

hipError_t launch_verify_timed(int curve, const BatchIn& in, const Work& w, const uint32_t* gtab,
                               uint32_t n, uint32_t chunk, uint64_t* bitmap, uint8_t* reason,
                               hipStream_t s, hipEvent_t ev[4]) {
  if (curve != 0) return hipErrorInvalidValue;
  const dim3 blk(256);
  const dim3 grd((n + 255) / 256);
  const uint32_t nchunks = (n + chunk - 1) / chunk;
  const dim3 grc((nchunks + 255) / 256);
  if (hipError_t e = hipEventRecord(ev[0], s)) return e;
  hipLaunchKernelGGL((k_prep<F30_p256, Fn_p256, Cv_p256>), grd, blk, 0, s, in, w, n);
  if (hipError_t e = hipEventRecord(ev[1], s)) return e;
  hipLaunchKernelGGL((k_inv<Fn_p256>), grc, blk, 0, s, w, n, chunk);
  if (hipError_t e = hipEventRecord(ev[2], s)) return e;
  hipLaunchKernelGGL((k_ladder<F30_p256>), grd, blk, 0, s, w, gtab, n, bitmap,
                     reason);
  if (hipError_t e = hipEventRecord(ev[3], s)) return e;
  return hipGetLastError();
}

hipError_t launch_stage(int stage, const BatchIn& in, const Work& w, const uint32_t* gtab,
                        uint32_t n, uint32_t chunk, uint64_t* bitmap, uint8_t* reason,
                        hipStream_t s) {
  const dim3 blk(256);
  const dim3 grd((n + 255) / 256);
  const uint32_t nchunks = (n + chunk - 1) / chunk;
  const dim3 grc((nchunks + 255) / 256);
  if (stage == 0)
    hipLaunchKernelGGL((k_prep<F30_p256, Fn_p256, Cv_p256>), grd, blk, 0, s, in, w, n);
  else if (stage == 1)
    hipLaunchKernelGGL((k_inv<Fn_p256>), grc, blk, 0, s, w, n, chunk);
  else
    hipLaunchKernelGGL((k_ladder<F30_p256>), grd, blk, 0, s, w, gtab, n, bitmap,
                       reason);
  return hipGetLastError();
}

}  // namespace bh
