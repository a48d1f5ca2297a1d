// Common macros for the bdls-hip device code.
//
// Every arithmetic header in this directory compiles two ways:
//   * as HIP device code for gfx950 (the product: libbdlship.so), and
//   * as plain host C++ with amdclang++ for the TEST-ONLY host harness
//     (tests/native/hostsim.cpp), so the arithmetic can be checked against the
//     oracle in a container without a GPU. The product library never calls the
//     host instantiation: there is no CPU fallback on the verify path.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BH_HD __host__ __device__ __forceinline__
#define BH_HDNI __host__ __device__ __attribute__((noinline))
#define BH_HDM __host__ __device__ __forceinline__  // member functions
#else
#define BH_HD static inline __attribute__((always_inline))
#define BH_HDNI static __attribute__((noinline))
#define BH_HDM inline __attribute__((always_inline))
#endif

namespace bh {

// (hi:lo) >> 8*sh, low 32 bits (sh in 0..3): one v_alignbyte_b32 on gfx950.
BH_HD uint32_t funnel_bytes(uint32_t lo, uint32_t hi, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
#endif
}

BH_HD uint32_t ld_aligned_u32(const uint8_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *reinterpret_cast<const uint32_t*>(p);
#else
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
#endif
}

// NW little-endian 32-bit words from byte address p of any alignment, with
// dword loads only (aligned dwords overlapping [p, p + 4 NW), so nothing past
// the dword holding the last byte is touched) and one funnel shift per word.
// Replaces 4 NW byte loads on the hashing paths.
template <int NW>
BH_HD void load_le_words(uint32_t* out, const uint8_t* p) {
  const uint32_t a = (uint32_t)((uintptr_t)p & 3u);
  const uint8_t* q = p - a;
  uint32_t prev = ld_aligned_u32(q);
#pragma unroll
  for (int i = 0; i < NW; i++) {
    const uint32_t nxt = (i + 1 < NW || a != 0u) ? ld_aligned_u32(q + 4 * (i + 1)) : 0u;
    out[i] = funnel_bytes(prev, nxt, a);
    prev = nxt;
  }
}

BH_HD uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

// Reason codes: identical to include/bdls_hip.h (BH_R_*) and oracle/ecdsa_ref.py.
enum : uint8_t {
  R_OK = 0,
  R_EMPTY_SIG = 1,
  R_EMPTY_DIGEST = 2,
  R_DER = 3,
  R_R_NONPOS = 4,
  R_S_NONPOS = 5,
  R_HIGH_S = 6,
  R_BAD_KEY = 7,
  R_R_RANGE = 8,
  R_MATH = 9,
  R_S_RANGE = 10,
};

}  // namespace bh
