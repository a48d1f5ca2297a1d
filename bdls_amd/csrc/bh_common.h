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
#else
#define BH_HD static inline __attribute__((always_inline))
#define BH_HDNI static __attribute__((noinline))
#endif

namespace bh {

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
