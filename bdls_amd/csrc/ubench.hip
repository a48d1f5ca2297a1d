// Micro-benchmarks for the roofline basis (run on the MI355X box):
//   mad   : v_mad_u64_u32 throughput (32x32+64 -> 64, the CIOS product step)
//   add   : v_add_co_u32 / v_addc_co_u32 carry-chain throughput
//   fmul  : P-256 Montgomery multiplications per second (mont_mul<Fp_p256>)
//   fsqr  : P-256 Montgomery squarings per second
//   dbl   : P-256 Jacobian doublings per second
// Prints one JSON object. Peak figures = ops / kernel time with the whole chip
// busy (grid = 256 CUs x 8 blocks x 256 threads).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ec.h"

using namespace bh;

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                          \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ __launch_bounds__(256) void k_mad(uint64_t* out, int iters) {
  uint32_t a = threadIdx.x * 2654435761u + blockIdx.x, b = a ^ 0x9e3779b9u;
  uint64_t acc[8];
  uint32_t x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    acc[k] = a + k;
    x[k] = b + 3 * k;
  }
  // 8 independent chains; the multiplicand depends on the previous result so
  // nothing folds: acc = lo(acc) * x + acc  (one v_mad_u64_u32 each)
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) acc[k] = (uint64_t)(uint32_t)acc[k] * x[k] + acc[k];
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(uint64_t* out, int iters) {
  uint32_t x[8], y[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    x[k] = threadIdx.x + k;
    y[k] = blockIdx.x * 77 + k;
  }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = __builtin_addc(x[k], y[k], c, &c);
      y[0] ^= c;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int SQR>
__global__ __launch_bounds__(256) void k_fmul(uint64_t* out, int iters) {
  uint32_t a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    a[k] = (threadIdx.x + 1) * (k + 3);
    b[k] = (blockIdx.x + 7) * (k + 11);
  }
  a[7] &= 0x7fffffffu;
  b[7] &= 0x7fffffffu;
  for (int i = 0; i < iters; i++) {
    if (SQR) mont_sqr<Fp_p256>(a, a);
    else mont_mul<Fp_p256>(a, a, b);
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_dbl(uint64_t* out, int iters) {
  Jac P;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    P.X[k] = (threadIdx.x + 1) * (k + 3);
    P.Y[k] = (blockIdx.x + 7) * (k + 11);
    P.Z[k] = k + 1;
  }
  P.X[7] &= 0x7fffffffu;
  P.Y[7] &= 0x7fffffffu;
  for (int i = 0; i < iters; i++) pt_dbl<Fp_p256, Cv_p256>(P, P);
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= P.X[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
double time_kernel(K kern, int blocks, int iters, uint64_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 2);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters);
  CHK(hipEventRecord(b, 0));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e-3;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;
  const double threads = (double)blocks * 256;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  const int it_mad = 4000, it_add = 4000, it_f = 20000, it_d = 2000;
  double t_mad = time_kernel(k_mad, blocks, it_mad, out);
  double t_add = time_kernel(k_add, blocks, it_add, out);
  double t_mul = time_kernel(k_fmul<0>, blocks, it_f, out);
  double t_sqr = time_kernel(k_fmul<1>, blocks, it_f, out);
  double t_dbl = time_kernel(k_dbl, blocks, it_d, out);
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, "
         "\"mad_u64_u32_per_s\": %.4e, \"addc_per_s\": %.4e, "
         "\"p256_mont_mul_per_s\": %.4e, \"p256_mont_sqr_per_s\": %.4e, "
         "\"p256_dbl_per_s\": %.4e}\n",
         prop.gcnArchName, cus, prop.clockRate, threads * it_mad * 16 * 8 / t_mad,
         threads * it_add * 16 * 8 / t_add, threads * it_f / t_mul, threads * it_f / t_sqr,
         threads * it_d / t_dbl);
  return 0;
}
