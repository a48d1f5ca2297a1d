// Micro-benchmarks for the roofline basis, run on the MI355X box.
//
//   mad_tput   v_mad_u64_u32 throughput: NCH independent chains per lane,
//              8 waves/SIMD, results kept live (no folding)
//   mad_lat    one dependent chain per lane, 1 wave/SIMD -> cycles per mad
//   add_tput   v_add_u32 throughput, 16 independent chains, 8 waves/SIMD
//   f30_mul    radix-2^30 P-256 Montgomery products per second (fp30.h)
//   clock      in-kernel s_memtime / s_memrealtime (100 MHz) ratio
// One JSON object on stdout. Rates are lane-operations per second, chip-wide.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "fp30.h"

using namespace bh;

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                          \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

template <int NCH>
__global__ __launch_bounds__(256) void k_mad(uint64_t* out, int iters) {
  uint64_t acc[NCH];
  uint32_t x[NCH];
#pragma unroll
  for (int k = 0; k < NCH; k++) {
    acc[k] = threadIdx.x * 2654435761u + blockIdx.x + k;
    x[k] = (threadIdx.x ^ 0x9e3779b9u) + 3 * k;
  }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int k = 0; k < NCH; k++) acc[k] = (uint64_t)(uint32_t)acc[k] * x[k] + acc[k];
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < NCH; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(uint64_t* out, int iters) {
  uint32_t x[16], y[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    x[k] = threadIdx.x + k;
    y[k] = blockIdx.x * 77 + k * 13;
  }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int k = 0; k < 16; k++) x[k] = (x[k] + y[k]) ^ (uint32_t)r;  // add + xor
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) s ^= x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NIND>
__global__ __launch_bounds__(256) void k_f30(uint64_t* out, int iters) {
  uint32_t a[NIND][9], b[9];
#pragma unroll
  for (int k = 0; k < 9; k++) b[k] = ((blockIdx.x + 7) * (k + 11)) & kM30;
#pragma unroll
  for (int c = 0; c < NIND; c++)
#pragma unroll
    for (int k = 0; k < 9; k++) a[c][k] = ((threadIdx.x + 1 + c) * (k + 3)) & kM30;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int c = 0; c < NIND; c++) f_mul<F30_p256>(a[c], a[c], b);
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < NIND; c++)
#pragma unroll
    for (int k = 0; k < 9; k++) s ^= a[c][k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_clock(uint64_t* out, int iters) {
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t acc = threadIdx.x;
  for (int i = 0; i < iters; i++) acc = (uint64_t)(uint32_t)(acc >> 3) * 2654435761u + acc;
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (acc == 42) out[0] = 0;
}

template <class K>
double time_kernel(K kern, int blocks, int threads, int iters, uint64_t* out) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 2);  // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters);
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
  const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
  const double lanes = (double)blocks * 256;
  uint64_t* out;
  CHK(hipMalloc(&out, (size_t)blocks * 256 * 8));
  const int it = 2000;
  double t16 = time_kernel(k_mad<16>, blocks, 256, it, out);
  double t32 = time_kernel(k_mad<32>, blocks, 256, it, out);
  // latency: 1 chain per lane, one 64-thread block per SIMD (1 wave/SIMD)
  double tl = time_kernel(k_mad<1>, cus * 4, 64, it * 4, out);
  double ta = time_kernel(k_add, blocks, 256, it, out);
  double tf1 = time_kernel(k_f30<1>, blocks, 256, 2000, out);
  double tf2 = time_kernel(k_f30<2>, blocks, 256, 2000, out);
  double tf1_lo = time_kernel(k_f30<1>, cus * 2, 256, 2000, out);  // 2 waves/SIMD
  // in-kernel clock under the mad load
  hipLaunchKernelGGL(k_clock, dim3(blocks), dim3(256), 0, 0, out, 200000);
  CHK(hipDeviceSynchronize());
  uint64_t h[2];
  CHK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
  const double ghz = (double)h[0] / (double)h[1] * 0.1;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz_nominal\": %d, \"clock_ghz_in_kernel\": %.3f, "
         "\"mad_u64_u32_per_s\": %.4e, \"mad_u64_u32_per_s_32ch\": %.4e, "
         "\"mad_dep_cycles_at_nominal\": %.2f, \"xad_u32_per_s\": %.4e, "
         "\"f30_mul_per_s\": %.4e, \"f30_mul_per_s_2ind\": %.4e, \"f30_mul_per_s_2waves\": %.4e}\n",
         prop.gcnArchName, cus, prop.clockRate, ghz, lanes * it * 8 * 16 / t16,
         lanes * it * 8 * 32 / t32, tl * 2.4e9 / (it * 4 * 8.0),
         lanes * it * 8 * 16 / ta, lanes * 2000 / tf1, lanes * 2000 * 2 / tf2,
         (double)cus * 2 * 256 * 2000 / tf1_lo);
  return 0;
}
