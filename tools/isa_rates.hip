// Issue-rate micro-benchmark for the VALU instructions the field arithmetic
// uses (gfx950): NCH independent chains of one instruction per lane, 8 waves
// per SIMD, results kept live. Prints lane-operations per cycle per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define NCH 12
#define ITERS 2048

#define KERNEL(NAME, DECL, INIT, BODY, FOLD)                                   \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t s) {    \
    DECL;                                                                     \
    for (int k = 0; k < NCH; k++) { INIT; }                                   \
    for (int i = 0; i < ITERS; i++) {                                         \
      _Pragma("unroll") for (int r = 0; r < 8; r++) {                         \
        _Pragma("unroll") for (int k = 0; k < NCH; k++) { BODY; }             \
      }                                                                       \
    }                                                                         \
    uint64_t acc = 0;                                                         \
    for (int k = 0; k < NCH; k++) { FOLD; }                                   \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                         \
  }

KERNEL(k_add, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(s)), acc ^= x[k])
KERNEL(k_and, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[k]) : "v"(s)), acc ^= x[k])
KERNEL(k_xad, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x[k]) : "v"(s)), acc ^= x[k])
KERNEL(k_shr64, uint64_t x[NCH], x[k] = threadIdx.x + ((uint64_t)k << 40) * s,
       asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(x[k])), acc ^= x[k])
KERNEL(k_ladd64, uint64_t x[NCH], x[k] = threadIdx.x + ((uint64_t)k << 40) * s,
       asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(x[k])), acc ^= x[k])
KERNEL(k_mad64, uint64_t x[NCH], x[k] = threadIdx.x + ((uint64_t)k << 40) * s,
       asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(x[k]) : "v"(s) : "vcc"), acc ^= x[k])
KERNEL(k_mul_lo, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(s)), acc ^= x[k])
KERNEL(k_mul_hi, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[k]) : "v"(s)), acc ^= x[k])
KERNEL(k_mad24, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x[k]) : "v"(s)), acc ^= x[k])
KERNEL(k_fma64, double x[NCH], x[k] = threadIdx.x + k * (double)s,
       asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(x[k]) : "v"((double)s)), acc ^= (uint64_t)x[k])
KERNEL(k_pkfma, uint64_t x[NCH], x[k] = threadIdx.x + ((uint64_t)k << 40) * s,
       asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(x[k])), acc ^= x[k])
KERNEL(k_cnd, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(s) : "vcc"), acc ^= x[k])
KERNEL(k_addco, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[k]) : "v"(s) : "vcc"), acc ^= x[k])
KERNEL(k_bfe, uint32_t x[NCH], x[k] = threadIdx.x + k * s,
       asm volatile("v_bfe_u32 %0, %0, 3, 30" : "+v"(x[k])), acc ^= x[k])

typedef void (*K)(uint64_t*, uint32_t);
int main() {
  int dev = 0, cus = 0, clk = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  const int blocks = cus * 8;  // 8 x 256 threads per CU = 8 waves per SIMD
  uint64_t* out;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  struct { const char* n; K k; } ks[] = {
      {"v_add_u32", k_add}, {"v_and_b32", k_and}, {"v_xad_u32", k_xad},
      {"v_lshrrev_b64", k_shr64}, {"v_lshl_add_u64", k_ladd64}, {"v_mad_u64_u32", k_mad64},
      {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi}, {"v_mad_u32_u24", k_mad24},
      {"v_fma_f64", k_fma64}, {"v_pk_fma_f32", k_pkfma}, {"v_cndmask_b32", k_cnd},
      {"v_add_co_u32", k_addco}, {"v_bfe_u32", k_bfe}};
  printf("{\"cus\": %d, \"clock_khz\": %d", cus, clk);
  for (auto& e : ks) {
    hipLaunchKernelGGL(e.k, dim3(blocks), dim3(256), 0, 0, out, 3u);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(e.k, dim3(blocks), dim3(256), 0, 0, out, 3u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = 3.0 * blocks * 256.0 * ITERS * 8 * NCH;
    const double per_cyc_simd = lane_ops / (ms * 1e-3) / (cus * 4.0 * clk * 1e3);
    printf(", \"%s\": %.2f", e.n, per_cyc_simd);
  }
  printf("}\n");
  return 0;
}
