// Single-wave dependent-chain latency (gfx950): one wave alone on the device
// runs a chain in which every instruction needs the previous result, and
// reads the shader clock before and after. Prints cycles per chained
// operation -- what bounds a lone lane's serial work (a table build's
// doubling chain, a registration, a small batch's ladder), against the
// issue-rate numbers of tools/isa_rates.hip (many waves, independent chains).
//   hipcc --offload-arch=gfx950 -O3 -I bdls_amd/csrc tools/lat_chain.hip -o tools/lat_chain
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "verify.h"

using namespace bh;

#define N 4096

__global__ void k_mad64(uint64_t* out, uint32_t s, uint64_t* cyc) {
  uint64_t x = threadIdx.x + 1;
  const uint64_t t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; i++)
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(x) : "v"(s) : "vcc");
  const uint64_t t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_add32(uint64_t* out, uint32_t s, uint64_t* cyc) {
  uint32_t x = threadIdx.x + 1;
  const uint64_t t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; i++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(s));
  const uint64_t t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_add64(uint64_t* out, uint32_t s, uint64_t* cyc) {
  uint64_t x = threadIdx.x + 1;
  const uint64_t t0 = clock64();
#pragma unroll 16
  for (int i = 0; i < N; i++) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(x));
  const uint64_t t1 = clock64();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// F_p products: CH independent chains of N / 16 dependent f_mul each
template <int CH>
__global__ void k_fmul(uint64_t* out, uint32_t s, uint64_t* cyc) {
  uint32_t a[CH][9];
  for (int c = 0; c < CH; c++)
    for (int k = 0; k < 9; k++) a[c][k] = (threadIdx.x * 7 + k * s + c) & kM30;
  const uint64_t t0 = clock64();
  for (int i = 0; i < N / 16; i++) {
#pragma unroll
    for (int c = 0; c < CH; c++) f_mul<F30_p256>(a[c], a[c], a[c]);
  }
  const uint64_t t1 = clock64();
  uint64_t acc = 0;
  for (int c = 0; c < CH; c++)
    for (int k = 0; k < 9; k++) acc ^= a[c][k];
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// Jacobian doublings (P-256, a = -3): one chain of N / 16
__global__ void k_dbl(uint64_t* out, uint32_t s, uint64_t* cyc) {
  J30 B;
  for (int k = 0; k < 9; k++) {
    B.X[k] = (threadIdx.x * 5 + k * s) & kM30;
    B.Y[k] = (threadIdx.x * 3 + k * s + 1) & kM30;
    B.Z[k] = (k == 0) ? 1u : 0u;
  }
  const uint64_t t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < N / 16; i++) j_dbl<F30_p256>(B, B);
  const uint64_t t1 = clock64();
  uint64_t acc = 0;
  for (int k = 0; k < 9; k++) acc ^= B.X[k] ^ B.Y[k] ^ B.Z[k];
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// field inversions by safegcd (verify.h f_inv_sg): a chain of N / 256
__global__ void k_finv(uint64_t* out, uint32_t s, uint64_t* cyc) {
  uint32_t a[9];
  for (int k = 0; k < 9; k++) a[k] = (threadIdx.x * 11 + k * s + 1) & kM30;
  const uint64_t t0 = clock64();
#pragma unroll 1
  for (int i = 0; i < N / 256; i++) {
    uint32_t r[9];
    f_inv_sg<F30_p256>(r, a);
    a[0] = r[0] + 1u;
    for (int k = 1; k < 9; k++) a[k] = r[k];
  }
  const uint64_t t1 = clock64();
  uint64_t acc = 0;
  for (int k = 0; k < 9; k++) acc ^= a[k];
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// a Lim-Lee comb table build (verify.h lltab_build) on one lane: scratch in
// the slot (global memory) or in LDS
__device__ uint32_t g_tab[kKTabWords];
__device__ uint32_t g_q[2 * 9 * 64];
template <bool LDS>
__global__ void k_comb(uint64_t* out, uint32_t s, uint64_t* cyc) {
  __shared__ __attribute__((aligned(16))) uint32_t s_comb[kLLPre + 12u * kLLEnt];
  Work w{};
  w.ns = 64;
  w.qx = g_q;
  w.qy = g_q + 9 * 64;
  if (threadIdx.x == 0) {  // Q = G (Montgomery form): a valid key
    for (int k = 0; k < 9; k++) {
      g_q[k * 64] = F30_p256::gx_m[k];
      g_q[9 * 64 + k * 64] = F30_p256::gy_m[k];
    }
  }
  __syncthreads();
  uint32_t rec = 0;
  asm volatile("" : "+v"(rec));  // a per-lane record index: VALU code, as in k_ktab_ladder
  const uint64_t t0 = clock64();
  if (threadIdx.x == 0) lltab_build<F30_p256>(g_tab, w, rec, LDS ? s_comb : nullptr);
  const uint64_t t1 = clock64();
  out[threadIdx.x] = g_tab[threadIdx.x];
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// lltab_build's first phase alone (the 222-doubling chain with its raw
// stores and Z products), LDS scratch
__global__ void k_comb_chain(uint64_t* out, uint32_t s, uint64_t* cyc) {
  __shared__ __attribute__((aligned(16))) uint32_t scr[kLLPre + 12u * kLLEnt];
  if (threadIdx.x != 0) return;
  J30 B;
  for (int k = 0; k < 9; k++) {
    B.X[k] = F30_p256::gx_m[k];
    B.Y[k] = F30_p256::gy_m[k];
    B.Z[k] = F30_p256::r1[k];
    // per-lane values: without this the uniform chain is compiled to SALU code
    asm volatile("" : "+v"(B.X[k]), "+v"(B.Y[k]), "+v"(B.Z[k]));
  }
  uint32_t z[9];
  const uint64_t t0 = clock64();
#pragma unroll 1
  for (uint32_t i = 0; i + 1 < (uint32_t)kLLTeeth; i++) {
    j_dbl<F30_p256>(B, B);
    llraw_store(scr, 2u * i, B);
    if (i == 0) f_copy(z, B.Z);
    else f_mul<F30_p256>(z, z, B.Z);
    llpre_store(scr, 2u * i, z);
#pragma unroll 1
    for (int d = 1; d < kLLSpace; d++) j_dbl<F30_p256>(B, B);
    llraw_store(scr, 2u * i + 1u, B);
    f_mul<F30_p256>(z, z, B.Z);
    llpre_store(scr, 2u * i + 1u, z);
  }
  const uint64_t t1 = clock64();
  out[0] = z[0] ^ B.X[0];
  cyc[0] = t1 - t0;
}

typedef void (*K)(uint64_t*, uint32_t, uint64_t*);

int main() {
  uint64_t *out, *cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  struct {
    const char* name;
    K k;
    double ops;
  } ks[] = {{"v_mad_u64_u32", k_mad64, N},     {"v_add_u32", k_add32, N},
            {"v_lshl_add_u64", k_add64, N},    {"f_mul x1 chain", k_fmul<1>, N / 16},
            {"f_mul x2 chains", k_fmul<2>, 2 * (N / 16)}, {"f_mul x4 chains", k_fmul<4>, 4 * (N / 16)},
            {"j_dbl chain", k_dbl, N / 16}, {"f_inv_sg chain", k_finv, N / 256},
            {"lltab_build, global scratch (per table)", k_comb<false>, 1},
            {"lltab_build, LDS scratch (per table)", k_comb<true>, 1},
            {"lltab_build phase 1 (222 doublings), LDS", k_comb_chain, 1}};
  const int nk = (int)(sizeof(ks) / sizeof(ks[0]));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("{\n");
  for (int r = 0; r < nk; r++) {
    uint64_t best = ~0ull;
    float best_ms = 1e9f;
    for (int rep = 0; rep < 5; rep++) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(ks[r].k, dim3(1), dim3(64), 0, 0, out, 3u, cyc);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      uint64_t c = 0;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      if (c < best) best = c;
      if (ms < best_ms) best_ms = ms;
    }
    printf(" \"%s\": {\"cycles_per_op\": %.2f, \"ns_per_op\": %.1f}%s\n", ks[r].name,
           (double)best / ks[r].ops, 1e6 * best_ms / ks[r].ops, r + 1 < nk ? "," : "");
  }
  printf("}\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
