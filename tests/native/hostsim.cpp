// TEST-ONLY host harness: runs the exact per-record stage functions of
// bdls_amd/csrc/verify.h (the code the HIP kernels execute) sequentially on the
// CPU, so the arithmetic can be checked against the oracle in a container with
// no GPU. Never linked into libbdlship.so; the product path has no CPU fallback.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../bdls_amd/csrc/verify.h"

using namespace bh;

static std::vector<uint32_t> g_gtab;

template <class F, class C>
static void build_gtab() {
  g_gtab.assign((size_t)kCombWindows * kCombEntries * 16, 0);
  for (uint32_t t = 0; t < (uint32_t)(kCombWindows * kCombEntries); t++) {
    const uint32_t win = t / kCombEntries, j = t % kCombEntries;
    Jac B;
    load_const8(B.X, C::gx_m);
    load_const8(B.Y, C::gy_m);
    load_const8(B.Z, F::r1);
    for (uint32_t d = 0; d < 8 * win; d++) pt_dbl<F, C>(B, B);
    const uint32_t k = j + 1;
    int top = 31 - __builtin_clz(k);
    Jac A;
    jac_copy(A, B);
    for (int b = top - 1; b >= 0; b--) {
      pt_dbl<F, C>(A, A);
      if ((k >> b) & 1u) {
        bool same;
        Jac R;
        pt_add<F>(R, A, B, &same);
        jac_copy(A, R);
      }
    }
    uint32_t zi[8], zi2[8], x[8], y[8];
    mont_inv<F>(zi, A.Z);
    mont_sqr<F>(zi2, zi);
    mont_mul<F>(x, A.X, zi2);
    mont_mul<F>(zi2, zi2, zi);
    mont_mul<F>(y, A.Y, zi2);
    for (int q = 0; q < 8; q++) {
      g_gtab[(size_t)t * 16 + q] = x[q];
      g_gtab[(size_t)t * 16 + 8 + q] = y[q];
    }
  }
}

extern "C" int hs_verify_dump(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                              const uint32_t* slen, const uint8_t* msg, const uint64_t* moff,
                              const uint32_t* mlen, uint32_t n, uint32_t flags, uint32_t chunk,
                              uint8_t* reason, uint32_t* dump);
extern "C" int hs_verify(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                         const uint32_t* slen, const uint8_t* msg, const uint64_t* moff,
                         const uint32_t* mlen, uint32_t n, uint32_t flags, uint32_t chunk,
                         uint8_t* reason) {
  return hs_verify_dump(pub, sig, soff, slen, msg, moff, mlen, n, flags, chunk, reason, nullptr);
}
extern "C" int hs_verify_dump(const uint8_t* pub, const uint8_t* sig, const uint64_t* soff,
                              const uint32_t* slen, const uint8_t* msg, const uint64_t* moff,
                              const uint32_t* mlen, uint32_t n, uint32_t flags, uint32_t chunk,
                              uint8_t* reason, uint32_t* dump) {
  if (g_gtab.empty()) build_gtab<Fp_p256, Cv_p256>();
  const uint32_t ns = (n + 63) & ~63u;
  std::vector<uint32_t> buf((size_t)9 * 8 * ns + (size_t)(ns / 64) * kQTab * 24 * 64);
  std::vector<uint8_t> st(ns);
  Work w;
  w.ns = ns;
  uint32_t* p = buf.data();
  w.e = p; p += 8 * ns;
  w.r = p; p += 8 * ns;
  w.sm = p; p += 8 * ns;
  w.pre = p; p += 8 * ns;
  w.qx = p; p += 8 * ns;
  w.qy = p; p += 8 * ns;
  w.rm = p; p += 8 * ns;
  w.r2m = p; p += 8 * ns;
  p += 8 * ns;
  w.qtab = p;
  w.st = st.data();
  BatchIn in{pub, sig, soff, slen, msg, moff, mlen, flags};
  uint32_t* arrs[6] = {w.e, w.r, w.sm, w.qx, w.qy, w.rm};
  auto snap = [&](int stage) {
    if (!dump) return;
    for (int a = 0; a < 6; a++)
      std::memcpy(dump + ((size_t)stage * 6 + a) * 8 * ns, arrs[a], 8 * (size_t)ns * 4);
    std::memcpy((uint8_t*)(dump + 3 * 6 * 8 * (size_t)ns) + stage * ns, w.st, ns);
  };
  for (uint32_t i = 0; i < n; i++) stage_prep<Fp_p256, Fn_p256, Cv_p256>(in, w, i);
  snap(0);
  for (uint32_t lo = 0; lo < n; lo += chunk)
    stage_inv<Fn_p256>(w, lo, lo + chunk < n ? lo + chunk : n);
  snap(1);
  for (uint32_t i = 0; i < n; i++) {
    const bool pre_ok = (w.st[i] & 0x7f) == R_OK;
    bool ok = stage_ladder<Fp_p256, Fn_p256, Cv_p256>(w, g_gtab.data(), i, i / 64, i % 64);
    reason[i] = pre_ok ? (ok ? R_OK : R_MATH) : (uint8_t)(w.st[i] & 0x7f);
  }
  snap(2);
  return 0;
}
