// Philox4x32-10 counter-based generator (Salmon et al., SC'11; Random123 constants) and the
// build's fixed uniform -> normal mapping. Host+device. The numpy twin lives in
// oracle/fakepta_oracle.py (philox4x32_10, box_muller) and is pinned by the Random123
// known-answer vectors; tests/test_gpu_parity.py checks this device version bit-for-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpta {

struct u32x4 {
  uint32_t x, y, z, w;
};

__host__ __device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    u32x4 n;
#if defined(__HIP_DEVICE_COMPILE__) && __has_builtin(__builtin_amdgcn_bitop3_b32)
    // gfx950's three-input bitwise op (truth table 0x96 = a ^ b ^ c): one instruction per word instead of two (a
    // target without it, e.g. ARCH=gfx942, takes the two-XOR form below: the same words)
    n.x = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96);
    n.z = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96);
#else
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
#endif
    n.y = (uint32_t)p1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// u1 in (0,1] from (x,y), u2 in [0,1) from (z,w); z0 = r cos(2 pi u2), z1 = r sin(2 pi u2).
__device__ __forceinline__ void box_muller(u32x4 v, double& z0, double& z1) {
  const uint64_t a = (uint64_t)v.x | ((uint64_t)v.y << 32);
  const uint64_t b = (uint64_t)v.z | ((uint64_t)v.w << 32);
  const double u1 = (double)((a >> 11) + 1ull) * 0x1.0p-53;
  const double u2 = (double)(b >> 11) * 0x1.0p-53;
  const double r = sqrt(-2.0 * log(u1));
  // cos/sin(2 pi u2) as sincospi(2 u2): the argument is already reduced, so this skips the general
  // range reduction; equal to the oracle's np.cos(2*pi*u2) to ~1 ulp of the unit-circle value
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// The build's uniform -> normal map (oracle: normals4, bm_log_u32, bm_sincos2pi_u32, operation for operation except
// the division in the logarithm and the square root, which are within an ulp of the oracle's IEEE results): two
// Box-Muller pairs per Philox call from 32-bit uniforms u1 = (a + 1) 2^-32 in (0, 1], u2 = b 2^-32 in [0, 1), with
// the logarithm and sine / cosine as fixed fp64 polynomials (~3e-14 relative): about half the VALU work per normal of
// box_muller (one Philox call per two normals, library log and sincospi).
__device__ __forceinline__ double bm_log_u32(uint32_t a) {
  const double n = (double)a + 1.0;  // exact
  int e;
  double m = frexp(n, &e);  // n = m 2^e, m in [0.5, 1)
  if (m < 0.7071067811865476) {
    m *= 2.0;
    e -= 1;
  }
  const double k = (double)(e - 32);
  // s = (m - 1) / (m + 1) from v_rcp_f64 and two Newton steps (m + 1 in [1.7, 2.5]: no scaling) plus one residual
  // correction: within an ulp of the correctly rounded quotient the oracle takes, in 7 instructions instead of 10
  const double num = m - 1.0, den = m + 1.0;
  double rc = __builtin_amdgcn_rcp(den);
  rc = fma(rc, fma(-den, rc, 1.0), rc);
  rc = fma(rc, fma(-den, rc, 1.0), rc);
  double s = num * rc;
  s = fma(fma(-den, s, num), rc, s);
  const double s2 = s * s;
  const double p =
      s2 * (1.0 / 3.0 +
            s2 * (1.0 / 5.0 + s2 * (1.0 / 7.0 + s2 * (1.0 / 9.0 + s2 * (1.0 / 11.0 + s2 * (1.0 / 13.0 + s2 * (1.0 / 15.0)))))));
  const double lm = 2.0 * s + 2.0 * s * p;
  return k * 6.93147180369123816490e-01 + (k * 1.90821492927058770002e-10 + lm);
}

__device__ __forceinline__ void bm_sincos2pi_u32(uint32_t b, double& sn, double& cs) {
  const double u = (double)b * 0x1.0p-32;  // [0, 1), exact
  const double q = rint(4.0 * u);          // nearest quarter turn 0 .. 4
  const double y = u - 0.25 * q;           // exact, [-1/8, 1/8]
  const double a = y * 6.283185307179586;
  const double x2 = a * a;
  const double sa =
      a + a * x2 *
              (-1.0 / 6.0 +
               x2 * (1.0 / 120.0 +
                     x2 * (-1.0 / 5040.0 + x2 * (1.0 / 362880.0 + x2 * (-1.0 / 39916800.0 + x2 * (1.0 / 6227020800.0))))));
  const double ca =
      1.0 + x2 * (-1.0 / 2.0 +
                  x2 * (1.0 / 24.0 +
                        x2 * (-1.0 / 720.0 +
                              x2 * (1.0 / 40320.0 +
                                    x2 * (-1.0 / 3628800.0 + x2 * (1.0 / 479001600.0 + x2 * (-1.0 / 87178291200.0)))))));
  // quadrant qi: (sn, cs) = (sa, ca), (ca, -sa), (-sa, -ca), (-ca, sa) as a swap and two sign-bit flips (no
  // divergent branches; the same values)
  const int qi = (int)q & 3;
  const bool sw = (qi & 1) != 0;
  const double s0 = sw ? ca : sa;
  const double c0 = sw ? sa : ca;
  sn = __longlong_as_double(__double_as_longlong(s0) ^ ((long long)(qi & 2) << 62));
  cs = __longlong_as_double(__double_as_longlong(c0) ^ ((long long)((qi + 1) & 2) << 62));
}

// sqrt(x) for x = -2 log u1 in [0, 45]: v_rsq_f64, one Goldschmidt step and one residual correction (within an ulp
// of the correctly rounded root; x = 0 exactly when u1 = 1)
__device__ __forceinline__ double bm_sqrt(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-g, h, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  g = fma(fma(-g, g, x), h, g);
  return x > 0.0 ? g : 0.0;
}

// four standard normals of one Philox output: (z0, z1) from (x, y), (z2, z3) from (z, w)
__device__ __forceinline__ void normals4(u32x4 v, double (&z)[4]) {
  double s, c;
  const double r0 = bm_sqrt(-2.0 * bm_log_u32(v.x));
  bm_sincos2pi_u32(v.y, s, c);
  z[0] = r0 * c;
  z[1] = r0 * s;
#ifndef FPTA_NORMALS4_SPLIT
#define FPTA_NORMALS4_SPLIT 1  // variant builds: 0 lets the scheduler interleave the two Box-Muller pairs
#endif
  if (FPTA_NORMALS4_SPLIT) __builtin_amdgcn_sched_barrier(0);  // the two pairs one after the other: half the live temporaries
  const double r1 = bm_sqrt(-2.0 * bm_log_u32(v.z));
  bm_sincos2pi_u32(v.w, s, c);
  z[2] = r1 * c;
  z[3] = r1 * s;
}

// GP coefficient normals (oracle gp_normals): ctr = (mode, pulsar, signal, g >> 1); realization g takes normals
// 2 (g & 1), 2 (g & 1) + 1 as (cos, sin). gp_pair2: both realizations g, g + 1 of an even g from one call.
// (gp_normal2 transforms only the half of the Philox output realization g takes: normals4's operations on those two
// words, so the same values as normals4's z[2 (g & 1)], z[2 (g & 1) + 1] for half the fp64 work)
__device__ __forceinline__ void gp_normal2(uint32_t k, uint32_t p, uint32_t seg, uint64_t g, uint32_t k0, uint32_t k1,
                                           double& zc, double& zs) {
  const u32x4 v = philox4x32_10({k, p, seg, (uint32_t)(g >> 1)}, k0, k1);
  const bool odd = (g & 1) != 0;
  double s, c;
  const double r = bm_sqrt(-2.0 * bm_log_u32(odd ? v.z : v.x));
  bm_sincos2pi_u32(odd ? v.w : v.y, s, c);
  zc = r * c;
  zs = r * s;
}
__device__ __forceinline__ void gp_pair2(uint32_t k, uint32_t p, uint32_t seg, uint64_t g_even, uint32_t k0,
                                         uint32_t k1, double (&z)[4]) {
  normals4(philox4x32_10({k, p, seg, (uint32_t)(g_even >> 1)}, k0, k1), z);
}

// Stream words for the non-GP draws (kept identical to the oracle).
constexpr uint32_t kWhitePsrWord = 0xFFFFFFFFu;
constexpr uint32_t kWhiteStream = 0xFFFFFFF0u;
constexpr uint32_t kEcorrStream = 0xFFFFFFF1u;
constexpr uint32_t kDenseStream = 0xFFFFFFF2u;  // dense-covariance draws (fpta_noise_draw)

}  // namespace fpta

namespace fpta {
// One normal of an indexed stream paired over both index and realization (oracle quad_normals): ctr = (i >> 1,
// 0xFFFFFFFF, stream, g >> 1), normal 2 (i & 1) + (g & 1). quad4: the four normals (i, g), (i, g + 1), (i + 1, g),
// (i + 1, g + 1) of even i and g from one call.
__device__ __forceinline__ double quad_normal(uint64_t i, uint32_t stream, uint64_t g, uint32_t k0, uint32_t k1) {
  double z[4];
  normals4(philox4x32_10({(uint32_t)(i >> 1), kWhitePsrWord, stream, (uint32_t)(g >> 1)}, k0, k1), z);
  // a select, not z[k]: a lane-dependent index into a private array is a scratch (stack) object, and each inlined
  // copy would get its own
  const double lo = (g & 1) ? z[1] : z[0], hi = (g & 1) ? z[3] : z[2];
  return (i & 1) ? hi : lo;
}
__device__ __forceinline__ void quad4(uint64_t i_even, uint32_t stream, uint64_t g_even, uint32_t k0, uint32_t k1,
                                      double (&z)[4]) {
  normals4(philox4x32_10({(uint32_t)(i_even >> 1), kWhitePsrWord, stream, (uint32_t)(g_even >> 1)}, k0, k1), z);
}
}  // namespace fpta
