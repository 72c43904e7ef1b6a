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
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
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

// Stream words for the non-GP draws (kept identical to the oracle).
constexpr uint32_t kWhitePsrWord = 0xFFFFFFFFu;
constexpr uint32_t kWhiteStream = 0xFFFFFFF0u;
constexpr uint32_t kEcorrStream = 0xFFFFFFF1u;
constexpr uint32_t kDenseStream = 0xFFFFFFF2u;  // dense-covariance draws (fpta_noise_draw)

}  // namespace fpta
