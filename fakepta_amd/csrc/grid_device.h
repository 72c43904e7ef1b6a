// Device helpers of the gridded-path kernels (grid_mfma.hip, grid_fused.hip): wave-uniform table reads, the
// interpolation tile and its residual store, and the coefficient draw of a grid signal's terms. Header-only (inline /
// templates), so every translation unit that includes it compiles the same instructions.
#pragma once
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "fpta_internal.h"
#include "philox.h"

namespace fpta {

typedef double dbl2 __attribute__((ext_vector_type(2)));

// A wave-uniform read of a table the kernel never writes, through the constant address space: a scalar load
// (lgkmcnt). A plain load of it is a vector load once the kernel has stores the compiler cannot rule out as aliasing,
// and waiting for it (vmcnt) then also waits for every store issued before it.
template <class T>
__device__ __forceinline__ T ld_uniform(const T* p) {
  return *(const __attribute__((address_space(4))) T*)p;
}
// A per-lane read through the global address space: a pointer chosen among several (a select or a branch) is generic,
// and a generic (flat) load counts on both vmcnt and lgkmcnt, so every LDS wait after it would also wait for it.
template <class T>
__device__ __forceinline__ T ld_global(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int4 ld_uniform4(const void* p) {
  const i32x4 v = ld_uniform((const i32x4*)p);
  return make_int4(v.x, v.y, v.z, v.w);
}

// An opaque value: a product stored through it is rounded before any later add (no fma contraction), as k_gen stores
// a coefficient and k_coef_merge adds it.
__device__ __forceinline__ double opaque(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

// The (cos, sin) coefficients of mode m of one grid signal for the batch realizations r, r + 1 (r even), summed over the
// signal's terms in its summation order (the anchor first, then the other members in layout order): a generated term
// (kind 0, a per-pulsar member) is amp * z from k_gen's Philox counter {mode, pulsar, signal, realization} (the same
// draws), its product rounded before the sum; a loaded term (kind 1) is the member's column pair of the coefficient
// buffer. T: any struct with DftGenArgs' term fields (n_terms, term_kind, term_seg, term_nm, term_col0, term_amp).
// Modes past nm and padding realizations (r >= n_real) give 0 for generated terms, as k_gen writes them.
template <class T>
__device__ __forceinline__ void grid_term_coefs(const T& d, int nm, const double* __restrict__ coef, int32_t K,
                                                int32_t R_pad, int32_t n_real, int64_t real0, uint32_t k0, uint32_t k1,
                                                int p, int m, int r, double (&bc)[2], double (&bs)[2]) {
  bc[0] = bc[1] = bs[0] = bs[1] = 0.0;
  if (m >= nm) return;
  bool first = true;
  for (int i = 0; i < d.n_terms; ++i) {
    if (m >= d.term_nm[i]) continue;
    double pc[2], ps[2];
    if (d.term_kind[i] == 0) {
      double z[4] = {0.0, 0.0, 0.0, 0.0};
      const uint64_t g = (uint64_t)(real0 + r);
      if (r < n_real) {  // padding realizations: zero, as k_gen writes them
        if ((g & 1) == 0) {
          gp_pair2((uint32_t)m, (uint32_t)p, (uint32_t)d.term_seg[i], g, k0, k1, z);
        } else {
          gp_normal2((uint32_t)m, (uint32_t)p, (uint32_t)d.term_seg[i], g, k0, k1, z[0], z[1]);
          gp_normal2((uint32_t)m, (uint32_t)p, (uint32_t)d.term_seg[i], g + 1, k0, k1, z[2], z[3]);
        }
        if (r + 1 >= n_real) z[2] = z[3] = 0.0;
      }
      const double a = d.term_amp[i][(int64_t)p * d.term_nm[i] + m];
      pc[0] = opaque(a * z[0]);
      ps[0] = opaque(a * z[1]);
      pc[1] = opaque(a * z[2]);
      ps[1] = opaque(a * z[3]);
    } else {
      const double* cp = coef + ((int64_t)p * K + d.term_col0[i] + 2 * m) * R_pad + r;
      const dbl2 vc = *(const dbl2*)cp, vs = *(const dbl2*)(cp + R_pad);
      pc[0] = vc.x;
      pc[1] = vc.y;
      ps[0] = vs.x;
      ps[1] = vs.y;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bc[h] = first ? pc[h] : bc[h] + pc[h];
      bs[h] = first ? ps[h] : bs[h] + ps[h];
    }
    first = false;
  }
}

// One interpolation tile: a chunk of <= kGridTT TOAs x 16 RW realizations (wave-uniform fields).
template <int RW>
struct InterpTile {
  int c, p, r0, nq, cnt, y;
  // partial-checksum row of the tile's chunk group and the chunk's place in it (first: start the row's sums, last:
  // store them); the diagnostic kernels take one chunk per row
  int pg = -1, pfirst = 1, plast = 1;
  int rr[kGridVMax / 64];
  const double* G0;
  const double* Wp;
};

// The tile's sums acc[e][i] (TOA parity e, realization tile i; lane (lr, lg) register g = TOA 2 lr + e of realization
// r0 + 32 (i >> 1) + 2 (lg + 4 g) + (i & 1)) stored into the residual block.
// PACE > 0 (k_grid_interp_st's storer waves): s_sleep PACE (x 64 cycles) after each 1 KB store of the fast path, so a
// CU's stores enter the memory pipeline at about the rate the write path drains them. A store that waits at the head
// of the CU's vector-memory queue holds every load behind it, including the compute waves' operand loads.
template <int RW, int PACE = 0>
__device__ __forceinline__ void interp_store_rows(const SynthArgs& a, double* __restrict__ out,
                                                  const InterpTile<RW>& t, const d4 (&acc)[2][RW]) {
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int tt = 2 * lr;  // this lane's even TOA in the chunk; tt + 1 the odd one
  if (tt >= t.cnt) return;
  const int64_t tg = ld_uniform(a.offs + t.p) + t.y + tt;
  // fast path (full chunk, every realization of the tile stored, no accumulate, 16-byte aligned rows): straight-line
  // 16-byte stores from a wave-uniform row base plus one 32-bit lane offset, no per-store tests. The general path
  // below spends ~28 instructions and several branches per store, which held the SIMD's issue while the partner
  // wave's MFMAs needed it.
  {
    const int64_t t0 = tg - tt;  // wave-uniform first sample of the chunk
    const bool fast = t.cnt == kGridTT && !a.accumulate && t.r0 + 16 * RW <= a.n_real &&
                      ((((uintptr_t)(out + t0)) | ((uintptr_t)a.ldo << 3)) & 15) == 0 &&
                      a.ldo < ((int64_t)1 << 26);  // lane offsets (< 6 ldo + 32 doubles) fit 32 bits
    if (__builtin_amdgcn_readfirstlane(fast ? 1 : 0)) {
      const uint32_t vo = (uint32_t)(((int64_t)2 * lg * a.ldo + tt) * 8);
      const char* base = (const char*)(out + t0 + (int64_t)t.r0 * a.ldo);
#pragma unroll
      for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int k = 32 * (i >> 1) + 8 * g + (i & 1);  // row of (tile i, register g) past r0 + 2 lg
          // non-temporal: the block is never re-read by this kernel, and L2-allocating 1.6 GB of stores would evict
          // the grid rows the next chunks re-read (they then queue behind the write stream: tools/mfma_store_probe)
          __builtin_nontemporal_store(dbl2{acc[0][i][g], acc[1][i][g]},
                                      (dbl2*)((char*)base + (int64_t)k * a.ldo * 8 + vo));
          if constexpr (PACE > 0) __builtin_amdgcn_s_sleep(PACE);
        }
      return;
    }
  }
  // one 16-byte store per (lane, realization) when both TOAs exist and the row offset r * ldo + tg keeps 16-byte
  // alignment (ldo and tg even), else the pair is stored as two 8-byte stores
  double* __restrict__ ocol = out + tg;
  const bool pair = tt + 1 < t.cnt;
  const bool vec = pair && ((((uintptr_t)ocol) | ((uintptr_t)a.ldo << 3)) & 15) == 0;
#pragma unroll
  for (int i = 0; i < RW; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int r = t.r0 + 32 * (i >> 1) + 2 * (lg + 4 * g) + (i & 1);
      if (r < a.n_real) {
        double* o = ocol + (int64_t)r * a.ldo;
        double v0 = acc[0][i][g], v1 = acc[1][i][g];
        if (a.accumulate) {
          v0 += o[0];
          if (pair) v1 += o[1];
        }
        if (vec) {
          *(dbl2*)o = dbl2{v0, v1};
        } else {
          o[0] = v0;
          if (pair) o[1] = v1;
        }
      }
    }
  }
}

}  // namespace fpta
