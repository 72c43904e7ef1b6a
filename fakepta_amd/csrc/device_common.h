// Device helpers shared by the kernel translation units (kernels.hip, dense.hip).
#pragma once
#include <hip/hip_runtime.h>

// Device-side bounds checks of the debug build (make debug, -DFPTA_DEBUG): a failed check prints the
// kernel, the index and the bound, then traps (the launch reports a device fault). Release builds
// compile them out.
#ifdef FPTA_DEBUG
#include <cstdio>
#define FPTA_DCHECK(cond, what, idx, bound)                                                          \
  do {                                                                                               \
    if (!(cond)) {                                                                                   \
      printf("FPTA_DCHECK %s: index %lld outside [0, %lld) (block %u thread %u)\n", what,           \
             (long long)(idx), (long long)(bound), blockIdx.x, threadIdx.x);                          \
      __builtin_trap();                                                                              \
    }                                                                                                \
  } while (0)
#else
#define FPTA_DCHECK(cond, what, idx, bound) \
  do {                                      \
  } while (0)
#endif

namespace fpta {

typedef double d4 __attribute__((ext_vector_type(4)));

// (freqf / nu)^idx with numpy's scalar-power fast paths (idx 0 -> 1, idx 2 -> square).
__device__ __forceinline__ double chrom_factor(double freqf, double nu, double idx) {
  if (idx == 0.0) return 1.0;
  const double x = freqf / nu;
  if (idx == 2.0) return x * x;
  if (idx == 1.0) return x;
  return pow(x, idx);
}

// Interpolation weight of row i of a TOA's window (exponential-of-semicircle kernel, width 2 hw cells, shape beta):
// ch phi((d - i) / hw), d the TOA's offset from the window's first row. One definition for k_grid_weights (the weight
// tables) and k_grid_interp_u (weights made on the fly), so both give the same doubles.
__device__ __forceinline__ double es_weight(double d, int i, double hw, double beta, double ch) {
  const double z = (d - (double)i) / hw;
  const double s = 1.0 - z * z;
  return s > 0.0 ? ch * exp(beta * (sqrt(s) - 1.0)) : 0.0;
}

}  // namespace fpta
