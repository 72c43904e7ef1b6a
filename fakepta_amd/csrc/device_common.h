// Device helpers shared by the kernel translation units (kernels.hip, dense.hip).
#pragma once
#include <hip/hip_runtime.h>

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

}  // namespace fpta
