// Calibration probe (not part of the product): fp64 MFMA vs fp64 VALU throughput on gfx950,
// and whether the two co-issue. Build: hipcc --offload-arch=gfx950 -O3 tools/fp64_probe.hip -o /tmp/fp64_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC, int NVALU>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double seed, unsigned long long* clk) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), t0 = __builtin_amdgcn_s_memrealtime();
  d4 acc[NACC > 0 ? NACC : 1];
  for (int i = 0; i < (NACC > 0 ? NACC : 1); ++i) acc[i] = d4{0, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-3, b = seed * 0.5 + threadIdx.x * 2e-3;
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = seed + i * 0.01 + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
    for (int k = 0; k < NVALU; ++k) v[k & 7] = fma(v[k & 7], 0.999999, 1e-9);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {  // shader cycles and 100 MHz ticks of this workgroup: the clock it ran at
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - t0;
  }
}

template <int NACC, int NVALU>
void run(const char* name, double* d, unsigned long long* clk, int blocks, int iters = 2000) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<NACC, NVALU>), dim3(blocks), dim3(256), 0, 0, d, 10, 1.0, clk);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL((probe<NACC, NVALU>), dim3(blocks), dim3(256), 0, 0, d, iters, 1.0, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[2 * 8192];
  hipMemcpy(h, clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost);
  double cyc = 0, ticks = 0;
  for (int b = 0; b < blocks; ++b) {
    cyc += (double)h[2 * b];
    ticks += (double)h[2 * b + 1];
  }
  const double ghz = cyc / (ticks * 10.0);  // s_memrealtime: 100 MHz
  const double waves = blocks * 4.0;
  const double mfma_flop = waves * 5 * iters * NACC * 2048.0;
  const double valu_flop = waves * 5 * iters * NVALU * 128.0;
  printf("%-28s blocks=%5d iters=%6d %9.3f ms  MFMA %7.2f TF  VALU %7.2f TF  total %7.2f TF  clock %.2f GHz (last launch)\n",
         name, blocks, iters, ms, mfma_flop / ms / 1e9, valu_flop / ms / 1e9, (mfma_flop + valu_flop) / ms / 1e9, ghz);
}

int main() {
  double* d;
  unsigned long long* clk;
  hipMalloc(&d, sizeof(double) * 256 * 8192);
  hipMalloc(&clk, sizeof(unsigned long long) * 2 * 8192);
  for (int blocks : {1024, 2048, 4096}) {
    run<8, 0>("mfma x8", d, clk, blocks);
    run<4, 0>("mfma x4", d, clk, blocks);
    run<0, 32>("valu fma x32", d, clk, blocks);
    run<8, 8>("mfma x8 + valu x8", d, clk, blocks);
    run<8, 16>("mfma x8 + valu x16", d, clk, blocks);
    run<8, 32>("mfma x8 + valu x32", d, clk, blocks);
    run<8, 64>("mfma x8 + valu x64", d, clk, blocks);
  }
  // sustained (~0.1-0.3 s per line): the clock the power limit leaves under each mix
  run<8, 0>("mfma x8 (sustained)", d, clk, 1024, 40000);
  run<0, 32>("valu fma x32 (sustained)", d, clk, 1024, 40000);
  run<8, 16>("mfma x8 + valu x16 (sust.)", d, clk, 1024, 40000);
  hipFree(clk);
  hipFree(d);
  return 0;
}
