// Calibration probe (not part of the product): throughput of the fp64 FMA forms the gridded interpolation
// can use on gfx950: plain v_fmac_f64 (VGPR x VGPR), v_fmac_f64 with an SGPR operand, and v_fmac_f64_dpp
// row_newbcast (the broadcast weight of k_grid_interp_sparse), with 8 or 2 independent accumulators.
// Build: hipcc --offload-arch=gfx950 -O3 tools/fp64_dpp_probe.hip -o /tmp/fp64_dpp_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define DPP(acc, g, i) "v_fmac_f64_dpp " acc ", %[w], " g " row_newbcast:" #i " row_mask:0xf bank_mask:0xf\n\t"

template <int MODE, int NACC>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double seed) {
  double acc[8], g[8];
  for (int i = 0; i < 8; ++i) {
    acc[i] = 0.0;
    g[i] = seed + i * 0.01 + threadIdx.x * 1e-3;
  }
  double w = seed * 0.5 + (threadIdx.x & 15) * 1e-3;
  const double ws = __builtin_amdgcn_readfirstlane((int)(seed * 3)) * 1e-3;  // wave-uniform (SGPR)
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep) {
      if constexpr (MODE == 0) {  // plain VGPR x VGPR
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k % NACC] = fma(w, g[k], acc[k % NACC]);
      } else if constexpr (MODE == 1) {  // SGPR operand
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k % NACC] = fma(ws, g[k], acc[k % NACC]);
      } else if constexpr (NACC == 8) {  // DPP broadcast, 8 independent accumulators
        asm(DPP("%[a0]", "%[g0]", 0) DPP("%[a1]", "%[g1]", 1) DPP("%[a2]", "%[g2]", 2) DPP("%[a3]", "%[g3]", 3)
                DPP("%[a4]", "%[g4]", 4) DPP("%[a5]", "%[g5]", 5) DPP("%[a6]", "%[g6]", 6) DPP("%[a7]", "%[g7]", 7)
            : [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]),
              [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7])
            : [w] "v"(w), [g0] "v"(g[0]), [g1] "v"(g[1]), [g2] "v"(g[2]), [g3] "v"(g[3]), [g4] "v"(g[4]),
              [g5] "v"(g[5]), [g6] "v"(g[6]), [g7] "v"(g[7]));
      } else {  // DPP broadcast, 2 accumulators (the kernel's even/odd chains)
        asm(DPP("%[a0]", "%[g0]", 0) DPP("%[a1]", "%[g1]", 1) DPP("%[a0]", "%[g2]", 2) DPP("%[a1]", "%[g3]", 3)
                DPP("%[a0]", "%[g4]", 4) DPP("%[a1]", "%[g5]", 5) DPP("%[a0]", "%[g6]", 6) DPP("%[a1]", "%[g7]", 7)
            : [a0] "+v"(acc[0]), [a1] "+v"(acc[1])
            : [w] "v"(w), [g0] "v"(g[0]), [g1] "v"(g[1]), [g2] "v"(g[2]), [g3] "v"(g[3]), [g4] "v"(g[4]),
              [g5] "v"(g[5]), [g6] "v"(g[6]), [g7] "v"(g[7]));
      }
    }
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int NACC>
void run(const char* name, double* d, int blocks) {
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<MODE, NACC>), dim3(blocks), dim3(256), 0, 0, d, 10, 1.0);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((probe<MODE, NACC>), dim3(blocks), dim3(256), 0, 0, d, iters, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = blocks * 256.0 * 5 * iters * 32 * 2.0;
  printf("%-34s blocks=%5d  %8.3f ms  %7.2f TF\n", name, blocks, ms, flop / ms / 1e9);
}

int main() {
  double* d;
  hipMalloc(&d, sizeof(double) * 256 * 8192);
  for (int blocks : {1024, 4096}) {
    run<0, 8>("v_fmac_f64 vgpr, 8 acc", d, blocks);
    run<0, 2>("v_fmac_f64 vgpr, 2 acc", d, blocks);
    run<1, 8>("v_fmac_f64 sgpr, 8 acc", d, blocks);
    run<2, 8>("v_fmac_f64_dpp newbcast, 8 acc", d, blocks);
    run<2, 2>("v_fmac_f64_dpp newbcast, 2 acc", d, blocks);
  }
  hipFree(d);
  return 0;
}
