// Gridded (factored) synthesis for harmonic grids: the same sums as k_synth_valu_seeded,
//   r(t) = ch(t) sum_{k=1..N} c_k cos(k theta) + s_k sin(k theta),  theta = w0 t,
// evaluated as a type-2 non-uniform FFT factorisation F ~= W E:
//
//   k_grid_weights  once per layout: dense banded interpolation weights W (chromatic factor and
//                   mask folded in) for every chunk of <= kGridTT (32) consecutive TOAs of one pulsar
//   k_grid_dft      per batch: grid values g_j = sum_k q_k (c_k cos(k x_j) + s_k sin(k x_j)),
//                   x_j = 2 pi j / nf, for every (pulsar, realization) - a real DFT done as a GEMM
//                   against the shared table E (both halves of the grid from one pass: the cos and
//                   sin partial sums give g_j and g_{nf-j})
//   interpolation   per batch: r(t) = sum_i W[t][i] g[J_t + i] for all signals, white noise / ECORR in
//                   the epilogue, one store per sample: k_grid_interp_mfma (grid_mfma.hip, dense 4-row band
//                   steps on the fp64 matrix cores)
//
// Kernel: exponential of semicircle phi(z) = exp(beta (sqrt(1 - z^2) - 1)), |z| <= 1, width w grid
// cells, oversampling nf >= sigma (2N + 1); q_k = (2 pi / nf) / phi_hat(k) deconvolves it.
// A-priori relative aliasing bound exp(-pi w sqrt(1 - 1/sigma)): 1.5e-12 at the default w = 15, sigma = 1.5
// (measured flat-spectrum worst case ~4x the bound; tests/test_gpu_grid.py, tools/sweep_grid.py).
// Per sample the interpolation costs sum_s rows_s FMAs (rows ~ w + cells spanned by the chunk)
// instead of sum_s 2 N_s for the direct contraction.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "fpta_internal.h"
#include "philox.h"

namespace fpta {

typedef double dbl2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------------------- k_grid_weights
// One thread per TOA of the segment: W[chunk][row + i][tt] = ch(t) phi((d - i) / (w / 2)), i < w; row = the
// signal's band offset in the chunk + the TOA's first row in that band (host plan), pitch vmax rows per chunk.
// dch (optional, k_grid_interp_u's on-the-fly weights): {d, ch} of the TOA for signal s_idx of n_sig at
// [(chunk * n_sig + s_idx) * kGridTT + tt].
// half (k_grid_fused's half-chunk bands): chunk_of is a half-chunk (2 chunk + h) of <= 16 TOAs, tt < 16, and its
// vmax x 16 weights are laid out by pairs of band steps, fused_half_weight_index: lane (tt, j) reads steps 2 qp and
// 2 qp + 1 of its band rows 4 q + j with one 16-byte load.
__global__ __launch_bounds__(256) void k_grid_weights(SegDesc sd, int64_t n_toa, const double* __restrict__ nu,
                                                      const int32_t* __restrict__ chunk_of,
                                                      const int32_t* __restrict__ tt_of,
                                                      const int32_t* __restrict__ row_of,
                                                      const double* __restrict__ d_of, int32_t w, double beta,
                                                      int32_t vmax, double* __restrict__ wd, dbl2* __restrict__ dch,
                                                      int32_t s_idx, int32_t n_sig, int32_t half) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_toa) return;
  double ch = chrom_factor(sd.freqf, nu[t], sd.idx);
  if (sd.mask && !sd.mask[t]) ch = 0.0;
  const double d = d_of[t];
  const double hw = 0.5 * (double)w;
  if (half) {
    double* dst = wd + (int64_t)chunk_of[t] * vmax * kFusedHalfTT;
    for (int i = 0; i < w; ++i) dst[fused_half_weight_index(row_of[t] + i, tt_of[t])] = es_weight(d, i, hw, beta, ch);
    return;
  }
  double* dst = wd + ((int64_t)chunk_of[t] * vmax + row_of[t]) * kGridTT + tt_of[t];
  for (int i = 0; i < w; ++i) dst[(int64_t)i * kGridTT] = es_weight(d, i, hw, beta, ch);
  if (dch) dch[((int64_t)chunk_of[t] * n_sig + s_idx) * kGridTT + tt_of[t]] = dbl2{d, ch};
}

// ----------------------------------------------------------------------------- k_grid_dft
// grid (ceil((half + 1) / (4 MI)), P, R_pad / 128), 4 waves. A wave owns MI grid rows j0.. of the
// half range [0, nf/2] and 128 realizations (lane: the adjacent pair r, r + 1). Table values are
// wave-uniform (scalar loads into v_fma_f64 SGPR operands), coefficients are one 16-byte load per
// lane per column. g_j = C_j + S_j and g_{nf-j} = C_j - S_j (cos even, sin odd in j).
template <int MI>
__global__ __launch_bounds__(256) void k_grid_dft(GridSegs gsegs, const double* __restrict__ coef, int32_t K,
                                                  int32_t R_pad) {
  // blockIdx.z enumerates the row tiles of every signal in turn (one launch for all signals). The 4 waves
  // of a workgroup share the row tile (same table slice: scalar-cache hits) and take 4 consecutive
  // 128-realization blocks; blockIdx.x (fastest) walks realization groups, so concurrently resident
  // workgroups mostly share the row tile too.
  int bz = blockIdx.z, s = 0;
  while (s + 1 < gsegs.n && bz >= gsegs.s[s].nblk) bz -= gsegs.s[s++].nblk;
  const GridSegDev& gs = gsegs.s[s];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int j0 = bz * MI;
  const int rblk = blockIdx.x * 4 + wave;
  if (rblk * 128 >= R_pad) return;
  const int p = blockIdx.y;
  const int r = rblk * 128 + 2 * lane;
  const double* __restrict__ cp = coef + ((int64_t)p * K + gs.col0) * R_pad + r;
  dbl2 C[MI], S[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    C[i] = (dbl2){0.0, 0.0};
    S[i] = (dbl2){0.0, 0.0};
  }
  const double* __restrict__ ec = gs.ecos + j0;
  const double* __restrict__ es = gs.esin + j0;
  // nm is even (host padding): modes in pairs, two register sets alternate so every coefficient
  // load is issued one mode ahead of its FMAs (the last prefetches re-read modes 0 and 1)
  dbl2 bc0 = *(const dbl2*)cp, bs0 = *(const dbl2*)(cp + R_pad);
  dbl2 bc1 = *(const dbl2*)(cp + 2 * (int64_t)R_pad), bs1 = *(const dbl2*)(cp + 3 * (int64_t)R_pad);
  for (int m = 0; m < gs.nm; m += 2) {
    const int mn = m + 2 < gs.nm ? m + 2 : 0;
    const double* __restrict__ cn = cp + (int64_t)(2 * mn) * R_pad;
    const dbl2 bc0n = *(const dbl2*)cn, bs0n = *(const dbl2*)(cn + R_pad);
    const double* __restrict__ ecm = ec + (int64_t)m * gs.lde;
    const double* __restrict__ esm = es + (int64_t)m * gs.lde;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      C[i].x = fma(ecm[i], bc0.x, C[i].x);
      C[i].y = fma(ecm[i], bc0.y, C[i].y);
      S[i].x = fma(esm[i], bs0.x, S[i].x);
      S[i].y = fma(esm[i], bs0.y, S[i].y);
    }
    const dbl2 bc1n = *(const dbl2*)(cn + 2 * (int64_t)R_pad), bs1n = *(const dbl2*)(cn + 3 * (int64_t)R_pad);
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      C[i].x = fma(ecm[gs.lde + i], bc1.x, C[i].x);
      C[i].y = fma(ecm[gs.lde + i], bc1.y, C[i].y);
      S[i].x = fma(esm[gs.lde + i], bs1.x, S[i].x);
      S[i].y = fma(esm[gs.lde + i], bs1.y, S[i].y);
    }
    bc0 = bc0n;
    bs0 = bs0n;
    bc1 = bc1n;
    bs1 = bs1n;
  }
  double* __restrict__ gp = gs.g + (int64_t)p * gs.nf * R_pad + r;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int j = j0 + i;
    if (j <= gs.half) *(dbl2*)(gp + (int64_t)j * R_pad) = C[i] + S[i];
    if (j > 0 && 2 * j < gs.nf) *(dbl2*)(gp + (int64_t)(gs.nf - j) * R_pad) = C[i] - S[i];
  }
}

hipError_t launch_grid_weights(hipStream_t st, const SegDesc& sd, int64_t n_toa, const double* nu,
                               const int32_t* chunk_of, const int32_t* tt_of, const int32_t* row_of,
                               const double* d_of, int32_t w, double beta, int32_t vmax, double* wd, double* dch,
                               int32_t s_idx, int32_t n_sig, int32_t half) {
  if (half && (vmax % 8 != 0 || dch)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_grid_weights, dim3((unsigned)((n_toa + 255) / 256)), dim3(256), 0, st, sd, n_toa, nu,
                     chunk_of, tt_of, row_of, d_of, w, beta, vmax, wd, (dbl2*)dch, s_idx, n_sig, half);
  return hipGetLastError();
}

hipError_t launch_grid_dft(hipStream_t st, GridSegs gsegs, int32_t P, const double* coef, int32_t K, int32_t R_pad) {
  if (R_pad % 128 != 0 || gsegs.n <= 0 || gsegs.n > kGridMaxSeg) return hipErrorInvalidValue;
  int64_t gx = 0;
  for (int s = 0; s < gsegs.n; ++s) {
    GridSegDev& g = gsegs.s[s];
    if (g.lde < (g.half + kGridMI) / kGridMI * kGridMI || g.nm % 2) return hipErrorInvalidValue;
    g.nblk = (g.half + 1 + kGridMI - 1) / kGridMI;
    gx += g.nblk;
  }
  if (gx > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_grid_dft<kGridMI>), dim3((unsigned)((R_pad / 128 + 3) / 4), (unsigned)P, (unsigned)gx), dim3(256),
                     0, st, gsegs, coef, K, R_pad);
  return hipGetLastError();
}

}  // namespace fpta
