// Gridded synthesis (grid.hip) on the fp64 matrix cores: both per-batch GEMMs of the factorisation
// F ~= W E as v_mfma_f64_16x16x4_f64 chains.
//
//   k_grid_dft_mfma     grid values G[p][j][r] (half-range real DFT, both grid halves per pass)
//   k_grid_interp_mfma  residuals out[r][t] = sum_s sum_i W_s[t][i] G_s[J + i][r] (+ white / ECORR)
//
// Fragment maps of v_mfma_f64_16x16x4_f64 (cdna_hip_programming.md §3): A[i = l & 15][k = l >> 4],
// B[k = l >> 4][j = l & 15], D: col = l & 15, row = (l >> 4) + 4 reg.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdlib>

#include "grid_device.h"

namespace fpta {

// k_grid_interp_mfma: 32 TOAs x 16 kInterpRW realizations per wave, kInterpWPC persistent workgroups per CU
// (compile-time; archived tools/experiments_archive.sh interp_variants built the alternatives it measured)
#ifndef FPTA_INTERP_RW
#define FPTA_INTERP_RW 8
#endif
#ifndef FPTA_INTERP_WPC
#define FPTA_INTERP_WPC 2
#endif
#ifndef FPTA_INTERP_DEPTH
#define FPTA_INTERP_DEPTH 2
#endif
constexpr int kInterpRW = FPTA_INTERP_RW;
constexpr int kInterpDepth = FPTA_INTERP_DEPTH;  // k_grid_interp_mfma: steps of operand prefetch (2 or 3)
constexpr int kInterpWPC = FPTA_INTERP_WPC;
#ifndef FPTA_WHITE_WPC
#define FPTA_WHITE_WPC 2  // persistent workgroups per CU of the white-epilogue interpolation
#endif
#ifndef FPTA_ECORR_AHEAD
#define FPTA_ECORR_AHEAD 1  // white / ECORR epilogue: groups of epoch normals loaded ahead (1 or 2)
#endif

// ----------------------------------------------------------------------------- k_grid_dft_mfma
// Quarter-range real DFT (one radix-2 step, then GEMMs): with nf = 4 Q and theta = 2 pi k j / nf, the modes of odd k
// (m = k - 1 even) and of even k (m odd) give per grid row j in [0, Q]
//   Oc_j = sum_{k odd} q_k c_k cos theta,  Os_j = sum_{k odd} q_k s_k sin theta,  Ec_j, Es_j likewise for k even,
// and, as even-k terms repeat with period nf / 2 and odd-k terms change sign (cos even, sin odd in j),
//   g_j = E + O,  g_{nf/2 + j} = E - O,  g_{nf/2 - j} = (Ec - Es) - (Oc - Os),  g_{nf - j} = (Ec - Es) + (Oc - Os)
// (E = Ec + Es, O = Oc + Os): nf nm / 2 multiply-adds per (pulsar, realization), half the half-range DFT's.
// A = table (grid row, mode of one parity), B = coefficients (mode, realization), four GEMMs sharing the output tile.
// Both operands come in tile pairs from one 16-byte load per lane: lane (lr, lg) loads table rows 2 lr, 2 lr + 1
// (.x row tile 2u, .y row tile 2u + 1) and realizations 2 lr, 2 lr + 1 (.x realization tile 2m, .y tile 2m + 1), so
// a 4-mode step issues MJ + MR loads for 2 MJ MR MFMAs. D of (row tile 2u + h, realization tile 2m + e): lane
// (lr, lg) register g holds grid row j0 + 32 u + 2 (lg + 4 g) + h, realization r0 + 32 m + 2 lr + e, so the two
// realization tiles of a pair store one 16-byte value per lane (256-byte runs per grid row). Wave tile 16 MJ rows x
// 16 MR realizations. Tables tq[4][ntq][ldq] (odd-k cos, odd-k sin, even-k cos, even-k sin) are zero-padded to ntq
// (multiple of 8) modes per parity and ldq (multiple of 16 MJ) rows; padded modes re-read the parity's last mode
// (finite) against zero table rows.
// Grid (1-D, XCD-grouped): a coefficient tile T = (pulsar, 64 MR-realization block) has nz row blocks over all
// signals, which read the same coefficients; workgroup b runs on XCD b % 8 and the nz row blocks of one tile are
// consecutive workgroups of one XCD, so the tile is read from HBM once and re-read from that XCD's L2.
template <int PJ, int PR>
__device__ __forceinline__ void dft_parity(d4 (&C)[2 * PJ][2 * PR], d4 (&S)[2 * PJ][2 * PR],
                                           const double* __restrict__ cb, const double* __restrict__ tc,
                                           const double* __restrict__ ts, int n, int par, int ldq, int R_pad, int lg) {
  struct Ops {
    dbl2 bc[PR], bs[PR], ac[PJ], as[PJ];
  };
  auto mfma = [&](const Ops& o) {
#pragma unroll
    for (int u = 0; u < PJ; ++u)
#pragma unroll
      for (int i = 0; i < PR; ++i) {
        C[2 * u][2 * i] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac[u].x, o.bc[i].x, C[2 * u][2 * i], 0, 0, 0);
        C[2 * u][2 * i + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac[u].x, o.bc[i].y, C[2 * u][2 * i + 1], 0, 0, 0);
        C[2 * u + 1][2 * i] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac[u].y, o.bc[i].x, C[2 * u + 1][2 * i], 0, 0, 0);
        C[2 * u + 1][2 * i + 1] =
            __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac[u].y, o.bc[i].y, C[2 * u + 1][2 * i + 1], 0, 0, 0);
        S[2 * u][2 * i] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.as[u].x, o.bs[i].x, S[2 * u][2 * i], 0, 0, 0);
        S[2 * u][2 * i + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.as[u].x, o.bs[i].y, S[2 * u][2 * i + 1], 0, 0, 0);
        S[2 * u + 1][2 * i] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.as[u].y, o.bs[i].x, S[2 * u + 1][2 * i], 0, 0, 0);
        S[2 * u + 1][2 * i + 1] =
            __builtin_amdgcn_mfma_f64_16x16x4f64(o.as[u].y, o.bs[i].y, S[2 * u + 1][2 * i + 1], 0, 0, 0);
      }
  };
  // operands of k-step q: modes of this parity t = 4 q + lg (m = 2 t + par), clamped to the parity's last mode (a
  // valid, finite value that meets a zero table row), so every load is unconditional and the next step's loads stay
  // in flight across the current step's MFMAs; two operand sets alternate (no register copies)
  auto load = [&](int qq, Ops& o) {
    const int m = 2 * min(4 * qq + lg, n - 1) + par;
    const double* __restrict__ cq = cb + (int64_t)(2 * m) * R_pad;
#pragma unroll
    for (int i = 0; i < PR; ++i) {
      o.bc[i] = *(const dbl2*)(cq + 32 * i);
      o.bs[i] = *(const dbl2*)(cq + R_pad + 32 * i);
    }
    const int64_t eo = (int64_t)(4 * qq) * ldq;
#pragma unroll
    for (int u = 0; u < PJ; ++u) {
      o.ac[u] = *(const dbl2*)(tc + eo + 32 * u);
      o.as[u] = *(const dbl2*)(ts + eo + 32 * u);
    }
  };
  const int nq = ((n + 7) >> 3) << 1;  // even: the tables hold ntq >= n rounded up to 8 modes (zero rows)
  Ops o0, o1;
  load(0, o0);
  for (int q = 0; q < nq; q += 2) {
    load(min(q + 1, nq - 1), o1);
    mfma(o0);
    load(min(q + 2, nq - 1), o0);
    mfma(o1);
  }
}

template <int MJ, int MR>
__global__ __launch_bounds__(256, 3) void k_grid_dft_mfma(GridSegs gsegs, const double* __restrict__ coef,
                                                          int32_t K, int32_t R_pad, int32_t n_xb, int32_t P,
                                                          int32_t nz) {
  static_assert(MJ % 2 == 0 && MR % 2 == 0, "operands come in tile pairs");
  constexpr int PJ = MJ / 2, PR = MR / 2;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int tile = (slot / nz) * 8 + xcd;
  if (tile >= n_xb * P) return;
  const int bx = tile % n_xb, p = tile / n_xb;
  int bz = slot - (slot / nz) * nz, s = 0;
  while (s + 1 < gsegs.n && bz >= gsegs.s[s].nblk) bz -= gsegs.s[s++].nblk;
  const GridSegDev& gs = gsegs.s[s];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int r0 = (bx * 4 + wave) * 16 * MR;
  if (r0 >= R_pad) return;
  const int j0 = bz * 16 * MJ;
  const double* __restrict__ cb = coef + ((int64_t)p * K + gs.col0) * R_pad + r0 + 2 * lr;
  // [0] odd k (m even), [1] even k (m odd): cos and sin accumulators
  d4 C[2][MJ][MR], S[2][MJ][MR];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int u = 0; u < MJ; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        C[a][u][i] = d4{0.0, 0.0, 0.0, 0.0};
        S[a][u][i] = d4{0.0, 0.0, 0.0, 0.0};
      }
  const int64_t tstride = (int64_t)gs.ntq * gs.ldq;
  const double* __restrict__ t0 = gs.tq + (int64_t)lg * gs.ldq + j0 + 2 * lr;
  const int n_odd = (gs.nm + 1) >> 1, n_even = gs.nm >> 1;
  dft_parity<PJ, PR>(C[0], S[0], cb, t0, t0 + tstride, n_odd, 0, gs.ldq, R_pad, lg);
  if (n_even > 0) dft_parity<PJ, PR>(C[1], S[1], cb, t0 + 2 * tstride, t0 + 3 * tstride, n_even, 1, gs.ldq, R_pad, lg);
  const int Q = gs.nf >> 2, H = gs.nf >> 1;
  double* __restrict__ gp = gs.g + (int64_t)p * gs.nf * R_pad + r0 + 2 * lr;
#pragma unroll
  for (int u = 0; u < PJ; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + 32 * u + 2 * (lg + 4 * g) + h;
        if (j > Q) continue;
#pragma unroll
        for (int i = 0; i < PR; ++i) {
          double pe[2], me[2], po[2], mo[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const double oc = C[0][2 * u + h][2 * i + e][g], os = S[0][2 * u + h][2 * i + e][g];
            const double ec = C[1][2 * u + h][2 * i + e][g], es = S[1][2 * u + h][2 * i + e][g];
            pe[e] = ec + es;
            me[e] = ec - es;
            po[e] = oc + os;
            mo[e] = oc - os;
          }
          *(dbl2*)(gp + (int64_t)j * R_pad + 32 * i) = dbl2{pe[0] + po[0], pe[1] + po[1]};
          *(dbl2*)(gp + (int64_t)(H + j) * R_pad + 32 * i) = dbl2{pe[0] - po[0], pe[1] - po[1]};
          if (j > 0 && j < Q) {
            *(dbl2*)(gp + (int64_t)(H - j) * R_pad + 32 * i) = dbl2{me[0] - mo[0], me[1] - mo[1]};
            *(dbl2*)(gp + (int64_t)(gs.nf - j) * R_pad + 32 * i) = dbl2{me[0] + mo[0], me[1] + mo[1]};
          }
        }
      }
}

// ----------------------------------------------------------------------------- k_grid_dft_gen
// The quarter-range DFT of k_grid_dft_mfma with the coefficients made on chip (DftGenArgs). A workgroup owns 16
// realizations of one pulsar and nw <= 4 waves:
//  1. every thread draws (mode, realization) coefficient pairs of the grid signal into LDS, term by term in the
//     grid signal's summation order (per-pulsar members: Philox + Box-Muller with k_gen's counter; common members:
//     their mixed coefficients loaded from the coefficient buffer), so each coefficient is made once per workgroup;
//  2. wave w takes 32-row chunks w, w + nw, ... of the quarter range (rows 0 .. nf / 4): per 4-mode k-step of one
//     parity, B[k = lg][j = lr] = the (cos, sin) pair of mode 2 (4 q + lg) + parity, realization r0 + lr (one
//     ds_read_b128), A = table rows in pairs (one 16-byte load per table: row tile 0 -> rows j0 + 2 lr, tile 1 ->
//     j0 + 2 lr + 1), and the same butterfly as k_grid_dft_mfma writes the grid rows.
// D of tile h: lane (lr, lg) register g = grid row j0 + 2 (lg + 4 g) + h, realization r0 + lr (16 consecutive
// realizations of a row per store instruction). A term's product is rounded before the sum, as k_gen stores it and
// k_coef_merge adds it.
constexpr int kDftGenMaxModes = 512;  // LDS: [modes][16 realizations][cos, sin] = 256 B per mode (128 KB at most)

__global__ __launch_bounds__(256, 2) void k_grid_dft_gen(DftGenArgs d) {
  extern __shared__ __attribute__((aligned(16))) double Bs[];  // [ntq * 2 (both parities)][16][2]
  const int nthr = blockDim.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = nthr >> 6;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int n_xb = d.R_pad >> 4;
  const int p = blockIdx.x / n_xb, r0 = (blockIdx.x - p * n_xb) * 16;
  const GridSegDev& gs = d.g;
  const int n_modes = 2 * gs.ntq;  // modes held: both parities' padded range (padding modes are zero)
  // 1. coefficients of every mode for the workgroup's 16 realizations, a realization pair per thread and mode (one
  //    Philox call per pair and generated term)
  for (int idx = threadIdx.x; idx < n_modes * 8; idx += nthr) {
    const int m = idx >> 3, rl = 2 * (idx & 7);
    double bc[2], bs[2];
    grid_term_coefs(d, gs.nm, d.coef, d.K, d.R_pad, d.n_real, d.real0, d.k0, d.k1, p, m, r0 + rl, bc, bs);
    *(dbl2*)(Bs + 2 * (m * 16 + rl)) = dbl2{bc[0], bs[0]};
    *(dbl2*)(Bs + 2 * (m * 16 + rl + 1)) = dbl2{bc[1], bs[1]};
  }
  __syncthreads();
  // 2. quarter-range rows, 32 per chunk
  const int Q = gs.nf >> 2, H = gs.nf >> 1;
  const int n_rc = (Q + 32) >> 5;
  const int64_t tstride = (int64_t)gs.ntq * gs.ldq;
  const int n_par[2] = {(gs.nm + 1) >> 1, gs.nm >> 1};  // modes of odd k (m = 2 t) and of even k (m = 2 t + 1)
  double* __restrict__ gp = gs.g + (int64_t)p * gs.nf * d.R_pad + r0 + lr;
  for (int rc = wave; rc < n_rc; rc += nw) {
    const int j0 = 32 * rc;
    d4 C[2][2], S[2][2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        C[par][h] = d4{0.0, 0.0, 0.0, 0.0};
        S[par][h] = d4{0.0, 0.0, 0.0, 0.0};
      }
      const double* __restrict__ tc = gs.tq + (int64_t)(2 * par) * tstride + (int64_t)lg * gs.ldq + j0 + 2 * lr;
      const double* __restrict__ ts = tc + tstride;
      const int nq = (n_par[par] + 3) >> 2;
      // operands of step q + 2 in flight while step q's MFMAs run (three sets, rotated)
      dbl2 ac[3], as[3], bb[3];
      auto fetch = [&](int q, int k) {
        const int qq = min(q, nq - 1);
        ac[k] = *(const dbl2*)(tc + (int64_t)(4 * qq) * gs.ldq);
        as[k] = *(const dbl2*)(ts + (int64_t)(4 * qq) * gs.ldq);
        bb[k] = *(const dbl2*)(Bs + 2 * ((2 * (4 * qq + lg) + par) * 16 + lr));
      };
      if (nq > 0) {
        fetch(0, 0);
        fetch(1, 1);
      }
      for (int q = 0; q < nq; q += 3) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (q + k >= nq) break;
          fetch(q + k + 2, (k + 2) % 3);
          C[par][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[k].x, bb[k].x, C[par][0], 0, 0, 0);
          C[par][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[k].y, bb[k].x, C[par][1], 0, 0, 0);
          S[par][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(as[k].x, bb[k].y, S[par][0], 0, 0, 0);
          S[par][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(as[k].y, bb[k].y, S[par][1], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + 2 * (lg + 4 * g) + h;
        if (j > Q) continue;
        const double oc = C[0][h][g], os = S[0][h][g], ec = C[1][h][g], es = S[1][h][g];
        const double pe = ec + es, me = ec - es, po = oc + os, mo = oc - os;
        gp[(int64_t)j * d.R_pad] = pe + po;
        gp[(int64_t)(H + j) * d.R_pad] = pe - po;
        if (j > 0 && j < Q) {
          gp[(int64_t)(H - j) * d.R_pad] = me - mo;
          gp[(int64_t)(gs.nf - j) * d.R_pad] = me + mo;
        }
      }
  }
}

hipError_t launch_grid_dft_gen(hipStream_t st, const DftGenArgs& a) {
  const int32_t Q = a.g.nf / 4, n_rc = (Q + 32) / 32;
  if (a.g.nf % 4 != 0 || !a.g.tq || a.R_pad % 16 != 0 || a.n_terms <= 0 || a.n_terms > kDftGenTerms || a.P <= 0 ||
      a.g.ldq < 32 * n_rc || a.g.ntq < ((((a.g.nm + 1) >> 1) + 3) & ~3) || 2 * a.g.ntq > kDftGenMaxModes)
    return hipErrorInvalidValue;
  for (int i = 0; i < a.n_terms; ++i)
    if (a.term_nm[i] <= 0 || a.term_nm[i] > a.g.nm || (a.term_kind[i] == 0 && !a.term_amp[i]) ||
        (a.term_kind[i] == 1 && (!a.coef || a.term_col0[i] < 0 || a.term_col0[i] + 2 * a.term_nm[i] > a.K)))
      return hipErrorInvalidValue;
  const int64_t blocks = (int64_t)a.P * (a.R_pad / 16);
  if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
  const int nw = std::min<int32_t>(4, n_rc);
  const size_t lds = sizeof(double) * 2 * 16 * 2 * (size_t)a.g.ntq;
  hipLaunchKernelGGL(k_grid_dft_gen, dim3((unsigned)blocks), dim3(64 * nw), lds, st, a);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- k_coef_merge
// Coalesced grid signal: the anchor's coefficient columns += every other member's (same modes k = m + 1, same w0,
// same chromatic weight per TOA), summed in member order. Thread = 2 adjacent realizations of one column.
__global__ __launch_bounds__(256) void k_coef_merge(CoefMerge m, int32_t K, int32_t R_pad,
                                                    double* __restrict__ coef) {
  const int r = (blockIdx.x * 256 + threadIdx.x) * 2;
  if (r >= R_pad) return;
  const int j = blockIdx.y;
  const int64_t prow = (int64_t)blockIdx.z * K;
  double* __restrict__ dst = coef + (prow + m.dst + j) * R_pad + r;
  dbl2 acc = *(const dbl2*)dst;
  for (int i = 0; i < m.n; ++i)
    if (j < m.ncol[i]) acc += *(const dbl2*)(coef + (prow + m.src[i] + j) * R_pad + r);
  *(dbl2*)dst = acc;
}

hipError_t launch_coef_merge(hipStream_t st, const CoefMerge& m, int32_t P, int32_t K, int32_t R_pad, double* coef) {
  if (m.n <= 0 || m.n > kGridMaxSeg || R_pad % 2 != 0 || P <= 0 || P > 65535) return hipErrorInvalidValue;
  int32_t jmax = 0;
  for (int i = 0; i < m.n; ++i) {
    if (m.src[i] < 0 || m.ncol[i] <= 0 || m.src[i] + m.ncol[i] > K || m.dst + m.ncol[i] > K) return hipErrorInvalidValue;
    jmax = std::max(jmax, m.ncol[i]);
  }
  hipLaunchKernelGGL(k_coef_merge, dim3((unsigned)((R_pad / 2 + 255) / 256), (unsigned)jmax, (unsigned)P), dim3(256),
                     0, st, m, K, R_pad, coef);
  return hipGetLastError();
}

// White-noise normals (oracle quad_normals on the white stream, the words of kernels.hip white_pair).
// quad: the white normals of TOAs t, t + 1 and realizations g, g + 1 (z[2 e + h]: TOA t + e, realization g + h) from one
// Philox call when t and g are even.
// the misaligned case out of line: one Philox call per value (a pulsar's first chunk at an odd TOA offset, or an odd
// first realization), so its temporaries never weigh on the interpolation kernels' register budget
__device__ __attribute__((noinline)) double white_one(uint64_t t, uint64_t g, uint32_t k0, uint32_t k1) {
  return quad_normal(t, kWhiteStream, g, k0, k1);
}
__device__ __forceinline__ void white_quad(int64_t t, int64_t g, uint32_t k0, uint32_t k1, double (&z)[4]) {
  if (((t | g) & 1) == 0) {
    quad4((uint64_t)t, kWhiteStream, (uint64_t)g, k0, k1, z);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = white_one((uint64_t)(t + (i >> 1)), (uint64_t)(g + (i & 1)), k0, k1);
  }
}

// ----------------------------------------------------------------------------- k_grid_interp_mfma
// out[r][t] = sum_v W[chunk][v][tt] G[row(chunk, v)][r] over the chunk's band rows v < V: every signal's band
// back to back (host plan), so one flat loop of V / 4 MFMA steps covers all signals. Per step A = grid values
// (realization, row), B = weights (row, TOA):
//  * the grid rows of a chunk sit in registers (lane l holds band row l + 64 i in rr[i], V <= kGridVMax) and a
//    step's 4 rows come from one ds_bpermute, so signals need no separate pipeline fill and the band is padded to
//    4 rows once per chunk, not per signal;
//  * the chunk's even and odd TOAs are two B-tiles (column j = TOA 2j, 2j + 1) over the same rows, so one set
//    of grid loads feeds both. Lane (lr, lg) loads W[v = 4q + lg][2 lr .. 2 lr + 1] with one 16-byte load
//    (.x even tile, .y odd tile);
//  * realization tiles come in pairs: lane (lr, lg) loads the adjacent realizations 2 lr, 2 lr + 1 of a
//    32-realization block with one 16-byte load (.x tile 2m, .y tile 2m + 1). D row rho of tile 2m + h is then
//    realization 32 m + 2 rho + h;
//  * D's register g of lane l holds TOA 2 (l & 15) + e of realization 32 m + 2 (lg + 4 g) + h in acc[e][2m + h]:
//    the two TOA parities of a lane are adjacent samples of one realization row (one 16-byte store, 256-byte
//    runs per row), and the two tiles of a realization pair sit in the same lane and register (one Philox call
//    per pair for the white epilogue).
// Wave tile = chunk x 16 RW realizations. Software pipeline: a step's operands are loaded two steps ahead (two
// register sets), and a wave sets up its NEXT tile and issues that tile's first two steps of loads before it
// stores the current tile. Loads and stores retire through one in-order counter (vmcnt), so loads issued after
// the 32 stores of an epilogue would wait for them; issued before, the next tile's first 32 MFMAs run while the
// stores drain (profiles/r02_interp_diag2.txt: without stores the kernel takes 0.42 ms, with them 0.63).
// White noise + ECORR added to the tile's sums in registers (before the next tile's operands are loaded: the
// Philox rounds and those operands do not fit in the register budget together).
template <int RW>
__device__ __forceinline__ void interp_white(const SynthArgs& a, const InterpTile<RW>& t, d4 (&acc)[2][RW]) {
  constexpr int NP = RW / 2;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int tt = 2 * lr;  // this lane's even TOA in the chunk; tt + 1 the odd one
  if (tt >= t.cnt) return;
  const int64_t tg = ld_uniform(a.offs + t.p) + t.y + tt;
  const bool two = tt + 1 < t.cnt;
  double sg[2] = {0.0, 0.0}, es[2] = {0.0, 0.0};
  int ep[2] = {-1, -1};
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    if (e == 1 && !two) break;
    sg[e] = a.w_sigma ? a.w_sigma[tg + e] : 0.0;
    ep[e] = a.w_block_of ? a.w_block_of[tg + e] : -1;
    es[e] = ep[e] >= 0 ? a.w_esig[ep[e]] : 0.0;
  }
  // ECORR epoch normals of group (m, g), loaded FPTA_ECORR_AHEAD groups ahead so their latency hides behind a group's Philox rounds
  // (one group at a time, each waiting for its own loads, left the tile's 16 gathers' latencies exposed). The loads are
  // unconditional: rows past n_real are clamped (those realizations are never stored) and a TOA without an epoch reads
  // epoch 0 against es = 0.
  const bool ecorr = a.w_block_of != nullptr;
  const int64_t e0 = ep[0] >= 0 ? ep[0] : 0, e1 = ep[1] >= 0 ? ep[1] : 0;
  auto zb_load = [&](int mg, double (&z)[2][2]) {
    const int rl = t.r0 + 32 * (mg >> 2) + 2 * (lg + 4 * (mg & 3));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double* row = a.w_zb + (int64_t)min(rl + h, a.n_real - 1) * a.w_nblocks;
      z[0][h] = row[e0];
      z[1][h] = row[e1];
    }
  };
  constexpr int D = FPTA_ECORR_AHEAD;  // groups of epoch normals in flight ahead of the one being added
  double zq[D + 1][2][2];
  if (ecorr)
#pragma unroll
    for (int i = 0; i < D; ++i) zb_load(i, zq[i]);
#pragma unroll
  for (int m = 0; m < NP; ++m) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int mg = 4 * m + g;
      if (ecorr && mg + D < 4 * NP) zb_load(mg + D, zq[(mg + D) % (D + 1)]);
      // acc[e][2m + h][g]: TOA tg + e, batch realization rl + h
      const int rl = t.r0 + 32 * m + 2 * (lg + 4 * g);
      if (a.w_sigma) {
        double z[4];
        white_quad(tg, a.real0 + rl, a.k0, a.k1, z);
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int h = 0; h < 2; ++h) acc[e][2 * m + h][g] = fma(sg[e], z[2 * e + h], acc[e][2 * m + h][g]);
      }
      if (ecorr) {
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int h = 0; h < 2; ++h) acc[e][2 * m + h][g] = fma(es[e], zq[mg % (D + 1)][e][h], acc[e][2 * m + h][g]);
      }
      // one (m, g) group at a time: no Philox state hoisted across groups (register budget)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// 64-bit DPP move within a row of 16 lanes (two 32-bit halves); CTRL: row_mirror 0x140 (lane l <- 15 - l),
// row_half_mirror 0x141 (l <- 7 - l within each 8), quad_perm 0x4E (l <- l ^ 2), 0xB1 (l <- l ^ 1). Every pairing
// is symmetric, so each step of a reduce-scatter exchanges complementary halves between two lanes.
template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// One reduce-scatter step: the lane keeps half `up` (0: x[0 .. H), 1: x[H .. 2H)) of its 2H values plus the
// partner's copy of that half, and hands the partner the other half.
template <int CTRL, int H>
__device__ __forceinline__ void rs_step(double (&x)[2 * H], bool up) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const double keep = up ? x[j + H] : x[j], send = up ? x[j] : x[j + H];
    x[j] = keep + dpp64<CTRL>(send);
  }
}

// Partial checksums of the tile's chunk, after its stores (the accumulators then die as the first
// reduce-scatter step consumes them). A wave takes the chunks of a partial group (GridBand::pgfirst: consecutive
// chunks of one pulsar) one after another for the same realizations: their partials add up in ps, in chunk order, and
// the group's last chunk stores the row (C3, groups of 16: 1/16 of the per-chunk rows' 0.41 GB per batch).
template <int RW>
__device__ __forceinline__ void interp_partials(const SynthArgs& a, const InterpTile<RW>& t, const d4 (&acc)[2][RW],
                                                double (&ps)[RW / 2]) {
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int tt = 2 * lr;
  {
    // partial checksums of this chunk: per realization the sum and sum of squares over the chunk's TOAs (lanes
    // without a TOA add 0), reduced over the 16 lanes of each row by a reduce-scatter (row_mirror, half_mirror,
    // xor 2, xor 1). Value k = 2 c + {0: sum, 1: sumsq} of combination c = 2 (4 m + g) + h (tile 2m + h,
    // register g), NV = 8 RW values; lane lr ends with k in [NV / 16 lr, NV / 16 (lr + 1)). RW = 8: the realization
    // pair of tiles (2m, 2m + 1) at register g for m = lr >> 2, g = lr & 3 (two 16-byte stores); RW = 4: combination
    // c = lr (one 16-byte store). Every value is summed over the 16 lanes by the same pairing tree whatever RW (each
    // step pairs the same lanes; only which half a lane keeps differs), so both give the same bits.
    static_assert(RW == 8 || RW == 4, "16 lanes of a row hold 16 RW / 2 values after the first step");
    constexpr int H1 = 4 * RW;  // values per lane after the first step
    double* __restrict__ pp = a.part + ((int64_t)(t.pg >= 0 ? t.pg : t.c) * a.R_pad + t.r0) * 2;
    const bool ok0 = tt < t.cnt, ok1 = tt + 1 < t.cnt;
    double x[H1];
    {
      // first step straight from the accumulators (the NV values are never all live): lanes 8..15 keep the upper
      // half of the combinations, lanes 0..7 the lower
      const bool up = lr >= 8;
#pragma unroll
      for (int j = 0; j < H1; ++j) {
        const int k0 = j, k1 = j + H1;  // the two values of this slot: kept or sent
        auto value = [&](int k) {
          const int c = k >> 1, h = c & 1, mg = c >> 1, m = mg >> 2, g = mg & 3;
          const double v0 = ok0 ? acc[0][2 * m + h][g] : 0.0, v1 = ok1 ? acc[1][2 * m + h][g] : 0.0;
          return (k & 1) ? fma(v0, v0, v1 * v1) : v0 + v1;
        };
        const double lo = value(k0), hi = value(k1);
        x[j] = (up ? hi : lo) + dpp64<0x140>(up ? lo : hi);
      }
    }
    {
      double (&y)[H1] = x;
      rs_step<0x141, H1 / 2>(y, (lr & 7) >= 4);
      double (&z)[H1 / 2] = *reinterpret_cast<double(*)[H1 / 2]>(&y[0]);
      rs_step<0x4E, H1 / 4>(z, (lr & 3) >= 2);
      double (&w)[H1 / 4] = *reinterpret_cast<double(*)[H1 / 4]>(&z[0]);
      rs_step<0xB1, H1 / 8>(w, (lr & 1) != 0);
    }
#pragma unroll
    for (int i = 0; i < RW / 2; ++i) ps[i] = t.pfirst ? x[i] : ps[i] + x[i];
    if (!t.plast) return;
    // non-temporal, as the block's own stores: the partials are read back by k_part_reduce from HBM, and
    // L2-allocating them would evict the grid rows the next chunks re-read
    if constexpr (RW == 8) {
      const int mm = lr >> 2, gg = lr & 3;
      const int rl = 32 * mm + 2 * (lg + 4 * gg);  // realization of (tile 2mm, register gg); rl + 1: tile 2mm + 1
      __builtin_nontemporal_store(dbl2{ps[0], ps[1]}, (dbl2*)(pp + 2 * rl));
      __builtin_nontemporal_store(dbl2{ps[2], ps[3]}, (dbl2*)(pp + 2 * rl + 2));
    } else {
      const int h = lr & 1, mg = lr >> 1;
      const int rl = 32 * (mg >> 2) + 2 * (lg + 4 * (mg & 3)) + h;
      __builtin_nontemporal_store(dbl2{ps[0], ps[1]}, (dbl2*)(pp + 2 * rl));
    }
  }
}

// The tile's epilogue: its block rows, then (FPTA_OPT_FUSE_CHECKSUMS) its partial checksums.
template <bool PART, int RW, int PACE = 0>
__device__ __forceinline__ void interp_store(const SynthArgs& a, double* __restrict__ out, const InterpTile<RW>& t,
                                             const d4 (&acc)[2][RW], double (&ps)[RW / 2]) {
  interp_store_rows<RW, PACE>(a, out, t, acc);
  if constexpr (PART) interp_partials<RW>(a, t, acc, ps);
}
// one chunk per partial row (the diagnostic kernels)
template <bool PART, int RW, int PACE = 0>
__device__ __forceinline__ void interp_store(const SynthArgs& a, double* __restrict__ out, const InterpTile<RW>& t,
                                             const d4 (&acc)[2][RW]) {
  double ps[RW / 2];
  interp_store<PART, RW, PACE>(a, out, t, acc, ps);
}

// Tile walk of the persistent interpolation kernels. Work item = (partial group, realization block), items
// group-major (the realization blocks of a group run side by side on one XCD and share its weights and grid rows in
// L2); a wave takes its item's chunks in order. Groups come from GridBand::pgfirst for fused partial checksums (PART),
// else a group is one chunk (item = chunk x realization block). Every field is wave-uniform.
struct TileWalk {
  int item, k, c0, c1;  // work item; chunk c0 + k of its group's chunks [c0, c1)
  template <bool PART>
  __device__ __forceinline__ void start(const GridBand& band, int n_rb, int end) {
    k = 0;
    if (item >= end) return;
    const int g = item / n_rb;
    if constexpr (PART) {
      c0 = ld_uniform(band.pgfirst + g);
      c1 = ld_uniform(band.pgfirst + g + 1);
    } else {
      c0 = g;
      c1 = g + 1;
    }
  }
  __device__ __forceinline__ int group(int n_rb) const { return item / n_rb; }
  __device__ __forceinline__ int chunk() const { return c0 + k; }
  __device__ __forceinline__ bool first() const { return k == 0; }
  __device__ __forceinline__ bool last() const { return c0 + k + 1 >= c1; }  // the tile's chunk ends its group
  template <bool PART>
  __device__ __forceinline__ void next(const GridBand& band, int n_rb, int stride, int end) {
    if (last()) {
      item += stride;
      start<PART>(band, n_rb, end);
    } else {
      ++k;
    }
  }
};

// Persistent launch: gridDim.x (a multiple of 8) workgroups, about as many as are co-resident; workgroup
// b runs on XCD b % 8 and walks that XCD's contiguous range of tiles (consecutive chunks: their grid rows
// overlap, so they stay in the XCD's L2). One tile per short-lived workgroup instead left the CUs mostly
// empty (SQ_WAVE_CYCLES ~ 0.7 resident waves per SIMD): workgroup dispatch, not the memory system, paced it.
// Every wave of a workgroup walks the same tiles (its own 16 RW realizations of each); a wave whose realization
// block lies past R_pad exits at once (no barrier in the kernel).
template <bool WHITE, bool PART, int RW>
__global__ __launch_bounds__(256, FPTA_INTERP_WPC) void k_grid_interp_mfma(SynthArgs a, GridBand band, int32_t n_tiles,
                                                                         int32_t R_pad, double* __restrict__ out) {
  static_assert(RW % 2 == 0, "realization tiles come in pairs");
  static_assert(kGridTT == 32, "two 16-TOA B-tiles per chunk");
  constexpr int NP = RW / 2;
  // n_tiles: work items (TileWalk), partial groups (or chunks) x realization blocks
  const int n_rb = (R_pad + 64 * RW - 1) / (64 * RW);
  const int per = (n_tiles + 7) >> 3;
  const int x = blockIdx.x & 7;
  const int stride = gridDim.x >> 3;
  const int end = min(n_tiles, (x + 1) * per);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;

  auto setup = [&](const TileWalk& tw, InterpTile<RW>& t) {
    // chunk-(group-)major tiles: the realization blocks of one chunk are consecutive tiles, so they run together on
    // one XCD and the chunk's weights are read from HBM once (realization-block-major read them once per block)
    const int grp = __builtin_amdgcn_readfirstlane(tw.group(n_rb));
    t.c = __builtin_amdgcn_readfirstlane(tw.chunk());
    const int rb = __builtin_amdgcn_readfirstlane(tw.item - grp * n_rb);  // realization block of 64 RW
    t.pg = grp;
    t.pfirst = tw.first();
    t.plast = tw.last();
    t.r0 = (rb * 4 + wave) * 16 * RW;
    const int4 ci = band.chunks[t.c];
    t.p = __builtin_amdgcn_readfirstlane(ci.x);
    t.y = __builtin_amdgcn_readfirstlane(ci.y);
    t.cnt = __builtin_amdgcn_readfirstlane(ci.z);
    t.nq = __builtin_amdgcn_readfirstlane(ci.w) >> 2;
    FPTA_DCHECK(4 * t.nq <= band.vmax && t.nq > 0, "k_grid_interp_mfma band rows", 4 * t.nq, band.vmax + 1);
    const int32_t* __restrict__ rt = band.rows + (int64_t)t.c * band.vmax;
#pragma unroll
    for (int i = 0; i < kGridVMax / 64; ++i) t.rr[i] = rt[min(64 * i + lane, 4 * t.nq - 1)];
    // a realization block past R_pad (R_pad not a multiple of 64 RW): this wave computes on block 0's columns and
    // stores nothing. Tiles of one wave alternate realization blocks, so this is decided per tile, never by exiting
    // (an exit on the first tile's block dropped the wave's later valid tiles, and a later invalid tile read past
    // its rows and wrote another chunk's partial checksums)
    t.G0 = band.g + (t.r0 < R_pad ? t.r0 : 0) + 2 * lr;
    t.Wp = band.wd + ((int64_t)t.c * band.vmax + lg) * kGridTT + 2 * lr;
  };
  auto load = [&](const InterpTile<RW>& t, int qq, dbl2(&av)[NP], dbl2& bv) {
    const int blk = qq >> 4;  // 64-row block of the step's rows (uniform)
    const int src = blk == 0 ? t.rr[0] : (blk == 1 ? t.rr[1] : (blk == 2 ? t.rr[2] : t.rr[3]));
    const int row = __builtin_amdgcn_ds_bpermute(((4 * qq + lg) & 63) << 2, src);
    FPTA_DCHECK(row >= 0 && row < band.grid_rows, "k_grid_interp_mfma grid row", row, band.grid_rows);
    const double* __restrict__ gr = t.G0 + (int64_t)row * R_pad;
#pragma unroll
    for (int m = 0; m < NP; ++m) av[m] = *(const dbl2*)(gr + 32 * m);
    bv = *(const dbl2*)(t.Wp + 4 * kGridTT * qq);
  };
  d4 acc[2][RW];  // [TOA parity][realization tile]
  double ps[RW / 2];  // partial checksums of the chunk group so far (PART)
  auto mfma = [&](const dbl2(&av)[NP], const dbl2& bv) {
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      acc[0][2 * m] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].x, bv.x, acc[0][2 * m], 0, 0, 0);
      acc[0][2 * m + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].y, bv.x, acc[0][2 * m + 1], 0, 0, 0);
      acc[1][2 * m] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].x, bv.y, acc[1][2 * m], 0, 0, 0);
      acc[1][2 * m + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].y, bv.y, acc[1][2 * m + 1], 0, 0, 0);
    }
  };

  TileWalk tw{x * per + (int)(blockIdx.x >> 3)};
  if (tw.item >= end) return;
  tw.start<PART>(band, n_rb, end);
  InterpTile<RW> cur;
  setup(tw, cur);
  FPTA_DCHECK(R_pad % (16 * RW) == 0, "k_grid_interp_mfma realization padding", R_pad % (16 * RW), 1);
  // operand sets: step q's operands are loaded kInterpDepth steps ahead (FPTA_INTERP_DEPTH 2 or 3). After a tile's
  // epilogue the first load that waits (vmcnt) for its 32 stores is that of step kInterpDepth of the next tile.
  dbl2 a0[NP], a1[NP], b0, b1;
#if FPTA_INTERP_DEPTH == 3
  dbl2 a2[NP], b2;
#endif
  auto prefetch = [&](const InterpTile<RW>& t) {
    load(t, 0, a0, b0);
    load(t, min(1, t.nq - 1), a1, b1);
#if FPTA_INTERP_DEPTH == 3
    load(t, min(2, t.nq - 1), a2, b2);
#endif
  };
  prefetch(cur);
  while (true) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < RW; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
    // each operand set is refilled kInterpDepth steps ahead right after its MFMAs
    for (int q = 0; q < cur.nq; q += kInterpDepth) {
      __builtin_amdgcn_sched_barrier(0);
      mfma(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (q + kInterpDepth < cur.nq) load(cur, q + kInterpDepth, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (q + 1 < cur.nq) {
        mfma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        if (q + 1 + kInterpDepth < cur.nq) load(cur, q + 1 + kInterpDepth, a1, b1);
      }
#if FPTA_INTERP_DEPTH == 3
      __builtin_amdgcn_sched_barrier(0);
      if (q + 2 < cur.nq) {
        mfma(a2, b2);
        __builtin_amdgcn_sched_barrier(0);
        if (q + 2 + kInterpDepth < cur.nq) load(cur, q + 2 + kInterpDepth, a2, b2);
      }
#endif
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (WHITE) {
      // the Philox rounds of the white epilogue and a second tile's operands do not fit in the register budget
      // together: this variant stores first, then starts the next tile
      if (cur.r0 < R_pad) {
        interp_white<RW>(a, cur, acc);
        interp_store<PART, RW>(a, out, cur, acc, ps);
      }
      tw.next<PART>(band, n_rb, stride, end);
      if (tw.item >= end) break;
      setup(tw, cur);
      prefetch(cur);
    } else {
      // next tile: its first steps are in flight before this tile's stores enter the vmcnt queue
      tw.next<PART>(band, n_rb, stride, end);
      const bool more = tw.item < end;
      InterpTile<RW> nxt = cur;
      if (more) {
        setup(tw, nxt);
        prefetch(nxt);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (cur.r0 < R_pad) interp_store<PART, RW>(a, out, cur, acc, ps);
      if (!more) break;
      cur = nxt;
    }
  }
}

// ----------------------------------------------------------------------------- k_grid_interp_ws
// The interpolation with warp-specialised roles, so the residual stores never stall an operand load. In
// k_grid_interp_mfma a wave's loads and stores retire through one in-order counter (vmcnt): every load issued after
// a tile's 32 stores waits for them, and the MFMA and store streams serialise (0.42 ms without stores, 0.33 ms of
// stores alone, 0.63 ms together on C2). Here a workgroup (one per CU) has 4 compute waves and 4 producer waves:
//  * producer wave p loads, kWsLead steps ahead, the 4 grid rows of compute wave p's 128 realizations and weight
//    row p of the step, with direct-to-LDS loads (five wave-instructions per step) into a ring of kWsSlots slots;
//    it waits only for its own loads (vmcnt) and never stores;
//  * compute wave w reads its operands from LDS (lgkmcnt), runs the same MFMA steps as k_grid_interp_mfma (even /
//    odd TOA B-tiles, realization tile pairs) and stores the tile; it issues no global load, so it never waits for
//    its stores;
//  * one s_barrier per band step: before barrier S the producers' loads of step S + 1 have landed and the compute
//    waves' reads of step S are done, so slot (S + kWsLead) mod kWsSlots (step S - 1's) can be refilled after it.
// Every wave walks the same tiles and steps (a tile = one chunk x 512 realizations), so all issue the same number
// of barriers; compute waves whose realizations lie past R_pad compute on clamped rows and store nothing. The
// barrier is a plain s_barrier: __syncthreads() would add a workgroup fence, i.e. vmcnt(0) on the stores.
#ifndef FPTA_WS_LEAD
#define FPTA_WS_LEAD 3
#endif
constexpr int kWsLead = FPTA_WS_LEAD;  // 3: a 4-slot ring (68 KB) leaves a CU room for co-running DFT / draw waves
constexpr int kWsSlots = kWsLead + 1;
constexpr int kWsSlotGrid = 4 * 4 * 128;          // doubles: [band row j][compute wave][128 realizations]
constexpr int kWsSlot = kWsSlotGrid + 4 * kGridTT;  // + [band row j][32 TOAs] weights: 17 KB per slot
constexpr int kWsLoadsPerStep = 5;                // per producer: 4 grid rows + 1 weight row

// s_waitcnt with only vmcnt <= N (lgkmcnt, expcnt not waited), and with only lgkmcnt(0)
template <int N>
__device__ __forceinline__ void ws_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void ws_wait_lgkm0() { __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4)); }
__device__ __forceinline__ void ws_barrier() { asm volatile("s_barrier" ::: "memory"); }
// vmcnt <= kWsLoadsPerStep * n, n = the steps whose loads may stay in flight (0 .. kWsLead - 1)
__device__ __forceinline__ void ws_wait_steps(int n) {
  if (n <= 0) ws_wait_vm<0>();
  else if (n == 1) ws_wait_vm<kWsLoadsPerStep>();
  else if (n == 2) ws_wait_vm<2 * kWsLoadsPerStep>();
  else if (n == 3) ws_wait_vm<3 * kWsLoadsPerStep>();
  else if (n == 4) ws_wait_vm<4 * kWsLoadsPerStep>();
  else if (n == 5) ws_wait_vm<5 * kWsLoadsPerStep>();
  else ws_wait_vm<6 * kWsLoadsPerStep>();
  static_assert(kWsLead - 1 <= 6, "ws_wait_steps covers up to 6 steps in flight");
}

template <bool PART>
__global__ __launch_bounds__(512, 1) void k_grid_interp_ws(SynthArgs a, GridBand band, int32_t n_tiles, int32_t R_pad,
                                                           double* __restrict__ out) {
  constexpr int RW = 8, NP = RW / 2;
  static_assert(kGridTT == 32, "two 16-TOA B-tiles per chunk");
  __shared__ __attribute__((aligned(16))) double ring[kWsSlots * kWsSlot];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int per = (n_tiles + 7) >> 3;
  const int x = blockIdx.x & 7;
  const int stride = gridDim.x >> 3;
  const int end = min(n_tiles, (x + 1) * per);
  const int first = x * per + (int)(blockIdx.x >> 3);
  const int n_rb = (R_pad + 511) / 512;
  // n_tiles: work items (TileWalk)
  const bool producer = wave >= 4;
  const int w = wave & 3;  // compute wave w, or the producer serving it
  if (first >= end) return;  // no tile: every wave of the workgroup leaves (no barrier issued)

  if (producer) {
    // cursor of the step the producer loads next: tile, step q of nq, chunk, realization base. Everything it
    // reads besides the operands is wave-uniform (scalar loads), so its vmcnt counts the ring loads alone.
    TileWalk tw{first};
    tw.start<PART>(band, n_rb, end);
    int q = 0, nq = 0, c = 0, r0 = 0;
    auto setup = [&]() {
      const int grp = __builtin_amdgcn_readfirstlane(tw.group(n_rb));
      c = __builtin_amdgcn_readfirstlane(tw.chunk());
      const int rb = __builtin_amdgcn_readfirstlane(tw.item - grp * n_rb);
      r0 = rb * 512 + w * 128;
      if (r0 >= R_pad) r0 = 0;  // a compute wave past R_pad: valid rows, its sums are never stored
      nq = __builtin_amdgcn_readfirstlane(ld_uniform4(band.chunks + c).w) >> 2;
    };
    int issued = 0;  // steps whose loads are issued
    bool valid = true;
    setup();
    auto issue = [&]() {
      double* slot = ring + (issued % kWsSlots) * kWsSlot;
      const int4 r4 = ld_uniform4(band.rows + (int64_t)c * band.vmax + 4 * q);  // the step's 4 rows
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = __builtin_amdgcn_readfirstlane(j == 0 ? r4.x : (j == 1 ? r4.y : (j == 2 ? r4.z : r4.w)));
        FPTA_DCHECK(row >= 0 && row < band.grid_rows, "k_grid_interp_ws grid row", row, band.grid_rows);
        __builtin_amdgcn_global_load_lds((const void*)(band.g + (int64_t)row * R_pad + r0 + 2 * lane),
                                         (__attribute__((address_space(3))) void*)(slot + (j * 4 + w) * 128), 16, 0,
                                         0);
      }
      // weight row w of the step: 32 doubles = 64 dwords, one per lane
      __builtin_amdgcn_global_load_lds(
          (const void*)((const uint32_t*)(band.wd + ((int64_t)c * band.vmax + 4 * q + w) * kGridTT) + lane),
          (__attribute__((address_space(3))) void*)(slot + kWsSlotGrid + w * kGridTT), 4, 0, 0);
      ++issued;
      if (++q == nq) {
        q = 0;
        tw.next<PART>(band, n_rb, stride, end);
        valid = tw.item < end;
        if (valid) setup();
      }
    };
    for (int i = 0; i < kWsLead && valid; ++i) issue();
    ws_wait_steps(issued - 1);  // step 0 has landed
    ws_barrier();
    // iteration S: refill the slot of step S - 1 with step S + kWsLead, make sure step S + 1 has landed
    for (int S = 0;; ++S) {
      if (valid) issue();
      ws_wait_steps(issued - (S + 2));
      // the barrier count must equal the compute waves': one per step of the workgroup's tiles
      if (S + 1 >= issued && !valid) {
        ws_barrier();
        break;
      }
      ws_barrier();
    }
    return;
  }

  // compute wave
  d4 acc[2][RW];
  double ps[4];  // partial checksums of the chunk group so far (PART)
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int i = 0; i < RW; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
  auto read = [&](int S, dbl2(&av)[NP], dbl2& bv) {
    const double* slot = ring + (S % kWsSlots) * kWsSlot;
#pragma unroll
    for (int m = 0; m < NP; ++m) av[m] = *(const dbl2*)(slot + (lg * 4 + w) * 128 + 32 * m + 2 * lr);
    bv = *(const dbl2*)(slot + kWsSlotGrid + lg * kGridTT + 2 * lr);
  };
  auto mfma = [&](const dbl2(&av)[NP], const dbl2& bv) {
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      acc[0][2 * m] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].x, bv.x, acc[0][2 * m], 0, 0, 0);
      acc[0][2 * m + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].y, bv.x, acc[0][2 * m + 1], 0, 0, 0);
      acc[1][2 * m] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].x, bv.y, acc[1][2 * m], 0, 0, 0);
      acc[1][2 * m + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m].y, bv.y, acc[1][2 * m + 1], 0, 0, 0);
    }
  };
  dbl2 a0[NP], a1[NP], b0, b1;
  ws_barrier();  // step 0 has landed
  read(0, a0, b0);
  ws_wait_lgkm0();
  int S = 0;
  TileWalk tw{first};
  for (tw.start<PART>(band, n_rb, end); tw.item < end; tw.next<PART>(band, n_rb, stride, end)) {
    InterpTile<RW> t;
    const int grp = __builtin_amdgcn_readfirstlane(tw.group(n_rb));
    t.c = __builtin_amdgcn_readfirstlane(tw.chunk());
    const int rb = __builtin_amdgcn_readfirstlane(tw.item - grp * n_rb);
    t.pg = grp;
    t.pfirst = tw.first();
    t.plast = tw.last();
    t.r0 = rb * 512 + w * 128;
    const int4 ci = ld_uniform4(band.chunks + t.c);
    t.p = __builtin_amdgcn_readfirstlane(ci.x);
    t.y = __builtin_amdgcn_readfirstlane(ci.y);
    t.cnt = __builtin_amdgcn_readfirstlane(ci.z);
    t.nq = __builtin_amdgcn_readfirstlane(ci.w) >> 2;
    // step S's operands in (a0, b0); step S + 1's are read from LDS after barrier S, while step S's MFMAs run
    for (int q = 0; q < t.nq; ++q, ++S) {
      ws_barrier();  // step S + 1 has landed; step S - 1's slot may now be refilled
      read(S + 1, a1, b1);
      mfma(a0, b0);
      ws_wait_lgkm0();
#pragma unroll
      for (int m = 0; m < NP; ++m) a0[m] = a1[m];
      b0 = b1;
    }
    if (t.r0 < R_pad) interp_store<PART, RW>(a, out, t, acc, ps);
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < RW; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
  }
}

#ifdef FPTA_DIAG_KERNELS
#include "diag/interp_ws2.inc"
#endif

hipError_t launch_grid_interp_ws(hipStream_t st, const SynthArgs& a, const GridBand& band, int32_t R_pad, bool ws2) {
  if (band.n_chunks <= 0 || band.vmax < 4 || band.vmax % 4 != 0 || band.vmax > kGridVMax || R_pad % 128 != 0 ||
      a.w_on || a.accumulate)
    return hipErrorInvalidValue;
  if (a.part && (!band.pgfirst || band.n_pg <= 0)) return hipErrorInvalidValue;
  const int32_t n_rb = (R_pad + 511) / 512;
  const int64_t tiles = (int64_t)(a.part ? band.n_pg : band.n_chunks) * n_rb;  // work items (TileWalk)
  if (tiles > 0x7FFFFFFF) return hipErrorInvalidValue;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
  // persistent: one workgroup per CU (the 4-slot ring takes 4 x 17 KB = 68 KB of the 160 KB LDS)
  const int64_t grid = std::min<int64_t>((tiles + 7) / 8 * 8, ((int64_t)n_cu + 7) / 8 * 8);
  if (ws2) {  // 256-realization tiles, two workgroups per CU (diagnostic builds only)
#ifndef FPTA_DIAG_KERNELS
    return hipErrorInvalidValue;
#else
    if (a.part) return hipErrorInvalidValue;
    const int64_t tiles2 = (int64_t)band.n_chunks * ((R_pad + 255) / 256);
    if (tiles2 > 0x7FFFFFFF) return hipErrorInvalidValue;
    const int64_t grid2 = std::min<int64_t>((tiles2 + 7) / 8 * 8, (2 * (int64_t)n_cu + 7) / 8 * 8);
    hipLaunchKernelGGL(k_grid_interp_ws2<false>, dim3((unsigned)grid2), dim3(512), 0, st, a, band, (int32_t)tiles2,
                       R_pad, a.out);
#endif
  } else if (a.part) {
    // fused partial checksums on this kernel: FPTA_OPT_INTERP_WS 2, variant builds only (slower than the register
    // kernel on C3); the instance is not in the product library
#ifdef FPTA_DIAG_KERNELS
    hipLaunchKernelGGL(k_grid_interp_ws<true>, dim3((unsigned)grid), dim3(512), 0, st, a, band, (int32_t)tiles, R_pad,
                       a.out);
#else
    return hipErrorInvalidValue;
#endif
  } else
    hipLaunchKernelGGL(k_grid_interp_ws<false>, dim3((unsigned)grid), dim3(512), 0, st, a, band, (int32_t)tiles, R_pad,
                       a.out);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- k_grid_interp_psr
// Layouts with one small grid signal (C3: the common GWB, nf = 124 grid points per pulsar): a workgroup owns one
// pulsar x 64 realizations, makes that pulsar's grid in LDS and interpolates every chunk of the pulsar from it. No grid
// buffer: the DFT launch (which could not co-run beside the 247-VGPR fused-checksum interpolation and followed it) and
// the grid's HBM round trip (0.41 GB written and read back per C3 batch) are gone.
//  1. wave w, realizations r0 + 16 w + lr: the quarter-range DFT of k_grid_dft_mfma (one 32-row block: nf <= 124) with
//     the same MFMA k-steps per parity (B = one realization's (cos, sin) coefficients per lane instead of a tile pair)
//     and the same butterfly into LDS rows j, H + j, H - j, nf - j: the grid values are k_grid_dft_mfma's, bit for bit;
//  2. one barrier; wave w takes the pulsar's partial groups w, w + 4, ... (chunks without partial checksums) and runs
//     k_grid_interp_mfma's MFMA steps at RW = 4 (64 realizations): A = two ds_read_b128 of a grid row, B = weights
//     from global memory, the next chunk's loaded before this chunk's stores; its grid-row indices come by scalar loads.
// The same operands in the same order as the two-kernel path: blocks and partial checksums are bit-identical to it.
constexpr int kPsrPitch = 66;   // doubles per LDS grid row: 64 realizations + 16 B (row starts 4 banks apart)
constexpr int kPsrMaxNf = 124;  // one quarter-range DFT block of 32 rows
template <bool PART, int NQ>
__global__ __launch_bounds__(256, 2) void k_grid_interp_psr(SynthArgs a, GridBand band, GridSegDev gs,
                                                            const int32_t* __restrict__ psr_grp, int32_t n_rb,
                                                            int32_t n_items, int32_t R_pad, double* __restrict__ out) {
  constexpr int RW = 4;
  extern __shared__ __attribute__((aligned(16))) double glds[];  // [nf][kPsrPitch]
  const int per = (n_items + 7) >> 3;
  const int item = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // a pulsar's blocks on one XCD
  if (item >= n_items) return;  // the whole workgroup, before its barrier
  const int p = item / n_rb, rb = item - p * n_rb;
  const int r0 = rb * 64;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int nf = gs.nf;
  {
    // 1. grid rows of pulsar p, realizations r0 + 16 wave + lr
    d4 C[2][2], S[2][2];  // [parity: 0 odd k, 1 even k][row tile h: rows 2 i + h]
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) C[q][h] = S[q][h] = d4{0.0, 0.0, 0.0, 0.0};
    const double* __restrict__ cb = a.coef + ((int64_t)p * a.K + gs.col0) * R_pad + r0 + 16 * wave + lr;
    const double* __restrict__ t0 = gs.tq + (int64_t)lg * gs.ldq + 2 * lr;
    const int64_t tstride = (int64_t)gs.ntq * gs.ldq;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int n = par ? gs.nm >> 1 : (gs.nm + 1) >> 1;
      const double* __restrict__ tc = t0 + 2 * par * tstride;
      const double* __restrict__ ts = tc + tstride;
      const int nq = ((n + 7) >> 3) << 1;
      for (int q = 0; q < nq; ++q) {
        const int m = 2 * min(4 * q + lg, n - 1) + par;  // clamped: a finite coefficient against a zero table row
        const double bc = cb[(int64_t)(2 * m) * R_pad], bs = cb[(int64_t)(2 * m + 1) * R_pad];
        const dbl2 ac = *(const dbl2*)(tc + (int64_t)(4 * q) * gs.ldq), as = *(const dbl2*)(ts + (int64_t)(4 * q) * gs.ldq);
        C[par][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac.x, bc, C[par][0], 0, 0, 0);
        C[par][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac.y, bc, C[par][1], 0, 0, 0);
        S[par][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(as.x, bs, S[par][0], 0, 0, 0);
        S[par][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(as.y, bs, S[par][1], 0, 0, 0);
      }
    }
    const int Q = nf >> 2, H = nf >> 1;
    double* __restrict__ gcol = glds + 16 * wave + lr;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = 2 * (lg + 4 * g) + h;
        if (j > Q) continue;
        const double oc = C[0][h][g], os = S[0][h][g], ec = C[1][h][g], es = S[1][h][g];
        const double pe = ec + es, me = ec - es, po = oc + os, mo = oc - os;
        gcol[j * kPsrPitch] = pe + po;
        gcol[(H + j) * kPsrPitch] = pe - po;
        if (j > 0 && j < Q) {
          gcol[(H - j) * kPsrPitch] = me - mo;
          gcol[(nf - j) * kPsrPitch] = me + mo;
        }
      }
  }
  __syncthreads();
  // 2. the pulsar's chunks; a wave's sequence: groups g0 + wave, g0 + wave + 4, ..., each group's chunks in order
  const int g1 = ld_uniform(psr_grp + p + 1);
  int g = ld_uniform(psr_grp + p) + wave;
  if (g >= g1) return;
  auto group_chunks = [&](int gg, int& c0, int& c1) {
    if constexpr (PART) {
      c0 = ld_uniform(band.pgfirst + gg);
      c1 = ld_uniform(band.pgfirst + gg + 1);
    } else {
      c0 = gg;
      c1 = gg + 1;
    }
  };
  const int rowbase = p * nf;  // grid-buffer row of the pulsar's first grid point (one grid signal: rowoff 0)
  struct Ops {
    int4 ci;
    int nq;
    dbl2 b[NQ];
    int row[NQ];  // LDS row of band row 4 q + lg
  };
  auto load = [&](int c, Ops& o) {
    o.ci = ld_uniform4(band.chunks + c);
    o.nq = __builtin_amdgcn_readfirstlane(o.ci.w) >> 2;
    FPTA_DCHECK(o.nq <= NQ && o.nq > 0, "k_grid_interp_psr band steps", o.nq, NQ + 1);
    const int32_t* __restrict__ rt = band.rows + (int64_t)c * band.vmax;
    const double* __restrict__ wp = band.wd + ((int64_t)c * band.vmax + lg) * kGridTT + 2 * lr;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int qq = min(q, o.nq - 1);  // steps past nq re-load the last one (never used)
      const int4 r4 = ld_uniform4(rt + 4 * qq);
      o.row[q] = (lg == 0 ? r4.x : lg == 1 ? r4.y : lg == 2 ? r4.z : r4.w) - rowbase;
      FPTA_DCHECK(o.row[q] >= 0 && o.row[q] < nf, "k_grid_interp_psr grid row", o.row[q], nf);
      o.b[q] = *(const dbl2*)(wp + 4 * kGridTT * qq);
    }
  };
  int c0, c1;
  group_chunks(g, c0, c1);
  int c = c0;
  Ops cur, nxt;
  load(c, cur);
  double ps[RW / 2];
  d4 acc[2][RW];
  while (true) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < RW; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < cur.nq) {
        const double* __restrict__ gr = glds + cur.row[q] * kPsrPitch + 2 * lr;
        const dbl2 av0 = *(const dbl2*)gr, av1 = *(const dbl2*)(gr + 32);
        const dbl2 bv = cur.b[q];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av0.x, bv.x, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av0.y, bv.x, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av0.x, bv.y, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av0.y, bv.y, acc[1][1], 0, 0, 0);
        acc[0][2] = __builtin_amdgcn_mfma_f64_16x16x4f64(av1.x, bv.x, acc[0][2], 0, 0, 0);
        acc[0][3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av1.y, bv.x, acc[0][3], 0, 0, 0);
        acc[1][2] = __builtin_amdgcn_mfma_f64_16x16x4f64(av1.x, bv.y, acc[1][2], 0, 0, 0);
        acc[1][3] = __builtin_amdgcn_mfma_f64_16x16x4f64(av1.y, bv.y, acc[1][3], 0, 0, 0);
      }
    }
    InterpTile<RW> t;
    t.c = c;
    t.p = p;
    t.r0 = r0;
    t.y = cur.ci.y;
    t.cnt = cur.ci.z;
    t.nq = cur.nq;
    t.pg = g;
    t.pfirst = c == c0;
    t.plast = c + 1 == c1;
    // next chunk: its operands are in flight before this chunk's stores enter the vmcnt queue
    bool more = true;
    if (c + 1 < c1) {
      ++c;
    } else {
      g += 4;
      more = g < g1;
      if (more) {
        group_chunks(g, c0, c1);
        c = c0;
      }
    }
    if (more) load(c, nxt);
    __builtin_amdgcn_sched_barrier(0);
    interp_store<PART, RW>(a, out, t, acc, ps);
    if (!more) break;
    cur = nxt;
  }
}

hipError_t launch_grid_interp_psr(hipStream_t st, const SynthArgs& a, const GridBand& band, const GridSegDev& gs,
                                  const int32_t* psr_grp, int32_t P, int32_t R_pad) {
  if (band.n_chunks <= 0 || band.vmax < 4 || band.vmax % 4 != 0 || band.vmax > 32 || R_pad % 64 != 0 || a.w_on ||
      gs.nf > kPsrMaxNf || gs.nf < 4 || gs.nf % 4 != 0 || gs.ldq != kGridDftRows || gs.nm <= 0 || !psr_grp ||
      (a.part && (!band.pgfirst || band.n_pg <= 0)))
    return hipErrorInvalidValue;
  const int32_t n_rb = R_pad / 64;
  const int64_t items = (int64_t)P * n_rb;
  if (items > 0x7FFFFFFF) return hipErrorInvalidValue;
  const int64_t grid = (items + 7) / 8 * 8;
  const size_t lds = sizeof(double) * (size_t)gs.nf * kPsrPitch;
  const bool small = band.vmax <= 16;
  auto kernel = a.part ? (small ? k_grid_interp_psr<true, 4> : k_grid_interp_psr<true, 8>)
                       : (small ? k_grid_interp_psr<false, 4> : k_grid_interp_psr<false, 8>);
  hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(256), lds, st, a, band, gs, psr_grp, n_rb, (int32_t)items,
                     R_pad, a.out);
  return hipGetLastError();
}

static_assert(16 * kDftMJ == kGridDftRows, "grid_build sizes grids to whole DFT row blocks");

hipError_t launch_grid_dft_mfma(hipStream_t st, GridSegs gsegs, int32_t P, const double* coef, int32_t K,
                                int32_t R_pad) {
  if (R_pad % (16 * kDftMR) != 0 || gsegs.n <= 0 || gsegs.n > kGridMaxSeg) return hipErrorInvalidValue;
  int64_t gz = 0;
  for (int s = 0; s < gsegs.n; ++s) {
    GridSegDev& g = gsegs.s[s];
    if (g.nf % 4 != 0 || !g.tq) return hipErrorInvalidValue;  // quarter-range tables
    g.nblk = (g.nf / 4 + 16 * kDftMJ) / (16 * kDftMJ);  // ceil((nf / 4 + 1) / (16 MJ))
    if (g.ldq < g.nblk * 16 * kDftMJ || g.ntq < ((((g.nm + 1) >> 1) + 7) & ~7)) return hipErrorInvalidValue;
    gz += g.nblk;
  }
  const int64_t n_xb = (R_pad + 64 * kDftMR - 1) / (64 * kDftMR);
  const int64_t n_tiles = n_xb * P;
  const int64_t blocks = (n_tiles + 7) / 8 * 8 * gz;  // 8 tiles (one per XCD) x gz row blocks per group of slots
  if (gz > 65535 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_grid_dft_mfma<kDftMJ, kDftMR>), dim3((unsigned)blocks), dim3(256), 0, st, gsegs, coef, K,
                     R_pad, (int32_t)n_xb, P, (int32_t)gz);
  return hipGetLastError();
}

hipError_t launch_grid_interp_mfma(hipStream_t st, const SynthArgs& a, const GridBand& band, int32_t R_pad) {
  constexpr int RW = kInterpRW;
  if (band.n_chunks <= 0 || band.vmax < 4 || band.vmax % 4 != 0 || R_pad % (16 * RW) != 0)
    return hipErrorInvalidValue;
  if (a.part && (!band.pgfirst || band.n_pg <= 0)) return hipErrorInvalidValue;
  const int32_t n_rb = (R_pad + 64 * RW - 1) / (64 * RW);
  const int64_t tiles = (int64_t)(a.part ? band.n_pg : band.n_chunks) * n_rb;  // work items (TileWalk)
  if (tiles > 0x7FFFFFFF) return hipErrorInvalidValue;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
  // persistent grid: kInterpWPC workgroups per CU (16-TOA tiles, profiles/r01_sweep_interp_wpc.txt: 1 -> 1.06 ms,
  // 2 -> 0.74, 3 -> 0.81; 32-TOA tiles: profiles/r02_interp_variants.txt)
  const int64_t want = (int64_t)n_cu * (a.w_on ? FPTA_WHITE_WPC : kInterpWPC);
  const int64_t grid = std::min<int64_t>((tiles + 7) / 8 * 8, (want + 7) / 8 * 8);
  // partial checksums are a separate instantiation: their reduce-scatter registers never weigh on the plain kernel
  auto kernel = a.w_on ? (a.part ? k_grid_interp_mfma<true, true, RW> : k_grid_interp_mfma<true, false, RW>)
                       : (a.part ? k_grid_interp_mfma<false, true, RW> : k_grid_interp_mfma<false, false, RW>);
  hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(256), 0, st, a, band, (int32_t)tiles, R_pad, a.out);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------- k_mix_mfma
// ORF mixing of a common signal on the fp64 matrix cores (large arrays, P >= kMixTiledMinP):
//   C[p][m] = sum_q L[p][q] Z[q][m],  m = jc R_pad + r (jc = 2 mode + cos/sin), coef[p][col0 + jc][r] = amp C,
// A = L (pulsar, q) from the zero-padded transpose L^T, B = Z (q, column), D[pulsar][column]. Both operands come
// in tile pairs from one 16-byte load: lane (lr, lg) loads L^T[q][p0 + 32 u + 2 lr .. + 1] (.x pulsar tile 2u,
// .y tile 2u + 1) and Z[q][m0 + 32 b + 2 lr .. + 1] (.x column tile 2b, .y tile 2b + 1) for q = q0 + lg. D of
// (pulsar tile 2u + e, column tile 2b + h): lane (lr, lg) register g = pulsar p0 + 32 u + 2 (lg + 4 g) + e,
// column m0 + 32 b + 2 lr + h, so one 16-byte store per (lane, pulsar) writes 256 contiguous bytes of a
// coefficient row. Wave tile 32 NU pulsars x 32 NB columns; workgroup = 4 waves along the columns.
// Grid: every pulsar tile of a column block runs on one XCD (block b: XCD b % 8), so the block's Z columns
// (P x 256 doubles) are read from HBM once and served to the other pulsar tiles from that XCD's L2. A lower-
// triangular factor (Cholesky of a positive-definite ORF) stops the q loop at the tile's last pulsar.
// o + (a v0, a v1) with the products rounded before the add (-ffp-contract=fast ignores contract pragmas), as
// k_coef_merge adds the stored coefficients a v: a block is bit-identical whichever of the two sums it
__device__ __forceinline__ dbl2 add_rounded_product(dbl2 o, double a, double v0, double v1) {
  double t0 = a * v0, t1 = a * v1;
  asm volatile("" : "+v"(t0), "+v"(t1));  // an opaque value: the add cannot fuse with the multiply
  return dbl2{o.x + t0, o.y + t1};
}

// OCC waves per SIMD: the small-array instance (<2, 1, 3>, 168 VGPRs) fits beside the warp-specialised interpolation
// of the previous block (2 x 168), so pipelined blocks' mixing co-runs with it instead of waiting for it.
template <int NU, int NB, int OCC>
__global__ __launch_bounds__(256, OCC) void k_mix_mfma(const double* __restrict__ LT, int32_t lt_ld,
                                                     const double* __restrict__ amp, int32_t P, int64_t M,
                                                     int32_t R_pad, int32_t lower, int32_t n_q, int32_t n_pt,
                                                     int32_t n_cb,
                                                     const double* __restrict__ zbuf, double* __restrict__ coef,
                                                     int32_t K, int32_t col0, double* __restrict__ x_out,
                                                     int32_t add_into) {
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int cb = (slot / n_pt) * 8 + xcd;
  const int pt = slot - (slot / n_pt) * n_pt;
  if (cb >= n_cb) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int p0 = pt * 32 * NU;
  const int64_t m0 = ((int64_t)cb * 4 + wave) * 32 * NB;
  const int qend = min(lower ? min(P, p0 + 32 * NU) : P, n_q);
  d4 acc[2 * NU][2 * NB];
#pragma unroll
  for (int u = 0; u < 2 * NU; ++u)
#pragma unroll
    for (int i = 0; i < 2 * NB; ++i) acc[u][i] = d4{0.0, 0.0, 0.0, 0.0};
  struct Ops {
    dbl2 a[NU], b[NB];
  };
  // q rows past P: L^T rows are zero there (padding); Z's row is clamped to P - 1 (finite x 0)
  auto load = [&](int q0, Ops& o) {
    const int q = q0 + lg;
    const double* __restrict__ lt = LT + (int64_t)q * lt_ld + p0 + 2 * lr;
#pragma unroll
    for (int u = 0; u < NU; ++u) o.a[u] = *(const dbl2*)(lt + 32 * u);
    const double* __restrict__ z = zbuf + (int64_t)min(q, P - 1) * M + m0 + 2 * lr;
#pragma unroll
    for (int b = 0; b < NB; ++b) o.b[b] = *(const dbl2*)(z + 32 * b);
  };
  auto mfma = [&](const Ops& o) {
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        acc[2 * u][2 * b] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a[u].x, o.b[b].x, acc[2 * u][2 * b], 0, 0, 0);
        acc[2 * u][2 * b + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a[u].x, o.b[b].y, acc[2 * u][2 * b + 1], 0, 0, 0);
        acc[2 * u + 1][2 * b] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.a[u].y, o.b[b].x, acc[2 * u + 1][2 * b], 0, 0, 0);
        acc[2 * u + 1][2 * b + 1] =
            __builtin_amdgcn_mfma_f64_16x16x4f64(o.a[u].y, o.b[b].y, acc[2 * u + 1][2 * b + 1], 0, 0, 0);
      }
  };
  Ops o0, o1;
  load(0, o0);
  for (int q0 = 0; q0 < qend; q0 += 8) {
    load(q0 + 4, o1);
    mfma(o0);
    load(q0 + 8, o0);
    if (q0 + 4 < qend) mfma(o1);
  }
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int p = p0 + 32 * u + 2 * (lg + 4 * g) + e;
        if (p >= P) continue;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const int64_t m = m0 + 32 * b + 2 * lr;  // columns m, m + 1 share jc (R_pad is even)
          const int jc = (int)(m / R_pad);
          const int r = (int)(m - (int64_t)jc * R_pad);
          const double a = amp[jc >> 1];
          const double v0 = acc[2 * u + e][2 * b][g], v1 = acc[2 * u + e][2 * b + 1][g];
          double* dst = coef + ((int64_t)p * K + col0 + jc) * R_pad + r;
          if (add_into) {  // into a coalesced grid signal's anchor columns
            const dbl2 o = *(const dbl2*)dst;
            *(dbl2*)dst = add_rounded_product(o, a, v0, v1);
          } else {
            *(dbl2*)dst = dbl2{a * v0, a * v1};
          }
          if (x_out) *(dbl2*)(x_out + (int64_t)p * M + m) = dbl2{v0, v1};
        }
      }
}

// k_gen_mix: draw + ORF mixing of a common signal in one kernel (arrays of kMixTiledMinP .. kGenMixMaxP pulsars). A
// workgroup owns mode k and 32 realizations r0 .. r0 + 31: its threads draw z[q][cos | sin][r] for every pulsar q with
// k_gen's counter {k, q, signal, realization} (the same draws) into LDS, then wave (pulsar tile u, column half h)
// computes coef[p][col0 + 2 k + h][r] = amp[k] sum_q L[p][q] z[q][h][r] for its 64 pulsars on fp64 MFMA (A = L from
// the zero-padded L^T, 16-byte pairs of pulsar tiles; B = z from LDS, 16-byte pairs of realization tiles), as
// k_mix_mfma does: the same products, summed in the same k-step order, stored as the rounded product amp * sum.
// The zbuf round trip (write + read of P x 2 N x R doubles) and a launch are gone.

// RH realization tiles of 16 per wave (RH = 2: waves (u, h) over 32 realizations; RH = 1: twice the waves, each on
// 16 realizations, so a workgroup's draws and MFMA steps spread over 8 waves per 64-pulsar tile pair). The products
// and their k-step order per coefficient are the same either way.
// RB realizations per workgroup (32, or 16 with RH = 1: a quarter of the LDS, 27 KB at P = 100, FPTA_OPT_GEN_MIX 3)
template <int RH, int RB>
__global__ __launch_bounds__(1024) void k_gen_mix(SegDesc sd, int32_t seg_id, int32_t P, int32_t n_real, int32_t R_pad,
                                                  int64_t real0, uint32_t k0, uint32_t k1, double* __restrict__ coef,
                                                  int32_t K) {
  static_assert(RB == 32 || (RB == 16 && RH == 1), "16-realization workgroups: one realization tile per wave");
  extern __shared__ __attribute__((aligned(16))) double Zs[];  // [q_pad][2 RB]: cos of RB realizations, then sin
  const int n_rb = R_pad / RB;
  const int k = blockIdx.x / n_rb, r0 = (blockIdx.x - k * n_rb) * RB;
  const int q_pad = (P + 7) & ~7;  // k-steps of 4 in pairs: the last step may read up to 8 rows past P
  for (int idx = threadIdx.x; idx < q_pad * (RB / 2); idx += blockDim.x) {  // a realization pair per thread and pulsar
    const int q = idx / (RB / 2), rl = 2 * (idx % (RB / 2));
    double z[4] = {0.0, 0.0, 0.0, 0.0};
    const int r = r0 + rl;
    if (q < sd.n_q && r < n_real) {  // columns q >= n_q of L are zero: their normals are never needed
      const uint64_t g = (uint64_t)(real0 + r);
      if ((g & 1) == 0) {
        gp_pair2((uint32_t)k, (uint32_t)q, (uint32_t)seg_id, g, k0, k1, z);
      } else {
        gp_normal2((uint32_t)k, (uint32_t)q, (uint32_t)seg_id, g, k0, k1, z[0], z[1]);
        gp_normal2((uint32_t)k, (uint32_t)q, (uint32_t)seg_id, g + 1, k0, k1, z[2], z[3]);
      }
      if (r + 1 >= n_real) z[2] = z[3] = 0.0;
    }
    *(dbl2*)(Zs + q * 2 * RB + rl) = dbl2{z[0], z[2]};
    *(dbl2*)(Zs + q * 2 * RB + RB + rl) = dbl2{z[1], z[3]};
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int NRH = RB / 16 / RH;  // realization tiles of 16 RH per (u, h)
  const int rh = wave % NRH, uh = wave / NRH;
  const int u = uh >> 1, h = uh & 1;  // pulsar tile (64 pulsars), column half (cos / sin)
  const int p0 = 64 * u;
  const int qend = min(sd.l_lower ? min(P, p0 + 64) : P, sd.n_q);
  d4 acc[4][RH];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < RH; ++e) acc[i][e] = d4{0.0, 0.0, 0.0, 0.0};
  const double* __restrict__ lt = sd.LT + p0 + 2 * lr;
  // B operand of realization tile e: RH = 2 realizations 2 lr + e (one 16-byte pair); RH = 1 realization 16 rh + lr
  const double* __restrict__ zb = Zs + RB * h + (RH == 2 ? 2 * lr : 16 * rh + lr);
  auto step = [&](int q0) {
    const int q = q0 + lg;
    const dbl2 a0 = *(const dbl2*)(lt + (int64_t)q * sd.lt_ld);
    const dbl2 a1 = *(const dbl2*)(lt + (int64_t)q * sd.lt_ld + 32);
    double b[RH];
    if constexpr (RH == 2) {
      const dbl2 bv = *(const dbl2*)(zb + q * 2 * RB);
      b[0] = bv.x;
      b[1] = bv.y;
    } else {
      b[0] = zb[q * 2 * RB];
    }
#pragma unroll
    for (int e = 0; e < RH; ++e) {
      acc[0][e] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.x, b[e], acc[0][e], 0, 0, 0);
      acc[1][e] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0.y, b[e], acc[1][e], 0, 0, 0);
      acc[2][e] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.x, b[e], acc[2][e], 0, 0, 0);
      acc[3][e] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1.y, b[e], acc[3][e], 0, 0, 0);
    }
  };
  for (int q0 = 0; q0 < qend; q0 += 4) step(q0);
  // D of (pulsar tile 2v + e', realization tile): lane (lr, lg) register g = pulsar p0 + 32 v + 2 (lg + 4 g) + e'
  const double a = sd.amp[k];
  const int jc = 2 * k + h;
#pragma unroll
  for (int v = 0; v < 2; ++v)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int p = p0 + 32 * v + 2 * (lg + 4 * g) + e;
        if (p >= P) continue;
        double* dst = coef + ((int64_t)p * K + sd.col0 + jc) * R_pad + r0;
        if constexpr (RH == 2) {  // realizations 2 lr, 2 lr + 1: one 16-byte store
          *(dbl2*)(dst + 2 * lr) = dbl2{a * acc[2 * v + e][0][g], a * acc[2 * v + e][1][g]};
        } else {
          dst[16 * rh + lr] = a * acc[2 * v + e][0][g];
        }
      }
}

hipError_t launch_gen_mix(hipStream_t st, const SegDesc& sd, int32_t seg_id, int32_t P, int32_t n_real, int32_t R_pad,
                          int64_t real0, uint32_t k0, uint32_t k1, double* coef, int32_t K, int rh, int rb,
                          hipEvent_t ev0, hipEvent_t ev1) {
  const int32_t n_pt = (P + 63) / 64;
  if (sd.kind != 1 || !sd.LT || P < 1 || P > kGenMixMaxP || R_pad % 32 != 0 || sd.lt_ld < 64 * n_pt ||
      sd.lt_rows < ((P + 7) & ~7) || sd.col0 < 0 || sd.col0 + 2 * sd.nm > K || (rh != 1 && rh != 2) ||
      (rb != 32 && (rb != 16 || rh != 1)))
    return hipErrorInvalidValue;
  const int64_t blocks = (int64_t)sd.nm * (R_pad / rb);
  if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
  const size_t lds = sizeof(double) * 2 * rb * (size_t)((P + 7) & ~7);
  if (rb == 16)
    hipExtLaunchKernelGGL((k_gen_mix<1, 16>), dim3((unsigned)blocks), dim3(128 * n_pt), (uint32_t)lds, st, ev0, ev1, 0u,
                          sd, seg_id, P, n_real, R_pad, real0, k0, k1, coef, K);
  else if (rh == 2)
    hipExtLaunchKernelGGL((k_gen_mix<2, 32>), dim3((unsigned)blocks), dim3(128 * n_pt), (uint32_t)lds, st, ev0, ev1, 0u,
                          sd, seg_id, P, n_real, R_pad, real0, k0, k1, coef, K);
  else
    hipExtLaunchKernelGGL((k_gen_mix<1, 32>), dim3((unsigned)blocks), dim3(256 * n_pt), (uint32_t)lds, st, ev0, ev1, 0u,
                          sd, seg_id, P, n_real, R_pad, real0, k0, k1, coef, K);
  return hipGetLastError();
}

template <int NU, int NB, int OCC>
hipError_t launch_mix_mfma_t(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                             double* coef, int32_t K, double* x_out, int32_t acc_col0) {
  const int64_t M = (int64_t)2 * sd.nm * R_pad;  // a multiple of 256: R_pad is a multiple of 128
  constexpr int kCols = 4 * 32 * NB, kRows = 32 * NU;
  if (P <= 0 || !sd.LT || M % kCols != 0) return hipErrorInvalidValue;
  const int64_t n_cb = M / kCols;
  const int32_t n_pt = (P + kRows - 1) / kRows;
  // operand loads stay inside L^T: pulsar columns up to n_pt * kRows, q rows up to the last k-step's + 4
  if (sd.lt_ld < n_pt * kRows || sd.lt_rows < (P + 7) / 8 * 8 + 4) return hipErrorInvalidValue;
  const int64_t blocks = (n_cb + 7) / 8 * 8 * n_pt;
  if (blocks > 0x7FFFFFFF || n_cb > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_mix_mfma<NU, NB, OCC>), dim3((unsigned)blocks), dim3(256), 0, st, sd.LT, sd.lt_ld, sd.amp, P,
                     M, R_pad, sd.l_lower, std::max(1, std::min(sd.n_q, P)), n_pt, (int32_t)n_cb, zbuf, coef, K,
                     acc_col0 >= 0 ? acc_col0 : sd.col0,
                     x_out, acc_col0 >= 0 ? 1 : 0);
  return hipGetLastError();
}

// Wave tile 64 pulsars x 64 columns at 2 waves per SIMD for large arrays (C4: the mix is a kernel of its own);
// 64 x 32 at 3 waves per SIMD for small ones, whose mixing co-runs with the previous block's interpolation.
#ifndef FPTA_MIX_LARGE_P
#define FPTA_MIX_LARGE_P 256
#endif
constexpr int kMixLargeP = FPTA_MIX_LARGE_P;

hipError_t launch_mix_mfma(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                           double* coef, int32_t K, double* x_out, int32_t acc_col0) {
  if (acc_col0 >= 0 && (x_out || acc_col0 + 2 * sd.nm > K)) return hipErrorInvalidValue;
  return P >= kMixLargeP ? launch_mix_mfma_t<2, 2, 2>(st, sd, P, R_pad, zbuf, coef, K, x_out, acc_col0)
                         : launch_mix_mfma_t<2, 1, 3>(st, sd, P, R_pad, zbuf, coef, K, x_out, acc_col0);
}

// ----------------------------------------------------------------------------- partial checksums
// Two fixed-order passes over the interpolation's partial rows: segment s of kPartSegs sums rows
// [s L, (s + 1) L) per realization, then the segments are summed in order. Threads run over realizations, so
// every pass reads consecutive 16-byte {sum, sumsq} pairs.
__global__ __launch_bounds__(256) void k_part_reduce(const double* __restrict__ part, int32_t n_rows, int32_t R_pad,
                                                     int32_t L, double* __restrict__ tmp) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= R_pad) return;
  const int s = blockIdx.y;
  const int c1 = min(n_rows, (s + 1) * L);
  double a = 0.0, b = 0.0;
#pragma unroll 8
  for (int c = s * L; c < c1; ++c) {
    const dbl2 v = *(const dbl2*)(part + ((int64_t)c * R_pad + r) * 2);
    a += v.x;
    b += v.y;
  }
  *(dbl2*)(tmp + ((int64_t)s * R_pad + r) * 2) = dbl2{a, b};
}

// 64-thread workgroups: C3's 4096 realizations make 64 of them (16 of 256 threads sat on a few CUs beside the next
// block's draws, 0.074 ms)
__global__ __launch_bounds__(64) void k_part_final(const double* __restrict__ tmp, int32_t n_seg, int32_t R_pad,
                                                   int32_t n_real, double* __restrict__ sums) {
  const int r = blockIdx.x * 64 + threadIdx.x;
  if (r >= n_real) return;
  double a = 0.0, b = 0.0;
#pragma unroll 8
  for (int s = 0; s < n_seg; ++s) {
    const dbl2 v = *(const dbl2*)(tmp + ((int64_t)s * R_pad + r) * 2);
    a += v.x;
    b += v.y;
  }
  sums[2 * r] = a;
  sums[2 * r + 1] = b;
}

// One pass for up to kPartOneRows rows: a workgroup is 16 realizations x kPartOneSegs row segments; thread (ri, s) sums
// rows [s L, (s + 1) L) of realization 16 b + ri in order, and the segment sums are added in segment order through
// LDS. A wave's load reads four 256-byte runs. One launch instead of two beside the streamed job's next block.
__global__ __launch_bounds__(256) void k_part_sums(const double* __restrict__ part, int32_t n_rows, int32_t R_pad,
                                                   int32_t L, int32_t n_real, double* __restrict__ sums) {
  static_assert(16 * kPartOneSegs == 256, "16 realizations x kPartOneSegs segments per workgroup");
  __shared__ dbl2 seg[kPartOneSegs][16];
  const int ri = threadIdx.x & 15, s = threadIdx.x >> 4;
  const int r = blockIdx.x * 16 + ri;
  double a = 0.0, b = 0.0;
  if (r < R_pad) {
    const int c1 = min(n_rows, (s + 1) * L);
#pragma unroll 8
    for (int c = s * L; c < c1; ++c) {
      const dbl2 v = *(const dbl2*)(part + ((int64_t)c * R_pad + r) * 2);
      a += v.x;
      b += v.y;
    }
  }
  seg[s][ri] = dbl2{a, b};
  __syncthreads();
  if (s == 0 && r < n_real) {
    double x = 0.0, y = 0.0;
#pragma unroll
    for (int k = 0; k < kPartOneSegs; ++k) {
      x += seg[k][ri].x;
      y += seg[k][ri].y;
    }
    *(dbl2*)(sums + 2 * (int64_t)r) = dbl2{x, y};
  }
}

hipError_t launch_part_checksums(hipStream_t st, const double* part, int32_t n_rows, int32_t R_pad, int32_t n_real,
                                 double* tmp, double* sums) {
  if (n_rows <= 0 || n_real <= 0 || n_real > R_pad) return hipErrorInvalidValue;
  if (n_rows <= kPartOneRows) {
    const int32_t L1 = (n_rows + kPartOneSegs - 1) / kPartOneSegs;
    hipLaunchKernelGGL(k_part_sums, dim3((unsigned)((n_real + 15) / 16)), dim3(256), 0, st, part, n_rows, R_pad, L1,
                       n_real, sums);
    return hipGetLastError();
  }
  const int32_t L = (n_rows + kPartSegs - 1) / kPartSegs;
  const int32_t n_seg = (n_rows + L - 1) / L;
  hipLaunchKernelGGL(k_part_reduce, dim3((unsigned)((R_pad + 255) / 256), (unsigned)n_seg), dim3(256), 0, st, part,
                     n_rows, R_pad, L, tmp);
  hipLaunchKernelGGL(k_part_final, dim3((unsigned)((n_real + 63) / 64)), dim3(64), 0, st, tmp, n_seg, R_pad, n_real,
                     sums);
  return hipGetLastError();
}

#ifdef FPTA_DIAG_KERNELS
#include "diag/interp_lds.inc"
#include "diag/interp_st.inc"
#include "diag/interp_u.inc"
#include "diag/interp_wr.inc"
#endif

}  // namespace fpta
