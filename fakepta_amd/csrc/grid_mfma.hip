// Gridded synthesis (grid.hip) on the fp64 matrix cores: both per-batch GEMMs of the factorisation
// F ~= W E as v_mfma_f64_16x16x4_f64 chains.
//
//   k_grid_dft_mfma     grid values G[p][j][r] (half-range real DFT, both grid halves per pass)
//   k_grid_interp_mfma  residuals out[r][t] = sum_s sum_i W_s[t][i] G_s[J + i][r] (+ white / ECORR)
//
// Fragment maps of v_mfma_f64_16x16x4_f64 (cdna_hip_programming.md §3): A[i = l & 15][k = l >> 4],
// B[k = l >> 4][j = l & 15], D: col = l & 15, row = (l >> 4) + 4 reg.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "fpta_internal.h"
#include "philox.h"

namespace fpta {

typedef double dbl2 __attribute__((ext_vector_type(2)));

// k_grid_interp_mfma: 32 TOAs x 16 kInterpRW realizations per wave, kInterpWPC persistent workgroups per CU
// (compile-time; tools/interp_variants.sh builds the alternatives it measures into build/diag)
#ifndef FPTA_INTERP_RW
#define FPTA_INTERP_RW 8
#endif
#ifndef FPTA_INTERP_WPC
#define FPTA_INTERP_WPC 2
#endif
#ifndef FPTA_INTERP_DIAG
#define FPTA_INTERP_DIAG 0  // 0 in every product build
#endif
constexpr int kInterpRW = FPTA_INTERP_RW;
constexpr int kInterpWPC = FPTA_INTERP_WPC;

// ----------------------------------------------------------------------------- k_grid_dft_mfma
// Per pulsar two GEMMs sharing the output tile (4 modes per MFMA):
//   Cj[j][r] = sum_k ecos[k][j] c_k[r],  Sj[j][r] = sum_k esin[k][j] s_k[r],
//   g_j = Cj + Sj, g_{nf - j} = Cj - Sj (cos even, sin odd in j).
// A = table (grid row, mode), B = coefficients (mode, realization). Both operands come in tile pairs from one
// 16-byte load per lane: lane (lr, lg) loads table rows 2 lr, 2 lr + 1 (.x row tile 2u, .y row tile 2u + 1) and
// realizations 2 lr, 2 lr + 1 (.x realization tile 2m, .y tile 2m + 1), so a 4-mode step issues MJ + MR loads
// for 2 MJ MR MFMAs (the one-double-per-lane version issued one load per MFMA and was address-unit bound).
// D of (row tile 2u + h, realization tile 2m + e): lane (lr, lg) register g holds grid row
// j0 + 32 u + 2 (lg + 4 g) + h, realization r0 + 32 m + 2 lr + e, so the two realization tiles of a pair store
// one 16-byte value per lane (256-byte runs per grid row). Wave tile 16 MJ rows x 16 MR realizations. The table
// is zero-padded to ntab (multiple of 8) modes and lde (multiple of 16 MJ) rows; padded coefficient modes
// re-read the signal's last mode (finite) against zero table rows.
template <int MJ, int MR>
__global__ __launch_bounds__(256, 2) void k_grid_dft_mfma(GridSegs gsegs, const double* __restrict__ coef,
                                                          int32_t K, int32_t R_pad) {
  static_assert(MJ % 2 == 0 && MR % 2 == 0, "operands come in tile pairs");
  constexpr int PJ = MJ / 2, PR = MR / 2;
  int bz = blockIdx.z, s = 0;
  while (s + 1 < gsegs.n && bz >= gsegs.s[s].nblk) bz -= gsegs.s[s++].nblk;
  const GridSegDev& gs = gsegs.s[s];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int r0 = (blockIdx.x * 4 + wave) * 16 * MR;
  if (r0 >= R_pad) return;
  const int p = blockIdx.y;
  const int j0 = bz * 16 * MJ;
  const double* __restrict__ cp = coef + ((int64_t)p * K + gs.col0 + 2 * lg) * R_pad + r0 + 2 * lr;
  const double* __restrict__ ec = gs.ecos + (int64_t)lg * gs.lde + j0 + 2 * lr;
  const double* __restrict__ es = gs.esin + (int64_t)lg * gs.lde + j0 + 2 * lr;
  d4 C[MJ][MR], S[MJ][MR];
#pragma unroll
  for (int u = 0; u < MJ; ++u)
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      C[u][i] = d4{0.0, 0.0, 0.0, 0.0};
      S[u][i] = d4{0.0, 0.0, 0.0, 0.0};
    }
  const int nq = ((gs.nm + 7) >> 3) << 1;  // even: the table has ntab >= nm rounded up to 8 modes (zero rows)
  // operands of k-step q; the coefficient row is clamped to the signal's last mode (a valid, finite value
  // that meets a zero table row), so every load is unconditional and the next step's loads stay in
  // flight across the current step's MFMAs. Two operand sets alternate (unrolled by 2: no register
  // copies, which would wait on the prefetch).
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
  auto load = [&](int qq, Ops& o) {
    const int m = min(4 * qq + lg, gs.nm - 1) - lg;  // mode of lane group 0 (clamped)
    const double* __restrict__ cq = cp + (int64_t)(2 * m) * R_pad;
    const int64_t eo = (int64_t)(4 * qq) * gs.lde;
#pragma unroll
    for (int i = 0; i < PR; ++i) {
      o.bc[i] = *(const dbl2*)(cq + 32 * i);
      o.bs[i] = *(const dbl2*)(cq + R_pad + 32 * i);
    }
#pragma unroll
    for (int u = 0; u < PJ; ++u) {
      o.ac[u] = *(const dbl2*)(ec + eo + 32 * u);
      o.as[u] = *(const dbl2*)(es + eo + 32 * u);
    }
  };
  Ops o0, o1;
  load(0, o0);
  for (int q = 0; q < nq; q += 2) {
    load(min(q + 1, nq - 1), o1);
    mfma(o0);
    load(min(q + 2, nq - 1), o0);
    mfma(o1);
  }
  double* __restrict__ gp = gs.g + (int64_t)p * gs.nf * R_pad + r0 + 2 * lr;
#pragma unroll
  for (int u = 0; u < PJ; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + 32 * u + 2 * (lg + 4 * g) + h;
#pragma unroll
        for (int i = 0; i < PR; ++i) {
          const double c0 = C[2 * u + h][2 * i][g], s0 = S[2 * u + h][2 * i][g];
          const double c1 = C[2 * u + h][2 * i + 1][g], s1 = S[2 * u + h][2 * i + 1][g];
          if (j <= gs.half) *(dbl2*)(gp + (int64_t)j * R_pad + 32 * i) = dbl2{c0 + s0, c1 + s1};
          if (j > 0 && 2 * j < gs.nf) *(dbl2*)(gp + (int64_t)(gs.nf - j) * R_pad + 32 * i) = dbl2{c0 - s0, c1 - s1};
        }
      }
}

// White-noise normals of (TOA t, global realizations g, g + 1 of the pair containing g): the
// realization-paired stream of oracle.white_normals_rpairs (same words as kernels.hip white_pair).
__device__ __forceinline__ void mfma_white_pair(int64_t t, int64_t g, uint32_t k0, uint32_t k1, double& z0,
                                                double& z1) {
  const u32x4 c = {(uint32_t)t, kWhitePsrWord, kWhiteStream, (uint32_t)(g >> 1)};
  box_muller(philox4x32_10(c, k0, k1), z0, z1);
}

// ----------------------------------------------------------------------------- k_grid_interp_mfma
// out[r][t] = sum_v W[chunk][v][tt] G[row(chunk, v)][r] over the chunk's band rows v < V: every signal's band
// back to back (host plan), so one flat loop of V / 4 MFMA steps covers all signals. Per step A = grid values
// (realization, row), B = weights (row, TOA):
//  * the grid rows of a step come from the chunk's row table with one scalar 16-byte load (4 rows, any
//    signal: each lane group loads its own row), so signals need no separate pipeline fill and the band is
//    padded to 4 rows once per chunk, not per signal;
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
// Wave tile = chunk x 16 RW realizations; the next step's operands are loaded before the current step's MFMAs
// (two register sets, unrolled by 2; the last prefetch re-reads the final step, the odd last step is skipped by
// a uniform branch).
template <bool WHITE, int RW>
__device__ __forceinline__ void interp_tile(const SynthArgs& a, const GridBand& band, int32_t R_pad,
                                            double* __restrict__ out, int tile) {
  static_assert(RW % 2 == 0, "realization tiles come in pairs");
  static_assert(kGridTT == 32, "two 16-TOA B-tiles per chunk");
  constexpr int NP = RW / 2;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int rb = __builtin_amdgcn_readfirstlane(tile / band.n_chunks);  // realization block of 64 RW
  const int c = __builtin_amdgcn_readfirstlane(tile - rb * band.n_chunks);
  const int r0 = (rb * 4 + wave) * 16 * RW;
  if (r0 >= R_pad) return;
  FPTA_DCHECK(r0 + 16 * RW <= R_pad, "k_grid_interp_mfma realization block", r0 + 16 * RW, R_pad + 1);
  const int4 ci = band.chunks[c];
  const int p = __builtin_amdgcn_readfirstlane(ci.x);
  const int nq = __builtin_amdgcn_readfirstlane(ci.w) >> 2;
  FPTA_DCHECK(4 * nq <= band.vmax, "k_grid_interp_mfma band rows", 4 * nq, band.vmax + 1);
  const int64_t base = a.offs[p];

  d4 acc[2][RW];  // [TOA parity][realization tile]
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int i = 0; i < RW; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};

  // the chunk's row table in registers: lane l holds band row l + 64 i in rr[i] (V <= kGridVMax = 256, host
  // plan); a step's rows then come from one ds_bpermute (no address-unit work, no vmcnt wait on the grid
  // prefetch). A per-step scalar load of the table compiled to a vector load + vmcnt(0) behind the epilogue's
  // stores.
  const int32_t* __restrict__ rt = band.rows + (int64_t)c * band.vmax;
  const int V = 4 * nq;
  int rr[kGridVMax / 64];
#pragma unroll
  for (int i = 0; i < kGridVMax / 64; ++i) rr[i] = rt[min(64 * i + lane, V - 1)];
  const double* __restrict__ G0 = band.g + r0 + 2 * lr;
  const double* __restrict__ Wp = band.wd + ((int64_t)c * band.vmax + lg) * kGridTT + 2 * lr;
  dbl2 a0[NP], a1[NP], b0, b1;
  auto row_of = [&](int qq) {  // grid row of this lane's k index in step qq
    const int blk = qq >> 4;     // 64-row block of the step's rows (uniform)
    const int src = blk == 0 ? rr[0] : (blk == 1 ? rr[1] : (blk == 2 ? rr[2] : rr[3]));
    return __builtin_amdgcn_ds_bpermute(((4 * qq + lg) & 63) << 2, src);
  };
  auto load = [&](int qq, int row, dbl2(&av)[NP], dbl2& bv) {
    FPTA_DCHECK(row >= 0 && row < band.grid_rows, "k_grid_interp_mfma grid row", row, band.grid_rows);
#if FPTA_INTERP_DIAG == 1  // diagnostic build only (tools/interp_variants.sh): every step reads one L1-resident row
    const double* __restrict__ gr = G0 + (int64_t)(row & 3) * R_pad;
#else
    const double* __restrict__ gr = G0 + (int64_t)row * R_pad;
#endif
#pragma unroll
    for (int m = 0; m < NP; ++m) av[m] = *(const dbl2*)(gr + 32 * m);
    bv = *(const dbl2*)(Wp + 4 * kGridTT * qq);
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
  // rows are looked up one step ahead of their loads, loads one step ahead of their MFMAs; the scheduling
  // barriers keep each step's loads issued before the MFMAs of the step before (else the first MFMA, hoisted
  // above them, waits for every outstanding load)
  int row1 = row_of(min(1, nq - 1));
  load(0, row_of(0), a0, b0);
  for (int q = 0; q < nq; q += 2) {
    const int row2 = row_of(min(q + 2, nq - 1));
    load(min(q + 1, nq - 1), row1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mfma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    row1 = row_of(min(q + 3, nq - 1));
    load(min(q + 2, nq - 1), row2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    if (q + 1 < nq) mfma(a1, b1);  // odd step count: skip the re-read last step (wave-uniform branch)
    __builtin_amdgcn_sched_barrier(0);
  }

  const int cnt = __builtin_amdgcn_readfirstlane(ci.z);
  const int tt = 2 * lr;  // this lane's even TOA in the chunk; tt + 1 the odd one
  if (tt >= cnt) return;
  const int64_t tg = base + ci.y + tt;
  if constexpr (WHITE) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (tt + e >= cnt) break;
      const int64_t te = tg + e;
      const double sg = a.w_sigma ? a.w_sigma[te] : 0.0;
      const int ep = a.w_block_of ? a.w_block_of[te] : -1;
      const double es = ep >= 0 ? a.w_esig[ep] : 0.0;
#pragma unroll
      for (int m = 0; m < NP; ++m) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int rl = r0 + 32 * m + 2 * (lg + 4 * g);  // batch index of acc[e][2m][g]; acc[e][2m + 1][g]: rl + 1
          double x0 = acc[e][2 * m][g], x1 = acc[e][2 * m + 1][g];
          if (a.w_sigma) {
            const int64_t g0 = a.real0 + rl;  // parity uniform over the launch (rl even)
            double z0, z1;
            mfma_white_pair(te, g0, a.k0, a.k1, z0, z1);
            if (g0 & 1) {  // (g0, g0 + 1) straddle two pairs
              double y0, y1;
              mfma_white_pair(te, g0 + 1, a.k0, a.k1, y0, y1);
              x0 = fma(sg, z1, x0);
              x1 = fma(sg, y0, x1);
            } else {
              x0 = fma(sg, z0, x0);
              x1 = fma(sg, z1, x1);
            }
          }
          if (ep >= 0) {
            if (rl < a.n_real) x0 = fma(es, a.w_zb[(int64_t)rl * a.w_nblocks + ep], x0);
            if (rl + 1 < a.n_real) x1 = fma(es, a.w_zb[(int64_t)(rl + 1) * a.w_nblocks + ep], x1);
          }
          acc[e][2 * m][g] = x0;
          acc[e][2 * m + 1][g] = x1;
        }
      }
    }
  }
  // one 16-byte store per (lane, realization) when both TOAs exist and the row offset r * ldo + tg keeps 16-byte
  // alignment (ldo and tg even), else the pair is stored as two 8-byte stores
#if FPTA_INTERP_DIAG == 2  // diagnostic build only: no stores (one conditional store keeps the sums live)
  if (acc[0][0][0] == 12345.678) out[tg] = acc[0][RW - 1][3] + acc[1][RW - 1][3];
  return;
#endif
  double* __restrict__ ocol = out + tg;
  const bool pair = tt + 1 < cnt;
  const bool vec = pair && ((((uintptr_t)ocol) | ((uintptr_t)a.ldo << 3)) & 15) == 0;
#pragma unroll
  for (int i = 0; i < RW; ++i) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int r = r0 + 32 * (i >> 1) + 2 * (lg + 4 * g) + (i & 1);
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

// Persistent launch: gridDim.x (a multiple of 8) workgroups, about as many as are co-resident; workgroup
// b runs on XCD b % 8 and walks that XCD's contiguous range of tiles (consecutive chunks: their grid rows
// overlap, so they stay in the XCD's L2). One tile per short-lived workgroup instead left the CUs mostly
// empty (SQ_WAVE_CYCLES ~ 0.7 resident waves per SIMD): workgroup dispatch, not the memory system, paced it.
template <bool WHITE, int RW>
__global__ __launch_bounds__(256, FPTA_INTERP_WPC) void k_grid_interp_mfma(SynthArgs a, GridBand band, int32_t n_tiles,
                                                                         int32_t R_pad, double* __restrict__ out) {
  const int per = (n_tiles + 7) >> 3;
  const int x = blockIdx.x & 7;
  const int step = gridDim.x >> 3;
  const int end = min(n_tiles, (x + 1) * per);
  for (int tile = x * per + (int)(blockIdx.x >> 3); tile < end; tile += step)
    interp_tile<WHITE, RW>(a, band, R_pad, out, tile);
}

constexpr int kDftMJ = 2, kDftMR = 4;  // k_grid_dft_mfma wave tile: 32 grid rows x 64 realizations

hipError_t launch_grid_dft_mfma(hipStream_t st, GridSegs gsegs, int32_t P, const double* coef, int32_t K,
                                int32_t R_pad) {
  if (R_pad % (16 * kDftMR) != 0 || gsegs.n <= 0 || gsegs.n > kGridMaxSeg) return hipErrorInvalidValue;
  int64_t gz = 0;
  for (int s = 0; s < gsegs.n; ++s) {
    GridSegDev& g = gsegs.s[s];
    g.nblk = (g.half + 16 * kDftMJ) / (16 * kDftMJ);  // ceil((half + 1) / (16 MJ))
    if (g.lde < g.nblk * 16 * kDftMJ || g.ntab < ((g.nm + 7) & ~7)) return hipErrorInvalidValue;
    gz += g.nblk;
  }
  if (gz > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_grid_dft_mfma<kDftMJ, kDftMR>),
                     dim3((unsigned)((R_pad + 64 * kDftMR - 1) / (64 * kDftMR)), (unsigned)P, (unsigned)gz), dim3(256),
                     0, st, gsegs, coef, K, R_pad);
  return hipGetLastError();
}

hipError_t launch_grid_interp_mfma(hipStream_t st, const SynthArgs& a, const GridBand& band, int32_t R_pad) {
  constexpr int RW = kInterpRW;
  if (band.n_chunks <= 0 || band.vmax < 4 || band.vmax % 4 != 0 || R_pad % (16 * RW) != 0)
    return hipErrorInvalidValue;
  const int32_t n_rb = (R_pad + 64 * RW - 1) / (64 * RW);
  const int64_t tiles = (int64_t)band.n_chunks * n_rb;
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
  const int64_t want = (int64_t)n_cu * kInterpWPC;
  const int64_t grid = std::min<int64_t>((tiles + 7) / 8 * 8, (want + 7) / 8 * 8);
  if (a.w_on)
    hipLaunchKernelGGL((k_grid_interp_mfma<true, RW>), dim3((unsigned)grid), dim3(256), 0, st, a, band,
                       (int32_t)tiles, R_pad, a.out);
  else
    hipLaunchKernelGGL((k_grid_interp_mfma<false, RW>), dim3((unsigned)grid), dim3(256), 0, st, a, band,
                       (int32_t)tiles, R_pad, a.out);
  return hipGetLastError();
}

}  // namespace fpta
