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

// ----------------------------------------------------------------------------- k_grid_dft_mfma
// Per pulsar two GEMMs sharing the output tile (4 modes per MFMA):
//   Cj[j][r] = sum_k ecos[k][j] c_k[r],  Sj[j][r] = sum_k esin[k][j] s_k[r],
//   g_j = Cj + Sj, g_{nf - j} = Cj - Sj (cos even, sin odd in j).
// A = table (row j, mode), B = coefficients (mode, realization), D: lane holds rows j = (l >> 4) + 4 g of
// realization l & 15, so every store instruction writes 4 runs of 128 bytes. Wave tile 16 MJ rows x 16 MR
// realizations. The table is zero-padded to ntab (multiple of 8) modes and lde (multiple of 16 MJ) rows;
// padded coefficient modes re-read the signal's last mode (finite) against zero table rows.
template <int MJ, int MR>
__global__ __launch_bounds__(256) void k_grid_dft_mfma(GridSegs gsegs, const double* __restrict__ coef, int32_t K,
                                                       int32_t R_pad) {
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
  const double* __restrict__ cp = coef + ((int64_t)p * K + gs.col0 + 2 * lg) * R_pad + r0 + lr;
  const double* __restrict__ ec = gs.ecos + (int64_t)lg * gs.lde + j0 + lr;
  const double* __restrict__ es = gs.esin + (int64_t)lg * gs.lde + j0 + lr;
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
    double bc[MR], bs[MR], ac[MJ], as[MJ];
  };
  auto mfma = [&](const Ops& o) {
#pragma unroll
    for (int u = 0; u < MJ; ++u)
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        C[u][i] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac[u], o.bc[i], C[u][i], 0, 0, 0);
        S[u][i] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.as[u], o.bs[i], S[u][i], 0, 0, 0);
      }
  };
  auto load = [&](int qq, Ops& o) {
    const int m = min(4 * qq + lg, gs.nm - 1) - lg;  // mode of lane group 0 (clamped)
    const double* __restrict__ cq = cp + (int64_t)(2 * m) * R_pad;
    const int64_t eo = (int64_t)(4 * qq) * gs.lde;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      o.bc[i] = cq[16 * i];
      o.bs[i] = cq[R_pad + 16 * i];
    }
#pragma unroll
    for (int u = 0; u < MJ; ++u) {
      o.ac[u] = ec[eo + 16 * u];
      o.as[u] = es[eo + 16 * u];
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
  double* __restrict__ gp = gs.g + (int64_t)p * gs.nf * R_pad + r0 + lr;
#pragma unroll
  for (int u = 0; u < MJ; ++u)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int j = j0 + 16 * u + lg + 4 * g;
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const double cv = C[u][i][g], sv = S[u][i][g];
        if (j <= gs.half) gp[(int64_t)j * R_pad + 16 * i] = cv + sv;
        if (j > 0 && 2 * j < gs.nf) gp[(int64_t)(gs.nf - j) * R_pad + 16 * i] = cv - sv;
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
// out[r][t] = sum_s sum_i W_s[chunk][i][tt] G_s[(J_s + i) mod nf][r] for a chunk of <= 32 TOAs: per 4 band
// rows, A = grid values (realization, row), B = weights (row, TOA).
//  * The chunk's even and odd TOAs are two B-tiles (column j = TOA 2j, 2j + 1) over the same band rows, so one
//    set of grid loads feeds both: the address unit, the busiest block of the 16-TOA version (one dbl2 grid
//    load per 2 MFMAs), now sees one per 4. Lane (lr, lg) loads W[row lg][2 lr .. 2 lr + 1] with one 16-byte
//    load (.x even tile, .y odd tile).
//  * Realization tiles come in pairs: lane (lr, lg) loads the adjacent realizations 2 lr, 2 lr + 1 of a
//    32-realization block with one 16-byte load (.x tile 2m, .y tile 2m + 1). D row rho of tile 2m + h is then
//    realization 32 m + 2 rho + h.
//  * D's register g of lane l holds TOA 2 (l & 15) + e of realization 32 m + 2 (lg + 4 g) + h in acc[e][2m + h]:
//    the two TOA parities of a lane are adjacent samples of one realization row (one 16-byte store, 256-byte
//    runs per row), and the two tiles of a realization pair sit in the same lane and register (one Philox call
//    per pair for the white epilogue).
// Wave tile = chunk x 16 RW realizations; per signal the next 4-row step's operands are loaded before the
// current step's MFMAs (two register sets, unrolled by 2, the odd last step skipped by a uniform branch).
template <bool WHITE, int RW>
__device__ __forceinline__ void interp_tile(const SynthArgs& a, const int4* __restrict__ chunks, int32_t n_chunks,
                                            const GridSegs& gsegs, int32_t R_pad, double* __restrict__ out,
                                            int tile) {
  static_assert(RW % 2 == 0, "realization tiles come in pairs");
  static_assert(kGridTT == 32, "two 16-TOA B-tiles per chunk");
  constexpr int NP = RW / 2;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  const int rb = __builtin_amdgcn_readfirstlane(tile / n_chunks);  // realization block of 64 RW
  const int c = __builtin_amdgcn_readfirstlane(tile - rb * n_chunks);
  const int r0 = (rb * 4 + wave) * 16 * RW;
  if (r0 >= R_pad) return;
  FPTA_DCHECK(r0 + 16 * RW <= R_pad, "k_grid_interp_mfma realization block", r0 + 16 * RW, R_pad + 1);
  const int4 ci = chunks[c];
  const int p = __builtin_amdgcn_readfirstlane(ci.x);
  const int64_t base = a.offs[p];

  d4 acc[2][RW];  // [TOA parity][realization tile]
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int i = 0; i < RW; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};

  for (int si = 0; si < gsegs.n; ++si) {
    const GridSegDev& gs = gsegs.s[si];
    const int2 jr = gs.js[c];
    const int nq = __builtin_amdgcn_readfirstlane(jr.y) >> 2;
    if (nq == 0) continue;
    const int nf = gs.nf;
    const double* __restrict__ Gp = gs.g + (int64_t)p * nf * R_pad + r0 + 2 * lr;
    const double* __restrict__ Wp = gs.wd + (int64_t)c * gs.rmax * kGridTT + lg * kGridTT + 2 * lr;
    int j = __builtin_amdgcn_readfirstlane(jr.x) + lg;  // grid row of this lane's k index
    if (j >= nf) j -= nf;
    dbl2 a0[NP], a1[NP], b0, b1;
    auto load = [&](int qq, dbl2(&av)[NP], dbl2& bv) {
      int jj = j + 4 * qq;
      while (jj >= nf) jj -= nf;
      const double* __restrict__ gr = Gp + (int64_t)jj * R_pad;
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
    load(0, a0, b0);
    for (int q = 0; q < nq; q += 2) {
      load(min(q + 1, nq - 1), a1, b1);
      mfma(a0, b0);
      load(min(q + 2, nq - 1), a0, b0);
      if (q + 1 < nq) mfma(a1, b1);  // odd step count: skip the re-read last step (wave-uniform branch)
    }
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
  // one 16-byte store per (lane, realization) when both TOAs exist: the row offset r * ldo + tg is even
  // whenever ldo and tg are, else the pair is stored as two 8-byte stores
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
__global__ __launch_bounds__(256, 2) void k_grid_interp_mfma(SynthArgs a, const int4* __restrict__ chunks,
                                                          int32_t n_chunks, int32_t n_tiles, GridSegs gsegs,
                                                          int32_t R_pad, double* __restrict__ out) {
  const int per = (n_tiles + 7) >> 3;
  const int x = blockIdx.x & 7;
  const int step = gridDim.x >> 3;
  const int end = min(n_tiles, (x + 1) * per);
  for (int tile = x * per + (int)(blockIdx.x >> 3); tile < end; tile += step)
    interp_tile<WHITE, RW>(a, chunks, n_chunks, gsegs, R_pad, out, tile);
}


constexpr int kDftMJ = 2, kDftMR = 2;  // k_grid_dft_mfma wave tile: 32 grid rows x 32 realizations
constexpr int kInterpRW = 8;           // k_grid_interp_mfma: 32 TOAs x 128 realizations per wave

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

template <int RW>
hipError_t launch_interp_rw(hipStream_t st, const SynthArgs& a, const int4* chunks, int32_t n_chunks,
                            const GridSegs& gsegs, int32_t R_pad) {
  if (R_pad % (16 * RW) != 0) return hipErrorInvalidValue;
  const int32_t n_rb = (R_pad + 64 * RW - 1) / (64 * RW);
  const int64_t tiles = (int64_t)n_chunks * n_rb;
  if (tiles > 0x7FFFFFFF) return hipErrorInvalidValue;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
  // persistent grid: 2 workgroups per CU (profiles/r01_sweep_interp_wpc.txt: 1 -> 1.06 ms, 2 -> 0.74, 3 -> 0.81)
  const int64_t want = (int64_t)n_cu * 2;
  const int64_t grid = std::min<int64_t>((tiles + 7) / 8 * 8, (want + 7) / 8 * 8);
  if (a.w_on)
    hipLaunchKernelGGL((k_grid_interp_mfma<true, RW>), dim3((unsigned)grid), dim3(256), 0, st, a, chunks, n_chunks,
                       (int32_t)tiles, gsegs, R_pad, a.out);
  else
    hipLaunchKernelGGL((k_grid_interp_mfma<false, RW>), dim3((unsigned)grid), dim3(256), 0, st, a, chunks,
                       n_chunks, (int32_t)tiles, gsegs, R_pad, a.out);
  return hipGetLastError();
}

hipError_t launch_grid_interp_mfma(hipStream_t st, const SynthArgs& a, const int4* chunks, int32_t n_chunks,
                                   const GridSegs& gsegs, int32_t R_pad) {
  if (n_chunks <= 0 || gsegs.n < 0 || gsegs.n > kGridMaxSeg) return hipErrorInvalidValue;
  for (int s = 0; s < gsegs.n; ++s)
    if (gsegs.s[s].rmax % 4 != 0 || gsegs.s[s].nf < 4) return hipErrorInvalidValue;
  return launch_interp_rw<kInterpRW>(st, a, chunks, n_chunks, gsegs, R_pad);
}

}  // namespace fpta
