// Gridded (factored) synthesis for harmonic grids: the same sums as k_synth_valu_seeded,
//   r(t) = ch(t) sum_{k=1..N} c_k cos(k theta) + s_k sin(k theta),  theta = w0 t,
// evaluated as a type-2 non-uniform FFT factorisation F ~= W E:
//
//   k_grid_weights  once per layout: dense banded interpolation weights W (chromatic factor and
//                   mask folded in) for every chunk of <= 16 consecutive TOAs of one pulsar
//   k_grid_dft      per batch: grid values g_j = sum_k q_k (c_k cos(k x_j) + s_k sin(k x_j)),
//                   x_j = 2 pi j / nf, for every (pulsar, realization) - a real DFT done as a GEMM
//                   against the shared table E (both halves of the grid from one pass: the cos and
//                   sin partial sums give g_j and g_{nf-j})
//   k_grid_interp   per batch: r(t) = sum_i W[t][i] g[J_t + i] for all signals of the chunk, white
//                   noise / ECORR added in the epilogue, one store per sample
//
// Kernel: exponential of semicircle phi(z) = exp(beta (sqrt(1 - z^2) - 1)), |z| <= 1, width w grid
// cells, oversampling nf >= sigma (2N + 1); q_k = (2 pi / nf) / phi_hat(k) deconvolves it.
// Aliasing error <= ~1e-12 relative at the default w = 14, sigma = 1.5 (and at w = 13, sigma = 2;
// tests/test_gpu_grid.py, tools/sweep_grid.py).
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
// One thread per TOA of the segment: W[chunk][row + i][tt] = ch(t) phi((d - i) / (w / 2)), i < w.
__global__ __launch_bounds__(256) void k_grid_weights(SegDesc sd, int64_t n_toa, const double* __restrict__ nu,
                                                      const int32_t* __restrict__ chunk_of,
                                                      const int32_t* __restrict__ tt_of,
                                                      const int32_t* __restrict__ row_of,
                                                      const double* __restrict__ d_of, int32_t w, double beta,
                                                      int32_t rmax, double* __restrict__ wd) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_toa) return;
  double ch = chrom_factor(sd.freqf, nu[t], sd.idx);
  if (sd.mask && !sd.mask[t]) ch = 0.0;
  const double d = d_of[t];
  const double hw = 0.5 * (double)w;
  double* dst = wd + ((int64_t)chunk_of[t] * rmax + row_of[t]) * kGridTT + tt_of[t];
  for (int i = 0; i < w; ++i) {
    const double z = (d - (double)i) / hw;
    const double s = 1.0 - z * z;
    dst[(int64_t)i * kGridTT] = s > 0.0 ? ch * exp(beta * (sqrt(s) - 1.0)) : 0.0;
  }
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

__device__ __forceinline__ void grid_white_pair(int64_t t, int64_t g, uint32_t k0, uint32_t k1, double& z0,
                                                double& z1) {
  const u32x4 c = {(uint32_t)t, kWhitePsrWord, kWhiteStream, (uint32_t)(g >> 1)};
  box_muller(philox4x32_10(c, k0, k1), z0, z1);
}

// ----------------------------------------------------------------------------- k_grid_interp
// 1-D grid of n_chunks * ceil(R_pad / 512) tiles (padded to a multiple of 8), XCD-swizzled so that an
// XCD walks consecutive chunks of the same pulsar (their grid rows overlap: L2 reuse). Wave = 128
// realizations (lane: adjacent pair) x the chunk's TT TOAs; per grid row one 16-byte load per lane and
// TT wave-uniform weights (scalar loads), 2 TT FMAs.
template <bool WHITE, int DBG, int H = kGridTT / 2, bool NT = false, bool PRIO = false>
__global__ __launch_bounds__(256) void k_grid_interp(SynthArgs a, const int4* __restrict__ chunks, int32_t n_chunks,
                                                     int32_t n_rb, GridSegs gsegs, int32_t R_pad, int32_t n_lin_stagger,
                                                     int32_t stagger, double* __restrict__ out) {
  // `out` (= a.out) as a noalias argument: the stores of one tile cannot clobber the tables read by the
  // next, so the weight loads stay scalar (s_load) inside the persistent loop
  // Workgroups of the first dispatch round (blockIdx.x < stagger_n) start staggered by (b / 8) % 4
  // quarter-periods. All tiles cost the same, so without it the store bursts of the resident
  // workgroups stay in phase (compute, then all store together); a new workgroup starts when an old
  // one exits, so the first round's stagger carries over to the whole grid.
  // The delay is a scalar-ALU recurrence: s_sleep (builtin or asm) counts as a memory side effect and
  // would turn every later table load of the kernel into a vector load.
  if ((int)blockIdx.x < n_lin_stagger) {
    uint32_t x = blockIdx.x;
    const int n = ((blockIdx.x >> 3) & 3) * stagger * 256;
    for (int k = 0; k < n; ++k) x = x * 1664525u + 1013904223u;
    if (x == 0x7FFFFFFFu && n < 0) return;  // never taken; keeps the loop
  }
  const int per = gridDim.x >> 3;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  {
  const int lin = blockIdx.x;
  const int tile = (lin & 7) * per + (lin >> 3);
  if (tile >= n_chunks * n_rb) return;
  // wave-uniform by construction; readfirstlane keeps the divergence analysis from losing that inside
  // the persistent loop (the band loop below must stay scalar: scalar weight loads, SGPR operands)
  const int rb = __builtin_amdgcn_readfirstlane(tile / n_chunks);
  const int c = __builtin_amdgcn_readfirstlane(tile - rb * n_chunks);
  const int r0 = (rb * 4 + wave) * 128;
  if (r0 >= R_pad) return;
  const int4 ci = chunks[c];
  const int p = __builtin_amdgcn_readfirstlane(ci.x);
  const int64_t base = a.offs[p];
  const int rl = r0 + 2 * lane;

  dbl2 acc[kGridTT];
#pragma unroll
  for (int tt = 0; tt < kGridTT; ++tt) acc[tt] = (dbl2){0.0, 0.0};

  // segment tables come from the kernel arguments (constant address space): wave-uniform scalar loads
  for (int s = 0; s < (DBG == 4 ? 0 : gsegs.n); ++s) {
    const GridSegDev& gs = gsegs.s[s];
    const int2 jr0 = gs.js[c];
    const int2 jr = make_int2(__builtin_amdgcn_readfirstlane(jr0.x), __builtin_amdgcn_readfirstlane(jr0.y));
    const double* __restrict__ W = gs.wd + (int64_t)c * gs.rmax * kGridTT;
    const double* __restrict__ G = gs.g + (int64_t)p * gs.nf * R_pad + rl;
    // rows come in pairs (the host pads every band to an even row count with zero weights); two
    // register sets alternate so each row's load is issued one row ahead of its FMAs
    int j = jr.x;
    dbl2 ga = *(const dbl2*)(G + (int64_t)j * R_pad);
    if (++j == gs.nf) j = 0;
    dbl2 gb = *(const dbl2*)(G + (int64_t)j * R_pad);
    for (int i = 0; i < jr.y; i += 2) {
      const double* __restrict__ Wi = DBG == 2 ? W : W + i * kGridTT;
      if (++j == gs.nf) j = 0;
      const dbl2 gan = DBG == 1 ? (dbl2){1.0 * i, 2.0} : *(const dbl2*)(G + (int64_t)j * R_pad);  // rows past the band are valid grid rows
#pragma unroll
      for (int tt = 0; tt < kGridTT; ++tt) {
        acc[tt].x = fma(Wi[tt], ga.x, acc[tt].x);
        acc[tt].y = fma(Wi[tt], ga.y, acc[tt].y);
      }
      if (++j == gs.nf) j = 0;
      const dbl2 gbn = DBG == 1 ? (dbl2){2.0 * i, 1.0} : *(const dbl2*)(G + (int64_t)j * R_pad);
#pragma unroll
      for (int tt = 0; tt < kGridTT; ++tt) {
        acc[tt].x = fma(Wi[kGridTT + tt], gb.x, acc[tt].x);
        acc[tt].y = fma(Wi[kGridTT + tt], gb.y, acc[tt].y);
      }
      ga = gan;
      gb = gbn;
    }
  }

  const int cnt = __builtin_amdgcn_readfirstlane(ci.z);
  if constexpr (WHITE) {
    const int64_t g0 = a.real0 + rl;  // parity is wave-uniform (r0 and 2 lane are even)
#pragma unroll
    for (int tt = 0; tt < kGridTT; ++tt) {
      if (tt < cnt) {
        const int64_t tg = base + ci.y + tt;
        if (a.w_sigma) {
          const double sg = a.w_sigma[tg];
          double z0, z1, y0, y1;
          grid_white_pair(tg, g0, a.k0, a.k1, z0, z1);
          if (g0 & 1) {  // (g0, g0 + 1) straddle two pairs
            grid_white_pair(tg, g0 + 1, a.k0, a.k1, y0, y1);
            acc[tt].x = fma(sg, z1, acc[tt].x);
            acc[tt].y = fma(sg, y0, acc[tt].y);
          } else {
            acc[tt].x = fma(sg, z0, acc[tt].x);
            acc[tt].y = fma(sg, z1, acc[tt].y);
          }
        }
        const int ep = a.w_block_of ? a.w_block_of[tg] : -1;
        if (ep >= 0) {
          const double e = a.w_esig[ep];
          if (rl < a.n_real) acc[tt].x = fma(e, a.w_zb[(int64_t)rl * a.w_nblocks + ep], acc[tt].x);
          if (rl + 1 < a.n_real) acc[tt].y = fma(e, a.w_zb[(int64_t)(rl + 1) * a.w_nblocks + ep], acc[tt].y);
        }
      }
    }
  }

  // Store through LDS in two halves of kGridTT/2 TOAs: lane l then writes TOA (l % 8) of realization
  // 8 i + l / 8, i.e. 64-byte runs of one realization row instead of 64 scattered 8-byte words
  // (8x fewer L2 write requests). Each wave uses its own LDS slice; no cross-wave synchronisation.
  if constexpr (DBG == 10) {  // coalesced scratch layout [chunk][tt][R_pad] (diagnostic)
    const int64_t lim = (int64_t)a.n_real * a.ldo;
#pragma unroll
    for (int tt = 0; tt < kGridTT; ++tt) {
      const int64_t o = ((int64_t)c * kGridTT + tt) * R_pad + rl;
      if (o + 1 < lim) *(dbl2*)(out + o) = acc[tt];
    }
    return;
  }
  if constexpr (DBG == 3) {
    double sum = 0.0;
#pragma unroll
    for (int tt = 0; tt < kGridTT; ++tt) sum += acc[tt].x + acc[tt].y;
    if (sum == 123.456) out[rl] = sum;
    return;
  }
  // PAR: transpose even and odd realizations in separate passes (half the LDS per wave)
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
  constexpr int NP = kGridTT / H;      // TOA passes
  constexpr int LPR = H;               // lanes per realization row in a store instruction
  constexpr int RPI = 64 / LPR;        // realization rows per store instruction
  __shared__ double tbuf[4][64][H + 1];
  double(*tb)[H + 1] = tbuf[wave];
  const int q = lane / LPR, th = lane % LPR;
#pragma unroll
  for (int h = 0; h < NP; ++h) {
#pragma unroll
    for (int par = 0; par < 2; ++par) {
#pragma unroll
      for (int u = 0; u < H; ++u) tb[lane][u] = par ? acc[h * H + u].y : acc[h * H + u].x;
      __builtin_amdgcn_wave_barrier();
      const int tt = h * H + th;
      if (tt < cnt) {
        double* ocol = out + base + ci.y + tt;
#pragma unroll 4
        for (int i = 0; i < 64 / RPI; ++i) {
          const int rr = RPI * i + q;          // lane rr of the wave holds realization 2 rr + par
          const int r = r0 + 2 * rr + par;
          if (r < a.n_real) {
            double* o = ocol + (int64_t)r * a.ldo;
            const double v = a.accumulate ? *o + tb[rr][th] : tb[rr][th];
            if constexpr (NT)
              __builtin_nontemporal_store(v, o);
            else
              *o = v;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  }
}

hipError_t launch_grid_weights(hipStream_t st, const SegDesc& sd, int64_t n_toa, const double* nu,
                               const int32_t* chunk_of, const int32_t* tt_of, const int32_t* row_of,
                               const double* d_of, int32_t w, double beta, int32_t rmax, double* wd) {
  hipLaunchKernelGGL(k_grid_weights, dim3((unsigned)((n_toa + 255) / 256)), dim3(256), 0, st, sd, n_toa, nu,
                     chunk_of, tt_of, row_of, d_of, w, beta, rmax, wd);
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

hipError_t launch_grid_interp(hipStream_t st, const SynthArgs& a, const int4* chunks, int32_t n_chunks,
                              const GridSegs& gsegs, int32_t R_pad) {
  if (R_pad % 128 != 0 || n_chunks <= 0 || gsegs.n < 0 || gsegs.n > kGridMaxSeg) return hipErrorInvalidValue;
  const int32_t n_rb = (R_pad + 511) / 512;
  const int64_t tiles = (int64_t)n_chunks * n_rb;
  const int64_t n_lin = (tiles + 7) / 8 * 8;
  if (n_lin > 0x7FFFFFFF) return hipErrorInvalidValue;
  static const int cfg_stagger = [] { const char* e = getenv("FPTA_GRID_STAGGER"); return e ? atoi(e) : 2; }();
  static const int cfg_wpc = [] { const char* e = getenv("FPTA_GRID_WPC"); return e ? atoi(e) : 4; }();
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
      n_cu = 256;
  }
  const int64_t grid = n_lin;
  const int32_t stagger = cfg_stagger;
  const int32_t nl = (int32_t)std::min<int64_t>(n_lin, (int64_t)n_cu * cfg_wpc);  // first dispatch round
  static const int dbg = [] { const char* e = getenv("FPTA_GRID_DBG"); return e ? atoi(e) : 0; }();
#define L_(...) hipLaunchKernelGGL((k_grid_interp<__VA_ARGS__>), dim3((unsigned)grid), dim3(256), 0, st, a, chunks, n_chunks, n_rb, gsegs, R_pad, nl, stagger, a.out)
  switch (dbg) {
    case 1: L_(false, 1); break;
    case 2: L_(false, 2); break;
    case 3: L_(false, 3); break;
    case 4: L_(false, 4); break;
    case 5: L_(false, 0, 8, true); break;
    case 6: L_(false, 0, 4, false); break;
    case 7: L_(false, 0, 4, true); break;
    case 8: L_(false, 4, 4, false); break;
    case 9: L_(false, 4, 8, true); break;
    case 10: L_(false, 10); break;
    case 11: L_(false, 0, 8, false, true); break;
    case 12: L_(false, 0, 8, false, false); break;
    case 13: L_(false, 4, 16, false, false); break;
    default:
      if (a.w_on) L_(true, 0, 16); else L_(false, 0, 16);
  }
#undef L_
  return hipGetLastError();
}

}  // namespace fpta
