// HIP kernels for gfx950 (MI355X): Fourier-basis GP residual synthesis.
//
//   k_gen          Philox4x32-10 -> Box-Muller -> coefficient scaling  (north-star step 1)
//   k_mix          ORF factor applied to the common-signal draws       (step 2)
//   k_synth_mfma   fused basis generation + contraction on fp64 MFMA   (steps 3/4)
//   k_synth_direct one sincos per basis element, used for few realizations and
//                  for the drop-in single-realization calls (exact reference phases)
//   k_white        white noise + ECORR epochs                          (step 4)
//
// Reference semantics: fakepta/fake_pta.py:357-387 (per-pulsar GP), :526-555
// (reconstruct_signal), :201-230 (white noise); fakepta/correlated_noises.py:111-160
// (common GP). See DESIGN.md for layouts and rooflines.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "fpta_internal.h"
#include "philox.h"

namespace fpta {

// ----------------------------------------------------------------------------- k_gen
// grid (ceil(R_pad/512), nm, P): thread = realization pair (r, r + 1), r even. One Philox call per (mode, pulsar,
// segment, global realization pair) gives the (cos, sin) pairs of both realizations (philox.h gp_pair2). Writes every
// entry of the realization padding.
__global__ __launch_bounds__(256) void k_gen(SegDesc sd, int32_t seg_id, int32_t P, int32_t n_real,
                                             int32_t R_pad, int64_t real0, uint32_t k0, uint32_t k1,
                                             const double* __restrict__ zin, int32_t zin_nseg,
                                             int32_t zin_nm, double* __restrict__ coef, int32_t K,
                                             double* __restrict__ zbuf) {
  const int r = (blockIdx.x * 256 + threadIdx.x) * 2;
  if (r >= R_pad) return;
  const int k = blockIdx.y;
  const int p = blockIdx.z;
  double zc[2] = {0.0, 0.0}, zs[2] = {0.0, 0.0};
  if (zin) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (r + h < n_real && k < zin_nm) {
        const double* zz = zin + ((((int64_t)(r + h) * zin_nseg + seg_id) * P + p) * zin_nm + k) * 2;
        zc[h] = zz[0];
        zs[h] = zz[1];
      }
  } else if (r < n_real) {
    const uint64_t g = (uint64_t)(real0 + r);
    if ((g & 1) == 0) {
      double z[4];
      gp_pair2((uint32_t)k, (uint32_t)p, (uint32_t)seg_id, g, k0, k1, z);
      zc[0] = z[0];
      zs[0] = z[1];
      zc[1] = z[2];
      zs[1] = z[3];
    } else {
      gp_normal2((uint32_t)k, (uint32_t)p, (uint32_t)seg_id, g, k0, k1, zc[0], zs[0]);
      gp_normal2((uint32_t)k, (uint32_t)p, (uint32_t)seg_id, g + 1, k0, k1, zc[1], zs[1]);
    }
    if (r + 1 >= n_real) zc[1] = zs[1] = 0.0;
  }
  if (sd.kind == 0) {
    const double a = sd.amp[(int64_t)p * sd.nm + k];
    double* cp = coef + ((int64_t)p * K + sd.col0 + 2 * k) * R_pad + r;
    *(double2*)cp = make_double2(a * zc[0], a * zc[1]);
    *(double2*)(cp + R_pad) = make_double2(a * zs[0], a * zs[1]);
  } else {
    double* zp = zbuf + ((int64_t)p * sd.nm + k) * 2 * R_pad + r;
    *(double2*)zp = make_double2(zc[0], zc[1]);
    *(double2*)(zp + R_pad) = make_double2(zs[0], zs[1]);
  }
}

// ----------------------------------------------------------------------------- k_mix
// coef[p][col0 + j][r] = amp[j/2] * sum_q L[p][q] zbuf[q][j][r],  j = 2k + (0 cos | 1 sin).
// One thread per (j, r) column, MIX_PT pulsar rows per block; L tiles broadcast from LDS.
constexpr int MIX_PT = 16;
constexpr int MIX_QT = 64;
__global__ __launch_bounds__(256) void k_mix(const double* __restrict__ L, const double* __restrict__ amp,
                                             int32_t P, int64_t M, int32_t R_pad,
                                             const double* __restrict__ zbuf, double* __restrict__ coef,
                                             int32_t K, int32_t col0, double* __restrict__ x_out) {
  __shared__ double Ls[MIX_PT][MIX_QT];
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int p0 = blockIdx.y * MIX_PT;
  double acc[MIX_PT];
#pragma unroll
  for (int i = 0; i < MIX_PT; ++i) acc[i] = 0.0;
  for (int q0 = 0; q0 < P; q0 += MIX_QT) {
    for (int e = threadIdx.x; e < MIX_PT * MIX_QT; e += 256) {
      const int i = e / MIX_QT, jj = e % MIX_QT;
      const int p = p0 + i, q = q0 + jj;
      Ls[i][jj] = (p < P && q < P) ? L[(int64_t)p * P + q] : 0.0;
    }
    __syncthreads();
    if (m < M) {
      const int qmax = min(MIX_QT, P - q0);
      const double* zp = zbuf + (int64_t)q0 * M + m;
      for (int jj = 0; jj < qmax; ++jj) {
        const double zv = zp[(int64_t)jj * M];
#pragma unroll
        for (int i = 0; i < MIX_PT; ++i) acc[i] = fma(Ls[i][jj], zv, acc[i]);
      }
    }
    __syncthreads();
  }
  if (m < M) {
    const int j = (int)(m / R_pad);
    const int r = (int)(m % R_pad);
    const double a = amp[j >> 1];
#pragma unroll
    for (int i = 0; i < MIX_PT; ++i) {
      const int p = p0 + i;
      if (p < P) {
        coef[((int64_t)p * K + col0 + j) * R_pad + r] = a * acc[i];
        if (x_out) x_out[(int64_t)p * M + m] = acc[i];
      }
    }
  }
}

// ----------------------------------------------------------------------------- k_mix_tiled
// The same product as k_mix as a register/LDS-tiled fp64 GEMM for large arrays (C4: P = 1000):
// C[P x M] = L[P x P] Z[P x M], block tile 128 rows x 128 columns, 8 x 8 outputs per thread,
// q-chunks of 16 staged through LDS (L transposed), next chunk prefetched into registers.
// Each Z element is re-read P/128 times instead of P/16. With a lower-triangular L (Cholesky of
// a positive-definite ORF) the q loop stops at the tile's last row: half the work.
// LDS reads are ds_read_b128: L rows ty*8.. are broadcast within a 16-lane group, Z columns
// {2tx, 2tx+1} + 32 jj give every 16-lane group 256 contiguous bytes (conflict-free).
constexpr int MT_P = 128, MT_M = 128, MT_Q = 16;
__global__ __launch_bounds__(256) void k_mix_tiled(const double* __restrict__ L, const double* __restrict__ amp,
                                                   int32_t P, int64_t M, int32_t R_pad, int32_t lower,
                                                   const double* __restrict__ zbuf, double* __restrict__ coef,
                                                   int32_t K, int32_t col0, double* __restrict__ x_out) {
  __shared__ __attribute__((aligned(16))) double Ls[MT_Q][MT_P + 2];  // +2: transposed writes spread banks
  __shared__ __attribute__((aligned(16))) double Zs[MT_Q][MT_M];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int p0 = blockIdx.y * MT_P;
  const int64_t m0 = (int64_t)blockIdx.x * MT_M;
  const int qend = lower ? min(P, p0 + MT_P) : P;
  double acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0;
  double lreg[8], zreg[8];
  auto fetch = [&](int q0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = tid + 256 * e;
      const int i = idx >> 4, jj = idx & 15;  // L[p0 + i][q0 + jj]
      const int p = p0 + i, q = q0 + jj;
      lreg[e] = (p < P && q < P) ? L[(int64_t)p * P + q] : 0.0;
      const int zq = idx >> 7, c = idx & 127;  // Z[q0 + zq][m0 + c]
      zreg[e] = (q0 + zq < P) ? zbuf[(int64_t)(q0 + zq) * M + m0 + c] : 0.0;
    }
  };
  fetch(0);
  for (int q0 = 0; q0 < qend; q0 += MT_Q) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = tid + 256 * e;
      Ls[idx & 15][idx >> 4] = lreg[e];
      Zs[idx >> 7][idx & 127] = zreg[e];
    }
    __syncthreads();
    if (q0 + MT_Q < qend) fetch(q0 + MT_Q);
#pragma unroll
    for (int q = 0; q < MT_Q; ++q) {
      double lv[8], zv[8];
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const double2 a = *reinterpret_cast<const double2*>(&Ls[q][ty * 8 + i]);
        lv[i] = a.x;
        lv[i + 1] = a.y;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double2 b = *reinterpret_cast<const double2*>(&Zs[q][2 * tx + 32 * j]);
        zv[2 * j] = b.x;
        zv[2 * j + 1] = b.y;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = fma(lv[i], zv[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = p0 + ty * 8 + i;
    if (p >= P) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + 2 * tx + 32 * j;  // columns m, m+1 share j (R_pad is even)
      const int jc = (int)(m / R_pad);
      const int r = (int)(m % R_pad);
      const double a = amp[jc >> 1];
      double2 v = make_double2(a * acc[i][2 * j], a * acc[i][2 * j + 1]);
      *reinterpret_cast<double2*>(&coef[((int64_t)p * K + col0 + jc) * R_pad + r]) = v;
      if (x_out) *reinterpret_cast<double2*>(&x_out[(int64_t)p * M + m]) = make_double2(acc[i][2 * j], acc[i][2 * j + 1]);
    }
  }
}

// ----------------------------------------------------------------------------- k_synth_direct
// grid (ceil(n_toa/256), n_real). One thread per (TOA, realization); the phase of every basis
// element is (2 pi f_k) t computed exactly as fake_pta.py:386, then sincos.
__global__ __launch_bounds__(256) void k_synth_direct(SynthArgs a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y;
  if (t >= a.n_toa) return;
  const int p = a.psr_of[t];
  const double toa = a.toas[t];
  const double nu = a.nu[t];
  const double* cbase = a.coef + (int64_t)p * a.K * a.R_pad + r;
  double acc = 0.0;
  for (int s = 0; s < a.n_seg; ++s) {
    const SegDesc sd = a.segs[s];
    if (sd.mask && !sd.mask[t]) continue;
    const double ch = chrom_factor(sd.freqf, nu, sd.idx);
    const double* w = sd.w + (int64_t)p * sd.w_pstride;
    const double* cs = cbase + (int64_t)sd.col0 * a.R_pad;
    double accs = 0.0;
    for (int k = 0; k < sd.nm; ++k) {
      double sn, cn;
      sincos(w[k] * toa, &sn, &cn);
      accs = fma(cs[(int64_t)(2 * k) * a.R_pad], cn, accs);
      accs = fma(cs[(int64_t)(2 * k + 1) * a.R_pad], sn, accs);
    }
    acc = fma(ch, accs, acc);
  }
  double* o = a.out + (int64_t)r * a.ldo + t;
  *o = a.accumulate ? *o + acc : acc;
}

// ----------------------------------------------------------------------------- k_synth_mfma
// out^T tile [realizations x TOAs] = A [realizations x K] * B [K x TOAs] on
// v_mfma_f64_16x16x4_f64, where A = coefficients (read from L2) and B = chromatic Fourier basis
// generated in registers: lane l owns TOA (l & 15) and basis column (l >> 4) of each 4-column
// K-step (cos m, sin m, cos m+1, sin m+1). On harmonic grids the lane's phasor
// ch * exp(i w_m t) is advanced two modes per K-step by one complex multiply with
// exp(i 2 w_0 t), and re-anchored to an exact sincos every `anchor` K-steps.
// Fragment maps (cdna_hip_programming.md §3): A[i = l&15][k = l>>4], B[k = l>>4][j = l&15],
// D: col = l&15 (TOA), row = (l>>4) + 4*reg (realization).
template <int WR, int WT>
__global__ __launch_bounds__(256, 2) void k_synth_mfma(SynthArgs a, const int4* __restrict__ tiles) {
  const int4 tl = tiles[blockIdx.x];
  const int p = tl.x;
  if (p < 0) return;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15;
  const int lg = lane >> 4;
  const int64_t base = a.offs[p];
  const int np_ = (int)(a.offs[p + 1] - base);
  const int tw0 = tl.y + wave * WT * 16;
  const int r0 = tl.z;
  FPTA_DCHECK(a.tile_toa == kWaves * WT * 16 && a.tile_real == WR * 16, "k_synth_mfma tile geometry", a.tile_real,
              WR * 16 + 1);
  FPTA_DCHECK(r0 + WR * 16 <= a.R_pad, "k_synth_mfma realization block", r0 + WR * 16, a.R_pad + 1);
  if (tw0 >= np_) return;  // whole wave past the pulsar's last TOA (no cross-wave sync below)

  double t[WT], nuv[WT];
  int tc[WT];
#pragma unroll
  for (int f = 0; f < WT; ++f) {
    const int tloc = tw0 + f * 16 + lr;
    tc[f] = tloc < np_ ? tloc : np_ - 1;
    t[f] = a.toas[base + tc[f]];
    nuv[f] = a.nu[base + tc[f]];
  }
  d4 acc[WR][WT];
#pragma unroll
  for (int i = 0; i < WR; ++i)
#pragma unroll
    for (int f = 0; f < WT; ++f) acc[i][f] = d4{0.0, 0.0, 0.0, 0.0};

  const int moff = lg >> 1;
  const bool is_sin = (lg & 1) != 0;
  const double* cp = a.coef + (int64_t)p * a.K * a.R_pad + r0 + lr;

  for (int s = 0; s < a.n_seg; ++s) {
    const SegDesc sd = a.segs[s];
    const double* w = sd.w + (int64_t)p * sd.w_pstride;
    double ch[WT];
#pragma unroll
    for (int f = 0; f < WT; ++f) {
      ch[f] = chrom_factor(sd.freqf, nuv[f], sd.idx);
      if (sd.mask && !sd.mask[base + tc[f]]) ch[f] = 0.0;
    }
    const bool harm = sd.harmonic != 0;
    const int anchor = harm ? (a.anchor > 0 ? a.anchor : 0x7fffffff) : 1;
    double rr[WT], ri[WT], zr[WT], zi[WT];
    const double* cs = cp + (int64_t)(sd.col0 + lg) * a.R_pad;
    const int nsteps = sd.nm >> 1;
    for (int j = 0; j < nsteps; ++j) {
      double av[WR];
      const double* cj = cs + (int64_t)(4 * j) * a.R_pad;
#pragma unroll
      for (int i = 0; i < WR; ++i) av[i] = cj[i * 16];
      if (j % anchor == 0) {
        const double wk = w[2 * j + moff];
#pragma unroll
        for (int f = 0; f < WT; ++f) {
          double sn, cn;
          sincos(wk * t[f], &sn, &cn);
          zr[f] = ch[f] * cn;
          zi[f] = ch[f] * sn;
          if (j == 0) {
            // step exp(i 2 w_0 t): the square of the mode-0 phasor, or the mode-1 phasor itself
            rr[f] = moff ? cn : fma(cn, cn, -sn * sn);
            ri[f] = moff ? sn : 2.0 * cn * sn;
          }
        }
      } else {
#pragma unroll
        for (int f = 0; f < WT; ++f) {
          const double nr = fma(zr[f], rr[f], -zi[f] * ri[f]);
          const double ni = fma(zr[f], ri[f], zi[f] * rr[f]);
          zr[f] = nr;
          zi[f] = ni;
        }
      }
#pragma unroll
      for (int f = 0; f < WT; ++f) {
        const double b = is_sin ? zi[f] : zr[f];
#pragma unroll
        for (int i = 0; i < WR; ++i) acc[i][f] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], b, acc[i][f], 0, 0, 0);
      }
    }
  }

#pragma unroll
  for (int i = 0; i < WR; ++i) {
#pragma unroll
    for (int f = 0; f < WT; ++f) {
      const int tloc = tw0 + f * 16 + lr;
      if (tloc >= np_) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int r = r0 + i * 16 + lg + 4 * g;
        if (r < a.n_real) {
          double* o = a.out + (int64_t)r * a.ldo + base + tloc;
          *o = a.accumulate ? *o + acc[i][f][g] : acc[i][f][g];
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------- k_synth_valu
// Fused basis + contraction on the fp64 VALU (v_fma_f64 runs faster than v_mfma_f64 on gfx950:
// DESIGN.md §Calibration). Lane l owns TOAs t0 + l + 64 m (m < MT); the wave owns NT
// realizations, so every coefficient is wave-uniform and is read with scalar loads straight
// into SGPR operands of v_fma_f64. Per mode k each lane advances its phasors
// z_m = ch_m exp(i w_k t_m) by one complex multiply (harmonic grids), then
//   acc[m][n] += Re z_m * A[2k][n] + Im z_m * A[2k+1][n]
// i.e. 2*NT FMAs per 4 recurrence ops per TOA. Workgroup = 4 waves on the same TOAs,
// realizations r0 + NT * wave.
template <int MT, int NT>
__global__ __launch_bounds__(256) void k_synth_valu(SynthArgs a, const int4* __restrict__ tiles) {
  const int4 tl = tiles[blockIdx.x];
  const int p = tl.x;
  if (p < 0) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t base = a.offs[p];
  const int np_ = (int)(a.offs[p + 1] - base);
  const int r0 = tl.z + wave * NT;
  FPTA_DCHECK(a.tile_toa == 64 * MT && a.tile_real == 4 * NT, "k_synth_valu tile geometry", a.tile_real, 4 * NT + 1);
  if (r0 >= a.n_real) return;
  // every coefficient read below is cb[col * R_pad + n], n < NT: the wave's realizations must lie in the padding
  FPTA_DCHECK(r0 + NT <= a.R_pad, "k_synth_valu realization block", r0 + NT, a.R_pad + 1);

  double t[MT], nuv[MT];
  int tc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int tloc = tl.y + lane + 64 * m;
    tc[m] = tloc < np_ ? tloc : np_ - 1;
    t[m] = a.toas[base + tc[m]];
    nuv[m] = a.nu[base + tc[m]];
  }
  double acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = 0.0;

  const double* __restrict__ cb = a.coef + (int64_t)p * a.K * a.R_pad + r0;
  for (int s = 0; s < a.n_seg; ++s) {
    const SegDesc sd = a.segs[s];
    const double* w = sd.w + (int64_t)p * sd.w_pstride;
    double ch[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      ch[m] = chrom_factor(sd.freqf, nuv[m], sd.idx);
      if (sd.mask && !sd.mask[base + tc[m]]) ch[m] = 0.0;
    }
    const bool harm = sd.harmonic != 0;
    const int anchor = harm ? (a.anchor > 0 ? 2 * a.anchor : 0x7fffffff) : 1;
    double zr[MT], zi[MT], rr[MT], ri[MT];
    const double* ck = cb + (int64_t)sd.col0 * a.R_pad;
    for (int k = 0; k < sd.nm; ++k, ck += 2 * (int64_t)a.R_pad) {
      if (k % anchor == 0) {
        const double wk = w[k];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          double sn, cn;
          sincos(wk * t[m], &sn, &cn);
          zr[m] = ch[m] * cn;
          zi[m] = ch[m] * sn;
          if (k == 0) {
            rr[m] = cn;
            ri[m] = sn;
          }
        }
      } else {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          const double nr = fma(zr[m], rr[m], -zi[m] * ri[m]);
          const double ni = fma(zr[m], ri[m], zi[m] * rr[m]);
          zr[m] = nr;
          zi[m] = ni;
        }
      }
      double cc[NT], cs[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        cc[n] = ck[n];
        cs[n] = ck[a.R_pad + n];
      }
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][n] = fma(zi[m], cs[n], fma(zr[m], cc[n], acc[m][n]));
    }
  }

#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int r = r0 + n;
    if (r >= a.n_real) break;
    double* orow = a.out + (int64_t)r * a.ldo + base;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int tloc = tl.y + lane + 64 * m;
      if (tloc < np_) orow[tloc] = a.accumulate ? orow[tloc] + acc[m][n] : acc[m][n];
    }
  }
}

// ----------------------------------------------------------------------------- k_seeds
// Per (segment, TOA) recurrence seed, computed once per layout (TOAs and grids are fixed across
// batches): {ch cos(w0 t), ch sin(w0 t), 2 cos(w0 t), ch} with ch = (freqf/nu)^idx * mask and
// w0 = the segment's first angular frequency for the TOA's pulsar. grid (ceil(n_toa/256), n_seg).
__global__ __launch_bounds__(256) void k_seeds(const SegDesc* __restrict__ segs, const int32_t* __restrict__ psr_of,
                                               const double* __restrict__ toas, const double* __restrict__ nu,
                                               int64_t n_toa, double4* __restrict__ seeds) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int s = blockIdx.y;
  if (t >= n_toa) return;
  const SegDesc sd = segs[s];
  const int p = psr_of[t];
  double ch = chrom_factor(sd.freqf, nu[t], sd.idx);
  if (sd.mask && !sd.mask[t]) ch = 0.0;
  double sn, cn;
  sincos(sd.w[(int64_t)p * sd.w_pstride] * toas[t], &sn, &cn);
  seeds[(int64_t)s * n_toa + t] = make_double4(ch * cn, ch * sn, 2.0 * cn, ch);
}

// White-noise normals of TOA t for the realization pair containing g (oracle quad_normals on the white stream):
// (z for the even realization, z for the odd one), two of the four normals of one Philox call.
__device__ __forceinline__ void white_pair(int64_t t, int64_t g, uint32_t k0, uint32_t k1, double& z0, double& z1) {
  double z[4];
  quad4((uint64_t)t & ~(uint64_t)1, kWhiteStream, (uint64_t)g & ~(uint64_t)1, k0, k1, z);
  z0 = z[2 * (t & 1)];
  z1 = z[2 * (t & 1) + 1];
}

// ----------------------------------------------------------------------------- k_synth_valu_seeded
// The production fused kernel for harmonic grids (every f_k = k/T signal of fake_pta.py:264 and
// correlated_noises.py:120). No transcendental in the kernel: each lane loads its TOA's seed and
// advances the phasor one mode per complex multiply. Workgroup = 4 waves on 4 consecutive TOA
// blocks (64*MT TOAs each) sharing the same NT realizations, so the wave-uniform coefficient
// stream (scalar loads into v_fma_f64 SGPR operands) is shared through the scalar cache.
// WHITE: the epilogue adds sigma*z + ECORR (fake_pta.py:201-230) before the single store, so the
// block is written once instead of re-read and re-written by a separate white-noise pass.
template <int MT, int NT, bool WHITE>
__global__ __launch_bounds__(256) void k_synth_valu_seeded(SynthArgs a, const int4* __restrict__ tiles,
                                                           const double4* __restrict__ seeds) {
  const int4 tl = tiles[blockIdx.x];
  const int p = tl.x;
  if (p < 0) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t base = a.offs[p];
  const int np_ = (int)(a.offs[p + 1] - base);
  const int tw0 = tl.y + wave * 64 * MT;
  const int r0 = tl.z;
  FPTA_DCHECK(a.tile_toa == 256 * MT && a.tile_real == NT, "k_synth_valu_seeded tile geometry", a.tile_real, NT + 1);
  FPTA_DCHECK(r0 + NT <= a.R_pad, "k_synth_valu_seeded realization block", r0 + NT, a.R_pad + 1);
  FPTA_DCHECK((int64_t)(p + 1) * a.K * a.R_pad <= a.coef_len, "k_synth_valu_seeded coefficient rows",
              (int64_t)(p + 1) * a.K * a.R_pad, a.coef_len + 1);
  if (tw0 >= np_) return;  // whole wave past the pulsar's last TOA (no cross-wave sync below)

  int tc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int tloc = tw0 + lane + 64 * m;
    tc[m] = tloc < np_ ? tloc : np_ - 1;
  }
  double acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = 0.0;

  const double* __restrict__ cb = a.coef + (int64_t)p * a.K * a.R_pad + r0;
  for (int s = 0; s < a.n_seg; ++s) {
    const SegDesc sd = a.segs[s];
    // three-term recurrence z_{k+1} = 2 cos(w0 t) z_k - z_{k-1} (2 FMAs per mode and TOA), started
    // from z_{-1} = (ch, 0) (frequency 0) and z_0 = ch exp(i w0 t). A rounding error made at step j
    // reaches step k multiplied by U_{k-j-1}(cos w0 t), |U_n| <= n + 1: the error stays below
    // ~k^2/2 ulp (5e-13 at 100 modes) for every phase, including w0 t near 0 or pi.
    double zr[MT], zi[MT], pr[MT], pi_[MT], c2[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const double4 q = seeds[(int64_t)s * a.n_toa + base + tc[m]];
      zr[m] = q.x;
      zi[m] = q.y;
      c2[m] = q.z;
      pr[m] = q.w;
      pi_[m] = 0.0;
    }
    const double* ck = cb + (int64_t)sd.col0 * a.R_pad;
    // nm is even (padded on the host): two modes per trip; the halves alternate which register
    // pair holds the current mode, so the recurrence needs no copies
    for (int k = 0; k < sd.nm; k += 2, ck += 4 * (int64_t)a.R_pad) {
      double cc[NT], cs[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        cc[n] = ck[n];
        cs[n] = ck[a.R_pad + n];
      }
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][n] = fma(zi[m], cs[n], fma(zr[m], cc[n], acc[m][n]));
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        pr[m] = fma(c2[m], zr[m], -pr[m]);
        pi_[m] = fma(c2[m], zi[m], -pi_[m]);
      }
      const double* ck1 = ck + 2 * (int64_t)a.R_pad;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        cc[n] = ck1[n];
        cs[n] = ck1[a.R_pad + n];
      }
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][n] = fma(pi_[m], cs[n], fma(pr[m], cc[n], acc[m][n]));
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        zr[m] = fma(c2[m], pr[m], -zr[m]);
        zi[m] = fma(c2[m], pi_[m], -zi[m]);
      }
    }
  }

  if constexpr (WHITE) {
    double sg[MT], es[MT];
    int ep[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int64_t tg = base + tc[m];
      sg[m] = a.w_sigma ? a.w_sigma[tg] : 0.0;
      ep[m] = a.w_block_of ? a.w_block_of[tg] : -1;
      es[m] = ep[m] >= 0 ? a.w_esig[ep[m]] : 0.0;
    }
    double z0[MT], z1[MT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int r = r0 + n;
      if (r >= a.n_real) break;
      const int64_t g = a.real0 + r;  // wave-uniform: the branches below do not diverge
      if (a.w_sigma && (n == 0 || (g & 1) == 0)) {
#pragma unroll
        for (int m = 0; m < MT; ++m) white_pair(base + tc[m], g, a.k0, a.k1, z0[m], z1[m]);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        double v = acc[m][n];
        if (a.w_sigma) v = fma(sg[m], (g & 1) ? z1[m] : z0[m], v);
        if (ep[m] >= 0) v = fma(es[m], a.w_zb[(int64_t)r * a.w_nblocks + ep[m]], v);
        acc[m][n] = v;
      }
    }
  }

#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int r = r0 + n;
    if (r >= a.n_real) break;
    double* orow = a.out + (int64_t)r * a.ldo + base;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int tloc = tw0 + lane + 64 * m;
      if (tloc < np_) orow[tloc] = a.accumulate ? orow[tloc] + acc[m][n] : acc[m][n];
    }
  }
}

// ----------------------------------------------------------------------------- k_white
// grid (ceil(n_toa/256), n_real). out[r][t] += sigma[t] z(t, r) + ecorr[b(t)] zb(b(t), r).
__global__ __launch_bounds__(256) void k_white(const double* __restrict__ sigma,
                                               const int32_t* __restrict__ block_of,
                                               const double* __restrict__ esig, const double* __restrict__ z,
                                               const double* __restrict__ zb, double* __restrict__ out,
                                               int64_t ldo, int64_t n_toa, int64_t real0, uint32_t k0,
                                               uint32_t k1) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int r = blockIdx.y;
  if (t >= n_toa) return;
  double v = 0.0;
  if (sigma) {
    double zt;
    if (z) {
      zt = z[(int64_t)r * n_toa + t];
    } else {
      zt = quad_normal((uint64_t)t, kWhiteStream, (uint64_t)(real0 + r), k0, k1);
    }
    v = sigma[t] * zt;
  }
  if (block_of) {
    const int b = block_of[t];
    if (b >= 0) {
      double zbv;
      if (zb) {
        zbv = zb[b];
      } else {
        zbv = quad_normal((uint64_t)b, kEcorrStream, (uint64_t)(real0 + r), k0, k1);
      }
      v = fma(esig[b], zbv, v);
    }
  }
  out[(int64_t)r * ldo + t] += v;
}

// ----------------------------------------------------------------------------- batch white / ECORR
// k_epoch_normals: zb[r][b] for every ECORR epoch (oracle quad_normals on the ECORR stream), one Philox call per
// (epoch pair, global realization pair): four normals. grid (ceil(ceil(n_blocks/2)/256), realization pairs touched).
__global__ __launch_bounds__(256) void k_epoch_normals(int64_t n_blocks, int32_t n_real, int64_t real0, uint32_t k0,
                                                       uint32_t k1, double* __restrict__ zb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // epoch pair
  if (2 * i >= n_blocks) return;
  const int64_t g0 = ((real0 >> 1) + blockIdx.y) * 2;  // even global realization of this pair
  double z[4];
  quad4((uint64_t)(2 * i), kEcorrStream, (uint64_t)g0, k0, k1, z);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t r = g0 + h - real0;
    if (r < 0 || r >= n_real) continue;
    double* row = zb + r * n_blocks;
    row[2 * i] = z[h];
    if (2 * i + 1 < n_blocks) row[2 * i + 1] = z[2 + h];
  }
}

// k_white_pairs: out[r][t] += sigma[t] z(t, real0 + r) + ecorr[b(t)] zb[r][b(t)], one thread per
// (TOA, global realization pair). grid (ceil(n_toa/256), number of realization pairs touched).
__global__ __launch_bounds__(256) void k_white_pairs(const double* __restrict__ sigma,
                                                     const int32_t* __restrict__ block_of,
                                                     const double* __restrict__ esig, const double* __restrict__ zb,
                                                     int64_t n_blocks, double* __restrict__ out, int64_t ldo,
                                                     int64_t n_toa, int32_t n_real, int64_t real0, uint32_t k0,
                                                     uint32_t k1) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_toa) return;
  const int64_t g0 = ((real0 >> 1) + blockIdx.y) * 2;  // even global realization of this pair
  double z[2] = {0.0, 0.0};
  if (sigma) white_pair(t, g0, k0, k1, z[0], z[1]);
  const double s = sigma ? sigma[t] : 0.0;
  const int b = block_of ? block_of[t] : -1;
  const double e = b >= 0 ? esig[b] : 0.0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t r = g0 + h - real0;
    if (r < 0 || r >= n_real) continue;
    double v = s * z[h];
    if (b >= 0) v = fma(e, zb[r * n_blocks + b], v);
    out[r * ldo + t] += v;
  }
}

// ----------------------------------------------------------------------------- correlation statistics
// The estimator of correlated_noises.py:14-34 on device, for arrays whose pulsars share the TOA
// count n: C_r[a][b] = sum_t x_r[a][t] x_r[b][t] / n per realization r of the last block.
// k_autos: auto[r][p] = C_r[p][p]. grid (P, n_real), one block per (pulsar, realization).
__global__ __launch_bounds__(256) void k_autos(const double* __restrict__ out, int64_t ldo, int32_t n,
                                               double* __restrict__ autos, int32_t P) {
  __shared__ double red[256];
  const int p = blockIdx.x, r = blockIdx.y;
  const double* x = out + (int64_t)r * ldo + (int64_t)p * n;
  double s = 0.0;
  for (int t = threadIdx.x; t < n; t += 256) s = fma(x[t], x[t], s);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) autos[(int64_t)r * P + p] = red[0] / n;
}

// k_xcorr: 64 x 64 tiles (ta <= tb) of C_r, 4 x 4 outputs per thread, TOA chunks of 32 staged in LDS.
// mode 0: write C_r per realization [n_real][P][P]; mode 1: accumulate sum_r C_r; mode 2: accumulate
// sum_r C_r[a][b] / sqrt(auto_r[a] auto_r[b]). Modes 1/2 loop over `rper` realizations per block and
// write one partial [chunk][P][P] (summed in a fixed order afterwards: deterministic).
constexpr int XC_T = 64, XC_K = 32;
__global__ __launch_bounds__(256) void k_xcorr(const double* __restrict__ out, int64_t ldo, int32_t n, int32_t P,
                                               int32_t n_real, int32_t mode, int32_t rper,
                                               const double* __restrict__ autos, double* __restrict__ dst) {
  __shared__ double Xa[XC_K][XC_T + 1];
  __shared__ double Xb[XC_K][XC_T + 1];
  // decode the upper-triangular tile pair
  const int nt = (P + XC_T - 1) / XC_T;
  int pair = blockIdx.x, ta = 0;
  while (pair >= nt - ta) {
    pair -= nt - ta;
    ++ta;
  }
  const int tb = ta + pair;
  const int a0 = ta * XC_T, b0 = tb * XC_T;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int rbeg = blockIdx.y * rper, rend = min(n_real, rbeg + rper);
  double tot[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) tot[i][j] = 0.0;
  for (int r = rbeg; r < rend; ++r) {
    const double* xr = out + (int64_t)r * ldo;
    double acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
    for (int t0 = 0; t0 < n; t0 += XC_K) {
      __syncthreads();
      for (int e = threadIdx.x; e < XC_T * XC_K; e += 256) {
        const int row = e / XC_K, k = e % XC_K;
        const int t = t0 + k;
        Xa[k][row] = (a0 + row < P && t < n) ? xr[(int64_t)(a0 + row) * n + t] : 0.0;
        Xb[k][row] = (b0 + row < P && t < n) ? xr[(int64_t)(b0 + row) * n + t] : 0.0;
      }
      __syncthreads();
#pragma unroll 4
      for (int k = 0; k < XC_K; ++k) {
        double av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[i] = Xa[k][ty + 16 * i];
          bv[i] = Xb[k][tx + 16 * i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fma(av[i], bv[j], acc[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a = a0 + ty + 16 * i;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = b0 + tx + 16 * j;
        if (a >= P || b >= P) continue;
        const double c = acc[i][j] / n;
        if (mode == 0) {
          dst[((int64_t)r * P + a) * P + b] = c;
          dst[((int64_t)r * P + b) * P + a] = c;
        } else if (mode == 1) {
          tot[i][j] += c;
        } else {
          tot[i][j] += c / sqrt(autos[(int64_t)r * P + a] * autos[(int64_t)r * P + b]);
        }
      }
    }
  }
  if (mode != 0) {
    double* part = dst + (int64_t)blockIdx.y * P * P;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a = a0 + ty + 16 * i;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int b = b0 + tx + 16 * j;
        if (a >= P || b >= P) continue;
        part[(int64_t)a * P + b] = tot[i][j];
        part[(int64_t)b * P + a] = tot[i][j];
      }
    }
  }
}

// sum of `nparts` [P*P] partials in index order (deterministic)
__global__ __launch_bounds__(256) void k_sum_parts(const double* __restrict__ parts, int32_t nparts, int64_t len,
                                                   double* __restrict__ res) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= len) return;
  double s = 0.0;
  for (int c = 0; c < nparts; ++c) s += parts[(int64_t)c * len + i];
  res[i] = s;
}

// ----------------------------------------------------------------------------- k_checksums
__global__ __launch_bounds__(256) void k_checksums(const double* __restrict__ out, int64_t ldo, int64_t n_toa,
                                                   double* __restrict__ sums) {
  __shared__ double s1[256], s2[256];
  const int r = blockIdx.x;
  double a = 0.0, b = 0.0;
  for (int64_t t = threadIdx.x; t < n_toa; t += 256) {
    const double v = out[(int64_t)r * ldo + t];
    a += v;
    b = fma(v, v, b);
  }
  s1[threadIdx.x] = a;
  s2[threadIdx.x] = b;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s1[threadIdx.x] += s1[threadIdx.x + w];
      s2[threadIdx.x] += s2[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sums[2 * r] = s1[0];
    sums[2 * r + 1] = s2[0];
  }
}

__global__ void k_philox(int64_t n, const uint32_t* __restrict__ ctr, uint32_t k0, uint32_t k1,
                         uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 c = {ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]};
  const u32x4 v = philox4x32_10(c, k0, k1);
  out[4 * i] = v.x;
  out[4 * i + 1] = v.y;
  out[4 * i + 2] = v.z;
  out[4 * i + 3] = v.w;
}

// k_normals4: the build's uniform -> normal map on given Philox words (fpta_debug_normals): out[4 i .. 4 i + 3] =
// normals4(words[4 i .. 4 i + 3]), the map every device draw uses
__global__ void k_normals4(int64_t n, const uint32_t* __restrict__ words, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = {words[4 * i], words[4 * i + 1], words[4 * i + 2], words[4 * i + 3]};
  double z[4];
  normals4(v, z);
#pragma unroll
  for (int k = 0; k < 4; ++k) out[4 * i + k] = z[k];
}

// ----------------------------------------------------------------------------- launchers

hipError_t launch_gen(hipStream_t st, const SegDesc& sd, int32_t seg_id, int32_t P, int32_t n_real,
                      int32_t R_pad, int64_t real0, uint32_t k0, uint32_t k1, const double* zin,
                      int32_t zin_nseg, int32_t zin_nm, double* coef, int32_t K, double* zbuf) {
  if (R_pad % 2 != 0) return hipErrorInvalidValue;  // realization pairs
  dim3 grid((R_pad / 2 + 255) / 256, sd.nm, P);
  hipLaunchKernelGGL(k_gen, grid, dim3(256), 0, st, sd, seg_id, P, n_real, R_pad, real0, k0, k1, zin,
                     zin_nseg, zin_nm, coef, K, zbuf);
  return hipGetLastError();
}

hipError_t launch_mix(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                      double* coef, int32_t K, double* x_out) {
  const int64_t M = (int64_t)2 * sd.nm * R_pad;
  dim3 grid((unsigned)((M + 255) / 256), (P + MIX_PT - 1) / MIX_PT);
  hipLaunchKernelGGL(k_mix, grid, dim3(256), 0, st, sd.L, sd.amp, P, M, R_pad, zbuf, coef, K, sd.col0,
                     x_out);
  return hipGetLastError();
}

hipError_t launch_mix_tiled(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                            double* coef, int32_t K, double* x_out) {
  const int64_t M = (int64_t)2 * sd.nm * R_pad;  // multiple of 256: R_pad is a multiple of 128
  dim3 grid((unsigned)(M / MT_M), (P + MT_P - 1) / MT_P);
  hipLaunchKernelGGL(k_mix_tiled, grid, dim3(256), 0, st, sd.L, sd.amp, P, M, R_pad, sd.l_lower, zbuf, coef, K,
                     sd.col0, x_out);
  return hipGetLastError();
}

// k_epoch_normals_t: the same normals epoch-major, zb[b][r] (pitch ldz): one thread per (global realization pair,
// epoch pair), realization pairs fastest, so a wave's stores are contiguous. grid (ceil(pairs / 256), epoch pairs).
__global__ __launch_bounds__(256) void k_epoch_normals_t(int64_t n_blocks, int32_t n_real, int64_t real0, uint32_t k0,
                                                         uint32_t k1, double* __restrict__ zb, int64_t ldz,
                                                         int64_t npairs) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;  // realization pair
  const int64_t i = blockIdx.y;                               // epoch pair
  if (j >= npairs) return;
  const int64_t g0 = ((real0 >> 1) + j) * 2;  // even global realization of this pair
  double z[4];
  quad4((uint64_t)(2 * i), kEcorrStream, (uint64_t)g0, k0, k1, z);
  const int64_t r = g0 - real0;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    if (2 * i + e >= n_blocks) continue;
    double* row = zb + (2 * i + e) * ldz;
    if (r >= 0 && r + 1 < n_real && (r & 1) == 0) {
      *(double2*)(row + r) = make_double2(z[2 * e], z[2 * e + 1]);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (r + h >= 0 && r + h < n_real) row[r + h] = z[2 * e + h];
    }
  }
}

hipError_t launch_epoch_normals_t(hipStream_t st, int64_t n_blocks, int32_t n_real, int64_t real0, uint32_t k0,
                                  uint32_t k1, double* zb, int64_t ldz) {
  const int64_t npairs = ((real0 + n_real + 1) >> 1) - (real0 >> 1);
  if (ldz < n_real || (n_blocks + 1) / 2 > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_epoch_normals_t, dim3((unsigned)((npairs + 255) / 256), (unsigned)((n_blocks + 1) / 2)),
                     dim3(256), 0, st, n_blocks, n_real, real0, k0, k1, zb, ldz, npairs);
  return hipGetLastError();
}

hipError_t launch_epoch_normals(hipStream_t st, int64_t n_blocks, int32_t n_real, int64_t real0, uint32_t k0,
                                uint32_t k1, double* zb) {
  const int64_t npairs = ((real0 + n_real + 1) >> 1) - (real0 >> 1);
  hipLaunchKernelGGL(k_epoch_normals, dim3((unsigned)(((n_blocks + 1) / 2 + 255) / 256), (unsigned)npairs), dim3(256), 0,
                     st, n_blocks, n_real, real0, k0, k1, zb);
  return hipGetLastError();
}

hipError_t launch_white_pairs(hipStream_t st, const double* sigma, const int32_t* block_of, const double* esig,
                              int64_t n_blocks, const double* zb, double* out, int64_t ldo, int64_t n_toa,
                              int32_t n_real, int64_t real0, uint32_t k0, uint32_t k1) {
  const int64_t npairs = ((real0 + n_real - 1) >> 1) - (real0 >> 1) + 1;
  hipLaunchKernelGGL(k_white_pairs, dim3((unsigned)((n_toa + 255) / 256), (unsigned)npairs), dim3(256), 0, st, sigma,
                     n_blocks > 0 ? block_of : nullptr, esig, n_blocks > 0 ? zb : nullptr, n_blocks, out, ldo, n_toa,
                     n_real, real0, k0, k1);
  return hipGetLastError();
}

hipError_t launch_synth_direct(hipStream_t st, const SynthArgs& a) {
  dim3 grid((unsigned)((a.n_toa + 255) / 256), a.n_real);
  hipLaunchKernelGGL(k_synth_direct, grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_synth_mfma(hipStream_t st, const SynthArgs& a, const int4* tiles, int32_t n_tiles) {
  hipLaunchKernelGGL((k_synth_mfma<kWR, kWT>), dim3(n_tiles), dim3(kWaves * 64), 0, st, a, tiles);
  return hipGetLastError();
}

hipError_t launch_synth_valu(hipStream_t st, const SynthArgs& a, const int4* tiles, int32_t n_tiles, int variant) {
  switch (variant) {
#define FPTA_VALU_CASE(i)                                                                          \
  case i:                                                                                          \
    hipLaunchKernelGGL((k_synth_valu<kValuVariants[i].mt, kValuVariants[i].nt>), dim3(n_tiles), dim3(256), 0, \
                       st, a, tiles);                                                              \
    break;
    FPTA_VALU_CASE(0)
    FPTA_VALU_CASE(1)
    FPTA_VALU_CASE(2)
    FPTA_VALU_CASE(3)
    FPTA_VALU_CASE(4)
    FPTA_VALU_CASE(5)
#undef FPTA_VALU_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_seeds(hipStream_t st, const SegDesc* segs, int32_t n_seg, const int32_t* psr_of,
                        const double* toas, const double* nu, int64_t n_toa, double4* seeds) {
  hipLaunchKernelGGL(k_seeds, dim3((unsigned)((n_toa + 255) / 256), n_seg), dim3(256), 0, st, segs, psr_of, toas,
                     nu, n_toa, seeds);
  return hipGetLastError();
}

hipError_t launch_synth_valu_seeded(hipStream_t st, const SynthArgs& a, const int4* tiles, int32_t n_tiles,
                                    const double4* seeds, int variant) {
  switch (variant) {
#define FPTA_SEEDED_CASE(i)                                                                                     \
  case i:                                                                                                       \
    if (a.w_on)                                                                                                 \
      hipLaunchKernelGGL((k_synth_valu_seeded<kSeededVariants[i].mt, kSeededVariants[i].nt, true>), dim3(n_tiles), \
                         dim3(256), 0, st, a, tiles, seeds);                                                    \
    else                                                                                                        \
      hipLaunchKernelGGL((k_synth_valu_seeded<kSeededVariants[i].mt, kSeededVariants[i].nt, false>),             \
                         dim3(n_tiles), dim3(256), 0, st, a, tiles, seeds);                                     \
    break;
    FPTA_SEEDED_CASE(0)
    FPTA_SEEDED_CASE(1)
    FPTA_SEEDED_CASE(2)
    FPTA_SEEDED_CASE(3)
    FPTA_SEEDED_CASE(4)
    FPTA_SEEDED_CASE(5)
#undef FPTA_SEEDED_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_white(hipStream_t st, const double* sigma, const int32_t* block_of, const double* esig,
                        const double* z, const double* zb, double* out, int64_t ldo, int64_t n_toa,
                        int32_t n_real, int64_t real0, uint32_t k0, uint32_t k1) {
  dim3 grid((unsigned)((n_toa + 255) / 256), n_real);
  hipLaunchKernelGGL(k_white, grid, dim3(256), 0, st, sigma, block_of, esig, z, zb, out, ldo, n_toa, real0,
                     k0, k1);
  return hipGetLastError();
}

hipError_t launch_correlations(hipStream_t st, const double* out, int64_t ldo, int32_t n, int32_t P, int32_t n_real,
                               int32_t mode, double* autos, double* parts, int32_t nparts, double* dst) {
  if (mode == 2 || mode == 3) {
    hipLaunchKernelGGL(k_autos, dim3(P, n_real), dim3(256), 0, st, out, ldo, n, autos, P);
    if (mode == 3) return hipGetLastError();
  }
  const int nt = (P + XC_T - 1) / XC_T;
  const int npairs = nt * (nt + 1) / 2;
  if (mode == 0) {
    hipLaunchKernelGGL(k_xcorr, dim3(npairs, n_real), dim3(256), 0, st, out, ldo, n, P, n_real, 0, 1, autos, dst);
  } else {
    const int rper = (n_real + nparts - 1) / nparts;
    hipLaunchKernelGGL(k_xcorr, dim3(npairs, nparts), dim3(256), 0, st, out, ldo, n, P, n_real, mode, rper, autos,
                       parts);
    const int64_t len = (int64_t)P * P;
    hipLaunchKernelGGL(k_sum_parts, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, st, parts, nparts, len, dst);
  }
  return hipGetLastError();
}

hipError_t launch_checksums(hipStream_t st, const double* out, int64_t ldo, int64_t n_toa, int32_t n_real,
                            double* sums) {
  hipLaunchKernelGGL(k_checksums, dim3(n_real), dim3(256), 0, st, out, ldo, n_toa, sums);
  return hipGetLastError();
}

hipError_t launch_philox(hipStream_t st, int64_t n, const uint32_t* ctr, uint32_t k0, uint32_t k1,
                         uint32_t* out) {
  hipLaunchKernelGGL(k_philox, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, ctr, k0, k1, out);
  return hipGetLastError();
}

hipError_t launch_normals4(hipStream_t st, int64_t n, const uint32_t* words, double* out) {
  if (n <= 0 || (n + 255) / 256 > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_normals4, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, words, out);
  return hipGetLastError();
}

}  // namespace fpta
