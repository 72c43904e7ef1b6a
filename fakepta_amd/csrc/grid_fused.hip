// k_grid_fused: the whole gridded synthesis of one pulsar x kFusedReal realizations in one workgroup (C2: RN + GWB in
// one grid signal of nf = 124 points, DM in one of nf = 380; 129 KB of LDS grid for 32 realizations).
//
// The two-kernel path writes every grid (C2: 0.41 GB per block of 1024 realizations) to HBM from k_grid_dft_gen and
// reads it back in k_grid_interp_ws: with the 1.64 GB of residuals, 2.5 GB of HBM traffic per block, and the DFTs of
// block b + 1 co-run beside the interpolation of block b on the leftover registers of one wave slot per SIMD. Here the
// grid lives in LDS only; HBM sees the residual stores, the interpolation weights (read once per pulsar per XCD, the
// 32 realization blocks of a pulsar run side by side on one XCD) and the mixed common coefficients.
//
// Phases of a workgroup (8 waves, one workgroup per CU):
//  1. draws: every thread makes (mode, realization pair) coefficient pairs of every grid signal into LDS staging,
//     [2 ntq][32 realizations][cos, sin] per signal, with grid_term_coefs (k_grid_dft_gen's terms and order);
//  2. DFT: wave w takes job w = (grid signal, 32-row chunk rc of its quarter range) for both 16-realization tiles:
//     k_grid_dft_gen's MFMA k-steps per parity (A = table row pairs from global / L2, B = the (cos, sin) pair of a
//     realization from LDS), the accumulators kept in registers; a barrier (the staging may lie under the grids), then
//     k_grid_dft_gen's butterfly writes grid rows j, H + j, H - j, nf - j into LDS row lrow0 + j;
//  3. interpolation: wave w takes the pulsar's chunks c0 + w, c0 + w + 8, ...: per band step A = the dbl2 pair of
//     realizations (2 lr, 2 lr + 1) of LDS row lrows[c][4 q + lg] (one ds_read_b128), B = the weight pair of TOAs
//     (2 lr, 2 lr + 1) from global memory, four MFMAs (even / odd TOA x realization tile) as k_grid_interp_ws; the next
//     chunk's weights are loaded before this chunk's eight 16-byte stores enter the vmcnt queue.
// Every value is made by the same operations in the same order as k_grid_dft_gen (or k_grid_dft_mfma from the merged
// anchor columns) + k_grid_interp_ws: the block is bit-identical to theirs (tests/test_gpu_grid.py).
#include <hip/hip_runtime.h>
#include <algorithm>

#include "grid_device.h"

namespace fpta {

template <int NQ>
__global__ __launch_bounds__(64 * kFusedWaves, 1) void k_grid_fused(SynthArgs a, GridBand band, FusedArgs f,
                                                                    int32_t n_rb, int32_t n_items) {
  static_assert(kFusedReal == 32 && kFusedPitch == 32, "two realization tiles per LDS grid row");
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int per = (n_items + 7) >> 3;
  const int item = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // a pulsar's blocks on one XCD
  if (item >= n_items) return;  // the whole workgroup, before its first barrier
  const int p = item / n_rb, rb = item - p * n_rb;
  const int r0 = rb * kFusedReal;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;

  // 1. coefficients of every grid signal, a realization pair per thread and mode
  for (int s = 0; s < f.n_sig; ++s) {
    const FusedSig& fs = f.s[s];
    double* __restrict__ bs_lds = lds + fs.stage;
    const int n_items_s = 2 * fs.ntq * (kFusedReal / 2);
    for (int idx = threadIdx.x; idx < n_items_s; idx += 64 * kFusedWaves) {
      const int m = idx >> 4, rl = 2 * (idx & 15);
      double bc[2], bs[2];
      grid_term_coefs(fs, fs.nm, a.coef, a.K, a.R_pad, a.n_real, f.real0, f.k0, f.k1, p, m, r0 + rl, bc, bs);
      *(dbl2*)(bs_lds + 2 * (m * kFusedReal + rl)) = dbl2{bc[0], bs[0]};
      *(dbl2*)(bs_lds + 2 * (m * kFusedReal + rl + 1)) = dbl2{bc[1], bs[1]};
    }
  }
  __syncthreads();

  // 2. DFT job of this wave: grid signal js, quarter-range rows 32 jrc .. 32 jrc + 31, both realization tiles
  int js = -1, jrc = 0;
  {
    int j = wave;
    for (int s = 0; s < f.n_sig; ++s) {
      if (js < 0 && j < f.s[s].n_rc) {
        js = s;
        jrc = j;
      }
      j -= f.s[s].n_rc;
    }
  }
  js = __builtin_amdgcn_readfirstlane(js);
  jrc = __builtin_amdgcn_readfirstlane(jrc);
  d4 C[2][2][2], S[2][2][2];  // [parity: 0 odd k, 1 even k][row tile h: rows 2 i + h][realization tile t]
  if (js >= 0) {
    const FusedSig& fs = f.s[js];
    const int j0 = 32 * jrc;
    const double* __restrict__ bsrc = lds + fs.stage;
    const int64_t tstride = (int64_t)fs.ntq * fs.ldq;
    const int n_par[2] = {(fs.nm + 1) >> 1, fs.nm >> 1};  // modes of odd k (m = 2 t) and of even k (m = 2 t + 1)
#pragma unroll
    for (int par = 0; par < 2; ++par) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int t = 0; t < 2; ++t) C[par][h][t] = S[par][h][t] = d4{0.0, 0.0, 0.0, 0.0};
      const double* __restrict__ tc = fs.tq + (int64_t)(2 * par) * tstride + (int64_t)lg * fs.ldq + j0 + 2 * lr;
      const double* __restrict__ ts = tc + tstride;
      const int nq = (n_par[par] + 3) >> 2;
      // operands of step q + 1 in flight while step q's MFMAs run (two sets, alternating)
      struct Ops {
        dbl2 ac, as, b[2];
      };
      auto fetch = [&](int q, Ops& o) {
        const int qq = min(q, nq - 1);
        o.ac = *(const dbl2*)(tc + (int64_t)(4 * qq) * fs.ldq);
        o.as = *(const dbl2*)(ts + (int64_t)(4 * qq) * fs.ldq);
        const double* bm = bsrc + 2 * ((2 * (4 * qq + lg) + par) * kFusedReal + lr);
        o.b[0] = *(const dbl2*)bm;
        o.b[1] = *(const dbl2*)(bm + 2 * 16);
      };
      auto mfma = [&](const Ops& o) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          C[par][0][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac.x, o.b[t].x, C[par][0][t], 0, 0, 0);
          C[par][1][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.ac.y, o.b[t].x, C[par][1][t], 0, 0, 0);
          S[par][0][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.as.x, o.b[t].y, S[par][0][t], 0, 0, 0);
          S[par][1][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(o.as.y, o.b[t].y, S[par][1][t], 0, 0, 0);
        }
      };
      if (nq > 0) {
        Ops o0, o1;
        fetch(0, o0);
        for (int q = 0; q < nq; q += 2) {
          fetch(q + 1, o1);
          mfma(o0);
          if (q + 1 < nq) {
            fetch(q + 2, o0);
            mfma(o1);
          }
        }
      }
    }
  }
  __syncthreads();  // every staging read is done: the grids may overlay the staging
  if (js >= 0) {
    const FusedSig& fs = f.s[js];
    const int j0 = 32 * jrc;
    const int nf = fs.nf, Q = nf >> 2, H = nf >> 1;
    double* __restrict__ gcol = lds + (int64_t)fs.lrow0 * kFusedPitch + lr;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = j0 + 2 * (lg + 4 * g) + h;
        if (j > Q) continue;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const double oc = C[0][h][t][g], os = S[0][h][t][g], ec = C[1][h][t][g], es = S[1][h][t][g];
          const double pe = ec + es, me = ec - es, po = oc + os, mo = oc - os;
          gcol[j * kFusedPitch + 16 * t] = pe + po;
          gcol[(H + j) * kFusedPitch + 16 * t] = pe - po;
          if (j > 0 && j < Q) {
            gcol[(H - j) * kFusedPitch + 16 * t] = me - mo;
            gcol[(nf - j) * kFusedPitch + 16 * t] = me + mo;
          }
        }
      }
  }
  __syncthreads();

  // 3. the pulsar's chunks, wave w: c0 + w, c0 + w + kFusedWaves, ...
  const int c_end = ld_uniform(f.psr_c0 + p + 1);
  int c = ld_uniform(f.psr_c0 + p) + wave;
  if (c >= c_end) return;
  struct Ops {
    int4 ci;
    int nq;
    dbl2 b[NQ];
    int row[NQ];  // LDS offset (doubles) of band row 4 (q0 + q) + lg, realization pair 2 lr
  };
  // operands of band steps q0 .. q0 + NQ - 1 of chunk cc (steps past nq re-load the last one, never used)
  auto load = [&](int cc, int q0, Ops& o) {
    o.ci = ld_uniform4(band.chunks + cc);
    o.nq = __builtin_amdgcn_readfirstlane(o.ci.w) >> 2;
    FPTA_DCHECK(o.nq > 0, "k_grid_fused band steps", o.nq, 1 << 20);
    const int32_t* __restrict__ rt = f.lrows + (int64_t)cc * band.vmax;
    const double* __restrict__ wp = band.wd + ((int64_t)cc * band.vmax + lg) * kGridTT + 2 * lr;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int qq = min(q0 + q, o.nq - 1);
      const int4 r4 = ld_uniform4(rt + 4 * qq);
      o.row[q] = (lg == 0 ? r4.x : lg == 1 ? r4.y : lg == 2 ? r4.z : r4.w) * kFusedPitch + 2 * lr;
      o.b[q] = *(const dbl2*)(wp + 4 * kGridTT * qq);
    }
  };
  Ops cur, nxt;
  load(c, 0, cur);
  d4 acc[2][2];  // [TOA parity][realization tile]
  while (true) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
    for (int q0 = 0;; q0 += NQ) {
      // step q's A operand is read from LDS ahead of step q - 1's MFMAs (rows past nq are valid clamped rows)
      dbl2 an = *(const dbl2*)(lds + cur.row[0]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q0 + q < cur.nq) {
          const dbl2 av = an;
          if (q + 1 < NQ) an = *(const dbl2*)(lds + cur.row[q + 1]);
          const dbl2 bv = cur.b[q];
          acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.y, acc[1][1], 0, 0, 0);
        }
      }
      if (q0 + NQ >= cur.nq) break;
      load(c, q0 + NQ, cur);  // a chunk wider than NQ steps (sparse pulsars): its next steps' operands
    }
    InterpTile<2> t;
    t.c = c;
    t.p = p;
    t.r0 = r0;
    t.y = cur.ci.y;
    t.cnt = cur.ci.z;
    t.nq = cur.nq;
    // next chunk: its operands are in flight before this chunk's stores enter the vmcnt queue
    c += kFusedWaves;
    const bool more = c < c_end;
    if (more) load(c, 0, nxt);
    __builtin_amdgcn_sched_barrier(0);
    interp_store_rows<2>(a, a.out, t, acc);
    if (!more) break;
    cur = nxt;
  }
}

hipError_t launch_grid_fused(hipStream_t st, const SynthArgs& a, const GridBand& band, const FusedArgs& f,
                             int32_t nq_max, size_t lds_bytes) {
  if (band.n_chunks <= 0 || band.vmax < 4 || band.vmax % 4 != 0 || a.R_pad % kFusedReal != 0 || a.w_on ||
      a.accumulate || a.part || !f.lrows || !f.psr_c0 || f.n_sig <= 0 || f.n_sig > kFusedMaxSig ||
      lds_bytes > (size_t)kFusedLdsMax || nq_max <= 0)
    return hipErrorInvalidValue;
  int jobs = 0;
  for (int s = 0; s < f.n_sig; ++s) {
    const FusedSig& fs = f.s[s];
    if (fs.nf % 4 != 0 || !fs.tq || fs.n_rc != (fs.nf / 4 + 32) / 32 || fs.ldq < 32 * fs.n_rc ||
        fs.ntq < ((((fs.nm + 1) >> 1) + 3) & ~3) || fs.n_terms <= 0 || fs.n_terms > kDftGenTerms ||
        fs.lrow0 < 0 || fs.stage < 0 ||
        (size_t)(fs.stage + 2 * fs.ntq * kFusedReal * 2) * sizeof(double) > lds_bytes ||
        (size_t)(fs.lrow0 + fs.nf) * kFusedPitch * sizeof(double) > lds_bytes)
      return hipErrorInvalidValue;
    for (int i = 0; i < fs.n_terms; ++i)
      if (fs.term_nm[i] <= 0 || fs.term_nm[i] > fs.nm || (fs.term_kind[i] == 0 && !fs.term_amp[i]) ||
          (fs.term_kind[i] == 1 && (!a.coef || fs.term_col0[i] < 0 || fs.term_col0[i] + 2 * fs.term_nm[i] > a.K)))
        return hipErrorInvalidValue;
    jobs += fs.n_rc;
  }
  if (jobs > kFusedWaves) return hipErrorInvalidValue;
  const int32_t n_rb = a.R_pad / kFusedReal;
  const int64_t items = (int64_t)a.P * n_rb;
  if (items > 0x7FFFFFFF || items <= 0) return hipErrorInvalidValue;
  const int64_t grid = (items + 7) / 8 * 8;
  // NQ: band steps whose operands a wave holds (a wider chunk takes them NQ at a time)
  auto kernel = nq_max <= 8 ? k_grid_fused<8> : k_grid_fused<12>;
  static bool attr_set[2] = {false, false};
  const int ki = nq_max <= 8 ? 0 : 1;
  if (!attr_set[ki]) {  // dynamic LDS beyond 64 KB
    hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLdsMax);
    if (e != hipSuccess) return e;
    attr_set[ki] = true;
  }
  hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(64 * kFusedWaves), lds_bytes, st, a, band, f, n_rb,
                     (int32_t)items);
  return hipGetLastError();
}

}  // namespace fpta
