// k_grid_fused_w: k_grid_fused for gridded blocks with white noise / ECORR (C5: RN + the HD, monopole and dipole
// common signals in one grid signal of nf = 124, DM and Sv in two of nf = 380, white + ECORR: 884 grid rows).
//
// The two-kernel white path writes every grid (C5: 0.72 GB per block of 1024 realizations) from three k_grid_dft_gen
// launches and reads it back in k_grid_interp_mfma<true, ..>, whose 256-VGPR waves leave no room beside them: the
// next block's DFTs ran after the interpolation, not beside it. Here, as in k_grid_fused, the grids live in LDS only:
// items are (pulsar, kFusedWReal = 16 realizations) so that C5's three grids (113 KB) fit beside a draw ring of
// 32-mode groups (48 KB).
//
// Roles (one wave of each per SIMD, one workgroup per CU, items from per-XCD ticket queues):
//  * DFT waves: up to two 32-row quarter-range jobs each (C5: seven jobs). Ring iteration g draws 32-mode group g + 1
//    of every grid signal (one (mode, realization pair) per lane: k_grid_dft_gen's terms and order) while the wave's
//    MFMAs run group g of its jobs in four units of two k-steps (a unit's table operands loaded one unit ahead), and
//    write the next item's grids at the item boundary; they interpolate chunks of the current item first while
//    enough are left (FusedArgs::join_reserve).
//  * interpolation waves: per band step A = the grid value of the lane's realization (LDS column w_col(lr)), B = the
//    weights of TOAs (2 lr, 2 lr + 1), two MFMAs; even and odd steps on separate accumulators (four independent chains,
//    added at the end). Then the white epilogue: sigma z (one Philox call per TOA pair and realization pair, the
//    white stream of k_grid_interp_mfma<true, ..>) and ECORR from the block's epoch normals, as interp_white; 16-byte
//    stores.
// Sums agree with the two-kernel white path to rounding (the band steps are summed in two chains); the white and
// ECORR terms are the same operations on the same normals (tests/test_gpu_fused_w.py). DESIGN.md §5a.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <atomic>

#include "fused_device.h"

namespace fpta {

namespace {

// members of a grid signal whose draw inputs the DFT waves load with the iteration's other loads (the others: inline)
constexpr int kFusedWTerms = 1;
#ifndef FPTA_W_JOIN
#define FPTA_W_JOIN 1
#endif
#ifndef FPTA_W_AHEAD
#define FPTA_W_AHEAD 1  // interpolation band steps between an A operand's LDS read and its MFMAs
#endif
#ifndef FPTA_W_PAIRS_TOGETHER
#define FPTA_W_PAIRS_TOGETHER 0  // 1: the two realization pairs' white-noise Philox rounds scheduled together
#endif

// A row i of the interpolation MFMA reads LDS column (realization) w_col(i): D register g of lane (lr, lg) (row
// lg + 4 g) is then realization w_real(lg, g) = 2 lg + 8 (g >> 1) + (g & 1), so a lane holds the realization pairs
// (2 lg, 2 lg + 1) and (8 + 2 lg, 9 + 2 lg): one white-noise Philox call per (TOA pair, realization pair)
__device__ __forceinline__ int w_col(int i) { return 2 * (i & 3) + 8 * (i >> 3) + ((i >> 2) & 1); }
__device__ __forceinline__ int w_real(int lg, int g) { return 2 * lg + 8 * (g >> 1) + (g & 1); }

template <int NS>
struct WOps {
  int c;        // chunk (wave-uniform)
  i32x4 ci;     // band.chunks[c] {pulsar, first TOA, count, band rows}
  dbl2 b[NS];   // weights of TOAs (2 lr, 2 lr + 1) at band row 4 q + lg
  int row[NS];  // LDS grid row of band row 4 q + lg
};

// white-stream normals of TOAs t, t + 1 and realizations g, g + 1 (k_grid_interp_mfma's white_quad: one Philox call
// when t and g are even, the misaligned case one call per value)
__device__ __attribute__((noinline)) double w_white_one(uint64_t t, uint64_t g, uint32_t k0, uint32_t k1) {
  return quad_normal(t, kWhiteStream, g, k0, k1);
}
__device__ __forceinline__ void w_white_quad(int64_t t, int64_t g, uint32_t k0, uint32_t k1, double (&z)[4]) {
  if (((t | g) & 1) == 0) {
    quad4((uint64_t)t, kWhiteStream, (uint64_t)g, k0, k1, z);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = w_white_one((uint64_t)(t + (i >> 1)), (uint64_t)(g + (i & 1)), k0, k1);
  }
}

}  // namespace

template <int NQ, bool ODD>
__global__ __launch_bounds__(64 * (kFusedIW + kFusedDW), 1) void k_grid_fused_w(SynthArgs a, GridBand band,
                                                                               FusedArgs f, int32_t n_rb,
                                                                               int32_t n_items) {
  static_assert(kFusedWReal == 16 && kFusedWPitch == 16 && kFusedWGroupModes * kFusedWReal / 2 == 64 * kFusedDW,
                "one realization tile; one (mode, realization pair) of a 32-mode group per DFT lane");
  // [grid rows][16] | ring [2][kFusedWMaxSig][kFusedWSlot] | sync word, 3 pad | item ring [4] | chunk tickets [2], 2 pad
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const FusedQueue queue(n_items, f.queue);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  double* __restrict__ ring = lds + f.ring_off;
  uint32_t* sync = (uint32_t*)(ring + 2 * kFusedWMaxSig * kFusedWSlot);
  volatile int* qitem = (volatile int*)(sync + 4);
  if (threadIdx.x == 0) {
    *sync = 0u;
    ((volatile int*)sync)[8] = 0;
    ((volatile int*)sync)[9] = 0;
    qitem[0] = queue.fetch();
    qitem[1] = qitem[0] >= 0 ? queue.fetch() : -1;
  }
  __syncthreads();
  auto item_of = [&](int k) { return __builtin_amdgcn_readfirstlane(qitem[k & 3]); };
  auto finish = [&]() {
    if (threadIdx.x == 0) {
      __threadfence();
      const uint32_t done = __hip_atomic_fetch_add(f.queue + 8, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (done == gridDim.x - 1)
        for (int i = 0; i < kFusedQueueWords; ++i)
          __hip_atomic_store(f.queue + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  if (item_of(0) < 0) {
    finish();
    return;
  }

  // ------------------------------------------------------------------ chunks (both roles), as k_grid_fused
  volatile int* ccnt = (volatile int*)(sync + 8);
  struct Geo {
    int p, r0, c0, n;
    int64_t toa0;
    bool valid;
  };
  auto geo = [&](int k) {
    Geo g;
    const int item = item_of(k);
    g.valid = item >= 0;
    const int it = g.valid ? item : 0;
    g.p = it / n_rb;
    g.r0 = (it - g.p * n_rb) * kFusedWReal;
    g.c0 = ld_uniform(f.psr_c0 + g.p);
    g.n = g.valid ? ld_uniform(f.psr_c0 + g.p + 1) - g.c0 : 0;
    g.toa0 = ld_uniform(a.offs + g.p);
    return g;
  };
  auto ticket = [&](int k) {
    int t = 0;
    if (lane == 0)
      t = __hip_atomic_fetch_add((int*)ccnt + (k & 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return __builtin_amdgcn_readfirstlane(t);
  };
  auto lane_now = [&]() {
    int v = lane;
    asm volatile("" : "+v"(v));
    return v;
  };
  using Ops = WOps<NQ>;
  auto load = [&](int cc, Ops& o, int ln) {
    o.c = cc;
    o.ci = *(const i32x4*)(band.chunks + cc);
    const int lgo = ln >> 4, lro = ln & 15;
    const i32x4* __restrict__ rt = (const i32x4*)(f.lrows + ((int64_t)cc * 4 + lgo) * f.fq);
    const double* __restrict__ wp = band.wd + ((int64_t)cc * band.vmax + lgo) * kGridTT + 2 * lro;
#pragma unroll
    for (int q4 = 0; q4 < NQ / 4; ++q4) {
      const i32x4 r4 = rt[q4];
      o.row[4 * q4] = r4.x;
      o.row[4 * q4 + 1] = r4.y;
      o.row[4 * q4 + 2] = r4.z;
      o.row[4 * q4 + 3] = r4.w;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) o.b[q] = *(const dbl2*)(wp + 4 * kGridTT * q);
  };
  // A chunk is processed in two parts, so that one operand set suffices: mfma_chunk (the band steps of chunk cur into
  // sum), then the next chunk's operands are loaded into the same registers, then epilogue (white noise + ECORR + the
  // stores of sum), whose Philox rounds cover those loads' latency; the loads precede the stores in the vmcnt queue.
  auto mfma_chunk = [&](const Ops& cur, int ln, d4 (&sum)[2], auto& pf) {
    const int lgl = ln >> 4, lrl = ln & 15;
    const int col = w_col(lrl);
    const int nq = __builtin_amdgcn_readfirstlane(cur.ci.w) >> 2;
    FPTA_DCHECK(nq > 0, "k_grid_fused_w band steps", nq, 1 << 20);
    d4 acc[2][2];  // [TOA parity][step parity]
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
    {
      // step q's A operand read from LDS kWAhead steps ahead (rows past nq are valid repeated rows)
      constexpr int DA = FPTA_W_AHEAD;
      double an[NQ];
#pragma unroll
      for (int q = 0; q < DA && q < NQ; ++q) an[q] = lds[cur.row[q] * kFusedWPitch + col];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q < nq) {
          if (q + DA < NQ) an[q + DA] = lds[cur.row[q + DA] * kFusedWPitch + col];
          const dbl2 bv = cur.b[q];
          acc[0][q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[q], bv.x, acc[0][q & 1], 0, 0, 0);
          acc[1][q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[q], bv.y, acc[1][q & 1], 0, 0, 0);
        }
      }
    }
    // a chunk wider than NQ steps: its further steps one at a time
    for (int q = NQ; q < nq; ++q) {
      const int v = 4 * q + lgl;
      const int row = f.lrows[((int64_t)cur.c * 4 + lgl) * f.fq + q];
      const dbl2 bv = *(const dbl2*)(band.wd + ((int64_t)cur.c * band.vmax + v) * kGridTT + 2 * lrl);
      const double av = lds[row * kFusedWPitch + col];
      acc[0][q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv.x, acc[0][q & 1], 0, 0, 0);
      acc[1][q & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv.y, acc[1][q & 1], 0, 0, 0);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) sum[e] = acc[e][0] + acc[e][1];
    pf.lap(1);
  };
  // The epilogue's inputs, loaded without conditions (absent white noise or ECORR reads a valid dummy address and
  // selects zero afterwards: a load under a branch makes the compiler's vmcnt waits after the join wait for everything):
  // epi_toa before the chunk's MFMAs (sigma and epoch of the lane's TOAs), epi_gather right after them (the epoch's
  // ECORR sigma and normals, which depend on the epoch), so both land while the next chunk's operand loads (issued
  // after them) are in flight.
  struct Epi {
    double sg[2], es[2], zb[2][2][2];  // zb [realization pair j][TOA e][realization of the pair h]
    int ep[2];
  };
  auto epi_toa = [&](const Geo& g, int ty, int tc, int ln, Epi& x) {
    const int tt = 2 * (ln & 15);
    const int64_t tg = g.toa0 + ty + min(tt, tc - 1);
    const int64_t t1 = g.toa0 + ty + min(tt + 1, tc - 1);
    const double* sp = a.w_sigma ? a.w_sigma : a.toas;
    const int32_t* bp = a.w_block_of ? a.w_block_of : a.psr_of;
    const double s0 = ld_global(sp + tg), s1 = ld_global(sp + t1);
    const int b0 = ld_global(bp + tg), b1 = ld_global(bp + t1);
    x.sg[0] = a.w_sigma ? s0 : 0.0;
    x.sg[1] = a.w_sigma && tt + 1 < tc ? s1 : 0.0;
    x.ep[0] = a.w_block_of ? b0 : -1;
    x.ep[1] = a.w_block_of && tt + 1 < tc ? b1 : -1;
  };
  // epoch normals epoch-major (SynthArgs::w_zb_ld, launch_epoch_normals_t): a realization pair of an epoch is one
  // 16-byte load (padding realizations past n_real are read, never stored)
  auto epi_gather = [&](const Geo& g, int ln, Epi& x) {
    const int lgl = ln >> 4;
    const bool ecorr = a.w_block_of != nullptr;
    const double* ebase = ecorr ? a.w_esig : a.toas;
    const double* zbase = ecorr ? a.w_zb : a.toas;
    const int64_t ld = ecorr ? a.w_zb_ld : 0;
    const int64_t e0 = x.ep[0] >= 0 ? x.ep[0] : 0, e1 = x.ep[1] >= 0 ? x.ep[1] : 0;
    const double q0 = ld_global(ebase + e0), q1 = ld_global(ebase + e1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t r = ecorr ? g.r0 + w_real(lgl, 2 * j) : 0;
      const dbl2 z0 = ld_global((const dbl2*)(zbase + e0 * ld + r));
      const dbl2 z1 = ld_global((const dbl2*)(zbase + e1 * ld + r));
      x.zb[j][0][0] = z0.x;
      x.zb[j][0][1] = z0.y;
      x.zb[j][1][0] = z1.x;
      x.zb[j][1][1] = z1.y;
    }
    x.es[0] = x.ep[0] >= 0 ? q0 : 0.0;
    x.es[1] = x.ep[1] >= 0 ? q1 : 0.0;
  };
  // white noise + ECORR (interp_white's operations: sigma z, then ecorr zb) and the stores of chunk (first TOA ty,
  // count tc) of item g. Lane TOAs tg, tg + 1; realization pairs (2 lg, 2 lg + 1) and (8 + 2 lg, 9 + 2 lg) of the item
  // (registers 0, 1 and 2, 3).
  auto epilogue = [&](const Geo& g, int ty, int tc, int ln, d4 (&sum)[2], const Epi& x, auto& pf) {
    const int lgl = ln >> 4, lrl = ln & 15;
    const int tt = 2 * lrl;
    const int64_t t0 = g.toa0 + ty;
    if (tt < tc) {
      const int64_t tg = t0 + tt;
      const bool ecorr = a.w_block_of != nullptr;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int rl = g.r0 + w_real(lgl, 2 * j);  // even realization of the pair
        if (a.w_sigma) {
          double z[4];
          w_white_quad(tg, a.real0 + rl, a.k0, a.k1, z);
#pragma unroll
          for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int h = 0; h < 2; ++h) sum[e][2 * j + h] = fma(x.sg[e], z[2 * e + h], sum[e][2 * j + h]);
        }
        if (ecorr) {
#pragma unroll
          for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int h = 0; h < 2; ++h) sum[e][2 * j + h] = fma(x.es[e], x.zb[j][e][h], sum[e][2 * j + h]);
        }
        if (!FPTA_W_PAIRS_TOGETHER) __builtin_amdgcn_sched_barrier(0);  // one pair at a time (register budget)
      }
    }
    // stores: a full chunk, every realization of the item, 16-byte aligned rows: four 16-byte non-temporal stores
    if (tc == kGridTT && g.r0 + kFusedWReal <= a.n_real && ((t0 | a.ldo) & 1) == 0 && a.ldo < ((int64_t)1 << 26)) {
      const char* base = (const char*)(a.out + t0 + (int64_t)g.r0 * a.ldo);
#pragma unroll
      for (int gg = 0; gg < 4; ++gg)
        __builtin_nontemporal_store(
            dbl2{sum[0][gg], sum[1][gg]},
            (dbl2*)((char*)base + ((int64_t)w_real(lgl, gg) * a.ldo + tt) * 8));
    } else if (tt < tc) {
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int r = g.r0 + w_real(lgl, gg);
        if (r >= a.n_real) continue;
        double* o = a.out + t0 + tt + (int64_t)r * a.ldo;
        o[0] = sum[0][gg];
        if (tt + 1 < tc) o[1] = sum[1][gg];
      }
    }
    pf.lap(2);
  };

  if (wave >= kFusedIW) {
    // ---------------------------------------------------------------- DFT waves
    const int dw = wave - kFusedIW;
    __builtin_amdgcn_s_setprio(3);
    Prof pf;  // -DFPTA_FUSED_PROF: 0 loads issue, 1 MFMA steps (DFT units and joined chunks), 2 ring sync / joined
              // chunks' epilogues, 3 grid writes, 4 barriers, 5 iterations, 6 draws, 7 joined chunks (count)
    pf.start();
    // this wave's jobs: u = 0 job dw, u = 1 job dw + kFusedDW (grid signal js[u], quarter-range rows 32 jrc[u] ..)
    int js[2] = {-1, -1}, jrc[2] = {0, 0};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int j = dw + kFusedDW * u;
#pragma unroll
      for (int s = 0; s < kFusedWMaxSig; ++s) {
        if (s < f.n_sig && js[u] < 0 && j < f.s[s].n_rc) {
          js[u] = s;
          jrc[u] = j;
        }
        if (s < f.n_sig) j -= f.s[s].n_rc;
      }
      js[u] = __builtin_amdgcn_readfirstlane(js[u]);
      jrc[u] = __builtin_amdgcn_readfirstlane(jrc[u]);
    }
    uint32_t epoch = 0;
    auto dsync = [&]() {
      fused_wait_lgkm0();
      if (lane == 0) __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      epoch += kFusedDW;
      while ((uint32_t)__builtin_amdgcn_readfirstlane(
                 (int)__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < epoch)
        __builtin_amdgcn_s_sleep(1);
    };
    // groups of 32 modes (four 4-mode k-steps of both parities)
    auto n_groups = [&](int nm) { return (nm + kFusedWGroupModes - 1) / kFusedWGroupModes; };
    int ng[kFusedWMaxSig];
    int n_it = 0;
#pragma unroll
    for (int s = 0; s < kFusedWMaxSig; ++s) {
      ng[s] = s < f.n_sig ? n_groups(f.s[s].nm) : 0;
      n_it = max(n_it, ng[s]);
    }
    // per job: k-steps per parity, the table base (re-derived where used: see k_grid_fused)
    int jnq0[2], jnq1[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const FusedSig& jf = f.s[js[u] < 0 ? 0 : js[u]];
      jnq0[u] = js[u] < 0 ? 0 : (((jf.nm + 1) >> 1) + 3) >> 2;
      jnq1[u] = js[u] < 0 ? 0 : ((jf.nm >> 1) + 3) >> 2;
    }
    auto jtab = [&](int u, int q, int par, dbl2& ac, dbl2& as) {  // table operands of job u's k-step q (clamped)
      const FusedSig& jf = f.s[js[u] < 0 ? js[0] : js[u]];
      const int jr = js[u] < 0 ? jrc[0] : jrc[u];
      const int ln = lane_now();
      const int64_t jts = (int64_t)jf.ntq * jf.ldq;
      const int qc = max(0, min(q, (js[u] < 0 ? jnq0[0] : jnq0[u]) - 1));
      const double* __restrict__ tc =
          jf.tq + (int64_t)(ln >> 4) * jf.ldq + 32 * jr + 2 * (ln & 15) + (int64_t)(2 * par) * jts + (int64_t)qc * 4 * jf.ldq;
      ac = ld_global((const dbl2*)tc);
      as = ld_global((const dbl2*)(tc + jts));
    };
    d4 C[2][2][2], S[2][2][2];  // [job][parity: 0 odd k, 1 even k][row tile h: rows 2 i + h]
    struct DrawIn {
      dbl2 x0[kFusedWTerms], x1[kFusedWTerms];
    };
    auto draw_load = [&](const FusedSig& fs, int g, int p, int r0, DrawIn& in) {
      const int didx = dw * 64 + lane_now(), dmm = didx >> 3, drl = 2 * (didx & 7);
      const int m = kFusedWGroupModes * g + dmm, r = r0 + drl;
#pragma unroll
      for (int i = 0; i < kFusedWTerms; ++i) {
        const bool on = i < fs.n_terms;
        const int nmi = on ? fs.term_nm[i] : 2;
        const int mi = min(m, nmi - 1);
        const double* src0;
        int64_t step;
        if (on && fs.term_kind[i] == 1) {
          src0 = a.coef + ((int64_t)p * a.K + fs.term_col0[i] + 2 * mi) * a.R_pad + r;
          step = a.R_pad;
        } else {
          src0 = (on ? fs.term_amp[i] : a.coef) + (int64_t)p * nmi + (mi & ~1);
          step = 0;
        }
        in.x0[i] = ld_global((const dbl2*)src0);
        in.x1[i] = ld_global((const dbl2*)(src0 + step));
      }
    };
    auto draw_finish = [&](const FusedSig& fs, int g, int p, int r0, double* __restrict__ slot_s, const DrawIn& in) {
      const int didx = dw * 64 + lane_now(), dmm = didx >> 3, drl = 2 * (didx & 7);
      const int m = kFusedWGroupModes * g + dmm, r = r0 + drl;
      const uint64_t gr = (uint64_t)(f.real0 + r);
      double bc[2] = {0.0, 0.0}, bs[2] = {0.0, 0.0};
      bool first = true;
      auto add = [&](bool use, const double (&pc)[2], const double (&ps)[2]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          bc[h] = use ? (first ? pc[h] : bc[h] + pc[h]) : bc[h];
          bs[h] = use ? (first ? ps[h] : bs[h] + ps[h]) : bs[h];
        }
        first = first && !use;
      };
      const bool ok0 = r < a.n_real, ok1 = r + 1 < a.n_real;
      auto normals = [&](int seg, double (&z)[4]) {
        if (!ODD) {
          gp_pair2((uint32_t)m, (uint32_t)p, (uint32_t)seg, gr, f.k0, f.k1, z);
        } else {
          gp_normal2((uint32_t)m, (uint32_t)p, (uint32_t)seg, gr, f.k0, f.k1, z[0], z[1]);
          gp_normal2((uint32_t)m, (uint32_t)p, (uint32_t)seg, gr + 1, f.k0, f.k1, z[2], z[3]);
        }
        z[0] = ok0 ? z[0] : 0.0;
        z[1] = ok0 ? z[1] : 0.0;
        z[2] = ok1 ? z[2] : 0.0;
        z[3] = ok1 ? z[3] : 0.0;
      };
#pragma unroll
      for (int i = 0; i < kFusedWTerms; ++i) {
        if (i >= fs.n_terms) continue;
        double pc[2], ps[2];
        if (fs.term_kind[i] == 0) {
          double z[4];
          normals(fs.term_seg[i], z);
          const double amp = (m & 1) ? in.x0[i].y : in.x0[i].x;
          pc[0] = opaque(amp * z[0]);
          ps[0] = opaque(amp * z[1]);
          pc[1] = opaque(amp * z[2]);
          ps[1] = opaque(amp * z[3]);
        } else {
          pc[0] = in.x0[i].x;
          pc[1] = in.x0[i].y;
          ps[0] = in.x1[i].x;
          ps[1] = in.x1[i].y;
        }
        add(m < fs.nm && m < fs.term_nm[i], pc, ps);
      }
      for (int i = kFusedWTerms; i < fs.n_terms; ++i) {
        const int mi = min(m, fs.term_nm[i] - 1);
        double pc[2], ps[2];
        if (fs.term_kind[i] == 0) {
          double z[4];
          normals(fs.term_seg[i], z);
          const double amp = ld_global(fs.term_amp[i] + (int64_t)p * fs.term_nm[i] + mi);
          pc[0] = opaque(amp * z[0]);
          ps[0] = opaque(amp * z[1]);
          pc[1] = opaque(amp * z[2]);
          ps[1] = opaque(amp * z[3]);
        } else {
          const double* cp = a.coef + ((int64_t)p * a.K + fs.term_col0[i] + 2 * mi) * a.R_pad + r;
          const dbl2 vc = ld_global((const dbl2*)cp), vs = ld_global((const dbl2*)(cp + a.R_pad));
          pc[0] = vc.x;
          pc[1] = vc.y;
          ps[0] = vs.x;
          ps[1] = vs.y;
        }
        add(m < fs.nm && m < fs.term_nm[i], pc, ps);
      }
      double* __restrict__ dst = slot_s + 2 * (dmm * kFusedWReal + drl);
      *(dbl2*)dst = dbl2{bc[0], bs[0]};
      *(dbl2*)(dst + 2) = dbl2{bc[1], bs[1]};
    };
    auto slot_of = [&](int k, int s) { return ring + ((k & 1) * kFusedWMaxSig + s) * kFusedWSlot; };
    // A unit is one k-step (h4) of both parities of one job (u = unit >> 2): q = 4 g + h4
    struct Tabs {
      dbl2 ac[2], as[2];  // [parity]
    };
    auto unit_tables = [&](int g, int unit, Tabs& tb) {
      const int u = unit >> 2, h4 = unit & 3;
#pragma unroll
      for (int par = 0; par < 2; ++par) jtab(u, 4 * g + h4, par, tb.ac[par], tb.as[par]);
    };
    auto unit_steps = [&](int slot, int g, int unit, const Tabs& tb) {
      const int u = unit >> 2, h4 = unit & 3;
      if (js[u] < 0) return;
      const double* __restrict__ bsrc = slot_of(slot, js[u]);
      const int q = 4 * g + h4;
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        if (q >= (par ? jnq1[u] : jnq0[u])) continue;
        const dbl2 ac = tb.ac[par], as = tb.as[par];
        // mode 32 g + 2 (4 h4 + lg) + par = 2 (4 q + lg) + par of the group, realization lr
        const dbl2 bv = *(const dbl2*)(bsrc + 2 * ((2 * (4 * h4 + lg) + par) * kFusedWReal + lr));
        C[u][par][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac.x, bv.x, C[u][par][0], 0, 0, 0);
        C[u][par][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac.y, bv.x, C[u][par][1], 0, 0, 0);
        S[u][par][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(as.x, bv.y, S[u][par][0], 0, 0, 0);
        S[u][par][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(as.y, bv.y, S[u][par][1], 0, 0, 0);
      }
    };
    int sb = 0;
    auto build = [&](int k) {
      const int item = item_of(k);
      const int p = item / n_rb, r0 = (item - p * n_rb) * kFusedWReal;
      const int item1n = item_of(k + 1);
      const bool nx = item1n >= 0;
      const int item1 = nx ? item1n : item;
      const int p1 = item1 / n_rb, r1 = (item1 - p1 * n_rb) * kFusedWReal;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int par = 0; par < 2; ++par)
#pragma unroll
          for (int h = 0; h < 2; ++h) C[u][par][h] = S[u][par][h] = d4{0.0, 0.0, 0.0, 0.0};
      if (k == 0) {
#pragma unroll
        for (int s = 0; s < kFusedWMaxSig; ++s) {
          if (s >= f.n_sig) continue;
          DrawIn in;
          draw_load(f.s[s], 0, p, r0, in);
          draw_finish(f.s[s], 0, p, r0, slot_of(sb, s), in);
        }
        dsync();
        pf.lap(2);
      }
      Tabs tb[2];
      unit_tables(0, 0, tb[0]);
      for (int g = 0; g < n_it; ++g) {
        const bool last = g + 1 == n_it;
        const int dp = last ? p1 : p, dr = last ? r1 : r0;
        DrawIn in[kFusedWMaxSig];
#pragma unroll
        for (int s = 0; s < kFusedWMaxSig; ++s)  // an unused descriptor is a copy of the first
          draw_load(f.s[s], last ? 0 : min(g + 1, max(ng[s], 1) - 1), dp, dr, in[s]);
        pf.lap(0);
        // eight units (four k-steps of each job), each one's tables loaded before the previous one's MFMAs (the next
        // iteration's first unit during this one's last)
#pragma unroll
        for (int unit = 0; unit < 8; ++unit) {
          if (unit < 7)
            unit_tables(g, unit + 1, tb[(unit + 1) & 1]);
          else
            unit_tables(g + 1 < n_it ? g + 1 : g, 0, tb[0]);
          unit_steps(sb + g, g, unit, tb[unit & 1]);
        }
        pf.lap(1);
#pragma unroll
        for (int s = 0; s < kFusedWMaxSig; ++s)
          if (last ? nx && s < f.n_sig : g + 1 < ng[s])
            draw_finish(f.s[s], last ? 0 : g + 1, dp, dr, slot_of(sb + g + 1, s), in[s]);
        pf.lap(6);
        dsync();
        pf.lap(2);
        pf.count(5);
      }
      sb = (sb + n_it) & 1;
    };
    auto write_grid = [&]() {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (js[u] < 0) continue;
        const FusedSig& jf = f.s[js[u]];
        const int j0 = 32 * jrc[u];
        const int nf = jf.nf, Q = nf >> 2, H = nf >> 1;
        double* __restrict__ gcol = lds + (int64_t)jf.lrow0 * kFusedWPitch + lr;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const int j = j0 + 2 * (lg + 4 * gg) + h;
            if (j > Q) continue;
            const double oc = C[u][0][h][gg], os = S[u][0][h][gg], ec = C[u][1][h][gg], es = S[u][1][h][gg];
            const double pe = ec + es, me = ec - es, po = oc + os, mo = oc - os;
            gcol[j * kFusedWPitch] = pe + po;
            gcol[(H + j) * kFusedWPitch] = pe - po;
            if (j > 0 && j < Q) {
              gcol[(H - j) * kFusedWPitch] = me - mo;
              gcol[(nf - j) * kFusedWPitch] = me + mo;
            }
          }
      }
      fused_wait_lgkm0();
    };
    auto join = [&](int k) {
      const Geo g = geo(k);
      auto take = [&]() {
        if (__builtin_amdgcn_readfirstlane(ccnt[k & 1]) >= g.n - f.join_reserve) return -1;
        const int t = ticket(k);
        return t < g.n ? t : -1;
      };
      int t = take();
      if (t < 0) return;
      Ops o;
      load(g.c0 + t, o, lane_now());
      for (;;) {
        const int ty = __builtin_amdgcn_readfirstlane(o.ci.y), tc = __builtin_amdgcn_readfirstlane(o.ci.z);
        Epi x;
        epi_toa(g, ty, tc, lane_now(), x);
        d4 sum[2];
        mfma_chunk(o, lane_now(), sum, pf);
        epi_gather(g, lane_now(), x);
        t = take();
        load(t >= 0 ? g.c0 + t : o.c, o, lane_now());
        epilogue(g, ty, tc, lane_now(), sum, x, pf);
        pf.count(7);
        if (t < 0) return;
      }
    };
    auto barrier_a = [&](int k) {
      fused_barrier();  // A(k): item k is interpolated
      pf.lap(4);
      if (dw == 0 && lane == 0) ccnt[k & 1] = 0;
    };
    for (int k = -1;; ++k) {
      const bool next = item_of(k + 1) >= 0;
      if (dw == 0 && lane == 0) qitem[(k + 3) & 3] = item_of(k + 2) >= 0 ? queue.fetch() : -1;
      if (FPTA_W_JOIN && k >= 0) join(k);
      if (!next) {
        if (k >= 0) barrier_a(k);
        fused_wait_lgkm0();
        fused_barrier();  // B(k)
        break;
      }
      build(k + 1);
      if (k >= 0) barrier_a(k);
      write_grid();
      pf.lap(3);
      fused_barrier();  // B(k)
      pf.lap(4);
    }
    pf.flush(f.prof, wave);
    return;
  }

  // ------------------------------------------------------------------ interpolation waves (as k_grid_fused)
  Prof pf;  // -DFPTA_FUSED_PROF: 0 next-chunk loads, 1 MFMA steps, 2 white epilogue + stores, 3 barriers, 5 chunks,
            // 6 epilogue input loads + ticket
  pf.start();
  fused_barrier();  // B(-1)
  pf.lap(3);
  int k = 0;
  Geo g0 = geo(0), g1 = geo(1);
  bool ex0 = false, ex1 = false;
  auto next = [&](int& kn) {
    if (!ex0) {
      const int t = ticket(k);
      if (t < g0.n) {
        kn = k;
        return g0.c0 + t;
      }
      ex0 = true;
    }
    if (!ex1 && g1.valid) {
      const int t = ticket(k + 1);
      if (t < g1.n) {
        kn = k + 1;
        return g1.c0 + t;
      }
      ex1 = true;
    }
    kn = -1;
    return -1;
  };
  Ops o;   // the operands of chunk o.c (item kc)
  int kc;  // -1: none
  {
    const int cc = next(kc);
    load(cc >= 0 ? cc : g0.c0, o, lane);
  }
  for (;;) {
    while (kc == k) {
      const int ty = __builtin_amdgcn_readfirstlane(o.ci.y), tc = __builtin_amdgcn_readfirstlane(o.ci.z);
      Epi x;
      epi_toa(g0, ty, tc, lane, x);
      pf.lap(6);
      d4 sum[2];
      mfma_chunk(o, lane, sum, pf);
      epi_gather(g0, lane, x);
      int kn;
      const int cn = next(kn);
      pf.lap(6);
      load(cn >= 0 ? cn : o.c, o, lane);  // never conditional (exact vmcnt waits)
      pf.lap(0);
      pf.count(5);
      epilogue(g0, ty, tc, lane, sum, x, pf);
      kc = kn;
    }
    fused_wait_lgkm0();
    pf.lap(6);
    fused_barrier();  // A(k)
    fused_barrier();  // B(k)
    pf.lap(3);
    ++k;
    g0 = g1;
    g1 = geo(k + 1);
    ex0 = ex1;
    ex1 = false;
    if (!g0.valid) break;
    if (kc < 0) {
      const int cc = next(kc);
      load(cc >= 0 ? cc : g0.c0, o, lane);
    }
  }
  pf.flush(f.prof, wave);
  finish();
}

hipError_t launch_grid_fused_w(hipStream_t st, const SynthArgs& a, const GridBand& band, const FusedArgs& f,
                               int32_t nq_max, size_t lds_bytes, hipEvent_t ev0, hipEvent_t ev1, int* kernel_out) {
  if (band.n_chunks <= 0 || band.vmax < 4 || f.join_reserve < 0 || band.vmax % 4 != 0 ||
      a.R_pad % kFusedWReal != 0 || a.accumulate || a.part || !f.lrows || !f.psr_c0 || f.n_sig <= 0 ||
      f.n_sig > kFusedWMaxSig || lds_bytes > (size_t)kFusedLdsMax || nq_max <= 0 || f.ring_off < 0 ||
      f.fq < kFusedWNQ || f.fq % 4 != 0 || !f.queue ||
      (size_t)(f.ring_off + 2 * kFusedWMaxSig * kFusedWSlot) * sizeof(double) + 48 > lds_bytes ||
      (a.w_block_of && (!a.w_zb || !a.w_esig || a.w_nblocks <= 0 || a.w_zb_ld < a.R_pad || a.w_zb_ld % 2)))
    return hipErrorInvalidValue;
  int jobs = 0;
  for (int s = 0; s < f.n_sig; ++s) {
    const FusedSig& fs = f.s[s];
    const int nq = ((((fs.nm + 1) >> 1) + 3) >> 2);
    if (fs.nf % 4 != 0 || !fs.tq || fs.n_rc != (fs.nf / 4 + 32) / 32 || fs.ldq < 32 * fs.n_rc ||
        4 * nq > fs.ntq || fs.n_terms <= 0 || fs.n_terms > kDftGenTerms ||
        fs.lrow0 < 0 || (fs.lrow0 + fs.nf) * kFusedWPitch > f.ring_off)
      return hipErrorInvalidValue;
    for (int i = 0; i < fs.n_terms; ++i)
      if (fs.term_nm[i] <= 0 || fs.term_nm[i] > fs.nm || (fs.term_kind[i] == 0 && (!fs.term_amp[i] || fs.term_nm[i] % 2)) ||
          (fs.term_kind[i] == 1 && (!a.coef || fs.term_col0[i] < 0 || fs.term_col0[i] + 2 * fs.term_nm[i] > a.K)))
        return hipErrorInvalidValue;
    jobs += fs.n_rc;
  }
  if (jobs > kFusedWJobs) return hipErrorInvalidValue;
  const int32_t n_rb = a.R_pad / kFusedWReal;
  const int64_t items = (int64_t)a.P * n_rb;
  if (items > 0x7FFFFFFF || items <= 0) return hipErrorInvalidValue;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  static std::atomic<int> n_cus[64];
  static std::atomic<bool> attr_set[64][kFusedWKernels];
  int n_cu = n_cus[dev].load(std::memory_order_relaxed);
  if (n_cu <= 0) {
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
    n_cus[dev].store(n_cu, std::memory_order_relaxed);
  }
  const int64_t grid = std::min<int64_t>((items + 7) / 8 * 8, ((int64_t)n_cu + 7) / 8 * 8);
  const int ki = (f.real0 & 1) ? 1 : 0;
  using K = void (*)(SynthArgs, GridBand, FusedArgs, int32_t, int32_t);
  static const K kernels[kFusedWKernels] = {k_grid_fused_w<kFusedWNQ, false>, k_grid_fused_w<kFusedWNQ, true>};
  const K kernel = kernels[ki];
  if (!attr_set[dev][ki].load(std::memory_order_acquire)) {
    hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLdsMax);
    if (e != hipSuccess) return e;
    attr_set[dev][ki].store(true, std::memory_order_release);
  }
  FusedArgs fa = f;
  for (int s = f.n_sig; s < kFusedArgSig; ++s) fa.s[s] = f.s[0];
  int32_t n_rb_arg = n_rb, items_arg = (int32_t)items;
  SynthArgs aa = a;
  GridBand bb = band;
  void* args[] = {(void*)&aa, (void*)&bb, (void*)&fa, (void*)&n_rb_arg, (void*)&items_arg};
  (void)hipGetLastError();
  const hipError_t e = hipExtLaunchKernel((const void*)kernel, dim3((unsigned)grid),
                                          dim3(64 * (kFusedIW + kFusedDW)), args, lds_bytes, st, ev0, ev1, 0);
  if (e == hipSuccess && kernel_out) *kernel_out = ki;
  return e;
}

}  // namespace fpta
