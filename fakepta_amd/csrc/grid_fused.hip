// k_grid_fused: the whole gridded synthesis of items = (pulsar, kFusedReal realizations) in persistent workgroups (C2:
// RN + GWB in one grid signal of nf = 124 points, DM in one of nf = 380; 129 KB of LDS grid per item).
//
// The two-kernel path writes every grid (C2: 0.41 GB per block of 1024 realizations) to HBM from k_grid_dft_gen and
// reads it back in k_grid_interp_ws: with the 1.64 GB of residuals, 2.5 GB of HBM traffic per block, and the DFTs of
// block b + 1 co-run beside the interpolation of block b on the leftover registers of one wave slot per SIMD. Here the
// grid lives in LDS only; HBM sees the residual stores, the interpolation weights (read once per pulsar per XCD: the 32
// items of a pulsar run side by side on one XCD) and the mixed common coefficients.
//
// A workgroup (one per CU) has two roles, one wave of each per SIMD; items come from per-XCD ticket queues:
//  * DFT waves (kFusedDW): build item k + 1's grids while item k is interpolated. Ring iteration g draws 16-mode group
//    g + 1 of every grid signal (one (mode, realization pair) per lane, grid_term_coefs: k_grid_dft_gen's terms and
//    order) into one slot of a two-slot LDS ring while the waves' MFMAs read group g from the other; the DFT waves meet
//    at an LDS counter after each iteration (the interpolation waves take no part). Wave d's job is the d-th 32-row
//    chunk of the quarter ranges: k_grid_dft_gen's MFMA k-steps for both realization tiles (A = table row pairs from
//    global memory / L2, B = the (cos, sin) pair of a realization from the ring), the accumulators kept in registers
//    until the item boundary, then k_grid_dft_gen's butterfly writes grid rows j, H + j, H - j, nf - j into LDS. Before
//    building, they interpolate chunks of item k while enough are left (light DFTs, C4).
//  * interpolation waves (kFusedIW): the item's chunks by LDS tickets: per band step A = the dbl2 pair of realizations
//    (2 lr, 2 lr + 1) of LDS row lrows[c][4 q + lg] (one ds_read_b128), B = the weight pair of TOAs (2 lr, 2 lr + 1)
//    from global memory, four MFMAs (even / odd TOA x realization tile) as k_grid_interp_ws; the next chunk's operands
//    are loaded before this chunk's eight 16-byte stores enter the vmcnt queue.
// Two s_barriers per item separate the roles: A (item k interpolated, item k + 1's accumulators ready), after which the
// DFT waves overwrite the grids, and B (the new grids written). DESIGN.md §5a.
// Every value is made by the same operations in the same order as k_grid_dft_gen (or k_grid_dft_mfma from the merged
// anchor columns) + k_grid_interp_ws: the block is bit-identical to theirs (tests/test_gpu_fused.py).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <atomic>
#include <type_traits>

#include "fused_device.h"

namespace fpta {

#ifndef FPTA_FUSED_DFT_PRIO
#define FPTA_FUSED_DFT_PRIO 3  // issue priority of the DFT waves (round 5: 3 beat 1 and 0 on C2)
#endif
#ifndef FPTA_HALF_STORE16
#define FPTA_HALF_STORE16 0  // HALF: 1 = lanes swap values (DPP) for 16-byte stores (measured slower than 8-byte stores)
#endif
#ifndef FPTA_HALF_AHEAD
#define FPTA_HALF_AHEAD 2  // HALF: band steps (four MFMAs each, both halves) between an A operand's LDS read and its use
#endif
constexpr int kFusedHalfAhead = FPTA_HALF_AHEAD;
#ifndef FPTA_HALF_PIN
#define FPTA_HALF_PIN 0  // HALF: 1 = a scheduling barrier keeps each step's look-ahead LDS reads before its MFMAs
#endif

#ifndef FPTA_FUSED_CUT
#define FPTA_FUSED_CUT 0  // diagnostic variant builds only (make variant DEFS=-DFPTA_FUSED_CUT=n): 1 no DFT builds, 2 no interpolation,
                          // 8 no output stores
#endif

namespace {

// A chunk's operands for band steps 0 .. NS - 1 (further steps of a wider chunk are loaded one at a time)
template <int NS>
struct FusedOps {
  int c;        // chunk (wave-uniform)
  i32x4 ci;     // band.chunks[c] {pulsar, first TOA, count, band rows} (a vector load: every lane the same address)
  dbl2 b[NS];   // weights of TOAs (2 lr, 2 lr + 1) at band row 4 q + lg
  int row[NS];  // LDS grid row of band row 4 q + lg
};
// The same with half-chunk bands (HALF): band steps 0 .. NS - 1 of each half
template <int NS>
struct FusedOpsH {
  int c;
  i32x4 ci;            // FusedHalf::chunks[c] {pulsar, first TOA, count, nq0 | nq1 << 16}
  dbl2 b[2][NS / 2];   // [half h][step pair qp]: weights of TOA 16 h + lr at band rows 4 (2 qp) + lg, 4 (2 qp + 1) + lg
  int row[2][NS];      // LDS grid row of band row 4 q + lg of half h
};

// One ticket of the successor block's mix (FusedMix): mode k, realizations 16 rg .. 16 rg + 15, pulsars
// kFusedMixGroup pg .. (seven 16-pulsar tiles), both columns. Lane (lr, lg) draws realization 16 rg + lr at k-step row
// q0 + lg: k_gen_mix's normals of (k, q, g) are the B operand; A = L^T[q][16 t + lr] of tile t, one MFMA per (tile,
// column) while the tile's k-steps last (k_gen_mix's bound at 16-pulsar granularity: the steps it runs past them have
// zero factors there). Two k-steps per trip: with an even first realization the lanes of a realization pair share
// Philox counters, so each computes one of the two steps' Philox calls and they swap the halves the other needs (one
// DPP exchange of two words); each lane then transforms its own half (normals4's operations: gp_normal2's values).
__device__ __forceinline__ uint32_t dpp_u32_xor1(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ void bm_half(uint32_t wl, uint32_t wa, double& zc, double& zs) {
  double sn, cs;
  const double r = bm_sqrt(-2.0 * bm_log_u32(wl));
  bm_sincos2pi_u32(wa, sn, cs);
  zc = r * cs;
  zs = r * sn;
}
__device__ __forceinline__ void fused_mix_tile(const FusedMix& m, int k, int rg, int pg, int lane) {
  constexpr int NT = kFusedMixGroup / 16;
  const int lr = lane & 15, lg = lane >> 4;
  const int r = 16 * rg + lr;
  const bool rv = r < m.n_real;  // padding realizations: zero, as k_gen_mix writes them
  const uint64_t g = (uint64_t)(m.real0 + r);
  const int p0 = kFusedMixGroup * pg;
  int qe[NT];
  int qmax = 0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int pt = p0 + 16 * t;
    qe[t] = pt < m.P ? min(m.lower ? min(m.P, pt + 16) : m.P, m.n_q) : 0;
    qmax = max(qmax, qe[t]);
  }
  d4 acc[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t][0] = acc[t][1] = d4{0.0, 0.0, 0.0, 0.0};
  const double* __restrict__ lt = m.LT + p0 + lr;
  const bool paired = (m.real0 & 1) == 0;  // lanes 2 i, 2 i + 1: realizations g, g + 1 of one Philox counter
  const int e = lr & 1;
  const uint32_t ctr3 = (uint32_t)(g >> 1);
  // rows q0 + lg of k-steps q0 < qe[t] <= P only: up to 4 ceil(P / 4) - 1 < lt_rows (launch check), zero past P
  for (int q0 = 0; q0 < qmax; q0 += 8) {
    double a0[NT], a1[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      a0[t] = q0 < qe[t] ? ld_global(lt + (int64_t)(q0 + lg) * m.lt_ld + 16 * t) : 0.0;
      a1[t] = q0 + 4 < qe[t] ? ld_global(lt + (int64_t)(q0 + 4 + lg) * m.lt_ld + 16 * t) : 0.0;
    }
    double zc0, zs0, zc1, zs1;
    if (paired) {
      const u32x4 v = philox4x32_10({(uint32_t)k, (uint32_t)(q0 + 4 * e + lg), (uint32_t)m.seg, ctr3}, m.k0, m.k1);
      const uint32_t r0 = dpp_u32_xor1(e ? v.x : v.z), r1 = dpp_u32_xor1(e ? v.y : v.w);
      bm_half(e ? r0 : v.x, e ? r1 : v.y, zc0, zs0);  // step q0: (x, y) of an even realization, (z, w) of an odd one
      bm_half(e ? v.z : r0, e ? v.w : r1, zc1, zs1);  // step q0 + 4
    } else {
      gp_normal2((uint32_t)k, (uint32_t)(q0 + lg), (uint32_t)m.seg, g, m.k0, m.k1, zc0, zs0);
      gp_normal2((uint32_t)k, (uint32_t)(q0 + 4 + lg), (uint32_t)m.seg, g, m.k0, m.k1, zc1, zs1);
    }
    const bool ok0 = rv && q0 + lg < m.n_q, ok1 = rv && q0 + 4 + lg < m.n_q;
    zc0 = ok0 ? zc0 : 0.0;
    zs0 = ok0 ? zs0 : 0.0;
    zc1 = ok1 ? zc1 : 0.0;
    zs1 = ok1 ? zs1 : 0.0;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (q0 < qe[t]) {
        acc[t][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[t], zc0, acc[t][0], 0, 0, 0);
        acc[t][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[t], zs0, acc[t][1], 0, 0, 0);
      }
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (q0 + 4 < qe[t]) {
        acc[t][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[t], zc1, acc[t][0], 0, 0, 0);
        acc[t][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[t], zs1, acc[t][1], 0, 0, 0);
      }
  }
  // D of tile t: lane (lr, lg) register gg = pulsar p0 + 16 t + lg + 4 gg, realization r; stored as amp * sum
  // (k_gen_mix's rounding)
  const double am = ld_global(m.amp + k);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int p = p0 + 16 * t + lg + 4 * gg;
        if (p < m.P) m.coef[((int64_t)p * m.K + m.col0 + 2 * k + h) * m.R_pad + r] = am * acc[t][h][gg];
      }
}

}  // namespace

// NQ: band steps whose operands an interpolation wave holds (HALF: per half); ODD: the first realization is odd (GEN
// only); GEN: some grid signal draws its own coefficients (a per-pulsar member, C2). Without generated terms (C4: one
// mixed common signal, loaded) the draws' Philox and Box-Muller code is compiled out. HALF: half-chunk bands
// (FusedHalf): per band step of half h, A = the realization pair of the half's band row, B = the weight of TOA 16 h +
// lr, two MFMAs (C2: 2 x 8 steps x 2 instead of 9 steps x 4 MFMAs per chunk); 8-byte stores (a lane holds TOAs lr
// and 16 + lr of each realization).
template <int NQ, bool ODD, bool GEN, bool HALF>
__global__ __launch_bounds__(64 * (kFusedIW + kFusedDW), 1) void k_grid_fused(SynthArgs a, GridBand band, FusedArgs f,
                                                                             int32_t n_rb, int32_t n_items) {
  static_assert(kFusedReal == 32 && kFusedPitch == 32 && kFusedGroupModes * kFusedReal / 2 == 64 * kFusedDW,
                "two realization tiles; one (mode, realization pair) of a 16-mode group per DFT lane");
  static_assert(!HALF || (NQ % 4 == 0 && kGridTT == 2 * kFusedHalfTT), "half bands: whole row groups, two halves");
  // [grid rows][32] | ring [2][kFusedMaxSig][kFusedSlot] | sync word, 3 pad | item ring [4] | chunk tickets [2], 2 pad
  // (48 bytes past the ring)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const FusedQueue queue(n_items, f.queue);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  double* __restrict__ ring = lds + f.ring_off;
  uint32_t* sync = (uint32_t*)(ring + 2 * kFusedMaxSig * kFusedSlot);
  volatile int* qitem = (volatile int*)(sync + 4);  // item k at [k & 3]
  if (threadIdx.x == 0) {
    *sync = 0u;
    ((volatile int*)sync)[8] = 0;  // chunk tickets of items 0 and 1
    ((volatile int*)sync)[9] = 0;
    qitem[0] = queue.fetch();
    qitem[1] = qitem[0] >= 0 ? queue.fetch() : -1;
  }
  __syncthreads();
  // item k of this workgroup (k >= -1; -1 = none): items 0 and 1 are fetched here, item k + 3 by the DFT waves' loop
  // trip k (before item k + 1's build), ahead of the ring syncs and barriers that publish it to the other waves
  auto item_of = [&](int k) { return __builtin_amdgcn_readfirstlane(qitem[k & 3]); };
  // the launch's last workgroup to finish zeroes the queues for the next launch (every workgroup's fetches precede
  // its count)
  auto finish = [&]() {
    if (threadIdx.x == 0) {
      __threadfence();
      const uint32_t done = __hip_atomic_fetch_add(f.queue + 8, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (done == gridDim.x - 1)
        for (int i = 0; i < kFusedQueueWords; ++i)
          __hip_atomic_store(f.queue + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  // The successor block's mix tickets (FusedMix), taken by every wave once it has nothing left of this block: the DFT
  // waves from the last item's interpolation on, the interpolation waves after it (at the lowest issue priority: the
  // last chunks go first). The launch's last workgroup zeroes the ticket counter with the queues (finish). (Tickets
  // taken by interpolation waves waiting for a build, while enough of it was left, measured no faster, and one call
  // site keeps the 112-pulsar accumulators within the registers.)
  auto mix_tiles = [&]() {
    if (f.mix.n_tiles <= 0) return;
    __builtin_amdgcn_s_setprio(0);
    // ticket t: pulsar group t % n_pg, then realization tile, then mode
    const int n_pg = (f.mix.P + kFusedMixGroup - 1) / kFusedMixGroup, n_rg = f.mix.R_pad >> 4;
    for (;;) {
      int t = 0;
      if (lane == 0)
        t = (int)__hip_atomic_fetch_add(f.queue + kFusedMixWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = __builtin_amdgcn_readfirstlane(t);
      if (t >= f.mix.n_tiles) break;
      const int pg = t % n_pg, kr = t / n_pg;
      const int k = kr / n_rg;
      fused_mix_tile(f.mix, k, kr - k * n_rg, pg, lane);
    }
  };
  if (item_of(0) < 0) {  // the whole workgroup, before its first barrier (the other workgroups take the mix tickets)
    finish();
    return;
  }

  // ------------------------------------------------------------------ chunks (both roles)
  // Item k's chunks are handed out by an LDS ticket counter, ccnt[k & 1]: the interpolation waves take them, and so do
  // the DFT waves before they build item k + 1 while more than FusedArgs::join_reserve are left (a layout of light DFTs,
  // e.g. C4's one common signal, then gets eight interpolating waves). A wave takes tickets of its grid item k and of
  // k + 1 only; counter k & 1 is zeroed by the DFT waves between barriers A(k - 2) and B(k - 2), after item k - 2's last
  // ticket and before item k's first.
  volatile int* ccnt = (volatile int*)(sync + 8);
  struct Geo {          // item k
    int p, r0, c0, n;   // pulsar, first realization, first chunk, chunks
    int64_t toa0;       // the pulsar's first TOA (residual column)
    bool valid;
  };
  auto geo = [&](int k) {
    Geo g;
    const int item = item_of(k);
    g.valid = item >= 0;
    const int it = g.valid ? item : 0;
    g.p = it / n_rb;
    g.r0 = (it - g.p * n_rb) * kFusedReal;
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
  // Every operand of a chunk's band steps comes through vector loads (vmcnt): a scalar load waits lgkmcnt(0) (scalar
  // loads return out of order), which also waits for the LDS grid reads. The chunk's table entry {pulsar, first TOA,
  // count, band rows} is a vector load too (every lane the same address), issued with the operands and read at process.
  // lane-derived addresses from an opaque copy of the lane index, re-derived where used: hoisted out of the roles' item
  // loops they would stay live across everything in them (the DFT waves' builds and joined chunks) and spill
  auto lane_now = [&]() {
    int v = lane;
    asm volatile("" : "+v"(v));
    return v;
  };
  using Ops = typename std::conditional<HALF, FusedOpsH<NQ>, FusedOps<NQ>>::type;
  // the DFT waves' joined chunks (fewer registers beside their own state)
  using OpsJ = typename std::conditional<HALF, FusedOpsH<NQ>, FusedOps<(NQ < 8 ? NQ : 8)>>::type;
  // operands of band steps 0 .. NS - 1 of chunk cc, at constant offsets from two addresses (steps past the chunk's
  // read the next chunk's or the tables' padding rows: never used)
  // ln: the lane index (the DFT waves pass an opaque copy, lane_now)
  auto load_half = [&](int cc, auto& o, int ln) {
    {
      constexpr int NS = sizeof(o.row[0]) / sizeof(o.row[0][0]);
      o.c = cc;
      o.ci = *(const i32x4*)(f.h.chunks + cc);
      const int lgo = ln >> 4, lro = ln & 15;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const i32x4* __restrict__ rt = (const i32x4*)(f.h.lrows + (((int64_t)cc * 2 + h) * 4 + lgo) * f.h.fq);
#pragma unroll
        for (int q4 = 0; q4 < NS / 4; ++q4) {
          const i32x4 r4 = rt[q4];
          o.row[h][4 * q4] = r4.x;
          o.row[h][4 * q4 + 1] = r4.y;
          o.row[h][4 * q4 + 2] = r4.z;
          o.row[h][4 * q4 + 3] = r4.w;
        }
        const double* __restrict__ wp =
            f.h.wd + ((int64_t)cc * 2 + h) * f.h.vmax * kFusedHalfTT + (lgo * kFusedHalfTT + lro) * 2;
#pragma unroll
        for (int qp = 0; qp < NS / 2; ++qp) o.b[h][qp] = *(const dbl2*)(wp + qp * 8 * kFusedHalfTT);
      }
    }
  };
  auto load_full = [&](int cc, auto& o, int ln) {
    constexpr int NS = sizeof(o.row) / sizeof(o.row[0]);
    o.c = cc;
    o.ci = *(const i32x4*)(band.chunks + cc);
    const int lgo = ln >> 4, lro = ln & 15;
    const i32x4* __restrict__ rt = (const i32x4*)(f.lrows + ((int64_t)cc * 4 + lgo) * f.fq);
    const double* __restrict__ wp = band.wd + ((int64_t)cc * band.vmax + lgo) * kGridTT + 2 * lro;
#pragma unroll
    for (int q4 = 0; q4 < NS / 4; ++q4) {
      const i32x4 r4 = rt[q4];
      o.row[4 * q4] = r4.x;
      o.row[4 * q4 + 1] = r4.y;
      o.row[4 * q4 + 2] = r4.z;
      o.row[4 * q4 + 3] = r4.w;
    }
#pragma unroll
    for (int q = 0; q < NS; ++q) o.b[q] = *(const dbl2*)(wp + 4 * kGridTT * q);
  };
  auto load = [&](int cc, auto& o, int ln) {
    if constexpr (HALF)
      load_half(cc, o, ln);
    else
      load_full(cc, o, ln);
  };
  // chunk cur of item g: k_grid_interp_ws's MFMA steps (A = the realization pair's dbl2 of the LDS grid row, B = the
  // TOA pair's weights) and stores
  // HALF: the same per half h on its own band rows, TOA 16 h + lr per lane
  auto process_half = [&](const Geo& g, const auto& cur, auto& pf, int ln) {
    constexpr int NS = sizeof(cur.row[0]) / sizeof(cur.row[0][0]);
    const int lg = ln >> 4, lr = ln & 15;
    const int lds_lane = 2 * lr;
    const int ty = __builtin_amdgcn_readfirstlane(cur.ci.y), tc = __builtin_amdgcn_readfirstlane(cur.ci.z);
    const int nqw = __builtin_amdgcn_readfirstlane(cur.ci.w);
    const int nq[2] = {nqw & 0xFFFF, nqw >> 16};
    FPTA_DCHECK(nq[0] > 0, "k_grid_fused half band steps", nq[0], 1 << 20);
    d4 acc[2][2];  // [half][realization tile]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[h][i] = d4{0.0, 0.0, 0.0, 0.0};
    {
      // band step q of both halves: four MFMAs back to back on four accumulators, as the whole-band kernel's steps
      // (one half at a time left two MFMAs per basic block, with hazard nops between them). Both halves run
      // max(nq0, nq1) steps: a half's steps past its own nq have zero weights (its weight rows up to the table's vmax
      // are zero, its LDS rows valid repeats), so they add exactly zero. A step's A operands are read from LDS
      // kFusedHalfAhead steps ahead (reads are unconditional).
      constexpr int DA = kFusedHalfAhead;
      const int nqm = min(max(nq[0], nq[1]), NS);
      dbl2 an[2][NS];
      auto rd = [&](int q) {
#pragma unroll
        for (int h = 0; h < 2; ++h) an[h][q] = *(const dbl2*)(lds + cur.row[h][q] * kFusedPitch + lds_lane);
      };
#pragma unroll
      for (int q = 0; q < DA && q < NS; ++q) rd(q);
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        if (q < nqm) {
          if (q + DA < NS) rd(q + DA);
          if (FPTA_HALF_PIN) __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of this step's MFMAs
          const double b0 = (q & 1) ? cur.b[0][q >> 1].y : cur.b[0][q >> 1].x;
          const double b1 = (q & 1) ? cur.b[1][q >> 1].y : cur.b[1][q >> 1].x;
          acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[0][q].x, b0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[0][q].y, b0, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[1][q].x, b1, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(an[1][q].y, b1, acc[1][1], 0, 0, 0);
        }
      }
    }
    pf.lap(1);
    // a half wider than NS steps: its further steps one at a time
#pragma unroll
    for (int h = 0; h < 2; ++h)
      for (int q = NS; q < nq[h]; ++q) {
        const int64_t hc = (int64_t)cur.c * 2 + h;
        const int row = f.h.lrows[(hc * 4 + lg) * f.h.fq + q];
        const double bv = f.h.wd[hc * f.h.vmax * kFusedHalfTT + fused_half_weight_index(4 * q + lg, lr)];
        const dbl2 av = *(const dbl2*)(lds + row * kFusedPitch + lds_lane);
        acc[h][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv, acc[h][0], 0, 0, 0);
        acc[h][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv, acc[h][1], 0, 0, 0);
      }
    pf.lap(4);
    __builtin_amdgcn_sched_barrier(0);
    const int64_t t0 = g.toa0 + ty;
    if ((FPTA_FUSED_CUT & 8) && acc[0][0][0] != -1.25e300) return;  // diagnostic: no stores (the sums stay live)
    // acc[h][i][gg]: TOA 16 h + lr of realization r0 + 2 (lg + 4 gg) + i
    if (FPTA_HALF_STORE16 && tc == kGridTT && g.r0 + kFusedReal <= a.n_real && ((t0 | a.ldo) & 1) == 0 &&
        a.ldo < ((int64_t)1 << 26)) {
      // a full chunk, every realization of the item, 16-byte aligned rows: lanes 2k and 2k + 1 swap TOA 16 + 2k for
      // TOA 2k + 1 (one DPP exchange per value), so lane 2k holds TOAs 2k, 2k + 1 and lane 2k + 1 holds TOAs 16 + 2k,
      // 17 + 2k: eight 16-byte non-temporal stores from one row base, as the whole-band kernel
      const bool odd = lr & 1;
      const uint32_t vo = (uint32_t)(((int64_t)2 * lg * a.ldo + (odd ? 15 + lr : lr)) * 8);
      const char* base = (const char*)(a.out + t0 + (int64_t)g.r0 * a.ldo);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const double send = odd ? acc[0][i][gg] : acc[1][i][gg];
          const double recv = dpp_xor1(send);
          const dbl2 v = odd ? dbl2{recv, acc[1][i][gg]} : dbl2{acc[0][i][gg], recv};
          __builtin_nontemporal_store(v, (dbl2*)((char*)base + (int64_t)(8 * gg + i) * a.ldo * 8 + vo));
        }
    } else if (tc == kGridTT && g.r0 + kFusedReal <= a.n_real && a.ldo < ((int64_t)1 << 26)) {
      // a full chunk, every realization of the item: 8-byte non-temporal stores from one row base (each 16-lane row
      // writes 128 contiguous bytes)
      const uint32_t vo = (uint32_t)(((int64_t)2 * lg * a.ldo + lr) * 8);
      const char* base = (const char*)(a.out + t0 + (int64_t)g.r0 * a.ldo);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg)
            __builtin_nontemporal_store(acc[h][i][gg],
                                        (double*)((char*)base + ((int64_t)(8 * gg + i) * a.ldo + 16 * h) * 8 + vo));
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (16 * h + lr >= tc) continue;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const int r = g.r0 + 2 * (lg + 4 * gg) + i;
            if (r < a.n_real) a.out[t0 + 16 * h + lr + (int64_t)r * a.ldo] = acc[h][i][gg];
          }
      }
    }
    pf.lap(2);
  };
  auto process_full = [&](const Geo& g, const auto& cur, auto& pf, int ln) {
    constexpr int NS = sizeof(cur.row) / sizeof(cur.row[0]);
    const int lg = ln >> 4, lr = ln & 15;
    const int lds_lane = 2 * lr;  // this lane's realization pair in an LDS grid row
    const int ty = __builtin_amdgcn_readfirstlane(cur.ci.y), tc = __builtin_amdgcn_readfirstlane(cur.ci.z);
    const int nq = __builtin_amdgcn_readfirstlane(cur.ci.w) >> 2;
    FPTA_DCHECK(nq > 0, "k_grid_fused band steps", nq, 1 << 20);
    d4 acc[2][2];  // [TOA parity][realization tile]
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[e][i] = d4{0.0, 0.0, 0.0, 0.0};
    {
      // step q's A operand is read from LDS ahead of step q - 1's MFMAs (rows past nq are valid clamped rows)
      dbl2 an = *(const dbl2*)(lds + cur.row[0] * kFusedPitch + lds_lane);
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        if (q < nq) {
          const dbl2 av = an;
          if (q + 1 < NS) an = *(const dbl2*)(lds + cur.row[q + 1] * kFusedPitch + lds_lane);
          const dbl2 bv = cur.b[q];
          acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.y, acc[1][1], 0, 0, 0);
        }
      }
    }
    pf.lap(1);
    // a chunk wider than NS steps (sparse pulsars): its further steps one at a time, each operand loaded and waited for
    // here (off the common path, whose operands all arrive one chunk ahead)
    for (int q = NS; q < nq; ++q) {
      const int v = 4 * q + lg;
      const int row = f.lrows[((int64_t)cur.c * 4 + lg) * f.fq + q];
      const dbl2 bv = *(const dbl2*)(band.wd + ((int64_t)cur.c * band.vmax + v) * kGridTT + 2 * lr);
      const dbl2 av = *(const dbl2*)(lds + row * kFusedPitch + lds_lane);
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.x, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.x, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bv.y, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bv.y, acc[1][1], 0, 0, 0);
    }
    pf.lap(4);
    __builtin_amdgcn_sched_barrier(0);
    // interp_store_rows' fast path from the item's first TOA: a full chunk, every realization of the item stored,
    // 16-byte aligned rows: eight 16-byte non-temporal stores from one row base
    const int64_t t0 = g.toa0 + ty;
    if ((FPTA_FUSED_CUT & 8) && acc[0][0][0] != -1.25e300) return;  // diagnostic: no stores (the sums stay live)
    if (FPTA_HALF_STORE16 && tc == kGridTT && g.r0 + kFusedReal <= a.n_real && ((t0 | a.ldo) & 1) == 0 &&
        a.ldo < ((int64_t)1 << 26)) {
      const uint32_t vo = (uint32_t)(((int64_t)2 * lg * a.ldo + 2 * lr) * 8);
      const char* base = (const char*)(a.out + t0 + (int64_t)g.r0 * a.ldo);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg)
          __builtin_nontemporal_store(dbl2{acc[0][i][gg], acc[1][i][gg]},
                                      (dbl2*)((char*)base + (int64_t)(8 * gg + i) * a.ldo * 8 + vo));
    } else {
      InterpTile<2> t;
      t.c = cur.c;
      t.p = g.p;
      t.r0 = g.r0;
      t.y = ty;
      t.cnt = tc;
      t.nq = nq;
      interp_store_rows<2>(a, a.out, t, acc);
    }
    pf.lap(2);
  };
  auto process = [&](const Geo& g, const auto& cur, auto& pf, int ln) {
    if constexpr (HALF)
      process_half(g, cur, pf, ln);
    else
      process_full(g, cur, pf, ln);
  };

  if (wave >= kFusedIW) {
    // ---------------------------------------------------------------- DFT waves
    const int dw = wave - kFusedIW;
    // the DFT waves are the item's critical path (the interpolation waves wait at barrier A): first claim on the SIMD's
    // issue slots, the interpolation waves fill the gaps (C2 kernel -3%)
    __builtin_amdgcn_s_setprio(FPTA_FUSED_DFT_PRIO);
    int js = -1, jrc = 0;  // this wave's job: grid signal js, quarter-range rows 32 jrc .. 32 jrc + 31
    {
      int j = dw;
#pragma unroll
      for (int s = 0; s < kFusedMaxSig; ++s) {
        if (s < f.n_sig && js < 0 && j < f.s[s].n_rc) {
          js = s;
          jrc = j;
        }
        if (s < f.n_sig) j -= f.s[s].n_rc;
      }
    }
    js = __builtin_amdgcn_readfirstlane(js);
    jrc = __builtin_amdgcn_readfirstlane(jrc);
    Prof pf;  // DFT waves: 0 loads issue, 1 MFMA steps (DFT and joined chunks), 2 ring sync / joined chunks' stores, 3 grid
              // writes, 4 barriers / joined wide chunks, 5 iterations, 6 draws, 7 joined chunks (count)
    pf.start();
    uint32_t epoch = 0;
    // every DFT wave's ring writes and reads so far are done (an LDS counter; the interpolation waves run on)
    auto dsync = [&]() {
      fused_wait_lgkm0();
      if (lane == 0) __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      epoch += kFusedDW;
      while ((uint32_t)__builtin_amdgcn_readfirstlane(
                 (int)__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < epoch)
        __builtin_amdgcn_s_sleep(1);
    };
    // groups of 16 modes (two 4-mode k-steps of both parities) of grid signal s
    auto n_groups = [&](int nm) { return (((((nm + 1) >> 1) + 3) >> 2) + 1) >> 1; };
    int ng[kFusedMaxSig];
    int n_it = 0;  // iterations per item: iteration g draws group g + 1 of every signal and runs group g's steps
#pragma unroll
    for (int s = 0; s < kFusedMaxSig; ++s) {
      ng[s] = s < f.n_sig ? n_groups(f.s[s].nm) : 0;
      n_it = max(n_it, ng[s]);
    }
    // this wave's job, hoisted: its table rows (parity 0 cos, t = lg, rows 32 jrc + 2 lr) and k-steps per parity
    const FusedSig& jf = f.s[js < 0 ? 0 : js];
    const int64_t jts = (int64_t)jf.ntq * jf.ldq, jld4 = 4 * (int64_t)jf.ldq;
    // Lane-derived addresses are re-derived where used from an opaque copy of the lane index: hoisted out of the item
    // loop they would stay live across the joined chunks (see join) and spill
    auto jtq_now = [&]() {
      const int ln = lane_now();
      return jf.tq + (int64_t)(ln >> 4) * jf.ldq + 32 * jrc + 2 * (ln & 15);
    };
    const int jnq0 = (((jf.nm + 1) >> 1) + 3) >> 2, jnq1 = ((jf.nm >> 1) + 3) >> 2;
    const int jng = js < 0 ? 0 : (jnq0 + 1) >> 1;
    // [parity: 0 odd k, 1 even k][row tile h: rows 2 i + h][realization tile t]
    d4 C[2][2][2], S[2][2][2];
    // Group g of signal s: modes 16 g .. 16 g + 15 x realizations r0 .. r0 + 31, one (mode m, realization pair r) per
    // lane, k_grid_dft_gen's coefficient (grid_term_coefs: the same operations) in three parts:
    //  draw_load: every term slot's inputs, two 16-byte loads each whatever the term (a fixed count keeps the compiler's
    //             vmcnt waits for the table operands exact): a generated term's amplitude, a loaded term's columns;
    //             issued with the tables of the steps before them, so the latencies overlap;
    //  draw_normals: the generated terms' normals (no memory);
    //  draw_store: amp * z (rounded) and the loaded values summed in the terms' order, into the ring.
    // The signal index is a constant wherever these run (loops over kFusedMaxSig unrolled): the descriptor's fields are
    // scalar loads at fixed kernel-argument offsets, not re-read by computed index in every group.
    struct DrawIn {
      dbl2 x0[kFusedTerms], x1[kFusedTerms];  // generated: x0.x amplitude pair; loaded: x0 cos pair, x1 sin pair
    };
    auto draw_load = [&](const FusedSig& fs, int g, int p, int r0, DrawIn& in) {
      const int didx = dw * 64 + lane_now(), dmm = didx >> 4, drl = 2 * (didx & 15);
      const int m = kFusedGroupModes * g + dmm, r = r0 + drl;
#pragma unroll
      for (int i = 0; i < kFusedTerms; ++i) {
        const bool on = i < fs.n_terms;
        const int nmi = on ? fs.term_nm[i] : 2;
        const int mi = min(m, nmi - 1);  // clamped: a mode past the term's is never used
        const double* src0;
        int64_t step;
        if (on && fs.term_kind[i] == 1) {
          src0 = a.coef + ((int64_t)p * a.K + fs.term_col0[i] + 2 * mi) * a.R_pad + r;
          step = a.R_pad;
        } else {  // the amplitude pair (mi, mi + 1) of a generated term: .x is amp[mi] (rows are padded to even nm)
          src0 = (on ? fs.term_amp[i] : a.coef) + (int64_t)p * nmi + (mi & ~1);
          step = 0;
        }
        in.x0[i] = ld_global((const dbl2*)src0);
        in.x1[i] = ld_global((const dbl2*)(src0 + step));
      }
    };
    auto draw_finish = [&](const FusedSig& fs, int g, int p, int r0, double* __restrict__ slot_s, const DrawIn& in) {
      const int didx = dw * 64 + lane_now(), dmm = didx >> 4, drl = 2 * (didx & 15);
      const int m = kFusedGroupModes * g + dmm, r = r0 + drl;
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
      const bool ok0 = r < a.n_real, ok1 = r + 1 < a.n_real;  // padding realizations: zero, as k_gen writes them
      auto normals = [&](int seg, double (&z)[4]) {
        if (!ODD) {  // r0 and r are even: the first realization's parity is the launch's
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
      for (int i = 0; i < kFusedTerms; ++i) {
        if (i >= fs.n_terms) continue;
        double pc[2], ps[2];
        if (GEN && fs.term_kind[i] == 0) {
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
      // members past kFusedTerms (a grid signal of three or more, e.g. coalesced RN + DM + GWB at one radio frequency):
      // loaded and drawn here, in order, with the same operations
      for (int i = kFusedTerms; i < fs.n_terms; ++i) {
        const int mi = min(m, fs.term_nm[i] - 1);
        double pc[2], ps[2];
        if (GEN && fs.term_kind[i] == 0) {
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
      double* __restrict__ dst = slot_s + 2 * (dmm * kFusedReal + drl);
      *(dbl2*)dst = dbl2{bc[0], bs[0]};
      *(dbl2*)(dst + 2) = dbl2{bc[1], bs[1]};
    };
    // ring slot k: [signal][16 modes][32 realizations][cos, sin]
    auto slot_of = [&](int k, int s) { return ring + ((k & 1) * kFusedMaxSig + s) * kFusedSlot; };
    // the table operands of this wave's k-steps q = 2 g, 2 g + 1 (clamped: a step past the parity's is never used)
    struct Tabs {
      dbl2 ac[2][2], as[2][2];  // [k-step h2][parity]
    };
    auto tables = [&](int g, Tabs& tb) {
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int q = max(0, min(2 * g + h2, jnq0 - 1));
#pragma unroll
        for (int par = 0; par < 2; ++par) {
          const double* __restrict__ tc = jtq_now() + (int64_t)(2 * par) * jts + q * jld4;
          tb.ac[h2][par] = ld_global((const dbl2*)tc);
          tb.as[h2][par] = ld_global((const dbl2*)(tc + jts));
        }
      }
    };
    // k_grid_dft_gen's MFMA k-steps q = 2 g, 2 g + 1 of the job on the job signal's group g in ring slot `slot`
    auto steps = [&](int slot, int g, const Tabs& tb) {
      const double* __restrict__ bsrc = slot_of(slot, js);
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int q = 2 * g + h2;
#pragma unroll
        for (int par = 0; par < 2; ++par) {
          if (q >= (par ? jnq1 : jnq0)) continue;
          const dbl2 ac = tb.ac[h2][par], as = tb.as[h2][par];
          // mode 16 g + 2 (4 h2 + lg) + par = 2 (4 q + lg) + par, realizations lr and 16 + lr
          const double* bm = bsrc + 2 * ((2 * (4 * h2 + lg) + par) * kFusedReal + lr);
          const dbl2 b[2] = {*(const dbl2*)bm, *(const dbl2*)(bm + 2 * 16)};
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            C[par][0][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac.x, b[t].x, C[par][0][t], 0, 0, 0);
            C[par][1][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac.y, b[t].x, C[par][1][t], 0, 0, 0);
            S[par][0][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(as.x, b[t].y, S[par][0][t], 0, 0, 0);
            S[par][1][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(as.y, b[t].y, S[par][1][t], 0, 0, 0);
          }
        }
      }
    };
    // Item k's accumulators of this wave's job. Iteration g runs the job signal's group g from ring slot sb + g and
    // draws group g + 1 of every signal into slot sb + g + 1; the last iteration draws group 0 of item k + 1 instead
    // (its MFMA steps have no draws of their own to overlap), so only the first item's group 0 is drawn alone. All
    // loads of an iteration are issued before its steps.
    int sb = 0;  // ring slot of the item's group 0
    auto build = [&](int k) {
      const int item = item_of(k);
      const int p = item / n_rb, r0 = (item - p * n_rb) * kFusedReal;
      const int item1n = item_of(k + 1);
      const bool nx = item1n >= 0;
      const int item1 = nx ? item1n : item;
      const int p1 = item1 / n_rb, r1 = (item1 - p1 * n_rb) * kFusedReal;
#pragma unroll
      for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int t = 0; t < 2; ++t) C[par][h][t] = S[par][h][t] = d4{0.0, 0.0, 0.0, 0.0};
      if (k == 0) {
#pragma unroll
        for (int s = 0; s < kFusedMaxSig; ++s) {
          if (s >= f.n_sig) continue;
          DrawIn in;
          draw_load(f.s[s], 0, p, r0, in);
          draw_finish(f.s[s], 0, p, r0, slot_of(sb, s), in);
        }
        pf.lap(6);
        dsync();
        pf.lap(2);
      }
      for (int g = 0; g < n_it; ++g) {
        const bool last = g + 1 == n_it;
        const int dp = last ? p1 : p, dr = last ? r1 : r0;
        Tabs tb;
        tables(g, tb);
        DrawIn in[kFusedMaxSig];
#pragma unroll
        for (int s = 0; s < kFusedMaxSig; ++s)  // an unused descriptor is a copy of the first
          draw_load(f.s[s], last ? 0 : min(g + 1, max(ng[s], 1) - 1), dp, dr, in[s]);
        pf.lap(0);
        if (g < jng) steps(sb + g, g, tb);
        pf.lap(1);
#pragma unroll
        for (int s = 0; s < kFusedMaxSig; ++s)
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
      if (js >= 0) {
        const int j0 = 32 * jrc;
        const int nf = jf.nf, Q = nf >> 2, H = nf >> 1;
        double* __restrict__ gcol = lds + (int64_t)jf.lrow0 * kFusedPitch + lr;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const int j = j0 + 2 * (lg + 4 * gg) + h;
            if (j > Q) continue;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              const double oc = C[0][h][t][gg], os = S[0][h][t][gg], ec = C[1][h][t][gg], es = S[1][h][t][gg];
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
      fused_wait_lgkm0();
    };
    // item k + 1's draws and steps run while the interpolation waves read item k's grids (one build site: the
    // draws are most of the kernel's code)
    // Before building item k + 1 (its accumulators not yet live), chunks of item k while more than f.join_reserve of
    // its tickets are left: the interpolation waves keep that many for the build's duration (host estimate; a layout
    // whose DFTs take as long as its interpolation, C2, never joins). The counter is peeked first, so a ticket taken is
    // always processed.
    auto join = [&](int k) {
      if (FPTA_FUSED_CUT & 6) return;
      const Geo g = geo(k);
      auto take = [&]() {  // a ticket while more than the reserve are left, else -1
        if (__builtin_amdgcn_readfirstlane(ccnt[k & 1]) >= g.n - f.join_reserve) return -1;
        const int t = ticket(k);
        return t < g.n ? t : -1;
      };
      int t = take();
      if (t < 0) return;
      // two operand sets in turn, the next chunk's loaded before this one's stores (as the interpolation waves)
      OpsJ o0, o1;
      load(g.c0 + t, o0, lane_now());
      for (;;) {
        t = take();
        load(t >= 0 ? g.c0 + t : o0.c, o1, lane_now());
        process(g, o0, pf, lane_now());
        pf.count(7);
        if (t < 0) return;
        t = take();
        load(t >= 0 ? g.c0 + t : o1.c, o0, lane_now());
        process(g, o1, pf, lane_now());
        pf.count(7);
        if (t < 0) return;
      }
    };
    // (one build site and one grid write per trip, on one path: the accumulators are dead from the write to the next
    // build, so the joined chunks have the registers)
    auto barrier_a = [&](int k) {
      fused_barrier();  // A(k): item k is interpolated
      pf.lap(4);
      if (dw == 0 && lane == 0) ccnt[k & 1] = 0;  // item k + 2's tickets (item k's are all taken)
    };
    for (int k = -1;; ++k) {
      const bool next = item_of(k + 1) >= 0;
      // item k + 3 into the slot of item k - 1 (no wave reads it after barrier B(k - 1)); published to the other waves
      // by the waits before the ring syncs and barriers that follow
      if (dw == 0 && lane == 0) qitem[(k + 3) & 3] = item_of(k + 2) >= 0 ? queue.fetch() : -1;
      if (k >= 0) join(k);
      if (!next) break;  // the last item: no build, no grid write, no barriers (the roles meet after it, below)
      if (!(FPTA_FUSED_CUT & 1)) build(k + 1);  // build and write on one path: the accumulators die at the write
      if (k >= 0) barrier_a(k);
      write_grid();
      pf.lap(3);
      fused_barrier();  // B(k): item k + 1's grids are written
      pf.lap(4);
    }
    pf.flush(f.prof, wave);
  } else {
  // ------------------------------------------------------------------ interpolation waves
  Prof pf;  // interpolation waves: 0 next-chunk loads, 1 MFMA steps, 2 stores, 3 barriers, 4 wide-chunk steps, 5 chunks,
            // 6 ticket + stream
  pf.start();
  fused_barrier();  // B(-1)
  pf.lap(3);
  int k = 0;                        // the item whose grids are in LDS (between barriers B(k - 1) and A(k))
  Geo g0 = geo(0), g1 = geo(1);     // items k, k + 1
  bool ex0 = false, ex1 = false;    // this wave found no ticket left in item k / k + 1
  // the next chunk for this wave: a ticket of item k, else of k + 1 (never further: item k + 2's counter is zeroed
  // after A(k)); -1 none. kn = its item.
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
  // chunk cur of item k; the next one's operands (this item's or the next item's) are loaded into nxt first, so their
  // latency hides behind this chunk's MFMAs and they precede this chunk's stores in the vmcnt queue. Loads are never
  // conditional (a load on one side of a branch makes the compiler's vmcnt wait after the join count from the side
  // without it): without a next chunk the current one's operands are loaded again (never used).
  auto step = [&](Ops& cur, Ops& nxt, int& kc) {
    pf.lap(6);
    int kn;
    const int cn = next(kn);
    load(cn >= 0 ? cn : cur.c, nxt, lane);
    pf.lap(0);
    pf.count(5);
    if (!(FPTA_FUSED_CUT & 2)) process(g0, cur, pf, lane);
    kc = kn;
  };
  Ops o0, o1;  // operand sets in turn (two chunks per loop trip: no register copies but at item crossings)
  int kc;      // item of the chunk in o0 (-1: none)
  {
    const int cc = next(kc);
    load(cc >= 0 ? cc : g0.c0, o0, lane);
  }
  for (;;) {
    while (kc == k) {
      step(o0, o1, kc);
      if (kc != k) {
        o0 = o1;  // the next item's chunk (or none): once per item crossing
        break;
      }
      step(o1, o0, kc);
    }
    // no chunk of item k left for this wave: cross A(k), B(k) (not after the last item: nothing follows it)
    if (!g1.valid) break;
    fused_wait_lgkm0();  // every grid read of the item is done
    pf.lap(6);
    fused_barrier();  // A(k)
    fused_barrier();  // B(k)
    pf.lap(3);
    ++k;
    g0 = g1;
    g1 = geo(k + 1);
    ex0 = ex1;
    ex1 = false;
    if (kc < 0) {
      const int cc = next(kc);
      load(cc >= 0 ? cc : g0.c0, o0, lane);
    }
  }
  pf.flush(f.prof, wave);
  }
  // both roles: the successor's mix tickets, then the last barrier
  mix_tiles();
  fused_barrier();
  if (wave < kFusedIW) finish();  // thread 0: after the last barrier, so after every fetch of the workgroup
}

hipError_t launch_grid_fused(hipStream_t st, const SynthArgs& a, const GridBand& band, const FusedArgs& f,
                             int32_t nq_max, size_t lds_bytes, hipEvent_t ev0, hipEvent_t ev1, bool half,
                             int* kernel_out) {
  if (band.n_chunks <= 0 || band.vmax < 4 || f.join_reserve < 0 || band.vmax % 4 != 0 || a.R_pad % kFusedReal != 0 || a.w_on ||
      a.accumulate || a.part || !f.lrows || !f.psr_c0 || f.n_sig <= 0 || f.n_sig > kFusedMaxSig ||
      lds_bytes > (size_t)kFusedLdsMax || nq_max <= 0 || f.ring_off < 0 || f.fq < kFusedNQ || f.fq % 4 != 0 ||
      !f.queue || (size_t)(f.ring_off + 2 * kFusedMaxSig * kFusedSlot) * sizeof(double) + 48 > lds_bytes)
    return hipErrorInvalidValue;
  // half-chunk bands: the kernel holds kFusedHalfNQ steps of each half (a wider half takes the rest one at a time) and
  // loads that many unconditionally (lrows entries, weight rows: the tables are padded past the last half)
  if (half && (!f.h.chunks || !f.h.lrows || !f.h.wd || f.h.fq < kFusedHalfNQ || f.h.fq % 4 != 0 || f.h.vmax < 8 ||
               f.h.vmax % 8 != 0))
    return hipErrorInvalidValue;
  int jobs = 0;
  for (int s = 0; s < f.n_sig; ++s) {
    const FusedSig& fs = f.s[s];
    const int nq = ((((fs.nm + 1) >> 1) + 3) >> 2);  // k-steps of the odd-k parity (the larger)
    if (fs.nf % 4 != 0 || !fs.tq || fs.n_rc != (fs.nf / 4 + 32) / 32 || fs.ldq < 32 * fs.n_rc || 4 * nq > fs.ntq ||
        fs.n_terms <= 0 || fs.n_terms > kDftGenTerms || fs.lrow0 < 0 || (fs.lrow0 + fs.nf) * kFusedPitch > f.ring_off)
      return hipErrorInvalidValue;
    for (int i = 0; i < fs.n_terms; ++i)
      if (fs.term_nm[i] <= 0 || fs.term_nm[i] > fs.nm || (fs.term_kind[i] == 0 && (!fs.term_amp[i] || fs.term_nm[i] % 2)) ||
          (fs.term_kind[i] == 1 && (!a.coef || fs.term_col0[i] < 0 || fs.term_col0[i] + 2 * fs.term_nm[i] > a.K)))
        return hipErrorInvalidValue;
    jobs += fs.n_rc;
  }
  if (jobs > kFusedDW) return hipErrorInvalidValue;
  // the successor's mix: the L^T columns of its 16-pulsar tiles and rows of its k-steps, 16-realization tickets over
  // its R_pad, its columns inside its coefficient rows
  const FusedMix& m = f.mix;
  if (m.n_tiles != 0 &&
      (m.n_tiles < 0 || !m.LT || !m.amp || !m.coef || m.P <= 0 || m.P > kFusedMixMaxP || m.lt_ld < 16 * ((m.P + 15) / 16) ||
       m.lt_rows < 4 * ((m.P + 3) / 4) || m.n_q <= 0 || m.n_q > m.P || m.nm <= 0 || m.R_pad <= 0 ||
       m.R_pad % 16 != 0 || m.n_real <= 0 || m.n_real > m.R_pad || (int64_t)m.n_tiles != (int64_t)m.nm * (m.R_pad / 16) * ((m.P + kFusedMixGroup - 1) / kFusedMixGroup) ||
       m.col0 < 0 || m.col0 + 2 * m.nm > m.K || m.real0 < 0 || m.real0 + m.n_real > ((int64_t)1 << 32)))
    return hipErrorInvalidValue;
  const int32_t n_rb = a.R_pad / kFusedReal;
  const int64_t items = (int64_t)a.P * n_rb;
  if (items > 0x7FFFFFFF || items <= 0) return hipErrorInvalidValue;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  // per device (one process may drive several devices from several threads, fpta_multi_*): its CU count, and whether
  // each instance's dynamic LDS limit is raised past 64 KB
  static std::atomic<int> n_cus[64];
  static std::atomic<bool> attr_set[64][kFusedKernels];
  int n_cu = n_cus[dev].load(std::memory_order_relaxed);
  if (n_cu <= 0) {
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
    n_cus[dev].store(n_cu, std::memory_order_relaxed);
  }
  // persistent: one workgroup per CU (the grids take most of the LDS)
  const int64_t cus = f.cu_pct > 0 && f.cu_pct < 100 ? std::max<int64_t>(8, (int64_t)n_cu * f.cu_pct / 100) : n_cu;
  const int64_t grid = std::min<int64_t>((items + 7) / 8 * 8, (cus + 7) / 8 * 8);
  // NQ: band steps whose operands an interpolation wave holds (a wider chunk takes them NQ at a time)
  // ODD: the first realization is odd, so no lane's realization pair is one Philox pair (the draws take two)
  // GEN: some term is drawn in the kernel
  bool gen = false;
  for (int s = 0; s < f.n_sig; ++s)
    for (int i = 0; i < f.s[s].n_terms; ++i) gen = gen || f.s[s].term_kind[i] == 0;
  const bool odd = gen && (f.real0 & 1);
  const int ki = half ? 6 + (gen ? 1 + odd : 0) : (nq_max <= 8 ? 0 : 3) + (gen ? 1 + odd : 0);
  using K = void (*)(SynthArgs, GridBand, FusedArgs, int32_t, int32_t);
  static const K kernels[kFusedKernels] = {
      k_grid_fused<8, false, false, false>,  k_grid_fused<8, false, true, false>,  k_grid_fused<8, true, true, false>,
      k_grid_fused<12, false, false, false>, k_grid_fused<12, false, true, false>, k_grid_fused<12, true, true, false>,
      k_grid_fused<kFusedHalfNQ, false, false, true>, k_grid_fused<kFusedHalfNQ, false, true, true>,
      k_grid_fused<kFusedHalfNQ, true, true, true>};
  const K kernel = kernels[ki];
  if (!attr_set[dev][ki].load(std::memory_order_acquire)) {
    hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLdsMax);
    if (e != hipSuccess) return e;
    attr_set[dev][ki].store(true, std::memory_order_release);
  }
  // unused descriptors are copies of the first: the kernel's unconditional draw loads read valid memory through them
  FusedArgs fa = f;
  for (int s = f.n_sig; s < kFusedMaxSig; ++s) fa.s[s] = f.s[0];
  (void)hipGetLastError();  // a stale error of an earlier call must not make this launch look failed
  int32_t n_rb_arg = n_rb, items_arg = (int32_t)items;
  void* args[] = {(void*)&a, (void*)&band, (void*)&fa, (void*)&n_rb_arg, (void*)&items_arg};
  // the launch's own status (hipExtLaunchKernelGGL returns none, and hipGetLastError after it could report a stale
  // error while the dispatch still holds the events)
  const hipError_t e = hipExtLaunchKernel((const void*)kernel, dim3((unsigned)grid),
                                          dim3(64 * (kFusedIW + kFusedDW)), args, lds_bytes, st, ev0, ev1, 0);
  if (e == hipSuccess && kernel_out) *kernel_out = ki;
  return e;
}

}  // namespace fpta
