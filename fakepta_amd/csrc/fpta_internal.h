// Internal declarations shared by kernels.hip (device code + launchers) and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpta {

// One GP signal ("segment") of a layout, as the kernels see it.
struct SegDesc {
  const double* w;      // angular frequencies 2*pi*f: kind 0 -> [P][nm], kind 1 -> [nm]
  const double* amp;    // coefficient std-devs sqrt(S*df): same shape as w
  const double* L;      // kind 1: ORF factor [P][P] row-major (x = L z); else null
  const double* LT;     // kind 1: L transposed, zero-padded [lt_rows][lt_ld] (k_mix_mfma operand); else null
  int32_t lt_ld, lt_rows;
  const uint8_t* mask;  // [n_toa_total] or null
  int64_t w_pstride;    // nm (kind 0) or 0 (kind 1)
  double idx;           // chromatic index
  double freqf;         // reference radio frequency (MHz)
  int32_t nm;           // modes, padded to even (padding modes have amp 0)
  int32_t kind;         // 0 per-pulsar, 1 common
  int32_t col0;         // first coefficient column of this segment (cos of mode 0)
  int32_t harmonic;     // 1: w[k] == (k+1) w[0] to rounding -> angle-addition recurrence
  int32_t l_lower;      // kind 1: L is lower-triangular (Cholesky factor) -> triangular mixing
  int32_t n_q;          // kind 1: columns of L up to its last nonzero one (a rank-r factor of a singular ORF, e.g.
                        // monopole r = 1, dipole r = 3): the mix sums q < n_q and draws no normals past them
};

struct SynthArgs {
  const int64_t* offs;    // [P+1]
  const int32_t* psr_of;  // [n_toa]
  const double* toas;     // [n_toa] seconds
  const double* nu;       // [n_toa] MHz
  const SegDesc* segs;    // [n_seg] (device)
  int32_t n_seg;
  int32_t P;
  int64_t n_toa;
  const double* coef;  // [P][K][R_pad]
  int32_t K;
  int32_t R_pad;
  double* out;  // [n_real][ldo]
  int64_t ldo;
  int32_t n_real;
  int32_t accumulate;
  int32_t anchor;
  // white noise + ECORR fused into the epilogue of the seeded VALU kernel (w_on = 1)
  int32_t w_on;
  const double* w_sigma;       // [n_toa] or null
  const int32_t* w_block_of;   // [n_toa] epoch of each TOA (-1: none) or null
  const double* w_esig;        // [n_blocks]
  const double* w_zb;          // [n_real][n_blocks] epoch normals of this batch (w_zb_ld > 0: [n_blocks][w_zb_ld])
  int64_t w_nblocks;
  int64_t w_zb_ld;             // 0: realization-major epoch normals; > 0 epoch-major with this pitch (k_grid_fused_w)
  int64_t real0;               // global index of realization 0 of the batch
  uint32_t k0, k1;             // Philox key (seed)
  // geometry checked by the debug build (FPTA_DCHECK): coefficient values P*K*R_pad, and the TOA x
  // realization tile the tile table was built for (0 when the kernel takes no tile table)
  int64_t coef_len;
  int32_t tile_toa, tile_real;
  // gridded interpolation: partial checksums {sum, sum of squares} of the stored block per (partial group of chunks,
  // realization) [GridBand::n_pg][R_pad], or null (FPTA_OPT_FUSE_CHECKSUMS)
  double* part;
};

// MFMA tile geometry
constexpr int kWR = 4;                  // 16-realization fragments per wave
constexpr int kWT = 2;                  // 16-TOA fragments per wave
constexpr int kWaves = 4;               // waves per workgroup
constexpr int kTileReal = kWR * 16;     // realizations per workgroup
constexpr int kTileToa = kWaves * kWT * 16;  // TOAs per workgroup
constexpr int kRealPad = 128;           // R_pad granularity (multiple of every realization tile)
constexpr int kMixTiledMinP = 64;       // ORF mixing: tiled GEMM from this many pulsars up

// VALU fused-kernel variants: (TOAs per lane MT, realizations per wave NT); workgroup tile is
// 64*MT TOAs x 4*NT realizations.
struct ValuVariant {
  int mt, nt;
};
constexpr ValuVariant kValuVariants[] = {{2, 16}, {4, 16}, {4, 8}, {2, 8}, {1, 32}, {1, 16}};
constexpr int kNumValuVariants = sizeof(kValuVariants) / sizeof(kValuVariants[0]);
// Seeded VALU kernel (harmonic grids): (MT, NT); workgroup tile 256*MT TOAs x NT realizations.
constexpr ValuVariant kSeededVariants[] = {{1, 16}, {2, 16}, {1, 8}, {2, 8}, {1, 32}, {4, 16}};
static_assert(sizeof(kSeededVariants) == sizeof(kValuVariants), "one variant index selects both tables");

// Gridded synthesis (grid.hip): one signal's tables as the kernels see them.
constexpr int kGridVMax = 256;  // band rows per chunk, all signals (k_grid_interp_mfma keeps them in 4 VGPRs)
constexpr int kGridMinV = 16;  // band rows per chunk at least (k_grid_interp_st: 4 MFMA steps, its lookahead + 1)
constexpr int kGridTT = 32;  // TOAs per interpolation chunk (k_grid_interp_mfma: even / odd TOAs = two MFMA B-tiles)
constexpr int kGridMI = 8;   // grid rows per wave in k_grid_dft
#ifndef FPTA_DFT_MJ
#define FPTA_DFT_MJ 2
#endif
constexpr int kDftMJ = FPTA_DFT_MJ;      // k_grid_dft_mfma wave tile: 16 MJ grid rows x 16 kDftMR realizations
constexpr int kDftMR = 4 / FPTA_DFT_MJ;  // (the accumulators stay at 4 MJ MR = 16 tiles: two parities, cos and sin)
constexpr int kGridDftRows = 16 * kDftMJ;  // grid rows per k_grid_dft_mfma row block (quarter range) and k_grid_dft (half)
struct GridSegDev {
  const double* ecos;  // [nm][lde] q_k cos(2 pi k j / nf), k = m + 1 (zero-padded columns)
  const double* esin;  // [nm][lde] q_k sin(2 pi k j / nf)
  double* g;           // [P][nf][R_pad] grid values of the batch (this signal's block of the grid buffer)
  int32_t nf, half, lde, nm, col0;
  int32_t ntab;        // mode rows of ecos/esin (nm zero-padded to a multiple of 8)
  int32_t nblk;        // k_grid_dft row blocks of this signal (set by launch_grid_dft*)
  const double* tq;    // k_grid_dft_mfma: [4][ntq][ldq] q_k cos / sin(2 pi k j / nf), j <= nf / 4, for the modes of
                       // odd k (m = 2 t) and of even k (m = 2 t + 1), t < ntq (zero-padded)
  int32_t ldq, ntq;
};
constexpr int kGridMaxSeg = 16;  // signals per layout on the gridded path (passed by value as kernel arguments)
struct GridSegs {
  GridSegDev s[kGridMaxSeg];
  int32_t n;
};

// Coalesced grid signal (FPTA_OPT_GRID_COALESCE): coef[p][dst + j][r] += sum_i coef[p][src_i + j][r], j < ncol_i,
// in source order (deterministic), before the DFT of the group reads columns dst ..
struct CoefMerge {
  int32_t dst;               // first coefficient column of the group's anchor (largest mode count)
  int32_t n;                 // other members
  int32_t src[kGridMaxSeg];  // first column of each other member
  int32_t ncol[kGridMaxSeg]; // its columns (2 x padded modes)
};
hipError_t launch_coef_merge(hipStream_t st, const CoefMerge& m, int32_t P, int32_t K, int32_t R_pad, double* coef);

hipError_t launch_grid_weights(hipStream_t st, const SegDesc& sd, int64_t n_toa, const double* nu,
                               const int32_t* chunk_of, const int32_t* tt_of, const int32_t* row_of,
                               const double* d_of, int32_t w, double beta, int32_t vmax, double* wd,
                               double* dch = nullptr, int32_t s_idx = 0, int32_t n_sig = 1, int32_t half = 0);
hipError_t launch_grid_dft(hipStream_t st, GridSegs gsegs, int32_t P, const double* coef, int32_t K, int32_t R_pad);
// the same two steps on v_mfma_f64_16x16x4_f64 (grid_mfma.hip)
hipError_t launch_grid_dft_mfma(hipStream_t st, GridSegs gsegs, int32_t P, const double* coef, int32_t K,
                                int32_t R_pad);
// Fused draw + DFT of one grid signal with at least one per-pulsar member (k_grid_dft_gen): the B operand of every
// MFMA step is built in registers, term by term in the grid signal's summation order (anchor first, then the other
// members in layout order): a per-pulsar member's coefficient amp * z from its own Philox stream (the k_gen counter
// {mode, pulsar, signal, realization}: the same draws), a common member's mixed coefficients loaded from its own
// columns of the coefficient buffer. No k_gen launch and no coefficient round trip for per-pulsar members.
constexpr int kDftGenTerms = 8;
struct DftGenArgs {
  GridSegDev g;             // the grid signal's tables and its block of the grid buffer (nm: the anchor's modes)
  int32_t n_terms;
  int32_t term_kind[kDftGenTerms];   // 0: generated (per-pulsar member), 1: loaded (mixed common member)
  int32_t term_seg[kDftGenTerms];    // layout index of the member (Philox counter word 2)
  int32_t term_nm[kDftGenTerms];     // the member's padded modes
  int32_t term_col0[kDftGenTerms];   // loaded: first coefficient column
  const double* term_amp[kDftGenTerms];  // generated: [P][term_nm] sqrt(S df)
  const double* coef;       // [P][K][R_pad]
  int32_t P, K, R_pad, n_real;
  int64_t real0;
  uint32_t k0, k1;
};
hipError_t launch_grid_dft_gen(hipStream_t st, const DftGenArgs& a);

// Interpolation band of the whole layout: per chunk of <= kGridTT TOAs the band rows of every signal back to back
// (V rows, a multiple of 4), the grid-buffer row of each and the weights of each (row, TOA).
struct GridBand {
  const int4* chunks;   // [n_chunks] {pulsar, first TOA (pulsar-local), count, V}
  const int32_t* rows;  // [n_chunks][vmax] grid-buffer row of band row v
  const double* wd;     // [n_chunks][vmax][kGridTT] weights
  const double* g;      // [grid_rows][R_pad] grid values (all signals)
  int32_t n_chunks, vmax;
  int64_t grid_rows;
  // fused partial checksums: [n_pg + 1] first chunk of each partial group (runs of consecutive chunks of one pulsar,
  // one partial row each); null: one chunk per group (n_pg = n_chunks)
  const int32_t* pgfirst;
  int32_t n_pg;
};
hipError_t launch_grid_interp_mfma(hipStream_t st, const SynthArgs& a, const GridBand& band, int32_t R_pad);
// Warp-specialised variant (producer waves stage operands in an LDS ring, compute waves never load from global memory,
// so their stores never hold up an operand); no white epilogue, no accumulate
// ws2: k_grid_interp_ws2 (64-realization compute tiles, two workgroups per CU), plain blocks only
hipError_t launch_grid_interp_ws(hipStream_t st, const SynthArgs& a, const GridBand& band, int32_t R_pad,
                                 bool ws2 = false);
// Window-ring variant (k_grid_interp_wr, diagnostic builds only): a workgroup walks a contiguous range of chunks for 256 realizations; each
// grid signal's band rows stay in a ring of kWrSlots LDS rows (slot = unwrapped row mod kWrSlots), so producer waves
// load only the rows the previous chunk's band did not hold, plus the chunk's weights; one barrier per chunk (two
// when the bands do not fit one window). Plain blocks, <= kWrMaxSig grid signals, R_pad a multiple of 256.
constexpr int kWrSlots = 32, kWrMaxSig = 2, kWrVMax = 40, kWrReal = 256;  // 128 + 30 KB of LDS
constexpr int kWrFresh = 1 << 30;  // GridWindow::meta .w flag: load every band row, after the previous chunk is done
constexpr int kWrFar = 1 << 29;    // .w flag: the new rows may load only once the chunk two back is done
constexpr int kWrBufs = 3;         // weight buffers: the chunk being computed, the next one, the one after
struct GridWindow {
  const int4* meta;    // [n_chunks] {full list offset, full count, new list offset, new count | kWrFresh}
  const int2* list;    // {LDS slot, grid-buffer row} load items
  const int32_t* slot; // [n_chunks][vmax] LDS slot of each band row
};
hipError_t launch_grid_interp_wr(hipStream_t st, const SynthArgs& a, const GridBand& band, const GridWindow& wr,
                                 int32_t R_pad);
// Per-pulsar variant for one small grid signal (nf <= 124, vmax <= 32, no white epilogue): a workgroup makes one
// pulsar's grid for 64 realizations in LDS (k_grid_dft_mfma's quarter-range DFT from the coefficient buffer) and
// interpolates the pulsar's chunks from it; no grid buffer. psr_grp [P + 1]: the first partial group (a.part) or chunk
// of each pulsar. Bit-identical to k_grid_dft_mfma + k_grid_interp_mfma.
hipError_t launch_grid_interp_psr(hipStream_t st, const SynthArgs& a, const GridBand& band, const GridSegDev& gs,
                                  const int32_t* psr_grp, int32_t P, int32_t R_pad);
// Fused per-pulsar synthesis (k_grid_fused, grid_fused.hip): persistent workgroups, each walking items = (pulsar,
// kFusedReal realizations). Per item, kFusedDW DFT waves draw every grid signal's coefficients (k_grid_dft_gen's terms
// and order) through a two-slot LDS ring and run the signal's quarter-range DFT on fp64 MFMA into registers (one
// 32-row chunk each); kFusedIW interpolation waves meanwhile interpolate the previous item's chunks from its LDS grid
// (k_grid_interp_ws's MFMA steps). At the item boundary the DFT waves write the next grid. No grid buffer, no DFT
// launch; bit-identical to the two-kernel path.
constexpr int kFusedMaxSig = 2;    // grid signals (the draw ring holds a group of each)
constexpr int kFusedReal = 32;     // realizations per item (two 16-realization MFMA tiles)
constexpr int kFusedPitch = 32;    // doubles per LDS grid row
constexpr int kFusedIW = 4;        // interpolation waves per workgroup
constexpr int kFusedDW = 4;        // DFT waves per workgroup = DFT jobs (32-row quarter-range chunks) at most
constexpr int kFusedGroupModes = 16;  // modes per draw group: two 4-mode k-steps of both parities
constexpr int kFusedSlot = kFusedGroupModes * kFusedReal * 2;  // doubles per signal of a ring slot [16 modes][32][cos, sin]
constexpr int kFusedLdsMax = 160 * 1024;
constexpr int kFusedNQ = 12;       // band steps whose operands an interpolation wave holds (a wider chunk: the rest one
                                   // step at a time)
constexpr int kFusedWdPad = 4 * 16;  // band rows of zero weights past the last chunk (GridPlan::wd): the most
                                     // unconditional band-step loads of a fused kernel (kFusedWNQ)
constexpr int kFusedTerms = 2;     // members of a grid signal whose inputs the DFT waves prefetch (the others: inline)
struct FusedSig {
  const double* tq;  // quarter-range tables [4][ntq][ldq] (GridSegDev::tq)
  int32_t ldq, ntq, nf, nm;  // nm: the anchor's padded modes
  int32_t lrow0;     // first LDS grid row of the signal
  int32_t n_rc;      // 32-row chunks of its quarter range (one DFT job each)
  int32_t n_terms;   // as DftGenArgs: generated (per-pulsar) and loaded (coefficient-buffer) terms, summation order
  int32_t term_kind[kDftGenTerms];
  int32_t term_seg[kDftGenTerms];
  int32_t term_nm[kDftGenTerms];
  int32_t term_col0[kDftGenTerms];
  const double* term_amp[kDftGenTerms];
};
// Half-chunk bands (k_grid_fused<.., HALF = true>): each 32-TOA chunk's TOAs 0..15 and 16..31 have bands of their own
// (C2: 32 instead of 36 band rows per chunk and half, 11 % fewer interpolation MFMAs). A half's weights are [vmax_h][16
// TOAs], laid out by pairs of band steps so that lane (TOA tt, row group j) reads steps 2 qp and 2 qp + 1 of band rows
// 4 q + j with one 16-byte load: element (v, tt) at ((v / 8 * 4 + v % 4) * 16 + tt) * 2 + (v / 4) % 2.
constexpr int kFusedHalfTT = 16;
constexpr int kFusedHalfNQ = 8;  // band steps of each half whose operands an interpolation wave holds
__host__ __device__ __forceinline__ int64_t fused_half_weight_index(int32_t v, int32_t tt) {
  return ((int64_t)((v >> 3) * 4 + (v & 3)) * kFusedHalfTT + tt) * 2 + ((v >> 2) & 1);
}
struct FusedHalf {
  const int4* chunks;    // [n_chunks] {pulsar, first TOA, count, nq0 | nq1 << 16}: band steps of each half
  const int32_t* lrows;  // [n_chunks][2][4][fq] LDS grid row of band row 4 q + j of half h at [h][j][q]
  const double* wd;      // [2 n_chunks][vmax][16] weights (fused_half_weight_index), + zero rows past the last
  int32_t fq, vmax;      // band steps per (chunk, half, j) in lrows (a multiple of 4); band rows per half (mult. of 8)
};
// The next block's common-signal draws + ORF mix (k_gen_mix's work for one signal) as spare-time tickets of
// k_grid_fused: a pipelined block whose successor is predictable (the same key, the next realizations) lets its
// kernel's waves with nothing left to interpolate or build make that block's mixed coefficients, so the successor
// launches no k_gen_mix. A ticket is one (mode, 16 realizations, 64 pulsars) tile: the pulsars' coefficients of both
// columns, the draws in registers (one Philox call per lane and k-step), the mix on fp64 MFMA per 16-pulsar tile.
// Bit-identical to k_gen_mix (the same normals, the same products per k-step in the same order: k-steps past a
// triangular factor's diagonal add exact zeros there). DESIGN.md §5a.
constexpr int kFusedMixMaxP = 256;   // pulsars of a signal whose mix k_grid_fused makes (k_gen_mix's limit)
constexpr int kFusedMixGroup = 112;  // pulsars per ticket (seven 16-pulsar MFMA tiles, both columns: 112 VGPRs of sums)
struct FusedMix {
  const double* LT;     // SegDesc::LT of the signal (zero-padded L^T)
  const double* amp;    // [nm] mode amplitudes
  double* coef;         // the successor's coefficient buffer [P][K][R_pad]
  int64_t real0;        // the successor's first realization
  uint32_t k0, k1;      // its Philox key
  int32_t lt_ld, lt_rows, P, K, col0, R_pad, n_real, n_q, lower, seg, nm;
  int32_t n_tiles;      // nm x R_pad / 16 x ceil(P / 64) tickets; 0: no successor mix in this launch
};
constexpr int kFusedArgSig = 3;  // grid signal descriptors a FusedArgs holds (k_grid_fused takes kFusedMaxSig of them)
struct FusedArgs {
  FusedSig s[kFusedArgSig];
  int32_t n_sig;
  int32_t ring_off;       // LDS offset (doubles) of the draw ring (past the grids); a sync word follows it
  const int32_t* lrows;   // [n_chunks][4][fq] LDS grid row of band row 4 q + j at [j][q]
  int32_t fq;             // band steps per (chunk, j) in lrows (a multiple of 4, >= kFusedNQ)
  const int32_t* psr_c0;  // [P + 1] first chunk of each pulsar
  int64_t real0;          // the batch's first realization (Philox counter)
  uint32_t k0, k1;
  unsigned long long* prof;  // -DFPTA_FUSED_PROF builds only: per-wave cycle counters [gridDim][8 waves][8]; else null
  uint32_t* queue;           // [kFusedQueueWords], zero at launch; the kernel's last workgroup zeroes it again
  int32_t join_reserve;      // the DFT waves interpolate an item's chunks while more than this many are left
  FusedHalf h;               // half-chunk bands (HALF kernels only; else zero)
  int32_t cu_pct;            // host only: workgroups for this percentage of the CUs (0 = all), leaving the rest to a
                             // co-running kernel (the next block's ORF mix)
  FusedMix mix;              // the successor block's common-signal mix (k_grid_fused only; n_tiles 0 = none)
};
#ifndef FPTA_FUSED_MIX_CU_PCT
#define FPTA_FUSED_MIX_CU_PCT 100  // CUs of k_grid_fused's grid while the next block's k_mix_mfma may co-run
#endif
constexpr int kFusedQueueWords = 10;  // 8 per-XCD item tickets, the count of finished workgroups, the mix tickets
constexpr int kFusedMixWord = 9;
#ifndef FPTA_FUSED_JOIN_SAFETY
#define FPTA_FUSED_JOIN_SAFETY 1.5  // measured best of 0.5 .. 5 on C2 and C4 (profiles/round5/r5mn_*); variants may change it (make variant DEFS=-DFPTA_FUSED_JOIN_SAFETY=...)
#endif
constexpr double kFusedJoinSafety = FPTA_FUSED_JOIN_SAFETY;  // FusedArgs::join_reserve over the estimated need
#ifndef FPTA_FUSED_W_JOIN_SAFETY
#define FPTA_FUSED_W_JOIN_SAFETY 1.5  // the same for k_grid_fused_w
#endif
constexpr double kFusedWJoinSafety = FPTA_FUSED_W_JOIN_SAFETY;
// nq_max: band steps of the widest chunk (vmax / 4; the kernel holds up to 12 steps' operands and takes a wider chunk's
// in turns); lds_bytes: grids + ring + sync word; ev0 / ev1: timing events bound to the dispatch (hipExtLaunchKernel)
// half: the HALF kernel on f.h (nq_max: band steps of the widest half); *kernel_out (optional): the instance launched,
// fused_kernel_name's index
hipError_t launch_grid_fused(hipStream_t st, const SynthArgs& a, const GridBand& band, const FusedArgs& f,
                             int32_t nq_max, size_t lds_bytes, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                             bool half = false, int* kernel_out = nullptr);
// White-epilogue variant (k_grid_fused_w, grid_fused_w.hip): gridded blocks with white noise / ECORR (C5: RN + three
// common signals, DM and Sv: three grid signals of 884 rows). Items are (pulsar, kFusedWReal realizations), so every
// grid signal's grid fits in LDS; up to kFusedWMaxSig grid signals and 2 kFusedDW DFT jobs (two per DFT wave); draw
// groups of kFusedWGroupModes modes (one (mode, realization pair) per DFT lane); the interpolation waves add white
// noise and ECORR (epoch normals from the block's SynthArgs::w_zb) before their stores.
constexpr int kFusedWReal = 16, kFusedWPitch = 16, kFusedWMaxSig = 3, kFusedWGroupModes = 32;
constexpr int kFusedWSlot = kFusedWGroupModes * kFusedWReal * 2;  // doubles per signal of a ring slot [32][16][cos, sin]
constexpr int kFusedWJobs = 2 * kFusedDW;
constexpr int kFusedWNQ = 16;  // band steps whose operands an interpolation wave holds
hipError_t launch_grid_fused_w(hipStream_t st, const SynthArgs& a, const GridBand& band, const FusedArgs& f,
                               int32_t nq_max, size_t lds_bytes, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                               int* kernel_out = nullptr);
constexpr int kFusedWKernels = 2;  // instances: draws from an even / odd first realization
constexpr int kFusedKernels = 9;  // instances: {NQ 8, NQ 12} x {no draws, draws, draws from an odd realization},
                                  // then HALF (NQ 8 per half) x the same three
// Storer-wave variant: compute waves hand finished sums to storer waves through LDS; every block kind (white / ECORR
// epilogue, partial checksums, accumulate) with R_pad a multiple of 128
hipError_t launch_grid_interp_st(hipStream_t st, const SynthArgs& a, const GridBand& band, int32_t R_pad);
// LDS-staged variant: the 4 waves of a workgroup take <= kLdsGroup consecutive chunks of one pulsar for the same
// realizations; the union of their band rows (<= kLdsRowsMax) is loaded once into LDS
constexpr int kLdsGroup = 4, kLdsRowsMax = 144;
struct GridLds {
  const int4* groups;   // [n_groups] {first chunk, chunks, union rows U, offset into urows}
  const int32_t* urows; // grid-buffer rows of each group's union
  const int32_t* lrows; // [n_chunks][vmax] union slot of each band row
  int32_t n_groups, lds_rows;
};
hipError_t launch_grid_interp_lds(hipStream_t st, const SynthArgs& a, const GridBand& band, const GridLds& lds,
                                  int32_t R_pad);
// Union-row interpolation (k_grid_interp_u): a workgroup takes a group of <= kUnionGroup consecutive chunks of one
// pulsar for 128 realizations, stages the union of their band rows (<= kUnionRowsMax rows over all signals) in LDS
// once, and each compute wave interpolates one chunk from it with its weights made on the fly (es_weight); layouts of
// <= kUnionSigMax grid signals.
constexpr int kUnionGroup = 4, kUnionRowsMax = 76, kUnionSigMax = 2, kUnionPitch = 130;
struct GridUnion {
  const int4* groups;    // [n_groups] {first chunk, chunks, union rows U, offset into urows}
  const int32_t* urows;  // grid-buffer rows of each group's union (signal by signal)
  const int32_t* cbase;  // [n_chunks][2 kUnionSigMax] per signal: first band row voff_s, union slot of band row 0 of
                         // the signal's band minus voff_s (slot = v + base)
  const double* dch;     // [n_chunks][n_sig][kGridTT] {d, ch} per TOA slot (double pairs)
  const int32_t* wrow;   // [n_chunks][n_sig][kGridTT] band row of the TOA's window start (voff_s included; empty slot:
                         // a large negative value, so every weight is 0)
  int32_t n_groups, n_sig;
  int32_t w[kUnionSigMax];
  double hw[kUnionSigMax], beta[kUnionSigMax];
};
hipError_t launch_grid_interp_u(hipStream_t st, const SynthArgs& a, const GridBand& band, const GridUnion& un,
                                int32_t R_pad);
// checksums [n_real][2] from the interpolation's partials [n_rows][R_pad][2] (one row per group of part_group
// consecutive chunks), summed over rows in a fixed order: one pass (k_part_sums) for n_rows <= kPartOneRows, else two
// (tmp: kPartSegs * R_pad * 2 doubles). sums may be pinned host memory.
constexpr int kPartSegs = 64;
constexpr int kPartOneSegs = 16, kPartOneRows = 16 * 48;
constexpr int kPartGroup = 16, kPartGroupMax = 16;
hipError_t launch_part_checksums(hipStream_t st, const double* part, int32_t n_rows, int32_t R_pad, int32_t n_real,
                                 double* tmp, double* sums);

hipError_t launch_seeds(hipStream_t st, const SegDesc* segs, int32_t n_seg, const int32_t* psr_of,
                        const double* toas, const double* nu, int64_t n_toa, double4* seeds);
hipError_t launch_synth_valu_seeded(hipStream_t st, const SynthArgs& a, const int4* tiles, int32_t n_tiles,
                                    const double4* seeds, int variant);

hipError_t launch_gen(hipStream_t st, const SegDesc& sd, int32_t seg_id, int32_t P, int32_t n_real,
                      int32_t R_pad, int64_t real0, uint32_t k0, uint32_t k1, const double* zin,
                      int32_t zin_nseg, int32_t zin_nm, double* coef, int32_t K, double* zbuf);
hipError_t launch_mix(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                      double* coef, int32_t K, double* x_out);
// the same product on v_mfma_f64_16x16x4_f64 (grid_mfma.hip), the large-array path. acc_col0 >= 0: add the mixed
// coefficients into columns acc_col0 .. (a coalesced grid signal's anchor) instead of writing the signal's own
hipError_t launch_mix_mfma(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                           double* coef, int32_t K, double* x_out, int32_t acc_col0 = -1);
// draw + mixing of a common signal in one kernel (kMixTiledMinP <= P <= kGenMixMaxP): writes the signal's own columns
constexpr int kGenMixMaxP = 256;
hipError_t launch_gen_mix(hipStream_t st, const SegDesc& sd, int32_t seg_id, int32_t P, int32_t n_real, int32_t R_pad,
                          int64_t real0, uint32_t k0, uint32_t k1, double* coef, int32_t K, int rh = 2, int rb = 32,
                          hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
hipError_t launch_mix_tiled(hipStream_t st, const SegDesc& sd, int32_t P, int32_t R_pad, const double* zbuf,
                            double* coef, int32_t K, double* x_out);
// epoch-major [n_blocks][ldz] (ldz >= n_real, even): a realization's normals of one epoch are contiguous, so
// k_grid_fused_w's gathers of an epoch's realization pairs are 16-byte loads (the same normals as launch_epoch_normals)
hipError_t launch_epoch_normals_t(hipStream_t st, int64_t n_blocks, int32_t n_real, int64_t real0, uint32_t k0,
                                  uint32_t k1, double* zb, int64_t ldz);
hipError_t launch_epoch_normals(hipStream_t st, int64_t n_blocks, int32_t n_real, int64_t real0, uint32_t k0,
                                uint32_t k1, double* zb);
hipError_t launch_white_pairs(hipStream_t st, const double* sigma, const int32_t* block_of, const double* esig,
                              int64_t n_blocks, const double* zb, double* out, int64_t ldo, int64_t n_toa,
                              int32_t n_real, int64_t real0, uint32_t k0, uint32_t k1);
hipError_t launch_synth_direct(hipStream_t st, const SynthArgs& a);
hipError_t launch_synth_mfma(hipStream_t st, const SynthArgs& a, const int4* tiles, int32_t n_tiles);
hipError_t launch_synth_valu(hipStream_t st, const SynthArgs& a, const int4* tiles, int32_t n_tiles, int variant);
hipError_t launch_white(hipStream_t st, const double* sigma, const int32_t* block_of, const double* esig,
                        const double* z, const double* zb, double* out, int64_t ldo, int64_t n_toa,
                        int32_t n_real, int64_t real0, uint32_t k0, uint32_t k1);
hipError_t launch_checksums(hipStream_t st, const double* out, int64_t ldo, int64_t n_toa, int32_t n_real,
                            double* sums);
hipError_t launch_correlations(hipStream_t st, const double* out, int64_t ldo, int32_t n, int32_t P, int32_t n_real,
                               int32_t mode, double* autos, double* parts, int32_t nparts, double* dst);
hipError_t launch_philox(hipStream_t st, int64_t n, const uint32_t* ctr, uint32_t k0, uint32_t k1,
                         uint32_t* out);
hipError_t launch_normals4(hipStream_t st, int64_t n, const uint32_t* words, double* out);

// dense-covariance path (dense.hip)
hipError_t launch_cov_basis(hipStream_t st, const double* toas, const double* nu, int64_t n, const double* f,
                            const double* sw, const int32_t* seg_of, const double* seg_idx, const double* seg_freqf,
                            int32_t n_modes, int32_t k_pad, double* GT, int64_t ldn);
hipError_t launch_gemm_tn(hipStream_t st, const double* a, int64_t lda, const double* b, int64_t ldb, bool b_rows,
                          bool b_tri, double* c, int64_t ldc, int64_t m, int64_t n, int32_t k4, int32_t lower,
                          int32_t tile0, int32_t mode, const double* diag);
hipError_t launch_potrf_block(hipStream_t st, double* C, int64_t ldc, int64_t n, int64_t k0, int* info);
hipError_t launch_trsm_panel(hipStream_t st, double* C, int64_t ldc, int64_t n, int64_t k0, double* PT,
                             int64_t ldp);
hipError_t launch_chol_solve(hipStream_t st, const double* C, int64_t ldc, int64_t n, const double* r,
                             const double* white, double* y, double* out);
hipError_t launch_dense_normals(hipStream_t st, int64_t n, int64_t rows, int32_t n_real, int64_t real0, uint32_t k0,
                                uint32_t k1, double* ZT, int64_t ldz);

}  // namespace fpta
