// Host side of libfakepta_amd.so shared by its translation units (not part of the C-ABI): capi.hip (context, options,
// drop-in and batch entry points, path selection, dense covariance), grid_host.hip (the gridded plan and its launches)
// and multi.hip (several devices in one process; one process per GPU over RCCL). All arithmetic on the path runs in
// the kernels (kernels.hip, grid_mfma.hip, grid_fused.hip, dense.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fakepta_amd.h"
#include "fpta_internal.h"

using namespace fpta;

namespace __attribute__((visibility("hidden"))) capi {  // library-internal: not exported

extern thread_local std::string g_err;  // the last error of a call without a context

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
  }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap && p) return hipSuccess;
    release();
    size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct Seg {
  SegDesc d{};
  int32_t nm_orig = 0;
  std::vector<double> h_w0;  // first angular frequency per row ([P] for kind 0, [1] for kind 1)
  std::vector<uint8_t> h_mask;  // host copy of the TOA mask (empty: none), for grid coalescing
  DevBuf w, amp, L, LT, mask;
};

// Gridded-synthesis tables of one signal (grid.hip): real-DFT table E; its grid block starts at row rowoff of
// the plan's grid buffer.
struct GridSeg {
  int32_t nf = 0, half = 0, lde = 0, ntab = 0;
  int64_t rowoff = 0;
  DevBuf ecos, esin;  // half-range tables (k_grid_dft)
  int32_t ldq = 0, ntq = 0;
  DevBuf tq;          // quarter-range tables by mode parity (k_grid_dft_mfma)
};

// Gridded-synthesis plan of a layout (built once per layout, reused by every batch).
// fpta_batch_grid_info_n slot 15 (1 + 4 kind + 2 white + part): kinds 0 .. 10 the interpolation kernels
// (_capi.interp_kernel_name), kInterpKindFused0 + i k_grid_fused instance i of launch_grid_fused's table
constexpr int kInterpKindFused0 = 11;
struct GridPlan {
  bool built = false;
  bool ok = false;           // usable for this layout (harmonic, <= kGridMaxSeg signals)
  std::string why;           // reason when !ok
  int32_t w = 0;             // kernel width (grid cells)
  double sigma = 0.0;        // oversampling
  int32_t n_chunks = 0;
  DevBuf chunks;             // int4 {pulsar, first TOA (pulsar-local), count, band rows V (multiple of 4)}
  int32_t vmax = 0;          // largest V: row pitch of the row-index and weight tables
  int64_t grid_rows = 0;     // rows of the grid buffer: sum over signals of P nf
  DevBuf rows;               // [n_chunks][vmax] int32 grid-buffer row of each band row (all signals back to back)
  DevBuf wd;                 // [n_chunks][vmax][kGridTT] interpolation weights (chromatic factor, mask folded in)
  DevBuf g, g2;              // [grid_rows][R_pad] grid values of the batch (two buffers when pipelined)
  std::vector<int32_t> psr_chunk0;  // [P + 1] first chunk of each pulsar (chunks are pulsar-major)
  // partial-checksum groups (FPTA_OPT_FUSE_CHECKSUMS): <= pg_size consecutive chunks of one pulsar each; pgfirst
  // [n_pg + 1] the first chunk of each group, psr_pg [P + 1] the first group of each pulsar
  int32_t pg_size = 0, n_pg = 0;
  DevBuf pgfirst, psr_pg;
  DevBuf psr_c0;  // device copy of psr_chunk0 (k_grid_interp_psr without partial checksums)
  // k_grid_fused plan (FPTA_OPT_INTERP_FUSED): every grid signal's grid for kFusedReal realizations in LDS (signal s
  // at LDS row fused_lrow0[s]), the draw ring after them; frows [n_chunks][vmax] the LDS row of each band row;
  // fused_lds the workgroup's LDS bytes
  bool fused_ok = false;
  size_t fused_lds = 0;
  bool fused_w_ok = false;  // k_grid_fused_w's plan (16-realization grids, <= 3 grid signals); frows serves both
  size_t fused_w_lds = 0;
  bool frows_ok = false;
  int32_t fused_fq = 0;  // band steps per (chunk, lane group) in frows
  std::vector<int32_t> fused_lrow0;
  DevBuf frows;
  // half-chunk bands of the fused kernel (FusedHalf): hchunks {pulsar, first TOA, count, nq0 | nq1 << 16}, hrows
  // [n_chunks][2][4][fused_hfq], hwd [2 n_chunks][fused_hvmax][16] (+ padding); fused_half_gain = the interpolation
  // MFMAs of whole-chunk bands over those of half-chunk bands
  bool fused_half_ok = false;
  int32_t fused_hfq = 0, fused_hvmax = 0, fused_hnq = 0;
  double fused_half_gain = 0.0;
  double fma_interp_half = 0.0;  // interpolation FMAs per realization on half-chunk bands (both halves run max(nq0, nq1) steps)
  DevBuf hchunks, hrows, hwd;
  // k_grid_interp_wr plan (GridWindow): <= 2 grid signals, each signal's band rows in a ring of kWrSlots LDS slots by
  // unwrapped row; per chunk the slot of each band row, and the rows to load: all its band rows (full) or those not in
  // the previous chunk's band (new; = full and flagged fresh when the two bands do not fit one ring window)
  bool wr_ok = false;
  DevBuf wr_meta, wr_list, wr_slot;
  // k_grid_interp_lds plan: groups int4 {first chunk, chunks, union rows U, offset into urows}; urows the grid-
  // buffer rows of each group's union; lrows [n_chunks][vmax] the union slot of each band row
  bool lds_ok = false;
  int32_t n_groups = 0, lds_rows = 0;
  DevBuf groups, urows, lrows;
  // k_grid_interp_u plan (GridUnion): groups of <= kUnionGroup chunks with <= kUnionRowsMax union rows; per chunk the
  // signals' band offsets and union bases; per (chunk, signal, TOA slot) the window's first band row and {d, ch}
  bool u_ok = false;
  int32_t u_groups = 0, u_sig = 0;
  DevBuf ugroups, uurows, ucbase, udch, uwrow;
  int32_t u_w[kUnionSigMax] = {0, 0};
  double u_hw[kUnionSigMax] = {0.0, 0.0}, u_beta[kUnionSigMax] = {0.0, 0.0};
  std::vector<GridSeg*> segs;  // one per grid signal
  // grid signals (FPTA_OPT_GRID_COALESCE): members (layout signal indices, ascending), the anchor (the member with
  // the most modes: its coefficient columns receive the others' and its grid/weights serve the group) and the last
  // member (the group's coefficients are complete once it is drawn)
  std::vector<std::vector<int32_t>> members;
  std::vector<int32_t> anchor, last;
  bool merges = false;       // some grid signal has > 1 member
  double mean_v = 0.0;       // mean band rows per chunk
  double fma_grid = 0.0;     // FMAs per realization: DFT + interpolation
  double fma_dft = 0.0;      // FMAs per realization in k_grid_dft
  double fma_interp = 0.0;   // FMAs per realization in k_grid_interp (dense band, padded TOA slots)
  double grid_vals = 0.0;    // grid values per realization (sum over signals of P nf)
  double weight_bytes = 0.0; // interpolation weight tables
  double fma_direct = 0.0;   // FMAs per realization of the direct contraction
  double err_bound = 1.0;    // a-priori relative aliasing bound of the ES kernel, exp(-pi w sqrt(1 - 1/sigma))
  int64_t g_rpad = 0;        // R_pad the grid buffers are sized for
  ~GridPlan() { clear(); }
  void clear() {
    for (GridSeg* g : segs) delete g;
    segs.clear();
    built = ok = false;
    n_chunks = 0;
    vmax = 0;
    lds_ok = false;
    n_groups = lds_rows = 0;
    u_ok = false;
    u_groups = u_sig = 0;
    grid_rows = 0;
    g_rpad = 0;
    psr_chunk0.clear();
    pg_size = n_pg = 0;
    wr_ok = false;
    fused_ok = false;
    fused_lds = 0;
    fused_w_ok = false;
    fused_w_lds = 0;
    frows_ok = false;
    fused_lrow0.clear();
    fused_half_ok = false;
    fused_hfq = fused_hvmax = fused_hnq = 0;
    fused_half_gain = 0.0;
    fma_interp_half = 0.0;
    members.clear();
    anchor.clear();
    last.clear();
    merges = false;
    mean_v = 0.0;
    // the plan figures accumulate over signals in grid_build: a rebuilt plan must start from zero
    fma_grid = fma_dft = fma_interp = grid_vals = weight_bytes = fma_direct = 0.0;
    err_bound = 1.0;
    why.clear();
  }
};

// A device-resident pulsar array plus its GP signals.
struct Layout {
  int32_t P = 0;
  int64_t n_toa = 0;
  int64_t max_np = 0;
  std::vector<int64_t> h_offs;
  std::vector<double> h_toas, h_nu;
  DevBuf offs, toas, nu, psr_of;
  std::vector<Seg*> segs;
  DevBuf segdesc;
  int32_t K = 0;
  bool dirty = true;
  uint64_t version = 0;  // bumped by every layout_finalize that rebuilds (signals, TOAs changed)
  // recurrence seeds [n_seg][n_toa] (double4), valid when every segment is harmonic
  DevBuf seeds;
  bool all_harmonic = false;
  // tile table cache of the tiled synthesis kernels: valid for (tiles_toa, tiles_real, tiles_n_real)
  DevBuf tiles;
  int32_t n_tiles = 0;
  int32_t tiles_toa = 0, tiles_real = 0;
  int64_t tiles_n_real = -1;
  GridPlan grid;
  ~Layout() { clear_signals(); }
  void clear_signals() {
    for (Seg* s : segs) delete s;
    segs.clear();
    K = 0;
    dirty = true;
    tiles_n_real = -1;
    grid.clear();
  }
};

}  // namespace capi

using namespace capi;

struct fpta_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  Layout batch, scratch;
  // batch white noise
  DevBuf sigma, block_of, esig, zb_epochs, corr_autos, corr_parts, corr_dst;
  bool has_sigma = false, has_blocks = false;
  int64_t n_blocks = 0;
  // work buffers
  DevBuf coef, zbuf, out, sums, zin, xout, hostz, scratch_out, scratch_z, scratch_zb, scratch_sigma,
      scratch_block_of, scratch_esig, dbg_a, dbg_b;
  DevBuf fused_q;  // k_grid_fused's item queues: 8 per-XCD tickets + a done counter, zero between launches
  bool fused_q_ready = false;
  int32_t out_R = 0;
  int64_t out_ld = 0;
  // options
  int synth_path = 0;
  int mfma_min_real = 16;
  int profile = 0;
  int anchor = 0;  // 0: phasor recurrence anchored once per segment
  int valu_variant = 1;  // seeded (MT 2, NT 16): fastest on C2 (profiles/r01_sweep_*.txt)
  int fuse_white = 1;    // add white/ECORR in the seeded kernel's epilogue
  int fuse_sums = 0;     // gridded path: interpolation writes partial checksums (FPTA_OPT_FUSE_CHECKSUMS)
  int mix_mfma = 1;      // ORF mixing of large arrays on fp64 MFMA (k_mix_mfma) or VALU (k_mix_tiled)
  // batch coefficients on a side stream (FPTA_OPT_OVERLAP): gen / mix of signal i run there and signal i's
  // consumer on the ctx stream waits for ev_sig[i] only, so the gridded DFT of one signal overlaps the draws of
  // the next (VALU Philox beside fp64 MFMA). ev_begin orders the side stream after everything queued before.
  int overlap = 1;
  int interp_ws = 1;      // gridded interpolation on the warp-specialised kernel (FPTA_OPT_INTERP_WS)
  int last_interp = 0;    // interpolation kernel of the last gridded block: 1 + 4 kind + 2 white + part (0: none)
  int fused_white = 0;  // k_grid_fused_w for white / ECORR and three-grid-signal blocks (FPTA_OPT_FUSED_WHITE)
  double last_fma_interp = 0.0;  // its interpolation MFMA FMAs per realization as run (half-chunk bands: both halves)
  int grid_coalesce = 1;  // gridded path: signals sharing w0 and the chromatic weight share one grid (FPTA_OPT_GRID_COALESCE)
  int part_group = kPartGroup;  // fused partial checksums: consecutive chunks per partial row (FPTA_OPT_PART_GROUP)
  int interp_psr = 1;  // k_grid_interp_psr where the layout allows it (FPTA_OPT_INTERP_PSR)
  int interp_wr = 0;   // k_grid_interp_wr for plain blocks where the plan allows it (FPTA_OPT_INTERP_WR)
  int interp_fused = 1;  // k_grid_fused for plain blocks where the plan allows it (FPTA_OPT_INTERP_FUSED): 1 with
                         // half-chunk bands where they save >= 3 % of the interpolation MFMAs, 2 whole-chunk bands, 3
                         // half-chunk bands whenever planned
  // pipelined per-pulsar blocks read their coefficients in the interpolation (ctx stream): two coefficient buffers,
  // coef2 the other one; coef_slot = the grid-buffer index whose block owns c->coef; prev_psr: the last pipelined
  // block ran that way (its draws waited for the interpolation two blocks back, not for the whole ctx stream)
  DevBuf coef2;
  int coef_slot = 0;
  bool prev_psr = false;
  // FPTA_OPT_FUSED_NEXT_MIX: the last k_grid_fused launch also made the mix of common signal `seg` for the block
  // (layout, version, seed, real0, n_real, R_pad) into buffer `buf` (c->coef2 then, c->coef once that block swaps).
  // run_coefficients takes it when the next block has exactly that key; otherwise the side streams wait for that
  // kernel (event `done`) before they write a coefficient buffer.
  int fused_next_mix = 1;
  struct NextMix {
    bool valid = false;
    const Layout* layout = nullptr;
    uint64_t version = 0, seed = 0;
    int64_t real0 = 0;
    int32_t n_real = 0, R_pad = 0, seg = -1;
    const void* buf = nullptr;
    hipEvent_t done = nullptr;  // recorded on the ctx stream after that kernel (a miss makes the side streams wait for it)
  } next_mix;
  // the last batch block (seed, first realization, size): the next block's first realization is predicted at this
  // block's stride (simulate_sharded: the batch; bench.py on G ranks: G x R)
  struct LastBlock {
    bool valid = false;
    uint64_t seed = 0;
    int64_t real0 = 0;
    int32_t n_real = 0;
  } last_blk;
  bool next_mix_made = false, next_mix_used = false;  // fpta_batch_grid_info_n slots 17, 18 of the last block
  bool coef_queued = true;  // the last run_coefficients queued work (a pipelined block that queued none: no grid-ready wait)
  int async_sums = 0;    // streamed jobs: partial-checksum reductions on their own stream (FPTA_OPT_ASYNC_SUMS; measured
                         // no faster on C3, profiles/r03h_ab_c3_async_sums.txt: the reductions then compete with the interpolation)
  int gen_mix = 2;       // common signals of 64..256 pulsars: draws and ORF mixing in one kernel (k_gen_mix,
                         // FPTA_OPT_GEN_MIX; 2: 16-realization waves, C3 -3.7 % vs 1, profiles/r03z_gen_mix_waves.txt);
                         // 0 k_gen into zbuf, then k_mix_mfma
  int dft_gen = 1;       // gridded path: grid signals with a per-pulsar member draw their coefficients inside the DFT
                         // (k_grid_dft_gen, FPTA_OPT_DFT_GEN): no k_gen launch, no coefficient round trip for them
  bool gen_fused = false;  // the current block runs k_grid_dft_gen for those grid signals (set by batch_common)
  int64_t blk_real0 = 0;   // the current block's first realization and Philox key (k_grid_dft_gen draws)
  uint32_t blk_k0 = 0, blk_k1 = 0;
  int interp_lds = 0;    // gridded interpolation with the grid rows staged in LDS where the plan allows (measured
                         // slower on C2: 0.745 vs 0.67 ms, profiles/r02g_*; kept as an option)
  hipStream_t side = nullptr;
  hipEvent_t ev_begin = nullptr;
  std::vector<hipEvent_t> ev_sig;
  bool coef_side = false;  // the last coefficients were made on the side stream and are not all waited for
  // recorded on the ctx stream right after the last reader of the coefficient buffer was queued (the gridded
  // DFT, or the coefficient download): the next block's draws wait for it instead of for the whole previous
  // block, so they overlap that block's interpolation
  hipEvent_t ev_coef_free = nullptr;
  bool coef_free_set = false;
  // pipelined gridded batches (FPTA_OPT_OVERLAP, path 4): the draws, merges and DFT of a block all run on the side
  // stream, into one of two grid buffers, so they overlap the previous block's interpolation on the ctx stream.
  // ev_gready: the block's DFT is done (its interpolation waits); ev_gfree[i]: the interpolation reading grid
  // buffer i is done (the DFT that next writes buffer i waits); coef_last_side: the last reader of coef was a
  // side-stream DFT, so the next block's draws need no ctx-stream wait.
  hipEvent_t ev_gready = nullptr;
  hipEvent_t ev_gfree[2] = {nullptr, nullptr};
  bool gfree_set[2] = {false, false};
  int gbuf = 0;
  bool coef_last_side = false;
  // FPTA_OPT_SIDE_SPLIT: grid signal split_g (per-pulsar members only) of the current pipelined block runs its draws
  // and DFT on side2. At each block start side waits for side2's previous work (ev_s2done) and side2 for side's
  // (ev_s2begin), so a layout change never lets one stream write columns the other still reads; ev_gready2: side2's
  // DFT is done. side_split 2: side2's DFT also waits for the common signals' draws queued on side before it
  // (ev_s2mix), so those draws get the room beside the previous block's interpolation first.
  int side_split = 2;
  hipStream_t side2 = nullptr;
  hipEvent_t ev_s2begin = nullptr, ev_s2done = nullptr, ev_gready2 = nullptr, ev_s2mix = nullptr;
  bool s2done_set = false;
  int32_t split_g = -1;
  bool coef_copy_pending = false;  // the block's coefficients are still to be downloaded after the synthesis
  DevBuf part[2], part_tmp; // partial checksums [n_chunks][R_pad][2] (two buffers, by block), reduction scratch
  bool part_ready = false;  // part[part_cur] holds the partials of the current block (c->out, out_R)
  int32_t part_chunks = 0, part_rpad = 0;
  int part_cur = 0, part_next = 0;
  // streamed jobs reduce a block's partials on their own stream (red), beside the next block's interpolation, which
  // writes the other partials buffer; ev_pfree[i]: the reduction reading part[i] is done (the interpolation that next
  // writes part[i] waits for it); red_pending: red has work the ctx stream has not joined
  hipStream_t red = nullptr;
  hipEvent_t ev_pready = nullptr, ev_pfree[2] = {nullptr, nullptr}, ev_red = nullptr;
  bool pfree_set[2] = {false, false};
  bool red_pending = false;
  int last_path = 0;     // synthesis path of the last batch (1 direct, 2 MFMA, 3 VALU, 4 gridded)
  std::string path_reason;  // why the last batch did not take the gridded path (empty if it did)
  // gridded path defaults: w = 15 at sigma = 1.5 (a-priori bound 1.5e-12). The measured flat-spectrum worst case at
  // real-MJD epochs is <= ~6e-12 relative (tests/test_gpu_grid.py at the shipped defaults; the numpy model of
  // oracle.grid_synth and the GPU agree); w = 14 (bound 9.4e-12) is refused by the auto path. sigma = 1.5 keeps the
  // grid (DFT) a quarter smaller than sigma = 2 (tools/sweep_grid.py --params, profiles/r01_sweep_wsig.txt)
  int grid_w = 15;       // gridded path: kernel width in grid cells
  int grid_sigma100 = 150;  // gridded path: oversampling x 100
  int grid_mfma = 1;     // gridded path: bit 0 k_grid_dft_mfma (else k_grid_dft); the interpolation is always on
                         // MFMA (k_grid_interp_ws / k_grid_interp_mfma)
  // profiling
  struct Pending {
    int which;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
  int64_t kcount[FPTA_K_N] = {};
  double kms[FPTA_K_N] = {};
  // dense-covariance path: inputs, basis G^T [k_pad][n_pad], matrix C [n_pad][n_pad], panel, draws
  DevBuf dn_toas, dn_nu, dn_f, dn_sw, dn_segof, dn_segidx, dn_segff, dn_white, dn_GT, dn_C, dn_PT, dn_info, dn_r,
      dn_y, dn_out, dn_Z;
};

namespace __attribute__((visibility("hidden"))) capi {  // library-internal: not exported

int fail(fpta_ctx* c, int code, const std::string& msg);
int hip_fail(fpta_ctx* c, hipError_t e, const char* what);

// Debug build (make debug, -DFPTA_DEBUG): synchronize after every launch so a device fault is
// reported by the launch that caused it, and the kernels' FPTA_DCHECK bounds checks are compiled in.
// Release builds read no environment variable and never add work or synchronisation.
#ifdef FPTA_DEBUG
constexpr bool debug_sync() { return true; }
#else
constexpr bool debug_sync() { return false; }
#endif

#define HIPCHK(ctx, expr, what)                                                           \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e == hipSuccess && debug_sync() && std::strstr(what, "launch"))                  \
      _e = hipStreamSynchronize((ctx)->stream);                                           \
    if (_e != hipSuccess) return hip_fail(ctx, _e, what);                                 \
  } while (0)

hipEvent_t get_event(fpta_ctx* c);

// Bracket a launch with HIP events on the ctx stream when profiling is on.
struct KTimer {
  fpta_ctx* c;
  int which;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  // ext: the events are handed to the launch (hipExtLaunchKernel: the kernel's own dispatch timestamps, no marker
  // packets between the step's kernels); unused (the launch took another path) they go back to the pool untimed
  bool ext = false, bound = false;
  KTimer(fpta_ctx* c_, int w, hipStream_t s = nullptr, bool ext_ = false)
      : c(c_), which(w), st(s ? s : c_->stream), ext(ext_) {
    if (c->profile) {
      a = get_event(c);
      b = get_event(c);
      if (a && !ext) (void)hipEventRecord(a, st);
    }
  }
  // the launch's start / stop events (null with profiling off)
  hipEvent_t start_ev() {
    bound = ext && a && b;
    return bound ? a : nullptr;
  }
  hipEvent_t stop_ev() const { return bound ? b : nullptr; }
  // the launch's result: a launch that failed recorded neither event, so they go back to the pool untimed
  hipError_t checked(hipError_t e) {
    if (e != hipSuccess) bound = false;
    return e;
  }
  ~KTimer() {
    if (!c->profile || !a || !b) return;
    if (!ext) (void)hipEventRecord(b, st);
    if (!ext || bound) {
      c->pending.push_back({which, a, b});
    } else {
      c->pool.push_back(a);
      c->pool.push_back(b);
    }
  }
};

// capi.hip
int join_red(fpta_ctx* c);
int upload(fpta_ctx* c, DevBuf& buf, const void* src, size_t bytes, const char* what);
int wait_coef(fpta_ctx* c, size_t i);
int wait_coef_all(fpta_ctx* c);
bool grid_gen_fused(const fpta_ctx* c, const Layout& L, size_t g);
bool psr_layout(const fpta_ctx* c, const Layout& L);
bool fused_layout(const fpta_ctx* c, const Layout& L);
bool fused_w_layout(const fpta_ctx* c, const Layout& L);
int32_t next_mix_seg(const fpta_ctx* c, const Layout& L, int32_t R_pad);
int batch_common(fpta_ctx* c, uint64_t seed, int64_t real0, int32_t n_real, const double* zin, int32_t zin_nm,
                 double* out, double* coeffs_out, bool white);
int launch_block_checksums(fpta_ctx* c, bool async = false, hipStream_t* used = nullptr, double* dst = nullptr,
                           bool* direct = nullptr);

// grid_host.hip
constexpr double kGridAutoRatio = 0.5;  // auto path: gridded when it needs < half the direct FMAs
// auto path: gridded only when the a-priori bound exp(-pi w sqrt(1 - 1/sigma)) of the width/oversampling pair is
// within this. The measured flat-spectrum worst case is ~3-4x the bound (w = 16, sigma = 1.5: bound 2.5e-13,
// measured <= 3.6e-12; w = 15: 1.5e-12 / 6e-12; w = 14: 9.4e-12 / 3.2e-11, refused). A forced path 4 runs any
// accepted pair: the caller opted in, and fpta_batch_grid_info reports the bound.
constexpr double kGridAutoMaxErr = 2e-12;
int grid_build(fpta_ctx* c, Layout& L);
int grid_part_groups(fpta_ctx* c, GridPlan& G, int32_t P, int32_t size);
int grid_run(fpta_ctx* c, Layout& L, SynthArgs& a, int32_t R_pad, bool pipe = false);

}  // namespace capi
