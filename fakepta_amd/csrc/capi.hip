// C-ABI of libfakepta_amd.so (declared in include/fakepta_amd.h).
// Host-side orchestration only: argument checking, device buffers, layout tables,
// kernel dispatch on the context's stream, HIP-event timing. All arithmetic on the
// path runs in kernels.hip.
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

namespace {

thread_local std::string g_err;

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
  int32_t fused_fq = 0;  // band steps per (chunk, lane group) in frows
  std::vector<int32_t> fused_lrow0;
  DevBuf frows;
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
    fused_lrow0.clear();
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

}  // namespace

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
  int grid_coalesce = 1;  // gridded path: signals sharing w0 and the chromatic weight share one grid (FPTA_OPT_GRID_COALESCE)
  int part_group = kPartGroup;  // fused partial checksums: consecutive chunks per partial row (FPTA_OPT_PART_GROUP)
  int interp_psr = 1;  // k_grid_interp_psr where the layout allows it (FPTA_OPT_INTERP_PSR)
  int interp_wr = 0;   // k_grid_interp_wr for plain blocks where the plan allows it (FPTA_OPT_INTERP_WR)
  int interp_fused = 1;  // k_grid_fused for plain blocks where the plan allows it (FPTA_OPT_INTERP_FUSED)
  // pipelined per-pulsar blocks read their coefficients in the interpolation (ctx stream): two coefficient buffers,
  // coef2 the other one; coef_slot = the grid-buffer index whose block owns c->coef; prev_psr: the last pipelined
  // block ran that way (its draws waited for the interpolation two blocks back, not for the whole ctx stream)
  DevBuf coef2;
  int coef_slot = 0;
  bool prev_psr = false;
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

namespace {

int fail(fpta_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  g_err = msg;
  return code;
}

int hip_fail(fpta_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(c, e == hipErrorOutOfMemory ? FPTA_ENOMEM : FPTA_EDEVICE, m);
}

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

hipEvent_t get_event(fpta_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Bracket a launch with HIP events on the ctx stream when profiling is on.
struct KTimer {
  fpta_ctx* c;
  int which;
  hipStream_t st;
  hipEvent_t a = nullptr, b = nullptr;
  KTimer(fpta_ctx* c_, int w, hipStream_t s = nullptr) : c(c_), which(w), st(s ? s : c_->stream) {
    if (c->profile) {
      a = get_event(c);
      b = get_event(c);
      if (a) (void)hipEventRecord(a, st);
    }
  }
  ~KTimer() {
    if (c->profile && a && b) {
      (void)hipEventRecord(b, st);
      c->pending.push_back({which, a, b});
    }
  }
};

// The ctx stream waits for everything queued on the red stream (partial-checksum reductions of streamed jobs).
int join_red(fpta_ctx* c) {
  if (!c->red_pending) return FPTA_OK;
  if (!c->ev_red) HIPCHK(c, hipEventCreateWithFlags(&c->ev_red, hipEventDisableTiming), "event create");
  HIPCHK(c, hipEventRecord(c->ev_red, c->red), "event record");
  HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_red, 0), "red join");
  c->red_pending = false;
  return FPTA_OK;
}

int upload(fpta_ctx* c, DevBuf& buf, const void* src, size_t bytes, const char* what) {
  HIPCHK(c, buf.ensure(bytes), what);
  if (bytes) HIPCHK(c, hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, c->stream), what);
  return FPTA_OK;
}

int layout_set_toas(fpta_ctx* c, Layout& L, int32_t P, const int64_t* offs, const double* toas,
                    const double* nu) {
  if (P <= 0 || !offs || !toas || !nu) return fail(c, FPTA_EINVAL, "set_toas: bad arguments");
  if (offs[0] != 0) return fail(c, FPTA_EINVAL, "set_toas: offs[0] must be 0");
  int64_t mx = 0;
  for (int32_t p = 0; p < P; ++p) {
    const int64_t n = offs[p + 1] - offs[p];
    if (n <= 0) return fail(c, FPTA_EINVAL, "set_toas: every pulsar needs >= 1 TOA");
    if (n > (int64_t)1 << 30) return fail(c, FPTA_EINVAL, "set_toas: too many TOAs in one pulsar");
    mx = std::max(mx, n);
  }
  const int64_t N = offs[P];
  L.clear_signals();
  L.P = P;
  L.n_toa = N;
  L.max_np = mx;
  L.h_offs.assign(offs, offs + P + 1);
  L.h_toas.assign(toas, toas + N);
  L.h_nu.assign(nu, nu + N);
  std::vector<int32_t> psr_of(N);
  for (int32_t p = 0; p < P; ++p)
    for (int64_t t = offs[p]; t < offs[p + 1]; ++t) psr_of[t] = p;
  int rc;
  if ((rc = upload(c, L.offs, offs, sizeof(int64_t) * (P + 1), "set_toas offs"))) return rc;
  if ((rc = upload(c, L.toas, toas, sizeof(double) * N, "set_toas toas"))) return rc;
  if ((rc = upload(c, L.nu, nu, sizeof(double) * N, "set_toas nu"))) return rc;
  if ((rc = upload(c, L.psr_of, psr_of.data(), sizeof(int32_t) * N, "set_toas psr_of"))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream), "set_toas sync");
  return FPTA_OK;
}

// Harmonic test: w[k] == (k+1) w[0] to a few ulp (the f_k = k/T grids of fake_pta.py:264).
bool is_harmonic(const double* w, int32_t nm) {
  if (nm < 2 || !(w[0] > 0.0)) return false;
  for (int32_t k = 1; k < nm; ++k) {
    const double want = (k + 1) * w[0];
    if (std::fabs(w[k] - want) > 8.0 * 2.220446049250313e-16 * std::fabs(want)) return false;
  }
  return true;
}

int layout_add_signal(fpta_ctx* c, Layout& L, int32_t kind, int32_t nm, const double* f, const double* amp,
                      double idx, double freqf, const double* Lmat, const uint8_t* mask) {
  if (L.P <= 0) return fail(c, FPTA_ESTATE, "add_signal: set_toas first");
  if ((kind != 0 && kind != 1) || nm <= 0 || !f || !amp)
    return fail(c, FPTA_EINVAL, "add_signal: bad kind / n_modes / arrays");
  if (kind == 1 && !Lmat) return fail(c, FPTA_EINVAL, "add_signal: common signal needs an ORF factor");
  if (L.segs.size() >= 4096) return fail(c, FPTA_EINVAL, "add_signal: too many signals");
  const int32_t P = L.P;
  const int32_t nmp = nm + (nm & 1);
  const int32_t rows = kind == 0 ? P : 1;
  std::vector<double> w((size_t)rows * nmp), a((size_t)rows * nmp, 0.0);
  bool harm = true;
  for (int32_t r = 0; r < rows; ++r) {
    for (int32_t k = 0; k < nm; ++k) {
      // 2*pi*f in the reference's operation order: (2*np.pi) * f  (fake_pta.py:386)
      w[(size_t)r * nmp + k] = (2.0 * M_PI) * f[(size_t)r * nm + k];
      a[(size_t)r * nmp + k] = amp[(size_t)r * nm + k];
      if (!std::isfinite(w[(size_t)r * nmp + k]) || !std::isfinite(a[(size_t)r * nmp + k]))
        return fail(c, FPTA_EINVAL, "add_signal: non-finite frequency or amplitude");
    }
    if (nmp != nm) {  // padding mode: amplitude 0, frequency continues the grid
      const double w0 = w[(size_t)r * nmp];
      w[(size_t)r * nmp + nm] = w[(size_t)r * nmp + nm - 1] + w0;
    }
    harm = harm && is_harmonic(&w[(size_t)r * nmp], nmp);
  }
  Seg* s = new Seg();
  s->nm_orig = nm;
  for (int32_t r = 0; r < rows; ++r) s->h_w0.push_back(w[(size_t)r * nmp]);
  if (mask) s->h_mask.assign(mask, mask + L.n_toa);
  int rc;
  if ((rc = upload(c, s->w, w.data(), sizeof(double) * w.size(), "add_signal w")) ||
      (rc = upload(c, s->amp, a.data(), sizeof(double) * a.size(), "add_signal amp"))) {
    delete s;
    return rc;
  }
  if (kind == 1 && (rc = upload(c, s->L, Lmat, sizeof(double) * (size_t)P * P, "add_signal L"))) {
    delete s;
    return rc;
  }
  // L^T zero-padded to whole 64-pulsar tiles (columns) plus one 16-row block of k-steps: every k_mix_mfma
  // operand load is a 16-byte pair inside the buffer, and pad rows / columns weigh 0
  int32_t lt_ld = 0, lt_rows = 0;
  if (kind == 1) {
    lt_ld = (P + 63) / 64 * 64;
    lt_rows = lt_ld + 16;
    std::vector<double> lt((size_t)lt_rows * lt_ld, 0.0);
    for (int32_t p = 0; p < P; ++p)
      for (int32_t q = 0; q < P; ++q) lt[(size_t)q * lt_ld + p] = Lmat[(size_t)p * P + q];
    if ((rc = upload(c, s->LT, lt.data(), sizeof(double) * lt.size(), "add_signal L^T"))) {
      delete s;
      return rc;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream), "add_signal L^T sync");  // lt goes out of scope
  }
  if (mask && (rc = upload(c, s->mask, mask, (size_t)L.n_toa, "add_signal mask"))) {
    delete s;
    return rc;
  }
  SegDesc& d = s->d;
  d.w = s->w.as<double>();
  d.amp = s->amp.as<double>();
  d.L = kind == 1 ? s->L.as<double>() : nullptr;
  d.LT = kind == 1 ? s->LT.as<double>() : nullptr;
  d.lt_ld = lt_ld;
  d.lt_rows = lt_rows;
  d.mask = mask ? s->mask.as<uint8_t>() : nullptr;
  d.w_pstride = kind == 0 ? nmp : 0;
  d.idx = idx;
  d.freqf = freqf;
  d.nm = nmp;
  d.kind = kind;
  d.col0 = L.K;
  d.harmonic = harm ? 1 : 0;
  d.l_lower = 0;
  if (kind == 1) {  // a Cholesky factor (exact zeros above the diagonal) allows triangular mixing
    bool low = true;
    for (int32_t p = 0; p < P && low; ++p)
      for (int32_t q = p + 1; q < P; ++q)
        if (Lmat[(size_t)p * P + q] != 0.0) {
          low = false;
          break;
        }
    d.l_lower = low ? 1 : 0;
    // trailing all-zero columns of L (exact zeros): skipping them changes no sum
    int32_t nq = 0;
    for (int32_t p = 0; p < P; ++p)
      for (int32_t q = P - 1; q >= nq; --q)
        if (Lmat[(size_t)p * P + q] != 0.0) {
          nq = q + 1;
          break;
        }
    d.n_q = std::max(nq, 1);
  }
  L.K += 2 * nmp;
  L.segs.push_back(s);
  L.dirty = true;
  HIPCHK(c, hipStreamSynchronize(c->stream), "add_signal sync");  // host vectors go out of scope
  return (int)(L.segs.size() - 1);
}

int layout_finalize(fpta_ctx* c, Layout& L) {
  if (!L.dirty) return FPTA_OK;
  L.grid.clear();
  std::vector<SegDesc> d;
  bool harm = !L.segs.empty();
  for (Seg* s : L.segs) {
    d.push_back(s->d);
    harm = harm && s->d.harmonic;
  }
  int rc = upload(c, L.segdesc, d.data(), sizeof(SegDesc) * d.size(), "segdesc");
  if (rc) return rc;
  L.all_harmonic = harm;
  if (harm) {
    HIPCHK(c, L.seeds.ensure(sizeof(double4) * (size_t)L.n_toa * d.size()), "seeds alloc");
    HIPCHK(c,
           launch_seeds(c->stream, L.segdesc.as<SegDesc>(), (int32_t)d.size(), L.psr_of.as<int32_t>(),
                        L.toas.as<double>(), L.nu.as<double>(), L.n_toa, L.seeds.as<double4>()),
           "k_seeds launch");
  }
  HIPCHK(c, hipStreamSynchronize(c->stream), "segdesc sync");
  L.dirty = false;
  return FPTA_OK;
}

int32_t pad_to(int32_t x, int32_t m) { return (x + m - 1) / m * m; }

// Draw + mix every segment into c->coef [P][K][R_pad].
// The ctx stream waits for signal i's coefficients (side-stream draws), or for all of them.
int wait_coef(fpta_ctx* c, size_t i) {
  if (c->coef_side && i < c->ev_sig.size()) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_sig[i], 0), "coef wait");
  return FPTA_OK;
}
int wait_coef_all(fpta_ctx* c) {
  if (!c->coef_side) return FPTA_OK;
  for (size_t i = 0; i < c->ev_sig.size(); ++i) {
    int rc = wait_coef(c, i);
    if (rc) return rc;
  }
  c->coef_side = false;
  return FPTA_OK;
}

// Grid signal g of L draws inside its DFT (k_grid_dft_gen) in a gen_fused block: it has a per-pulsar member, at most
// kDftGenTerms members and a coefficient tile that fits the kernel's LDS.
bool grid_gen_fused(const fpta_ctx* c, const Layout& L, size_t g) {
  if (!c->gen_fused || !L.grid.built || !L.grid.ok || g >= L.grid.members.size()) return false;
  const std::vector<int32_t>& m = L.grid.members[g];
  if (m.size() > (size_t)kDftGenTerms || 2 * L.grid.segs[g]->ntq > 512) return false;
  for (int32_t i : m)
    if (L.segs[i]->d.kind == 0) return true;
  return false;
}

// The gridded plan of L runs on k_grid_interp_psr (FPTA_OPT_INTERP_PSR): one grid signal whose coefficients come
// from the coefficient buffer through the MFMA DFT (the kernel reproduces k_grid_dft_mfma), one 32-row DFT block
// (nf <= 124), bands of <= 32 rows, and no diagnostic interpolation kernel chosen.
bool psr_layout(const fpta_ctx* c, const Layout& L) {
  const GridPlan& G = L.grid;
  if (!c->interp_psr || !G.built || !G.ok || G.segs.size() != 1 || grid_gen_fused(c, L, 0) || !(c->grid_mfma & 1) ||
      c->interp_lds || c->interp_ws >= 4)
    return false;
  const GridSeg* gs = G.segs[0];
  return gs->nf <= 124 && gs->nf % 4 == 0 && gs->ldq == kGridDftRows && G.vmax <= 32 && gs->rowoff == 0;
}

// The gridded plan of L runs on k_grid_fused (FPTA_OPT_INTERP_FUSED): its grids and coefficient staging for
// kFusedReal realizations fit in LDS (GridPlan::fused_ok), no per-pulsar (psr) or diagnostic kernel chosen. Blocks
// with white noise, fused checksums or accumulation take the other kernels (grid_run).
bool fused_layout(const fpta_ctx* c, const Layout& L) {
  const GridPlan& G = L.grid;
  return c->interp_fused && G.built && G.ok && G.fused_ok && (c->grid_mfma & 1) && !c->interp_lds &&
         c->interp_ws < 4 && !c->interp_wr && !psr_layout(c, L);
}

// The interpolation kernel reads the block's coefficients (pipelined blocks alternate two coefficient buffers)
bool coef_in_interp(const fpta_ctx* c, const Layout& L) { return psr_layout(c, L) || fused_layout(c, L); }

// merge: the gridded plan of L coalesces signals (GridPlan::members): after the last member of a grid signal is
// drawn, k_coef_merge adds the other members' columns into the anchor's. coef_host (optional, with merge): the
// per-signal coefficients [P][K][R] are downloaded before any merge and *coef_done is set.
// pipe: a pipelined gridded block (side stream even for one signal; grid_run runs its DFT there too).
int run_coefficients(fpta_ctx* c, Layout& L, uint64_t seed, int64_t real0, int32_t R, int32_t R_pad,
                     const double* zin, int32_t zin_nm, double* x_out, bool side = false, bool merge = false,
                     double* coef_host = nullptr, bool* coef_done = nullptr, bool pipe = false) {
  const int32_t P = L.P;
  int rc0 = wait_coef_all(c);  // a previous block's draws are fully ordered before this one's
  if (rc0) return rc0;
  hipStream_t st = c->stream;
  const bool use_side = side && (L.segs.size() > 1 || pipe);
  const bool last_side = c->coef_last_side;
  c->coef_last_side = false;
  if (!use_side) c->coef_free_set = false;  // coef is written on the ctx stream from here on
  // a pipelined per-pulsar block draws into the coefficient buffer of its grid-buffer index (the interpolation of the
  // previous block may still read the other one)
  const bool psr = pipe && use_side && !zin && !x_out && !coef_host && coef_in_interp(c, L);
  if (psr && c->coef_slot != c->gbuf) {
    c->coef.swap(c->coef2);
    c->coef_slot = c->gbuf;
  }
  const size_t coef_bytes = sizeof(double) * (size_t)P * std::max(L.K, 1) * R_pad;
  if (c->side && c->coef.cap < coef_bytes) HIPCHK(c, hipStreamSynchronize(c->side), "side sync");  // before a regrow
  if (c->side2 && c->coef.cap < coef_bytes) HIPCHK(c, hipStreamSynchronize(c->side2), "side sync");
  if (use_side) {
    if (!c->side) HIPCHK(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking), "side stream create");
    if (!c->ev_begin) HIPCHK(c, hipEventCreateWithFlags(&c->ev_begin, hipEventDisableTiming), "event create");
    while (c->ev_sig.size() < L.segs.size()) {
      hipEvent_t e = nullptr;
      HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), "event create");
      c->ev_sig.push_back(e);
    }
    // the previous block's last reader of coef (its DFT or download) comes first; without one recorded,
    // everything queued on the ctx stream. A pipelined block whose DFT (on this stream) was that reader needs no
    // wait, unless the draws read a ctx-stream upload (zin)
    // (a per-pulsar block after another: its buffer's last reader was the interpolation two blocks back)
    if (!(pipe && last_side && !c->coef_free_set && !zin) && !(psr && c->prev_psr)) {
      if (!c->coef_free_set) HIPCHK(c, hipEventRecord(c->ev_begin, c->stream), "event record");
      HIPCHK(c, hipStreamWaitEvent(c->side, c->coef_free_set ? c->ev_coef_free : c->ev_begin, 0), "side wait");
    }
    if (psr && c->gfree_set[c->gbuf])
      HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_gfree[c->gbuf], 0), "coefficient buffer wait");
    c->coef_free_set = false;
    // the previous split block's second side stream (its draws and DFT) comes first as well
    if (c->s2done_set) HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_gready2, 0), "side wait");
    c->s2done_set = false;
    st = c->side;
  }
  HIPCHK(c, c->coef.ensure(coef_bytes), "coef alloc");
  size_t zb = 0;
  for (Seg* s : L.segs)
    if (s->d.kind == 1) zb = std::max(zb, sizeof(double) * (size_t)P * 2 * s->d.nm * R_pad);
  if (zb) HIPCHK(c, c->zbuf.ensure(zb), "zbuf alloc");
  const uint32_t k0 = (uint32_t)(seed & 0xFFFFFFFFull), k1 = (uint32_t)(seed >> 32);
  const GridPlan& G = L.grid;
  merge = merge && G.built && G.ok && G.merges;
  // the download of per-signal coefficients must precede every merge: then all events wait for the end
  const bool defer = merge && coef_host;
  // A common (kind-1) member of a coalesced grid signal adds into the anchor's columns inside its own k_mix_mfma
  // (no k_coef_merge pass over it) when the anchor is drawn before it and every member before it (index order,
  // anchor excluded) does the same: the sums then run in k_coef_merge's order, bit for bit. Not when the
  // per-signal coefficients are downloaded (they are taken before any merge) or mixed draws are returned.
  const bool mfma_mix = P >= kMixTiledMinP && R_pad % 128 == 0 && c->mix_mfma;
  // members of grid signals that draw inside their DFT (k_grid_dft_gen): per-pulsar members are not drawn here, and
  // the common members' mixed coefficients stay in their own columns (the DFT adds them in the merge order)
  std::vector<char> in_fused(L.segs.size(), 0), fused_g(G.members.size(), 0);
  for (size_t g = 0; g < G.members.size(); ++g)
    if (grid_gen_fused(c, L, g)) {
      fused_g[g] = 1;
      for (int32_t i : G.members[g]) in_fused[i] = 1;
    }
  std::vector<int32_t> fuse_into(L.segs.size(), -1);
  if (merge && !defer && mfma_mix && !x_out)
    for (size_t g = 0; g < G.members.size(); ++g) {
      if (fused_g[g]) continue;
      bool prefix = true;
      for (int32_t i : G.members[g]) {
        if (i == G.anchor[g]) continue;
        prefix = prefix && L.segs[i]->d.kind == 1 && G.anchor[g] < i;
        if (prefix) fuse_into[i] = L.segs[G.anchor[g]]->d.col0;
      }
    }
  // FPTA_OPT_SIDE_SPLIT: in a pipelined block, the grid signal with the largest DFT (half range x modes) whose
  // members are all per-pulsar signals (no zbuf, no mixing) is drawn, merged and transformed on side2, beside the
  // other signals' chain on side. Both streams start after everything before the block on side.
  c->split_g = -1;
  std::vector<int32_t> group_of(L.segs.size(), -1);
  for (size_t g = 0; g < G.members.size(); ++g)
    for (int32_t i : G.members[g]) group_of[i] = (int32_t)g;
  if (pipe && use_side && c->side_split && G.built && G.ok && G.members.size() > 1 && !zin && !x_out && !coef_host &&
      !psr) {
    int64_t best = -1;
    for (size_t g = 0; g < G.members.size(); ++g) {
      bool per_pulsar = true;
      for (int32_t i : G.members[g]) per_pulsar = per_pulsar && L.segs[i]->d.kind == 0;
      const int64_t cost = (int64_t)G.segs[g]->half * L.segs[G.anchor[g]]->d.nm;
      if (per_pulsar && cost > best) {
        best = cost;
        c->split_g = (int32_t)g;
      }
    }
  }
  if (c->split_g >= 0) {
    if (!c->side2) {  // at the highest priority: its chain (the largest DFT) is the longer one (profiles/r02n_*)
      int lo = 0, hi = 0;
      HIPCHK(c, hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priority range");
      HIPCHK(c, hipStreamCreateWithPriority(&c->side2, hipStreamNonBlocking, hi), "side stream create");
    }
    for (hipEvent_t* e : {&c->ev_s2begin, &c->ev_gready2})
      if (!*e) HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming), "event create");
    HIPCHK(c, hipEventRecord(c->ev_s2begin, c->side), "event record");
    HIPCHK(c, hipStreamWaitEvent(c->side2, c->ev_s2begin, 0), "side wait");
  }
  auto stream_of = [&](int32_t g) { return g >= 0 && g == c->split_g ? c->side2 : st; };
  auto merge_group = [&](size_t g) -> int {
    CoefMerge m{};
    m.dst = L.segs[G.anchor[g]]->d.col0;
    for (int32_t i : G.members[g])
      if (i != G.anchor[g] && fuse_into[i] < 0) {
        if (m.n >= kGridMaxSeg) return fail(c, FPTA_EINVAL, "coef merge: more than kGridMaxSeg members");
        m.src[m.n] = L.segs[i]->d.col0;
        m.ncol[m.n++] = 2 * L.segs[i]->d.nm;
      }
    if (m.n == 0) return FPTA_OK;  // every member was added inside its mix
    hipStream_t sg = stream_of((int32_t)g);
    KTimer kt(c, FPTA_K_GEN, sg);
    HIPCHK(c, launch_coef_merge(sg, m, P, L.K, R_pad, c->coef.as<double>()), "k_coef_merge launch");
    return FPTA_OK;
  };
  for (size_t i = 0; i < L.segs.size(); ++i) {
    const SegDesc& d = L.segs[i]->d;
    hipStream_t si = stream_of(group_of[i]);  // side2 only for members of split_g (kind 0: no mixing below)
    if (in_fused[i] && d.kind == 0) continue;  // drawn inside its grid signal's DFT
    if (d.kind == 1 && c->gen_mix && mfma_mix && !zin && !x_out && fuse_into[i] < 0 && P <= kGenMixMaxP) {
      KTimer kt(c, FPTA_K_MIX, st);  // draws + mixing in one kernel, into the signal's own columns
      // 16-realization workgroups (FPTA_OPT_GEN_MIX 3: they fit in the LDS two k_grid_interp_psr workgroups leave;
      // C3 measured the same either way, profiles/round4/R5d)
      const int rb = c->gen_mix == 3 ? 16 : 32;
      HIPCHK(c, launch_gen_mix(st, d, (int32_t)i, P, R, R_pad, real0, k0, k1, c->coef.as<double>(), L.K,
                               c->gen_mix == 1 ? 2 : 1, rb),
             "k_gen_mix launch");
    } else {
    {
      KTimer kt(c, FPTA_K_GEN, si);
      HIPCHK(c,
             launch_gen(si, d, (int32_t)i, P, R, R_pad, real0, k0, k1, zin, (int32_t)L.segs.size(), zin_nm,
                        c->coef.as<double>(), L.K, c->zbuf.as<double>()),
             "k_gen launch");
    }
    if (d.kind == 1) {
      KTimer kt(c, FPTA_K_MIX, st);
      if (mfma_mix)
        HIPCHK(c,
               launch_mix_mfma(st, d, P, R_pad, c->zbuf.as<double>(), c->coef.as<double>(), L.K, x_out, fuse_into[i]),
               "k_mix_mfma launch");
      else if (P >= kMixTiledMinP && R_pad % 128 == 0)
        HIPCHK(c, launch_mix_tiled(st, d, P, R_pad, c->zbuf.as<double>(), c->coef.as<double>(), L.K, x_out),
               "k_mix_tiled launch");
      else
        HIPCHK(c, launch_mix(st, d, P, R_pad, c->zbuf.as<double>(), c->coef.as<double>(), L.K, x_out),
               "k_mix launch");
    }
    }
    if (merge && !defer)
      for (size_t g = 0; g < G.members.size(); ++g)
        if (!fused_g[g] && G.members[g].size() > 1 && G.last[g] == (int32_t)i) {
          int rc = merge_group(g);
          if (rc) return rc;
        }
    if (st != c->stream && !defer && !pipe) HIPCHK(c, hipEventRecord(c->ev_sig[i], st), "event record");
  }
  if (defer) {
    HIPCHK(c,
           hipMemcpy2DAsync(coef_host, sizeof(double) * R, c->coef.p, sizeof(double) * R_pad, sizeof(double) * R,
                            (size_t)P * L.K, hipMemcpyDeviceToHost, st),
           "coef download");
    if (coef_done) *coef_done = true;
    for (size_t g = 0; g < G.members.size(); ++g)
      if (!fused_g[g] && G.members[g].size() > 1) {
        int rc = merge_group(g);
        if (rc) return rc;
      }
    if (st != c->stream && !pipe)
      for (size_t i = 0; i < L.segs.size(); ++i) HIPCHK(c, hipEventRecord(c->ev_sig[i], st), "event record");
  }
  c->coef_side = st != c->stream && !pipe;  // pipelined: the DFT follows on the same stream, no per-signal events
  c->prev_psr = psr;
  return FPTA_OK;
}

// Tile table of (pulsar, first TOA, first realization) for a kernel whose workgroup covers tile_toa TOAs x
// tile_real realizations. The cache is keyed on the whole geometry: a table built for one kernel must never
// drive another (with a key of n_real alone, the tile table of k_synth_mfma drove
// k_synth_valu<1,32>, whose 128-realization workgroups then read coefficients past the padded block).
int build_tiles(fpta_ctx* c, Layout& L, int32_t R, int32_t tile_toa, int32_t tile_real) {
  if (L.tiles_n_real == R && L.tiles_toa == tile_toa && L.tiles_real == tile_real) return FPTA_OK;
  L.tiles_n_real = -1;
  std::vector<int4> t;
  for (int32_t p = 0; p < L.P; ++p) {
    const int64_t np_ = L.h_offs[p + 1] - L.h_offs[p];
    for (int32_t r0 = 0; r0 < R; r0 += tile_real)
      for (int64_t t0 = 0; t0 < np_; t0 += tile_toa) t.push_back(make_int4(p, (int)t0, r0, 0));
  }
  // XCD-aware order: workgroups b, b+8, b+16, ... share an XCD's L2 (round-robin dispatch), so give
  // them consecutive tiles (same pulsar and realization tile -> same coefficient block).
  const size_t n = t.size();
  const size_t per = (n + 7) / 8;
  std::vector<int4> o(per * 8, make_int4(-1, 0, 0, 0));
  for (size_t b = 0; b < o.size(); ++b) {
    const size_t tile = (b % 8) * per + b / 8;
    if (tile < n) o[b] = t[tile];
  }
  int rc = upload(c, L.tiles, o.data(), sizeof(int4) * o.size(), "tiles");
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream), "tiles sync");
  L.n_tiles = (int32_t)o.size();
  L.tiles_toa = tile_toa;
  L.tiles_real = tile_real;
  L.tiles_n_real = R;
  return FPTA_OK;
}

// The tile table in the cache was built for exactly this kernel geometry (checked before every tiled launch).
int check_tiles(fpta_ctx* c, const Layout& L, int32_t R, int32_t tile_toa, int32_t tile_real, SynthArgs& a) {
  if (L.tiles_n_real != R || L.tiles_toa != tile_toa || L.tiles_real != tile_real)
    return fail(c, FPTA_ESTATE, "synth: tile table does not match the kernel's tile geometry");
  a.tile_toa = tile_toa;
  a.tile_real = tile_real;
  return FPTA_OK;
}


// ------------------------------------------------------------------------------- gridded plan
// Gauss-Legendre nodes/weights on [-1, 1] (Newton on P_n; host, once per plan).
void gauss_legendre(int n, std::vector<double>& x, std::vector<double>& wt) {
  x.assign(n, 0.0);
  wt.assign(n, 0.0);
  for (int i = 0; i < (n + 1) / 2; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5)), dp = 1.0;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = z;
      for (int k = 2; k <= n; ++k) {
        const double p2 = ((2.0 * k - 1.0) * z * p1 - (k - 1.0) * p0) / k;
        p0 = p1;
        p1 = p2;
      }
      dp = n * (z * p1 - p0) / (z * z - 1.0);
      const double dz = p1 / dp;
      z -= dz;
      if (std::fabs(dz) < 1e-16) break;
    }
    x[i] = -z;
    x[n - 1 - i] = z;
    wt[i] = wt[n - 1 - i] = 2.0 / ((1.0 - z * z) * dp * dp);
  }
}

// Build the gridded plan (grid.hip) of layout L: per signal the grid size nf, the deconvolved real-DFT
// table, the chunking of every pulsar's TOAs into runs of <= kGridTT whose interpolation rows span at
// most kGridRowCap cells, and the dense banded weights (device). Not usable -> ok = false + why.
constexpr int kGridRowCap = 48;
constexpr double kGridAutoRatio = 0.5;  // auto path: gridded when it needs < half the direct FMAs
// auto path: gridded only when the a-priori bound exp(-pi w sqrt(1 - 1/sigma)) of the width/oversampling pair is
// within this. The measured flat-spectrum worst case is ~3-4x the bound (w = 16, sigma = 1.5: bound 2.5e-13,
// measured <= 3.6e-12; w = 15: 1.5e-12 / 6e-12; w = 14: 9.4e-12 / 3.2e-11, refused). A forced path 4 runs any
// accepted pair: the caller opted in, and fpta_batch_grid_info reports the bound.
constexpr double kGridAutoMaxErr = 2e-12;
int grid_build(fpta_ctx* c, Layout& L) {
  GridPlan& G = L.grid;
  if (G.built && G.w == c->grid_w && G.sigma == c->grid_sigma100 / 100.0) return FPTA_OK;
  G.clear();
  G.built = true;
  G.w = c->grid_w;
  G.sigma = c->grid_sigma100 / 100.0;
  G.err_bound = std::exp(-M_PI * G.w * std::sqrt(1.0 - 1.0 / G.sigma));
  if (L.segs.empty()) {
    G.why = "gridded path: no signals";
    return FPTA_OK;
  }
  for (Seg* sg : L.segs)
    if (!sg->d.harmonic) {
      G.why = "gridded path: every signal needs a harmonic grid f_k = k f_1";
      return FPTA_OK;
    }
  // grid signals: with FPTA_OPT_GRID_COALESCE, a signal joins the first earlier grid signal with the same base
  // frequency w0 on every pulsar and the same chromatic weight (factor x mask) on every TOA. Their sums
  // ch(t) sum_k c_k cos(k w0 t) + s_k sin(k w0 t) then add in coefficient space (k_coef_merge): one DFT, one band.
  {
    const int32_t n_layout = (int32_t)L.segs.size();
    std::vector<std::vector<double>> chv(n_layout);
    auto ch_of = [&](int32_t i) -> const std::vector<double>& {
      if (chv[i].empty()) {
        const SegDesc& d = L.segs[i]->d;
        const std::vector<uint8_t>& m = L.segs[i]->h_mask;
        chv[i].resize(L.n_toa);
        for (int64_t t = 0; t < L.n_toa; ++t) {
          double ch = 1.0;  // chrom_factor (device_common.h), same operations
          if (d.idx != 0.0) {
            const double x = d.freqf / L.h_nu[t];
            ch = d.idx == 2.0 ? x * x : d.idx == 1.0 ? x : std::pow(x, d.idx);
          }
          chv[i][t] = (!m.empty() && !m[t]) ? 0.0 : ch;
        }
      }
      return chv[i];
    };
    auto w0_of = [&](int32_t i, int32_t p) { return L.segs[i]->h_w0[L.segs[i]->d.kind == 0 ? p : 0]; };
    for (int32_t i = 0; i < n_layout; ++i) {
      int32_t join = -1;
      for (size_t g = 0; c->grid_coalesce && g < G.members.size() && join < 0; ++g) {
        // a grid signal merges at most kGridMaxSeg other members (CoefMerge::src): a full group starts a new one
        if (G.members[g].size() > (size_t)kGridMaxSeg) continue;
        const int32_t f = G.members[g][0];
        bool same = true;
        for (int32_t p = 0; p < L.P && same; ++p) same = w0_of(i, p) == w0_of(f, p);
        if (same) same = ch_of(i) == ch_of(f);
        if (same) join = (int32_t)g;
      }
      if (join < 0) {
        G.members.push_back({i});
      } else {
        G.members[join].push_back(i);
        G.merges = true;
      }
    }
    for (const std::vector<int32_t>& m : G.members) {
      int32_t a = m[0];
      for (int32_t i : m)
        if (L.segs[i]->d.nm > L.segs[a]->d.nm) a = i;
      G.anchor.push_back(a);
      G.last.push_back(m.back());
    }
  }
  const int32_t n_seg = (int32_t)G.members.size();  // grid signals from here on
  if (n_seg > kGridMaxSeg) {
    G.why = "gridded path: needs 1.." + std::to_string(kGridMaxSeg) + " grid signals (after coalescing)";
    return FPTA_OK;
  }
  const int64_t N = L.n_toa;
  // per (segment, TOA): first interpolation row J (unwrapped) and offset d = u - J, u = theta / h
  std::vector<std::vector<int64_t>> J(n_seg, std::vector<int64_t>(N));
  std::vector<std::vector<double>> D(n_seg, std::vector<double>(N));
  std::vector<int32_t> nf(n_seg), ws(n_seg);
  std::vector<double> betas(n_seg);
  // Per grid signal: the options' (w, sigma) give nf0 = sigma (2 N + 1) grid points, a multiple of 4 (the MFMA DFT
  // runs on the quarter range); it computes whole blocks of kGridDftRows rows of the quarter range, so nf1 = 4 (rows
  // of those blocks - 1) points cost it nothing more. The larger effective oversampling sigma1 = nf1 / (2 N + 1)
  // reaches the options' a-priori bound with a narrower kernel w1; the signal takes (nf1, w1) when its interpolation
  // band (w + the cells a 32-TOA chunk spans) is estimated narrower.
  const double bound_target = G.err_bound;
  G.err_bound = 0.0;
  for (int32_t s = 0; s < n_seg; ++s) {
    const Seg* sg = L.segs[G.anchor[s]];
    const SegDesc& d = sg->d;
    int32_t n = (int32_t)std::ceil(G.sigma * (2.0 * d.nm + 1.0));
    int32_t n0 = (std::max(n, 2 * G.w + 2) + 3) / 4 * 4, w0 = G.w;
    // grid cells per TOA per grid point: mean over pulsars of w0 dt / (2 pi), dt the mean TOA spacing
    double rho = 0.0;
    for (int32_t p = 0; p < L.P; ++p) {
      const int64_t a0 = L.h_offs[p], a1 = L.h_offs[p + 1];
      double tmin = L.h_toas[a0], tmax = L.h_toas[a0];
      for (int64_t t = a0; t < a1; ++t) {
        tmin = std::min(tmin, L.h_toas[t]);
        tmax = std::max(tmax, L.h_toas[t]);
      }
      if (a1 - a0 > 1) rho += sg->h_w0[d.kind == 0 ? p : 0] * (tmax - tmin) / (double)(a1 - a0 - 1) / (2.0 * M_PI);
    }
    rho /= L.P;
    const int32_t blocks = (n0 / 4 + kGridDftRows) / kGridDftRows;  // ceil((nf / 4 + 1) / rows per block)
    const int32_t n1 = 4 * (blocks * kGridDftRows - 1);
    const double sig1 = n1 / (2.0 * d.nm + 1.0);
    int32_t w1 = G.w;
    while (w1 > 4 && std::exp(-M_PI * (w1 - 1) * std::sqrt(1.0 - 1.0 / sig1)) <= bound_target) --w1;
    const bool fill = n1 > n0 && 2 * w1 + 2 <= n1 && w1 + kGridTT * n1 * rho < w0 + kGridTT * n0 * rho - 0.25;
    nf[s] = fill ? n1 : n0;
    ws[s] = fill ? w1 : w0;
    const double sig = nf[s] / (2.0 * d.nm + 1.0);
    // shape parameter of the exponential-of-semicircle kernel for oversampling sigma (2.31 w at sigma = 2)
    betas[s] = 0.98 * M_PI * ws[s] * (1.0 - 0.5 / sig);
    G.err_bound = std::max(G.err_bound, std::exp(-M_PI * ws[s] * std::sqrt(1.0 - 1.0 / sig)));
    const double hw = 0.5 * ws[s];
    const double h = 2.0 * M_PI / nf[s];
    for (int32_t p = 0; p < L.P; ++p) {
      const double w0 = sg->h_w0[d.kind == 0 ? p : 0];
      for (int64_t t = L.h_offs[p]; t < L.h_offs[p + 1]; ++t) {
        const double u = (w0 * L.h_toas[t]) / h;
        if (!std::isfinite(u) || std::fabs(u) > 1e15) {
          G.why = "gridded path: phase out of range";
          return FPTA_OK;
        }
        const int64_t j = (int64_t)std::floor(u - hw) + 1;
        J[s][t] = j;
        D[s][t] = u - (double)j;
      }
    }
  }
  // chunks: <= kGridTT consecutive TOAs of one pulsar, every signal's band <= kGridRowCap rows
  std::vector<int4> chunks;
  std::vector<int32_t> chunk_of(N), tt_of(N);
  std::vector<std::vector<int64_t>> band_lo(n_seg);  // per chunk: first grid row (unwrapped) of each signal
  std::vector<std::vector<int32_t>> band_n(n_seg);   // per chunk: band rows of each signal (span + w)
  std::vector<int64_t> lo(n_seg), hi(n_seg);
  for (int32_t p = 0; p < L.P; ++p) {
    int64_t t = L.h_offs[p];
    const int64_t t_end = L.h_offs[p + 1];
    while (t < t_end) {
      const int64_t t0 = t;
      for (int32_t s = 0; s < n_seg; ++s) lo[s] = hi[s] = J[s][t];
      ++t;
      // chunks end on multiples of kGridTT in the global TOA index: every full chunk then writes whole
      // 256-byte runs of each realization row
      const int64_t t_lim = std::min(t_end, (t0 / kGridTT + 1) * kGridTT);
      while (t < t_lim) {
        bool fits = true;
        for (int32_t s = 0; s < n_seg && fits; ++s)
          fits = std::max(hi[s], J[s][t]) - std::min(lo[s], J[s][t]) + ws[s] + 1 <= kGridRowCap;
        if (!fits) break;
        for (int32_t s = 0; s < n_seg; ++s) {
          lo[s] = std::min(lo[s], J[s][t]);
          hi[s] = std::max(hi[s], J[s][t]);
        }
        ++t;
      }
      const int32_t ci = (int32_t)chunks.size();
      chunks.push_back(make_int4(p, (int)(t0 - L.h_offs[p]), (int)(t - t0), 0));
      for (int64_t u = t0; u < t; ++u) {
        chunk_of[u] = ci;
        tt_of[u] = (int32_t)(u - t0);
      }
      for (int32_t s = 0; s < n_seg; ++s) {
        band_lo[s].push_back(lo[s]);
        band_n[s].push_back((int32_t)(hi[s] - lo[s]) + ws[s]);
        for (int64_t u = t0; u < t; ++u) J[s][u] -= lo[s];  // row of the TOA's first weight in its band
      }
    }
  }
  if (chunks.size() > (size_t)0x7FFFFFFF / 8) {
    G.why = "gridded path: too many chunks";
    return FPTA_OK;
  }
  G.n_chunks = (int32_t)chunks.size();
  G.psr_chunk0.assign((size_t)L.P + 1, 0);
  for (int32_t ci = (int32_t)chunks.size() - 1; ci >= 0; --ci) G.psr_chunk0[chunks[ci].x] = ci;
  G.psr_chunk0[L.P] = G.n_chunks;
  for (int32_t p = L.P - 1; p >= 0; --p)  // a pulsar without TOAs has no chunk: it starts where the next one does
    if (L.h_offs[p + 1] == L.h_offs[p]) G.psr_chunk0[p] = G.psr_chunk0[p + 1];
  if (int rc0 = upload(c, G.psr_c0, G.psr_chunk0.data(), sizeof(int32_t) * G.psr_chunk0.size(), "pulsar chunks"))
    return rc0;
  const int32_t n_chunks = G.n_chunks;
  // band rows of a chunk: every signal's band back to back (virtual rows voff_s ..), padded to a multiple of
  // 4 once per chunk (k_grid_interp_mfma: 4 rows per MFMA step; pad rows re-read a valid row at weight 0), and in
  // diagnostic builds to at least kGridMinV rows (k_grid_interp_st's operand lookahead never passes the next chunk; the
  // product kernels would only run zero-weight steps on them)
  std::vector<int32_t> voff((size_t)n_seg * n_chunks);
  int32_t vmax = 4;
  for (int32_t ci = 0; ci < n_chunks; ++ci) {
    int32_t v = 0;
    for (int32_t s = 0; s < n_seg; ++s) {
      voff[(size_t)s * n_chunks + ci] = v;
      v += band_n[s][ci];
    }
#ifdef FPTA_DIAG_KERNELS
    chunks[ci].w = std::max(kGridMinV, (v + 3) & ~3);
#else
    chunks[ci].w = (v + 3) & ~3;
#endif
    vmax = std::max(vmax, chunks[ci].w);
  }
  if (vmax > kGridVMax) {
    G.why = "gridded path: a chunk's band rows over all signals exceed " + std::to_string(kGridVMax);
    return FPTA_OK;
  }
  G.vmax = vmax;
  std::vector<int64_t> rowoff(n_seg);
  int64_t grid_rows = 0;
  for (int32_t s = 0; s < n_seg; ++s) {
    rowoff[s] = grid_rows;
    grid_rows += (int64_t)L.P * nf[s];
  }
  if (grid_rows > 0x7FFFFFFF) {
    G.why = "gridded path: grid too large";
    return FPTA_OK;
  }
  G.grid_rows = grid_rows;
  std::vector<int32_t> rt((size_t)n_chunks * vmax);
  for (int32_t ci = 0; ci < n_chunks; ++ci) {
    int32_t* r = rt.data() + (size_t)ci * vmax;
    const int32_t p = chunks[ci].x;
    int32_t v = 0;
    for (int32_t s = 0; s < n_seg; ++s)
      for (int32_t i = 0; i < band_n[s][ci]; ++i) {
        const int64_t j = ((band_lo[s][ci] + i) % nf[s] + nf[s]) % nf[s];
        r[v++] = (int32_t)(rowoff[s] + (int64_t)p * nf[s] + j);
      }
    for (; v < vmax; ++v) r[v] = r[0];
  }
  // k_grid_interp_wr (diagnostic kernel): ring slot kWrSlots s + (unwrapped row mod kWrSlots) per band row; load
  // lists per chunk
  std::vector<int4> wr_meta;
  std::vector<int2> wr_list;
  std::vector<int32_t> wr_slot;
#ifdef FPTA_DIAG_KERNELS
  bool wr_ok = n_seg <= kWrMaxSig && vmax <= kWrVMax;
#else
  bool wr_ok = false;
#endif
  for (int32_t s = 0; s < n_seg && wr_ok; ++s)
    for (int32_t ci = 0; ci < n_chunks && wr_ok; ++ci) wr_ok = band_n[s][ci] <= kWrSlots;
  if (wr_ok) {
    wr_meta.resize(n_chunks);
    wr_slot.assign((size_t)n_chunks * vmax, 0);
    for (int32_t ci = 0; ci < n_chunks; ++ci) {
      const int32_t p = chunks[ci].x;
      int32_t* sl = wr_slot.data() + (size_t)ci * vmax;
      int32_t v = 0;
      for (int32_t s = 0; s < n_seg; ++s)
        for (int32_t i = 0; i < band_n[s][ci]; ++i)
          sl[v++] = kWrSlots * s + (int32_t)((band_lo[s][ci] + i) & (kWrSlots - 1));
      for (; v < vmax; ++v) sl[v] = sl[0];
      // the bands of chunks ci - back .. ci (same pulsar) in one ring window per signal: compat (back 1) = only the rows
      // the previous band does not hold load, after the chunk before has been computed; near (back 2) = they may load
      // while the chunk two back is computed
      auto window = [&](int32_t back) {
        if (ci < back) return false;
        for (int32_t b = 1; b <= back; ++b)
          if (chunks[ci - b].x != p) return false;
        for (int32_t s = 0; s < n_seg; ++s) {
          int64_t lo = band_lo[s][ci], hi = band_lo[s][ci] + band_n[s][ci];
          for (int32_t b = 1; b <= back; ++b) {
            lo = std::min(lo, band_lo[s][ci - b]);
            hi = std::max(hi, band_lo[s][ci - b] + (int64_t)band_n[s][ci - b]);
          }
          if (hi - lo > kWrSlots) return false;
        }
        return true;
      };
      const bool compat = window(1), near = compat && window(2);
      auto add_rows = [&](bool only_new) {
        int32_t n = 0;
        for (int32_t s = 0; s < n_seg; ++s)
          for (int32_t i = 0; i < band_n[s][ci]; ++i) {
            const int64_t u = band_lo[s][ci] + i;
            if (only_new && u >= band_lo[s][ci - 1] && u < band_lo[s][ci - 1] + band_n[s][ci - 1]) continue;
            const int64_t j = (u % nf[s] + nf[s]) % nf[s];
            wr_list.push_back(make_int2(kWrSlots * s + (int32_t)(u & (kWrSlots - 1)),
                                        (int32_t)(rowoff[s] + (int64_t)p * nf[s] + j)));
            ++n;
          }
        return n;
      };
      const int32_t full_off = (int32_t)wr_list.size();
      const int32_t full_n = add_rows(false);
      int32_t new_off = full_off, new_n = full_n;
      if (compat) {
        new_off = (int32_t)wr_list.size();
        new_n = add_rows(true);
      }
      wr_meta[ci] = make_int4(full_off, full_n, new_off, new_n | (compat ? 0 : kWrFresh) | (near ? 0 : kWrFar));
    }
  }
  // LDS-staged interpolation (k_grid_interp_lds): groups of <= kLdsGroup consecutive chunks of one pulsar whose
  // bands, over all signals, unite to <= kLdsRowsMax rows. Per group the union's grid-buffer rows (signal by
  // signal, each signal's rows one contiguous unwrapped range), per chunk the union slot of each band row.
  std::vector<int4> groups;
  std::vector<int32_t> urows, lrt((size_t)n_chunks * vmax);
  int32_t umax = 0;
  bool lds_ok = true;
  for (int32_t ci = 0; ci < n_chunks && lds_ok;) {
    const int32_t p = chunks[ci].x;
    auto union_rows = [&](int32_t n) {
      int64_t u = 0;
      for (int32_t s = 0; s < n_seg; ++s) {
        int64_t lo = band_lo[s][ci], end = band_lo[s][ci] + band_n[s][ci];
        for (int32_t k = 1; k < n; ++k) {
          lo = std::min(lo, band_lo[s][ci + k]);
          end = std::max(end, band_lo[s][ci + k] + (int64_t)band_n[s][ci + k]);
        }
        u += end - lo;
      }
      return u;
    };
    int32_t n = 1;
    while (n < kLdsGroup && ci + n < n_chunks && chunks[ci + n].x == p && union_rows(n + 1) <= kLdsRowsMax) ++n;
    const int64_t U = union_rows(n);
    if (U > kLdsRowsMax) {
      lds_ok = false;  // one chunk's bands alone exceed the LDS budget: the register-tiled kernel serves the layout
      break;
    }
    groups.push_back(make_int4(ci, n, (int32_t)U, (int32_t)urows.size()));
    umax = std::max(umax, (int32_t)U);
    int32_t uoff = 0;
    for (int32_t s = 0; s < n_seg; ++s) {
      int64_t lo = band_lo[s][ci], end = band_lo[s][ci] + band_n[s][ci];
      for (int32_t k = 1; k < n; ++k) {
        lo = std::min(lo, band_lo[s][ci + k]);
        end = std::max(end, band_lo[s][ci + k] + (int64_t)band_n[s][ci + k]);
      }
      for (int64_t j = lo; j < end; ++j)
        urows.push_back((int32_t)(rowoff[s] + (int64_t)p * nf[s] + ((j % nf[s]) + nf[s]) % nf[s]));
      for (int32_t k = 0; k < n; ++k) {  // chunk ci + k: signal s's band rows start at slot uoff + (its lo - lo)
        int32_t v = 0;
        for (int32_t s2 = 0; s2 < s; ++s2) v += band_n[s2][ci + k];
        for (int32_t i = 0; i < band_n[s][ci + k]; ++i)
          lrt[(size_t)(ci + k) * vmax + v + i] = uoff + (int32_t)(band_lo[s][ci + k] - lo) + i;
      }
      uoff += (int32_t)(end - lo);
    }
    for (int32_t k = 0; k < n; ++k) {  // pad rows: any valid slot (weight 0)
      int32_t* r = lrt.data() + (size_t)(ci + k) * vmax;
      int32_t v = 0;
      for (int32_t s = 0; s < n_seg; ++s) v += band_n[s][ci + k];
      for (; v < vmax; ++v) r[v] = r[0];
    }
    ci += n;
  }
  G.lds_ok = lds_ok && !groups.empty();
  G.n_groups = (int32_t)groups.size();
  G.lds_rows = umax;
  // k_grid_interp_u plan (diagnostic builds): the same grouping under the tighter LDS budget of two workgroups per CU
  std::vector<int4> ug;
  std::vector<int32_t> uur, ucb, uwr;
#ifdef FPTA_DIAG_KERNELS
  bool u_ok = n_seg <= kUnionSigMax;
#else
  bool u_ok = false;
#endif
  for (int32_t ci = 0; ci < n_chunks && u_ok;) {
    const int32_t p = chunks[ci].x;
    auto span = [&](int32_t s, int32_t n, int64_t& lo, int64_t& end) {
      lo = band_lo[s][ci];
      end = band_lo[s][ci] + band_n[s][ci];
      for (int32_t k = 1; k < n; ++k) {
        lo = std::min(lo, band_lo[s][ci + k]);
        end = std::max(end, band_lo[s][ci + k] + (int64_t)band_n[s][ci + k]);
      }
    };
    auto union_rows = [&](int32_t n) {
      int64_t u = 0, lo, end;
      for (int32_t s = 0; s < n_seg; ++s) {
        span(s, n, lo, end);
        u += end - lo;
      }
      return u;
    };
    int32_t n = 1;
    while (n < kUnionGroup && ci + n < n_chunks && chunks[ci + n].x == p && union_rows(n + 1) <= kUnionRowsMax) ++n;
    const int64_t U = union_rows(n);
    if (U > kUnionRowsMax) {
      u_ok = false;
      break;
    }
    ug.push_back(make_int4(ci, n, (int32_t)U, (int32_t)uur.size()));
    int32_t uoff = 0;
    std::vector<int32_t> cb((size_t)n * 2 * kUnionSigMax, 0);
    for (int32_t s = 0; s < n_seg; ++s) {
      int64_t lo, end;
      span(s, n, lo, end);
      for (int64_t j = lo; j < end; ++j)
        uur.push_back((int32_t)(rowoff[s] + (int64_t)p * nf[s] + ((j % nf[s]) + nf[s]) % nf[s]));
      for (int32_t k = 0; k < n; ++k) {
        const int32_t vo = voff[(size_t)s * n_chunks + ci + k];
        cb[(size_t)k * 2 * kUnionSigMax + s] = vo;
        cb[(size_t)k * 2 * kUnionSigMax + kUnionSigMax + s] = uoff + (int32_t)(band_lo[s][ci + k] - lo) - vo;
      }
      uoff += (int32_t)(end - lo);
    }
    for (int32_t k = 0; k < n; ++k)
      for (int32_t s = n_seg; s < kUnionSigMax; ++s) {  // absent signals: never selected (offset past every row)
        cb[(size_t)k * 2 * kUnionSigMax + s] = 1 << 20;
        cb[(size_t)k * 2 * kUnionSigMax + kUnionSigMax + s] = 0;
      }
    ucb.insert(ucb.end(), cb.begin(), cb.end());
    ci += n;
  }
  G.u_ok = u_ok && !ug.empty();
  G.u_groups = (int32_t)ug.size();
  G.u_sig = n_seg;
  if (G.u_ok) {
    uwr.assign((size_t)n_chunks * n_seg * kGridTT, -(1 << 20));  // empty TOA slots: every weight 0
    for (int32_t s = 0; s < n_seg; ++s)
      for (int64_t t = 0; t < N; ++t)
        uwr[((size_t)chunk_of[t] * n_seg + s) * kGridTT + tt_of[t]] =
            (int32_t)J[s][t] + voff[(size_t)s * n_chunks + chunk_of[t]];
    for (int32_t s = 0; s < n_seg; ++s) {
      G.u_w[s] = ws[s];
      G.u_hw[s] = 0.5 * (double)ws[s];
      G.u_beta[s] = betas[s];
    }
  }
  int rc;
  G.wr_ok = wr_ok;
  if (wr_ok && ((rc = upload(c, G.wr_meta, wr_meta.data(), sizeof(int4) * wr_meta.size(), "window plan")) ||
                (rc = upload(c, G.wr_list, wr_list.data(), sizeof(int2) * std::max<size_t>(wr_list.size(), 1),
                             "window rows")) ||
                (rc = upload(c, G.wr_slot, wr_slot.data(), sizeof(int32_t) * wr_slot.size(), "window slots"))))
    return rc;
  if ((rc = upload(c, G.chunks, chunks.data(), sizeof(int4) * chunks.size(), "grid chunks")) ||
      (rc = upload(c, G.rows, rt.data(), sizeof(int32_t) * rt.size(), "grid band rows")))
    return rc;
  if (G.lds_ok && ((rc = upload(c, G.groups, groups.data(), sizeof(int4) * groups.size(), "grid groups")) ||
                   (rc = upload(c, G.urows, urows.data(), sizeof(int32_t) * urows.size(), "grid union rows")) ||
                   (rc = upload(c, G.lrows, lrt.data(), sizeof(int32_t) * lrt.size(), "grid LDS rows"))))
    return rc;
  if (G.u_ok) {
    if ((rc = upload(c, G.ugroups, ug.data(), sizeof(int4) * ug.size(), "union groups")) ||
        (rc = upload(c, G.uurows, uur.data(), sizeof(int32_t) * uur.size(), "union rows")) ||
        (rc = upload(c, G.ucbase, ucb.data(), sizeof(int32_t) * ucb.size(), "union bases")) ||
        (rc = upload(c, G.uwrow, uwr.data(), sizeof(int32_t) * uwr.size(), "union window rows")))
      return rc;
    const size_t dbytes = sizeof(double) * 2 * (size_t)n_chunks * n_seg * kGridTT;
    HIPCHK(c, G.udch.ensure(dbytes), "union weight parameters alloc");
    HIPCHK(c, hipMemsetAsync(G.udch.p, 0, dbytes, c->stream), "union weight parameters memset");
  }
  DevBuf d_chunk_of, d_tt_of, d_row, d_d;
  if ((rc = upload(c, d_chunk_of, chunk_of.data(), sizeof(int32_t) * N, "grid chunk_of")) ||
      (rc = upload(c, d_tt_of, tt_of.data(), sizeof(int32_t) * N, "grid tt_of")))
    return rc;
  // + kFusedWdPad band rows after the last chunk: k_grid_fused loads NQ band steps' weights of every chunk unclamped
  const size_t wbytes = sizeof(double) * ((size_t)n_chunks * vmax + kFusedWdPad) * kGridTT;
  HIPCHK(c, G.wd.ensure(wbytes), "grid weights alloc");
  HIPCHK(c, hipMemsetAsync(G.wd.p, 0, wbytes, c->stream), "grid weights memset");
  std::vector<double> gx, gw;
  gauss_legendre(256, gx, gw);
  G.fma_direct = 0.0;
  G.fma_grid = 0.0;
  G.fma_interp = 0.0;
  G.fma_dft = 0.0;
  G.grid_vals = 0.0;
  for (int32_t ci = 0; ci < n_chunks; ++ci) G.fma_interp += (double)chunks[ci].w * kGridTT;
  G.mean_v = G.fma_interp / kGridTT / std::max(n_chunks, 1);
  G.weight_bytes = (double)wbytes;
  for (Seg* sg : L.segs) G.fma_direct += 2.0 * sg->d.nm * (double)N;
  for (int32_t s = 0; s < n_seg; ++s) {
    const SegDesc& d = L.segs[G.anchor[s]]->d;
    GridSeg* gs = new GridSeg();
    G.segs.push_back(gs);
    gs->nf = nf[s];
    gs->half = nf[s] / 2;
    gs->lde = (gs->half + kGridDftRows) / kGridDftRows * kGridDftRows;  // row blocks of k_grid_dft_mfma and k_grid_dft
    gs->ntab = (d.nm + 7) / 8 * 8;         // whole pairs of 4-mode MFMA k-steps (zero rows)
    gs->rowoff = rowoff[s];
    // q_k = (2 pi / nf) / phi_hat(k), phi_hat(k) = alpha int_{-1}^{1} phi(z) cos(k alpha z) dz, alpha = pi w / nf
    const double alpha = M_PI * ws[s] / nf[s], beta = betas[s];
    std::vector<double> ec((size_t)gs->ntab * gs->lde, 0.0), es((size_t)gs->ntab * gs->lde, 0.0);
    for (int32_t m = 0; m < d.nm; ++m) {
      const int64_t k = m + 1;
      double ph = 0.0;
      for (size_t q = 0; q < gx.size(); ++q)
        ph += gw[q] * std::exp(beta * (std::sqrt(1.0 - gx[q] * gx[q]) - 1.0)) * std::cos(k * alpha * gx[q]);
      const double qk = (2.0 * M_PI / nf[s]) / (alpha * ph);
      for (int32_t j = 0; j <= gs->half; ++j) {
        const double a = 2.0 * M_PI * (double)((k * j) % nf[s]) / nf[s];  // exact argument reduction
        ec[(size_t)m * gs->lde + j] = qk * std::cos(a);
        es[(size_t)m * gs->lde + j] = qk * std::sin(a);
      }
    }
    if ((rc = upload(c, gs->ecos, ec.data(), sizeof(double) * ec.size(), "grid ecos")) ||
        (rc = upload(c, gs->esin, es.data(), sizeof(double) * es.size(), "grid esin")))
      return rc;
    // quarter-range tables by parity: [0] cos / [1] sin of odd k = 2 t + 1 (m = 2 t), [2] / [3] of even k = 2 t + 2
    gs->ldq = (nf[s] / 4 + kGridDftRows) / kGridDftRows * kGridDftRows;
    gs->ntq = ((d.nm + 1) / 2 + 7) / 8 * 8;
    std::vector<double> tq((size_t)4 * gs->ntq * gs->ldq, 0.0);
    for (int32_t m = 0; m < d.nm; ++m) {
      const int32_t par = m & 1, t = m >> 1;
      for (int32_t j = 0; j <= nf[s] / 4; ++j) {
        tq[((size_t)(2 * par) * gs->ntq + t) * gs->ldq + j] = ec[(size_t)m * gs->lde + j];
        tq[((size_t)(2 * par + 1) * gs->ntq + t) * gs->ldq + j] = es[(size_t)m * gs->lde + j];
      }
    }
    if ((rc = upload(c, gs->tq, tq.data(), sizeof(double) * tq.size(), "grid quarter tables"))) return rc;
    // weight rows of signal s: its band's virtual offset in the chunk + the TOA's first row in the band
    std::vector<int32_t> row(N);
    for (int64_t t = 0; t < N; ++t) row[t] = (int32_t)J[s][t] + voff[(size_t)s * n_chunks + chunk_of[t]];
    if ((rc = upload(c, d_row, row.data(), sizeof(int32_t) * N, "grid rows")) ||
        (rc = upload(c, d_d, D[s].data(), sizeof(double) * N, "grid offsets")))
      return rc;
    HIPCHK(c,
           launch_grid_weights(c->stream, d, N, L.nu.as<double>(), d_chunk_of.as<int32_t>(), d_tt_of.as<int32_t>(),
                               d_row.as<int32_t>(), d_d.as<double>(), ws[s], beta, vmax, G.wd.as<double>(),
                               G.u_ok ? G.udch.as<double>() : nullptr, s, n_seg),
           "k_grid_weights launch");
    HIPCHK(c, hipStreamSynchronize(c->stream), "grid weights sync");  // d_row / d_d are reused
    // multiply-adds per realization: quarter range by parity on MFMA, half range on VALU
    G.fma_dft += (double)L.P * ((c->grid_mfma & 1) ? (gs->nf / 4 + 1) * 2.0 * d.nm : (gs->half + 1) * 2.0 * d.nm);
    G.grid_vals += (double)L.P * gs->nf;
    G.fma_grid = G.fma_dft + G.fma_interp;
  }
  // k_grid_fused: the grids of kFusedReal realizations plus the draw ring fit in LDS, n_seg <= kFusedMaxSig, and every
  // 32-row DFT chunk is one DFT wave's job
  {
    int32_t jobs = 0, rows = 0;
    bool ok = n_seg <= kFusedMaxSig;
    for (int32_t s = 0; s < n_seg && ok; ++s) {
      const GridSeg* gs = G.segs[s];
      ok = gs->nf % 4 == 0 && gs->ldq == (gs->nf / 4 + 32) / 32 * 32;
      G.fused_lrow0.push_back(rows);
      jobs += (gs->nf / 4 + 32) / 32;
      rows += gs->nf;
    }
    const size_t lds = sizeof(double) * ((size_t)rows * kFusedPitch + 2 * kFusedMaxSig * kFusedSlot) + 16;
    for (const std::vector<int32_t>& m : G.members) ok = ok && m.size() <= (size_t)kDftGenTerms;
    ok = ok && jobs <= kFusedDW && lds <= (size_t)kFusedLdsMax;
    if (ok) {
      // [n_chunks][4][fq]: band row 4 q + j of a chunk at [j][q] (a lane's rows of consecutive steps contiguous: 16-byte
      // loads), fq = the band steps rounded up to 4 and at least kFusedNQ; steps past the chunk's repeat its first row
      const int32_t fq = std::max(kFusedNQ, (vmax / 4 + 3) & ~3);
      std::vector<int32_t> band_row(vmax);
      std::vector<int32_t> lrt((size_t)n_chunks * 4 * fq);
      for (int32_t ci = 0; ci < n_chunks; ++ci) {
        int32_t v = 0;
        for (int32_t s = 0; s < n_seg; ++s)
          for (int32_t i = 0; i < band_n[s][ci]; ++i)
            band_row[v++] = G.fused_lrow0[s] + (int32_t)(((band_lo[s][ci] + i) % nf[s] + nf[s]) % nf[s]);
        for (; v < vmax; ++v) band_row[v] = band_row[0];
        int32_t* r = lrt.data() + (size_t)ci * 4 * fq;
        for (int32_t j = 0; j < 4; ++j)
          for (int32_t q = 0; q < fq; ++q) r[j * fq + q] = 4 * q + j < vmax ? band_row[4 * q + j] : band_row[0];
      }
      if ((rc = upload(c, G.frows, lrt.data(), sizeof(int32_t) * lrt.size(), "fused LDS rows"))) return rc;
      G.fused_fq = fq;
      G.fused_lds = lds;
    }
    G.fused_ok = ok;
  }
  G.ok = true;
  return FPTA_OK;
}

// Partial-checksum groups of G: each pulsar's chunks cut into runs of <= size consecutive chunks (a group never spans
// two pulsars, so a workgroup that owns a pulsar owns its groups), uploaded once per (plan, size).
int grid_part_groups(fpta_ctx* c, GridPlan& G, int32_t P, int32_t size) {
  if (G.pg_size == size) return FPTA_OK;
  std::vector<int32_t> first, psr((size_t)P + 1);
  for (int32_t p = 0; p < P; ++p) {
    psr[p] = (int32_t)first.size();
    for (int32_t ci = G.psr_chunk0[p]; ci < G.psr_chunk0[p + 1]; ci += size) first.push_back(ci);
  }
  psr[P] = (int32_t)first.size();
  first.push_back(G.n_chunks);
  int rc;
  if ((rc = upload(c, G.pgfirst, first.data(), sizeof(int32_t) * first.size(), "partial groups")) ||
      (rc = upload(c, G.psr_pg, psr.data(), sizeof(int32_t) * psr.size(), "partial groups of pulsars")))
    return rc;
  G.n_pg = (int32_t)first.size() - 1;
  G.pg_size = size;
  return FPTA_OK;
}

// Run the gridded synthesis: one DFT launch per grid signal, then one interpolation launch for all.
// pipe (run_coefficients drew this block on the side stream in pipelined mode): the DFTs follow there, into grid
// buffer c->gbuf, and the interpolation on the ctx stream waits only for them.
int grid_run(fpta_ctx* c, Layout& L, SynthArgs& a, int32_t R_pad, bool pipe = false) {
  GridPlan& G = L.grid;
  GridSegs gsegs{};
  gsegs.n = (int32_t)G.segs.size();
  const size_t gbytes = sizeof(double) * (size_t)G.grid_rows * R_pad;
  // k_grid_interp_psr: no DFT launch, no grid buffer; in a pipelined block the coefficients drawn on the side stream
  // into buffer gi are this block's (run_coefficients)
  const bool psr = psr_layout(c, L) && !a.w_on && !a.accumulate && (!pipe || c->prev_psr);
  // k_grid_fused: the DFTs run inside the synthesis kernel too (plain blocks: no white epilogue, no partial checksums)
  const bool fused = !psr && fused_layout(c, L) && !a.w_on && !a.accumulate &&
                     !(c->fuse_sums && a.out == c->out.as<double>()) && (!pipe || c->prev_psr);
  // grid buffers only for the kernels that read one (two of 0.41 GB each on C2)
  if (!psr && !fused && (G.g_rpad != R_pad || (pipe && G.g2.cap < gbytes))) {
    if (c->side) HIPCHK(c, hipStreamSynchronize(c->side), "side sync");  // no reader of a buffer being regrown
    if (c->side2) HIPCHK(c, hipStreamSynchronize(c->side2), "side sync");
    HIPCHK(c, hipStreamSynchronize(c->stream), "grid regrow sync");
    HIPCHK(c, G.g.ensure(gbytes), "grid alloc");
    if (pipe) HIPCHK(c, G.g2.ensure(gbytes), "grid alloc");
    G.g_rpad = R_pad;
  }
  const int gi = pipe ? c->gbuf : 0;
  double* const gbase = gi ? G.g2.as<double>() : G.g.as<double>();
  if (pipe) {
    for (hipEvent_t* e : {&c->ev_gready, &c->ev_gfree[0], &c->ev_gfree[1]})
      if (!*e) HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming), "event create");
    // the DFT overwrites buffer gi: the interpolation that last read it (two blocks back) must be done
    if (c->gfree_set[gi]) HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_gfree[gi], 0), "grid buffer wait");
  }
  if (psr || fused) {
    GridSeg* gs = G.segs[0];
    GridSegDev& g = gsegs.s[0];
    g.g = nullptr;
    g.nf = gs->nf;
    g.half = gs->half;
    g.nm = L.segs[G.anchor[0]]->d.nm;
    g.col0 = L.segs[G.anchor[0]]->d.col0;
    g.tq = gs->tq.as<double>();
    g.ldq = gs->ldq;
    g.ntq = gs->ntq;
    if (pipe) {
      HIPCHK(c, hipEventRecord(c->ev_gready, c->side), "event record");
      c->coef_last_side = false;  // the interpolation on the ctx stream reads the coefficients
    } else {
      int rc = wait_coef_all(c);
      if (rc) return rc;
    }
  } else {
    KTimer kt(c, FPTA_K_GRID, pipe ? c->side : c->stream);
    for (size_t s = 0; s < G.segs.size(); ++s) {
      GridSeg* gs = G.segs[s];
      const SegDesc& d = L.segs[G.anchor[s]]->d;  // a coalesced grid signal reads its anchor's merged columns
      GridSegDev& g = gsegs.s[s];
      g.ecos = gs->ecos.as<double>();
      g.esin = gs->esin.as<double>();
      g.g = gbase + gs->rowoff * R_pad;
      g.nf = gs->nf;
      g.half = gs->half;
      g.lde = gs->lde;
      g.nm = d.nm;
      g.col0 = d.col0;
      g.ntab = gs->ntab;
      g.tq = gs->tq.as<double>();
      g.ldq = gs->ldq;
      g.ntq = gs->ntq;
    }
    const bool early_free = c->coef_side && !c->coef_copy_pending;
    const int32_t split = pipe && c->split_g < gsegs.n ? c->split_g : -1;
    c->split_g = -1;
    // the DFTs of a set of grid signals on one stream: each k_grid_dft_gen signal its own launch, the others in one
    // k_grid_dft_mfma / k_grid_dft launch
    auto dfts = [&](hipStream_t sd, const std::vector<int32_t>& sigs) -> int {
      GridSegs rest{};
      for (int32_t s : sigs) {
        if (!grid_gen_fused(c, L, (size_t)s)) {
          rest.s[rest.n++] = gsegs.s[s];
          continue;
        }
        DftGenArgs d{};
        d.g = gsegs.s[s];
        std::vector<int32_t> order{G.anchor[s]};  // the merge order: anchor, then the others in layout order
        for (int32_t i : G.members[s])
          if (i != G.anchor[s]) order.push_back(i);
        for (int32_t i : order) {
          const SegDesc& sd2 = L.segs[i]->d;
          d.term_kind[d.n_terms] = sd2.kind;
          d.term_seg[d.n_terms] = i;
          d.term_nm[d.n_terms] = sd2.nm;
          d.term_col0[d.n_terms] = sd2.col0;
          d.term_amp[d.n_terms] = sd2.amp;
          ++d.n_terms;
        }
        d.coef = a.coef;
        d.P = L.P;
        d.K = a.K;
        d.R_pad = R_pad;
        d.n_real = a.n_real;
        d.real0 = c->blk_real0;
        d.k0 = c->blk_k0;
        d.k1 = c->blk_k1;
        HIPCHK(c, launch_grid_dft_gen(sd, d), "k_grid_dft_gen launch");
      }
      if (rest.n)
        HIPCHK(c,
               (c->grid_mfma & 1) ? launch_grid_dft_mfma(sd, rest, L.P, a.coef, a.K, R_pad)
                                  : launch_grid_dft(sd, rest, L.P, a.coef, a.K, R_pad),
               "k_grid_dft launch");
      return FPTA_OK;
    };
    std::vector<int32_t> all_sigs(gsegs.n);
    for (int32_t s = 0; s < gsegs.n; ++s) all_sigs[s] = s;
    if (pipe && split >= 0) {
      // the split signal's DFT on side2 (after its draws there), the others' on side
      std::vector<int32_t> rest_sigs;
      for (int32_t s = 0; s < gsegs.n; ++s)
        if (s != split) rest_sigs.push_back(s);
      {
        if (c->gfree_set[gi]) HIPCHK(c, hipStreamWaitEvent(c->side2, c->ev_gfree[gi], 0), "grid buffer wait");
        if (c->side_split == 2) {
          if (!c->ev_s2mix) HIPCHK(c, hipEventCreateWithFlags(&c->ev_s2mix, hipEventDisableTiming), "event create");
          HIPCHK(c, hipEventRecord(c->ev_s2mix, c->side), "event record");
          HIPCHK(c, hipStreamWaitEvent(c->side2, c->ev_s2mix, 0), "side wait");
        }
        KTimer kt2(c, FPTA_K_GRID, c->side2);
        int rc = dfts(c->side2, {split});
        if (rc) return rc;
      }
      HIPCHK(c, hipEventRecord(c->ev_gready2, c->side2), "event record");
      c->s2done_set = true;
      int rc = dfts(c->side, rest_sigs);
      if (rc) return rc;
    } else if (pipe) {
      int rc = dfts(c->side, all_sigs);
      if (rc) return rc;
    } else if (c->coef_side) {
      // one DFT launch per grid signal, each after that signal's draws (and merge) only (side stream); in the
      // order their draws complete
      std::vector<int32_t> order(gsegs.n);
      for (int32_t s = 0; s < gsegs.n; ++s) order[s] = s;
      std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return G.last[x] < G.last[y]; });
      for (int32_t s : order) {
        GridSegs one{};
        one.s[0] = gsegs.s[s];
        one.n = 1;
        int rc = wait_coef(c, (size_t)G.last[s]);
        if (rc) return rc;
        HIPCHK(c,
               (c->grid_mfma & 1) ? launch_grid_dft_mfma(c->stream, one, L.P, a.coef, a.K, R_pad)
                                  : launch_grid_dft(c->stream, one, L.P, a.coef, a.K, R_pad),
               "k_grid_dft launch");
      }
      c->coef_side = false;
    } else {
      int rc = dfts(c->stream, all_sigs);
      if (rc) return rc;
    }
    if (pipe) {
      HIPCHK(c, hipEventRecord(c->ev_gready, c->side), "event record");
      c->coef_last_side = !c->coef_copy_pending;  // else the download on the ctx stream is the last reader
    } else if (early_free) {  // the DFT was the last reader of coef: the next block may draw during the interpolation
      if (!c->ev_coef_free) HIPCHK(c, hipEventCreateWithFlags(&c->ev_coef_free, hipEventDisableTiming), "event create");
      HIPCHK(c, hipEventRecord(c->ev_coef_free, c->stream), "event record");
      c->coef_free_set = true;
    }
  }
  // partial checksums of a batch block (written into the context's own block, not accumulated)
  if (c->fuse_sums && a.out == c->out.as<double>() && !a.accumulate) {
    const int pi = c->part_next;
    DevBuf& pb = c->part[pi];
    const size_t pbytes = sizeof(double) * 2 * (size_t)G.n_chunks * R_pad;
    if (pb.cap < pbytes && c->red) HIPCHK(c, hipStreamSynchronize(c->red), "partials regrow sync");
    HIPCHK(c, pb.ensure(pbytes), "partial checksums alloc");
    // the reduction of the block that last wrote this buffer (on the red stream) must have read it
    if (c->pfree_set[pi]) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_pfree[pi], 0), "partials buffer wait");
    a.part = pb.as<double>();
    int rc = grid_part_groups(c, G, L.P, c->part_group);
    if (rc) return rc;
    c->part_cur = pi;
    c->part_next = pi ^ 1;
  }
  if (pipe) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_gready, 0), "grid ready wait");
  if (pipe && c->s2done_set) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_gready2, 0), "grid ready wait");
  KTimer kt(c, FPTA_K_SYNTH);
  GridBand band{G.chunks.as<int4>(), G.rows.as<int32_t>(), G.wd.as<double>(), gbase, G.n_chunks, G.vmax,
                G.grid_rows, a.part ? G.pgfirst.as<int32_t>() : nullptr, a.part ? G.n_pg : G.n_chunks};
  // the warp-specialised kernel for plain blocks; with fused partial checksums its reduce-scatter temporaries take
  // its VGPRs to 230 and the register kernel is faster (C3: 47.9 vs 52.5 ms per job, profiles/r02k_ab_c2c3_ws.txt)
  // k_grid_interp_ws tiles 512 realizations (4 compute waves x 128): when R_pad leaves some of the last tile's compute
  // waves idle, the 256-realization tiles of k_grid_interp_ws2 waste less (C4, R_pad = 256: half of every ws tile;
  // 6.8-7.4 vs 8.4 ms/step, profiles/r04a_c4_ws2.txt)
  const bool ws2_fits = c->interp_ws == 1 && (R_pad + 255) / 256 * 256 - R_pad < (R_pad + 511) / 512 * 512 - R_pad;
  int kind;  // the interpolation kernel (fpta_batch_grid_info_n slot 15)
  if (false) {
#ifdef FPTA_DIAG_KERNELS
  } else if (c->interp_ws == 5 && !c->interp_lds && G.u_ok && !a.w_on) {
    kind = 5;
    band.pgfirst = nullptr;  // the diagnostic kernels write one partial row per chunk
    band.n_pg = G.n_chunks;
    GridUnion un{G.ugroups.as<int4>(), G.uurows.as<int32_t>(), G.ucbase.as<int32_t>(), G.udch.as<double>(),
                 G.uwrow.as<int32_t>(), G.u_groups, G.u_sig, {G.u_w[0], G.u_w[1]}, {G.u_hw[0], G.u_hw[1]},
                 {G.u_beta[0], G.u_beta[1]}};
    HIPCHK(c, launch_grid_interp_u(c->stream, a, band, un, R_pad), "k_grid_interp_u launch");
  } else if (c->interp_ws == 4 && !c->interp_lds) {
    kind = 4;
    band.pgfirst = nullptr;
    band.n_pg = G.n_chunks;
    HIPCHK(c, launch_grid_interp_st(c->stream, a, band, R_pad), "k_grid_interp_st launch");
  } else if (c->interp_wr && G.wr_ok && !c->interp_lds && c->interp_ws > 0 && !a.w_on && !a.accumulate && !a.part &&
             R_pad % kWrReal == 0 && !psr) {
    kind = 10;
    GridWindow wrp{G.wr_meta.as<int4>(), G.wr_list.as<int2>(), G.wr_slot.as<int32_t>()};
    HIPCHK(c, launch_grid_interp_wr(c->stream, a, band, wrp, R_pad), "k_grid_interp_wr launch");
#endif
  } else if (fused) {
    const int32_t nq = G.vmax / 4;
    kind = nq <= 8 ? 8 : 9;  // launch_grid_fused: NQ = 8 or 12 band steps at a time
    FusedArgs f{};
    f.n_sig = (int32_t)G.segs.size();
    for (int32_t s = 0; s < f.n_sig; ++s) {
      const GridSeg* gs = G.segs[s];
      const SegDesc& d = L.segs[G.anchor[s]]->d;
      FusedSig& fs = f.s[s];
      fs.tq = gs->tq.as<double>();
      fs.ldq = gs->ldq;
      fs.ntq = gs->ntq;
      fs.nf = gs->nf;
      fs.nm = d.nm;
      fs.lrow0 = G.fused_lrow0[s];
      fs.n_rc = (gs->nf / 4 + 32) / 32;
      if (grid_gen_fused(c, L, (size_t)s)) {  // k_grid_dft_gen's terms: the anchor, then the others in layout order
        std::vector<int32_t> order{G.anchor[s]};
        for (int32_t i : G.members[s])
          if (i != G.anchor[s]) order.push_back(i);
        for (int32_t i : order) {
          const SegDesc& sd2 = L.segs[i]->d;
          fs.term_kind[fs.n_terms] = sd2.kind;
          fs.term_seg[fs.n_terms] = i;
          fs.term_nm[fs.n_terms] = sd2.nm;
          fs.term_col0[fs.n_terms] = sd2.col0;
          fs.term_amp[fs.n_terms] = sd2.amp;
          ++fs.n_terms;
        }
      } else {  // k_grid_dft_mfma's operand: the anchor's (merged) columns of the coefficient buffer
        fs.term_kind[0] = 1;
        fs.term_seg[0] = G.anchor[s];
        fs.term_nm[0] = d.nm;
        fs.term_col0[0] = d.col0;
        fs.n_terms = 1;
      }
    }
    f.ring_off = (G.fused_lrow0.back() + G.segs.back()->nf) * kFusedPitch;
    f.lrows = G.frows.as<int32_t>();
    f.fq = G.fused_fq;
    f.psr_c0 = G.psr_c0.as<int32_t>();
    f.real0 = c->blk_real0;
    f.k0 = c->blk_k0;
    f.k1 = c->blk_k1;
#ifdef FPTA_FUSED_PROF
    HIPCHK(c, c->dbg_a.ensure(sizeof(unsigned long long) * 8 * 8 * 4096), "fused profile alloc");
    HIPCHK(c, hipMemsetAsync(c->dbg_a.p, 0, sizeof(unsigned long long) * 8 * 8 * 4096, c->stream), "profile memset");
    f.prof = c->dbg_a.as<unsigned long long>();
#endif
    HIPCHK(c, launch_grid_fused(c->stream, a, band, f, nq, G.fused_lds), "k_grid_fused launch");
  } else if (psr) {
    kind = G.vmax <= 16 ? 6 : 7;  // launch_grid_interp_psr: NQ = 4 or 8 band steps
    HIPCHK(c,
           launch_grid_interp_psr(c->stream, a, band, gsegs.s[0],
                                  a.part ? G.psr_pg.as<int32_t>() : G.psr_c0.as<int32_t>(), L.P, R_pad),
           "k_grid_interp_psr launch");
  } else if ((c->interp_ws == 3 || ws2_fits) && !c->interp_lds && !a.w_on && !a.accumulate && !a.part) {
    kind = 2;
    HIPCHK(c, launch_grid_interp_ws(c->stream, a, band, R_pad, true), "k_grid_interp_ws2 launch");
  } else if (c->interp_ws && !c->interp_lds && !a.w_on && !a.accumulate && (!a.part || c->interp_ws == 2)) {
    kind = 1;
    HIPCHK(c, launch_grid_interp_ws(c->stream, a, band, R_pad), "k_grid_interp_ws launch");
#ifdef FPTA_DIAG_KERNELS
  } else if (c->interp_lds && G.lds_ok && !a.w_on) {
    kind = 3;
    band.pgfirst = nullptr;
    band.n_pg = G.n_chunks;
    GridLds lds{G.groups.as<int4>(), G.urows.as<int32_t>(), G.lrows.as<int32_t>(), G.n_groups, G.lds_rows};
    HIPCHK(c, launch_grid_interp_lds(c->stream, a, band, lds, R_pad), "k_grid_interp_lds launch");
#endif
  } else {
    kind = 0;
    HIPCHK(c, launch_grid_interp_mfma(c->stream, a, band, R_pad), "k_grid_interp_mfma launch");
  }
  c->last_interp = 1 + kind * 4 + (a.w_on ? 2 : 0) + (a.part ? 1 : 0);
  if (pipe) {  // buffer gi is free once this interpolation is done; the next block's DFT writes the other one
    HIPCHK(c, hipEventRecord(c->ev_gfree[gi], c->stream), "event record");
    c->gfree_set[gi] = true;
    c->gbuf = gi ^ 1;
  }
  if (a.part) {
    c->part_ready = true;
    c->part_chunks = band.n_pg;  // partial rows
    c->part_rpad = R_pad;
  }
  return FPTA_OK;
}

// White noise + ECORR to fuse into the synthesis epilogue (batch path).
struct WhiteCfg {
  int32_t on = 0;
  const double* sigma = nullptr;
  const int32_t* block_of = nullptr;
  const double* esig = nullptr;
  const double* zb = nullptr;
  int64_t nblocks = 0;
  int64_t real0 = 0;
  uint32_t k0 = 0, k1 = 0;
};

// Synthesis path of a batch (before its coefficients are drawn: a gridded plan that coalesces signals merges
// their coefficient columns, run_coefficients).
int select_path(fpta_ctx* c, Layout& L, int32_t R, bool allow_mfma, int* out_path) {
  // path: 1 direct, 2 MFMA, 3 VALU, 4 gridded; auto (0) = gridded when its plan needs fewer than
  // kGridAutoRatio of the direct FMAs and its a-priori error bound is within kGridAutoMaxErr, else VALU,
  // for R >= mfma_min_real; direct below. c->path_reason says why auto did not take the gridded path.
  int path = c->synth_path;
  c->path_reason.clear();
  *out_path = 0;
  if (!allow_mfma) {
    path = 1;
    c->path_reason = "single-realization drop-in call: direct path (exact phases)";
  } else if (path == 4) {
    if (!L.all_harmonic) return fail(c, FPTA_EINVAL, "gridded path: every signal needs a harmonic grid f_k = k f_1");
    if (c->anchor != 0) return fail(c, FPTA_EINVAL, "gridded path: needs anchor 0");
    int rc = grid_build(c, L);
    if (rc) return rc;
    if (!L.grid.ok) return fail(c, FPTA_EINVAL, L.grid.why);
  } else if (path == 0) {
    path = 3;
    if (R < c->mfma_min_real) {
      path = 1;
      c->path_reason = "gridded path: n_real below FPTA_OPT_MFMA_MIN_REAL (direct path)";
    } else if (!L.all_harmonic) {
      c->path_reason = "gridded path: every signal needs a harmonic grid f_k = k f_1";
    } else if (c->anchor != 0) {
      c->path_reason = "gridded path: needs anchor 0";
    } else {
      int rc = grid_build(c, L);
      if (rc) return rc;
      if (!L.grid.ok)
        c->path_reason = L.grid.why;
      else if (L.grid.err_bound > kGridAutoMaxErr)
        c->path_reason = "gridded path: a-priori error bound " + std::to_string(L.grid.err_bound) +
                         " of the width/oversampling options exceeds " + std::to_string(kGridAutoMaxErr);
      else if (!(L.grid.fma_grid < kGridAutoRatio * L.grid.fma_direct))
        c->path_reason = "gridded path: not cheaper than the direct contraction for this layout";
      else
        path = 4;
    }
  }
  *out_path = path;
  return FPTA_OK;
}

// *fused is set when the kernel that ran also added `white` (the seeded VALU and gridded kernels do).
// path: the select_path result for this batch, or -1 to select here.
int run_synth(fpta_ctx* c, Layout& L, int32_t R, int32_t R_pad, double* out, int64_t ldo, int accumulate,
              bool allow_mfma, const WhiteCfg* white = nullptr, bool* fused = nullptr, int path = -1,
              bool pipe = false) {
  if (fused) *fused = false;
  SynthArgs a{};
  a.offs = L.offs.as<int64_t>();
  a.psr_of = L.psr_of.as<int32_t>();
  a.toas = L.toas.as<double>();
  a.nu = L.nu.as<double>();
  a.segs = L.segdesc.as<SegDesc>();
  a.n_seg = (int32_t)L.segs.size();
  a.P = L.P;
  a.n_toa = L.n_toa;
  a.coef = c->coef.as<double>();
  a.K = L.K;
  a.R_pad = R_pad;
  a.out = out;
  a.ldo = ldo;
  a.n_real = R;
  a.accumulate = accumulate;
  a.anchor = c->anchor;
  a.coef_len = (int64_t)L.P * std::max(L.K, 1) * R_pad;
  if (path < 0) {
    int rc = select_path(c, L, R, allow_mfma, &path);
    if (rc) return rc;
  }
  // host-side guards of what the tiled kernels assume (every tile's realization block lies inside
  // the coefficient padding; the coefficient buffer holds P*K*R_pad values)
  if (R_pad % kRealPad != 0 || R > R_pad || kRealPad % kTileReal != 0 ||
      kRealPad % (4 * kValuVariants[c->valu_variant].nt) != 0)
    return fail(c, FPTA_EINVAL, "synth: realization padding inconsistent with the tile geometry");
  if (c->coef.cap < sizeof(double) * (size_t)L.P * std::max(L.K, 1) * R_pad)
    return fail(c, FPTA_ESTATE, "synth: coefficient buffer smaller than P*K*R_pad");
  c->last_path = path;
  if (path != 4) {
    int rc = wait_coef_all(c);  // only the gridded DFT consumes side-stream draws signal by signal
    if (rc) return rc;
  }
  if (path == 4) {
    if (white && white->on && c->fuse_white) {
      a.w_on = 1;
      a.w_sigma = white->sigma;
      a.w_block_of = white->block_of;
      a.w_esig = white->esig;
      a.w_zb = white->zb;
      a.w_nblocks = white->nblocks;
      a.real0 = white->real0;
      a.k0 = white->k0;
      a.k1 = white->k1;
      if (fused) *fused = true;
    }
    return grid_run(c, L, a, R_pad, pipe);
  } else if (path == 2) {
    int rc = build_tiles(c, L, R, kTileToa, kTileReal);
    if (rc || (rc = check_tiles(c, L, R, kTileToa, kTileReal, a))) return rc;
    KTimer kt(c, FPTA_K_SYNTH);
    HIPCHK(c, launch_synth_mfma(c->stream, a, L.tiles.as<int4>(), L.n_tiles), "k_synth_mfma launch");
  } else if (path == 3 && L.all_harmonic && c->anchor == 0) {
    const ValuVariant v = kSeededVariants[c->valu_variant];
    int rc = build_tiles(c, L, R, 4 * 64 * v.mt, v.nt);
    if (rc || (rc = check_tiles(c, L, R, 4 * 64 * v.mt, v.nt, a))) return rc;
    if (white && white->on && c->fuse_white) {
      a.w_on = 1;
      a.w_sigma = white->sigma;
      a.w_block_of = white->block_of;
      a.w_esig = white->esig;
      a.w_zb = white->zb;
      a.w_nblocks = white->nblocks;
      a.real0 = white->real0;
      a.k0 = white->k0;
      a.k1 = white->k1;
      if (fused) *fused = true;
    }
    KTimer kt(c, FPTA_K_SYNTH);
    HIPCHK(c,
           launch_synth_valu_seeded(c->stream, a, L.tiles.as<int4>(), L.n_tiles, L.seeds.as<double4>(),
                                    c->valu_variant),
           "k_synth_valu_seeded launch");
  } else if (path == 3) {
    const ValuVariant v = kValuVariants[c->valu_variant];
    int rc = build_tiles(c, L, R, 64 * v.mt, 4 * v.nt);
    if (rc || (rc = check_tiles(c, L, R, 64 * v.mt, 4 * v.nt, a))) return rc;
    KTimer kt(c, FPTA_K_SYNTH);
    HIPCHK(c, launch_synth_valu(c->stream, a, L.tiles.as<int4>(), L.n_tiles, c->valu_variant),
           "k_synth_valu launch");
  } else {
    if (R > 65535) return fail(c, FPTA_EINVAL, "direct synthesis path: n_real > 65535");
    KTimer kt(c, FPTA_K_SYNTH);
    HIPCHK(c, launch_synth_direct(c->stream, a), "k_synth_direct launch");
  }
  return FPTA_OK;
}

int blocks_to_owner(fpta_ctx* c, int64_t n_toa, int64_t n_blocks, const int64_t* boffs, const int64_t* bidx,
                    std::vector<int32_t>& owner) {
  owner.assign(n_toa, -1);
  if (n_blocks > (int64_t)0x7FFFFFFF) return fail(c, FPTA_EINVAL, "white: too many ECORR blocks");
  if (n_blocks > 0 && (!boffs || !bidx || boffs[0] != 0))
    return fail(c, FPTA_EINVAL, "white: bad ECORR block CSR");
  for (int64_t b = 0; b < n_blocks; ++b) {
    if (boffs[b + 1] < boffs[b]) return fail(c, FPTA_EINVAL, "white: block offsets not monotone");
    for (int64_t j = boffs[b]; j < boffs[b + 1]; ++j) {
      const int64_t t = bidx[j];
      if (t < 0 || t >= n_toa) return fail(c, FPTA_EINVAL, "white: block TOA index out of range");
      if (owner[t] >= 0) return fail(c, FPTA_EINVAL, "white: a TOA belongs to two ECORR blocks");
      owner[t] = (int32_t)b;
    }
  }
  return FPTA_OK;
}

// ----------------------------------------------------------------------------- dense covariance
inline int64_t pad_i64(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct DenseDims {
  int64_t n = 0, n_pad = 0;
  int32_t n_modes = 0, k_pad = 0;
};

// Basis + Gram: C [n_pad][n_pad] on device = sum_s B_s diag(w_s) B_s^T (+ diag white), full symmetric,
// padding rows/columns zero (the factor and the draws read them).
int dense_build(fpta_ctx* c, int64_t n, const double* toas, const double* nu, int32_t n_seg,
                const int32_t* seg_nmodes, const double* f, const double* w, const double* seg_idx,
                const double* seg_freqf, const double* white_var, DenseDims& d) {
  if (n <= 0 || !toas || !nu || n_seg <= 0 || !seg_nmodes || !f || !w || !seg_idx || !seg_freqf)
    return fail(c, FPTA_EINVAL, "dense: bad arguments");
  if (n > (int64_t)1 << 17) return fail(c, FPTA_EINVAL, "dense: more than 131072 TOAs");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  int64_t M = 0;
  for (int32_t s = 0; s < n_seg; ++s) {
    if (seg_nmodes[s] <= 0) return fail(c, FPTA_EINVAL, "dense: segment with no modes");
    M += seg_nmodes[s];
  }
  if (M > (1 << 20)) return fail(c, FPTA_EINVAL, "dense: too many modes");
  std::vector<double> sw((size_t)M);
  std::vector<int32_t> seg_of((size_t)M);
  for (int32_t s = 0, m = 0; s < n_seg; ++s)
    for (int32_t k = 0; k < seg_nmodes[s]; ++k, ++m) {
      if (!(w[m] >= 0.0)) return fail(c, FPTA_EINVAL, "dense: psd * df must be >= 0");
      sw[m] = std::sqrt(w[m]);
      seg_of[m] = s;
    }
  d.n = n;
  d.n_pad = pad_i64(n, 256);
  d.n_modes = (int32_t)M;
  d.k_pad = (int32_t)pad_i64(2 * M, 4);
  int rc;
  if ((rc = upload(c, c->dn_toas, toas, sizeof(double) * n, "dense toas"))) return rc;
  if ((rc = upload(c, c->dn_nu, nu, sizeof(double) * n, "dense nu"))) return rc;
  if ((rc = upload(c, c->dn_f, f, sizeof(double) * M, "dense f"))) return rc;
  if ((rc = upload(c, c->dn_sw, sw.data(), sizeof(double) * M, "dense w"))) return rc;
  if ((rc = upload(c, c->dn_segof, seg_of.data(), sizeof(int32_t) * M, "dense segments"))) return rc;
  if ((rc = upload(c, c->dn_segidx, seg_idx, sizeof(double) * n_seg, "dense idx"))) return rc;
  if ((rc = upload(c, c->dn_segff, seg_freqf, sizeof(double) * n_seg, "dense freqf"))) return rc;
  if (white_var && (rc = upload(c, c->dn_white, white_var, sizeof(double) * n, "dense white"))) return rc;
  HIPCHK(c, c->dn_GT.ensure(sizeof(double) * (size_t)d.k_pad * d.n_pad), "dense basis alloc");
  HIPCHK(c, c->dn_C.ensure(sizeof(double) * (size_t)d.n_pad * d.n_pad), "dense matrix alloc");
  HIPCHK(c, hipMemsetAsync(c->dn_C.p, 0, sizeof(double) * (size_t)d.n_pad * d.n_pad, c->stream), "dense memset");
  KTimer kt(c, FPTA_K_DENSE);
  HIPCHK(c,
         launch_cov_basis(c->stream, c->dn_toas.as<double>(), c->dn_nu.as<double>(), n, c->dn_f.as<double>(),
                          c->dn_sw.as<double>(), c->dn_segof.as<int32_t>(), c->dn_segidx.as<double>(),
                          c->dn_segff.as<double>(), d.n_modes, d.k_pad, c->dn_GT.as<double>(), d.n_pad),
         "k_cov_basis launch");
  HIPCHK(c,
         launch_gemm_tn(c->stream, c->dn_GT.as<double>(), d.n_pad, c->dn_GT.as<double>(), d.n_pad, false, false,
                        c->dn_C.as<double>(), d.n_pad, n, n, d.k_pad / 4, 1, 0, 2,
                        white_var ? c->dn_white.as<double>() : nullptr),
         "k_gemm_tn (gram) launch");
  return FPTA_OK;
}

// In-place lower Cholesky of C (right-looking, 64-wide panels: diagonal block in LDS, panel solve,
// MFMA trailing update). Fails with FPTA_EINVAL when C is not numerically positive definite.
int dense_cholesky(fpta_ctx* c, const DenseDims& d) {
  double* C = c->dn_C.as<double>();
  const int64_t ld = d.n_pad;
  HIPCHK(c, c->dn_PT.ensure(sizeof(double) * 64 * (size_t)d.n_pad), "dense panel alloc");
  HIPCHK(c, c->dn_info.ensure(sizeof(int)), "dense info alloc");
  HIPCHK(c, hipMemsetAsync(c->dn_info.p, 0, sizeof(int), c->stream), "dense info memset");
  {
    KTimer kt(c, FPTA_K_DENSE);
    const int32_t T = (int32_t)((d.n + 63) / 64);
    for (int32_t kb = 0; kb < T; ++kb) {
      const int64_t k0 = (int64_t)kb * 64;
      HIPCHK(c, launch_potrf_block(c->stream, C, ld, d.n, k0, c->dn_info.as<int>()), "k_potrf_block launch");
      if (k0 + 64 >= d.n) break;
      HIPCHK(c, launch_trsm_panel(c->stream, C, ld, d.n, k0, c->dn_PT.as<double>(), d.n_pad), "k_trsm_panel launch");
      HIPCHK(c,
             launch_gemm_tn(c->stream, c->dn_PT.as<double>(), d.n_pad, c->dn_PT.as<double>(), d.n_pad, false, false, C,
                            ld, d.n, d.n, 16, 1, kb + 1, 1, nullptr),
             "k_gemm_tn (update) launch");
    }
  }
  int info = 0;
  HIPCHK(c, hipMemcpyAsync(&info, c->dn_info.p, sizeof(int), hipMemcpyDeviceToHost, c->stream), "dense info");
  HIPCHK(c, hipStreamSynchronize(c->stream), "dense cholesky sync");
  if (info)
    return fail(c, FPTA_EINVAL, "dense: covariance not positive definite (pivot " + std::to_string(info - 1) + ")");
  return FPTA_OK;
}

}  // namespace

// =============================================================================================== API
extern "C" {

int fpta_version(void) { return 10000; }

const char* fpta_last_error(const fpta_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int fpta_device_count(int* n) {
  if (!n) return fail(nullptr, FPTA_EINVAL, "device_count: null");
  int k = 0;
  hipError_t e = hipGetDeviceCount(&k);
  if (e != hipSuccess) {
    *n = 0;
    return hip_fail(nullptr, e, "hipGetDeviceCount");
  }
  *n = k;
  return FPTA_OK;
}

int fpta_create(int device, fpta_ctx** out) {
  if (!out) return fail(nullptr, FPTA_EINVAL, "create: null out");
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return fail(nullptr, FPTA_EDEVICE, "create: no HIP device visible");
  if (device < 0 || device >= n) return fail(nullptr, FPTA_EINVAL, "create: device index out of range");
  e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(nullptr, e, "hipSetDevice");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      return fail(nullptr, FPTA_EDEVICE, std::string("create: built for gfx950, device is ") + prop.gcnArchName);
  }
  fpta_ctx* c = new fpta_ctx();
  c->device = device;
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return hip_fail(nullptr, e, "hipStreamCreate");
  }
  *out = c;
  return FPTA_OK;
}

int fpta_destroy(fpta_ctx* c) {
  if (!c) return FPTA_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (auto& p : c->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto e : c->pool) (void)hipEventDestroy(e);
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  if (c->side2) {
    (void)hipStreamSynchronize(c->side2);
    (void)hipStreamDestroy(c->side2);
  }
  if (c->red) {
    (void)hipStreamSynchronize(c->red);
    (void)hipStreamDestroy(c->red);
  }
  for (hipEvent_t e : {c->ev_pready, c->ev_pfree[0], c->ev_pfree[1], c->ev_red})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {c->ev_s2begin, c->ev_s2done, c->ev_gready2, c->ev_s2mix})
    if (e) (void)hipEventDestroy(e);
  if (c->ev_begin) (void)hipEventDestroy(c->ev_begin);
  if (c->ev_coef_free) (void)hipEventDestroy(c->ev_coef_free);
  for (hipEvent_t e : {c->ev_gready, c->ev_gfree[0], c->ev_gfree[1]})
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->ev_sig) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return FPTA_OK;
}

int fpta_set_option(fpta_ctx* c, int32_t key, int64_t value) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "set_option: null ctx");
  switch (key) {
    case FPTA_OPT_SYNTH_PATH:
      if (value < 0 || value > 4) return fail(c, FPTA_EINVAL, "synth path must be 0, 1, 2, 3 or 4");
      c->synth_path = (int)value;
      return FPTA_OK;
    case FPTA_OPT_GRID_WIDTH:
      if (value < 4 || value > 24) return fail(c, FPTA_EINVAL, "grid width must be in [4, 24]");
      c->grid_w = (int)value;
      c->batch.grid.clear();
      return FPTA_OK;
    case FPTA_OPT_GRID_SIGMA:
      if (value < 125 || value > 400) return fail(c, FPTA_EINVAL, "grid oversampling (x100) must be in [125, 400]");
      c->grid_sigma100 = (int)value;
      c->batch.grid.clear();
      return FPTA_OK;
    case FPTA_OPT_FUSE_WHITE:
      c->fuse_white = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_GRID_MFMA:
      // bit 1 (the interpolation kernel in round 1) is accepted and ignored: the interpolation is always on MFMA
      if (value < 0 || value > 3) return fail(c, FPTA_EINVAL, "grid MFMA mask must be in 0..3");
      c->grid_mfma = (int)(value & 1);
      return FPTA_OK;
    case FPTA_OPT_FUSE_CHECKSUMS:
      c->fuse_sums = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_MIX_MFMA:
      c->mix_mfma = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_OVERLAP:
      c->overlap = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_INTERP_LDS:
#ifndef FPTA_DIAG_KERNELS
      if (value) return fail(c, FPTA_EINVAL, "interp_lds: k_grid_interp_lds is a diagnostic kernel, not in this build");
#endif
      c->interp_lds = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_DFT_GEN:
      c->dft_gen = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_GEN_MIX:
      if (value < 0 || value > 3) return fail(c, FPTA_EINVAL, "gen_mix must be 0 .. 3");
      c->gen_mix = (int)value;
      return FPTA_OK;
    case FPTA_OPT_ASYNC_SUMS:
      c->async_sums = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_PART_GROUP:
      if (value < 1 || value > kPartGroupMax) return fail(c, FPTA_EINVAL, "part_group must be 1 .. 16");
      c->part_group = (int)value;
      return FPTA_OK;
    case FPTA_OPT_INTERP_PSR:
      c->interp_psr = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_INTERP_FUSED:
      c->interp_fused = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_INTERP_WR:
#ifndef FPTA_DIAG_KERNELS
      if (value) return fail(c, FPTA_EINVAL, "interp_wr: k_grid_interp_wr is a diagnostic kernel, not in this build");
#endif
      c->interp_wr = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_GRID_COALESCE:
      c->grid_coalesce = value ? 1 : 0;
      c->batch.grid.clear();
      return FPTA_OK;
    case FPTA_OPT_INTERP_WS:
      if (value < 0 || value > 5) return fail(c, FPTA_EINVAL, "interp_ws must be 0 .. 5");
#ifndef FPTA_DIAG_KERNELS
      if (value > 3)
        return fail(c, FPTA_EINVAL, "interp_ws 4 / 5: k_grid_interp_st / _u are diagnostic kernels, not in this build");
#endif
      c->interp_ws = (int)value;
      return FPTA_OK;
    case FPTA_OPT_SIDE_SPLIT:
      if (value < 0 || value > 2) return fail(c, FPTA_EINVAL, "side_split must be 0 .. 2");
      c->side_split = (int)value;
      return FPTA_OK;
    case FPTA_OPT_VALU_VARIANT:
      if (value < 0 || value >= kNumValuVariants) return fail(c, FPTA_EINVAL, "unknown VALU variant");
      c->valu_variant = (int)value;
      return FPTA_OK;
    case FPTA_OPT_MFMA_MIN_REAL:
      c->mfma_min_real = (int)std::max<int64_t>(1, value);
      return FPTA_OK;
    case FPTA_OPT_PROFILE:
      c->profile = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_ANCHOR:
      if (value < 0 || value > 1 << 20) return fail(c, FPTA_EINVAL, "anchor must be >= 0");
      c->anchor = (int)value;
      return FPTA_OK;
  }
  return fail(c, FPTA_EINVAL, "set_option: unknown key");
}

int fpta_get_option(fpta_ctx* c, int32_t key, int64_t* value) {
  if (!c || !value) return fail(c, FPTA_EINVAL, "get_option: bad arguments");
  switch (key) {
    case FPTA_OPT_SYNTH_PATH: *value = c->synth_path; return FPTA_OK;
    case FPTA_OPT_MFMA_MIN_REAL: *value = c->mfma_min_real; return FPTA_OK;
    case FPTA_OPT_PROFILE: *value = c->profile; return FPTA_OK;
    case FPTA_OPT_ANCHOR: *value = c->anchor; return FPTA_OK;
    case FPTA_OPT_VALU_VARIANT: *value = c->valu_variant; return FPTA_OK;
    case FPTA_OPT_FUSE_WHITE: *value = c->fuse_white; return FPTA_OK;
    case FPTA_OPT_GRID_WIDTH: *value = c->grid_w; return FPTA_OK;
    case FPTA_OPT_GRID_SIGMA: *value = c->grid_sigma100; return FPTA_OK;
    case FPTA_OPT_GRID_MFMA: *value = c->grid_mfma; return FPTA_OK;
    case FPTA_OPT_FUSE_CHECKSUMS: *value = c->fuse_sums; return FPTA_OK;
    case FPTA_OPT_MIX_MFMA: *value = c->mix_mfma; return FPTA_OK;
    case FPTA_OPT_OVERLAP: *value = c->overlap; return FPTA_OK;
    case FPTA_OPT_INTERP_LDS: *value = c->interp_lds; return FPTA_OK;
    case FPTA_OPT_GRID_COALESCE: *value = c->grid_coalesce; return FPTA_OK;
    case FPTA_OPT_INTERP_WS: *value = c->interp_ws; return FPTA_OK;
    case FPTA_OPT_SIDE_SPLIT: *value = c->side_split; return FPTA_OK;
    case FPTA_OPT_DFT_GEN: *value = c->dft_gen; return FPTA_OK;
    case FPTA_OPT_GEN_MIX: *value = c->gen_mix; return FPTA_OK;
    case FPTA_OPT_ASYNC_SUMS: *value = c->async_sums; return FPTA_OK;
    case FPTA_OPT_PART_GROUP: *value = c->part_group; return FPTA_OK;
    case FPTA_OPT_INTERP_PSR: *value = c->interp_psr; return FPTA_OK;
    case FPTA_OPT_INTERP_WR: *value = c->interp_wr; return FPTA_OK;
    case FPTA_OPT_INTERP_FUSED: *value = c->interp_fused; return FPTA_OK;
  }
  return fail(c, FPTA_EINVAL, "get_option: unknown key");
}

int fpta_build_flags(void) {
  int f = 0;
#ifdef FPTA_DEBUG
  f |= FPTA_BUILD_DEBUG;
#endif
#ifdef FPTA_DIAG_KERNELS
  f |= FPTA_BUILD_DIAG;
#endif
  return f;
}

int fpta_synchronize(fpta_ctx* c) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  int rc = join_red(c);
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  return FPTA_OK;
}

int fpta_kernel_stats(fpta_ctx* c, int32_t which, int64_t* count, double* total_ms) {
  if (!c || which < 0 || which >= FPTA_K_N) return fail(c, FPTA_EINVAL, "kernel_stats: bad args");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  for (auto& p : c->pending) {
    HIPCHK(c, hipEventSynchronize(p.b), "hipEventSynchronize");
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, p.a, p.b), "hipEventElapsedTime");
    c->kcount[p.which] += 1;
    c->kms[p.which] += ms;
    c->pool.push_back(p.a);
    c->pool.push_back(p.b);
  }
  c->pending.clear();
  if (count) *count = c->kcount[which];
  if (total_ms) *total_ms = c->kms[which];
  return FPTA_OK;
}

int fpta_reset_stats(fpta_ctx* c) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  int rc = fpta_kernel_stats(c, 0, nullptr, nullptr);
  if (rc) return rc;
  for (int i = 0; i < FPTA_K_N; ++i) {
    c->kcount[i] = 0;
    c->kms[i] = 0;
  }
  return FPTA_OK;
}

// ------------------------------------------------------------------------------------ drop-in
int fpta_gp_accumulate(fpta_ctx* c, int64_t n_toa, const double* toas, const double* nu, int32_t n_seg,
                       const int32_t* seg_nmodes, const double* f, const double* ccos, const double* csin,
                       const double* seg_idx, const double* seg_freqf, const uint8_t* mask, double sign,
                       double* residuals) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  const int64_t offs[2] = {0, n_toa};
  return fpta_gp_accumulate_array(c, 1, offs, toas, nu, n_seg, seg_nmodes, f, ccos, csin, seg_idx, seg_freqf, mask,
                                  sign, residuals);
}

int fpta_gp_accumulate_array(fpta_ctx* c, int32_t n_psr, const int64_t* offs, const double* toas, const double* nu,
                             int32_t n_seg, const int32_t* seg_nmodes, const double* f, const double* ccos,
                             const double* csin, const double* seg_idx, const double* seg_freqf, const uint8_t* mask,
                             double sign, double* residuals) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (n_psr <= 0 || !offs || n_seg <= 0 || !toas || !nu || !seg_nmodes || !f || !ccos || !csin || !seg_idx ||
      !seg_freqf || !residuals)
    return fail(c, FPTA_EINVAL, "gp_accumulate: bad arguments");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  Layout& L = c->scratch;
  int rc = layout_set_toas(c, L, n_psr, offs, toas, nu);
  if (rc) return rc;
  const int64_t n_toa = offs[n_psr];
  int64_t m0 = 0, nmax = 0;
  for (int32_t s = 0; s < n_seg; ++s) {
    const int32_t nm = seg_nmodes[s];
    if (nm <= 0) return fail(c, FPTA_EINVAL, "gp_accumulate: segment with no modes");
    // coefficient = sign * (ccos, csin) through the from-z path (amplitude = sign, exact)
    std::vector<double> amp((size_t)n_psr * nm, sign);
    rc = layout_add_signal(c, L, 0, nm, f + m0, amp.data(), seg_idx[s], seg_freqf[s], nullptr,
                           mask ? mask + (size_t)s * n_toa : nullptr);
    if (rc < 0) return rc;
    m0 += (int64_t)n_psr * nm;
    nmax = std::max<int64_t>(nmax, nm + (nm & 1));
  }
  if ((rc = layout_finalize(c, L))) return rc;
  // z [1][n_seg][n_psr][nmax][2] = (ccos, csin)
  std::vector<double> z((size_t)n_seg * n_psr * nmax * 2, 0.0);
  m0 = 0;
  for (int32_t s = 0; s < n_seg; ++s) {
    const int32_t nm = seg_nmodes[s];
    for (int32_t p = 0; p < n_psr; ++p)
      for (int32_t k = 0; k < nm; ++k) {
        const size_t dst = (((size_t)s * n_psr + p) * nmax + k) * 2;
        z[dst] = ccos[m0 + (size_t)p * nm + k];
        z[dst + 1] = csin[m0 + (size_t)p * nm + k];
      }
    m0 += (int64_t)n_psr * nm;
  }
  if ((rc = upload(c, c->zin, z.data(), sizeof(double) * z.size(), "gp_accumulate z"))) return rc;
  if ((rc = run_coefficients(c, L, 0, 0, 1, kRealPad, c->zin.as<double>(), (int32_t)nmax, nullptr))) return rc;
  if ((rc = upload(c, c->scratch_out, residuals, sizeof(double) * n_toa, "gp_accumulate residuals"))) return rc;
  if ((rc = run_synth(c, L, 1, kRealPad, c->scratch_out.as<double>(), n_toa, 1, false))) return rc;
  HIPCHK(c, hipMemcpyAsync(residuals, c->scratch_out.p, sizeof(double) * n_toa, hipMemcpyDeviceToHost, c->stream),
         "gp_accumulate download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "gp_accumulate sync");
  return FPTA_OK;
}

int fpta_common_accumulate(fpta_ctx* c, int32_t n_psr, const int64_t* offs, const double* toas, const double* nu,
                           int32_t n_modes, const double* f, const double* amp, double idx, double freqf,
                           const double* Lmat, const double* z, double* residuals, double* x_out) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (n_psr <= 0 || n_modes <= 0 || !offs || !toas || !nu || !f || !amp || !Lmat || !z || !residuals)
    return fail(c, FPTA_EINVAL, "common_accumulate: bad arguments");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  Layout& L = c->scratch;
  int rc = layout_set_toas(c, L, n_psr, offs, toas, nu);
  if (rc) return rc;
  rc = layout_add_signal(c, L, 1, n_modes, f, amp, idx, freqf, Lmat, nullptr);
  if (rc < 0) return rc;
  if ((rc = layout_finalize(c, L))) return rc;
  const int32_t nmp = L.segs[0]->d.nm;
  // reference draw order z[k][0 = sin, 1 = cos][p] -> zin[0][0][p][k][0 = cos, 1 = sin]
  std::vector<double> zz((size_t)n_psr * nmp * 2, 0.0);
  for (int32_t k = 0; k < n_modes; ++k)
    for (int32_t p = 0; p < n_psr; ++p) {
      zz[((size_t)p * nmp + k) * 2] = z[((size_t)k * 2 + 1) * n_psr + p];
      zz[((size_t)p * nmp + k) * 2 + 1] = z[((size_t)k * 2 + 0) * n_psr + p];
    }
  if ((rc = upload(c, c->zin, zz.data(), sizeof(double) * zz.size(), "common z"))) return rc;
  const int64_t M = (int64_t)2 * nmp * kRealPad;
  double* xdev = nullptr;
  if (x_out) {
    HIPCHK(c, c->xout.ensure(sizeof(double) * (size_t)n_psr * M), "x_out alloc");
    xdev = c->xout.as<double>();
  }
  if ((rc = run_coefficients(c, L, 0, 0, 1, kRealPad, c->zin.as<double>(), nmp, xdev))) return rc;
  const int64_t N = offs[n_psr];
  if ((rc = upload(c, c->scratch_out, residuals, sizeof(double) * N, "common residuals"))) return rc;
  if ((rc = run_synth(c, L, 1, kRealPad, c->scratch_out.as<double>(), N, 1, false))) return rc;
  HIPCHK(c, hipMemcpyAsync(residuals, c->scratch_out.p, sizeof(double) * N, hipMemcpyDeviceToHost, c->stream),
         "common download");
  std::vector<double> xh;
  if (x_out) {
    xh.resize((size_t)n_psr * M);
    HIPCHK(c, hipMemcpyAsync(xh.data(), xdev, sizeof(double) * xh.size(), hipMemcpyDeviceToHost, c->stream),
           "x download");
  }
  HIPCHK(c, hipStreamSynchronize(c->stream), "common sync");
  if (x_out) {  // [p][j = 2k + c][r = 0] -> x_out[k][c][p]
    for (int32_t k = 0; k < n_modes; ++k)
      for (int32_t cc = 0; cc < 2; ++cc)
        for (int32_t p = 0; p < n_psr; ++p)
          x_out[((size_t)k * 2 + cc) * n_psr + p] = xh[(size_t)p * M + (size_t)(2 * k + cc) * kRealPad];
  }
  return FPTA_OK;
}

int fpta_white_accumulate(fpta_ctx* c, int64_t n_toa, const double* sigma, const double* z, int64_t n_blocks,
                          const int64_t* block_offs, const int64_t* block_idx, const double* ecorr_sigma,
                          const double* zb, double* residuals) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (n_toa <= 0 || !sigma || !z || !residuals || n_blocks < 0 || (n_blocks > 0 && (!ecorr_sigma || !zb)))
    return fail(c, FPTA_EINVAL, "white_accumulate: bad arguments");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  std::vector<int32_t> owner;
  int rc = blocks_to_owner(c, n_toa, n_blocks, block_offs, block_idx, owner);
  if (rc) return rc;
  if ((rc = upload(c, c->scratch_sigma, sigma, sizeof(double) * n_toa, "white sigma"))) return rc;
  if ((rc = upload(c, c->scratch_z, z, sizeof(double) * n_toa, "white z"))) return rc;
  if (n_blocks > 0) {
    if ((rc = upload(c, c->scratch_block_of, owner.data(), sizeof(int32_t) * n_toa, "white owner"))) return rc;
    if ((rc = upload(c, c->scratch_esig, ecorr_sigma, sizeof(double) * n_blocks, "white esig"))) return rc;
    if ((rc = upload(c, c->scratch_zb, zb, sizeof(double) * n_blocks, "white zb"))) return rc;
  }
  if ((rc = upload(c, c->scratch_out, residuals, sizeof(double) * n_toa, "white residuals"))) return rc;
  {
    KTimer kt(c, FPTA_K_WHITE);
    HIPCHK(c,
           launch_white(c->stream, c->scratch_sigma.as<double>(),
                        n_blocks > 0 ? c->scratch_block_of.as<int32_t>() : nullptr,
                        n_blocks > 0 ? c->scratch_esig.as<double>() : nullptr, c->scratch_z.as<double>(),
                        n_blocks > 0 ? c->scratch_zb.as<double>() : nullptr, c->scratch_out.as<double>(), n_toa,
                        n_toa, 1, 0, 0, 0),
           "k_white launch");
  }
  HIPCHK(c, hipMemcpyAsync(residuals, c->scratch_out.p, sizeof(double) * n_toa, hipMemcpyDeviceToHost, c->stream),
         "white download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "white sync");
  return FPTA_OK;
}

// ------------------------------------------------------------------------------------ batch
// ----------------------------------------------------------------------------- dense covariance
int fpta_gp_covariance(fpta_ctx* c, int64_t n_toa, const double* toas, const double* nu, int32_t n_seg,
                       const int32_t* seg_nmodes, const double* f, const double* w, const double* seg_idx,
                       const double* seg_freqf, const double* white_var, double* cov) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (!cov) return fail(c, FPTA_EINVAL, "gp_covariance: null output");
  DenseDims d;
  int rc = dense_build(c, n_toa, toas, nu, n_seg, seg_nmodes, f, w, seg_idx, seg_freqf, white_var, d);
  if (rc) return rc;
  HIPCHK(c,
         hipMemcpy2DAsync(cov, sizeof(double) * n_toa, c->dn_C.p, sizeof(double) * d.n_pad, sizeof(double) * n_toa,
                          n_toa, hipMemcpyDeviceToHost, c->stream),
         "gp_covariance download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "gp_covariance sync");
  return FPTA_OK;
}

int fpta_noise_wiener(fpta_ctx* c, int64_t n_toa, const double* toas, const double* nu, int32_t n_seg,
                      const int32_t* seg_nmodes, const double* f, const double* w, const double* seg_idx,
                      const double* seg_freqf, const double* white_var, const double* residuals, double* out) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (!white_var || !residuals || !out) return fail(c, FPTA_EINVAL, "noise_wiener: bad arguments");
  DenseDims d;
  int rc = dense_build(c, n_toa, toas, nu, n_seg, seg_nmodes, f, w, seg_idx, seg_freqf, white_var, d);
  if (rc) return rc;
  if ((rc = upload(c, c->dn_r, residuals, sizeof(double) * n_toa, "noise_wiener residuals"))) return rc;
  if ((rc = dense_cholesky(c, d))) return rc;
  HIPCHK(c, c->dn_y.ensure(sizeof(double) * n_toa), "noise_wiener scratch");
  HIPCHK(c, c->dn_out.ensure(sizeof(double) * n_toa), "noise_wiener out");
  {
    KTimer kt(c, FPTA_K_DENSE);
    HIPCHK(c,
           launch_chol_solve(c->stream, c->dn_C.as<double>(), d.n_pad, n_toa, c->dn_r.as<double>(),
                             c->dn_white.as<double>(), c->dn_y.as<double>(), c->dn_out.as<double>()),
           "k_chol_solve launch");
  }
  HIPCHK(c, hipMemcpyAsync(out, c->dn_out.p, sizeof(double) * n_toa, hipMemcpyDeviceToHost, c->stream),
         "noise_wiener download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "noise_wiener sync");
  return FPTA_OK;
}

int fpta_noise_draw(fpta_ctx* c, int64_t n_toa, const double* toas, const double* nu, int32_t n_seg,
                    const int32_t* seg_nmodes, const double* f, const double* w, const double* seg_idx,
                    const double* seg_freqf, const double* white_var, uint64_t seed, int64_t real0, int32_t n_real,
                    double* out) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (!out || n_real <= 0 || real0 < 0) return fail(c, FPTA_EINVAL, "noise_draw: bad arguments");
  if (real0 + n_real > ((int64_t)1 << 33)) return fail(c, FPTA_EINVAL, "noise_draw: realization index overflow");
  DenseDims d;
  int rc = dense_build(c, n_toa, toas, nu, n_seg, seg_nmodes, f, w, seg_idx, seg_freqf, white_var, d);
  if (rc) return rc;
  if ((rc = dense_cholesky(c, d))) return rc;
  const int64_t ldz = pad_i64(n_real, 256);
  HIPCHK(c, c->dn_Z.ensure(sizeof(double) * (size_t)d.n_pad * ldz), "noise_draw normals alloc");
  HIPCHK(c, c->dn_out.ensure(sizeof(double) * (size_t)n_real * n_toa), "noise_draw out alloc");
  {
    KTimer kt(c, FPTA_K_DENSE);
    HIPCHK(c,
           launch_dense_normals(c->stream, n_toa, d.n_pad, n_real, real0, (uint32_t)(seed & 0xFFFFFFFFull),
                                (uint32_t)(seed >> 32), c->dn_Z.as<double>(), ldz),
           "k_dense_normals launch");
    // X [n_real][n_toa] = Z L^T: A = Z (k-major: ZT[t][r]), B^T = L (rows), L lower-triangular
    HIPCHK(c,
           launch_gemm_tn(c->stream, c->dn_Z.as<double>(), ldz, c->dn_C.as<double>(), d.n_pad, true, true,
                          c->dn_out.as<double>(), n_toa, n_real, n_toa, (int32_t)(d.n_pad / 4), 0, 0, 0, nullptr),
           "k_gemm_tn (draws) launch");
  }
  HIPCHK(c, hipMemcpyAsync(out, c->dn_out.p, sizeof(double) * (size_t)n_real * n_toa, hipMemcpyDeviceToHost,
                           c->stream),
         "noise_draw download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "noise_draw sync");
  return FPTA_OK;
}

int fpta_batch_set_toas(fpta_ctx* c, int32_t n_psr, const int64_t* offs, const double* toas, const double* nu) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  c->has_sigma = c->has_blocks = false;
  c->out_R = 0;
  return layout_set_toas(c, c->batch, n_psr, offs, toas, nu);
}

int fpta_batch_add_signal(fpta_ctx* c, int32_t kind, int32_t n_modes, const double* f, const double* amp,
                          double idx, double freqf, const double* Lmat, const uint8_t* mask) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  return layout_add_signal(c, c->batch, kind, n_modes, f, amp, idx, freqf, Lmat, mask);
}

int fpta_batch_clear_signals(fpta_ctx* c) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  c->batch.clear_signals();
  c->has_sigma = c->has_blocks = false;
  return FPTA_OK;
}

int fpta_batch_set_white(fpta_ctx* c, const double* sigma, int64_t n_blocks, const int64_t* block_offs,
                         const int64_t* block_idx, const double* ecorr_sigma) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (c->batch.P <= 0) return fail(c, FPTA_ESTATE, "set_white: set_toas first");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int64_t N = c->batch.n_toa;
  int rc;
  c->has_sigma = sigma != nullptr;
  if (sigma && (rc = upload(c, c->sigma, sigma, sizeof(double) * N, "set_white sigma"))) return rc;
  c->has_blocks = n_blocks > 0;
  c->n_blocks = n_blocks;
  if (n_blocks > 0) {
    if (!ecorr_sigma) return fail(c, FPTA_EINVAL, "set_white: ecorr_sigma missing");
    std::vector<int32_t> owner;
    if ((rc = blocks_to_owner(c, N, n_blocks, block_offs, block_idx, owner))) return rc;
    if ((rc = upload(c, c->block_of, owner.data(), sizeof(int32_t) * N, "set_white owner"))) return rc;
    if ((rc = upload(c, c->esig, ecorr_sigma, sizeof(double) * n_blocks, "set_white esig"))) return rc;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream), "set_white sync");
  return FPTA_OK;
}

static int batch_common(fpta_ctx* c, uint64_t seed, int64_t real0, int32_t n_real, const double* zin,
                        int32_t zin_nm, double* out, double* coeffs_out, bool white) {
  double* const coeffs_host = coeffs_out;
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  Layout& L = c->batch;
  if (L.P <= 0) return fail(c, FPTA_ESTATE, "batch_synth: set_toas first");
  if (n_real <= 0) return fail(c, FPTA_EINVAL, "batch_synth: n_real must be > 0");
  if (real0 < 0 || real0 + n_real > ((int64_t)1 << 32))
    return fail(c, FPTA_EINVAL, "batch_synth: realization index exceeds the 32-bit Philox counter word");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  int rc = layout_finalize(c, L);
  if (rc) return rc;
  const int32_t R_pad = pad_to(n_real, kRealPad);
  const size_t out_bytes = sizeof(double) * (size_t)n_real * L.n_toa;
  HIPCHK(c, c->out.ensure(out_bytes), "out alloc");
  c->out_R = n_real;
  c->out_ld = L.n_toa;
  c->part_ready = false;  // set by the gridded interpolation when it writes this block's partial checksums
  const bool do_white = white && (c->has_sigma || c->has_blocks);
  const uint32_t k0 = (uint32_t)(seed & 0xFFFFFFFFull), k1 = (uint32_t)(seed >> 32);
  WhiteCfg wc{};
  if (do_white) {
    if (n_real > 65535) return fail(c, FPTA_EINVAL, "white: n_real > 65535 per call");
    wc.on = 1;
    wc.sigma = c->has_sigma ? c->sigma.as<double>() : nullptr;
    wc.block_of = c->has_blocks ? c->block_of.as<int32_t>() : nullptr;
    wc.esig = c->has_blocks ? c->esig.as<double>() : nullptr;
    wc.nblocks = c->has_blocks ? c->n_blocks : 0;
    wc.real0 = real0;
    wc.k0 = k0;
    wc.k1 = k1;
  }
  int path = 0;
  if (!L.segs.empty() && (rc = select_path(c, L, n_real, true, &path))) return rc;
  // ECORR epoch normals of this batch as a [R][n_epochs] block, read by every white path. (Making them from their
  // Philox counters inside the gridded epilogue instead was measured 2x slower on C5: the epilogue is VALU-bound,
  // profiles/round4/R4l_c5_storer_ecorr_inline_ab.txt.)
  if (do_white && c->has_blocks) {
    HIPCHK(c, c->zb_epochs.ensure(sizeof(double) * (size_t)n_real * c->n_blocks), "zb alloc");
    wc.zb = c->zb_epochs.as<double>();
    KTimer kt(c, FPTA_K_WHITE);
    HIPCHK(c, launch_epoch_normals(c->stream, c->n_blocks, n_real, real0, k0, k1, c->zb_epochs.as<double>()),
           "k_epoch_normals launch");
  }
  bool fused = false;
  if (L.segs.empty()) {
    HIPCHK(c, hipMemsetAsync(c->out.p, 0, out_bytes, c->stream), "out memset");
  } else {
    // grid signals with a per-pulsar member draw inside their DFT (not for validation draws or coefficient downloads,
    // which need every signal's coefficients in the buffer)
    c->gen_fused = path == 4 && !zin && !coeffs_out && c->dft_gen && (c->grid_mfma & 1);
    c->blk_real0 = real0;
    c->blk_k0 = k0;
    c->blk_k1 = k1;
    bool coef_done = false;
    // pipelined gridded block: draws, merges and DFT on the side stream, overlapping the previous block's
    // interpolation (not for zin blocks: their draws read an upload queued on the ctx stream)
    const bool pipe = c->overlap != 0 && path == 4 && !zin;
    if ((rc = run_coefficients(c, L, seed, real0, n_real, R_pad, zin, zin_nm, nullptr, c->overlap != 0, path == 4,
                               coeffs_out, &coef_done, pipe)))
      return rc;
    if (coef_done) coeffs_out = nullptr;  // downloaded before the coalesced grid signals were merged
    c->coef_copy_pending = coeffs_out != nullptr;
    if ((rc = run_synth(c, L, n_real, R_pad, c->out.as<double>(), L.n_toa, 0, true, do_white ? &wc : nullptr,
                        &fused, path, pipe)))
      return rc;
  }
  if (do_white && !fused) {
    c->part_ready = false;  // the separate pass changes the block after the partials were taken
    KTimer kt(c, FPTA_K_WHITE);
    HIPCHK(c,
           launch_white_pairs(c->stream, wc.sigma, wc.block_of, wc.esig, wc.nblocks, wc.zb, c->out.as<double>(),
                              L.n_toa, L.n_toa, n_real, real0, k0, k1),
           "k_white_pairs launch");
  }
  c->gen_fused = false;
  if (out) HIPCHK(c, hipMemcpyAsync(out, c->out.p, out_bytes, hipMemcpyDeviceToHost, c->stream), "out download");
  if (coeffs_out && L.K > 0) {
    // [P][K][R_pad] -> [P][K][n_real]
    HIPCHK(c,
           hipMemcpy2DAsync(coeffs_out, sizeof(double) * n_real, c->coef.p, sizeof(double) * R_pad,
                            sizeof(double) * n_real, (size_t)L.P * L.K, hipMemcpyDeviceToHost, c->stream),
           "coef download");
  }
  if (out || coeffs_out || coeffs_host) HIPCHK(c, hipStreamSynchronize(c->stream), "batch sync");
  return FPTA_OK;
}

int fpta_batch_synth(fpta_ctx* c, uint64_t seed, int64_t real0, int32_t n_real, double* out, double* coeffs_out) {
  return batch_common(c, seed, real0, n_real, nullptr, 0, out, coeffs_out, true);
}

int fpta_batch_synth_from_z(fpta_ctx* c, int32_t n_real, int32_t n_modes_max, const double* z, double* out) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (!z || n_modes_max <= 0 || n_real <= 0) return fail(c, FPTA_EINVAL, "synth_from_z: bad arguments");
  for (Seg* s : c->batch.segs)
    if (s->nm_orig > n_modes_max) return fail(c, FPTA_EINVAL, "synth_from_z: n_modes_max too small");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const size_t bytes = sizeof(double) * (size_t)n_real * c->batch.segs.size() * c->batch.P * n_modes_max * 2;
  int rc = upload(c, c->zin, z, bytes, "synth_from_z z");
  if (rc) return rc;
  return batch_common(c, 0, 0, n_real, c->zin.as<double>(), n_modes_max, out, nullptr, false);
}

int fpta_batch_download(fpta_ctx* c, int32_t r_begin, int32_t r_count, double* host) {
  if (!c || !host) return fail(c, FPTA_EINVAL, "download: bad arguments");
  if (!c->out_R) return fail(c, FPTA_ESTATE, "download: nothing synthesized yet");
  if (r_begin < 0 || r_count <= 0 || r_begin + r_count > c->out_R)
    return fail(c, FPTA_EINVAL, "download: realization range outside the last block");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const size_t row = sizeof(double) * (size_t)c->out_ld;
  HIPCHK(c,
         hipMemcpyAsync(host, c->out.as<char>() + row * r_begin, row * r_count, hipMemcpyDeviceToHost,
                        c->stream),
         "download copy");
  HIPCHK(c, hipStreamSynchronize(c->stream), "download sync");
  return FPTA_OK;
}

int fpta_batch_device_out(fpta_ctx* c, double** dptr, int64_t* ld, int32_t* n_real) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (!c->out_R) return fail(c, FPTA_ESTATE, "device_out: nothing synthesized yet");
  if (dptr) *dptr = c->out.as<double>();
  if (ld) *ld = c->out_ld;
  if (n_real) *n_real = c->out_R;
  return FPTA_OK;
}

// Per-realization {sum, sum of squares} of the context's last block into c->sums (device): from the interpolation's
// partial checksums when it wrote them for this block, else one pass over the block. On the ctx stream, or (async,
// streamed jobs with partials) on the red stream beside the next block's work; *used: the stream the sums are on.
// With dst (device or pinned host memory), sums from the partials are written there directly (*direct = true)
// instead of into c->sums.
static int launch_block_checksums(fpta_ctx* c, bool async = false, hipStream_t* used = nullptr, double* dst = nullptr,
                                  bool* direct = nullptr) {
  if (direct) *direct = false;
  hipStream_t st = c->stream;
  if (async && c->part_ready) {
    if (!c->red) HIPCHK(c, hipStreamCreateWithFlags(&c->red, hipStreamNonBlocking), "red stream create");
    for (hipEvent_t* e : {&c->ev_pready, &c->ev_pfree[0], &c->ev_pfree[1]})
      if (!*e) HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableTiming), "event create");
    HIPCHK(c, hipEventRecord(c->ev_pready, c->stream), "event record");
    HIPCHK(c, hipStreamWaitEvent(c->red, c->ev_pready, 0), "partials ready wait");
    st = c->red;
    c->red_pending = true;
  } else {
    int rc = join_red(c);  // sums / part_tmp / partials may still be in use there
    if (rc) return rc;
  }
  if (used) *used = st;
  if (c->part_ready && dst) {
    if (direct) *direct = true;
  } else if (c->sums.cap < sizeof(double) * 2 * c->out_R) {
    HIPCHK(c, hipStreamSynchronize(st), "sums regrow sync");
    HIPCHK(c, c->sums.ensure(sizeof(double) * 2 * c->out_R), "sums alloc");
  }
  if (c->part_ready) {
    const size_t tb = sizeof(double) * 2 * (size_t)kPartSegs * c->part_rpad;
    if (c->part_tmp.cap < tb) {
      HIPCHK(c, hipStreamSynchronize(st), "partials scratch regrow sync");
      HIPCHK(c, c->part_tmp.ensure(tb), "partials scratch alloc");
    }
    HIPCHK(c,
           launch_part_checksums(st, c->part[c->part_cur].as<double>(), c->part_chunks, c->part_rpad, c->out_R,
                                 c->part_tmp.as<double>(), dst ? dst : c->sums.as<double>()),
           "k_part_reduce launch");
    if (st == c->red) {
      HIPCHK(c, hipEventRecord(c->ev_pfree[c->part_cur], c->red), "event record");
      c->pfree_set[c->part_cur] = true;
    }
  } else {
    HIPCHK(c, launch_checksums(c->stream, c->out.as<double>(), c->out_ld, c->out_ld, c->out_R, c->sums.as<double>()),
           "k_checksums launch");
  }
  return FPTA_OK;
}

int fpta_batch_checksums(fpta_ctx* c, double* sums) {
  if (!c || !sums) return fail(c, FPTA_EINVAL, "checksums: bad arguments");
  if (!c->out_R) return fail(c, FPTA_ESTATE, "checksums: nothing synthesized yet");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  int rc = launch_block_checksums(c);
  if (rc) return rc;
  HIPCHK(c, hipMemcpyAsync(sums, c->sums.p, sizeof(double) * 2 * c->out_R, hipMemcpyDeviceToHost, c->stream),
         "sums download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "checksums sync");
  return FPTA_OK;
}

int fpta_batch_correlations(fpta_ctx* c, int32_t mode, double* out) {
  if (!c || !out || mode < 0 || mode > 3) return fail(c, FPTA_EINVAL, "correlations: bad arguments");
  if (!c->out_R) return fail(c, FPTA_ESTATE, "correlations: nothing synthesized yet");
  const Layout& L = c->batch;
  const int32_t P = L.P;
  const int64_t n = L.h_offs[1] - L.h_offs[0];
  for (int32_t p = 0; p < P; ++p)
    if (L.h_offs[p + 1] - L.h_offs[p] != n)
      return fail(c, FPTA_EINVAL, "correlations: every pulsar must have the same number of TOAs");
  if (n > 0x7FFFFFFF || c->out_R > 65535) return fail(c, FPTA_EINVAL, "correlations: block too large");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int32_t R = c->out_R;
  const int32_t nparts = std::min<int32_t>(R, 256);
  const size_t pp = (size_t)P * P;
  size_t dst_len = mode == 0 ? (size_t)R * pp : mode == 3 ? (size_t)R * P : pp;
  HIPCHK(c, c->corr_autos.ensure(sizeof(double) * (size_t)R * P), "autos alloc");
  HIPCHK(c, c->corr_parts.ensure(sizeof(double) * (size_t)nparts * pp), "parts alloc");
  HIPCHK(c, c->corr_dst.ensure(sizeof(double) * dst_len), "corr alloc");
  double* dst = mode == 3 ? c->corr_autos.as<double>() : c->corr_dst.as<double>();
  HIPCHK(c,
         launch_correlations(c->stream, c->out.as<double>(), c->out_ld, (int32_t)n, P, R, mode,
                             c->corr_autos.as<double>(), c->corr_parts.as<double>(), nparts, dst),
         "k_xcorr launch");
  HIPCHK(c, hipMemcpyAsync(out, dst, sizeof(double) * dst_len, hipMemcpyDeviceToHost, c->stream), "corr download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "corr sync");
  return FPTA_OK;
}

int fpta_batch_info(fpta_ctx* c, int64_t* info) {
  if (!c || !info) return fail(c, FPTA_EINVAL, "info: bad arguments");
  info[0] = c->batch.P;
  info[1] = c->batch.n_toa;
  info[2] = (int64_t)c->batch.segs.size();
  info[3] = c->batch.K;
  info[4] = c->batch.max_np;
  return FPTA_OK;
}

int fpta_batch_grid_info_n(fpta_ctx* c, double* dst, int32_t n_out) {
  if (!c || !dst || n_out < 0) return fail(c, FPTA_EINVAL, "grid_info: bad arguments");
  const GridPlan& G = c->batch.grid;
  const bool ok = G.built && G.ok;
  double out[FPTA_GRID_INFO_LEN];
  out[0] = c->last_path;
  out[1] = ok ? 1.0 : 0.0;
  out[2] = ok ? G.n_chunks : 0.0;
  out[3] = ok ? G.fma_dft : 0.0;
  out[4] = ok ? G.fma_interp : 0.0;
  out[5] = ok ? G.fma_direct : 0.0;
  out[6] = ok ? G.grid_vals : 0.0;
  out[7] = ok ? G.weight_bytes : 0.0;
  out[8] = c->grid_mfma;
  out[9] = std::exp(-M_PI * c->grid_w * std::sqrt(1.0 - 100.0 / c->grid_sigma100));
  out[10] = c->grid_w;
  out[11] = c->grid_sigma100 / 100.0;
  out[12] = ok ? (double)G.segs.size() : 0.0;
  out[13] = (double)c->batch.segs.size();
  out[14] = ok ? G.mean_v : 0.0;
  out[15] = c->last_interp;
  std::memcpy(dst, out, sizeof(double) * std::min<int32_t>(n_out, FPTA_GRID_INFO_LEN));
  return FPTA_GRID_INFO_LEN;
}

// the round-1 contract: 9 values (a caller's double[9] stays in bounds)
int fpta_batch_grid_info(fpta_ctx* c, double* out) {
  const int rc = fpta_batch_grid_info_n(c, out, 9);
  return rc < 0 ? rc : FPTA_OK;
}

const char* fpta_batch_path_reason(const fpta_ctx* c) { return c ? c->path_reason.c_str() : ""; }

#ifdef FPTA_FUSED_PROF
// k_grid_fused's per-wave cycle counters of the last fused block ([4096 workgroups][8 waves][8]; -DFPTA_FUSED_PROF
// variant builds only, tools/fused_prof.py)
extern "C" int fpta_debug_fused_prof(fpta_ctx* c, unsigned long long* host, int64_t n) {
  if (!c || !host || n <= 0 || !c->dbg_a.p || (size_t)n * 8 > c->dbg_a.cap) return FPTA_EINVAL;
  HIPCHK(c, hipMemcpy(host, c->dbg_a.p, (size_t)n * 8, hipMemcpyDeviceToHost), "profile download");
  return FPTA_OK;
}
#endif

int fpta_debug_fill_out(fpta_ctx* c, double value) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (!c->out_R) return fail(c, FPTA_ESTATE, "fill_out: nothing synthesized yet");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const size_t n = (size_t)c->out_R * c->out_ld;
  std::vector<double> v(std::min<size_t>(n, (size_t)1 << 20), value);
  for (size_t i = 0; i < n; i += v.size())
    HIPCHK(c,
           hipMemcpyAsync(c->out.as<double>() + i, v.data(), sizeof(double) * std::min(v.size(), n - i),
                          hipMemcpyHostToDevice, c->stream),
           "fill_out copy");
  HIPCHK(c, hipStreamSynchronize(c->stream), "fill_out sync");
  return FPTA_OK;
}

int fpta_debug_philox(fpta_ctx* c, int64_t n, const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  if (!c || n <= 0 || !ctr || !key || !out) return fail(c, FPTA_EINVAL, "debug_philox: bad arguments");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  int rc = upload(c, c->dbg_a, ctr, sizeof(uint32_t) * 4 * n, "philox ctr");
  if (rc) return rc;
  HIPCHK(c, c->dbg_b.ensure(sizeof(uint32_t) * 4 * n), "philox out");
  HIPCHK(c, launch_philox(c->stream, n, c->dbg_a.as<uint32_t>(), key[0], key[1], c->dbg_b.as<uint32_t>()),
         "k_philox launch");
  HIPCHK(c, hipMemcpyAsync(out, c->dbg_b.p, sizeof(uint32_t) * 4 * n, hipMemcpyDeviceToHost, c->stream),
         "philox download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "philox sync");
  return FPTA_OK;
}

int fpta_debug_normals(fpta_ctx* c, int64_t n, const uint32_t* words, double* out) {
  if (!c || n <= 0 || !words || !out) return fail(c, FPTA_EINVAL, "debug_normals: bad arguments");
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  int rc = upload(c, c->dbg_a, words, sizeof(uint32_t) * 4 * n, "normals words");
  if (rc) return rc;
  HIPCHK(c, c->dbg_b.ensure(sizeof(double) * 4 * n), "normals out");
  HIPCHK(c, launch_normals4(c->stream, n, c->dbg_a.as<uint32_t>(), c->dbg_b.as<double>()), "k_normals4 launch");
  HIPCHK(c, hipMemcpyAsync(out, c->dbg_b.p, sizeof(double) * 4 * n, hipMemcpyDeviceToHost, c->stream),
         "normals download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "normals sync");
  return FPTA_OK;
}


// ------------------------------------------------------------------------------------ multi-device
// One process driving several devices (SURVEY.md §8(b) fpta_multi_*, §8(e)): one context per listed
// device, the layout replicated on each, realizations sharded contiguously (device g of G owns
// [real0 + g n / G, real0 + (g + 1) n / G)) and streamed in batches. Only per-realization checksums
// leave the devices (async D2H into pinned host memory); the residual blocks stay resident. The work
// of all devices is issued round-robin from this thread on their own streams, so the devices run
// concurrently. Output is invariant to the device count and the batch size (Philox counters carry the
// global realization index). Processes that own one GPU each use fakepta_amd.batch.simulate_sharded
// (torch.distributed / RCCL) instead.
struct fpta_multi {
  std::vector<fpta_ctx*> ctx;
  std::string err;
  // checksum gather (fpta_multi_set_gather): FPTA_GATHER_AUTO = RCCL when the devices are distinct, else pinned host
  // staging; FPTA_GATHER_RCCL; FPTA_GATHER_HOST. comm: one RCCL communicator per device (ncclCommInitAll, made on
  // the first RCCL gather); shard: each device's checksums of its shard, gathered to device 0's root buffer
  int gather = FPTA_GATHER_AUTO;
  int last_gather = 0;
  std::vector<ncclComm_t> comm;
  std::vector<DevBuf*> shard;
  DevBuf root;
  ~fpta_multi() {
    for (size_t g = 0; g < comm.size(); ++g)
      if (comm[g]) (void)ncclCommDestroy(comm[g]);
    for (size_t g = 0; g < shard.size(); ++g) {
      if (g < ctx.size() && ctx[g]) (void)hipSetDevice(ctx[g]->device);
      delete shard[g];
    }
    if (!ctx.empty() && ctx[0]) (void)hipSetDevice(ctx[0]->device);
    root.release();
  }
};

// One process per GPU (fakepta_amd.batch.RcclComm): an RCCL communicator on a context's device and stream.
struct fpta_comm {
  ncclComm_t comm = nullptr;
  fpta_ctx* ctx = nullptr;
  int32_t nranks = 0, rank = 0;
  DevBuf send, recv;
  std::string err;
};

namespace {
int multi_fail(fpta_multi* m, int i, int rc) {
  if (m) m->err = "device context " + std::to_string(i) + ": " + fpta_last_error(m->ctx[i]);
  g_err = m ? m->err : g_err;
  return rc;
}

// checksums of the context's last block -> dst [n_real][2] (pinned host, or device with d2d), asynchronously: on the
// red stream beside the next block when the interpolation wrote partials, else on the ctx stream.
int checksums_async(fpta_ctx* c, double* dst, bool d2d = false) {
  hipStream_t st = nullptr;
  bool direct = false;
  int rc = launch_block_checksums(c, c->async_sums != 0, &st, dst, &direct);
  if (rc) return rc;
  if (direct) return FPTA_OK;  // the reduction wrote dst
  HIPCHK(c,
         hipMemcpyAsync(dst, c->sums.p, sizeof(double) * 2 * c->out_R,
                        d2d ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, st),
         "sums copy");
  return FPTA_OK;
}
}  // namespace

int fpta_multi_create(int32_t n_dev, const int32_t* devices, fpta_multi** out) {
  if (!out || n_dev <= 0 || !devices) return fail(nullptr, FPTA_EINVAL, "multi_create: bad arguments");
  *out = nullptr;
  fpta_multi* m = new fpta_multi();
  for (int32_t i = 0; i < n_dev; ++i) {
    fpta_ctx* c = nullptr;
    int rc = fpta_create(devices[i], &c);
    if (rc) {
      std::string msg = "multi_create: device " + std::to_string(devices[i]) + ": " + g_err;
      fpta_multi_destroy(m);
      return fail(nullptr, rc, msg);
    }
    m->ctx.push_back(c);
  }
  *out = m;
  return FPTA_OK;
}

int fpta_multi_destroy(fpta_multi* m) {
  if (!m) return FPTA_OK;
  std::vector<fpta_ctx*> ctx = m->ctx;
  delete m;  // communicators and device buffers first, then the contexts they were made on
  for (fpta_ctx* c : ctx) fpta_destroy(c);
  return FPTA_OK;
}

const char* fpta_multi_last_error(const fpta_multi* m) { return m ? m->err.c_str() : g_err.c_str(); }

int fpta_multi_size(const fpta_multi* m) { return m ? (int)m->ctx.size() : 0; }

fpta_ctx* fpta_multi_context(fpta_multi* m, int32_t i) {
  return (m && i >= 0 && i < (int32_t)m->ctx.size()) ? m->ctx[i] : nullptr;
}

int fpta_multi_set_toas(fpta_multi* m, int32_t n_psr, const int64_t* offs, const double* toas, const double* nu) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null multi");
  for (size_t i = 0; i < m->ctx.size(); ++i) {
    int rc = fpta_batch_set_toas(m->ctx[i], n_psr, offs, toas, nu);
    if (rc) return multi_fail(m, (int)i, rc);
  }
  return FPTA_OK;
}

int fpta_multi_add_signal(fpta_multi* m, int32_t kind, int32_t n_modes, const double* f, const double* amp,
                          double idx, double freqf, const double* Lmat, const uint8_t* mask) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null multi");
  int id = -1;
  for (size_t i = 0; i < m->ctx.size(); ++i) {
    int rc = fpta_batch_add_signal(m->ctx[i], kind, n_modes, f, amp, idx, freqf, Lmat, mask);
    if (rc < 0) return multi_fail(m, (int)i, rc);
    id = rc;
  }
  return id;
}

int fpta_multi_set_white(fpta_multi* m, const double* sigma, int64_t n_blocks, const int64_t* block_offs,
                         const int64_t* block_idx, const double* ecorr_sigma) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null multi");
  for (size_t i = 0; i < m->ctx.size(); ++i) {
    int rc = fpta_batch_set_white(m->ctx[i], sigma, n_blocks, block_offs, block_idx, ecorr_sigma);
    if (rc) return multi_fail(m, (int)i, rc);
  }
  return FPTA_OK;
}

int fpta_multi_set_option(fpta_multi* m, int32_t key, int64_t value) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null multi");
  for (size_t i = 0; i < m->ctx.size(); ++i) {
    int rc = fpta_set_option(m->ctx[i], key, value);
    if (rc) return multi_fail(m, (int)i, rc);
  }
  return FPTA_OK;
}

int fpta_multi_set_gather(fpta_multi* m, int32_t mode) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null multi");
  if (mode < FPTA_GATHER_AUTO || mode > FPTA_GATHER_HOST) {
    m->err = "multi_set_gather: mode must be FPTA_GATHER_AUTO, _RCCL or _HOST";
    return fail(nullptr, FPTA_EINVAL, m->err);
  }
  m->gather = mode;
  return FPTA_OK;
}

int fpta_multi_last_gather(const fpta_multi* m) { return m ? m->last_gather : 0; }

namespace {
int rccl_fail(std::string* err, ncclResult_t r, const char* what) {
  std::string msg = std::string(what) + ": " + ncclGetErrorString(r);
  if (err) *err = msg;
  return fail(nullptr, FPTA_EDEVICE, msg);
}

// ncclCommInitAll over m's devices (once)
int multi_rccl_init(fpta_multi* m) {
  if (!m->comm.empty()) return FPTA_OK;
  const int G = (int)m->ctx.size();
  std::vector<int> devs(G);
  for (int g = 0; g < G; ++g) devs[g] = m->ctx[g]->device;
  std::vector<ncclComm_t> comm(G, nullptr);
  ncclResult_t r = ncclCommInitAll(comm.data(), G, devs.data());
  if (r != ncclSuccess) return rccl_fail(&m->err, r, "multi_synth: ncclCommInitAll");
  m->comm = comm;
  return FPTA_OK;
}
}  // namespace

// Realizations real0 .. real0 + n_real - 1 split over m's contexts (context g: [g n / G, (g + 1) n / G)),
// streamed in batches of <= `batch` round-robin over the devices. Per-realization checksums (from the gridded
// interpolation's partial sums where it runs) either stay on each device and are gathered to device 0 by one
// ncclGather over xGMI at the end (RCCL mode), or are copied asynchronously into pinned host staging (host mode);
// one sync per device at the end either way: no host round trip between batches.
static int stream_checksums(fpta_multi* m, uint64_t seed, int64_t real0, int64_t n_real, int32_t batch,
                            double* checksums_out) {
  const int64_t G = (int64_t)m->ctx.size();
  std::vector<int64_t> beg(G + 1);
  for (int64_t g = 0; g <= G; ++g) beg[g] = g * n_real / G;
  int64_t n_max = 0;
  for (int64_t g = 0; g < G; ++g) n_max = std::max(n_max, beg[g + 1] - beg[g]);
  bool distinct = true;
  for (int64_t g = 0; g < G; ++g)
    for (int64_t h = 0; h < g; ++h) distinct = distinct && m->ctx[g]->device != m->ctx[h]->device;
  const bool use_rccl = m->gather == FPTA_GATHER_RCCL || (m->gather == FPTA_GATHER_AUTO && distinct);
  if (use_rccl && !distinct) {
    m->err = "multi_synth: the RCCL gather needs distinct devices (one communicator rank per device)";
    return fail(nullptr, FPTA_EINVAL, m->err);
  }
  if (use_rccl && n_max > ((int64_t)1 << 40) / (2 * G)) {
    m->err = "multi_synth: job too large for one gather";
    return fail(nullptr, FPTA_EINVAL, m->err);
  }
  int rc = use_rccl ? multi_rccl_init(m) : FPTA_OK;
  if (rc) return rc;
  m->last_gather = use_rccl ? FPTA_GATHER_RCCL : FPTA_GATHER_HOST;
  // RCCL: each device's shard of checksums [n_max][2] on the device, the gather target [G][n_max][2] on device 0,
  // and one pinned buffer for the root's download. Host: pinned staging for each device's shard
  std::vector<double*> stage(G, nullptr);
  double* root_host = nullptr;
  if (use_rccl) {
    while (m->shard.size() < (size_t)G) m->shard.push_back(new DevBuf());
    for (int64_t g = 0; g < G && !rc; ++g) {
      fpta_ctx* c = m->ctx[g];
      hipError_t e = hipSetDevice(c->device);
      if (e == hipSuccess) e = m->shard[g]->ensure(sizeof(double) * 2 * (size_t)n_max);
      if (e == hipSuccess && g == 0) e = m->root.ensure(sizeof(double) * 2 * (size_t)n_max * G);
      if (e == hipSuccess && g == 0)
        e = hipHostMalloc((void**)&root_host, sizeof(double) * 2 * (size_t)n_max * G, hipHostMallocDefault);
      if (e != hipSuccess) rc = multi_fail(m, (int)g, hip_fail(c, e, "multi_synth gather buffers"));
    }
  } else {
    for (int64_t g = 0; g < G && !rc; ++g) {
      const int64_t n = beg[g + 1] - beg[g];
      if (n == 0) continue;
      fpta_ctx* c = m->ctx[g];
      hipError_t e = hipSetDevice(c->device);
      // coherent: the partial-checksum reduction writes its sums here directly from the device (checksums_async)
      if (e == hipSuccess) e = hipHostMalloc((void**)&stage[g], sizeof(double) * 2 * n, hipHostMallocCoherent);
      if (e != hipSuccess) rc = multi_fail(m, (int)g, hip_fail(c, e, "multi_synth staging"));
    }
  }
  // a checksums-only job: the gridded interpolation writes partial checksums (no second pass over each block).
  // The path is chosen once for the job, not per batch: a tail batch below FPTA_OPT_MFMA_MIN_REAL would otherwise
  // take the direct path and its realizations (and checksums) would depend on the batch split and device count
  std::vector<int> fuse(G), min_real(G);
  for (int64_t g = 0; g < G; ++g) {
    fuse[g] = m->ctx[g]->fuse_sums;
    m->ctx[g]->fuse_sums = 1;
    min_real[g] = m->ctx[g]->mfma_min_real;
    m->ctx[g]->mfma_min_real = 1;
  }
  // round-robin: batch k of every device, then batch k + 1 (each device's stream orders its own work)
  for (int64_t k = 0; !rc; ++k) {
    bool any = false;
    for (int64_t g = 0; g < G && !rc; ++g) {
      const int64_t first = beg[g] + k * (int64_t)batch;
      if (first >= beg[g + 1]) continue;
      any = true;
      const int32_t n = (int32_t)std::min<int64_t>(batch, beg[g + 1] - first);
      fpta_ctx* c = m->ctx[g];
      if ((rc = batch_common(c, seed, real0 + first, n, nullptr, 0, nullptr, nullptr, true)))
        rc = multi_fail(m, (int)g, rc);
      else if (use_rccl) {
        if ((rc = checksums_async(c, m->shard[g]->as<double>() + 2 * (first - beg[g]), true)))
          rc = multi_fail(m, (int)g, rc);
      } else if ((rc = checksums_async(c, stage[g] + 2 * (first - beg[g])))) {
        rc = multi_fail(m, (int)g, rc);
      }
    }
    if (!any) break;
  }
  for (int64_t g = 0; g < G && !rc; ++g) {  // the reductions and copies on each device's red stream come first
    fpta_ctx* c = m->ctx[g];
    (void)hipSetDevice(c->device);
    if ((rc = join_red(c))) rc = multi_fail(m, (int)g, rc);
  }
  if (use_rccl && !rc) {
    // every device's shard to device 0 in one collective (pad rows beyond a shard's count are dropped below)
    ncclResult_t r = ncclGroupStart();
    for (int64_t g = 0; g < G && r == ncclSuccess; ++g) {
      (void)hipSetDevice(m->ctx[g]->device);
      r = ncclGather(m->shard[g]->p, g == 0 ? m->root.p : nullptr, 2 * (size_t)n_max, ncclFloat64, 0, m->comm[g],
                     m->ctx[g]->stream);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) {
      rccl_fail(&m->err, r, "multi_synth: ncclGather");
      rc = FPTA_EDEVICE;
    } else {
      fpta_ctx* c0 = m->ctx[0];
      (void)hipSetDevice(c0->device);
      hipError_t e = hipMemcpyAsync(root_host, m->root.p, sizeof(double) * 2 * (size_t)n_max * G,
                                    hipMemcpyDeviceToHost, c0->stream);
      if (e != hipSuccess) rc = multi_fail(m, 0, hip_fail(c0, e, "multi_synth root download"));
    }
  }
  for (int64_t g = 0; g < G; ++g) {
    if (!use_rccl && !stage[g]) continue;
    fpta_ctx* c = m->ctx[g];
    (void)hipSetDevice(c->device);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (!rc && e != hipSuccess) rc = multi_fail(m, (int)g, hip_fail(c, e, "multi_synth sync"));
    if (!use_rccl) {
      if (!rc) std::memcpy(checksums_out + 2 * beg[g], stage[g], sizeof(double) * 2 * (beg[g + 1] - beg[g]));
      (void)hipHostFree(stage[g]);
    }
  }
  if (use_rccl) {
    if (!rc)
      for (int64_t g = 0; g < G; ++g)
        std::memcpy(checksums_out + 2 * beg[g], root_host + 2 * (size_t)n_max * g,
                    sizeof(double) * 2 * (beg[g + 1] - beg[g]));
    if (root_host) {
      (void)hipSetDevice(m->ctx[0]->device);
      (void)hipHostFree(root_host);
    }
  }
  for (int64_t g = 0; g < G; ++g) {
    m->ctx[g]->fuse_sums = fuse[g];
    m->ctx[g]->mfma_min_real = min_real[g];
  }
  return rc;
}

int fpta_multi_synth(fpta_multi* m, uint64_t seed, int64_t real0, int64_t n_real, int32_t batch,
                     double* checksums_out) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null multi");
  if (n_real <= 0 || real0 < 0 || batch <= 0 || !checksums_out) {
    m->err = "multi_synth: bad arguments";
    return fail(nullptr, FPTA_EINVAL, m->err);
  }
  if (real0 + n_real > ((int64_t)1 << 32)) {
    m->err = "multi_synth: realization index exceeds the 32-bit Philox counter word";
    return fail(nullptr, FPTA_EINVAL, m->err);
  }
  return stream_checksums(m, seed, real0, n_real, batch, checksums_out);
}

// ----------------------------------------------------------------------------- one process per GPU: RCCL
int fpta_comm_unique_id(void* id) {
  if (!id) return fail(nullptr, FPTA_EINVAL, "comm_unique_id: null buffer");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return rccl_fail(nullptr, r, "ncclGetUniqueId");
  std::memcpy(id, u.internal, FPTA_COMM_ID_BYTES);
  return FPTA_OK;
}

int fpta_comm_init_rank(fpta_ctx* c, int32_t nranks, int32_t rank, const void* id, fpta_comm** out) {
  if (!c || !id || !out || nranks <= 0 || rank < 0 || rank >= nranks)
    return fail(c, FPTA_EINVAL, "comm_init_rank: bad arguments");
  *out = nullptr;
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  ncclUniqueId u;
  std::memcpy(u.internal, id, FPTA_COMM_ID_BYTES);
  ncclComm_t comm = nullptr;
  ncclResult_t r = ncclCommInitRank(&comm, nranks, u, rank);
  if (r != ncclSuccess) {
    rccl_fail(&c->err, r, "ncclCommInitRank");
    return FPTA_EDEVICE;
  }
  fpta_comm* m = new fpta_comm();
  m->comm = comm;
  m->ctx = c;
  m->nranks = nranks;
  m->rank = rank;
  *out = m;
  return FPTA_OK;
}

int fpta_comm_destroy(fpta_comm* m) {
  if (!m) return FPTA_OK;
  (void)hipSetDevice(m->ctx->device);
  if (m->comm) (void)ncclCommDestroy(m->comm);
  delete m;
  return FPTA_OK;
}

const char* fpta_comm_last_error(const fpta_comm* m) { return m ? m->err.c_str() : g_err.c_str(); }

int fpta_comm_size(const fpta_comm* m, int32_t* nranks, int32_t* rank) {
  if (!m) return fail(nullptr, FPTA_EINVAL, "null comm");
  if (nranks) *nranks = m->nranks;
  if (rank) *rank = m->rank;
  return FPTA_OK;
}

// max over ranks of *value (host), on the context's stream after all its queued work: also the job barrier
int fpta_comm_max(fpta_comm* m, double* value) {
  if (!m || !value) return fail(nullptr, FPTA_EINVAL, "comm_max: bad arguments");
  fpta_ctx* c = m->ctx;
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(c, m->send.ensure(sizeof(double)), "comm_max buffer");
  HIPCHK(c, hipMemcpyAsync(m->send.p, value, sizeof(double), hipMemcpyHostToDevice, c->stream), "comm_max upload");
  ncclResult_t r = ncclAllReduce(m->send.p, m->send.p, 1, ncclFloat64, ncclMax, m->comm, c->stream);
  if (r != ncclSuccess) return rccl_fail(&m->err, r, "ncclAllReduce");
  HIPCHK(c, hipMemcpyAsync(value, m->send.p, sizeof(double), hipMemcpyDeviceToHost, c->stream), "comm_max download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "comm_max sync");
  return FPTA_OK;
}

// every rank sends `count` doubles (host); rank 0 receives nranks * count in rank order into recv (host; ignored
// on the other ranks)
int fpta_comm_gather(fpta_comm* m, const double* send, int64_t count, double* recv) {
  if (!m || count < 0 || (count && !send) || (m->rank == 0 && count && !recv))
    return fail(nullptr, FPTA_EINVAL, "comm_gather: bad arguments");
  fpta_ctx* c = m->ctx;
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const size_t bytes = sizeof(double) * (size_t)std::max<int64_t>(count, 1);
  HIPCHK(c, m->send.ensure(bytes), "comm_gather buffer");
  if (m->rank == 0) HIPCHK(c, m->recv.ensure(bytes * m->nranks), "comm_gather buffer");
  if (count)
    HIPCHK(c, hipMemcpyAsync(m->send.p, send, sizeof(double) * count, hipMemcpyHostToDevice, c->stream),
           "comm_gather upload");
  ncclResult_t r = ncclGather(m->send.p, m->rank == 0 ? m->recv.p : nullptr, (size_t)count, ncclFloat64, 0, m->comm,
                              c->stream);
  if (r != ncclSuccess) return rccl_fail(&m->err, r, "ncclGather");
  if (m->rank == 0 && count)
    HIPCHK(c,
           hipMemcpyAsync(recv, m->recv.p, sizeof(double) * count * m->nranks, hipMemcpyDeviceToHost, c->stream),
           "comm_gather download");
  HIPCHK(c, hipStreamSynchronize(c->stream), "comm_gather sync");
  return FPTA_OK;
}

int fpta_batch_synth_checksums(fpta_ctx* c, uint64_t seed, int64_t real0, int64_t n_real, int32_t batch,
                               double* sums) {
  if (!c) return fail(nullptr, FPTA_EINVAL, "null ctx");
  if (n_real <= 0 || real0 < 0 || batch <= 0 || !sums)
    return fail(c, FPTA_EINVAL, "batch_synth_checksums: bad arguments");
  if (real0 + n_real > ((int64_t)1 << 32))
    return fail(c, FPTA_EINVAL, "batch_synth_checksums: realization index exceeds the 32-bit Philox counter word");
  fpta_multi one;
  one.ctx.push_back(c);
  one.gather = FPTA_GATHER_HOST;  // one device: nothing to gather
  const int rc = stream_checksums(&one, seed, real0, n_real, batch, sums);  // a failing step set c's last error
  one.ctx.clear();  // the context is the caller's
  return rc;
}

}  // extern "C"
