// C-ABI of libfakepta_amd.so (declared in include/fakepta_amd.h): contexts and options, the drop-in entry points, the
// batch entry points and path selection, dense covariance. The gridded plan is grid_host.hip, several devices and RCCL
// ranks multi.hip; host-side orchestration only (argument checking, device buffers, layout tables, kernel dispatch on
// the context's stream, HIP-event timing).
#include "capi_host.h"

namespace __attribute__((visibility("hidden"))) capi {  // library-internal: not exported

thread_local std::string g_err;


int fail(fpta_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  g_err = msg;
  return code;
}

int hip_fail(fpta_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(c, e == hipErrorOutOfMemory ? FPTA_ENOMEM : FPTA_EDEVICE, m);
}

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
  ++L.version;
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

// The gridded plan of L runs white / ECORR blocks (and plain blocks k_grid_fused does not take: three grid signals)
// on k_grid_fused_w: its 16-realization grids and draw ring fit in LDS (GridPlan::fused_w_ok).
bool fused_w_layout(const fpta_ctx* c, const Layout& L) {
  const GridPlan& G = L.grid;
  return c->fused_white && c->interp_fused && G.built && G.ok && G.fused_w_ok && (c->grid_mfma & 1) && !c->interp_lds &&
         c->interp_ws < 4 && !c->interp_wr && !psr_layout(c, L);
}

// The interpolation kernel reads the block's coefficients (pipelined blocks alternate two coefficient buffers)
bool coef_in_interp(const fpta_ctx* c, const Layout& L) {
  return psr_layout(c, L) || fused_layout(c, L) || fused_w_layout(c, L);
}

// FPTA_OPT_FUSED_NEXT_MIX: the common signal whose k_gen_mix a pipelined block of L (R_pad realizations) can take from
// the previous block's k_grid_fused (FusedMix), or -1: the layout's only common signal, of kMixTiledMinP ..
// kFusedMixMaxP pulsars, mixed by k_gen_mix (run_coefficients' branch) into its own columns; every per-pulsar signal
// drawn inside its grid signal's DFT, so the block launches nothing else before its kernel.
int32_t next_mix_seg(const fpta_ctx* c, const Layout& L, int32_t R_pad) {
  if (!c->fused_next_mix || !c->overlap || !c->gen_mix || !c->mix_mfma || L.P < kMixTiledMinP || L.P > kFusedMixMaxP ||
      L.P > kGenMixMaxP || R_pad % 128 != 0 || !L.grid.built || !L.grid.ok || !fused_layout(c, L))
    return -1;
  int32_t seg = -1;
  for (size_t g = 0; g < L.grid.members.size(); ++g)
    for (int32_t i : L.grid.members[g]) {
      const SegDesc& d = L.segs[i]->d;
      if (d.kind == 1) {
        if (seg >= 0 || !d.LT || !grid_gen_fused(c, L, g)) return -1;
        seg = i;
      } else if (!grid_gen_fused(c, L, g)) {
        return -1;
      }
    }
  return seg;
}

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
  // FPTA_OPT_FUSED_NEXT_MIX: the previous block's k_grid_fused made this block's mix of common signal nm_seg if this
  // is the block it was made for (the key, pipelined, the buffer this block swaps in, k_gen_mix's branch below);
  // otherwise that kernel may still be writing the buffer: the ctx stream is waited for before anything here
  const fpta_ctx::NextMix nmx = c->next_mix;
  c->next_mix.valid = false;
  c->next_mix_used = false;
  int32_t nm_seg = -1;
  // a miss: the side streams wait for that kernel (ctx-stream work is ordered after it anyway); a coefficient buffer
  // that may be regrown below is not freed under it either (the whole ctx stream is waited for then)
  const size_t coef_need = sizeof(double) * (size_t)P * std::max(L.K, 1) * R_pad;
  auto next_mix_miss = [&]() -> int {
    if (c->coef.cap < coef_need || c->coef2.cap < coef_need || !nmx.done) {
      HIPCHK(c, hipStreamSynchronize(c->stream), "next mix sync");
    } else {
      if (c->side) HIPCHK(c, hipStreamWaitEvent(c->side, nmx.done, 0), "next mix wait");
      if (c->side2) HIPCHK(c, hipStreamWaitEvent(c->side2, nmx.done, 0), "next mix wait");
    }
    nm_seg = -1;
    return FPTA_OK;
  };
  if (nmx.valid) {
    if (nmx.layout == &L && nmx.version == L.version && nmx.seed == seed && nmx.real0 == real0 && nmx.n_real == R &&
        nmx.R_pad == R_pad && pipe && side && merge && !zin && !x_out && !coef_host && nmx.done &&
        nmx.seg == next_mix_seg(c, L, R_pad))
      nm_seg = nmx.seg;
    else if ((rc0 = next_mix_miss()))
      return rc0;
  }
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
  if (nm_seg >= 0 && !(psr && c->coef.p == nmx.buf) && (rc0 = next_mix_miss())) return rc0;
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
  int n_launch = 0;  // kernels (and copies) this call queues
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
    ++n_launch;
    hipStream_t sg = stream_of((int32_t)g);
    KTimer kt(c, FPTA_K_GEN, sg);
    HIPCHK(c, launch_coef_merge(sg, m, P, L.K, R_pad, c->coef.as<double>()), "k_coef_merge launch");
    return FPTA_OK;
  };
  auto gen_mix_branch = [&](size_t i) {
    const SegDesc& d = L.segs[i]->d;
    return d.kind == 1 && c->gen_mix && mfma_mix && !zin && !x_out && fuse_into[i] < 0 && P <= kGenMixMaxP;
  };
  if (nm_seg >= 0 && !gen_mix_branch((size_t)nm_seg) && (rc0 = next_mix_miss())) return rc0;
  for (size_t i = 0; i < L.segs.size(); ++i) {
    const SegDesc& d = L.segs[i]->d;
    hipStream_t si = stream_of(group_of[i]);  // side2 only for members of split_g (kind 0: no mixing below)
    if (in_fused[i] && d.kind == 0) continue;  // drawn inside its grid signal's DFT
    if ((int32_t)i == nm_seg) {
      // made by the previous block's kernel into this buffer: ordered before this block's ctx-stream work; a reader on
      // a side stream (the two-kernel path's DFT of a white block) waits for that kernel
      c->next_mix_used = true;
      if (c->side) HIPCHK(c, hipStreamWaitEvent(c->side, nmx.done, 0), "next mix wait");
      if (c->side2) HIPCHK(c, hipStreamWaitEvent(c->side2, nmx.done, 0), "next mix wait");
      continue;
    }
    ++n_launch;
    if (gen_mix_branch(i)) {
      KTimer kt(c, FPTA_K_MIX, st, true);  // draws + mixing in one kernel, into the signal's own columns
      // 16-realization workgroups (FPTA_OPT_GEN_MIX 3: they fit in the LDS two k_grid_interp_psr workgroups leave;
      // C3 measured the same either way, profiles/round4/R5d)
      const int rb = c->gen_mix == 3 ? 16 : 32;
      hipEvent_t e0 = kt.start_ev();
      HIPCHK(c,
             kt.checked(launch_gen_mix(st, d, (int32_t)i, P, R, R_pad, real0, k0, k1, c->coef.as<double>(), L.K,
                                       c->gen_mix == 1 ? 2 : 1, rb, e0, kt.stop_ev())),
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
  c->coef_queued = n_launch > 0 || defer;
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


// White noise + ECORR to fuse into the synthesis epilogue (batch path).
struct WhiteCfg {
  int32_t on = 0;
  const double* sigma = nullptr;
  const int32_t* block_of = nullptr;
  const double* esig = nullptr;
  const double* zb = nullptr;
  int64_t nblocks = 0;
  int64_t zb_ld = 0;  // 0: zb realization-major [R][nblocks]; > 0 epoch-major [nblocks][zb_ld] (k_grid_fused_w only)
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
      a.w_zb_ld = white->zb_ld;
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

}  // namespace capi

// =============================================================================================== API
extern "C" {

int fpta_version(void) { return FPTA_VERSION; }

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

// Option values measured slower than the shipped one exist for same-box A/B runs and the bitwise tests
// against the shipped kernels: variant builds only (make variant DEFS=-DFPTA_DIAG_KERNELS); the product refuses them.
static bool variant_value_ok(fpta_ctx* c, bool shipped, const char* what) {
#ifdef FPTA_DIAG_KERNELS
  (void)c;
  (void)shipped;
  (void)what;
  return true;
#else
  if (shipped) return true;
  fail(c, FPTA_EINVAL, std::string(what) + ": measured slower, a variant-build option (make variant DEFS=-DFPTA_DIAG_KERNELS)");
  return false;
#endif
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
      if (!variant_value_ok(c, value == 1, "dft_gen 0 (the draws through the coefficient buffer, +8 % on C2)"))
        return FPTA_EINVAL;
      c->dft_gen = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_GEN_MIX:
      if (value < 0 || value > 3) return fail(c, FPTA_EINVAL, "gen_mix must be 0 .. 3");
      if (!variant_value_ok(c, value == 2, "gen_mix 0 / 1 / 3 (equal or slower than 2)")) return FPTA_EINVAL;
      c->gen_mix = (int)value;
      return FPTA_OK;
    case FPTA_OPT_ASYNC_SUMS:
      if (!variant_value_ok(c, value == 0, "async_sums 1 (slower on C3)")) return FPTA_EINVAL;
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
      if (value < 0 || value > 3) return fail(c, FPTA_EINVAL, "interp_fused: 0 .. 3");
      c->interp_fused = (int)value;
      return FPTA_OK;
    case FPTA_OPT_FUSED_WHITE:
      c->fused_white = value ? 1 : 0;
      return FPTA_OK;
    case FPTA_OPT_FUSED_NEXT_MIX:
      c->fused_next_mix = value ? 1 : 0;
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
      if (!variant_value_ok(c, value == 1 || value > 3, "interp_ws 0 / 2 / 3 (slower on C2 / C3)")) return FPTA_EINVAL;
      c->interp_ws = (int)value;
      return FPTA_OK;
    case FPTA_OPT_SIDE_SPLIT:
      if (value < 0 || value > 2) return fail(c, FPTA_EINVAL, "side_split must be 0 .. 2");
      if (!variant_value_ok(c, value == 2, "side_split 0 / 1 (slower on C2 / C5)")) return FPTA_EINVAL;
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
    case FPTA_OPT_FUSED_WHITE: *value = c->fused_white; return FPTA_OK;
    case FPTA_OPT_FUSED_NEXT_MIX: *value = c->fused_next_mix; return FPTA_OK;
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

}  // extern "C"
namespace __attribute__((visibility("hidden"))) capi {  // library-internal: not exported

int batch_common(fpta_ctx* c, uint64_t seed, int64_t real0, int32_t n_real, const double* zin,
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
  c->next_mix_made = false;  // set by a k_grid_fused launch that also mixes the next block's common signal
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
  // k_grid_fused_w reads them epoch-major (an epoch's realizations contiguous: 16-byte gathers of realization pairs);
  // the block then runs on it (grid_run checks), no other kernel reads them
  if (do_white && c->has_blocks) {
    const bool zb_major = path == 4 && c->fuse_white && fused_w_layout(c, L) && !c->fuse_sums;
    const int64_t ldz = zb_major ? R_pad : 0;
    HIPCHK(c, c->zb_epochs.ensure(sizeof(double) * (size_t)(zb_major ? R_pad : n_real) * c->n_blocks), "zb alloc");
    wc.zb = c->zb_epochs.as<double>();
    wc.zb_ld = ldz;
    KTimer kt(c, FPTA_K_WHITE);
    if (zb_major)
      HIPCHK(c, launch_epoch_normals_t(c->stream, c->n_blocks, n_real, real0, k0, k1, c->zb_epochs.as<double>(), ldz),
             "k_epoch_normals_t launch");
    else
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
  c->last_blk = fpta_ctx::LastBlock{true, seed, real0, n_real};
  return FPTA_OK;
}

}  // namespace capi
extern "C" {

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

}  // extern "C"
namespace __attribute__((visibility("hidden"))) capi {  // library-internal: not exported

// Per-realization {sum, sum of squares} of the context's last block into c->sums (device): from the interpolation's
// partial checksums when it wrote them for this block, else one pass over the block. On the ctx stream, or (async,
// streamed jobs with partials) on the red stream beside the next block's work; *used: the stream the sums are on.
// With dst (device or pinned host memory), sums from the partials are written there directly (*direct = true)
// instead of into c->sums.
int launch_block_checksums(fpta_ctx* c, bool async, hipStream_t* used, double* dst, bool* direct) {
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

}  // namespace capi
extern "C" {

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
  out[16] = ok ? (c->last_fma_interp > 0.0 ? c->last_fma_interp : G.fma_interp) : 0.0;
  out[17] = c->next_mix_made ? 1.0 : 0.0;
  out[18] = c->next_mix_used ? 1.0 : 0.0;
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


}  // extern "C"
