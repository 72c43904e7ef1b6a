// The gridded path's host side: the plan of a layout (chunks, band rows, weights, grid signals, the fused kernel's
// plan) and the launches of one block (DFTs and interpolation). DESIGN.md §5c.
#include "capi_host.h"

namespace __attribute__((visibility("hidden"))) capi {  // library-internal: not exported

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
  // + kFusedWdPad band rows after the last chunk: k_grid_fused(_w) loads NQ band steps' weights of every chunk unclamped
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
    const size_t lds = sizeof(double) * ((size_t)rows * kFusedPitch + 2 * kFusedMaxSig * kFusedSlot) + 48;
    bool members_ok = true;
    for (const std::vector<int32_t>& m : G.members) members_ok = members_ok && m.size() <= (size_t)kDftGenTerms;
    // k_grid_fused_w (white / ECORR blocks, and plain blocks of three grid signals): the grids of kFusedWReal
    // realizations, <= kFusedWMaxSig grid signals, <= kFusedWJobs DFT jobs
    bool ok_w = n_seg <= kFusedWMaxSig && members_ok;
    int32_t jobs_w = 0, rows_w = 0;
    for (int32_t s = 0; s < n_seg && ok_w; ++s) {
      const GridSeg* gs = G.segs[s];
      ok_w = gs->nf % 4 == 0 && gs->ldq == (gs->nf / 4 + 32) / 32 * 32;
      jobs_w += (gs->nf / 4 + 32) / 32;
      rows_w += gs->nf;
    }
    const size_t lds_w = sizeof(double) * ((size_t)rows_w * kFusedWPitch + 2 * kFusedWMaxSig * kFusedWSlot) + 48;
    ok_w = ok_w && jobs_w <= kFusedWJobs && lds_w <= (size_t)kFusedLdsMax;
    if (ok_w && G.fused_lrow0.size() != (size_t)n_seg) {  // the LDS row of each grid signal (as k_grid_fused's)
      G.fused_lrow0.clear();
      for (int32_t s = 0, r = 0; s < n_seg; r += G.segs[s]->nf, ++s) G.fused_lrow0.push_back(r);
    }
    G.fused_w_ok = ok_w;
    G.fused_w_lds = lds_w;
    ok = ok && members_ok && jobs <= kFusedDW && lds <= (size_t)kFusedLdsMax;
    if (ok || ok_w) {
      // [n_chunks][4][fq]: band row 4 q + j of a chunk at [j][q] (a lane's rows of consecutive steps contiguous: 16-byte
      // loads), fq = the band steps rounded up to 4 and at least kFusedNQ; steps past the chunk's repeat its first row
      const int32_t fq = std::max(std::max(kFusedNQ, kFusedWNQ), (vmax / 4 + 3) & ~3);
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
    G.frows_ok = ok || ok_w;
    // Half-chunk bands (FusedHalf): TOAs 0..15 and 16..31 of each chunk get bands of their own (a 32-TOA chunk's band
    // is w + the cells its 32 TOAs span; a half's, w + the cells of 16). Per half the signals' bands back to back,
    // padded to whole band steps; the weights by the half-band layout of k_grid_weights.
    if (ok) {
      std::vector<int4> hch(n_chunks);
      std::vector<int32_t> hv((size_t)2 * n_chunks, 0);                    // band rows of each half (padded)
      std::vector<int32_t> hrow_of(N), hchunk_of(N), htt_of(N);            // per TOA (filled per signal below)
      std::vector<std::vector<int64_t>> hlo(n_seg, std::vector<int64_t>((size_t)2 * n_chunks, 0));
      std::vector<std::vector<int32_t>> hvoff(n_seg, std::vector<int32_t>((size_t)2 * n_chunks, 0));
      std::vector<std::vector<int32_t>> hn(n_seg, std::vector<int32_t>((size_t)2 * n_chunks, 0));
      double steps_full = 0.0, steps_half = 0.0;
      for (int32_t ci = 0; ci < n_chunks; ++ci) {
        const int64_t a0 = L.h_offs[chunks[ci].x] + chunks[ci].y, a1 = a0 + chunks[ci].z;
        int32_t nqh[2] = {0, 0};
        for (int32_t h = 0; h < 2; ++h) {
          const int64_t b0 = a0 + kFusedHalfTT * h, b1 = std::min(a1, b0 + kFusedHalfTT);
          if (b0 >= b1) continue;
          int32_t v = 0;
          for (int32_t s = 0; s < n_seg; ++s) {
            int64_t lo1 = INT64_MAX, hi1 = INT64_MIN;
            for (int64_t u = b0; u < b1; ++u) {
              const int64_t j = J[s][u] + band_lo[s][ci];  // unwrapped first row of the TOA
              lo1 = std::min(lo1, j);
              hi1 = std::max(hi1, j);
            }
            const size_t hc = (size_t)2 * ci + h;
            hlo[s][hc] = lo1;
            hvoff[s][hc] = v;
            hn[s][hc] = (int32_t)(hi1 - lo1) + ws[s];
            v += hn[s][hc];
          }
          hv[(size_t)2 * ci + h] = (v + 3) & ~3;
          nqh[h] = hv[(size_t)2 * ci + h] / 4;
          for (int64_t u = b0; u < b1; ++u) {
            hchunk_of[u] = 2 * ci + h;
            htt_of[u] = (int32_t)(u - b0);
          }
        }
        hch[ci] = make_int4(chunks[ci].x, chunks[ci].y, chunks[ci].z, nqh[0] | (nqh[1] << 16));
        steps_full += 4.0 * (chunks[ci].w / 4);
        steps_half += 4.0 * std::max(nqh[0], nqh[1]);  // the kernel runs both halves' longer step count
      }
      int32_t hvmax = 8;
      for (int32_t v : hv) hvmax = std::max(hvmax, (v + 7) & ~7);
      const int32_t hfq = std::max(kFusedHalfNQ, (hvmax / 4 + 3) & ~3);
      std::vector<int32_t> hrt((size_t)n_chunks * 2 * 4 * hfq);
      for (int32_t ci = 0; ci < n_chunks; ++ci)
        for (int32_t h = 0; h < 2; ++h) {
          const size_t hc = (size_t)2 * ci + h;
          std::vector<int32_t> band_row(std::max(hv[hc], 1), G.fused_lrow0[0]);
          int32_t v = 0;
          for (int32_t s = 0; s < n_seg; ++s)
            for (int32_t i = 0; i < hn[s][hc]; ++i)
              band_row[v++] = G.fused_lrow0[s] + (int32_t)(((hlo[s][hc] + i) % nf[s] + nf[s]) % nf[s]);
          for (; v < (int32_t)band_row.size(); ++v) band_row[v] = band_row[0];
          int32_t* r = hrt.data() + hc * 4 * hfq;
          for (int32_t j = 0; j < 4; ++j)
            for (int32_t q = 0; q < hfq; ++q)
              r[j * hfq + q] = 4 * q + j < hv[hc] ? band_row[4 * q + j] : band_row[0];
        }
      if ((rc = upload(c, G.hchunks, hch.data(), sizeof(int4) * hch.size(), "fused half chunks")) ||
          (rc = upload(c, G.hrows, hrt.data(), sizeof(int32_t) * hrt.size(), "fused half rows")))
        return rc;
      // + the rows the kernel's unconditional loads may read past the last half (kFusedHalfNQ steps)
      const size_t hbytes = sizeof(double) * ((size_t)2 * n_chunks * hvmax + 4 * kFusedHalfNQ) * kFusedHalfTT;
      HIPCHK(c, G.hwd.ensure(hbytes), "half weights alloc");
      HIPCHK(c, hipMemsetAsync(G.hwd.p, 0, hbytes, c->stream), "half weights memset");
      if ((rc = upload(c, d_chunk_of, hchunk_of.data(), sizeof(int32_t) * N, "half chunk_of")) ||
          (rc = upload(c, d_tt_of, htt_of.data(), sizeof(int32_t) * N, "half tt_of")))
        return rc;
      for (int32_t s = 0; s < n_seg; ++s) {
        const SegDesc& d = L.segs[G.anchor[s]]->d;
        for (int64_t t = 0; t < N; ++t) {
          const size_t hc = (size_t)hchunk_of[t];
          hrow_of[t] = (int32_t)(J[s][t] + band_lo[s][hc / 2] - hlo[s][hc]) + hvoff[s][hc];
        }
        if ((rc = upload(c, d_row, hrow_of.data(), sizeof(int32_t) * N, "half rows")) ||
            (rc = upload(c, d_d, D[s].data(), sizeof(double) * N, "grid offsets")))
          return rc;
        HIPCHK(c,
               launch_grid_weights(c->stream, d, N, L.nu.as<double>(), d_chunk_of.as<int32_t>(), d_tt_of.as<int32_t>(),
                                   d_row.as<int32_t>(), d_d.as<double>(), ws[s], betas[s], hvmax, G.hwd.as<double>(),
                                   nullptr, s, n_seg, 1),
               "k_grid_weights (half bands) launch");
        HIPCHK(c, hipStreamSynchronize(c->stream), "half weights sync");  // d_row / d_d are reused
      }
      int32_t hnq = 1;
      for (int32_t v : hv) hnq = std::max(hnq, v / 4);
      G.fused_hfq = hfq;
      G.fused_hvmax = hvmax;
      G.fused_hnq = hnq;
      G.fused_half_gain = steps_half > 0.0 ? steps_full / steps_half : 0.0;
      G.fma_interp_half = steps_half * 4.0 * kGridTT / 4.0;  // 4 rows x 32 TOAs per (both-halves) step
      G.fused_half_ok = true;
    }
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
int grid_run(fpta_ctx* c, Layout& L, SynthArgs& a, int32_t R_pad, bool pipe) {
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
  // k_grid_fused_w: the same for white / ECORR blocks and for plain blocks k_grid_fused does not take (three grid
  // signals, C5's shape)
  const bool fused_w = !psr && !fused && fused_w_layout(c, L) && !a.accumulate &&
                       !(c->fuse_sums && a.out == c->out.as<double>()) && (!pipe || c->prev_psr);
  if (a.w_on && a.w_zb_ld > 0 && !fused_w)  // batch_common wrote them for k_grid_fused_w only
    return fail(c, FPTA_ESTATE, "internal: epoch-major ECORR normals for a block k_grid_fused_w does not take");
  // grid buffers only for the kernels that read one (two of 0.41 GB each on C2)
  if (!psr && !fused && !fused_w && (G.g_rpad != R_pad || (pipe && G.g2.cap < gbytes))) {
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
  // a pipelined block whose draws and mixing queued nothing on the side stream (the previous block's kernel mixed its
  // common signal, FPTA_OPT_FUSED_NEXT_MIX; its other signals drawn inside the kernel): no grid-ready event to wait for
  bool gwait = pipe;
  if (psr || fused || fused_w) {
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
    gwait = pipe && c->coef_queued;
    if (gwait) HIPCHK(c, hipEventRecord(c->ev_gready, c->side), "event record");
    if (pipe) {
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
  if (gwait) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_gready, 0), "grid ready wait");
  if (pipe && c->s2done_set) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_gready2, 0), "grid ready wait");
  // the fused launch takes the timing events itself (no marker packets around it); the diagnostic options that take
  // another kernel for a fused layout time it with recorded events
#ifdef FPTA_DIAG_KERNELS
  const bool ext = (fused || fused_w) && c->interp_ws != 4 && c->interp_ws != 5 && !c->interp_wr;
#else
  const bool ext = fused || fused_w;
#endif
  KTimer kt(c, FPTA_K_SYNTH, nullptr, ext);
  GridBand band{G.chunks.as<int4>(), G.rows.as<int32_t>(), G.wd.as<double>(), gbase, G.n_chunks, G.vmax,
                G.grid_rows, a.part ? G.pgfirst.as<int32_t>() : nullptr, a.part ? G.n_pg : G.n_chunks};
  // the warp-specialised kernel for plain blocks; with fused partial checksums its reduce-scatter temporaries take
  // its VGPRs to 230 and the register kernel is faster (C3: 47.9 vs 52.5 ms per job, profiles/r02k_ab_c2c3_ws.txt)
  // k_grid_interp_ws tiles 512 realizations (4 compute waves x 128): when R_pad leaves some of the last tile's compute
  // waves idle, the 256-realization tiles of k_grid_interp_ws2 waste less (C4, R_pad = 256: half of every ws tile;
  // 6.8-7.4 vs 8.4 ms/step, profiles/r04a_c4_ws2.txt)
  // (the automatic k_grid_interp_ws2 choice for such R_pad, diagnostic builds only since round 6: no shipped layout
  // reaches it)
#ifdef FPTA_DIAG_KERNELS
  const bool ws2_fits = c->interp_ws == 1 && (R_pad + 255) / 256 * 256 - R_pad < (R_pad + 511) / 512 * 512 - R_pad;
#else
  const bool ws2_fits = false;
#endif
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
  } else if (fused || fused_w) {
    // half-chunk bands (FPTA_OPT_INTERP_FUSED 1: where they save >= 3 % of the interpolation MFMAs; 3: always)
    const bool half = fused && G.fused_half_ok &&
                      (c->interp_fused == 3 || (c->interp_fused == 1 && G.fused_half_gain >= 1.03));
    const int32_t nq = half ? G.fused_hnq : G.vmax / 4;
    FusedArgs f{};
    if (half) f.h = FusedHalf{G.hchunks.as<int4>(), G.hrows.as<int32_t>(), G.hwd.as<double>(), G.fused_hfq, G.fused_hvmax};
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
    // The DFT waves interpolate an item's chunks while more than join_reserve are left, then build the next item
    // while the interpolation waves take the rest. In MFMA-equivalents (64 cycles): a ring iteration of a DFT wave is
    // its 32 MFMAs + ~20 per generated term (a Philox call and two Box-Muller pairs per lane), a chunk 4 per band step
    // + ~12 (operand loads, stores). The reserve is kFusedJoinSafety times the chunks the interpolation waves do in a
    // build: C2 (~7 x 72 per build, ~48 per chunk: reserve 63 of its 63 chunks per item) hardly joins; C4 (~7 x 32,
    // ~32 per chunk: reserve ~42 of 313) joins for most of an item. (The estimate is about half the measured build
    // time on C2; the factor 1.5 was the best of 0.5 .. 5 on both, profiles/round5/r5mn_*.)
    // k_grid_fused_w (16-realization items): an iteration is up to 64 MFMAs (two jobs) + the draws, a chunk V / 2
    // MFMAs + ~12 + the white epilogue (two Philox calls per lane: ~40 on white blocks).
    {
      int it_max = 0, gen = 0;
      for (int32_t s = 0; s < f.n_sig; ++s) {
        const int nm = f.s[s].nm;
        it_max = std::max(it_max, fused_w ? (nm + kFusedWGroupModes - 1) / kFusedWGroupModes
                                          : (((((nm + 1) >> 1) + 3) >> 2) + 1) >> 1);
        for (int i = 0; i < f.s[s].n_terms; ++i) gen += f.s[s].term_kind[i] == 0;
      }
      const double build = it_max * ((fused_w ? 64.0 : 32.0) + 20.0 * gen);
      const double chunk = fused_w ? G.mean_v / 2 + 12.0 + (a.w_on ? 40.0 : 0.0) : G.mean_v + 12.0;
      f.join_reserve = (int32_t)std::min(
          1.0e6, std::ceil((fused_w ? kFusedWJoinSafety : kFusedJoinSafety) * kFusedIW * build / chunk));
    }
    f.ring_off = (G.fused_lrow0.back() + G.segs.back()->nf) * (fused_w ? kFusedWPitch : kFusedPitch);
    // a pipelined block whose common signals are mixed by a separate k_mix_mfma (P > kGenMixMaxP, C4): the next
    // block's mix is queued on the side stream while this kernel runs
    {
      bool sep_mix = false;
      for (const Seg* sg : L.segs) sep_mix = sep_mix || (sg->d.kind == 1 && L.P > kGenMixMaxP);
      f.cu_pct = pipe && sep_mix ? FPTA_FUSED_MIX_CU_PCT : 100;
    }
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
    // The item queues are zeroed once: every launch leaves them zero (its last workgroup resets them), which holds
    // because fused launches only go on the context stream, one after another. The debug build re-zeroes them before
    // every launch, so a launch that did not complete cannot make the next one skip items unnoticed.
#ifdef FPTA_DEBUG
    c->fused_q_ready = false;
#endif
    if (!c->fused_q_ready) {
      HIPCHK(c, c->fused_q.ensure(sizeof(uint32_t) * kFusedQueueWords), "fused queue alloc");
      HIPCHK(c, hipMemsetAsync(c->fused_q.p, 0, sizeof(uint32_t) * kFusedQueueWords, c->stream), "fused queue memset");
      c->fused_q_ready = true;
    }
    f.queue = c->fused_q.as<uint32_t>();
    // FPTA_OPT_FUSED_NEXT_MIX: the next block's common-signal mix (this seed and size) as spare-time tickets, into the
    // coefficient buffer that block swaps in (c->coef2: this block's kernel and k_gen_mix's of the block before read
    // it no more; grown already, so it is not reallocated under the kernel). The next block's first realization:
    // real0 + this block's stride from the last one of the same seed and size when that is a whole number of blocks
    // (G ranks' interleaved blocks), else real0 + n_real.
    c->next_mix_made = false;
    const int32_t nms = !fused_w && pipe && c->prev_psr ? next_mix_seg(c, L, R_pad) : -1;
    const size_t coef_bytes = sizeof(double) * (size_t)L.P * std::max(L.K, 1) * R_pad;
    const uint64_t blk_seed = (uint64_t)c->blk_k0 | ((uint64_t)c->blk_k1 << 32);
    const fpta_ctx::LastBlock& lb = c->last_blk;
    const int64_t step = c->blk_real0 - lb.real0;
    const int64_t stride =
        lb.valid && lb.seed == blk_seed && lb.n_real == a.n_real && step >= a.n_real && step % a.n_real == 0 ? step
                                                                                                         : a.n_real;
    if (nms >= 0 && c->coef2.cap >= coef_bytes && c->blk_real0 + stride + a.n_real <= ((int64_t)1 << 32)) {
      const SegDesc& d = L.segs[nms]->d;
      FusedMix& m = f.mix;
      m.LT = d.LT;
      m.amp = d.amp;
      m.coef = c->coef2.as<double>();
      m.real0 = c->blk_real0 + stride;
      m.k0 = c->blk_k0;
      m.k1 = c->blk_k1;
      m.lt_ld = d.lt_ld;
      m.lt_rows = d.lt_rows;
      m.P = L.P;
      m.K = a.K;
      m.col0 = d.col0;
      m.R_pad = R_pad;
      m.n_real = a.n_real;
      m.n_q = d.n_q;
      m.lower = d.l_lower;
      m.seg = nms;
      m.nm = d.nm;
      m.n_tiles = d.nm * (R_pad / 16) * ((L.P + kFusedMixGroup - 1) / kFusedMixGroup);
    }
    hipEvent_t e0 = kt.start_ev();
    int ki = 0;
    if (fused_w) {
      HIPCHK(c, kt.checked(launch_grid_fused_w(c->stream, a, band, f, nq, G.fused_w_lds, e0, kt.stop_ev(), &ki)),
             "k_grid_fused_w launch");
      kind = kInterpKindFused0 + kFusedKernels + ki;
    } else {
      HIPCHK(c, kt.checked(launch_grid_fused(c->stream, a, band, f, nq, G.fused_lds, e0, kt.stop_ev(), half, &ki)),
             "k_grid_fused launch");
      kind = kInterpKindFused0 + ki;  // fpta_batch_grid_info_n slot 15: the instance launched
      if (f.mix.n_tiles > 0) {
        fpta_ctx::NextMix& nx = c->next_mix;
        nx.valid = true;
        nx.layout = &L;
        nx.version = L.version;
        nx.seed = blk_seed;
        nx.real0 = f.mix.real0;
        nx.n_real = a.n_real;
        nx.R_pad = R_pad;
        nx.seg = nms;
        nx.buf = c->coef2.p;
        nx.done = nullptr;  // the event recorded after this launch (pipe: ev_gfree of this block's buffer index, below)
        c->next_mix_made = true;
      }
    }
    c->last_fma_interp = half ? G.fma_interp_half : G.fma_interp;
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
  if (kind < kInterpKindFused0) c->last_fma_interp = G.fma_interp;
  if (pipe) {  // buffer gi is free once this interpolation is done; the next block's DFT writes the other one
    HIPCHK(c, hipEventRecord(c->ev_gfree[gi], c->stream), "event record");
    if (c->next_mix_made) c->next_mix.done = c->ev_gfree[gi];  // the kernel that writes the next block's mix is done
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

}  // namespace capi
