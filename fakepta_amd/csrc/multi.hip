// Several devices in one process (fpta_multi_*) and one process per GPU over RCCL (fpta_comm_*). DESIGN.md §7.
#include "capi_host.h"

extern "C" {

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

}  // extern "C"
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
extern "C" {

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

}  // extern "C"
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
extern "C" {

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
