/*
 * fakepta_amd.h — C-ABI of libfakepta_amd.so, the MI355X (gfx950) Fourier-basis
 * Gaussian-process residual synthesis for pulsar-timing arrays.
 *
 * The reference (mfalxa/fakepta) has no FFI: its hot path is numpy loops inside
 * Python methods. Each entry point below names the reference code it replaces;
 * the Python host layer (fakepta_amd/fake_pta.py, correlated_noises.py, batch.py)
 * binds them through ctypes (fakepta_amd/_capi.py) behind the reference's own
 * method signatures. INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain pointers + sizes, no torch types. Host buffers are owned by the caller;
 *     the library copies inputs to device buffers owned by the context.
 *   - Every call returns 0 on success or a negative FPTA_E* code; the message is
 *     available from fpta_last_error(ctx) (or fpta_last_error(NULL) for calls
 *     that failed before a context existed). The library never aborts or exits.
 *   - A context owns one device and one HIP stream and is single-threaded; use
 *     one context per GPU (one process per GPU for multi-GPU).
 *   - All arithmetic is IEEE fp64.
 *   - Angular frequencies: the library computes the phase as (2*pi*f_k) * t with
 *     the same operation order as fakepta/fake_pta.py:386, so drop-in results
 *     match the numpy reference to rounding.
 */
#ifndef FAKEPTA_AMD_H
#define FAKEPTA_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FPTA_OK 0
#define FPTA_EINVAL (-22)   /* bad argument / shape */
#define FPTA_ENOMEM (-12)   /* device allocation failed */
#define FPTA_EDEVICE (-19)  /* no device / HIP runtime error */
#define FPTA_ESTATE (-77)   /* call out of order (e.g. synth before set_toas) */

typedef struct fpta_ctx fpta_ctx;

/* ------------------------------------------------------------------ lifetime */
/* 10000 * ABI major + 100 * behaviour revision (FPTA_VERSION): the major changes only if an entry point's signature
 * or buffer size changes; the revision when a call's accepted values or reported codes change. 10100 (round 6):
 * FPTA_OPT_INTERP_WS 0/2/3, DFT_GEN 0, GEN_MIX 0/1/3, ASYNC_SUMS 1 and SIDE_SPLIT 0/1 are refused (FPTA_EINVAL) by
 * the product library (variant builds accept them); FPTA_OPT_INTERP_FUSED takes 0 .. 3; fpta_batch_grid_info_n slot
 * 15 names each k_grid_fused instance (kinds 11 .. 19) instead of kinds 8 / 9. 10200 (round 6): option
 * FPTA_OPT_FUSED_NEXT_MIX; fpta_batch_grid_info_n slots 17 and 18 (FPTA_GRID_INFO_LEN 19). */
#define FPTA_VERSION 10200
int fpta_version(void);
int fpta_create(int device, fpta_ctx** out);
int fpta_destroy(fpta_ctx* ctx);
const char* fpta_last_error(const fpta_ctx* ctx);
int fpta_device_count(int* n);

/* ------------------------------------------------------------------ drop-in, one realization
 * These replace the per-call numpy loops of the reference; the host keeps the
 * reference's RNG draws (np.random legacy stream) and bookkeeping, so a seeded
 * script produces the same residuals.
 */

/* Replaces fakepta/fake_pta.py:385-387 (Pulsar.add_time_correlated_noise hot loop)
 * and fakepta/fake_pta.py:538-554 (Pulsar.reconstruct_signal GP branches).
 *   residuals[t] += sign * sum_s m_s(t) (freqf_s/nu_t)^idx_s *
 *                   sum_k ( ccos[k] cos(2 pi f[k] t) + csin[k] sin(2 pi f[k] t) )
 * Segments s are concatenated: seg_nmodes[n_seg]; f/ccos/csin hold sum(seg_nmodes)
 * values. ccos = sqrt(df)*coeffs[0::2] when injecting, df*fourier[0] when reconstructing.
 * mask: NULL, or uint8 [n_seg][n_toa] (1 = TOA belongs to the backend of that segment).
 * residuals: host fp64 [n_toa], read and written. */
int fpta_gp_accumulate(fpta_ctx* ctx, int64_t n_toa, const double* toas, const double* nu,
                       int32_t n_seg, const int32_t* seg_nmodes, const double* f,
                       const double* ccos, const double* csin, const double* seg_idx,
                       const double* seg_freqf, const uint8_t* mask, double sign,
                       double* residuals);

/* Array form of fpta_gp_accumulate (one launch for a whole array): replaces the per-pulsar
 * reconstruct_signal calls of correlated_noises.py:133-134 (replace-on-reinject) and of
 * remove_signal (fake_pta.py:557-567) over many pulsars. n_psr pulsars (CSR offs[n_psr+1]);
 * segment s has seg_nmodes[s] modes and contributes f/ccos/csin blocks of [n_psr][seg_nmodes[s]]
 * (concatenated over segments). mask: NULL or uint8 [n_seg][n_toa_total]. residuals [n_toa_total]. */
int fpta_gp_accumulate_array(fpta_ctx* ctx, int32_t n_psr, const int64_t* offs, const double* toas,
                             const double* nu, int32_t n_seg, const int32_t* seg_nmodes, const double* f,
                             const double* ccos, const double* csin, const double* seg_idx,
                             const double* seg_freqf, const uint8_t* mask, double sign, double* residuals);

/* Replaces fakepta/correlated_noises.py:146-160 (add_common_correlated_noise hot loop).
 * n_psr pulsars, CSR offsets offs[n_psr+1] into toas/nu (seconds / MHz).
 * For mode k: x_sin = L z[k][0], x_cos = L z[k][1] (z in the reference's draw order,
 * [n_modes][2][n_psr], sin vector drawn first), L = [n_psr][n_psr] row-major factor with
 * L L^T = ORF (for exact reference parity pass the transpose of numpy's SVD factor).
 *   residuals[t in p] += (freqf/nu_t)^idx * sum_k amp[k] ( x_cos[p] cos(2 pi f_k t)
 *                                                        + x_sin[p] sin(2 pi f_k t) )
 * with amp[k] = sqrt(df_k) * sqrt(psd_k) (the reference's df**0.5 * coeffs[2k]; cos and sin
 * share it because coeffs = sqrt(repeat(psd, 2)), correlated_noises.py:146-147).
 * x_out (optional, may be NULL): [n_modes][2][n_psr] mixed draws (cos, sin) for the
 * host's signal_model bookkeeping (correlated_noises.py:157-158). */
int fpta_common_accumulate(fpta_ctx* ctx, int32_t n_psr, const int64_t* offs, const double* toas,
                           const double* nu, int32_t n_modes, const double* f, const double* amp,
                           double idx, double freqf, const double* L,
                           const double* z, double* residuals, double* x_out);

/* Replaces fakepta/fake_pta.py:201-230 (add_white_noise), with ECORR fixed (defects D1/D2):
 *   residuals[t] += sigma[t] * z[t]  +  sum over blocks b containing t: ecorr_sigma[b] * zb[b]
 * Blocks are CSR: block_offs[n_blocks+1] into block_idx (TOA indices, any order).
 * n_blocks may be 0 (then block_* / ecorr_sigma / zb may be NULL). */
int fpta_white_accumulate(fpta_ctx* ctx, int64_t n_toa, const double* sigma, const double* z,
                          int64_t n_blocks, const int64_t* block_offs, const int64_t* block_idx,
                          const double* ecorr_sigma, const double* zb, double* residuals);

/* ------------------------------------------------------------------ dense covariance
 * The reference's covariance-matrix route (fakepta/fake_pta.py:389-420, :493-524). Signals are
 * given as segments like fpta_gp_accumulate: seg_nmodes[n_seg]; f and w hold sum(seg_nmodes)
 * values with w = psd * df (the reference's np.repeat(psd * df, 2)); seg_idx / seg_freqf give
 * each segment's chromatic factor (freqf/nu)^idx. For a backend's system noise pass only that
 * backend's TOAs (the reference builds the covariance of the masked TOAs, :398-405).
 * white_var: NULL or [n_toa] white-noise variances, added on the diagonal. */

/* Replaces make_time_correlated_noise_cov (fakepta/fake_pta.py:389-420) and, summed over
 * segments, the red part of make_noise_covariance_matrix (:493-513); with white_var, the
 * total covariance np.diag(white_cov) + red_cov of draw_noise_model (:517):
 *   cov[i][j] = sum_s ch_s(i) ch_s(j) sum_k w[k] (cos(2 pi f_k t_i) cos(2 pi f_k t_j)
 *                                                + sin(2 pi f_k t_i) sin(2 pi f_k t_j))
 *               + (i == j ? white_var[i] : 0)
 * Basis generation + fp64 MFMA Gram (lower tiles, mirrored). cov: host [n_toa][n_toa]. */
int fpta_gp_covariance(fpta_ctx* ctx, int64_t n_toa, const double* toas, const double* nu,
                       int32_t n_seg, const int32_t* seg_nmodes, const double* f, const double* w,
                       const double* seg_idx, const double* seg_freqf, const double* white_var,
                       double* cov);

/* Replaces draw_noise_model(residuals) (fakepta/fake_pta.py:520-523), the Wiener estimate
 *   out = red_cov^T C^-1 residuals,  C = red_cov + diag(white_var),
 * evaluated as residuals - white_var * C^-1 residuals (red_cov is symmetric) through a device
 * Cholesky factorisation of C instead of the reference's explicit inverse. white_var is
 * required. FPTA_EINVAL if C is not positive definite. out may alias residuals. */
int fpta_noise_wiener(fpta_ctx* ctx, int64_t n_toa, const double* toas, const double* nu,
                      int32_t n_seg, const int32_t* seg_nmodes, const double* f, const double* w,
                      const double* seg_idx, const double* seg_freqf, const double* white_var,
                      const double* residuals, double* out);

/* Batched draw_noise_model() (fakepta/fake_pta.py:518-519): n_real realizations of N(0, C),
 * C = red_cov + diag(white_var), as x = L z with L the device Cholesky factor of C and z
 * Philox normals ctr = (toa, 0xFFFFFFFF, 0xFFFFFFF2, g >> 1), pick [g & 1], g = real0 + r.
 * Same distribution as the reference's np.random.multivariate_normal (which factors C by SVD);
 * the draws themselves follow this library's stream. out: host [n_real][n_toa]. */
int fpta_noise_draw(fpta_ctx* ctx, int64_t n_toa, const double* toas, const double* nu,
                    int32_t n_seg, const int32_t* seg_nmodes, const double* f, const double* w,
                    const double* seg_idx, const double* seg_freqf, const double* white_var,
                    uint64_t seed, int64_t real0, int32_t n_real, double* out);

/* ------------------------------------------------------------------ batched realizations
 * Many independent realizations of the whole array on device (north-star steps 1-4):
 * Philox4x32-10 draws -> ORF mixing -> fused basis/contraction -> white/ECORR.
 * Draw streams (invariant to batching and to the number of GPUs):
 *   GP   : ctr = (mode, pulsar, segment, realization), key = seed -> (z_cos, z_sin)
 *   white: ctr = (toa, 0xFFFFFFFF, 0xFFFFFFF0, realization>>1), pick [realization&1]
 *   ECORR: ctr = (block>>1, 0xFFFFFFFF, 0xFFFFFFF1, realization), pick [block&1]
 * Replaces the Python loop of fakepta/fake_pta.py:648-668 + correlated_noises.py:153-160
 * when many realizations of one array are needed. */

/* Array layout: CSR offsets [n_psr+1], toas [s], nu [MHz]. Clears previously added signals. */
int fpta_batch_set_toas(fpta_ctx* ctx, int32_t n_psr, const int64_t* offs, const double* toas,
                        const double* nu);
/* kind 0 = per-pulsar GP: f, amp are [n_psr][n_modes] (amp 0 disables a pulsar);
 * kind 1 = common GP:    f, amp are [n_modes], L is [n_psr][n_psr] (x = L z).
 * amp = sqrt(psd * df). mask: NULL or uint8 [n_toa_total]. Returns the segment id (>= 0). */
int fpta_batch_add_signal(fpta_ctx* ctx, int32_t kind, int32_t n_modes, const double* f,
                          const double* amp, double idx, double freqf, const double* L,
                          const uint8_t* mask);
/* White noise sigma [n_toa_total] (NULL disables) and ECORR blocks (CSR over global TOA
 * indices, ecorr_sigma [n_blocks]; n_blocks 0 disables). */
int fpta_batch_set_white(fpta_ctx* ctx, const double* sigma, int64_t n_blocks,
                         const int64_t* block_offs, const int64_t* block_idx,
                         const double* ecorr_sigma);
int fpta_batch_clear_signals(fpta_ctx* ctx);
/* Synthesize realizations real0 .. real0+n_real-1 into the context's device buffer
 * [n_real][n_toa_total]. If out != NULL the result is also copied to host memory
 * (row-major, same shape). coeffs_out: NULL or host [n_psr][K][n_real] coefficient dump
 * (K = fpta_batch_info column count) for validation. */
int fpta_batch_synth(fpta_ctx* ctx, uint64_t seed, int64_t real0, int32_t n_real, double* out,
                     double* coeffs_out);
/* Validation mode: same as fpta_batch_synth but the standard normals come from the host:
 * z [n_real][n_seg][n_psr][n_modes_max][2] (cos, sin); white/ECORR are not added. */
int fpta_batch_synth_from_z(fpta_ctx* ctx, int32_t n_real, int32_t n_modes_max, const double* z,
                            double* out);
/* Copy realizations [r_begin, r_begin + r_count) of the last block to host [r_count][n_toa_total]
 * (the "residual block" gather of SURVEY.md §8(e); the full block can be tens of GB). */
int fpta_batch_download(fpta_ctx* ctx, int32_t r_begin, int32_t r_count, double* host);
/* Device pointer of the last synthesized block and its leading dimension (n_toa_total). */
int fpta_batch_device_out(fpta_ctx* ctx, double** dptr, int64_t* ld, int32_t* n_real);
/* Per-realization sum and sum of squares of the last block, computed on device
 * (deterministic order). sums: host [n_real][2]. */
int fpta_batch_checksums(fpta_ctx* ctx, double* sums);
/* Realizations real0 .. real0 + n_real - 1 streamed through this context in batches of <= batch (the context's
 * block then holds the last batch) with their checksums written to sums [n_real][2] (as fpta_batch_checksums,
 * from the gridded interpolation's partial sums where it runs): batches are queued back to back with no host
 * synchronisation in between (pinned staging, one sync at the end). The single-device form of
 * fpta_multi_synth; fakepta_amd.batch.simulate_sharded uses it when no per-batch consumer is given. */
int fpta_batch_synth_checksums(fpta_ctx* ctx, uint64_t seed, int64_t real0, int64_t n_real, int32_t batch,
                               double* sums);
/* Correlation statistics of the last block, the estimator of
 * fakepta/correlated_noises.py:14-34 (C_r[a][b] = dot(res_a, res_b) / n) for arrays whose pulsars
 * all have n TOAs (FPTA_EINVAL otherwise):
 *   mode 0: host out [n_real][P][P], C_r per realization
 *   mode 1: host out [P][P], sum over realizations of C_r
 *   mode 2: host out [P][P], sum over realizations of C_r[a][b] / sqrt(C_r[a][a] C_r[b][b])
 *   mode 3: host out [n_real][P], auto-correlations C_r[p][p]
 * Sums are formed in a fixed order (bitwise reproducible). */
int fpta_batch_correlations(fpta_ctx* ctx, int32_t mode, double* out);
/* info[0]=n_psr info[1]=n_toa_total info[2]=n_seg info[3]=K columns info[4]=max toas/pulsar */
int fpta_batch_info(fpta_ctx* ctx, int64_t* info);

/* Gridded-path plan of the batch layout and the path the last batch took (for rooflines):
 * out[0] synthesis path of the last batch (1 direct, 2 MFMA, 3 VALU, 4 gridded), out[1] plan usable,
 * out[2] interpolation chunks, out[3] k_grid_dft FMAs per realization, out[4] k_grid_interp FMAs per
 * realization, out[5] direct-contraction FMAs per realization, out[6] grid values per realization,
 * out[7] interpolation-weight bytes, out[8] the FPTA_OPT_GRID_MFMA mask in force, out[9] the a-priori
 * relative aliasing bound exp(-pi w sqrt(1 - 1/sigma)) of the width/oversampling options in force (auto
 * selection takes the gridded path only when it is <= 2e-12), out[10] width w, out[11] oversampling sigma,
 * out[12] grid signals of the plan (signals after FPTA_OPT_GRID_COALESCE), out[13] layout signals, out[14]
 * mean band rows per chunk (all grid signals, padded to 4), out[15] the interpolation kernel of the last gridded
 * block: 0 none, else 1 + 4 kind + 2 (white / ECORR epilogue) + (fused partial checksums), kind 0
 * k_grid_interp_mfma, 1 k_grid_interp_ws, 2 k_grid_interp_ws2, 3 k_grid_interp_lds, 4 k_grid_interp_st, 5
 * k_grid_interp_u, 6 / 7 k_grid_interp_psr with 4 / 8 band steps, 10 k_grid_interp_wr (diagnostic builds only),
 * 11 .. 19 the k_grid_fused<NQ, ODD, GEN, HALF> instances (8 / 12 band steps' operands x no draws / draws / draws
 * from an odd realization, then half-chunk bands x the same three), 20 / 21 k_grid_fused_w (white / ECORR epilogue;
 * even / odd first realization); out[16] (FPTA_VERSION 10100) the interpolation MFMA FMAs per realization of the
 * last gridded block as its kernel ran them (half-chunk bands: both halves' steps; else out[4]); out[17]
 * (FPTA_VERSION 10200) 1 when the last block's k_grid_fused also made the next block's common-signal mix
 * (FPTA_OPT_FUSED_NEXT_MIX), out[18] 1 when the last block took its common-signal mix from the previous block's kernel
 * (no k_gen_mix launch).
 * fpta_batch_grid_info_n writes the first min(n_out, FPTA_GRID_INFO_LEN) values and returns FPTA_GRID_INFO_LEN
 * (negative on error); fpta_batch_grid_info keeps the round-1 contract: out[0..8], host double[9]. */
#define FPTA_GRID_INFO_LEN 19
int fpta_batch_grid_info_n(fpta_ctx* ctx, double* out, int32_t n_out);
int fpta_batch_grid_info(fpta_ctx* ctx, double* out);
/* Why the last batch did not take the gridded path (signal count, non-harmonic grid, error bound, cost,
 * n_real below the threshold, ...); "" when it did. Owned by the context, valid until the next batch. */
const char* fpta_batch_path_reason(const fpta_ctx* ctx);

/* ------------------------------------------------------------------ multi-device (one process)
 * one context per listed device (a device may repeat), the layout replicated on
 * each, realizations [real0, real0 + n_real) sharded contiguously (device g of G owns
 * [real0 + g n/G, real0 + (g+1) n/G)) and streamed in batches of <= batch realizations; only the
 * per-realization checksums (sum, sum of squares; fpta_batch_checksums order) come back, in global
 * realization order: checksums_out host [n_real][2]. The result is bit-identical for every device
 * count and batch size. Replaces running the reference's make_fake_array / add_* loop once per
 * realization (fakepta/fake_pta.py:648-668, fakepta/correlated_noises.py:153-160) over a large
 * ensemble. One-process-per-GPU jobs (torchrun) use fakepta_amd.batch.simulate_sharded instead. */
typedef struct fpta_multi fpta_multi;
int fpta_multi_create(int32_t n_dev, const int32_t* devices, fpta_multi** out);
int fpta_multi_destroy(fpta_multi* m);
const char* fpta_multi_last_error(const fpta_multi* m);
int fpta_multi_size(const fpta_multi* m);
/* The i-th device context (options, kernel statistics, downloads of its last block). */
fpta_ctx* fpta_multi_context(fpta_multi* m, int32_t i);
int fpta_multi_set_toas(fpta_multi* m, int32_t n_psr, const int64_t* offs, const double* toas,
                        const double* nu);
int fpta_multi_add_signal(fpta_multi* m, int32_t kind, int32_t n_modes, const double* f,
                          const double* amp, double idx, double freqf, const double* L,
                          const uint8_t* mask);
int fpta_multi_set_white(fpta_multi* m, const double* sigma, int64_t n_blocks,
                         const int64_t* block_offs, const int64_t* block_idx,
                         const double* ecorr_sigma);
int fpta_multi_set_option(fpta_multi* m, int32_t key, int64_t value);
int fpta_multi_synth(fpta_multi* m, uint64_t seed, int64_t real0, int64_t n_real, int32_t batch,
                     double* checksums_out);
/* How fpta_multi_synth brings the checksums to the host: FPTA_GATHER_RCCL keeps each device's
 * shard on the device and gathers them to device 0 with one ncclGather over xGMI (communicators from
 * ncclCommInitAll over the listed devices, made on first use; the devices must be distinct);
 * FPTA_GATHER_HOST copies each device's checksums into pinned host staging; FPTA_GATHER_AUTO (default) takes
 * RCCL when the devices are distinct. fpta_multi_last_gather: the route the last fpta_multi_synth took. */
#define FPTA_GATHER_AUTO 0
#define FPTA_GATHER_RCCL 1
#define FPTA_GATHER_HOST 2
int fpta_multi_set_gather(fpta_multi* m, int32_t mode);
int fpta_multi_last_gather(const fpta_multi* m);

/* ------------------------------------------------------------------ one process per GPU: RCCL
 * The library's own RCCL (ROCm 7.2, the same HIP runtime as the kernels) for realization-sharded jobs with one
 * process per GPU (fakepta_amd.batch.RcclComm; the reference loop that shards: correlated_noises.py:153-160).
 * Rank 0 makes the 128-byte unique id (fpta_comm_unique_id) and hands it to the other ranks out of band; every
 * rank then calls fpta_comm_init_rank on its context. Collectives run on the context's stream after all work
 * queued there, and return when their result is on the host. Only the job barrier / max of the elapsed time and
 * the checksum gather go through them: the data path has no collective. */
typedef struct fpta_comm fpta_comm;
#define FPTA_COMM_ID_BYTES 128
int fpta_comm_unique_id(void* id);
int fpta_comm_init_rank(fpta_ctx* ctx, int32_t nranks, int32_t rank, const void* id, fpta_comm** out);
int fpta_comm_destroy(fpta_comm* comm);
const char* fpta_comm_last_error(const fpta_comm* comm);
int fpta_comm_size(const fpta_comm* comm, int32_t* nranks, int32_t* rank);
/* *value (host) <- max over ranks of *value. Also the barrier of a timed region. */
int fpta_comm_max(fpta_comm* comm, double* value);
/* Every rank sends `count` doubles (host); rank 0 receives nranks * count, in rank order, into recv (host). */
int fpta_comm_gather(fpta_comm* comm, const double* send, int64_t count, double* recv);

/* ------------------------------------------------------------------ tuning / profiling */
#define FPTA_OPT_SYNTH_PATH 1     /* 0 auto, 1 direct (sincos per basis element), 2 fp64 MFMA, 3 fp64 VALU fused,
                                     4 gridded (real DFT to an oversampled phase grid + banded interpolation,
                                     harmonic grids only; aliasing error <= ~6e-12 relative at the defaults) */
#define FPTA_OPT_MFMA_MIN_REAL 2  /* auto: MFMA path when n_real >= this (default 16) */
#define FPTA_OPT_PROFILE 3        /* 1: time every batch kernel with HIP events on the ctx stream */
#define FPTA_OPT_ANCHOR 4         /* recurrence re-anchor interval in K-steps of 2 modes (0 = once per signal, default) */
#define FPTA_OPT_VALU_VARIANT 5   /* tile variant of the VALU fused kernel (0..5) */
#define FPTA_OPT_FUSE_WHITE 6     /* 1 (default): white/ECORR added in the synthesis epilogue; 0: separate pass */
#define FPTA_OPT_GRID_WIDTH 7     /* gridded path: interpolation kernel width in grid cells (default 15) */
#define FPTA_OPT_GRID_SIGMA 8     /* gridded path: grid oversampling x 100 (default 150) */
#define FPTA_OPT_GRID_MFMA 9      /* gridded path: bit 0 runs the DFT on fp64 MFMA (else fp64 VALU); the
                                     interpolation always runs on fp64 MFMA. Default 1. */
#define FPTA_OPT_FUSE_CHECKSUMS 10 /* 1: the gridded interpolation also writes per-(chunk, realization) partial
                                     sums (sum, sum of squares) of the block it stores, and
                                     fpta_batch_checksums reduces those (in a fixed order: deterministic, batch-
                                     split invariant) instead of re-reading the block. Default 0; other paths
                                     always take the full pass. */
#define FPTA_OPT_MIX_MFMA 11      /* ORF mixing of common signals for P >= 64 pulsars: 1 (default) on fp64 MFMA
                                     (k_mix_mfma), 0 the register-tiled fp64 VALU GEMM (k_mix_tiled) */
#define FPTA_OPT_OVERLAP 12       /* batch synthesis with several signals: 1 (default) draws each signal's
                                     coefficients on a second stream so the gridded DFT of one signal overlaps
                                     the draws of the next; 0 one stream. Results are identical. */
#define FPTA_OPT_INTERP_LDS 13    /* diagnostic builds only (FPTA_BUILD_DIAG; the product library refuses 1):
                                     gridded interpolation: 1 stages each chunk group's grid rows in LDS
                                     (k_grid_interp_lds) where every group fits and no white noise is fused;
                                     0 (default, faster on MI355X) the register-tiled k_grid_interp_mfma.
                                     Results are identical. */
#define FPTA_OPT_GRID_COALESCE 14 /* gridded path: 1 (default) sums, in coefficient space, the signals of a pulsar
                                     that share the base frequency w0 and the chromatic weight on every TOA (e.g.
                                     red noise and a common GWB on the pulsar's own span, or DM noise at a single
                                     radio frequency): they then share one grid and one interpolation band. Exact
                                     algebra (the sum is linear); results agree with 0 to rounding. */
#define FPTA_OPT_INTERP_WS 15     /* gridded interpolation: 1 (default) the warp-specialised k_grid_interp_ws
                                     (producer waves stage the operands in an LDS ring, compute waves only store,
                                     so stores never delay an operand load) for blocks without fused white noise
                                     or fused partial checksums, or k_grid_interp_ws2 (256-realization tiles, two
                                     workgroups per CU) when the padded realization count leaves fewer idle
                                     compute waves in 256- than in 512-realization tiles (C4: R = 256); 2 ws also
                                     for blocks with fused partial checksums; 3 ws2 for every plain block; 0 the
                                     register-pipelined k_grid_interp_mfma; 4 k_grid_interp_st for every block
                                     (compute waves hand their sums to storer waves through LDS; the storers add
                                     white noise / ECORR, store and reduce partial checksums). Results are
                                     identical. Variant builds only (FPTA_BUILD_DIAG): 0, 2, 3 (measured slower)
                                     and 4; the product library refuses them. */
#define FPTA_OPT_SIDE_SPLIT 16    /* pipelined gridded blocks (FPTA_OPT_OVERLAP): 1 the grid signal with the
                                     largest DFT, when it has no common (ORF-mixed) member, is drawn and
                                     transformed on a second side stream, beside the other signals' draws, mixing
                                     and DFT; 2 (default) the same, its DFT started after the common signals'
                                     draws + mixing queued on the first side stream (they get the room beside the
                                     previous block's interpolation first: C2 -1.3 %, C5 -1.4 %); 0 one side
                                     stream for all. Results are identical. 0 and 1 (measured slower): variant
                                     builds only (FPTA_BUILD_DIAG); the product library refuses them. */
#define FPTA_OPT_DFT_GEN 17       /* gridded path: 1 (default) a grid signal with a per-pulsar member draws its
                                     coefficients inside its DFT kernel (k_grid_dft_gen: Philox + Box-Muller into
                                     LDS, same counters and draws as k_gen); 0 k_gen writes them to the coefficient
                                     buffer and k_grid_dft_mfma reads them back. Same draws; sums agree to rounding.
                                     0 (measured slower): variant builds only (FPTA_BUILD_DIAG). */
#define FPTA_OPT_GEN_MIX 18       /* common signals of 64..256 pulsars (fp64 MFMA mixing): 2 (default) draws and ORF
                                     mixing in one kernel (k_gen_mix: normals in LDS, no zbuf round trip), one wave per
                                     16 realizations, 32 realizations per workgroup; 3 the same with 16 realizations
                                     per workgroup (a quarter of the LDS);
                                     1 waves of 32 realizations; 0 k_gen then k_mix_mfma. Same draws and products;
                                     results identical. 0, 1, 3 (equal or slower): variant builds only. */
#define FPTA_OPT_ASYNC_SUMS 19    /* streamed jobs (fpta_batch_synth_checksums, fpta_multi_synth): 1 a block's partial
                                     checksums are reduced on a stream of their own, beside the next block, into one
                                     of two partials buffers; 0 (default) on the context stream. Identical results.
                                     1 (measured slower): variant builds only (FPTA_BUILD_DIAG). */
#define FPTA_OPT_PART_GROUP 20    /* fused partial checksums (FPTA_OPT_FUSE_CHECKSUMS): the interpolation sums the partials
                                     of this many consecutive chunks (1 .. 16, default 16) in registers, in chunk order,
                                     and writes one {sum, sum of squares} row per group; the reduction then sums the
                                     groups in order. Deterministic and batch-split invariant for every value; the
                                     value changes the order of the additions (checksums agree to rounding). */
#define FPTA_OPT_INTERP_PSR 21    /* gridded path with one grid signal of <= 124 grid points whose coefficients the MFMA
                                     DFT would read from the coefficient buffer (e.g. C3's common GWB), <= 32 band
                                     rows and no fused white noise: 1 (default) k_grid_interp_psr (a workgroup makes
                                     one pulsar's grid for 64 realizations in LDS and interpolates the pulsar's chunks
                                     from it: no grid buffer, no separate DFT launch; pipelined blocks alternate two
                                     coefficient buffers); 0 the DFT + interpolation kernels. Results are identical. */
#define FPTA_OPT_INTERP_WR 22     /* diagnostic builds only (FPTA_BUILD_DIAG; the product library refuses 1): gridded
                                     plain blocks of <= 2 grid signals, R_pad a multiple of 256: 1 k_grid_interp_wr
                                     (each grid signal's band rows kept in a ring of LDS rows across consecutive chunks:
                                     only the rows the previous chunk did not hold are loaded; measured slower); 0
                                     (default) the other kernels. Results are identical. */
#define FPTA_OPT_INTERP_FUSED 23  /* gridded plain blocks (no white epilogue, no fused checksums) whose grids for 32
                                     realizations fit in LDS beside the draw ring with at most 4 DFT jobs of 32
                                     quarter-range rows and 2 grid signals (C2: 129 KB of grids): 1 (default)
                                     k_grid_fused (persistent workgroups, one per CU: 4 DFT waves draw and transform
                                     the next pulsar x 32 realizations into LDS while 4 interpolation waves read the
                                     current one: no grid buffer, no DFT launch), its interpolation on half-chunk
                                     bands (TOAs 0..15 and 16..31 of a chunk each with their own band rows) where
                                     that saves at least 3 % of the interpolation's MFMAs (C2: 11 %); 2 k_grid_fused
                                     on whole-chunk bands only; 3 half-chunk bands whenever the plan has them; 0 the
                                     DFT + interpolation kernels. Whole-chunk bands are bit-identical to the DFT +
                                     interpolation kernels; half-chunk bands group the band rows differently (sums
                                     agree to rounding). A layout k_grid_interp_psr serves keeps it. */
#define FPTA_OPT_FUSED_WHITE 24   /* (FPTA_VERSION 10100) gridded white / ECORR blocks, and plain blocks of three grid
                                     signals, whose grids for 16 realizations fit in LDS (C5: 884 rows, 113 KB): 1
                                     k_grid_fused_w (k_grid_fused's design with 16-realization items, up to 8 DFT
                                     jobs, the white / ECORR epilogue in the interpolation waves, ECORR epoch normals
                                     epoch-major); 0 (default) the DFT + interpolation kernels (measured faster on C5:
                                     1.74 vs 2.05 ms per block). Sums agree to rounding (two summation
                                     chains per chunk), white / ECORR terms identical. */
#define FPTA_OPT_FUSED_NEXT_MIX 25 /* (FPTA_VERSION 10200) pipelined gridded blocks on k_grid_fused (FPTA_OPT_OVERLAP 1)
                                     with one ORF-mixed common signal of 64 .. 128 pulsars drawn by k_gen_mix (C2's
                                     GWB): 1 (default) the kernel's waves with nothing left of their block draw and
                                     mix that signal for the next block of the same seed and size (first realization
                                     real0 + the stride from the block before when that is a whole number of blocks,
                                     else real0 + n_real) into the coefficient buffer that block reads; a batch_synth
                                     with that key then launches no k_gen_mix; after any other call the side streams
                                     wait for the kernel.
                                     0: every block runs k_gen_mix. Results are identical. */
int fpta_set_option(fpta_ctx* ctx, int32_t key, int64_t value);
/* Current value of option `key` (same keys as fpta_set_option). */
int fpta_get_option(fpta_ctx* ctx, int32_t key, int64_t* value);
/* Build flags of the loaded library: FPTA_BUILD_DEBUG when built with -DFPTA_DEBUG (make debug: per-launch
 * synchronisation and device-side bounds checks; never used for measurements); FPTA_BUILD_DIAG when built with
 * -DFPTA_DIAG_KERNELS (make variant: the measured-and-not-adopted diagnostic kernels, e.g. FPTA_OPT_INTERP_LDS). */
#define FPTA_BUILD_DEBUG 1
#define FPTA_BUILD_DIAG 2
int fpta_build_flags(void);
/* Kernel ids for fpta_kernel_stats */
#define FPTA_K_GEN 0
#define FPTA_K_MIX 1
#define FPTA_K_SYNTH 2
#define FPTA_K_WHITE 3
#define FPTA_K_DENSE 4 /* dense covariance: basis + Gram, Cholesky, solves, draws */
#define FPTA_K_GRID 5  /* gridded path: real-DFT grid values (k_grid_dft); its interpolation counts as SYNTH */
#define FPTA_K_N 6
/* Accumulated launches and HIP-event milliseconds of kernel `which` since the last reset. */
int fpta_kernel_stats(fpta_ctx* ctx, int32_t which, int64_t* count, double* total_ms);
int fpta_reset_stats(fpta_ctx* ctx);
int fpta_synchronize(fpta_ctx* ctx);

/* ------------------------------------------------------------------ test hooks */
/* Philox4x32-10 on device: ctr [n][4], key [2] -> out [n][4]. */
int fpta_debug_philox(fpta_ctx* ctx, int64_t n, const uint32_t* ctr, const uint32_t* key,
                      uint32_t* out);
/* The uniform -> normal map of every device draw (philox.h normals4) on n given Philox outputs: out[4 i + k] for the
 * words words[4 i .. 4 i + 3] (validation of the map on chosen words, e.g. its end points; oracle normals4). */
int fpta_debug_normals(fpta_ctx* ctx, int64_t n, const uint32_t* words, double* out);
/* Fill the last synthesized device block with `value` (tests: a later batch must overwrite every sample). */
int fpta_debug_fill_out(fpta_ctx* ctx, double value);

#ifdef __cplusplus
}
#endif
#endif /* FAKEPTA_AMD_H */
