// HIP kernels for gfx950 (MI355X): the dense-covariance path.
//
//   k_cov_basis    G^T = (chromatic Fourier basis * sqrt(psd df))^T, k-major   (fake_pta.py:414-417)
//   k_gemm_tn      C (op)= A B on v_mfma_f64_16x16x4_f64, 64 x 64 output tiles:
//                    covariance  C = G G^T (+ diag white)   (fake_pta.py:418, :493-513, :517)
//                    Cholesky trailing update C22 -= L21 L21^T
//                    batched draws X = Z L^T (L lower-triangular)
//   k_potrf_block  Cholesky of one 64 x 64 diagonal block in LDS
//   k_trsm_panel   panel solve L21 = A21 L11^-T, one row per thread
//   k_chol_solve   C y = r by forward/backward substitution on the factor (one workgroup), fused with
//                  the Wiener output r - white * y = red_cov C^-1 r      (fake_pta.py:520-523)
//   k_dense_normals Philox normals for the batched draws
//
// The covariance is symmetric positive (semi-)definite; the factorisation reads and writes only its
// lower triangle and zeroes the upper triangle of each diagonal block, so the factor can be used as
// a dense lower-triangular matrix by k_gemm_tn.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "fpta_internal.h"
#include "philox.h"

namespace fpta {

// ----------------------------------------------------------------------------- k_cov_basis
// GT[2m][t] = ch_s(t) sqrt(w_m) cos((2 pi f_m) t), GT[2m+1][t] = ... sin(...), s = segment of mode m.
// The phase is evaluated exactly as the reference's 2*np.pi*f[i]*toas (fake_pta.py:416).
// grid (ldn / 256, K_pad / 2): rows of modes >= n_modes and columns t >= n are written as zeros.
__global__ __launch_bounds__(256) void k_cov_basis(const double* __restrict__ toas, const double* __restrict__ nu,
                                                   int64_t n, const double* __restrict__ f,
                                                   const double* __restrict__ sw, const int32_t* __restrict__ seg_of,
                                                   const double* __restrict__ seg_idx,
                                                   const double* __restrict__ seg_freqf, int32_t n_modes,
                                                   double* __restrict__ GT, int64_t ldn) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int m = blockIdx.y;
  double c = 0.0, s = 0.0;
  if (t < n && m < n_modes) {
    const int sg = seg_of[m];
    const double a = chrom_factor(seg_freqf[sg], nu[t], seg_idx[sg]) * sw[m];
    double sn, cn;
    sincos((2.0 * M_PI * f[m]) * toas[t], &sn, &cn);
    c = a * cn;
    s = a * sn;
  }
  GT[(int64_t)(2 * m) * ldn + t] = c;
  GT[(int64_t)(2 * m + 1) * ldn + t] = s;
}

// ----------------------------------------------------------------------------- k_gemm_tn
// C[i][j] (op)= sum_k A[i][k] B[k][j] with A given k-major (A_T[k][i], lda) and B k-major
// (B_T[k][j], ldb) or, with b_rows, row-major B^T (Brow[j][k], ldb). Workgroup = 64 x 64 tile,
// 4 waves of 32 x 32 = 2 x 2 MFMA fragments (cdna_hip_programming.md §3 fragment maps:
// A[i = l&15][k = l>>4], B[k = l>>4][j = l&15], D row = (l>>4) + 4 reg, col = l&15). Operands
// must be readable up to the tile edges (buffers padded to 64) and to 4*k4 rows; values there
// only reach outputs outside [0,m) x [0,n), which are not stored.
struct GemmTN {
  const double* a;
  int64_t lda;
  const double* b;
  int64_t ldb;
  double* c;
  int64_t ldc;
  int64_t m, n;        // stored output extent
  int32_t k4;          // reduction length / 4
  int32_t tiles_n;     // full grid: tiles per output row block (blockIdx.x = bi * tiles_n + bj)
  int32_t tile0;       // lower grid: first tile (rows and columns)
  int32_t lower;       // 1: blockIdx.x enumerates the tiles bi >= bj >= tile0 (triangular order)
  int32_t mode;        // 0 store, 1 subtract, 2 store + mirror (C symmetric)
  int32_t b_rows;      // B operand given as rows of B^T
  int32_t b_tri;       // B[k][j] == 0 for k > j: stop each wave's reduction after its last column
  const double* diag;  // modes 0/2: added on the diagonal (may be null)
};

__global__ __launch_bounds__(256) void k_gemm_tn(GemmTN g) {
  int bi, bj;
  if (g.lower) {
    const int64_t b = blockIdx.x;
    int q = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
    while ((int64_t)q * (q + 1) / 2 > b) --q;
    while ((int64_t)(q + 1) * (q + 2) / 2 <= b) ++q;
    bi = g.tile0 + q;
    bj = g.tile0 + (int)(b - (int64_t)q * (q + 1) / 2);
  } else {
    bi = blockIdx.x / g.tiles_n;
    bj = blockIdx.x % g.tiles_n;
  }
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int lr = lane & 15;
  const int lg = lane >> 4;
  const int64_t i0 = (int64_t)bi * 64 + (wave >> 1) * 32;
  const int64_t j0 = (int64_t)bj * 64 + (wave & 1) * 32;
  int k4 = g.k4;
  if (g.b_tri) k4 = min<int64_t>(k4, (j0 + 32) / 4);

  d4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = d4{0.0, 0.0, 0.0, 0.0};

  const double* pa = g.a + (int64_t)lg * g.lda + i0 + lr;
  const int64_t sa = 4 * g.lda;
  if (g.b_rows) {
    const double* pb0 = g.b + (j0 + lr) * g.ldb + lg;
    const double* pb1 = pb0 + 16 * g.ldb;
    for (int k = 0; k < k4; ++k, pa += sa, pb0 += 4, pb1 += 4) {
      const double a0 = pa[0], a1 = pa[16], b0 = *pb0, b1 = *pb1;
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
  } else {
    const double* pb = g.b + (int64_t)lg * g.ldb + j0 + lr;
    const int64_t sb = 4 * g.ldb;

    for (int k = 0; k < k4; ++k, pa += sa, pb += sb) {
      const double a0 = pa[0], a1 = pa[16], b0 = pb[0], b1 = pb[16];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
  }

  const bool mirror = g.mode == 2 && bi != bj;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int64_t j = j0 + y * 16 + lr;
      if (j >= g.n) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t i = i0 + x * 16 + lg + 4 * q;
        if (i >= g.m) continue;
        double v = acc[x][y][q];
        double* o = g.c + i * g.ldc + j;
        if (g.mode == 1) {
          *o -= v;
        } else {
          if (g.diag && i == j) v += g.diag[i];
          *o = v;
          if (mirror) g.c[j * g.ldc + i] = v;
        }
      }
    }
}

// ----------------------------------------------------------------------------- k_potrf_block
// Cholesky of the diagonal block C[k0:k0+nb, k0:k0+nb] (nb = min(64, n - k0)), right-looking in
// LDS. Writes the factor to the lower triangle and zeros above the diagonal of the block. A
// non-positive pivot sets *info = (row + 1) once (the host reports it); the factor is then invalid.
__global__ __launch_bounds__(256) void k_potrf_block(double* __restrict__ C, int64_t ldc, int64_t n, int64_t k0,
                                                     int* __restrict__ info) {
  __shared__ double A[64][65];
  const int nb = (int)min<int64_t>(64, n - k0);
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int i = e >> 6, j = e & 63;
    A[i][j] = (i < nb && j <= i) ? C[(k0 + i) * ldc + k0 + j] : (i == j ? 1.0 : 0.0);
  }
  __syncthreads();
  for (int j = 0; j < nb; ++j) {
    const double d = A[j][j];
    if (!(d > 0.0) && threadIdx.x == 0) atomicCAS(info, 0, (int)(k0 + j + 1));
    const double s = sqrt(d);
    __syncthreads();  // every thread has read A[j][j]
    for (int i = j + 1 + (int)threadIdx.x; i < nb; i += 256) A[i][j] /= s;
    if (threadIdx.x == 0) A[j][j] = s;
    __syncthreads();
    const int m = nb - j - 1;
    for (int e = threadIdx.x; e < m * m; e += 256) {
      const int ii = e / m, ll = e - ii * m;
      if (ll <= ii) A[j + 1 + ii][j + 1 + ll] = fma(-A[j + 1 + ii][j], A[j + 1 + ll][j], A[j + 1 + ii][j + 1 + ll]);
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < nb * nb; e += 256) {
    const int i = e / nb, j = e - i * nb;
    C[(k0 + i) * ldc + k0 + j] = j <= i ? A[i][j] : 0.0;
  }
}

// ----------------------------------------------------------------------------- k_trsm_panel
// Rows i >= k0 + 64 of the panel: x L11^T = a, i.e. x_l = (a_l - sum_{j<l} x_j L11[l][j]) / L11[l][l],
// right-looking so the 64 updates of each step are independent FMAs. One row per thread, held in
// registers. Writes the row back into C and k-major into PT[l][i] for the trailing update.
__global__ __launch_bounds__(256) void k_trsm_panel(double* __restrict__ C, int64_t ldc, int64_t n, int64_t k0,
                                                    double* __restrict__ PT, int64_t ldp) {
  __shared__ double LT[64][64];  // LT[l][j] = L11[j][l]
  __shared__ double inv[64];
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int j = e >> 6, l = e & 63;
    LT[l][j] = l <= j ? C[(k0 + j) * ldc + k0 + l] : 0.0;
  }
  if (threadIdx.x < 64) inv[threadIdx.x] = 1.0 / C[(k0 + threadIdx.x) * ldc + k0 + threadIdx.x];
  __syncthreads();
  const int64_t i = k0 + 64 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double* row = C + i * ldc + k0;
  double x[64];
#pragma unroll
  for (int l = 0; l < 64; ++l) x[l] = row[l];
#pragma unroll
  for (int l = 0; l < 64; ++l) {
    x[l] *= inv[l];
#pragma unroll
    for (int j = l + 1; j < 64; ++j) x[j] = fma(-x[l], LT[l][j], x[j]);
  }
#pragma unroll
  for (int l = 0; l < 64; ++l) {
    row[l] = x[l];
    PT[(int64_t)l * ldp + i] = x[l];
  }
}

// ----------------------------------------------------------------------------- k_chol_solve
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One workgroup of 1024 threads (16 waves): L u = r, L^T y = u on the lower factor, then
// out = r - white * y (= red_cov C^-1 r, since C = red_cov + diag(white)). y is global scratch:
// the waves of one workgroup share the CU's L1, so __syncthreads() orders its reads and writes.
__global__ __launch_bounds__(1024) void k_chol_solve(const double* __restrict__ C, int64_t ldc, int64_t n,
                                                     const double* __restrict__ r, const double* __restrict__ white,
                                                     double* __restrict__ y, double* __restrict__ out) {
  __shared__ double Ld[64][65];
  __shared__ double part[16][64];
  __shared__ double rhs[64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nblk = (int)((n + 63) / 64);
  // forward: L u = r (u kept in y)
  for (int b = 0; b < nblk; ++b) {
    const int64_t r0 = (int64_t)b * 64;
    const int nb = (int)min<int64_t>(64, n - r0);
    for (int e = threadIdx.x; e < nb * 64; e += 1024) {
      const int i = e >> 6, j = e & 63;
      Ld[i][j] = (j <= i) ? C[(r0 + i) * ldc + r0 + j] : 0.0;
    }
    for (int q = 0; q < 4; ++q) {
      const int ii = wave + 16 * q;
      double s = 0.0;
      if (ii < nb) {
        const double* row = C + (r0 + ii) * ldc;
        for (int64_t k = lane; k < r0; k += 64) s = fma(row[k], y[k], s);
      }
      s = wave_sum(s);
      if (lane == 0) rhs[ii] = s;
    }
    __syncthreads();
    if (wave == 0) {
      double v = lane < nb ? r[r0 + lane] - rhs[lane] : 0.0;
      double u = 0.0;
      for (int j = 0; j < nb; ++j) {
        const double uj = __shfl(v, j) / Ld[j][j];
        if (lane == j) u = uj;
        if (lane > j && lane < nb) v = fma(-Ld[lane][j], uj, v);
      }
      if (lane < nb) y[r0 + lane] = u;
    }
    __syncthreads();
  }
  // backward: L^T y = u
  for (int b = nblk - 1; b >= 0; --b) {
    const int64_t r0 = (int64_t)b * 64;
    const int nb = (int)min<int64_t>(64, n - r0);
    for (int e = threadIdx.x; e < nb * 64; e += 1024) {
      const int i = e >> 6, j = e & 63;
      Ld[i][j] = (j <= i) ? C[(r0 + i) * ldc + r0 + j] : 0.0;
    }
    double s = 0.0;  // lane = column r0 + lane of the block; wave strides the rows below it
    if (lane < nb)
      for (int64_t i = r0 + 64 + wave; i < n; i += 16) s = fma(C[i * ldc + r0 + lane], y[i], s);
    part[wave][lane] = s;
    __syncthreads();
    if (wave == 0) {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < 16; ++w) t += part[w][lane];
      double v = lane < nb ? y[r0 + lane] - t : 0.0;
      double yy = 0.0;
      for (int j = nb - 1; j >= 0; --j) {
        const double yj = __shfl(v, j) / Ld[j][j];
        if (lane == j) yy = yj;
        if (lane < j) v = fma(-Ld[j][lane], yj, v);
      }
      if (lane < nb) y[r0 + lane] = yy;
    }
    __syncthreads();
  }
  for (int64_t i = threadIdx.x; i < n; i += 1024) out[i] = white ? fma(-white[i], y[i], r[i]) : y[i];
}

// ----------------------------------------------------------------------------- k_dense_normals
// ZT[t][r] for the batched dense draws: quad_normal(t, DENSE stream, g), g = real0 + r (oracle:
// quad_normals(..., stream=DENSE_STREAM)). Zero outside
// [0,n) x [0,n_real). grid (ldz / 256, rows).
__global__ __launch_bounds__(256) void k_dense_normals(int64_t n, int32_t n_real, int64_t real0, uint32_t k0,
                                                       uint32_t k1, double* __restrict__ ZT, int64_t ldz) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t t = blockIdx.y;
  double z = 0.0;
  if (t < n && r < n_real) {
    z = quad_normal((uint64_t)t, kDenseStream, (uint64_t)(real0 + r), k0, k1);
  }
  ZT[t * ldz + r] = z;
}

// ----------------------------------------------------------------------------- launchers
hipError_t launch_cov_basis(hipStream_t st, const double* toas, const double* nu, int64_t n, const double* f,
                            const double* sw, const int32_t* seg_of, const double* seg_idx, const double* seg_freqf,
                            int32_t n_modes, int32_t k_pad, double* GT, int64_t ldn) {
  if (ldn % 256 || k_pad % 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_cov_basis, dim3((unsigned)(ldn / 256), (unsigned)(k_pad / 2)), dim3(256), 0, st, toas, nu, n,
                     f, sw, seg_of, seg_idx, seg_freqf, n_modes, GT, ldn);
  return hipGetLastError();
}

hipError_t launch_gemm_tn(hipStream_t st, const double* a, int64_t lda, const double* b, int64_t ldb, bool b_rows,
                          bool b_tri, double* c, int64_t ldc, int64_t m, int64_t n, int32_t k4, int32_t lower,
                          int32_t tile0, int32_t mode, const double* diag) {
  GemmTN g{a, lda, b, ldb, c, ldc, m, n, k4, 0, tile0, lower, mode, b_rows ? 1 : 0, b_tri ? 1 : 0, diag};
  const int64_t tm = (m + 63) / 64, tn = (n + 63) / 64;
  int64_t blocks;
  if (lower) {
    const int64_t t = tm - tile0;  // m == n for the lower grid
    if (t <= 0) return hipSuccess;
    blocks = t * (t + 1) / 2;
  } else {
    g.tiles_n = (int32_t)tn;
    blocks = tm * tn;
  }
  if (blocks <= 0) return hipSuccess;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gemm_tn, dim3((unsigned)blocks), dim3(256), 0, st, g);
  return hipGetLastError();
}

hipError_t launch_potrf_block(hipStream_t st, double* C, int64_t ldc, int64_t n, int64_t k0, int* info) {
  hipLaunchKernelGGL(k_potrf_block, dim3(1), dim3(256), 0, st, C, ldc, n, k0, info);
  return hipGetLastError();
}

hipError_t launch_trsm_panel(hipStream_t st, double* C, int64_t ldc, int64_t n, int64_t k0, double* PT,
                             int64_t ldp) {
  const int64_t rows = n - k0 - 64;
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_trsm_panel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, C, ldc, n, k0, PT, ldp);
  return hipGetLastError();
}

hipError_t launch_chol_solve(hipStream_t st, const double* C, int64_t ldc, int64_t n, const double* r,
                             const double* white, double* y, double* out) {
  hipLaunchKernelGGL(k_chol_solve, dim3(1), dim3(1024), 0, st, C, ldc, n, r, white, y, out);
  return hipGetLastError();
}

hipError_t launch_dense_normals(hipStream_t st, int64_t n, int64_t rows, int32_t n_real, int64_t real0, uint32_t k0,
                                uint32_t k1, double* ZT, int64_t ldz) {
  if (ldz % 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_dense_normals, dim3((unsigned)(ldz / 256), (unsigned)rows), dim3(256), 0, st, n, n_real, real0,
                     k0, k1, ZT, ldz);
  return hipGetLastError();
}

}  // namespace fpta
