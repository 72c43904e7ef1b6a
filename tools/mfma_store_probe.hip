// Probe (not part of the library): does an fp64 MFMA stream overlap a streaming-store stream on MI355X?
// Each workgroup has 8 waves (2 per SIMD), one workgroup per CU, persistent. Per "tile" a compute wave issues
// kMfmaPerTile v_mfma_f64_16x16x4_f64 on 16 independent accumulators and a store wave writes kStorePerTile 1 KB
// rows (16 B per lane) into a 2 GiB buffer, the interpolation kernel's ratio (160 MFMAs per 32 stores).
//   mode 0: every wave computes only         mode 1: every wave stores only
//   mode 2: waves 0-3 compute, 4-7 store     mode 3: every wave computes then stores (the interpolation's shape)
//   mode 4: waves 0-3 compute then store, waves 4-7 idle (one wave per SIMD)
//   mode 5: as mode 3, and every 16-MFMA step of a compute wave loads its operands (five 1 KB dbl2 loads from a 64 KB
//           L2-resident table, two steps ahead: the interpolation's operand stream)
//   mode 6: as mode 5 with the operands read from LDS (ds_read_b128) instead
//   mode 7: as mode 5 without stores
//   mode 9: as mode 8 with the operands read from a 256 MiB table (rows re-read ~5 times, as the grid rows are)
//   mode 10: as mode 9 without stores
//   modes 11-14: mode 9 with the stores' cache policy bits: nt / sc1 / sc0 sc1 / nt sc0 sc1
//   mode 8: as mode 5 with the interpolation's store addresses: out[r][t] with a row pitch of 200,000 doubles, a
//           wave's 128 realization rows (r0 + 32 m + 2 (lg + 4 g) + h) x the 32 TOAs of its chunk, chunks walked
//           as the persistent tiles are
// Prints per mode the time and the MFMA / store rates. hipcc --offload-arch=gfx950 -O3 tools/mfma_store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int kMfmaPerTile = 160, kStorePerTile = 32;

template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(double* __restrict__ out, long long n_rows, int tiles, double seed,
                                                 double* __restrict__ sink, const double* __restrict__ table,
                                                 const double* __restrict__ big) {
  __shared__ double lds[8192];  // 64 KB operand image (mode 6)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const bool compute = MODE == 0 || MODE == 3 || MODE >= 5 || ((MODE == 2 || MODE == 4) && wave < 4);
  const bool store = MODE == 1 || MODE == 3 || MODE == 5 || MODE == 6 || MODE == 8 || MODE == 9 || MODE >= 11 ||
                     (MODE == 2 && wave >= 4) ||
                     (MODE == 4 && wave < 4);
  constexpr bool LOADS = MODE >= 5;  // modes 5-10
  if (MODE == 6) {
    for (int i = threadIdx.x; i < 8192; i += 512) lds[i] = table[i];
    __syncthreads();
  }
  if (!compute && !store) return;
  d4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = d4{table[(lane + 64 * i) & 8191], table[(lane + 64 * i + 1) & 8191], 0.5, -0.25};
  const double a = table[(lane * 37 + wave * 11) & 8191] + seed * 1e-3, b = table[(lane * 53 + 5) & 8191] - seed * 1e-3;
  long long row = ((long long)blockIdx.x * 8 + wave) * 4;
  const long long stride = (long long)gridDim.x * 8 * 4;
  // operand stream: step k of tile t reads five 1 KB pieces of the table (wave- and step-dependent offsets)
  auto opnd = [&](int t, int k, dbl2 (&o)[5]) {
    const int base = ((t * 10 + k) * 5 + wave * 3) & 63;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int off = ((base + j) & 63) * 128 + 2 * lane;
      if (MODE == 6) {
        o[j] = *(const dbl2*)(lds + off);
      } else if (MODE >= 9) {  // 9 .. 14
        // 1 KB rows of a 256 MiB table: a tile walks ~37 rows of a 2.4 MB window that moves 1/5 of itself per tile
        const long long row = ((long long)blockIdx.x * 997 + (long long)t * 480 + (wave & 3) * 7 + k * 4 + j) % 262144;
        o[j] = *(const dbl2*)(big + row * 128 + 2 * lane);
      } else {
        o[j] = *(const dbl2*)(table + off);
      }
    }
  };
  dbl2 o0[5], o1[5];
  if (LOADS) {
    opnd(0, 0, o0);
    opnd(0, 1, o1);
  }
  for (int t = 0; t < tiles; ++t) {
    if (compute) {
      for (int k = 0; k < kMfmaPerTile / 16; ++k) {
        double x = a, y = b;
        if (LOADS) {
          dbl2(&o)[5] = (k & 1) ? o1 : o0;
          x = o[0].x + o[1].y + o[2].x;
          y = o[3].y + o[4].x;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[i], 0, 0, 0);
        if (LOADS) {
          const int nk = k + 2 < kMfmaPerTile / 16 ? k + 2 : k + 2 - kMfmaPerTile / 16;
          const int nt = k + 2 < kMfmaPerTile / 16 ? t : t + 1;
          if (k & 1) opnd(nt, nk, o1);
          else opnd(nt, nk, o0);
        }
      }
    }
    if (store) {
      if (MODE == 8 || MODE == 9 || MODE >= 11) {
        // tile t of this wave: chunk (blockIdx.x + gridDim.x * t) mod 6250, realization block (wave & 3) x 128 of
        // 1024 (waves 4-7 the same blocks on the next chunk), 200,000 TOAs per row
        const long long chunk = ((long long)blockIdx.x * 2 + (wave >> 2) + (long long)gridDim.x * 2 * t) % 6250;
        const int r0 = (wave & 3) * 128, lr = lane & 15, lg = lane >> 4;
#pragma unroll
        for (int s = 0; s < kStorePerTile; ++s) {
          const int i = s >> 2, g = s & 3;
          const int r = r0 + 32 * (i >> 1) + 2 * (lg + 4 * g) + (i & 1);
          const double v = acc[s & 15][s >> 4];
          dbl2* dst = (dbl2*)(out + (long long)r * 200000 + chunk * 32 + 2 * lr);
          const dbl2 val = dbl2{v, v + 1.0};
          if (MODE == 11) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(dst), "v"(val) : "memory");
          else if (MODE == 12) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(val) : "memory");
          else if (MODE == 13) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dst), "v"(val) : "memory");
          else if (MODE == 14) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(val) : "memory");
          else *dst = val;
        }
      } else
#pragma unroll
      for (int s = 0; s < kStorePerTile; ++s) {
        // 4 rows of 256 B per instruction (the interpolation's store shape), rows spread over the buffer
        const long long r = (row * 4 + (lane >> 4) + (long long)s * 4 * stride * tiles) & (n_rows - 1);
        const double v = acc[s & 15][s >> 4];
        *(dbl2*)(out + r * 32 + 2 * (lane & 15)) = dbl2{v, v + 1.0};
      }
      row += stride;
    }
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5678) sink[0] = s;  // keeps the MFMAs live
}

int main() {
  const long long bytes = 2LL << 30;
  const long long n_rows = bytes / 256;  // 256-B rows
  double *out, *sink, *table, *big;
  if (hipMalloc(&big, 256LL << 20) != hipSuccess || hipMemset(big, 0x3f, 256LL << 20) != hipSuccess) return 1;
  if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess ||
      hipMalloc(&table, 8192 * sizeof(double)) != hipSuccess)
    return 1;
  {  // random operands: zero data lets the chip hold a higher clock (MI355X_MICROARCH.md, DVFS)
    static double h[8192];
    unsigned long long x = 88172645463325252ull;
    for (int i = 0; i < 8192; ++i) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      h[i] = (double)(x >> 11) * (1.0 / 9007199254740992.0) - 0.5;
    }
    if (hipMemcpy(table, h, sizeof(h), hipMemcpyHostToDevice) != hipSuccess) return 1;
  }
  int n_cu = 256;
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int tiles = 400;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kernel, const char* name, int compute_waves, int store_waves) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kernel, dim3(n_cu), dim3(512), 0, 0, out, n_rows, tiles, 1.0 + rep, sink, table, big);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double mfma_flops = 2048.0 * kMfmaPerTile * tiles * compute_waves * n_cu;
      const double st_bytes = 1024.0 * kStorePerTile * tiles * store_waves * n_cu;
      if (rep == 2)
        printf("%-34s %8.3f ms  %6.1f TF/s  %6.2f TB/s\n", name, ms, mfma_flops / ms / 1e9, st_bytes / ms / 1e9);
    }
  };
  run(probe<0>, "mode 0 compute only (8 waves)", 8, 0);
  run(probe<1>, "mode 1 store only (8 waves)", 0, 8);
  run(probe<2>, "mode 2 4 compute + 4 store waves", 4, 4);
  run(probe<3>, "mode 3 compute then store (8 waves)", 8, 8);
  run(probe<4>, "mode 4 compute then store (4 waves)", 4, 4);
  run(probe<5>, "mode 5 + operand loads (global)", 8, 8);
  run(probe<6>, "mode 6 + operand loads (LDS)", 8, 8);
  run(probe<7>, "mode 7 operand loads, no stores", 8, 0);
  run(probe<8>, "mode 8 mode 5, interpolation addresses", 8, 8);
  run(probe<9>, "mode 9 mode 8, 256 MiB operand table", 8, 8);
  run(probe<10>, "mode 10 mode 9 without stores", 8, 0);
  run(probe<11>, "mode 11 mode 9, nt stores", 8, 8);
  run(probe<12>, "mode 12 mode 9, sc1 stores", 8, 8);
  run(probe<13>, "mode 13 mode 9, sc0 sc1 stores", 8, 8);
  run(probe<14>, "mode 14 mode 9, sc0 sc1 nt stores", 8, 8);
  run(probe<1>, "mode 1 store only (8 waves)", 0, 8);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  return 0;
}
