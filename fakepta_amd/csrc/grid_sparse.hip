// Gridded synthesis, interpolation step on the fp64 VALU:
//   out[r][t] = sum_s ch_s(t) sum_{i<w} phi_s(t, i) G_s[J_s(t) + i][r]
// with each TOA touching only the grid rows of its own chunk window (the dense-band MFMA form,
// k_grid_interp_mfma, multiplies every TOA of a chunk by 4-row steps of the whole band).
//
//   lane    = one realization; wave = 64 realizations x the TOAs of a work item (<= kSparseChunks chunks
//             of <= 16 consecutive TOAs of one pulsar)
//   window  = the WS_s = w + D_s grid rows of signal s that the chunk touches, in registers (one double
//             per row and lane, a 512-byte coalesced row load per wave); D_s = the largest offset of a
//             TOA's first row from its chunk's base row for that signal (<= kSparseD, host plan)
//   weights = per (signal, TOA) records of kSparseRec window slots (ch * mask * phi, zero outside the
//             TOA's w rows): the step's records go to the wave's LDS slice, lane l reads slot l mod 16
//             (and 16 + l mod 4), and v_fmac_f64 DPP row_newbcast:j hands slot j to every lane, so the
//             wave-uniform weights cost neither scalar-load latency per TOA nor LDS bandwidth per FMA
//   partial sums over signals accumulate in the wave's LDS tile T[16 TOAs][64 realizations], read
//   transposed at the end of a chunk so every store instruction writes four full 128-byte lines
// The next step's window rows and records are loaded while the current step computes (two register
// sets). White noise / ECORR (fake_pta.py:201-230) initialise the first signal's pass.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_common.h"
#include "fpta_internal.h"
#include "philox.h"

namespace fpta {

constexpr int kSparsePitch = 66;                 // LDS tile row pitch (doubles): conflict-free transposed reads
constexpr int kSparseWS = kSparseRec;            // largest window (w + D <= kSparseRec slots)
constexpr int kStepRec = kGridTT * kSparseRec;   // record doubles of one step (one chunk, one signal)
constexpr int kRecPerLane = (kStepRec + 63) / 64;

// one realization per lane: the pair stream of oracle.white_normals_rpairs, this lane's half
__device__ __forceinline__ double sparse_white(int64_t t, int64_t g, uint32_t k0, uint32_t k1) {
  const u32x4 c = {(uint32_t)t, kWhitePsrWord, kWhiteStream, (uint32_t)(g >> 1)};
  double z0, z1;
  box_muller(philox4x32_10(c, k0, k1), z0, z1);
  return (g & 1) ? z1 : z0;
}

// One TOA against a WS-row window: a0 / a1 += sum_j slot_j * win[j] (even slots into a0, odd into a1: two
// independent FMA chains). v_fmac_f64 with DPP row_newbcast:(j mod 16) broadcasts lane j mod 16 of every
// 16-lane row of the weight register (slots 0..15 in wa, 16.. in wb) into the FMA, so every lane uses slot j.
// One asm block per TOA (the compiler separates consecutive asm blocks by a wait state); it opens with the wait
// states of the DPP read-after-VALU-write hazard, in case the compiler copied a weight register just before.
// (generated: one specialisation per window size 12..20)
template <int WS>
__device__ __forceinline__ void window_dot(double& a0, double& a1, double wa, double wb,
                                           const double (&win)[kSparseWS]);

template <>
__device__ __forceinline__ void window_dot<12>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  (void)wb;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]));
}

template <>
__device__ __forceinline__ void window_dot<13>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  (void)wb;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]));
}

template <>
__device__ __forceinline__ void window_dot<14>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  (void)wb;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]));
}

template <>
__device__ __forceinline__ void window_dot<15>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  (void)wb;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]), [g14] "v"(win[14]));
}

template <>
__device__ __forceinline__ void window_dot<16>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  (void)wb;
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]), [g14] "v"(win[14]), [g15] "v"(win[15]));
}

template <>
__device__ __forceinline__ void window_dot<17>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wb], %[g16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [wb] "v"(wb), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]), [g14] "v"(win[14]), [g15] "v"(win[15]), [g16] "v"(win[16]));
}

template <>
__device__ __forceinline__ void window_dot<18>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wb], %[g16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wb], %[g17] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [wb] "v"(wb), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]), [g14] "v"(win[14]), [g15] "v"(win[15]), [g16] "v"(win[16]), [g17] "v"(win[17]));
}

template <>
__device__ __forceinline__ void window_dot<19>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wb], %[g16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wb], %[g17] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wb], %[g18] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [wb] "v"(wb), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]), [g14] "v"(win[14]), [g15] "v"(win[15]), [g16] "v"(win[16]), [g17] "v"(win[17]), [g18] "v"(win[18]));
}

template <>
__device__ __forceinline__ void window_dot<20>(double& a0, double& a1, double wa, double wb,
                                               const double (&win)[kSparseWS]) {
  
  asm("s_nop 1\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wa], %[g14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wa], %[g15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wb], %[g16] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wb], %[g17] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[wb], %[g18] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[wb], %[g19] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1)
      : [wa] "v"(wa), [wb] "v"(wb), [g0] "v"(win[0]), [g1] "v"(win[1]), [g2] "v"(win[2]), [g3] "v"(win[3]), [g4] "v"(win[4]), [g5] "v"(win[5]), [g6] "v"(win[6]), [g7] "v"(win[7]), [g8] "v"(win[8]), [g9] "v"(win[9]), [g10] "v"(win[10]), [g11] "v"(win[11]), [g12] "v"(win[12]), [g13] "v"(win[13]), [g14] "v"(win[14]), [g15] "v"(win[15]), [g16] "v"(win[16]), [g17] "v"(win[17]), [g18] "v"(win[18]), [g19] "v"(win[19]));
}

template <bool WHITE>
__global__ __launch_bounds__(256, 3) void k_grid_interp_sparse(SynthArgs a, const int4* __restrict__ chunks,
                                                               const int4* __restrict__ work, int32_t n_tiles,
                                                               int32_t n_rsb, SparseSegs ss, int32_t R_pad,
                                                               double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double T[4][kGridTT][kSparsePitch];
  __shared__ __attribute__((aligned(16))) double RL[4][kRecPerLane * 64];
  // XCD-aware: workgroup b runs on XCD b % 8, which walks a contiguous range of tiles (the realization blocks
  // of a work item and the work items of a pulsar share records and grid rows in that XCD's L2)
  const int per = gridDim.x >> 3;
  const int tile = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (tile >= n_tiles) return;
  const int wi = __builtin_amdgcn_readfirstlane(tile / n_rsb);
  const int rsb = __builtin_amdgcn_readfirstlane(tile - wi * n_rsb);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int r0 = (rsb * 4 + wave) * 64;
  if (r0 >= R_pad) return;  // whole wave (no cross-wave synchronisation below: the LDS slices are per wave)
  FPTA_DCHECK(r0 + 64 <= R_pad, "k_grid_interp_sparse realization block", r0 + 64, R_pad + 1);
  const int4 wk = work[wi];  // {first chunk, chunks, pulsar, 0}
  const int c0 = __builtin_amdgcn_readfirstlane(wk.x);
  const int p = __builtin_amdgcn_readfirstlane(wk.z);
  const int nseg = ss.n;
  const int Q = __builtin_amdgcn_readfirstlane(wk.y) * nseg;
  const int64_t pbase = a.offs[p];
  double(*Tw)[kSparsePitch] = T[wave];
  double* __restrict__ rl_ = RL[wave];
  const int rl = r0 + lane;

  // step q = (chunk q / nseg, signal q % nseg): window rows and the chunk's weight records into registers
  auto load = [&](int q, double(&win)[kSparseWS], double(&rs)[kRecPerLane]) {
    const int cq = __builtin_amdgcn_readfirstlane(q / nseg);
    const int s = __builtin_amdgcn_readfirstlane(q - cq * nseg);
    const SparseSegDev& sd = ss.s[s];
    // Every load is unconditional (rows past the signal's window are valid grid rows; the record array is padded
    // by one step): a fixed number of loads per step lets the compiler wait for exactly the older step's loads
    // (vmcnt(N)) instead of draining the next step's prefetch (vmcnt(0)) before every TOA.
    int j = __builtin_amdgcn_readfirstlane(sd.base[c0 + cq]);
    const double* __restrict__ G = sd.g + (int64_t)p * sd.nf * R_pad + rl;
#pragma unroll
    for (int i = 0; i < kSparseWS; ++i) {
      win[i] = G[(int64_t)j * R_pad];
      if (++j == sd.nf) j = 0;
    }
    const int4 ci = chunks[c0 + cq];
    const double* __restrict__ rec = sd.rec + (pbase + ci.y) * kSparseRec;
#pragma unroll
    for (int k = 0; k < kRecPerLane; ++k) rs[k] = rec[lane + 64 * k];
  };

  auto compute = [&](int q, const double(&win)[kSparseWS], const double(&rs)[kRecPerLane]) {
    const int cq = __builtin_amdgcn_readfirstlane(q / nseg);
    const int s = __builtin_amdgcn_readfirstlane(q - cq * nseg);
    const SparseSegDev& sd = ss.s[s];
    const int4 ci = chunks[c0 + cq];
    const int cnt = __builtin_amdgcn_readfirstlane(ci.z);
    const int64_t t0 = pbase + __builtin_amdgcn_readfirstlane(ci.y);
    const int ws = __builtin_amdgcn_readfirstlane(sd.ws);
    // the step's records to the wave's LDS slice (the previous step's reads of it are done: in-order DS)
#pragma unroll
    for (int k = 0; k < kRecPerLane; ++k) rl_[lane + 64 * k] = rs[k];
    const int sa = lane & 15, sb = 16 + (lane & 3);
    // TOA loop, two TOAs per trip with two register sets: the next TOA's weights and partial sum are read from
    // LDS before the current TOA's FMAs, so the LDS latency overlaps the FMA chain. Every read is unconditional
    // (index clamped to the chunk; an odd count recomputes the last TOA from the same inputs, an idempotent
    // rewrite) so the compiler can count the outstanding LDS operations instead of draining them.
    auto toas = [&](auto wsc, auto firstc) {
      constexpr int WS = decltype(wsc)::value;
      constexpr bool FIRST = decltype(firstc)::value;
      auto rd_a = [&](int tt) { return rl_[tt * kSparseRec + sa]; };
      auto rd_b = [&](int tt) { return WS > 16 ? rl_[tt * kSparseRec + sb] : 0.0; };
      auto rd_t = [&](int tt) { return FIRST ? 0.0 : Tw[tt][lane]; };
      auto one = [&](int tt, double wa, double wb, double acc) {
        double acc1 = 0.0;
        if constexpr (WHITE && FIRST) {
          const int64_t tg = t0 + tt;
          if (a.w_sigma) acc = a.w_sigma[tg] * sparse_white(tg, a.real0 + rl, a.k0, a.k1);
          const int ep = a.w_block_of ? a.w_block_of[tg] : -1;
          if (ep >= 0 && rl < a.n_real) acc = fma(a.w_esig[ep], a.w_zb[(int64_t)rl * a.w_nblocks + ep], acc);
        }
        window_dot<WS>(acc, acc1, wa, wb, win);
        Tw[tt][lane] = acc + acc1;
      };
      double wa0 = rd_a(0), wb0 = rd_b(0), ta0 = rd_t(0);
      for (int tt = 0; tt < cnt; tt += 2) {
        const int t1 = min(tt + 1, cnt - 1), t2 = min(tt + 2, cnt - 1);
        const double wa1 = rd_a(t1), wb1 = rd_b(t1), ta1 = rd_t(t1);
        __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the FMA chain that does not need them
        one(tt, wa0, wb0, ta0);
        wa0 = rd_a(t2);
        wb0 = rd_b(t2);
        ta0 = rd_t(t2);
        __builtin_amdgcn_sched_barrier(0);
        one(t1, wa1, wb1, ta1);
      }
    };
    auto toas_ws = [&](auto wsc) {
      if (s == 0)
        toas(wsc, std::true_type{});
      else
        toas(wsc, std::false_type{});
    };
    switch (ws) {  // wave-uniform, once per step: the FMA count of a TOA is the signal's window size
      case 12: toas_ws(std::integral_constant<int, 12>{}); break;
      case 13: toas_ws(std::integral_constant<int, 13>{}); break;
      case 14: toas_ws(std::integral_constant<int, 14>{}); break;
      case 15: toas_ws(std::integral_constant<int, 15>{}); break;
      case 16: toas_ws(std::integral_constant<int, 16>{}); break;
      case 17: toas_ws(std::integral_constant<int, 17>{}); break;
      case 18: toas_ws(std::integral_constant<int, 18>{}); break;
      case 19: toas_ws(std::integral_constant<int, 19>{}); break;
      default: toas_ws(std::integral_constant<int, 20>{}); break;
    }
    if (s == nseg - 1) {  // chunk complete: transposed store, 16 lanes per realization row (128-byte lines)
      const int tt = lane & 15;
      if (tt < cnt) {
        double* __restrict__ ocol = out + t0 + tt;
#pragma unroll 4
        for (int jr = 0; jr < 16; ++jr) {
          const int rr = 4 * jr + (lane >> 4);
          const int r = r0 + rr;
          if (r < a.n_real) ocol[(int64_t)r * a.ldo] = Tw[tt][rr];  // batch blocks are written, not accumulated
        }
      }
    }
  };

  // the prefetches are unconditional (the last ones re-read the final step): with the same loads on every path
  // the compiler can wait for the older register set alone instead of draining all outstanding loads
  double wa[kSparseWS], wb[kSparseWS], ra[kRecPerLane], rb[kRecPerLane];
  load(0, wa, ra);
  for (int q = 0; q < Q; q += 2) {
    load(min(q + 1, Q - 1), wb, rb);
    compute(q, wa, ra);
    load(min(q + 2, Q - 1), wa, ra);
    if (q + 1 < Q) compute(q + 1, wb, rb);
  }
}

// Per (signal, TOA) record of window slots: rec[t][j] = ch(t) mask(t) phi((d - (j - o)) / (w / 2)) for
// 0 <= j - o < w, zero elsewhere, o = the TOA's first row offset in its chunk window (off_of[t]); the
// chromatic factor and the backend mask folded in, as in k_grid_weights.
__global__ __launch_bounds__(256) void k_grid_records(SegDesc sd, int64_t n_toa, const double* __restrict__ nu,
                                                      const double* __restrict__ d_of,
                                                      const int32_t* __restrict__ off_of, int32_t w, double beta,
                                                      double* __restrict__ rec) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n_toa) return;
  double ch = chrom_factor(sd.freqf, nu[t], sd.idx);
  if (sd.mask && !sd.mask[t]) ch = 0.0;
  const double d = d_of[t];
  const int o = off_of[t];
  const double hw = 0.5 * (double)w;
  double* dst = rec + t * kSparseRec;
  for (int j = 0; j < kSparseRec; ++j) {
    const int i = j - o;
    const double z = (d - (double)i) / hw;
    const double s = 1.0 - z * z;
    dst[j] = (i >= 0 && i < w && s > 0.0) ? ch * exp(beta * (sqrt(s) - 1.0)) : 0.0;
  }
}

hipError_t launch_grid_records(hipStream_t st, const SegDesc& sd, int64_t n_toa, const double* nu,
                               const double* d_of, const int32_t* off_of, int32_t w, double beta, double* rec) {
  hipLaunchKernelGGL(k_grid_records, dim3((unsigned)((n_toa + 255) / 256)), dim3(256), 0, st, sd, n_toa, nu, d_of,
                     off_of, w, beta, rec);
  return hipGetLastError();
}

bool sparse_width_supported(int32_t w) { return w >= 12 && w + kSparseD <= kSparseWS; }

hipError_t launch_grid_interp_sparse(hipStream_t st, const SynthArgs& a, const int4* chunks, const int4* work,
                                     int32_t n_work, const SparseSegs& ss, int32_t R_pad) {
  if (R_pad % 128 != 0 || n_work <= 0 || ss.n <= 0 || ss.n > kGridMaxSeg) return hipErrorInvalidValue;
  for (int s = 0; s < ss.n; ++s)
    if (ss.s[s].ws < 12 || ss.s[s].ws > kSparseWS) return hipErrorInvalidValue;
  const int32_t n_rsb = (R_pad + 255) / 256;
  const int64_t tiles = (int64_t)n_work * n_rsb;
  const int64_t grid = (tiles + 7) / 8 * 8;
  if (grid > 0x7FFFFFFF) return hipErrorInvalidValue;
  if (a.w_on)
    hipLaunchKernelGGL((k_grid_interp_sparse<true>), dim3((unsigned)grid), dim3(256), 0, st, a, chunks, work,
                       (int32_t)tiles, n_rsb, ss, R_pad, a.out);
  else
    hipLaunchKernelGGL((k_grid_interp_sparse<false>), dim3((unsigned)grid), dim3(256), 0, st, a, chunks, work,
                       (int32_t)tiles, n_rsb, ss, R_pad, a.out);
  return hipGetLastError();
}

}  // namespace fpta
