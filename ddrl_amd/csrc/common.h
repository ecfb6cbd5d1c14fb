// Shared device helpers for the DDRL MI355X (gfx950 / CDNA4) kernels.
//
// Tiles are 16x16 fp32 on v_mfma_f32_16x16x4_f32 (exact f32, 64 FLOP/clk/SIMD).
// Lane l of a wave64: c = l & 15 (batch row inside a 16-row tile), q = l >> 4 (0..3).
//   A operand : A[i = c][k = q]            (16 x 4)
//   B operand : B[k = q][j = c]            (4 x 16)
//   C/D       : reg r -> C[row = 4q + r][col = c]
//
// Activations live "transposed" in registers: a 16(features) x 16(rows) C tile holds
// H^T[f = 16*fb + 4q + r][row = c].  That tile is directly the B operand of the next
// layer when the k-steps are enumerated as (fb, r) (lane l supplies feature 16fb+4q+r at
// k-step (fb, r)); the A operand (weights) is then read with the same permuted k.  So a
// whole MLP runs from registers with one LDS read per MFMA for the weights.
//
// LDS matrices with 64 columns are stored row-major with the column XOR-swizzled by the row
// inside its 16-column block (col' = col ^ swz(row), swz < 16), so every MFMA operand address
// is  (per-lane base) + (compile-time immediate).  A ds_read_b32 serves a wave in two groups of
// 32 lanes over 32 banks ((address / 4) mod 32), and every pattern below puts two 16-lane
// halves of a group on two different rows:
//   "R" reads  (row = 4s + q, col = 16t + c): forward weights, dW operands (rows 1 apart)
//   "W" access (row = 16u + c, col = 16t + 4q + r): activation stores, W2^T reads
//   "E" access (row = 16u + 4q + r, col = 16t + c): Adam's weights (rows 4 apart)
// Round 5 (DDRL_LDS_PAD, default 1): rows are DDRL_LRS = 80 floats apart (a
// stride of 16 banks) and row r starts 16 ((r >> 2) & 1) floats into its slot, so rows r and
// r + 1 and rows r and r + 4 start in opposite 16-bank halves; swz(row) = row & 0xB then makes
// the 8 rows of each half of a "W" group cover all 16 (col ^ swz) banks of the half: all three
// patterns are conflict-free.  The round-4 layout (64 floats per row, swz = ((row >> 1) & 7) << 1)
// left every one of them 2-way conflicted (SQ_LDS_BANK_CONFLICT 2.1x SQ_ACTIVE_INST_LDS).  The
// layout is a template parameter (PAD) of the helpers below, defaulting to DDRL_LDS_PAD: the
// fused update's A = 8 kernel without the row split keeps the compact one (its LDS budget has no
// room for the 25 % larger images).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

#define DDRL_H 64          // hidden width (fcnet_hiddens = [64, 64])
#ifndef DDRL_MB
#define DDRL_MB 128        // sgd_minibatch_size supported by the fused update kernel
#endif
#define DDRL_LOG2PI 1.8378770664093453

#ifndef DDRL_LDS_PAD
#define DDRL_LDS_PAD 1
#endif
constexpr bool kLdsPad = DDRL_LDS_PAD != 0;
__host__ __device__ constexpr int lds_rs(bool pad) { return pad ? 80 : 64; }           // floats per row
__host__ __device__ constexpr int lds_blk(bool pad) { return 16 * lds_rs(pad); }       // 16 rows
__host__ __device__ constexpr int lds_img(int rows, bool pad) { return rows * lds_rs(pad); }
#define DDRL_LBLK lds_blk(kLdsPad)
#define DDRL_LIMG(rows) lds_img(rows, kLdsPad)
template <bool PAD = kLdsPad>
__device__ __forceinline__ int swz(int row) { return PAD ? (row & 0xB) : (((row >> 1) & 7) << 1); }
template <bool PAD = kLdsPad>
__device__ __forceinline__ int lrow(int row) { return PAD ? row * 80 + ((row & 4) << 2) : row * 64; }
template <bool PAD = kLdsPad>
__device__ __forceinline__ int sidx(int row, int col) { return lrow<PAD>(row) + (col ^ swz<PAD>(row)); }

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Global-memory access through address space 1.  Pointers read from argument arrays are
// generic to the compiler, which then emits flat_* instructions; flat loads count against
// lgkmcnt as well as vmcnt, so every later LDS wait would also wait for them.
template <class T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ void gst(T* p, T v) {
  *(__attribute__((address_space(1))) T*)p = v;
}

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}
// LDS-DMA: 16 bytes per lane from gsrc into LDS at the wave-uniform byte address lds_dst +
// 16 * lane (global_load_lds_dwordx4).  Invisible to the compiler's s_waitcnt bookkeeping:
// the caller waits vmcnt itself before a barrier and the ds_reads of the data.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ floatx4 splat4(float v) { floatx4 r = {v, v, v, v}; return r; }

// tanh(x) = 2 / (1 + 2^(-2 log2(e) x)) - 1 with the hardware exp2 / reciprocal: 5
// instructions, absolute error ~1.5e-7 everywhere (no cancellation guard near 0 is needed at
// the 1e-5 parity bar: the error is absolute, like fp32 rounding of O(1) values); the
// saturated ends come out exactly: 2^(+inf) -> rcp 0 -> -1, 2^(-inf) -> 2 - 1 = 1.
__device__ __forceinline__ float tanh_fast(float x) {
#ifdef DDRL_ABL_NO_TANH   // ablation build (timing only)
  return x * 0.5f;
#endif
  const float e = __builtin_amdgcn_exp2f(fabsf(x) * 2.8853900817779268f);
  return copysignf(fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f), x);
}

// Cross-row pair sums with the gfx950 lane-swap instructions (VALU, no LDS round trip like
// the ds_bpermute a __shfl_xor becomes): v_permlane16_swap_b32 of v with itself leaves rows
// (0, 0, 2, 2) in one operand and (1, 1, 3, 3) in the other, so their sum is v + v[lane ^ 16];
// v_permlane32_swap_b32 likewise gives v + v[lane ^ 32].  Every lane gets the same bits as
// the shuffle form (the two addends are the same, in either order).
__device__ __forceinline__ float xor16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Sum over the 4 lanes that share c (q = 0..3): fixed order ((q0+q1)+(q2+q3)).
__device__ __forceinline__ float qsum(float v) { return xor32_sum(xor16_sum(v)); }

// Sum over the 16 lanes of a DPP row (lanes 16q .. 16q+15, i.e. over c for fixed q), every
// lane of the row receives the total.  Fixed order: xor 1, xor 2, half-mirror, mirror.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}

// Full wave64 sum, fixed order: the DPP row sum, then the rows in pairs (xor 16, xor 32).
__device__ __forceinline__ float wave_sum(float v) { return qsum(row16_sum(v)); }

// Transpose-reduce: v[0..15] in each lane of a DPP row (16 lanes, index c); afterwards lane c
// holds the sum over the row of v[c].  Four exchange steps (mirror, half-mirror, quad
// reverse, quad swap), each halving the live values: 15 DPP adds instead of 16 x 4.
__device__ __forceinline__ float row16_transpose_sum(float v[16]) {
  const int c = threadIdx.x & 15;
  // step 1: partner 15-c (bit 3 differs); keep the half selected by bit 3
  const bool b3 = c & 8, b2 = c & 4, b1 = c & 2, b0 = c & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float keep = b3 ? v[8 + k] : v[k];
    const float send = b3 ? v[k] : v[8 + k];
    v[k] = keep + dpp_mov<0x140>(send);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float keep = b2 ? v[4 + k] : v[k];
    const float send = b2 ? v[k] : v[4 + k];
    v[k] = keep + dpp_mov<0x141>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float keep = b1 ? v[2 + k] : v[k];
    const float send = b1 ? v[k] : v[2 + k];
    v[k] = keep + dpp_mov<0x1B>(send);   // quad_perm [3,2,1,0]
  }
  const float keep = b0 ? v[1] : v[0];
  const float send = b0 ? v[0] : v[1];
  return keep + dpp_mov<0xB1>(send);     // quad_perm [1,0,3,2]
}

// Full wave64 sum of a double, in registers: the DPP row sum (xor 1, xor 2, half-mirror,
// mirror) on both 32-bit halves, then the row pairs with the permlane swaps (xor 16, xor 32);
// every lane gets the same bits (no ds_bpermute round trips as __shfl_xor of a double takes).
template <int CTRL>
__device__ __forceinline__ double dpp_mov_d(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double xor_rows_sum_d(double v, bool x32) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  const auto rl = x32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                      : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = x32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                      : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double a = __builtin_bit_cast(double, ((unsigned long long)rh[0] << 32) | rl[0]);
  const double c = __builtin_bit_cast(double, ((unsigned long long)rh[1] << 32) | rl[1]);
  return a + c;
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_mov_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov_d<0x141>(v);  // row_half_mirror
  v += dpp_mov_d<0x140>(v);  // row_mirror
  return xor_rows_sum_d(xor_rows_sum_d(v, false), true);
}

// ------------------------------------------------------------------------------------
// Per-net weight image in LDS (one FFN branch: 2 hidden layers + linear head).
//   w1 : [kpad rows][64]  swizzled, rows >= d are zero
//   w2 : [64][64]         swizzled
//   b1, b2 : [64]
//   wo : [64][O] plain row-major (O <= 16),  bo : [O]
// ------------------------------------------------------------------------------------
struct NetLds {
  float* w1;
  float* w2;
  float* b1;
  float* b2;
  float* wo;
  float* bo;
  float* cup;   // update kernel, policy branch of the "cup" model: leg-coupling table [4][A]
};

// Per-lane LDS bases for the "R" pattern (row = 4s + q): rbase(v) = sidx(4v + q, c), valid for
// every s with s & 3 == v; the address of (s, block t) is
//   rbase(s & 3) + DDRL_LBLK * (s >> 2) + 16 * t.
template <bool PAD = kLdsPad>
__device__ __forceinline__ int rbase(int v) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  const int row = 4 * v + q;
  return lrow<PAD>(row) + (c ^ swz<PAD>(row));
}
// Per-lane LDS bases for the "W" pattern (row = 16u + c, col = 16t + 4q + r):
//   wbase(r) = sidx(c, 4q + r); address of (u, t) = wbase(r) + DDRL_LBLK u + 16 t.
template <bool PAD = kLdsPad>
__device__ __forceinline__ int wbase(int r) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  return lrow<PAD>(c) + ((4 * q + r) ^ swz<PAD>(c));
}

// Forward of one branch for RT row tiles (16 rows each) of this wave.
//   xop[t][s] : B operand of layer 1 at k-step s for row tile t, X[row = c][f = 4s + q]
//   KS1       : k-steps of layer 1 (ceil(d / 4)); W1 rows beyond d are zero in LDS
// Outputs h1[t][4], h2[t][4] (transposed activation tiles), out[t][O] (same in the 4 q-lanes).
// Every weight operand read from LDS feeds RT MFMAs.
template <int O, int KS1, int RT, bool PAD = kLdsPad>
__device__ __forceinline__ void ffn_fwd_rt(const NetLds& W, const float (*xop)[12],
                                           floatx4 (*h1)[4], floatx4 (*h2)[4], float (*out)[O]) {
  constexpr int BLK = lds_blk(PAD);
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const int o0 = 16 * ob + 4 * q;
    floatx4 b = {W.b1[o0], W.b1[o0 + 1], W.b1[o0 + 2], W.b1[o0 + 3]};
#pragma unroll
    for (int t = 0; t < RT; ++t) h1[t][ob] = b;
  }
  // Weight operands of k-step s + 2 are loaded while the MFMAs of step s issue (a 3-deep
  // register ring; the scheduling barrier keeps the compiler from sinking the loads next to
  // their MFMAs, which a single wave per SIMD cannot hide).
  const int rb[4] = {rbase<PAD>(0), rbase<PAD>(1), rbase<PAD>(2), rbase<PAD>(3)};
  auto ld1 = [&](int s, float* a) {
    const float* wp = W.w1 + rb[s & 3] + BLK * (s >> 2);
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) a[ob] = wp[16 * ob];
  };
  int fb_base[4];   // layer 2: row f = 16fb + 4q + r -> same swizzle as rbase with (4q + r) as the row
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * q + r;
    fb_base[r] = lrow<PAD>(row) + (c ^ swz<PAD>(row));
  }
  auto ld2 = [&](int k, float* a) {   // k = 4 fb + r
    const float* wp = W.w2 + fb_base[k & 3] + BLK * (k >> 2);
#pragma unroll
    for (int ob = 0; ob < 4; ++ob) a[ob] = wp[16 * ob];
  };
  float wr[3][4];
  {
    ld1(0, wr[0]);
    if (KS1 > 1) ld1(1, wr[1]);
#pragma unroll
    for (int s = 0; s < KS1; ++s) {
      if (s + 2 < KS1) ld1(s + 2, wr[(s + 2) % 3]);
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
#pragma unroll
        for (int t = 0; t < RT; ++t) h1[t][ob] = mfma4(wr[s % 3][ob], xop[t][s], h1[t][ob]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float wq[3][4];
  ld2(0, wq[0]);
  ld2(1, wq[1]);
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) h1[t][ob][r] = tanh_fast(h1[t][ob][r]);

#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const int o0 = 16 * ob + 4 * q;
    floatx4 b = {W.b2[o0], W.b2[o0 + 1], W.b2[o0 + 2], W.b2[o0 + 3]};
#pragma unroll
    for (int t = 0; t < RT; ++t) h2[t][ob] = b;
  }
  {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k + 2 < 16) ld2(k + 2, wq[(k + 2) % 3]);
#pragma unroll
      for (int ob = 0; ob < 4; ++ob)
#pragma unroll
        for (int t = 0; t < RT; ++t) h2[t][ob] = mfma4(wq[k % 3][ob], h1[t][k >> 2][k & 3], h2[t][ob]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int ob = 0; ob < 4; ++ob)
#pragma unroll
      for (int r = 0; r < 4; ++r) h2[t][ob][r] = tanh_fast(h2[t][ob][r]);

  // Linear head: partial dot over this lane's 16 features, then sum over q.
#pragma unroll
  for (int o = 0; o < O; ++o) {
    float acc[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[t] = 0.f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float wv = W.wo[(16 * fb + 4 * q + r) * O + o];
#pragma unroll
        for (int t = 0; t < RT; ++t) acc[t] = fmaf(h2[t][fb][r], wv, acc[t]);
      }
#pragma unroll
    for (int t = 0; t < RT; ++t) out[t][o] = qsum(acc[t]) + W.bo[o];
  }
}

// Single-tile form used by the rollout forward.
template <int O, int KS1>
__device__ __forceinline__ void ffn_branch_fwd(const NetLds& W, const float* xop,
                                               floatx4 h1[4], floatx4 h2[4], float out[O]) {
  ffn_fwd_rt<O, KS1, 1>(W, reinterpret_cast<const float (*)[12]>(xop),
                        reinterpret_cast<floatx4 (*)[4]>(h1), reinterpret_cast<floatx4 (*)[4]>(h2),
                        reinterpret_cast<float (*)[O]>(out));
}

// tanh derivative applied in place: d = d * (1 - h^2)
__device__ __forceinline__ void dtanh_inplace(floatx4 d[4], const floatx4 h[4]) {
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) d[b][r] = d[b][r] * (1.f - h[b][r] * h[b][r]);
}

// dH2^T = Wo . dout^T   (VALU; dout identical in the 4 q-lanes of a row)
template <int O>
__device__ __forceinline__ void head_bwd(const NetLds& W, const float* dout, floatx4 dh[4]) {
  const int q = (threadIdx.x & 63) >> 4;
#pragma unroll
  for (int fb = 0; fb < 4; ++fb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* wrow = W.wo + (16 * fb + 4 * q + r) * O;
      float acc = 0.f;
#pragma unroll
      for (int o = 0; o < O; ++o) acc = fmaf(wrow[o], dout[o], acc);
      dh[fb][r] = acc;
    }
}

// dH1^T = W2 . dZ2^T   (MFMA, A = W2[f = 16fb + c][o = 16ob + 4q + r], B = dZ2 tile regs)
template <int RT, bool PAD = kLdsPad>
__device__ __forceinline__ void layer2_bwd_rt(const NetLds& W, const floatx4 (*dz2)[4], floatx4 (*dh1)[4]) {
  constexpr int BLK = lds_blk(PAD);
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) dh1[t][fb] = splat4(0.f);
  const int wb[4] = {wbase<PAD>(0), wbase<PAD>(1), wbase<PAD>(2), wbase<PAD>(3)};
  auto ld = [&](int k, float* a) {   // k = 4 ob + r (operands prefetched two steps ahead)
    const float* wp = W.w2 + wb[k & 3] + 16 * (k >> 2);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) a[fb] = wp[BLK * fb];
  };
  float wr[3][4];
  ld(0, wr[0]);
  ld(1, wr[1]);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k + 2 < 16) ld(k + 2, wr[(k + 2) % 3]);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int t = 0; t < RT; ++t) dh1[t][fb] = mfma4(wr[k % 3][fb], dz2[t][k >> 2][k & 3], dh1[t][fb]);
    __builtin_amdgcn_sched_barrier(0);
  }
}
__device__ __forceinline__ void layer2_bwd(const NetLds& W, const floatx4 dz2[4], floatx4 dh1[4]) {
  layer2_bwd_rt<1>(W, reinterpret_cast<const floatx4 (*)[4]>(dz2), reinterpret_cast<floatx4 (*)[4]>(dh1));
}

// Write a transposed activation tile set (rows 16*tile + c, features 16fb+4q+r) into an
// LDS swizzled image (DDRL_LIMG(rows) floats) as row-major activations.
__device__ __forceinline__ void store_act(float* buf, int tile, const floatx4 v[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float* p = buf + wbase(r) + DDRL_LBLK * tile;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) p[16 * fb] = v[fb][r];
  }
}

// Feature-major activation image for the weight-gradient GEMMs: T[f][b], 128 rows b per
// feature plus 8 floats of padding (stride FM_LD = 136 == 8 mod 64 makes every ds_read_b128
// of the dW operands bank-conflict free).  The GEMM's k index is the row b; lane (c, q)
// takes rows 16u + 4q .. 16u + 4q + 3 for k-group u, i.e. ONE ds_read_b128 per operand per
// four MFMAs.
// (A 64-row image uses stride 72, also 8 mod 64.)
#define FM_LD 136
template <int LD = FM_LD>
__device__ __forceinline__ void store_act_fm(float* buf, int tile, const floatx4 v[4]) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  float* p = buf + (4 * q) * LD + 16 * tile + c;
#pragma unroll
  for (int fb = 0; fb < 4; ++fb)
#pragma unroll
    for (int r = 0; r < 4; ++r) p[(16 * fb + r) * LD] = v[fb][r];
}

// NT_ tiles dW[f = 16 fa_i + 4q + r][o = 16 fo + c] (one fo, NT_ fa's) over NROWS rows.
template <int NROWS, int NT_, int LD = NROWS + 8>
__device__ __forceinline__ void dw_tiles_fm(const float* A, const float* B, const int* fa, int fo, floatx4* out) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < NT_; ++i) out[i] = splat4(0.f);
  const float* bp = B + (16 * fo + c) * LD + 4 * q;
  const float* ap[NT_];
#pragma unroll
  for (int i = 0; i < NT_; ++i) ap[i] = A + (16 * fa[i] + c) * LD + 4 * q;
  // operands of row group u + 1 are loaded while the MFMAs of group u issue
  constexpr int NU = NROWS / 16;
  floatx4 bv[2], av[2][NT_];
  bv[0] = *reinterpret_cast<const floatx4*>(bp);
#pragma unroll
  for (int i = 0; i < NT_; ++i) av[0][i] = *reinterpret_cast<const floatx4*>(ap[i]);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    if (u + 1 < NU) {
      bv[(u + 1) & 1] = *reinterpret_cast<const floatx4*>(bp + 16 * (u + 1));
#pragma unroll
      for (int i = 0; i < NT_; ++i) av[(u + 1) & 1][i] = *reinterpret_cast<const floatx4*>(ap[i] + 16 * (u + 1));
    }
#pragma unroll
    for (int i = 0; i < NT_; ++i)
#pragma unroll
      for (int v = 0; v < 4; ++v) out[i] = mfma4(av[u & 1][i][v], bv[u & 1][v], out[i]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One 16x16 tile of dW = A^T B over NROWS rows:  dW[f = 16fa + 4q + r][o = 16fo + c]
//   A image: [rows][64] swizzled (A[b][f]),  B image: [rows][64] swizzled (B[b][o])
template <int NROWS>
__device__ __forceinline__ floatx4 dw_tile(const float* A, const float* B, int fa, int fo) {
  floatx4 acc = splat4(0.f);
  const int rb[4] = {rbase(0), rbase(1), rbase(2), rbase(3)};
  const float* ap = A + 16 * fa;
  const float* bp = B + 16 * fo;
#pragma unroll 2
  for (int u = 0; u < NROWS / 16; ++u) {
#pragma unroll
    for (int v = 0; v < 4; ++v) acc = mfma4(ap[rb[v] + DDRL_LBLK * u], bp[rb[v] + DDRL_LBLK * u], acc);
  }
  return acc;
}

// Two independent 16x16 dW tiles in one pass (two accumulation chains interleaved, so a
// single wave per SIMD keeps the MFMA pipe busy despite the 40-cycle dependent latency).
template <int NROWS>
__device__ __forceinline__ void dw_tile2(const float* A, const float* B, int fa0, int fo0, int fa1, int fo1,
                                         floatx4& t0, floatx4& t1) {
  floatx4 a0 = splat4(0.f), a1 = splat4(0.f);
  const int rb[4] = {rbase(0), rbase(1), rbase(2), rbase(3)};
  const float *ap0 = A + 16 * fa0, *bp0 = B + 16 * fo0, *ap1 = A + 16 * fa1, *bp1 = B + 16 * fo1;
#pragma unroll 2
  for (int u = 0; u < NROWS / 16; ++u) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int o = rb[v] + DDRL_LBLK * u;
      a0 = mfma4(ap0[o], bp0[o], a0);
      a1 = mfma4(ap1[o], bp1[o], a1);
    }
  }
  t0 = a0;
  t1 = a1;
}

// Same with B given as a plain [rows][O] (O <= 16) row-major array, zero beyond O.
template <int O, int NROWS>
__device__ __forceinline__ floatx4 dw_tile_head(const float* A, const float* D, int fa) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  floatx4 acc = splat4(0.f);
  const int rb[4] = {rbase(0), rbase(1), rbase(2), rbase(3)};
  const float* ap = A + 16 * fa;
  const bool cv = c < O;
  const float* dp = D + q * O + (cv ? c : 0);
#pragma unroll 2
  for (int u = 0; u < NROWS / 16; ++u) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float bv = cv ? dp[(16 * u + 4 * v) * O] : 0.f;
      acc = mfma4(ap[rb[v] + DDRL_LBLK * u], bv, acc);
    }
  }
  return acc;
}
