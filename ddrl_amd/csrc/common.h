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
// LDS matrices with 64 columns are stored row-major, 64 floats per row, with the column
// XOR-swizzled by the row:  col' = col ^ swz(row),  swz(row) = ((row >> 1) & 7) << 1.
// The XOR only touches bits 1..3, so it never moves a column out of its 16-column block
// and every MFMA operand address is  (per-lane base) + (compile-time immediate):
//   "R" reads  (row = 4s + q, col = 16t + c): forward weights, dW operands -> 2-way at most
//   "W" access (row = 16u + c, col = 16t + 4q + r): activation stores, W2^T reads -> 2-way
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define DDRL_H 64          // hidden width (fcnet_hiddens = [64, 64])
#define DDRL_MB 128        // sgd_minibatch_size supported by the fused update kernel
#define DDRL_LOG2PI 1.8378770664093453

__device__ __forceinline__ int swz(int row) { return ((row >> 1) & 7) << 1; }
__device__ __forceinline__ int sidx(int row, int col) { return row * 64 + (col ^ swz(row)); }

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ floatx4 splat4(float v) { floatx4 r = {v, v, v, v}; return r; }

// Sum over the 4 lanes that share c (q = 0..3): fixed order ((q0+q1)+(q2+q3)).
__device__ __forceinline__ float qsum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// Full wave64 sum, fixed butterfly order.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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
};

// Per-lane LDS bases for the "R" pattern (row = 4s + q): rbase(v) = (4v + q)*64 + (c ^ swz),
// valid for every s with s & 3 == v; the address of (s, block t) is
//   rbase(s & 3) + 1024 * (s >> 2) + 16 * t.
__device__ __forceinline__ int rbase(int v) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  const int row = 4 * v + q;
  return row * 64 + (c ^ swz(row));
}
// Per-lane LDS bases for the "W" pattern (row = 16u + c, col = 16t + 4q + r):
//   wbase(r) = c*64 + ((4q + r) ^ swz(c)); address of (u, t) = wbase(r) + 1024 u + 16 t.
__device__ __forceinline__ int wbase(int r) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  return c * 64 + ((4 * q + r) ^ swz(c));
}

// Forward of one branch for the 16 rows of this wave.
//   xop[s] : B operand of layer 1 at k-step s, i.e. X[row = c][f = 4s + q] (0 beyond d)
//   KS1    : k-steps of layer 1 (ceil(d / 4)); W1 rows beyond d are zero in LDS
// Outputs h1[4], h2[4] (transposed activation tiles), out[O] (identical in the 4 q-lanes).
template <int O, int KS1>
__device__ __forceinline__ void ffn_branch_fwd(const NetLds& W, const float* xop,
                                               floatx4 h1[4], floatx4 h2[4], float out[O]) {
  const int lane = threadIdx.x & 63, q = lane >> 4;
#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const int o0 = 16 * ob + 4 * q;
    floatx4 b = {W.b1[o0], W.b1[o0 + 1], W.b1[o0 + 2], W.b1[o0 + 3]};
    h1[ob] = b;
  }
  {
    const int rb[4] = {rbase(0), rbase(1), rbase(2), rbase(3)};
#pragma unroll
    for (int s = 0; s < KS1; ++s) {
      const float* wp = W.w1 + rb[s & 3] + 1024 * (s >> 2);
      const float bx = xop[s];
#pragma unroll
      for (int ob = 0; ob < 4; ++ob) h1[ob] = mfma4(wp[16 * ob], bx, h1[ob]);
    }
  }
#pragma unroll
  for (int ob = 0; ob < 4; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) h1[ob][r] = tanhf(h1[ob][r]);

#pragma unroll
  for (int ob = 0; ob < 4; ++ob) {
    const int o0 = 16 * ob + 4 * q;
    floatx4 b = {W.b2[o0], W.b2[o0 + 1], W.b2[o0 + 2], W.b2[o0 + 3]};
    h2[ob] = b;
  }
  {
    // row f = 16fb + 4q + r  ->  same swizzle as rbase with (4q + r) as the row
    const int c = lane & 15;
    int fb_base[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * q + r;
      fb_base[r] = row * 64 + (c ^ swz(row));
    }
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float* wp = W.w2 + fb_base[r] + 1024 * fb;
        const float bx = h1[fb][r];
#pragma unroll
        for (int ob = 0; ob < 4; ++ob) h2[ob] = mfma4(wp[16 * ob], bx, h2[ob]);
      }
  }
#pragma unroll
  for (int ob = 0; ob < 4; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) h2[ob][r] = tanhf(h2[ob][r]);

  // Linear head: partial dot over this lane's 16 features, then sum over q.
#pragma unroll
  for (int o = 0; o < O; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = fmaf(h2[fb][r], W.wo[(16 * fb + 4 * q + r) * O + o], acc);
    out[o] = qsum(acc) + W.bo[o];
  }
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
__device__ __forceinline__ void layer2_bwd(const NetLds& W, const floatx4 dz2[4], floatx4 dh1[4]) {
#pragma unroll
  for (int fb = 0; fb < 4; ++fb) dh1[fb] = splat4(0.f);
  const int wb[4] = {wbase(0), wbase(1), wbase(2), wbase(3)};
#pragma unroll 2
  for (int ob = 0; ob < 4; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float bx = dz2[ob][r];
      const float* wp = W.w2 + wb[r] + 16 * ob;
#pragma unroll
      for (int fb = 0; fb < 4; ++fb) dh1[fb] = mfma4(wp[1024 * fb], bx, dh1[fb]);
    }
}

// Write a transposed activation tile set (rows 16*tile + c, features 16fb+4q+r) into an
// LDS [128][64] swizzled image as row-major activations.
__device__ __forceinline__ void store_act(float* buf, int tile, const floatx4 v[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float* p = buf + wbase(r) + 1024 * tile;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) p[16 * fb] = v[fb][r];
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
    for (int v = 0; v < 4; ++v) acc = mfma4(ap[rb[v] + 1024 * u], bp[rb[v] + 1024 * u], acc);
  }
  return acc;
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
      acc = mfma4(ap[rb[v] + 1024 * u], bv, acc);
    }
  }
  return acc;
}
