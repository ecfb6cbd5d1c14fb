// a13-a17: fused PPO minibatch SGD for the fcnet policy/value model (persistent kernel).
//
// One launch runs the whole 10-epoch schedule of up to 4 policies.  Per policy the policy
// branch (fc_1, fc_2, fc_out) and the value branch (fc_value_1, fc_value_2, value_out) each run
// on KSP = 2 workgroups (the row split: 64 rows of the 128-row minibatch each, one 16-row MFMA
// tile per wave, one wave per SIMD); blocks p, p + 8, p + 16, p + 24 (the dispatcher's
// round robin puts them on one XCD, checked after every launch through HW_REG_XCC_ID).
//   * the row halves swap their partial gradients every step through tagged 16-byte
//     granules in the XCD's L2 (plain stores, sc1 polls; ppo_ffn_atomic.hip builds the same
//     source with relaxed agent-scope atomics, valid for any placement);
//   * the branches share only tf.clip_by_global_norm: one tagged 8-byte norm^2 granule
//     each way per step.  Tags carry a 12-bit launch epoch, so no memset per launch.
// Per minibatch step (RLlib TrainTFMultiGPU: row = shuffle[perm[e][b] * 128 + i]):
//   the step's records were gathered into LDS by LDS-DMA during the previous step;
//   forward (MFMA 16x16x4 f32, activations in registers, weights in a swizzled LDS image);
//   PPOLoss per row (RLlib 1.0) and dL/d(outputs); the policy head's dWo = H2^T dout as one
//   more 16x16 tile of the dW2 MFMA stream and dH2 = Wo dout^T on MFMA, the value head's by
//   DPP transpose-reductions; layer-2 backward from registers; H1/dZ2 then X/dZ1 through
//   feature-major LDS images for the weight-gradient tiles (K = 64 rows), owned per wave;
//   partner exchange; global-norm clip; tf1 Adam (m / v in the owning lanes' registers, two
//   elements per packed instruction, weights updated in place in LDS).
// ppo_ffn_impl.h holds the device code; DESIGN.md section 3 the measurements behind it.
#define DDRL_FFN_KSP 2   // the KSP = 1 kernels: ppo_ffn_k1.hip
#include "ppo_ffn_impl.h"


size_t gx_bytes(int P) { return sizeof(unsigned long long) * (size_t)P * 2 * 2 * 2 * GX_MAX_PAIRS * 256 * 2; }

// ------------------------------------------------------------------------------------
// DDP apply: tf.clip_by_global_norm + tf1 Adam on an all-reduced flat gradient.
// K = ceil(n / 1024) workgroups of 1024 threads.  Every workgroup computes the global norm
// itself, in one fixed order (thread t sums elements t + 1024 k in k order, DPP within the
// wave, the 16 wave sums in order), so all of them hold the same clip scale; workgroup b
// then updates elements [1024 b, 1024 b + 1024).  The gradient is read K times, from L2.
// beta_pow[2] counts the workgroups that have read beta1^t / beta2^t; the last to arrive
// advances them and resets the count (the next launch on the stream starts after this one).
// The grid is 8 K blocks of which only those on XCD `xcd` (block mod 8, the dispatcher's
// round robin) work: the update kernel of the same policy runs on that XCD, so the gradient
// it wrote and the weights it reads next stay in that XCD's L2 (spreading the slices over
// all XCDs cost the next gradient launch 3 us of weight misses).
// K = 0: one workgroup with a strided loop (vectors beyond 32 K elements).
// ------------------------------------------------------------------------------------
template <int K>
__global__ void __launch_bounds__(1024) k_apply_adam(const float* __restrict__ grad, int n,
                                                     float* theta, float* m, float* v,
                                                     float* beta_pow, UpdateHyper h, float gscale, int xcd,
                                                     const int* err) {
  __shared__ float red[16];
  if (K > 0 && (int)(blockIdx.x & 7) != xcd) return;   // not on the policy's XCD
  if (*err) return;   // the step's gradient launch failed: leave the weights (the host restores them)
  const int tid = threadIdx.x;
  const float b1p = beta_pow[0], b2p = beta_pow[1];
  const int i0 = K > 0 ? (int)(blockIdx.x >> 3) * 1024 + tid : tid;
  const bool own = i0 < n;
  float mm = 0.f, vv = 0.f, th = 0.f, go = 0.f;
  if (K > 0 && own) {   // this workgroup's slice, issued with the norm loads
    mm = m[i0];
    vv = v[i0];
    th = theta[i0];
    go = grad[i0];
  }
  float ss = 0.f;
  if constexpr (K > 0) {
    float g[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = tid + 1024 * k;
      g[k] = i < n ? grad[i] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float gi = g[k] * gscale;   // gscale: 1 / ranks of the "local" data-parallel mode
      ss += gi * gi;
    }
  } else {
    for (int i = tid; i < n; i += 1024) {
      const float gi = grad[i] * gscale;
      ss += gi * gi;
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  if (tid == 0) {
    float tot = 0.f;
    for (int i = 0; i < 16; ++i) tot += red[i];
    const float gn = sqrtf(tot);
    red[0] = h.grad_clip * fminf(1.f / gn, 1.f / h.grad_clip);
  }
  __syncthreads();
  const float scale = red[0];
  const float alpha = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float c1 = 1.f - h.b1, c2 = 1.f - h.b2;
  auto adam = [&](float gr, float& a, float& b, float& t) {
    const float gg = (gr * gscale) * scale;
    a = a + (gg - a) * c1;
    b = b + (gg * gg - b) * c2;
    t = t - (a * alpha) / (sqrtf(b) + h.eps);
  };
  if constexpr (K > 0) {
    if (own) {
      adam(go, mm, vv, th);
      m[i0] = mm;
      v[i0] = vv;
      theta[i0] = th;
    }
    if (tid == 0) {   // every thread of this workgroup has read beta_pow (barriers above)
      unsigned* cnt = reinterpret_cast<unsigned*>(beta_pow + 2);
      if (atomicAdd(cnt, 1u) == (unsigned)(gridDim.x >> 3) - 1) {
        beta_pow[0] = b1p * h.b1;
        beta_pow[1] = b2p * h.b2;
        *cnt = 0u;
      }
    }
  } else {
    for (int i = tid; i < n; i += 1024) {
      float a = m[i], b = v[i], t = theta[i];
      adam(grad[i], a, b, t);
      m[i] = a;
      v[i] = b;
      theta[i] = t;
    }
    __syncthreads();
    if (tid == 0) {
      beta_pow[0] = b1p * h.b1;
      beta_pow[1] = b2p * h.b2;
    }
  }
}

void launch_apply_adam(hipStream_t s, const float* grad, int n, float* theta, float* m, float* v,
                       float* beta_pow, const UpdateHyper& h, float gscale, int xcd, const int* err) {
  const int k = (n + 1023) / 1024;
  xcd &= 7;
  if (k <= 16)        // fcnet policies: 11,205 .. 15,057 parameters
    hipLaunchKernelGGL(k_apply_adam<16>, dim3(8 * k), dim3(1024), 0, s, grad, n, theta, m, v, beta_pow, h, gscale,
                       xcd, err);
  else if (k <= 32)   // GraphNet: 28,869 parameters
    hipLaunchKernelGGL(k_apply_adam<32>, dim3(8 * k), dim3(1024), 0, s, grad, n, theta, m, v, beta_pow, h, gscale,
                       xcd, err);
  else
    hipLaunchKernelGGL(k_apply_adam<0>, dim3(1), dim3(1024), 0, s, grad, n, theta, m, v, beta_pow, h, gscale, 0, err);
}

// Pre-gather of a run of data-parallel steps (ddrl_ppo_update_ddp): step k's m rows,
// dst[k][i][col] = rec[shuffle[perm[step0 + k] * m + i] * stride + col], so every one-step
// gradient launch stages its records from one contiguous slice instead of through the two
// dependent index loads (perm, then shuffle) ahead of its record gathers.  One float per thread.
__global__ void k_rows_gather(const float* __restrict__ rec, int stride, const int32_t* __restrict__ shuffle,
                              const int32_t* __restrict__ perm, int m, int step0, size_t n, float* __restrict__ dst) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n) return;
  const size_t rowg = gid / stride;
  const int col = (int)(gid - rowg * stride);
  const int k = (int)(rowg / m), i = (int)(rowg - (size_t)k * m);
  const int row = shuffle[(size_t)perm[step0 + k] * m + i];
  dst[gid] = rec[(size_t)row * stride + col];
}

void launch_rows_gather(hipStream_t s, const float* rec, int stride, const int32_t* shuffle, const int32_t* perm,
                        int m, int step0, int n_steps, float* dst) {
  const size_t n = (size_t)n_steps * m * stride;
  hipLaunchKernelGGL(k_rows_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rec, stride, shuffle, perm, m,
                     step0, n, dst);
}
