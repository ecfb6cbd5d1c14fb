// a13-a17: fused PPO minibatch SGD for the fcnet policy/value model (persistent kernel).
//
// Two workgroups per policy, on two CUs of one XCD: blockIdx = p + 8 branch, branch 0 = policy branch
// (fc_1, fc_2, fc_out), branch 1 = value branch (fc_value_1, fc_value_2, value_out).  The
// branches share no parameters, so each workgroup computes its own gradients and runs Adam
// on its own parameters; the only coupling is tf.clip_by_global_norm, which needs the
// squared norm over ALL variables: every step the two workgroups swap their partial
// squared norms through one tagged 8-byte granule each (plain store / sc1 poll, slots double
// buffered by step parity, zeroed by a memset before every launch, spins bounded).
//
// Per minibatch step (RLlib TrainTFMultiGPU: row = shuffle[perm[e][b] * 128 + i]):
//   rows of step s+1 are prefetched into registers while step s computes;
//   forward of the branch for 32 rows per wave, one wave per SIMD (MFMA 16x16x4 f32,
//   activations in registers, every weight operand read from LDS feeds two MFMAs);
//   PPOLoss per row (RLlib 1.0 ppo_tf_policy.PPOLoss) and analytic dL/d(outputs);
//   head / bias gradients and loss statistics by DPP row reductions (no LDS round trip);
//   layer-2 backward from registers; H1/dZ2 then X/dZ1 through LDS for the two weight-
//   gradient GEMMs (16x16 tiles, K = 128 rows); per-wave tile ownership;
//   global-norm clip; tf1 Adam (ApplyAdam) with m / v held in registers by the owning
//   lane and the weights updated in place in the LDS image.
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
