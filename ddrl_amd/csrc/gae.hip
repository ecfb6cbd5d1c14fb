// a11 / a12: GAE reverse scan over a time-major fragment, fused with the
// standardization statistics of the advantages.
//
// RLlib 1.0 compute_advantages (postprocess_ppo_gae, run once per agent trajectory segment):
//   delta_t = r_t + gamma * V_{t+1} - V_t, with V_T = last_r (0 after done, else V(s_T));
//   adv = lfilter([1], [1, -gamma*lambda], delta[::-1])[::-1]  in float64,
//   value_targets = float32(adv + vf_preds), adv = float32(adv).
// A fragment is split into episode segments at done flags; within one chain the
// recursion y_t = delta_t + gamma*lambda*y_{t+1} (reset after a done) is exactly lfilter's.
// One thread per chain; the loads over t are coalesced across chains (time-major rows).
// StandardizeFields: (adv - mean) / max(1e-4, std) over the policy's whole batch; the sums
// are fp64 and reduced in a fixed order (per-block partials + one finalize block).
#include "common.h"
#include "kernels.h"

#pragma clang fp contract(off)

__global__ void __launch_bounds__(256) k_gae(GaeArgs g) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (c < g.C) {
    const int e = c / g.k;
    double acc = 0.0;
    double nextv = (double)g.last_v[c];
    const double gl = g.gamma * g.lambda_;
    for (int t = g.T - 1; t >= 0; --t) {
      float* rp = g.rec + ((size_t)t * g.C + c) * g.lay.stride;
      const bool done = g.done_tn[(size_t)t * g.N + e] != 0;
      if (done) {
        acc = 0.0;
        nextv = 0.0;
      }
      const double v = (double)rp[g.lay.vf];
      const double delta = (double)rp[g.lay.rew] + g.gamma * nextv - v;
      acc = delta + gl * acc;
      const float a32 = (float)acc;
      rp[g.lay.adv] = a32;
      rp[g.lay.vt] = (float)(acc + v);
      s1 += (double)a32;
      s2 += (double)a32 * (double)a32;
      nextv = v;
    }
  }
  __shared__ double red[2][4];
  s1 = wave_sum_d(s1);
  s2 = wave_sum_d(s2);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s1;
    red[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    g.partials[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    g.partials[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__global__ void k_gae_finalize(GaeArgs g, int nblocks) {
  if (threadIdx.x != 0) return;
  double s1 = 0.0, s2 = 0.0;
  for (int b = 0; b < nblocks; ++b) {
    s1 += g.partials[2 * b];
    s2 += g.partials[2 * b + 1];
  }
  const double n = (double)g.C * (double)g.T;
  g.partials[2 * nblocks] = s1;        // for a cross-rank StandardizeFields
  g.partials[2 * nblocks + 1] = s2;
  g.partials[2 * nblocks + 2] = n;
  const double mean = s1 / n;
  double var = s2 / n - mean * mean;
  if (var < 0.0) var = 0.0;
  const float std32 = (float)sqrt(var);
  g.adv_norm[0] = (float)mean;
  g.adv_norm[1] = fmaxf(1e-4f, std32);
}

void launch_gae(hipStream_t s, const GaeArgs& g) {
  const int nblocks = (g.C + 255) / 256;
  hipLaunchKernelGGL(k_gae, dim3(nblocks), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_gae_finalize, dim3(1), dim3(64), 0, s, g, nblocks);
}
