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

// The record loads of a chunk of GAE_U time steps are issued one chunk ahead of the
// recursion (the stores of adv / vt may alias them as far as the compiler knows, so it would
// otherwise wait for every load in turn: one memory round trip per time step).
#define GAE_U 8
struct GaeChunk { float v[GAE_U], r[GAE_U]; bool d[GAE_U]; };

__device__ __forceinline__ void gae_load(const GaeArgs& g, int c, int e, int t0, GaeChunk& ch) {
#pragma unroll
  for (int u = 0; u < GAE_U; ++u) {
    const int t = t0 - u;
    if (t >= 0) {
      const float* rp = g.rec + ((size_t)t * g.C + c) * g.lay.stride;
      ch.v[u] = rp[g.lay.vf];
      ch.r[u] = rp[g.lay.rew];
      ch.d[u] = g.done_tn[(size_t)t * g.N + e] != 0;
    }
  }
}

__device__ __forceinline__ void gae_run(const GaeArgs& g, int c, int t0, const GaeChunk& ch, double& acc,
                                        double& nextv, double& s1, double& s2) {
  const double gl = g.gamma * g.lambda_;
#pragma unroll
  for (int u = 0; u < GAE_U; ++u) {
    const int t = t0 - u;
    if (t < 0) break;
    if (ch.d[u]) {
      acc = 0.0;
      nextv = 0.0;
    }
    const double v = (double)ch.v[u];
    const double delta = (double)ch.r[u] + g.gamma * nextv - v;
    acc = delta + gl * acc;
    const float a32 = (float)acc;
    float* rp = g.rec + ((size_t)t * g.C + c) * g.lay.stride;
    rp[g.lay.adv] = a32;
    rp[g.lay.vt] = (float)(acc + v);
    s1 += (double)a32;
    s2 += (double)a32 * (double)a32;
    nextv = v;
  }
}

__global__ void __launch_bounds__(256) k_gae(GaeArgs g) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (c < g.C) {
    const int e = c / g.k;
    double acc = 0.0;
    double nextv = (double)g.last_v[c];
    const int nch = (g.T + GAE_U - 1) / GAE_U;
    GaeChunk a, b;
    gae_load(g, c, e, g.T - 1, a);
    for (int k = 0; k < nch; k += 2) {
      const int ta = g.T - 1 - k * GAE_U, tb = ta - GAE_U;
      if (k + 1 < nch) gae_load(g, c, e, tb, b);
      gae_run(g, c, ta, a, acc, nextv, s1, s2);
      if (k + 1 >= nch) break;
      if (k + 2 < nch) gae_load(g, c, e, tb - GAE_U, a);
      gae_run(g, c, tb, b, acc, nextv, s1, s2);
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
