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
// are fp64 and reduced in a fixed order (per-wave partials + one finalize block per policy).
#include "common.h"
#include "kernels.h"

#pragma clang fp contract(off)

// The record loads of a chunk of GAE_U time steps are issued one chunk ahead of the
// recursion (the stores of adv / vt may alias them as far as the compiler knows, so it would
// otherwise wait for every load in turn: one memory round trip per time step).
#define GAE_U 16
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

// One launch for all policies (blockIdx.y), one wave per block: a policy's C chains spread
// over C / 64 workgroups (Local at 4096 envs: 256 CUs busy instead of 16, whose texture units
// serialized the strided record loads; 4 x 255 -> one ~60 us launch).  Each block writes its
// wave's (sum adv, sum adv^2); the finalize sums them four at a time as ((w0 + w1) + (w2 + w3))
// and then over the groups in order -- the 256-thread reduction's order, so adv_norm and the
// totals are bit-identical to it.
__global__ void __launch_bounds__(64) k_gae(GaeBatch gb) {
  const GaeArgs& g = gb.g[blockIdx.y];
  if ((int)blockIdx.x * 64 >= g.C) return;
  const int c = blockIdx.x * 64 + threadIdx.x;
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
  s1 = wave_sum_d(s1);
  s2 = wave_sum_d(s2);
  if (threadIdx.x == 0) {
    double* wp = g.partials + gae_wave_base(g.C) + 2 * blockIdx.x;
    wp[0] = s1;
    wp[1] = s2;
  }
}

__global__ void k_gae_finalize(GaeBatch gb) {
  if (threadIdx.x != 0) return;
  const GaeArgs& g = gb.g[blockIdx.x];
  const int nw = (g.C + 63) / 64, ngroups = (g.C + 255) / 256;
  const double* wp = g.partials + gae_wave_base(g.C);
  double s1 = 0.0, s2 = 0.0;
  for (int b = 0; b < ngroups; ++b) {
    double x[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int w = 4 * b + i;
      x[0][i] = w < nw ? wp[2 * w] : 0.0;
      x[1][i] = w < nw ? wp[2 * w + 1] : 0.0;
    }
    s1 += (x[0][0] + x[0][1]) + (x[0][2] + x[0][3]);
    s2 += (x[1][0] + x[1][1]) + (x[1][2] + x[1][3]);
  }
  const double n = (double)g.C * (double)g.T;
  double* tot = g.partials + 2 * ngroups;   // for a cross-rank StandardizeFields
  tot[0] = s1;
  tot[1] = s2;
  tot[2] = n;
  const double mean = s1 / n;
  double var = s2 / n - mean * mean;
  if (var < 0.0) var = 0.0;
  const float std32 = (float)sqrt(var);
  g.adv_norm[0] = (float)mean;
  g.adv_norm[1] = fmaxf(1e-4f, std32);
}

void launch_gae(hipStream_t s, const GaeBatch& gb) {
  int maxw = 1;
  for (int p = 0; p < gb.P; ++p) maxw = maxw > (gb.g[p].C + 63) / 64 ? maxw : (gb.g[p].C + 63) / 64;
  hipLaunchKernelGGL(k_gae, dim3(maxw, gb.P), dim3(64), 0, s, gb);
  hipLaunchKernelGGL(k_gae_finalize, dim3(gb.P), dim3(64), 0, s, gb);
}
