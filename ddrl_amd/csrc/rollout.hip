// Rollout-side kernels: env-side MeanStdFilter (a2), observation routing (a1/a3),
// fused per-policy forward + DiagGaussian sampling + action scatter (a4/a6/a7),
// per-leg rewards (a8).
//
// Reference: simulation_envs/quantruped_adaptor_multi_environment.py:83-85 (normalize),
// :124-136 (distribute_observations), :160-212 (contact cost, rewards, concatenate_actions);
// models/fcnet_glorot_uniform_init.py:120-125 (forward / value_function);
// RLlib DiagGaussian sampling with clip_actions=True.
#include "common.h"
#include "kernels.h"
#include "ffn.h"

// ------------------------------------------------------------------------------------
// a2: batched MeanStdFilter push, two launches.  k_filter_chunk: workgroup (j, s) reduces rows
// [256 s, 256 s + 256) of observation column j to the chunk's (mean, M2) in fp64 (two passes
// over one value per thread, fixed-order wave / workgroup sums).  k_filter_merge: one thread
// per column merges the chunks in order with Chan's formula into the batch's (mean, M2), then
// the batch into the running stat with RunningStat.update, and writes the normalization
// constants (mean, std + 1e-8) -- a batched MeanStdFilter call pushes every row before
// normalizing.  (Round 2 ran one workgroup per column over all rows: 14.4 us per env-step at
// 4096 envs.  The same chunks merged by the last-arriving workgroup of a column -- agent-scope
// acq_rel atomics, one L2 write-back per workgroup -- measured 18.3 us.)
// ------------------------------------------------------------------------------------
#define FP_ROWS 256   // rows per chunk: one per thread
__global__ void __launch_bounds__(256) k_filter_chunk(const float* __restrict__ obs, int N, int D,
                                                      double* __restrict__ part) {
  const int j = blockIdx.x, sc = blockIdx.y;
  __shared__ double red[4];
  const int tid = threadIdx.x, w = tid >> 6;
  const int e = sc * FP_ROWS + tid;
  const int n_c = min(FP_ROWS, N - sc * FP_ROWS);
  const float x = e < N ? obs[(size_t)e * D + j] : 0.f;
  double acc = wave_sum_d((double)x);
  if ((tid & 63) == 0) red[w] = acc;
  __syncthreads();
  const double mean_c = ((red[0] + red[1]) + (red[2] + red[3])) / (double)n_c;
  __syncthreads();
  const double dlt = e < N ? (double)x - mean_c : 0.0;
  acc = wave_sum_d(dlt * dlt);
  if ((tid & 63) == 0) red[w] = acc;
  __syncthreads();
  if (tid == 0) {
    double* pc = part + ((size_t)sc * D + j) * 2;
    pc[0] = mean_c;
    pc[1] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

__global__ void k_filter_merge(int N, int D, const double* __restrict__ part, double* n_run, double* M,
                               double* S, double* normc, int push, int enabled, double* dn, double* dM,
                               double* dS) {
  const int j = threadIdx.x;
  if (j >= D) return;
  double n1 = n_run[0];
  double Mj = M[j], Sj = S[j];
  if (push) {
    // the batch's (mean, M2): the chunks merged in order (Chan et al.)
    const int nchunks = (N + FP_ROWS - 1) / FP_ROWS;
    double nb = 0.0, mean_b = 0.0, s_b = 0.0;
    for (int c = 0; c < nchunks; ++c) {
      const double* pc = part + ((size_t)c * D + j) * 2;
      const double nc = (double)min(FP_ROWS, N - c * FP_ROWS), nn = nb + nc, d = pc[0] - mean_b;
      mean_b = (nb * mean_b + nc * pc[0]) / nn;
      s_b = s_b + pc[1] + d * d * nb * nc / nn;
      nb = nn;
    }
    const double n2 = (double)N, n = n1 + n2;
    const double delta = Mj - mean_b;
    Mj = (n1 * Mj + n2 * mean_b) / n;
    Sj = Sj + s_b + delta * delta * n1 * n2 / n;
    n1 = n;
    M[j] = Mj;
    S[j] = Sj;
    // the same batch merged into the delta buffer (pushes since the last filter sync)
    const double d1 = dn[0], dd = d1 + n2, ddl = dM[j] - mean_b;
    dM[j] = (d1 * dM[j] + n2 * mean_b) / dd;
    dS[j] = dS[j] + s_b + ddl * ddl * d1 * n2 / dd;
  }
  const double var = n1 > 1.0 ? Sj / (n1 - 1.0) : Mj * Mj;
  normc[2 * j] = enabled ? Mj : 0.0;
  normc[2 * j + 1] = enabled ? sqrt(var) + 1e-8 : 1.0;
}

size_t filter_part_doubles(int N, int D) { return (size_t)2 * D * ((N + FP_ROWS - 1) / FP_ROWS); }

void launch_filter_push(hipStream_t s, const float* obs, int N, int D, double* n_run, double* M,
                        double* S, double* normc, int update, int enabled, double* dn, double* dM,
                        double* dS, double* part) {
  const int push = enabled && update;
  if (push)
    hipLaunchKernelGGL(k_filter_chunk, dim3(D, (N + FP_ROWS - 1) / FP_ROWS), dim3(256), 0, s, obs, N, D, part);
  hipLaunchKernelGGL(k_filter_merge, dim3(1), dim3(64), 0, s, N, D, part, n_run, M, S, normc, push, enabled,
                     dn, dM, dS);
}

// The running count of the env-side filter advances after every column of k_filter_push has
// read it: the observe kernel that follows adds the batch (FilterCount: count = N, or 0 when
// the filter did not push).
__device__ __forceinline__ void filter_count(const FilterCount& fc) {
  if (fc.count && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    fc.n_run[0] += (double)fc.count;
    fc.dn[0] += (double)fc.count;
  }
}

__device__ __forceinline__ double norm_obs_d(float x, const double* normc, int idx, float clip) {
  double z = ((double)x - normc[2 * idx]) / normc[2 * idx + 1];
  if (clip > 0.f) z = fmin(fmax(z, -(double)clip), (double)clip);
  return z;
}
__device__ __forceinline__ float norm_obs(float x, const double* normc, int idx, float clip) {
  double z = ((double)x - normc[2 * idx]) / normc[2 * idx + 1];
  if (clip > 0.f) z = fmin(fmax(z, -(double)clip), (double)clip);
  return (float)z;
}

// a1: per-agent gather of the normalized observation into stage[p][c][f].
__global__ void k_observe_ffn(RouteArgs ra, const float* __restrict__ obs,
                              const double* __restrict__ normc, float clip, float* const* stage_tab,
                              const double* __restrict__ pf, FilterCount fc) {
  filter_count(fc);
  const int p = blockIdx.y;
  const PolicyRoute& pr = ra.pol[p];
  const int C = ra.N * pr.k;              // rows of the env range [e0, e0 + N)
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= C * pr.d) return;
  const int cl = gid / pr.d, f = gid - cl * pr.d;
  const int el = cl / pr.k, slot = cl - el * pr.k;
  const int e = ra.e0 + el, c = ra.e0 * pr.k + cl;
  const int idx = pr.obs_index[slot][f];
  float v;
  if (idx < 0) {
    v = idx == -2 ? 1.f : 0.f;
  } else if (pf) {   // RLlib MeanStdFilter on the fp64 env-normalized value
    const double* P = pf + (size_t)p * PF_STRIDE + PF_NORMC;
    v = (float)((norm_obs_d(obs[(size_t)e * ra.full_dim + idx], normc, idx, clip) - P[2 * f]) / P[2 * f + 1]);
  } else {
    v = norm_obs(obs[(size_t)e * ra.full_dim + idx], normc, idx, clip);
  }
  stage_tab[p][(size_t)c * pr.d + f] = v;
}

void launch_observe_ffn(hipStream_t s, const RouteArgs& ra, const float* obs, const double* normc,
                        float clip, float* const* stage, const double* pf, const FilterCount& fc) {
  int maxw = 0;
  for (int p = 0; p < ra.P; ++p) maxw = max(maxw, ra.N * ra.pol[p].k * ra.pol[p].d);
  dim3 grid((maxw + 255) / 256, ra.P);
  hipLaunchKernelGGL(k_observe_ffn, grid, dim3(256), 0, s, ra, obs, normc, clip, stage, pf, fc);
}

// ------------------------------------------------------------------------------------
// a2 (RLlib side): per-policy MeanStdFilter, unclipped (RLlib get_filter, clip=None).
// Policy p's rows at a step are its k agents' routed columns of every env, so the batch
// statistics of policy column f are sums of the env-normalized full-observation column
// statistics over the slots: one fp64 pass over obs [N][D] (k_zstats) serves every policy.
// The batch is merged with RunningStat.update (Chan), like the env-side filter.
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_zstats(const float* __restrict__ obs, int N, int D,
                                                const double* __restrict__ normc, float clip,
                                                double* __restrict__ zs) {
  const int j = blockIdx.x, tid = threadIdx.x;
  __shared__ double red[2][4];
  double s1 = 0.0, s2 = 0.0;
  for (int e = tid; e < N; e += 256) {
    const double z = norm_obs_d(obs[(size_t)e * D + j], normc, j, clip);
    s1 += z;
    s2 += z * z;
  }
  s1 = wave_sum_d(s1);
  s2 = wave_sum_d(s2);
  if ((tid & 63) == 0) { red[0][tid >> 6] = s1; red[1][tid >> 6] = s2; }
  __syncthreads();
  if (tid == 0) {
    zs[2 * j] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    zs[2 * j + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__device__ __forceinline__ void chan_merge(double& n, double& M, double& S, double nb, double mb, double sb) {
  const double tot = n + nb, delta = M - mb;
  M = (n * M + nb * mb) / tot;
  S = S + sb + delta * delta * n * nb / tot;
}

__global__ void k_pfilter(RouteArgs ra, const double* __restrict__ zs, double* pf, int update) {
  const int p = blockIdx.x, f = threadIdx.x;
  const PolicyRoute& pr = ra.pol[p];
  double* P = pf + (size_t)p * PF_STRIDE;
  const double n0 = P[PF_N], dn0 = P[PF_DN];
  const double nb = (double)ra.N * pr.k;
  __syncthreads();
  if (f < pr.d) {
    double M = P[PF_M + f], S = P[PF_S + f], n = n0;
    if (update) {
      double s1 = 0.0, s2 = 0.0;
      for (int s = 0; s < pr.k; ++s) {
        const int idx = pr.obs_index[s][f];
        s1 += zs[2 * idx];
        s2 += zs[2 * idx + 1];
      }
      const double mb = s1 / nb, sb = fmax(s2 - s1 * mb, 0.0);
      chan_merge(n, M, S, nb, mb, sb);
      double dn = dn0, dM = P[PF_DM + f], dS = P[PF_DS + f];
      chan_merge(dn, dM, dS, nb, mb, sb);
      P[PF_M + f] = M;
      P[PF_S + f] = S;
      P[PF_DM + f] = dM;
      P[PF_DS + f] = dS;
      n = n0 + nb;
    }
    const double var = n > 1.0 ? S / (n - 1.0) : M * M;
    P[PF_NORMC + 2 * f] = M;
    P[PF_NORMC + 2 * f + 1] = sqrt(var) + 1e-8;
  }
  __syncthreads();
  if (update && f == 0) {
    P[PF_N] = n0 + nb;
    P[PF_DN] = dn0 + nb;
  }
}

void launch_policy_filter(hipStream_t s, const RouteArgs& ra, const float* obs, const double* normc, float clip,
                          double* zs, double* pf, int update) {
  if (update) hipLaunchKernelGGL(k_zstats, dim3(ra.full_dim), dim3(256), 0, s, obs, ra.N, ra.full_dim, normc, clip, zs);
  hipLaunchKernelGGL(k_pfilter, dim3(ra.P), dim3(64), 0, s, ra, zs, pf, update);
}

// a3: graph observation X[env][node] = [normalized 19 features | ego quaternion (raw obs)].
__global__ void k_observe_gnn(RouteArgs ra, const float* __restrict__ obs,
                              const double* __restrict__ normc, float clip, float* __restrict__ X,
                              FilterCount fc) {
  filter_count(fc);
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= ra.N * 4) return;
  const int e = ra.e0 + (gid >> 2), n = gid & 3;
  const PolicyRoute& pr = ra.pol[0];
  const float* o = obs + (size_t)e * ra.full_dim;
  float* x = X + ((size_t)e * 4 + n) * 23;
  for (int f = 0; f < 19; ++f) {
    const int idx = pr.obs_index[n][f];
    x[f] = norm_obs(o[idx], normc, idx, clip);
  }
  // leg_encoding_ego: quat_mul(obs[1:5], [0, 0, sin(a/2), cos(a/2)]) in fp64
  const double rad = (double)ra.leg_angle[n] / 2.0 * (3.14159265358979323846 / 180.0);
  const double z2 = sin(rad), w2 = cos(rad);
  const double x1 = o[1], y1 = o[2], z1 = o[3], w1 = o[4];
  x[19] = (float)(x1 * w2 + y1 * z2 - z1 * 0.0 + w1 * 0.0);
  x[20] = (float)(-x1 * z2 + y1 * w2 + z1 * 0.0 + w1 * 0.0);
  x[21] = (float)(x1 * 0.0 - y1 * 0.0 + z1 * w2 + w1 * z2);
  x[22] = (float)(-x1 * 0.0 - y1 * 0.0 - z1 * z2 + w1 * w2);
}

void launch_observe_gnn(hipStream_t s, const RouteArgs& ra, const float* obs, const double* normc,
                        float clip, float* stage_x, const FilterCount& fc) {
  hipLaunchKernelGGL(k_observe_gnn, dim3((ra.N * 4 + 255) / 256), dim3(256), 0, s, ra, obs, normc,
                     clip, stage_x, fc);
}

// ------------------------------------------------------------------------------------
// a4 + a6 + a7: fused rollout forward.  Workgroup = 8 waves = 64 rows of ONE policy
// (grid.y = policy).  The policy's weights are staged once into LDS in the swizzled
// image; waves 0-3 run the policy branch and waves 4-7 the value branch of the same four
// 16-row tiles, from registers (MFMA 16x16x4 f32), so the two branch chains run side by side
// on each SIMD.  The policy waves sample a = mean + exp(log_std) * eps, compute logp, write
// the training record and scatter clip(a, -1, 1) into the env action vector.
// ------------------------------------------------------------------------------------
template <int A, int KS1>
__global__ void __launch_bounds__(512) k_act_ffn(RouteArgs ra, ActArgs aa) {
  constexpr int O = 2 * A;
  extern __shared__ float lds[];
  const int p = blockIdx.y;
  const PolicyRoute& pr = ra.pol[p];
  const int C = aa.C[p];
  const int row_hi = aa.e1 * pr.k;        // rows of the env range [e0, e1)
  const int row0 = aa.e0 * pr.k + blockIdx.x * 64;
  if (row0 >= row_hi) return;
  const int d = pr.d;
  NetLds PW, VW;
  stage_weights(aa.theta[p], d, A, lds, PW, VW, 512);
  __syncthreads();

  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4, w = threadIdx.x >> 6;
  const bool value_wave = w >= 4;
  if (aa.bootstrap && !value_wave) return;   // bootstrap: V(s_T) only
  const int row = row0 + 16 * (w & 3) + c;
  const bool valid = row < row_hi;
  const float* xs = aa.stage[p] + (size_t)(valid ? row : 0) * d;
  float xop[12];
#pragma unroll
  for (int s = 0; s < 12; ++s) {
    const int f = 4 * s + q;
    xop[s] = (s < KS1 && f < d && valid) ? xs[f] : 0.f;
  }
  floatx4 h1[4], h2[4];
  const RecLayout& L = aa.lay[p];
  if (value_wave) {
    float vout[1];
    ffn_branch_fwd<1, KS1>(VW, xop, h1, h2, vout);
    if (valid && q == 0) {
      if (aa.bootstrap) aa.last_v[p][row] = vout[0];
      else aa.rec[p][((size_t)aa.t * C + row) * L.stride + L.vf] = vout[0];
    }
    return;
  }
  float logits[O];
  ffn_branch_fwd<O, KS1>(PW, xop, h1, h2, logits);
  if (!valid) return;
  float* rp = aa.rec[p] + ((size_t)aa.t * C + row) * L.stride;
  const int e = row / pr.k, slot = row - e * pr.k;
  const int agent = pr.agent[slot];
  // "cup" model (coupling_net_glorot_uniform_init.py:22-30): mean_j *= coupling[leg][j], the
  // log-std half is padded with ones; leg = the agent's index in the env (one shared policy)
  if (aa.cup[p]) {
#pragma unroll
    for (int j = 0; j < A; ++j) logits[j] *= aa.cup[p][slot * A + j];
  }
  // sample + logp (DiagGaussian, RLlib 1.0): a = mean + std * eps
  float logp = -0.5f * (float)(DDRL_LOG2PI * A);
  float act[A];
#pragma unroll
  for (int j = 0; j < A; ++j) {
    const float mu = logits[j], ls = logits[A + j];
    const float sd = expf(ls);
    const float eps = aa.eps[((size_t)e * ra.n_agents + agent) * A + j];
    act[j] = mu + sd * eps;
    const float z = (act[j] - mu) / sd;
    logp -= 0.5f * z * z;
    logp -= ls;
  }
  // q-lanes split the record stores
  for (int f = q; f < d; f += 4) rp[L.obs + f] = xs[f];
  if (q == 0) {
#pragma unroll
    for (int j = 0; j < A; ++j) {
      rp[L.act + j] = act[j];
      const float ac = fminf(fmaxf(act[j], -1.f), 1.f);
      aa.actions[(size_t)e * 8 + pr.act_index[slot][j]] = (pr.act_neg[slot] >> j) & 1 ? -ac : ac;
    }
  } else if (q == 1) {
#pragma unroll
    for (int j = 0; j < O; ++j) rp[L.logit + j] = logits[j];
  } else if (q == 2) {
    rp[L.logp] = logp;
    if (L.cid >= 0) rp[L.cid] = (float)slot;
  }
}

template <int A, int KS1>
static void launch_act_t(hipStream_t s, dim3 grid, const RouteArgs& ra, const ActArgs& aa) {
  hipLaunchKernelGGL((k_act_ffn<A, KS1>), grid, dim3(512), LDS_WEIGHTS_FLOATS(2 * A) * 4, s, ra, aa);
}

void launch_act_ffn(hipStream_t s, const RouteArgs& ra, const ActArgs& aa) {
  int maxC = 0;
  for (int p = 0; p < ra.P; ++p) maxC = max(maxC, (aa.e1 - aa.e0) * ra.pol[p].k);
  dim3 grid((maxC + 63) / 64, ra.P);
  int maxd = 0;
  for (int p = 0; p < ra.P; ++p) maxd = max(maxd, ra.pol[p].d);
  DDRL_DISPATCH_A_KS1(ra.A, maxd, launch_act_t, s, grid, ra, aa);
}

// ------------------------------------------------------------------------------------
// a8: per-leg (or global / normalized) reward of each agent; fp64 like the reference.
// ------------------------------------------------------------------------------------
// One thread per (env, agent): the agent's control cost and its bodies' contact cost.
__global__ void k_reward(RewardArgs ra, const float* __restrict__ fw, const float* __restrict__ cfrc,
                         const float* __restrict__ actions, const uint8_t* __restrict__ done,
                         uint8_t* __restrict__ done_tn) {
  const int na = ra.n_agents;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= ra.n * na) return;
  const int el = gid / na, j = gid - el * na, e = ra.e0 + el;
  const float* cf = cfrc + (size_t)e * 14 * 6;
  const float* a8 = actions + (size_t)e * 8;
  const double fwd = fw[e];
  double r;
  if (ra.mode == 1) {
    double ctrl_all = 0.0, contact_all = 0.0;
    for (int i = 0; i < 8; ++i) ctrl_all += (double)a8[i] * a8[i];
    for (int i = 0; i < 14 * 6; ++i) {
      const double v = fmin(fmax((double)cf[i], -1.0), 1.0);
      contact_all += v * v;
    }
    contact_all *= ra.contact_w;
    r = (fwd - ra.ctrl_w * ctrl_all - contact_all) / na;
  } else {
    double ctrl = 0.0;
    for (int i = 0; i < ra.n_act[j]; ++i) {
      const double a = a8[ra.act_index[j][i]];
      ctrl += a * a;
    }
    double contact = 0.0;
    for (int b = 0; b < ra.n_contact[j]; ++b) {
      const float* body = cf + ra.contact_index[j][b] * 6;
      double sb = 0.0;
      for (int k = 0; k < 6; ++k) {
        const double v = fmin(fmax((double)body[k], -1.0), 1.0);
        sb += ra.contact_w * v * v * ra.contact_weight[j][b];
      }
      contact += sb;
    }
    r = ra.mode == 2 ? fwd - na * (ra.ctrl_w * ctrl + contact)
                     : fwd / na - ra.ctrl_w * ctrl - contact;
  }
  const int p = ra.policy_of_agent[j], slot = ra.slot_of_agent[j];
  const size_t C = (size_t)ra.N * ra.k[p];
  float* rp = ra.rec[p] + ((size_t)ra.t * C + (size_t)e * ra.k[p] + slot) * ra.lay[p].stride;
  rp[ra.lay[p].rew] = (float)r;
  if (j == 0) done_tn[(size_t)ra.t * ra.N + e] = done ? done[e] : 0;
}

void launch_reward(hipStream_t s, const RewardArgs& ra, const float* fw, const float* cfrc,
                   const float* actions, const uint8_t* done, uint8_t* done_tn) {
  const int n = ra.n * ra.n_agents;
  hipLaunchKernelGGL(k_reward, dim3((n + 255) / 256), dim3(256), 0, s, ra, fw, cfrc, actions,
                     done, done_tn);
}

// ------------------------------------------------------------------------------------
// ModelV2.forward + value_function (fcnet_glorot_uniform_init.py:120-125) on n rows.
// ------------------------------------------------------------------------------------
template <int A, int KS1>
__global__ void __launch_bounds__(256) k_forward_ffn(ForwardArgs fa) {
  constexpr int O = 2 * A;
  extern __shared__ float lds[];
  NetLds PW, VW;
  stage_weights(fa.theta, fa.d, A, lds, PW, VW, 256);
  __syncthreads();
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 64 + 16 * w + c;
  const bool valid = row < fa.n;
  const int d = fa.d;
  float xop[12];
#pragma unroll
  for (int s = 0; s < 12; ++s) {
    const int f = 4 * s + q;
    xop[s] = (valid && s < KS1 && f < d) ? fa.x[(size_t)row * d + f] : 0.f;
  }
  floatx4 h1[4], h2[4];
  float vout[1], logits[O];
  ffn_branch_fwd<1, KS1>(VW, xop, h1, h2, vout);
  ffn_branch_fwd<O, KS1>(PW, xop, h1, h2, logits);
  if (!valid) return;
  if (fa.cup) {   // "cup": leg index of the row (clamped to the table; the host validates it)
    const int leg = min(max(fa.node[row], 0), 3);
#pragma unroll
    for (int j = 0; j < A; ++j) logits[j] *= fa.cup[leg * A + j];
  }
  if (q == 0) fa.values[row] = vout[0];
  for (int j = q; j < O; j += 4) fa.logits[(size_t)row * O + j] = logits[j];
}

template <int A, int KS1>
static void launch_forward_t(hipStream_t s, dim3 grid, const ForwardArgs& fa) {
  hipLaunchKernelGGL((k_forward_ffn<A, KS1>), grid, dim3(256), LDS_WEIGHTS_FLOATS(2 * A) * 4, s, fa);
}

void launch_forward_ffn(hipStream_t s, const ForwardArgs& fa) {
  dim3 grid((fa.n + 63) / 64);
  DDRL_DISPATCH_A_KS1(fa.A, fa.d, launch_forward_t, s, grid, fa);
}
