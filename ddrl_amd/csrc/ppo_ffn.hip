// a13-a17: fused PPO minibatch SGD for the fcnet policy/value model.
//
// One persistent workgroup (8 waves, 512 threads) per policy runs the policy's whole
// minibatch schedule -- num_sgd_iter epochs x nb minibatches of 128 rows -- without
// returning to the host.  Per minibatch step:
//   gather 128 rows (row = shuffle[perm[e][b] * 128 + i], RLlib TrainTFMultiGPU slicing)
//   -> forward of the policy branch (MFMA, activations in registers, 16 rows per wave)
//   -> PPOLoss per row and analytic dL/dlogits (DiagGaussian logp / KL / entropy, clipped
//      surrogate; RLlib 1.0 ppo_tf_policy.PPOLoss)
//   -> backward (head VALU, layer 2 MFMA from registers), activations to LDS, weight
//      gradients as 16x16 MFMA tiles over the 128 rows (K = rows), bias column sums
//   -> the same for the value branch (PPO2 clipped value loss, vf_clip_param)
//   -> global-norm clip (tf.clip_by_global_norm(grads, 0.5)) via a workgroup reduction
//   -> tf1 Adam (ApplyAdam) on every parameter; weights updated in place in LDS,
//      m / v in HBM (L2 resident), beta powers as fp32 like the TF variables.
// Gradients never leave the registers of the wave that produced them.
#include "common.h"
#include "kernels.h"
#include "ffn.h"

struct UpdateBatch {
  const UpdateArgs* a;   // device array, one entry per workgroup (policy)
  UpdateHyper h;
  int nrows;      // rows per minibatch handled here (<= 128)
  float inv_n;    // 1 / sgd_minibatch_size (global minibatch)
};

#define NT 512
#define NW 8
#define SCR_ROWS 128

// Store a 16x16 gradient tile (C layout: dW[f = 16fa + 4q + r][o = 16fo + c]) of a
// row-major [rows][ncols] parameter block at global offset `off`; returns its sum of squares.
__device__ __forceinline__ float store_grad_tile(float* G, int off, int ncols, int nrows_valid,
                                                 int fa, int fo, const floatx4& t) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  const int o = 16 * fo + c;
  float ss = 0.f;
  if (o < ncols) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * fa + 4 * q + r;
      if (f < nrows_valid) {
        G[off + f * ncols + o] = t[r];
        ss += t[r] * t[r];
      }
    }
  }
  return ss;
}

// LDS location of parameter `i` (Keras flat order) inside the two-branch weight image.
template <int O>
__device__ __forceinline__ float* param_lds(int i, const FfnOffsets& of, const NetLds& P, const NetLds& V) {
  if (i < of.b1) return P.w1 + sidx(i >> 6, i & 63);
  if (i < of.vw1) return P.b1 + (i - of.b1);
  if (i < of.vb1) { const int j = i - of.vw1; return V.w1 + sidx(j >> 6, j & 63); }
  if (i < of.w2) return V.b1 + (i - of.vb1);
  if (i < of.b2) { const int j = i - of.w2; return P.w2 + sidx(j >> 6, j & 63); }
  if (i < of.vw2) return P.b2 + (i - of.b2);
  if (i < of.vb2) { const int j = i - of.vw2; return V.w2 + sidx(j >> 6, j & 63); }
  if (i < of.wo) return V.b2 + (i - of.vb2);
  if (i < of.bo) return P.wo + (i - of.wo);
  if (i < of.vo) return P.bo + (i - of.bo);
  if (i < of.vbo) return V.wo + (i - of.vo);
  return V.bo;
}

__device__ __forceinline__ void tile_coords(int t, int& type, int& fa, int& fo) {
  if (t < 4) { type = 0; fa = t; fo = 0; }
  else if (t < 20) { type = 1; fa = (t - 4) >> 2; fo = (t - 4) & 3; }
  else { type = 2; fa = (t - 20) >> 2; fo = (t - 20) & 3; }
}

template <int A, int KS1>
__global__ void __launch_bounds__(NT) k_update_ffn(UpdateBatch ub) {
  constexpr int O = 2 * A;
  extern __shared__ float lds[];
  const int p = blockIdx.x;
  const UpdateArgs U = ub.a[p];
  const UpdateHyper& H = ub.h;
  const int d = U.d;
  const FfnOffsets of = ffn_offsets(d, A);
  const int nf1 = (d + 15) >> 4;
  const int T_net = 20 + 4 * nf1;

  NetLds PW, VW;
  stage_weights(U.theta, d, A, lds, PW, VW, NT);
  float* bufA = lds + LDS_WEIGHTS_FLOATS(O);
  float* bufB = bufA + 128 * 64;
  float* D = bufB + 128 * 64;             // [128][O]
  float* scr = D + 128 * 16;              // [8][128] per-row stats
  float* red = scr + 8 * SCR_ROWS;        // [32]
  __syncthreads();

  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, q = lane >> 4, w = tid >> 6;
  const int row_l = 16 * w + c;            // row of this lane inside the minibatch
  const bool row_ok = row_l < ub.nrows;
  float b1p = U.beta_pow[0], b2p = U.beta_pow[1];
  const float adv_mean = U.adv_norm[0], adv_den = U.adv_norm[1];
  const float beta = U.kl_coeff;
  const float lo = 1.f - H.clip, hi = 1.f + H.clip;

  const int total_steps = U.n_epochs * U.nb;
  const int last = U.max_steps >= 0 ? min(total_steps, U.step0 + U.max_steps) : total_steps;
  for (int step = U.step0; step < last; ++step) {
    const int e = step / U.nb, b = step - e * U.nb;
    int ridx = 0;
    if (row_ok) ridx = U.shuffle[U.perm[e * U.nb + b] * DDRL_MB + row_l];
    const float* rp = U.rec + (size_t)ridx * U.lay.stride;
    float xop[12];
#pragma unroll
    for (int s = 0; s < 12; ++s) {
      const int f = 4 * s + q;
      xop[s] = (row_ok && s < KS1 && f < d) ? rp[U.lay.obs + f] : 0.f;
    }
    float act[A], olog[O];
#pragma unroll
    for (int j = 0; j < A; ++j) act[j] = rp[U.lay.act + j];
#pragma unroll
    for (int j = 0; j < O; ++j) olog[j] = rp[U.lay.logit + j];
    const float ologp = rp[U.lay.logp];
    const float vf_old = rp[U.lay.vf];
    const float adv = (rp[U.lay.adv] - adv_mean) / adv_den;
    const float vt = rp[U.lay.vt];

    // gradients go straight to G (L2-resident) as each tile / column sum completes
    float* G = U.grad_out ? U.grad_out : U.gscr;
    float ss = 0.f;   // this thread's share of the squared global norm

#pragma unroll
    for (int net = 0; net < 2; ++net) {
      const NetLds& W = net == 0 ? PW : VW;
      floatx4 h1[4], h2[4], dz2[4], dz1[4];
      float dout[O];
      if (net == 0) {
        float logits[O];
        ffn_branch_fwd<O, KS1>(W, xop, h1, h2, logits);
        // ---- PPOLoss (per row) and dL/dlogits ----
        float logp = -0.5f * (float)(DDRL_LOG2PI * A), klr = 0.f, ent = 0.f;
        float z[A], sd[A];
#pragma unroll
        for (int j = 0; j < A; ++j) {
          sd[j] = expf(logits[A + j]);
          z[j] = (act[j] - logits[j]) / sd[j];
          logp -= 0.5f * z[j] * z[j];
          logp -= logits[A + j];
          const float v0 = expf(olog[A + j]);
          const float dm = olog[j] - logits[j];
          klr += logits[A + j] - olog[A + j] + (v0 * v0 + dm * dm) / (2.f * sd[j] * sd[j]) - 0.5f;
          ent += logits[A + j] + 0.5f * (float)(DDRL_LOG2PI + 1.0);
        }
        const float ratio = expf(logp - ologp);
        const float cr = fminf(fmaxf(ratio, lo), hi);
        const float s1 = adv * ratio, s2 = adv * cr;
        const float surr = fminf(s1, s2);
        const float dr = (s1 <= s2) ? adv : ((ratio >= lo && ratio <= hi) ? adv : 0.f);
        const float glogp = -dr * ratio;
#pragma unroll
        for (int j = 0; j < A; ++j) {
          const float v0 = expf(olog[A + j]);
          const float dm = olog[j] - logits[j];
          const float var1 = sd[j] * sd[j];
          float dmu = glogp * (z[j] / sd[j]) + beta * ((logits[j] - olog[j]) / var1);
          float dls = glogp * (z[j] * z[j] - 1.f) + beta * (1.f - (v0 * v0 + dm * dm) / var1) - H.ent_coeff;
          dout[j] = row_ok ? dmu * ub.inv_n : 0.f;
          dout[A + j] = row_ok ? dls * ub.inv_n : 0.f;
        }
        if (q == 0 && row_ok) {
          scr[0 * SCR_ROWS + row_l] = -surr;
          scr[1 * SCR_ROWS + row_l] = klr;
          scr[2 * SCR_ROWS + row_l] = ent;
        }
      } else {
        float vo[1];
        ffn_branch_fwd<1, KS1>(W, xop, h1, h2, vo);
        const float V = vo[0];
        float vf, dvf;
        if (H.vf_mode == 0) {
          const float vf1 = (V - vt) * (V - vt);
          const float dv = V - vf_old;
          const float vcl = vf_old + fminf(fmaxf(dv, -H.vf_clip), H.vf_clip);
          const float vf2 = (vcl - vt) * (vcl - vt);
          vf = fmaxf(vf1, vf2);
          dvf = (vf1 >= vf2) ? 2.f * (V - vt)
                             : ((dv >= -H.vf_clip && dv <= H.vf_clip) ? 2.f * (vcl - vt) : 0.f);
        } else {
          const float sq = (V - vt) * (V - vt);
          vf = fminf(sq, H.vf_clip);
          dvf = sq <= H.vf_clip ? 2.f * (V - vt) : 0.f;
        }
        dout[0] = row_ok ? H.vf_coeff * dvf * ub.inv_n : 0.f;
        if (q == 0 && row_ok) {
          scr[3 * SCR_ROWS + row_l] = vf;
          scr[4 * SCR_ROWS + row_l] = V;
          scr[5 * SCR_ROWS + row_l] = vt;
        }
      }
      constexpr int OMAX = O;
      const int OO = net == 0 ? O : 1;
      // ---- backward through the head (registers), then publish H2 / dZ2 / dout ----
      if (net == 0) head_bwd<O>(W, dout, dz2);
      else head_bwd<1>(W, dout, dz2);
      dtanh_inplace(dz2, h2);
      __syncthreads();                       // previous phase readers of bufA/bufB/D done
      store_act(bufA, w, h2);
      store_act(bufB, w, dz2);
      if (q == 0) {
#pragma unroll
        for (int o = 0; o < OMAX; ++o)
          if (o < OO) D[row_l * OO + o] = dout[o];
      }
      layer2_bwd(W, dz2, dz1);
      dtanh_inplace(dz1, h1);
      __syncthreads();
      // ---- phase 0: dWo tiles (H2 x dout), db2, dbo ----
      const int boff = net == 0 ? 0 : 128;
#pragma unroll 1
      for (int i = 0; i < 4; ++i) {
        const int t = w + 8 * i;
        if (t < 4) {
          if (net == 0) ss += store_grad_tile(G, of.wo, O, 64, t, 0, dw_tile_head<O, DDRL_MB>(bufA, D, t));
          else ss += store_grad_tile(G, of.vo, 1, 64, t, 0, dw_tile_head<1, DDRL_MB>(bufA, D, t));
        }
      }
      if (tid >= boff && tid < boff + 64) {
        float s = 0.f;
        for (int r = 0; r < DDRL_MB; ++r) s += bufB[sidx(r, tid - boff)];
        G[(net ? of.vb2 : of.b2) + tid - boff] = s;   // db2
        ss += s * s;
      } else if (tid >= boff + 64 && tid < boff + 64 + OO) {
        float s = 0.f;
        for (int r = 0; r < DDRL_MB; ++r) s += D[r * OO + (tid - boff - 64)];
        G[(net ? of.vbo : of.bo) + tid - boff - 64] = s;   // dbo
        ss += s * s;
      }
      __syncthreads();
      // ---- phase 1: H1 -> A ; dW2 tiles (H1 x dZ2) ----
      store_act(bufA, w, h1);
      __syncthreads();
#pragma unroll 1
      for (int i = 0; i < 4; ++i) {
        const int t = w + 8 * i;
        if (t >= 4 && t < 20) {
          int type, fa, fo;
          tile_coords(t, type, fa, fo);
          ss += store_grad_tile(G, net ? of.vw2 : of.w2, 64, 64, fa, fo, dw_tile<DDRL_MB>(bufA, bufB, fa, fo));
        }
      }
      __syncthreads();
      // ---- phase 2: X -> A, dZ1 -> B ; dW1 tiles, db1 ----
      store_act(bufB, w, dz1);
#pragma unroll
      for (int s = 0; s < 12; ++s) bufA[sidx(row_l, 4 * s + q)] = xop[s];
      __syncthreads();
#pragma unroll 1
      for (int i = 0; i < 4; ++i) {
        const int t = w + 8 * i;
        if (t >= 20 && t < T_net) {
          int type, fa, fo;
          tile_coords(t, type, fa, fo);
          ss += store_grad_tile(G, net ? of.vw1 : of.w1, 64, d, fa, fo, dw_tile<DDRL_MB>(bufA, bufB, fa, fo));
        }
      }
      if (tid >= boff && tid < boff + 64) {
        float s = 0.f;
        for (int r = 0; r < DDRL_MB; ++r) s += bufB[sidx(r, tid - boff)];
        G[(net ? of.vb1 : of.b1) + tid - boff] = s;   // db1
        ss += s * s;
      }
    }

    // ---- DDP: raw gradients were written to grad_out; the caller all-reduces ----
    if (U.grad_out) return;

    // ---- global norm (tf.clip_by_global_norm) ----
    ss = wave_sum(ss);
    if (lane == 0) red[w] = ss;
    __syncthreads();   // also publishes G (workgroup scope, same CU)
    if (tid == 0) {
      float tot = 0.f;
      for (int i = 0; i < NW; ++i) tot += red[i];
      const float gn = sqrtf(tot);
      red[16] = gn;
      red[17] = H.grad_clip * fminf(1.f / gn, 1.f / H.grad_clip);
    }
    __syncthreads();
    const float scale = red[17];
    const float alpha = H.lr * sqrtf(1.f - b2p) / (1.f - b1p);
    const float c1 = 1.f - H.b1, c2 = 1.f - H.b2;

    // ---- tf1 Adam (ApplyAdam), coalesced over the flat parameter vector ----
    for (int i = tid; i < of.n; i += NT) {
      const float gg = G[i] * scale;
      float mi = U.m[i], vi = U.v[i];
      mi = mi + (gg - mi) * c1;
      vi = vi + (gg * gg - vi) * c2;
      U.m[i] = mi;
      U.v[i] = vi;
      float* lp = param_lds<O>(i, of, PW, VW);
      *lp = *lp - (mi * alpha) / (sqrtf(vi) + H.eps);
    }
    b1p = b1p * H.b1;
    b2p = b2p * H.b2;

    // ---- minibatch statistics (RLlib learner stats) ----
    if (w == 0) {
      const int n = ub.nrows;
      float sp = 0.f, sk = 0.f, se = 0.f, sv = 0.f, st = 0.f, sy = 0.f, sd = 0.f;
      for (int r = lane; r < n; r += 64) {
        const float pl = scr[r], kl = scr[SCR_ROWS + r], en = scr[2 * SCR_ROWS + r];
        const float vf = scr[3 * SCR_ROWS + r];
        sp += pl; sk += kl; se += en; sv += vf;
        st += pl + beta * kl + H.vf_coeff * vf - H.ent_coeff * en;
        sy += scr[5 * SCR_ROWS + r];
        sd += scr[5 * SCR_ROWS + r] - scr[4 * SCR_ROWS + r];
      }
      sp = wave_sum(sp); sk = wave_sum(sk); se = wave_sum(se); sv = wave_sum(sv);
      st = wave_sum(st); sy = wave_sum(sy); sd = wave_sum(sd);
      const float my = sy / n, md = sd / n;
      float vy = 0.f, vd = 0.f;
      for (int r = lane; r < n; r += 64) {
        const float y = scr[5 * SCR_ROWS + r], dd = y - scr[4 * SCR_ROWS + r];
        vy += (y - my) * (y - my);
        vd += (dd - md) * (dd - md);
      }
      vy = wave_sum(vy); vd = wave_sum(vd);
      if (lane == 0 && U.stats) {
        float* so = U.stats + (size_t)step * 8;
        so[0] = st / n; so[1] = sp / n; so[2] = sv / n; so[3] = sk / n; so[4] = se / n;
        so[5] = vy > 0.f ? fmaxf(-1.f, 1.f - vd / vy) : 0.f;
        so[6] = red[16];
        so[7] = scale;
      }
    }
    __syncthreads();
  }

  // ---- write back weights and beta powers ----
  if (U.grad_out) return;
  for (int i = tid; i < 48 * 64; i += NT) {
    const int f = i >> 6, col = i & 63;
    if (f < d) {
      U.theta[of.w1 + i] = PW.w1[sidx(f, col)];
      U.theta[of.vw1 + i] = VW.w1[sidx(f, col)];
    }
  }
  for (int i = tid; i < 64 * 64; i += NT) {
    const int f = i >> 6, col = i & 63;
    U.theta[of.w2 + i] = PW.w2[sidx(f, col)];
    U.theta[of.vw2 + i] = VW.w2[sidx(f, col)];
  }
  for (int i = tid; i < 64; i += NT) {
    U.theta[of.b1 + i] = PW.b1[i]; U.theta[of.b2 + i] = PW.b2[i];
    U.theta[of.vb1 + i] = VW.b1[i]; U.theta[of.vb2 + i] = VW.b2[i];
    U.theta[of.vo + i] = VW.wo[i];
  }
  for (int i = tid; i < 64 * O; i += NT) U.theta[of.wo + i] = PW.wo[i];
  for (int i = tid; i < O; i += NT) U.theta[of.bo + i] = PW.bo[i];
  if (tid == 0) {
    U.theta[of.vbo] = VW.bo[0];
    U.beta_pow[0] = b1p;
    U.beta_pow[1] = b2p;
  }
}

static size_t update_lds_bytes(int O) {
  return (size_t)(LDS_WEIGHTS_FLOATS(O) + 2 * 128 * 64 + 128 * 16 + 8 * SCR_ROWS + 32) * 4;
}

template <int A, int KS1>
static void launch_update_t(hipStream_t s, const UpdateBatch& ub, int P) {
  hipLaunchKernelGGL((k_update_ffn<A, KS1>), dim3(P), dim3(NT), update_lds_bytes(2 * A), s, ub);
}

void launch_update_ffn(hipStream_t s, const UpdateArgs* ua_dev, const UpdateHyper& h, int nrows, float inv_n,
                       int A, int d) {
  UpdateBatch ub;
  ub.a = ua_dev;
  ub.h = h;
  ub.nrows = nrows;
  ub.inv_n = inv_n;
  DDRL_DISPATCH_A_KS1(A, d, launch_update_t, s, ub, h.P);
}

// ------------------------------------------------------------------------------------
// DDP apply: tf.clip_by_global_norm + tf1 Adam on an all-reduced flat gradient.
// One workgroup; fixed-order reduction of the squared norm.
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_apply_adam(const float* __restrict__ grad, int n,
                                                     float* theta, float* m, float* v,
                                                     float* beta_pow, UpdateHyper h) {
  __shared__ float red[16];
  const int tid = threadIdx.x;
  float ss = 0.f;
  for (int i = tid; i < n; i += 1024) ss += grad[i] * grad[i];
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
  const float b1p = beta_pow[0], b2p = beta_pow[1];
  const float alpha = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float c1 = 1.f - h.b1, c2 = 1.f - h.b2;
  for (int i = tid; i < n; i += 1024) {
    const float g = grad[i] * scale;
    float mi = m[i], vi = v[i];
    mi = mi + (g - mi) * c1;
    vi = vi + (g * g - vi) * c2;
    m[i] = mi;
    v[i] = vi;
    theta[i] = theta[i] - (mi * alpha) / (sqrtf(vi) + h.eps);
  }
  __syncthreads();
  if (tid == 0) {
    beta_pow[0] = b1p * h.b1;
    beta_pow[1] = b2p * h.b2;
  }
}

void launch_apply_adam(hipStream_t s, const float* grad, int n, float* theta, float* m, float* v,
                       float* beta_pow, const UpdateHyper& h) {
  hipLaunchKernelGGL(k_apply_adam, dim3(1), dim3(1024), 0, s, grad, n, theta, m, v, beta_pow, h);
}
