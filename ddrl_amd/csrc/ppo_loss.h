// Per-row PPO loss (RLlib 1.0 ppo_tf_policy.PPOLoss) and its analytic output gradient,
// shared by the fcnet and GraphNet update kernels.
#pragma once
#include "common.h"
#include "kernels.h"

// Per-row PPO loss terms and output gradient (policy branch).
template <int A>
__device__ __forceinline__ void policy_loss_row(const float* out, const float* act, const float* ol,
                                                float logp_old, float adv, float beta, float lo, float hi,
                                                float ent_coeff, float inv_n, bool ok, float* dout, float* st) {
  // hardware exp / no divisions: 1 / sd = exp(-log_std), sd_old^2 = exp(2 log_std_old)
  float logp = -0.5f * (float)(DDRL_LOG2PI * A), klr = 0.f, ent = 0.f;
  float z[A], isd[A], q0[A];
#pragma unroll
  for (int j = 0; j < A; ++j) {
    isd[j] = __expf(-out[A + j]);
    z[j] = (act[j] - out[j]) * isd[j];
    logp -= 0.5f * z[j] * z[j];
    logp -= out[A + j];
    const float dm = ol[j] - out[j];
    q0[j] = __expf(2.f * ol[A + j]) + dm * dm;
    klr += out[A + j] - ol[A + j] + 0.5f * q0[j] * (isd[j] * isd[j]) - 0.5f;
    ent += out[A + j] + 0.5f * (float)(DDRL_LOG2PI + 1.0);
  }
  const float ratio = __expf(logp - logp_old);
  const float cr = fminf(fmaxf(ratio, lo), hi);
  const float s1 = adv * ratio, s2 = adv * cr;
  const float surr = fminf(s1, s2);
  const float dr = (s1 <= s2) ? adv : ((ratio >= lo && ratio <= hi) ? adv : 0.f);
  const float glogp = -dr * ratio;
#pragma unroll
  for (int j = 0; j < A; ++j) {
    const float iv = isd[j] * isd[j];
    const float dmu = glogp * (z[j] * isd[j]) + beta * ((out[j] - ol[j]) * iv);
    const float dls = glogp * (z[j] * z[j] - 1.f) + beta * (1.f - q0[j] * iv) - ent_coeff;
    dout[j] = ok ? dmu * inv_n : 0.f;
    dout[A + j] = ok ? dls * inv_n : 0.f;
  }
  st[0] = ok ? -surr : 0.f;
  st[1] = ok ? klr : 0.f;
  st[2] = ok ? ent : 0.f;
}

// Per-row clipped value loss (RLlib 1.0 PPO2 style, or later RLlib's clip of the square).
__device__ __forceinline__ void value_loss_row(float V, float vfo, float vtg, const UpdateHyper& H,
                                               float inv_n, bool ok, float* dout, float* st) {
  float vf, dvf;
  if (H.vf_mode == 0) {
    const float vf1 = (V - vtg) * (V - vtg);
    const float dv = V - vfo;
    const float vcl = vfo + fminf(fmaxf(dv, -H.vf_clip), H.vf_clip);
    const float vf2 = (vcl - vtg) * (vcl - vtg);
    vf = fmaxf(vf1, vf2);
    dvf = (vf1 >= vf2) ? 2.f * (V - vtg)
                       : ((dv >= -H.vf_clip && dv <= H.vf_clip) ? 2.f * (vcl - vtg) : 0.f);
  } else {
    const float sq = (V - vtg) * (V - vtg);
    vf = fminf(sq, H.vf_clip);
    dvf = sq <= H.vf_clip ? 2.f * (V - vtg) : 0.f;
  }
  dout[0] = ok ? H.vf_coeff * dvf * inv_n : 0.f;
  const float dd = vtg - V;
  st[0] = ok ? vf : 0.f;
  st[1] = ok ? vtg : 0.f;
  st[2] = ok ? vtg * vtg : 0.f;
  st[3] = ok ? dd : 0.f;
  st[4] = ok ? dd * dd : 0.f;
}

