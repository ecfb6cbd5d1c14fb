// f1: host env plane -- the clean-room vectorized QuAntruped stand-in and its thread pool
// (see hostenv.h), plus the C-ABI to create / reset / step it.  The pipelined rollout over
// it (ddrl_rollout_hostenv) lives in capi.cpp next to the context it drives.
#include "hostenv.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/ddrl_hip.h"

namespace hostenv {

Pool::Pool(int n_threads) {
  for (int i = 1; i < std::max(1, n_threads); ++i) workers_.emplace_back([this, i] { run(i); });
}

Pool::~Pool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void Pool::run(int) {
  // A worker takes chunks only of the generation it woke up for: a worker still looping after
  // the last chunk of generation g was finished must not pick up a chunk of g + 1 with g's job
  // (the caller's function object is gone by then).
  uint64_t seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || generation_ != seen; });
    if (stop_) return;
    seen = generation_;
    const std::function<void(int, int)>* job = job_;
    while (generation_ == seen && next_ < chunks_) {
      const int c = next_++, n = n_, ch = chunks_;
      lk.unlock();
      (*job)((int)((long long)n * c / ch), (int)((long long)n * (c + 1) / ch));
      lk.lock();
      if (++finished_ == ch) done_cv_.notify_all();
    }
  }
}

void Pool::parallel_for(int n, const std::function<void(int, int)>& fn) {
  if (n <= 0) return;
  if (workers_.empty()) {
    fn(0, n);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    job_ = &fn;
    n_ = n;
    chunks_ = std::min(n, 4 * size());
    next_ = 0;
    finished_ = 0;
    ++generation_;
  }
  cv_.notify_all();
  for (;;) {   // the caller works too
    int c;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (next_ >= chunks_) break;
      c = next_++;
    }
    const int lo = (int)((long long)n * c / chunks_), hi = (int)((long long)n * (c + 1) / chunks_);
    fn(lo, hi);
    std::lock_guard<std::mutex> lk(mu_);
    if (++finished_ == chunks_) done_cv_.notify_all();
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return finished_ == chunks_; });
  job_ = nullptr;
}

// counter-based generator: uniform in [-1, 1) from (seed, env, episode, draw)
static double hash_uniform(uint64_t seed, uint64_t env, uint64_t episode, uint64_t k) {
  uint64_t z = seed ^ (env * 0x9E3779B97F4A7C15ull) ^ (episode * 0xBF58476D1CE4E5B9ull) ^ (k * 0x94D049BB133111EBull);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

}  // namespace hostenv

using hostenv::EnvState;

namespace {
constexpr double kH = 0.01;           // integration step; frame_skip 5 -> 0.05 s per env step
constexpr int kFrameSkip = 5;
constexpr double kDt = kH * kFrameSkip;
constexpr int kTimeLimit = 1000;      // gym TimeLimit of the registered envs (simulation_envs/__init__.py:27-32)
constexpr double kQ0[8] = {0.0, 1.0, 0.0, -1.0, 0.0, -1.0, 0.0, 1.0};   // rest pose (knees bent)
constexpr double kGear = 30.0, kSpring = 8.0, kDamp = 1.5, kLimit = 1.4;
constexpr double kShin = 0.7, kHipOff = 0.08, kGround = 400.0, kGroundDamp = 8.0;
constexpr uint64_t kTvDraw = 1u << 20;   // counter index of the target-velocity draw (pose draws use 0..16)
}  // namespace

void ddrl_hostenv::reset_env(int e, bool draw_tv) {
  EnvState& s = st[e];
  const uint32_t ep = s.episode + 1;
  const double tv = s.tv;
  std::memset(&s, 0, sizeof(s));
  s.episode = ep;
  s.tv = tv;
  if (draw_tv) {
    // random.choice(target_velocity_list): every list position equally likely (a repeated value
    // counts once per position); draw index kTvDraw of the episode's counter stream
    const double u = 0.5 * (hostenv::hash_uniform(seed, e, ep, kTvDraw) + 1.0);   // [0, 1)
    const size_t n = tv_list.size();
    s.tv = tv_list[std::min(n - 1, (size_t)(u * (double)n))];
  }
  int k = 0;
  s.z = 0.57 + 0.01 * hostenv::hash_uniform(seed, e, ep, k++);
  for (int j = 0; j < 8; ++j) {
    s.q[j] = kQ0[j] + 0.1 * hostenv::hash_uniform(seed, e, ep, k++);
    s.qd[j] = 0.1 * hostenv::hash_uniform(seed, e, ep, k++);
  }
}

void ddrl_hostenv::write_obs(int e, const double* ctrl) {
  const EnvState& s = st[e];
  float* o = obs + (size_t)e * D;
  // quaternion (w, x, y, z) of roll about x then pitch about y
  const double cr = std::cos(0.5 * s.roll), sr = std::sin(0.5 * s.roll);
  const double cp = std::cos(0.5 * s.pitch), sp = std::sin(0.5 * s.pitch);
  const double qpos[13] = {s.z, cr * cp, sr * cp, cr * sp, -sr * sp, s.q[0], s.q[1], s.q[2], s.q[3],
                           s.q[4], s.q[5], s.q[6], s.q[7]};
  const double qvel[14] = {s.vx, s.vy, s.vz, s.wroll, s.wpitch, 0.0, s.qd[0], s.qd[1], s.qd[2], s.qd[3],
                           s.qd[4], s.qd[5], s.qd[6], s.qd[7]};
  int i = 0;
  for (double v : qpos) o[i++] = (float)v;
  for (double v : qvel) o[i++] = (float)v;
  for (int j = 0; j < 8; ++j) o[i++] = (float)s.qfrc[j];
  for (int j = 0; j < 8; ++j) o[i++] = (float)(ctrl ? ctrl[j] : 0.0);
  if (D > 43) o[i++] = (float)s.tv;
}

void ddrl_hostenv::step_env(int e, const float* a8) {
  EnvState& s = st[e];
  double a[8];
  for (int j = 0; j < 8; ++j) a[j] = std::min(1.0, std::max(-1.0, (double)a8[j]));
  const double x0 = s.x;
  for (int f = 0; f < kFrameSkip; ++f) {
    double thrust = 0.0, lift = 0.0, troll = 0.0, tpitch = 0.0;
    for (int leg = 0; leg < 4; ++leg) {
      const int hip = 2 * leg, knee = hip + 1;
      // foot height below the hip: shin along the knee angle, hip swing lifts it a little
      const double fz = s.z - kShin * std::cos(s.q[knee]) * std::cos(s.q[hip]) + kHipOff * std::fabs(std::sin(s.q[hip]));
      double force = 0.0;
      if (fz < 0.0) force = std::max(0.0, -kGround * fz - kGroundDamp * s.vz);
      s.foot[leg] = force;
      // a stance foot pushes the torso by the hip's backward swing
      thrust += force * 0.05 * (-s.qd[hip]) * std::cos(s.q[hip]);
      lift += force;
      const double side = (leg == 0 || leg == 1) ? 1.0 : -1.0;    // FL, HL left; HR, FR right
      const double front = (leg == 0 || leg == 3) ? 1.0 : -1.0;   // FL, FR front
      troll += side * force;
      tpitch += front * force;
    }
    for (int j = 0; j < 8; ++j) {
      const double tau = kGear * a[j];
      double qdd = tau - kSpring * (s.q[j] - kQ0[j]) - kDamp * s.qd[j];
      s.qd[j] += kH * qdd;
      s.q[j] += kH * s.qd[j];
      double constraint = 0.0;
      if (s.q[j] > kLimit || s.q[j] < -kLimit) {   // joint limit: stop and report the reaction
        const double lim = s.q[j] > 0 ? kLimit : -kLimit;
        constraint = -(s.q[j] - lim) / (kH * kH);
        s.q[j] = lim;
        s.qd[j] = 0.0;
      }
      s.qfrc[j] = tau + std::max(-100.0, std::min(100.0, constraint));
    }
    s.vx += kH * (thrust - 0.8 * s.vx);
    s.vy += kH * (-0.8 * s.vy + 0.02 * troll * std::sin(s.roll));
    s.vz += kH * (lift / 8.0 - 9.81 - 1.0 * s.vz);
    s.wroll += kH * (0.02 * troll - 4.0 * s.roll - 1.5 * s.wroll);
    s.wpitch += kH * (0.02 * tpitch - 4.0 * s.pitch - 1.5 * s.wpitch);
    s.x += kH * s.vx;
    s.y += kH * s.vy;
    s.z += kH * s.vz;
    s.roll += kH * s.wroll;
    s.pitch += kH * s.wpitch;
  }
  ++s.steps;
  // forward reward of the step (quantruped_v3.py:163-179): the torso's x velocity; the TVel
  // envs reward reaching the target velocity instead (QuAntrupedTVelEnv.compute_forward_reward,
  // quantruped_v3.py:391-392)
  const double vx = (s.x - x0) / kDt;
  if (D > 43) {
    const double tv = s.tv;
    fw[e] = (float)((1.0 + 1.0 / tv) * (1.0 / (std::fabs(vx - tv) + 1.0) - 1.0 / (tv + 1.0)));
  } else {
    fw[e] = (float)vx;
  }
  // cfrc_ext [14][6]: {floor, torso, then hip / leg / foot of FL, HL, HR, FR}; rotational then
  // linear part, the contact force on the foot bodies
  float* cf = cfrc + (size_t)e * 14 * 6;
  std::fill(cf, cf + 14 * 6, 0.f);
  for (int leg = 0; leg < 4; ++leg) {
    float* foot = cf + (4 + 3 * leg) * 6;
    const double f = s.foot[leg];
    foot[0] = (float)(0.01 * f * std::sin(s.q[2 * leg]));
    foot[3] = (float)(0.1 * f * std::sin(s.q[2 * leg]));
    foot[5] = (float)f;
    cf[1 * 6 + 5] += (float)(0.05 * f);
  }
  const bool unhealthy = !(s.z > 0.1 && s.z < 1.5) || !std::isfinite(s.z);
  const bool d = unhealthy || s.steps >= kTimeLimit;
  done[e] = d ? 1 : 0;
  if (d) {
    reset_env(e);
    write_obs(e, nullptr);
  } else {
    write_obs(e, a);
  }
}

void ddrl_hostenv::reset_all() {
  pool->parallel_for(N, [this](int lo, int hi) {
    for (int e = lo; e < hi; ++e) {
      st[e].episode = 0;
      reset_env(e);
      // staggered episode phases, like a long-running sampler (the synthetic rollouts too)
      st[e].steps = (int)(((uint64_t)e * 2654435761ull + seed) % kTimeLimit);
      write_obs(e, nullptr);
      done[e] = 0;
    }
  });
}

void ddrl_hostenv::reset_state() {
  pool->parallel_for(N, [this](int lo, int hi) {
    for (int e = lo; e < hi; ++e) reset_env(e, false);   // steps = 0: the TimeLimit count restarts too
  });
}

void ddrl_hostenv::step(int e0, int e1) {
  pool->parallel_for(e1 - e0, [this, e0](int lo, int hi) {
    for (int e = e0 + lo; e < e0 + hi; ++e) step_env(e, act + (size_t)e * 8);
  });
}

// ---- C-ABI ------------------------------------------------------------------------------
namespace {
thread_local std::string g_henv_err;
}
extern "C" const char* ddrl_hostenv_last_error(void) { return g_henv_err.c_str(); }

extern "C" int ddrl_hostenv_create(int n_envs, int obs_dim, int n_threads, uint64_t seed, float target_velocity,
                                   ddrl_hostenv** out) {
  if (!out || n_envs < 1 || (obs_dim != 43 && obs_dim != 44) || n_threads < 1 ||
      (obs_dim == 44 && !(target_velocity > 0.f))) {
    g_henv_err = "ddrl_hostenv_create: n_envs >= 1, obs_dim 43 or 44 (44: target_velocity > 0), n_threads >= 1";
    return -1;
  }
  auto* h = new ddrl_hostenv();
  h->N = n_envs;
  h->D = obs_dim;
  h->seed = seed;
  h->tv_list.assign(1, (double)target_velocity);
  h->st.assign(n_envs, EnvState{});
  // the create-time velocity until the first reset draws one (a step before any reset must not
  // divide by zero in the TVel reward)
  for (auto& s : h->st) s.tv = (double)target_velocity;
  const size_t N = n_envs;
  // pinned when a GPU is present (the DMA engines read / write them directly); without one
  // (CPU tests of the env plane) ordinary aligned host memory
  int ndev = 0;
  h->pinned = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
  auto alloc = [&](void** p, size_t bytes) {
    if (h->pinned) return hipHostMalloc(p, bytes, hipHostMallocDefault) == hipSuccess;
    *p = std::aligned_alloc(64, (bytes + 63) / 64 * 64);
    return *p != nullptr;
  };
  if (!alloc((void**)&h->obs, N * obs_dim * 4) || !alloc((void**)&h->act, N * 8 * 4) || !alloc((void**)&h->fw, N * 4) ||
      !alloc((void**)&h->cfrc, N * 14 * 6 * 4) || !alloc((void**)&h->done, N)) {
    g_henv_err = "ddrl_hostenv_create: host buffer allocation failed";
    ddrl_hostenv_destroy(h);
    return -1;
  }
  std::memset(h->act, 0, N * 8 * 4);
  h->pool = new hostenv::Pool(n_threads);
  *out = h;
  return 0;
}

extern "C" int ddrl_hostenv_destroy(ddrl_hostenv* h) {
  if (!h) return 0;
  delete h->pool;
  for (void* p : {(void*)h->obs, (void*)h->act, (void*)h->fw, (void*)h->cfrc, (void*)h->done}) {
    if (!p) continue;
    if (h->pinned) (void)hipHostFree(p);
    else std::free(p);
  }
  delete h;
  return 0;
}

extern "C" int ddrl_hostenv_buffers(ddrl_hostenv* h, float** obs, float** act, float** fw, float** cfrc,
                                    uint8_t** done) {
  if (!h) {
    g_henv_err = "null host env";
    return -1;
  }
  if (obs) *obs = h->obs;
  if (act) *act = h->act;
  if (fw) *fw = h->fw;
  if (cfrc) *cfrc = h->cfrc;
  if (done) *done = h->done;
  return 0;
}

extern "C" int ddrl_hostenv_reset(ddrl_hostenv* h) {
  if (!h) {
    g_henv_err = "null host env";
    return -1;
  }
  h->reset_all();
  return 0;
}

extern "C" int ddrl_hostenv_step(ddrl_hostenv* h, int e0, int e1) {
  if (!h || e0 < 0 || e1 > h->N || e0 >= e1) {
    g_henv_err = "ddrl_hostenv_step: bad env range";
    return -1;
  }
  h->step(e0, e1);
  return 0;
}

extern "C" int ddrl_hostenv_threads(ddrl_hostenv* h) { return h ? h->pool->size() : 0; }

extern "C" int ddrl_hostenv_set_target_velocities(ddrl_hostenv* h, const float* list, int n) {
  if (!h || !list || n < 1) {
    g_henv_err = "ddrl_hostenv_set_target_velocities: a list of n >= 1 values";
    return -1;
  }
  for (int i = 0; i < n; ++i) {
    if (h->D > 43 && !(list[i] > 0.f)) {
      g_henv_err = "ddrl_hostenv_set_target_velocities: obs_dim 44 needs target velocities > 0 "
                   "(the TVel reward divides by it)";
      return -1;
    }
  }
  h->tv_list.assign(list, list + n);
  return 0;
}

extern "C" int ddrl_hostenv_target_velocities(ddrl_hostenv* h, float* out, int n) {
  if (!h || !out || n != h->N) {
    g_henv_err = "ddrl_hostenv_target_velocities: out holds n_envs floats";
    return -1;
  }
  for (int e = 0; e < n; ++e) out[e] = (float)h->st[e].tv;
  return 0;
}

extern "C" int ddrl_hostenv_reset_state(ddrl_hostenv* h) {
  if (!h) {
    g_henv_err = "null host env";
    return -1;
  }
  h->reset_state();
  return 0;
}
