// f1: the host env plane -- a vectorized QuAntruped stand-in stepped by a pool of host
// threads into pinned buffers (the reference steps MuJoCo envs on its
// rollout workers' cores: simulation_envs/quantruped_v3.py:166-267, and the adaptor's
// step(action_dict) -> obs / reward / done dicts, quantruped_adaptor_multi_environment.py:220-250).
//
// MuJoCo is not in this image, so the dynamics are a clean-room stand-in with the reference
// env's interface and layout, NOT a physics engine: 8 actuated hip / knee joints driven by the
// clipped actions (gear, spring, damping, joint limits), a torso whose forward velocity is
// pushed by the feet that touch the ground and whose height / roll / pitch follow the legs,
// frame_skip 5 at dt 0.01 (0.05 s per env step, quantruped_v3.py's dt).  It emits exactly what
// the device path consumes: obs43 = [qpos[2:15] (z, quaternion w x y z, 8 joint angles),
// qvel (14), actuator + constraint forces (8), ctrl (8)] (+ target velocity as column 44 for the
// TVel envs), the forward reward fw = dx / dt (TVel: the target-velocity reward of
// quantruped_v3.py:391-392), cfrc_ext [14 bodies][6] (contact force on each
// foot body) and done (gym TimeLimit at 1000 steps, or torso height out of [0.1, 1.5]); a done
// env is reset at once (its next observation is the reset one), as RLlib's sampler does.
// Every env is a pure function of (seed, env index, its own actions): results do not depend on
// the thread count or on how the envs are grouped.
#pragma once
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace hostenv {

struct EnvState {
  double x, y, z, vx, vy, vz;       // torso position / velocity
  double roll, pitch, wroll, wpitch;
  double q[8], qd[8];               // joints: [FL hip, FL knee, HL hip, HL knee, HR hip, HR knee, FR hip, FR knee]
  double qfrc[8];                   // last actuator + constraint force per joint
  double foot[4];                   // last contact force per foot
  int steps;                        // steps in the current episode
  uint32_t episode;
  double tv;                        // target velocity of the current episode (TVel envs)
};

// Persistent worker threads; parallel_for splits [0, n) in contiguous chunks, the caller
// takes part, and returns when every chunk is done.
class Pool {
 public:
  explicit Pool(int n_threads);
  ~Pool();
  void parallel_for(int n, const std::function<void(int, int)>& fn);
  int size() const { return (int)workers_.size() + 1; }

 private:
  void run(int id);
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int, int)>* job_ = nullptr;
  int n_ = 0, chunks_ = 0, next_ = 0, finished_ = 0;
  uint64_t generation_ = 0;
  bool stop_ = false;
};

}  // namespace hostenv

struct ddrl_hostenv {
  int N = 0, D = 43;
  // target velocities an episode draws from (random.choice on every reset,
  // quantruped_adaptor_multi_environment.py:47-50, 214-216); one entry for a fixed velocity
  std::vector<double> tv_list{0.0};
  uint64_t seed = 0;
  std::vector<hostenv::EnvState> st;
  // pinned host buffers (hipHostMalloc): obs [N][D], act [N][8], fw [N], cfrc [N][14][6], done [N]
  float *obs = nullptr, *act = nullptr, *fw = nullptr, *cfrc = nullptr;
  uint8_t* done = nullptr;
  bool pinned = false;
  hostenv::Pool* pool = nullptr;

  // a fresh episode of env e: new initial pose and, when draw_tv, a new target velocity
  void reset_env(int e, bool draw_tv = true);
  void write_obs(int e, const double* ctrl);
  void step_env(int e, const float* a8);
  void reset_all();
  // update_environment_after_epoch (adaptor :97-122): every env's physical state and episode
  // step count restart (gym env.reset()), the target velocity stays (only the adaptor's own
  // reset() re-draws it), no done flag is raised and the observation buffer is not rewritten
  // (the adaptor discards env.reset()'s observation; the sampler acts on the last one it has)
  void reset_state();
  // step the envs [e0, e1) with the actions act[e][8]; writes obs / fw / cfrc / done of the range
  void step(int e0, int e1);
};
