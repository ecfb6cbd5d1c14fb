/* ddrl_hip.h -- C-ABI of libddrl_hip.so, the MI355X (gfx950) hot path of DDRL.
 *
 * This boundary replaces the numeric work that the reference delegates to RLlib 1.0.x and
 * TensorFlow 2.3, which run behind two plugin interfaces:
 *   (1) MultiAgentEnv: simulation_envs/quantruped_adaptor_multi_environment.py:8-272
 *       (distribute_observations :124-136, distribute_reward :173-203,
 *        concatenate_actions :205-212, step :220-250)
 *   (2) ModelV2: models/fcnet_glorot_uniform_init.py:10-125 ("ffn"),
 *       models/shared_graphnet_glorot_uniform_init.py:14-58 + graph_net.py + gcn.py ("gnn"),
 *       registered in models/__init__.py:7-13.
 * The RLlib side they plug into (sampling, GAE, PPOLoss, clip_gradients, Adam, minibatch
 * SGD, KL update) is rebuilt here as HIP kernels.  Host code -- Python through ctypes, or a
 * maintainer's own FFI binding -- drives these entry points.
 *
 * Conventions
 *   - Every function returns int status: 0 = OK, < 0 = error; ddrl_last_error() returns a
 *     thread-local message.  No exceptions cross the boundary.
 *   - Pointers named *_dev are device (HBM) pointers.  Pointers named *_host are host
 *     memory (pageable or pinned).  Work is enqueued on the context's stream
 *     (ddrl_set_stream) and is asynchronous unless stated otherwise.
 *   - One context = one device + one stream; calls on a context are serialized by the caller.
 */
#ifndef DDRL_HIP_H
#define DDRL_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DDRL_ABI_VERSION 4
#define DDRL_MAX_POLICIES 4
#define DDRL_MAX_AGENTS 4
#define DDRL_MAX_OBS 48

enum { DDRL_MODEL_FFN = 0, DDRL_MODEL_GNN = 1 };
enum { DDRL_REWARD_PER_LEG = 0, DDRL_REWARD_GLOBAL = 1, DDRL_REWARD_NORM = 2 };
enum { DDRL_VF_CLIP_RAY10 = 0, DDRL_VF_CLIP_SQUARED = 1 };
/* message-passing layer of the "gnn" model (models/graph_net.py:20 selects one of
 * models/gcn.py's layers: MPNN :39-94 (the reference's default), GCN :7-37, MPNN2 :96-150,
 * GAT1 :153-206) */
enum { DDRL_GNN_MPNN = 0, DDRL_GNN_GCN = 1, DDRL_GNN_MPNN2 = 2, DDRL_GNN_GAT1 = 3 };

/* Static configuration of one context (one env shard of one trainer). */
typedef struct ddrl_cfg {
  int32_t n_envs;        /* N: parallel environments on this device                      */
  int32_t frag_len;      /* T: rollout_fragment_length                                     */
  int32_t obs_full_dim;  /* 43 (44 with target velocity)                                   */
  int32_t n_agents;      /* agents per env: 4 (legs), 2 (sides/diagonals), 1 (centralized) */
  int32_t n_policies;    /* P                                                              */
  int32_t model_kind;    /* DDRL_MODEL_FFN | DDRL_MODEL_GNN                               */
  int32_t act_dim;       /* A: actions per agent (2, 4 or 8)                               */
  int32_t agent_policy[DDRL_MAX_AGENTS];           /* policy id of every agent            */
  int32_t obs_dim[DDRL_MAX_POLICIES];              /* d per policy (GNN: 19 per node)      */
  int32_t obs_index[DDRL_MAX_AGENTS][DDRL_MAX_OBS];/* gather table per agent (a1); entries
                                                      -1 / -2 are the constants 0 / 1 (the
                                                      one-hot leg id of the LegID env)      */
  int32_t act_index[DDRL_MAX_AGENTS][8];           /* scatter table per agent (a7)         */
  int32_t n_contact[DDRL_MAX_AGENTS];              /* contact-cost bodies per agent (a8)   */
  int32_t contact_index[DDRL_MAX_AGENTS][14];
  float contact_weight[DDRL_MAX_AGENTS][14];
  float leg_angle_deg[DDRL_MAX_AGENTS];            /* GNN ego encoding (FL,HL,HR,FR)       */
  int32_t filter_enabled;   /* env-side MeanStdFilter on the full observation (a2)         */
  int32_t filter_update;    /* push batches into the running statistics                   */
  float filter_clip;        /* 10 in the reference; 0 = no clip                            */
  int32_t reward_mode;      /* DDRL_REWARD_*                                                */
  float ctrl_cost_weight;
  float contact_cost_weight;
  float gamma, lambda_;
  float clip_param, vf_clip_param, vf_loss_coeff, entropy_coeff;
  float lr, grad_clip;
  float adam_beta1, adam_beta2, adam_eps;
  int32_t vf_clip_mode;     /* DDRL_VF_CLIP_*                                               */
  int32_t sgd_minibatch_size;  /* 128 (the fused update kernel is built for 128)          */
  int32_t num_sgd_iter;        /* 10                                                       */
  int32_t act_negate[DDRL_MAX_AGENTS][8];  /* 1: negate action j of the agent in the env action
                                              vector (LegTransforms: fr / hr knee)          */
  int32_t policy_filter;    /* RLlib observation_filter "MeanStdFilter" on every policy's
                               input (after the env-side filter; unclipped, fp64 stats)     */
  int32_t leg_coupling;     /* "cup" model (models/coupling_net_glorot_uniform_init.py:11-30,
                               registered models/__init__.py:10): the action means of the
                               shared leg policy are scaled by a trainable table [4][A],
                               row = the agent's leg index (SharedDecentralLegID env, :66-114);
                               the table follows the fcnet variables in the parameter vector */
  int32_t gnn_layer;        /* DDRL_GNN_* (model_kind GNN): the layer's kernels sit between the
                               state encoder and linear_out of each net, in Keras order */
} ddrl_cfg;

typedef struct ddrl_ctx ddrl_ctx;

int ddrl_abi_version(void);
const char* ddrl_last_error(void);

/* Context lifetime.  Allocates every device buffer for T x N rollouts. */
int ddrl_ctx_create(const ddrl_cfg* cfg, int device, ddrl_ctx** out);
int ddrl_ctx_destroy(ddrl_ctx* ctx);
int ddrl_set_stream(ddrl_ctx* ctx, void* hip_stream);
int ddrl_synchronize(ddrl_ctx* ctx);

/* Shapes.  layout_out[11] = {row_stride, off_obs, off_act, off_logits, off_logp, off_vf,
 * off_adv, off_vt, off_rew, rows_per_step (C = N*k), off_leg (leg index of the row, "cup"
 * model; -1 otherwise)}, all in floats. */
int ddrl_param_count(ddrl_ctx* ctx, int pid, int64_t* n_out);
int ddrl_record_layout(ddrl_ctx* ctx, int pid, int32_t* layout_out);

/* Parameter / optimizer / filter state, in the reference's Keras checkpoint order
 * (pid/fc_1/kernel [d,64], fc_1/bias, fc_value_1/..., fc_2/..., fc_value_2/...,
 *  fc_out/..., value_out/...), replacing Policy.get_weights/set_weights. */
int ddrl_params_set(ddrl_ctx* ctx, int pid, const float* host, size_t n);
int ddrl_params_get(ddrl_ctx* ctx, int pid, float* host, size_t n);
int ddrl_adam_set(ddrl_ctx* ctx, int pid, const float* m_host, const float* v_host, size_t n,
                  float beta1_power, float beta2_power);
int ddrl_adam_get(ddrl_ctx* ctx, int pid, float* m_host, float* v_host, size_t n,
                  float* beta1_power, float* beta2_power);
int ddrl_filter_set(ddrl_ctx* ctx, double n, const double* mean_host, const double* sq_host);
int ddrl_filter_get(ddrl_ctx* ctx, double* n, double* mean_host, double* sq_host);
/* Pushes since the last ddrl_filter_delta_reset, as their own running stat (RLlib's filter
 * "buffer"); a data-parallel trainer merges every rank's delta into the synced filter
 * (RunningStat.update in rank order) and resets (synchronize_filters, P_Local:160). */
int ddrl_filter_delta_get(ddrl_ctx* ctx, double* n, double* mean_host, double* sq_host);
int ddrl_filter_delta_reset(ddrl_ctx* ctx);
/* The per-policy RLlib MeanStdFilter (cfg.policy_filter): RunningStat of policy pid over its
 * obs_dim input columns, and its pushes since the last delta reset (same sync protocol). */
int ddrl_policy_filter_set(ddrl_ctx* ctx, int pid, double n, const double* mean_host, const double* sq_host);
int ddrl_policy_filter_get(ddrl_ctx* ctx, int pid, double* n, double* mean_host, double* sq_host);
int ddrl_policy_filter_delta_get(ddrl_ctx* ctx, int pid, double* n, double* mean_host, double* sq_host);
int ddrl_policy_filter_delta_reset(ddrl_ctx* ctx);

/* Rollout (per env step).
 * observe: env-side MeanStdFilter push + normalize + per-agent routing of the raw
 *          observations obs_dev[N][obs_full_dim] (a1/a2/a3).
 * act:     fused forward of every policy on the routed observations, DiagGaussian sample
 *          with explicit noise eps_dev[N][n_agents][A], logp, value; writes training row
 *          t and the clipped env actions actions_dev[N][8] (a4/a6/a7).
 * reward:  per-agent rewards for row t from forward reward fw_dev[N], contact forces
 *          cfrc_dev[N][14][6], the env actions and done flags done_dev[N] (a8).
 * bootstrap: V(s_T) of the routed observations -> last values for GAE. */
int ddrl_observe(ddrl_ctx* ctx, const float* obs_dev);
int ddrl_act(ddrl_ctx* ctx, int t, const float* eps_dev, float* actions_dev);
int ddrl_reward(ddrl_ctx* ctx, int t, const float* fw_dev, const float* cfrc_dev,
                const float* actions_dev, const uint8_t* done_dev);
int ddrl_bootstrap(ddrl_ctx* ctx);
/* The same over the envs [e0, e1) only, on full-size buffers (obs_dev[N][D], eps_dev, actions_dev,
 * fw_dev, cfrc_dev, done_dev): a pipelined host env plane (ddrl_rollout_hostenv) runs its env
 * groups through these so that one group's host step overlaps another group's device work.
 * The env-side filter pushes the range's rows as one batch (groups in call order). */
int ddrl_observe_range(ddrl_ctx* ctx, const float* obs_dev, int e0, int e1);
int ddrl_act_range(ddrl_ctx* ctx, int t, int e0, int e1, const float* eps_dev, float* actions_dev);
int ddrl_reward_range(ddrl_ctx* ctx, int t, int e0, int e1, const float* fw_dev, const float* cfrc_dev,
                      const float* actions_dev, const uint8_t* done_dev);
/* A whole fragment over device-resident env data (a device env, replayed transitions, the
 * synthetic benchmark): for t in [0, T): act(t), reward(t), observe(obs_dev[t + 1]); then
 * bootstrap.  Expects observe(obs_dev[0]) to have been called.  Layouts: obs_dev[T+1][N][D],
 * eps_dev[T][N][n_agents][A], fw_dev[T][N], cfrc_dev[T][N][14][6], done_dev[T][N] (may be
 * NULL), actions_dev[N][8] (scratch: the env actions of the last step).  One call instead of
 * 3 T host calls: the per-step launches stay in C++, captured once into a HIP graph that is
 * re-launched while the six buffer pointers are unchanged (contents may change between calls;
 * DDRL_ROLLOUT_GRAPH=0 at context creation issues the launches directly). */
int ddrl_rollout_fragment(ddrl_ctx* ctx, const float* obs_dev, const float* eps_dev, const float* fw_dev,
                          const float* cfrc_dev, const uint8_t* done_dev, float* actions_dev);
/* Host-buffer variants for a host-side env (MultiAgentEnv.step on host cores): pinned
 * buffers, hipMemcpyAsync on the context's stream, asynchronous like the device calls.
 *   step_host:     obs_host[N][D] in -> observe; eps_host in -> act(t); actions_host[N][8] out
 *                  (the reset observation and the first action of a fragment);
 *   act_host:      eps_host in -> act(t) on the staged observation -> actions_host out;
 *   env_step_host: the env's answer to the actions of step t: fw_host[N], cfrc_host[N][14][6],
 *                  done_host[N] (may be NULL) -> reward(t); obs_next_host[N][D] -> observe.
 * A loop over t: act_host(t) (step_host for t = 0), synchronize, step the envs on the host,
 * env_step_host(t). */
int ddrl_step_host(ddrl_ctx* ctx, int t, const float* obs_host, const float* eps_host,
                   float* actions_host);
int ddrl_act_host(ddrl_ctx* ctx, int t, const float* eps_host, float* actions_host);
int ddrl_env_step_host(ddrl_ctx* ctx, int t, const float* fw_host, const float* cfrc_host,
                       const uint8_t* done_host, const float* obs_next_host);

/* f1 host env plane (hostenv.cpp): a vectorized QuAntruped stand-in (clean-room kinematics in
 * the reference env's layout -- MuJoCo is absent; see hostenv.h) stepped by a pool of
 * n_threads host threads into pinned buffers obs[N][obs_dim], act[N][8], fw[N],
 * cfrc[N][14][6], done[N] (ddrl_hostenv_buffers).  Replaces the reference's per-worker
 * MuJoCo stepping (simulation_envs/quantruped_v3.py:166-267) and the adaptor's
 * step(action_dict) (quantruped_adaptor_multi_environment.py:220-250).
 *   step: the envs [e0, e1) with act[e][8] (clipped to [-1, 1]); a done env is reset at once.
 * ddrl_rollout_hostenv runs a whole fragment over it, pipelined over `groups` env groups (one
 * group's host step overlaps the other groups' device work and transfers), then bootstraps. */
typedef struct ddrl_hostenv ddrl_hostenv;
const char* ddrl_hostenv_last_error(void);
int ddrl_hostenv_create(int n_envs, int obs_dim, int n_threads, uint64_t seed, float target_velocity,
                        ddrl_hostenv** out);
int ddrl_hostenv_destroy(ddrl_hostenv* env);
int ddrl_hostenv_buffers(ddrl_hostenv* env, float** obs, float** act, float** fw, float** cfrc, uint8_t** done);
int ddrl_hostenv_reset(ddrl_hostenv* env);
int ddrl_hostenv_step(ddrl_hostenv* env, int e0, int e1);
int ddrl_hostenv_threads(ddrl_hostenv* env);
/* Target velocities of the TVel envs (obs_dim 44): every env draws its episode's velocity
 * uniformly from list[0..n) on every reset, the adaptor's random.choice(target_velocity_list)
 * at construction and in reset() (quantruped_adaptor_multi_environment.py:47-50, 214-216); the
 * draw takes effect at the next reset (ddrl_hostenv_reset, or an episode end).  create's
 * target_velocity is the list of one.  target_velocities: each env's current velocity. */
int ddrl_hostenv_set_target_velocities(ddrl_hostenv* env, const float* list, int n);
int ddrl_hostenv_target_velocities(ddrl_hostenv* env, float* out, int n_envs);
/* update_environment_after_epoch (quantruped_adaptor_multi_environment.py:97-122, after every
 * training iteration through on_train_result, train_experiment_1_architecture_on_flat.py:171-178):
 * every env's state and TimeLimit count restart (gym env.reset()), the target velocity is kept,
 * no done flag is raised and obs is not rewritten (the adaptor discards that observation).
 * The terrain regeneration of the same hook is MuJoCo-side (out of scope). */
int ddrl_hostenv_reset_state(ddrl_hostenv* env);
int ddrl_rollout_hostenv(ddrl_ctx* ctx, ddrl_hostenv* env, int groups, const float* eps_dev, int reset);

/* Postprocessing: GAE over the fragment for every policy + advantage standardization
 * statistics (a11/a12). */
int ddrl_gae(ddrl_ctx* ctx);
/* fp64 {sum adv, sum adv^2, count} of policy pid from the last ddrl_gae, for a cross-rank
 * StandardizeFields (the global {mean, max(1e-4, std)} goes back through adv_norm_set). */
int ddrl_adv_sums_get(ddrl_ctx* ctx, int pid, double* host3);

/* PPO update of policy pid_mask bits (a13-a17).  Per policy p (bit p set):
 *   shuffle_dev[p] : int32[R_p] row permutation (SampleBatch.shuffle)
 *   perm_dev[p]    : int32[num_sgd_iter][nb_p] minibatch-slot permutation per epoch,
 *                    nb_p = max(1, R_p / sgd_minibatch_size)
 *   kl_coeff[p]    : current KL coefficient
 * max_steps < 0 runs the whole schedule; >= 0 runs only the first max_steps minibatches.
 * All policies in the mask run concurrently (one persistent workgroup each). */
int ddrl_ppo_update(ddrl_ctx* ctx, int pid_mask, const int32_t* const* shuffle_dev,
                    const int32_t* const* perm_dev, const float* kl_coeff, int max_steps);
/* The same update resumed at minibatch step step0 of the schedule (step0 = e * nb + b), from the
 * weights, Adam state and beta powers the context holds (e.g. restored from a mid-update
 * checkpoint): bit-identical to steps step0 .. of one uninterrupted ddrl_ppo_update (round 6; the
 * fused exchange's tag bits follow the schedule step).  Learner statistics land in rows step0 ..;
 * max_steps counts from step0.  ddrl_ppo_update is ddrl_ppo_update_from(…, 0, max_steps). */
int ddrl_ppo_update_from(ddrl_ctx* ctx, int pid_mask, const int32_t* const* shuffle_dev,
                         const int32_t* const* perm_dev, const float* kl_coeff, int step0, int max_steps);
/* Per-minibatch learner stats of the last update: n_steps x 8 floats
 * {total_loss, policy_loss, vf_loss, kl, entropy, vf_explained_var, grad_gnorm, clip_scale}. */
int ddrl_ppo_stats(ddrl_ctx* ctx, int pid, float* host, size_t n_steps);
/* Rows [first, first + n_steps) of the same statistics: RLlib's learner stats and update_kl
 * (3p ppo.py update_kl, on the last epoch's mean KL) need only the last epoch's nb rows. */
int ddrl_ppo_stats_range(ddrl_ctx* ctx, int pid, size_t first, size_t n_steps, float* host);

/* Data-parallel (shared policy) primitives: gradient of (1/minibatch) * sum over the
 * given rows -> grad_dev[n_params]; after the caller's all-reduce (RCCL), apply clip +
 * Adam.  rows_dev holds n_rows (<= 128) record indices.  stats_step >= 0 also writes this
 * rank's loss statistics of the rows (means over n_rows) into stats row stats_step. */
int ddrl_ppo_grad(ddrl_ctx* ctx, int pid, const int32_t* rows_dev, int n_rows,
                  float kl_coeff, float* grad_dev, int stats_step);
int ddrl_ppo_apply(ddrl_ctx* ctx, int pid, const float* grad_dev);

/* RCCL communicator of a data-parallel learner (SURVEY 8(b) "ddrl_comm_init"; replaces the
 * GPU-tower gradient averaging of RLlib's TrainTFMultiGPU, 3p execution/train_ops.py, which
 * the reference sizes with ray.init(num_gpus=...) at train_experiment_1_architecture_on_flat.py:94
 * and the commented config['num_gpus'] at :103-106).  Rank 0 makes
 * the unique id (DDRL_COMM_ID_BYTES bytes, handed to the other ranks by the caller, e.g. a
 * torch.distributed broadcast), every rank joins with its rank; one communicator per context,
 * on the context's device.  comm_allreduce sums n floats in place on the context's stream. */
#define DDRL_COMM_ID_BYTES 128
int ddrl_comm_unique_id(void* id_out, size_t n);
int ddrl_comm_init(ddrl_ctx* ctx, const void* id, int rank, int nranks);
int ddrl_comm_allreduce(ddrl_ctx* ctx, float* buf_dev, size_t n);
/* The data-parallel minibatch SGD of policy pid, enqueued from C++ on the context's stream
 * (per step: gradient of this rank's rows -> RCCL all-reduce -> clip + Adam), the per-step
 * loop of ddrl_amd/ddp.py DataParallelLearner.learn without a host round trip per call.
 *   shuffle_dev: this rank's row permutation; perm_host[n_epochs][nb]: minibatch slots;
 *   rows_per_rank: 128 / ranks ("split") or 128 ("local"); grad_scale: 1 or 1 / ranks.
 * Learner statistics of the last epoch land in ddrl_ppo_stats rows 0 .. nb - 1.
 * The records of each run of up to 1,024 steps are gathered on the device into one chunk
 * (allocated by the first call: min(1024, steps) x rows_per_rank x record stride floats) before
 * that run's gradient launches; perm_host is copied to the device once per call. */
int ddrl_ppo_update_ddp(ddrl_ctx* ctx, int pid, const int32_t* shuffle_dev, const int32_t* perm_host,
                        int n_epochs, int nb, int rows_per_rank, float kl_coeff, float grad_scale);

/* Peer mode (round 5): the shared-policy minibatch SGD of two ranks as ONE
 * fused persistent update split across the ranks' contexts -- the reference's 128-row minibatch
 * ("split" semantics; train_shared_policy_architecture_on_flat.py:48,79 via RLlib's
 * TrainTFMultiGPU) with rank r's 64 rows of every minibatch in rank r's fused launch, which swaps
 * its partial gradients with the peer launch every step through shared outboxes (LSB-tagged
 * quads, system-scope stores and loads; no collective, no per-step launch), then runs the same
 * clip + Adam:
 * both ranks' weights stay bit-identical to each other and to one fused launch over the union
 * batch.  fcnet models, row split on (the default), two ranks.
 *   ddrl_peer_alloc: rank 0 allocates the outboxes (fine-grained device memory, cleared) and,
 *     with ipc_handle_out, exports them (DDRL_PEER_HANDLE_BYTES, hipIpcGetMemHandle);
 *   ddrl_peer_open: rank 1 maps rank 0's outboxes from that handle (another process);
 *   ddrl_peer_attach: both ranks, before their first peer update (a context in the same
 *     process passes rank 0's pointer directly); resets the launch tags; rank 0's attach also
 *     clears the outboxes, so rank 1 attaches after it (and after a failed update both re-attach);
 *     it reserves the buffers of num_sgd_iter epochs of R / 64 slots (a larger schedule grows
 *     them, which waits for the whole device: a stall for a peer context of the same process);
 *   ddrl_ppo_update_peer: shuffle_dev = this rank's nb * 64 row indices (minibatch slot b owns
 *     entries [64 b, 64 b + 64)), perm_dev[n_epochs][nb] = the slots, the same on both ranks.
 *     Both ranks must issue the same sequence of peer updates, and each launch needs its peer's
 *     launch to run concurrently (a wait abandoned after 3 s raises, with the snapshot restored).
 *     A failed peer update detaches the context: the next ddrl_ppo_update_peer is refused ("no
 *     peer") until both ranks have called ddrl_peer_attach again, which clears the outboxes. */
#define DDRL_PEER_HANDLE_BYTES 64
int ddrl_peer_alloc(ddrl_ctx* ctx, void** gx_out, void* ipc_handle_out);
int ddrl_peer_open(ddrl_ctx* ctx, const void* ipc_handle, void** gx_out);
int ddrl_peer_attach(ddrl_ctx* ctx, void* gx, int rank, int nranks);
int ddrl_ppo_update_peer(ddrl_ctx* ctx, int pid, const int32_t* shuffle_dev, const int32_t* perm_dev,
                         int n_epochs, int nb, float kl_coeff, int max_steps);

/* The GraphNet context's minibatch step as it runs now: *on = 1 for the one-launch step (the
 * gradient launch reduces over its tiles and runs clip + Adam in its tail), 0 for the three-launch
 * step (k_gnn + k_gnn_reduce + k_gnn_adam) -- DDRL_GNN_TAIL=0, an occupancy or owner-list refusal,
 * or a fallback after a failed one-launch step -- or before the first 128-row step has built
 * the owner lists; 0 for an fcnet context. */
int ddrl_gnn_one_launch(ddrl_ctx* ctx, int* on);

/* Model forward (ModelV2.forward + value_function) on arbitrary rows:
 * obs_dev[n][d] (ffn; + node_dev[n] = leg index with leg_coupling) or X_dev[n][4][23] +
 * node_dev[n] (gnn). */
int ddrl_policy_forward(ddrl_ctx* ctx, int pid, const float* obs_dev, const int32_t* node_dev,
                        int n, float* logits_dev, float* values_dev);

/* Training-row buffers (SampleBatch columns) of policy pid, [T*C][row_stride] floats:
 * read back for inspection, or loaded from an external batch (e.g. a replayed SampleBatch). */
int ddrl_records_get(ddrl_ctx* ctx, int pid, float* host, size_t n_floats);
int ddrl_records_set(ddrl_ctx* ctx, int pid, const float* host, size_t n_floats);
/* Advantage standardization constants {mean, max(1e-4, std)} of policy pid. */
int ddrl_adv_norm_get(ddrl_ctx* ctx, int pid, float* host2);
int ddrl_adv_norm_set(ddrl_ctx* ctx, int pid, float mean, float denom);
/* Bootstrap values V(s_T) of policy pid, C floats (set: for a replayed batch). */
int ddrl_last_values_get(ddrl_ctx* ctx, int pid, float* host, size_t n);
int ddrl_last_values_set(ddrl_ctx* ctx, int pid, const float* host, size_t n);
/* Episode-end flags of the fragment, [T][N] bytes (normally written by ddrl_reward). */
int ddrl_done_set(ddrl_ctx* ctx, const uint8_t* host, size_t n);

/* Direct device pointers (for zero-copy inspection and collectives). */
int ddrl_device_buffers(ddrl_ctx* ctx, int pid, void** records, void** last_v, void** params,
                        void** adv_norm);

#ifdef __cplusplus
}
#endif
#endif
