// Host-side launch wrappers shared between the kernel translation units and the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DDRL_MAXP 4       // policies per context
#define DDRL_MAXAG 4      // agents per env
#define DDRL_MAXD 48      // per-agent observation width
#define DDRL_MAXFULL 48   // full observation width (43 / 44)
#ifndef DDRL_MB
#define DDRL_MB 128       // sgd_minibatch_size supported by the update kernels
#endif

// Record (one training row) layout, in floats.  Rows are time-major:
//   row = t * C + c,  c = env * k + slot  (k agents of this policy per env).
struct RecLayout {
  int stride;      // floats per row (multiple of 4)
  int obs, act, logit, logp, vf, adv, vt, rew;
  int cid;         // leg index of the row ("cup" model), -1 when the model has no coupling
};

// Per-policy routing tables for the observe / act / reward kernels.
struct PolicyRoute {
  int k;                    // agents of this policy per env
  int d;                    // obs width per row (GNN: 19 features per node)
  int agent[DDRL_MAXAG];    // agent id of each slot
  int obs_index[DDRL_MAXAG][DDRL_MAXD];
  int act_index[DDRL_MAXAG][8];
  int act_neg[DDRL_MAXAG];         // bit j: negate action j in the env vector (LegTransforms)
};

struct RouteArgs {
  int P, N, A, full_dim, n_agents, model;   // model: 0 ffn, 1 gnn
  int e0;                                   // env range [e0, e0 + N) of a ranged observe (host env plane)
  PolicyRoute pol[DDRL_MAXP];
  float leg_angle[4];
};

// ---- filter / observe (rollout.hip) ----
// dn / dM / dS: a second running stat of the pushes since the last cross-rank filter sync
// part: filter_part_doubles(N, D) doubles of per-chunk (mean, M2) scratch
void launch_filter_push(hipStream_t s, const float* obs, int N, int D, double* n_run, double* M,
                        double* S, double* normc, int update, int enabled, double* dn, double* dM,
                        double* dS, double* part);
size_t filter_part_doubles(int N, int D);
// the batch count of the env-side filter push, added by the observe kernel
struct FilterCount { double* n_run; double* dn; int count; };
// pf: per-policy RLlib MeanStdFilter state (PF_* layout, nullptr when disabled)
void launch_observe_ffn(hipStream_t s, const RouteArgs& ra, const float* obs, const double* normc,
                        float clip, float* const* stage, const double* pf, const FilterCount& fc);
// per-policy filter: statistics of the env-normalized observation columns, then the
// RunningStat update + normalization constants of every policy column
#define PF_N 0
#define PF_M 1
#define PF_S (PF_M + DDRL_MAXD)
#define PF_DN (PF_S + DDRL_MAXD)
#define PF_DM (PF_DN + 1)
#define PF_DS (PF_DM + DDRL_MAXD)
#define PF_NORMC (PF_DS + DDRL_MAXD)
#define PF_STRIDE (PF_NORMC + 2 * DDRL_MAXD)
void launch_policy_filter(hipStream_t s, const RouteArgs& ra, const float* obs, const double* normc, float clip,
                          double* zs, double* pf, int update);
void launch_observe_gnn(hipStream_t s, const RouteArgs& ra, const float* obs, const double* normc,
                        float clip, float* stage_x /*[N][4][23]*/, const FilterCount& fc);

// ---- act (rollout forward + sample) ----
struct ActArgs {
  const float* theta[DDRL_MAXP];
  const float* stage[DDRL_MAXP];   // [C][d] (ffn) or [N][4][23] (gnn)
  float* rec[DDRL_MAXP];           // base of the record buffer of this policy
  const float* cup[DDRL_MAXP];     // "cup" leg-coupling table [4][A] (nullptr: none)
  float* last_v[DDRL_MAXP];
  RecLayout lay[DDRL_MAXP];
  int C[DDRL_MAXP];
  int t;                           // time index (record row block)
  const float* eps;                // [N][n_agents][A]
  float* actions;                  // [N][8]
  int bootstrap;                   // 1: only value -> last_v
  int e0, e1;                      // env range of this call ([0, N) for a whole step)
};
void launch_act_ffn(hipStream_t s, const RouteArgs& ra, const ActArgs& aa);
void launch_act_gnn(hipStream_t s, const RouteArgs& ra, const ActArgs& aa, int layer);

// ---- reward (a8) ----
struct RewardArgs {
  int P, N, n_agents, mode;         // mode: 0 per-leg, 1 global, 2 norm_reward
  float ctrl_w, contact_w;
  int policy_of_agent[DDRL_MAXAG];
  int slot_of_agent[DDRL_MAXAG];
  int k[DDRL_MAXP];
  int act_index[DDRL_MAXAG][8];
  int n_act[DDRL_MAXAG];
  int n_contact[DDRL_MAXAG];
  int contact_index[DDRL_MAXAG][14];
  float contact_weight[DDRL_MAXAG][14];
  float* rec[DDRL_MAXP];
  RecLayout lay[DDRL_MAXP];
  int t;
  int e0, n;                        // env range [e0, e0 + n) of this call (N: all envs)
};
void launch_reward(hipStream_t s, const RewardArgs& ra, const float* fw, const float* cfrc,
                   const float* actions, const uint8_t* done, uint8_t* done_tn);

// ---- GAE + standardization statistics ----
struct GaeArgs {
  float* rec; RecLayout lay; int C, T, N, k;
  const float* last_v; const uint8_t* done_tn;
  double gamma, lambda_;
  // totals {sum adv, sum adv^2, count} at [2 * ceil(C / 256)], per-wave partial sums
  // [ceil(C / 64)][2] from gae_wave_base(C); gae_partials_len(C) doubles in all
  double* partials;
  float* adv_norm;    // [2]: mean, max(1e-4, std)
};
__host__ __device__ inline int gae_wave_base(int C) { return 2 * ((C + 255) / 256) + 4; }
__host__ __device__ inline int gae_partials_len(int C) { return gae_wave_base(C) + 2 * ((C + 63) / 64); }
struct GaeBatch { GaeArgs g[DDRL_MAXP]; int P; };
void launch_gae(hipStream_t s, const GaeBatch& gb);   // every policy of the context, one launch

// ---- PPO update (fused persistent minibatch loop) ----
struct UpdateArgs {
  const float* rec; RecLayout lay;
  int d, A, R;                 // obs width, action dim, rows of this policy
  const int32_t* shuffle;      // [R]; null: the minibatch rows are rec[0 .. rows) (pre-gathered)
  const int32_t* perm;         // [E][nb]
  int nb, n_epochs, max_steps, step0;
  float* theta; float* m; float* v; float* beta_pow;   // beta_pow[2]
  float* stats;                // [steps][8]
  const float* adv_norm;       // [2]
  float* grad_out;             // optional: write raw (unclipped) grads and stop (DDP)
  float* gscr;                 // [n_params] gradient scratch (L2 resident)
  float kl_coeff;
  int cup;                     // "cup" model: the leg-coupling table follows the fcnet variables
};
struct UpdateHyper {
  float clip, vf_clip, vf_coeff, ent_coeff, lr, grad_clip, b1, b2, eps;
  int vf_mode;
  int P;
};
// ua: host array of h.P UpdateArgs (one persistent workgroup pair per entry), passed to the
//     kernel by value in its argument block (no device copy, nothing outlives the call)
// ksp: 1 = one workgroup per branch, 2 = row split over two (gx: gx_bytes(P) of exchange granules)
// d / stride: the widest obs width / record stride of the launched policies
// own_kq: -1 = both row halves in this launch; 0 / 1 = peer mode (that half only; gx shared with
// the peer context, whose launch runs the other half; launch_update_ffn_peer)
// lx_base: peer mode's global step count before this launch (0 otherwise)
void launch_update_ffn(hipStream_t s, const UpdateArgs* ua, const UpdateHyper& h, int nrows, float inv_n, int A, int d,
                       int stride, int cup, unsigned long long* xchg, unsigned long long* gx, int ksp, int* err,
                       unsigned* epoch_ctr, int* xcc, int own_kq = -1, unsigned lx_base = 0);
// the same with the relaxed system-scope atomic exchange (ppo_ffn_atomic.hip): any placement
void launch_update_ffn_atomic(hipStream_t s, const UpdateArgs* ua, const UpdateHyper& h, int nrows, float inv_n, int A,
                              int d, int stride, int cup, unsigned long long* xchg, unsigned long long* gx, int ksp,
                              int* err, unsigned* epoch_ctr, int* xcc, int own_kq = -1, unsigned lx_base = 0);
// the launches of launch_update_ffn other than the fused row split: KSP = 1 and gradient export (ppo_ffn_k1.hip)
void launch_update_ffn_k1(hipStream_t s, const UpdateArgs* ua, const UpdateHyper& h, int nrows, float inv_n, int A,
                          int d, int stride, int cup, unsigned long long* xchg, unsigned long long* gx, int ksp,
                          int* err, unsigned* epoch_ctr, int* xcc, int own_kq = -1, unsigned lx_base = 0);
// peer mode (ppo_ffn_peer.hip): the LSB-tagged quads at system scope, outboxes shared with the
// peer context's launch (fine-grained memory a peer GPU reads)
void launch_update_ffn_peer(hipStream_t s, const UpdateArgs* ua, const UpdateHyper& h, int nrows, float inv_n, int A,
                            int d, int stride, int cup, unsigned long long* xchg, unsigned long long* gx, int ksp,
                            int* err, unsigned* epoch_ctr, int* xcc, int own_kq = -1, unsigned lx_base = 0);
// epoch_ctr: per-context launch counter (granule tags)
size_t gx_bytes(int P);
// clip_by_global_norm + tf1 Adam on a flat (all-reduced) gradient vector
// gscale multiplies the gradient before the clip (1 / ranks in the "local" data-parallel mode)
// err: the context's error word -- a set word (a failed gradient launch) skips the update
void launch_apply_adam(hipStream_t s, const float* grad, int n, float* theta, float* m, float* v,
                       float* beta_pow, const UpdateHyper& h, float gscale, int xcd, const int* err);
// Bounds-checked diagnostic build (-DDDRL_BOUNDS): violation counters of the update kernel's
// staging / record / schedule / LDS indices (see ppo_ffn.hip); ddrl_diag_bounds reads them.
#define DDRL_NBOUNDS 6

// ---- ModelV2.forward / value_function on arbitrary rows ----
struct ForwardArgs {
  const float* theta; const float* x; const int32_t* node; int n, d, A;
  const float* cup;             // ffn: leg-coupling table [4][A] ("cup" model) or nullptr
  float* logits; float* values;
};
void launch_forward_ffn(hipStream_t s, const ForwardArgs& fa);
void launch_forward_gnn(hipStream_t s, const ForwardArgs& fa, int layer);

// ---- GraphNet (gnn.hip): per-tile kernels, one minibatch step = grad / reduce / Adam ----
struct GnnArgs {
  const float* theta;
  int n_graphs;                 // envs (act), rows (forward) or minibatch rows (grad)
  const float* x;               // act: stage [N][4][23]; forward: [n][4][23]
  const int32_t* node;          // forward: node of every row
  // act
  float* rec; RecLayout lay; int t; const float* eps; float* actions; int n_agents;
  int act_index[4][8]; int bootstrap; float* last_v;
  // forward
  float* logits; float* values;
  // grad
  UpdateArgs u; UpdateHyper h; int step; float inv_n;
  float* part; int part_stride;  // [tiles][n_params] partial gradients
  float* statp;                  // [2 nets][32 tiles][8]
  float* normp;                  // [reduce blocks] squared-norm partials
  float* bp_cur;                 // [2] beta powers of the current step
  float* grad;                   // reduced gradient (scratch or the DDP output)
  int act_e0, act_nfull;          // act: first env of the range, envs of the shard (record rows)
  // staged minibatch (fused update only): the records of this step, contiguous [128][stride]
  // (a slot of the pre-gathered chunk); null: gather through shuffle / perm
  const float* stage;
  // one-launch step (gnn.hip gnn_tail): arrival flags [256], norm^2 granules [256], this launch's
  // tag; the XCD-grouped 1-D grid (xgrid); the parameters of each (net, share) combination
  // (plist[poff[k] .. poff[k + 1]), k = 4 net + share) and the first reducer index of each (rbase)
  unsigned* flags; unsigned long long* gran; unsigned tag; int tail; int nred; int n_params; int ntiles; int* err;
  // xgrid: 1 = the XCD-grouped grid, 2 = test hook remapping each combination across every XCD;
  // xcc: [8 combinations][32 tiles] XCC id of the workgroup that ran each tile (placement record)
  int xgrid; int only_share; const int* plist; int poff[9]; int rbase[9]; int* xcc;
};
struct GnnScratch {
  float* part; int part_stride; float* statp; float* normp; float* bp_cur; float* grad;
  float* chunk;       // [chunk_steps][128][stride] records of a run of minibatch steps
  int chunk_steps;    // min(GNN_CHUNK_STEPS, the schedule's steps); chunk allocated on first use
  unsigned* flags;              // [256] arrival flags of the one-launch step (device)
  unsigned long long* gran;     // [256] tagged norm^2 partials {value, tag} of its reduction blocks
  unsigned seq;                 // tag of the last one-launch step (host; never 0)
  int* plist;                   // [n_params] parameters by (net, share) owner (device)
  int poff[9], rbase[9];        // list offsets / first reducer of each combination
  int lists;                    // 0: not built yet, 1: built, -1: unusable (three launches)
  int tail;           // 1: reduction + clip + Adam in the gradient launch (DDRL_GNN_TAIL, default 1)
  int* err;           // the context's error word
  int* xcc;           // [256] XCC id per (combination, tile) of the last one-launch step (device)
  int xcc_pending;    // a one-launch step ran since the host last checked its placement
  int misplace;       // test hook (DDRL_TEST_GNN_MISPLACE): every combination straddles the XCDs
};
#define GNN_CHUNK_STEPS 1024
int gnn_param_total(int A, int layer);   // layer: DDRL_GNN_*
// stage: the step's pre-gathered records (fused update) or null (data-parallel gradient of
// explicit rows)
void launch_step_gnn(hipStream_t s, const UpdateArgs& u, const UpdateHyper& h, int step, int nrows, float inv_n,
                     GnnScratch& sc, const float* stage, int layer);
// the records of minibatch steps [step0, step0 + n_steps) of the schedule -> dst
// ([n_steps][128][stride], n_steps <= GNN_CHUNK_STEPS): one bandwidth-bound gather per chunk
void launch_gnn_gather(hipStream_t s, const UpdateArgs& u, int step0, int n_steps, float* dst);
// data-parallel steps: step k's m minibatch rows gathered into dst[k][m][stride] (ppo_ffn.hip)
void launch_rows_gather(hipStream_t s, const float* rec, int stride, const int32_t* shuffle, const int32_t* perm,
                        int m, int step0, int n_steps, float* dst);
