// C-ABI of libddrl_hip.so (declared in include/ddrl_hip.h).
// Owns every device buffer of a training shard; all work is enqueued on one HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/ddrl_hip.h"
#include "hostenv.h"
#include "kernels.h"

namespace {
thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess)                                                           \
      return fail(std::string(#x) + ": " + hipGetErrorString(e_));                  \
  } while (0)

#define NCCLCHK(x)                                                                  \
  do {                                                                              \
    ncclResult_t r_ = (x);                                                          \
    if (r_ != ncclSuccess) return fail(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

#define CHK_CTX(c) \
  if (!(c)) return fail("null context")

int ffn_param_count(int d, int A) { return d * 64 * 2 + 128 + 2 * 4096 + 128 + 64 * 2 * A + 2 * A + 65; }
int gnn_param_count(int A, int layer) { return gnn_param_total(A, layer); }

struct Policy {
  int k = 0, d = 0, C = 0, n_params = 0, R = 0, nb = 0;
  int agents[DDRL_MAXAG] = {0};
  RecLayout lay{};
  float *theta = nullptr, *m = nullptr, *v = nullptr, *beta_pow = nullptr;
  float *rec = nullptr, *stage = nullptr, *last_v = nullptr, *adv_norm = nullptr;
  float *stats = nullptr, *grad = nullptr;
  double* partials = nullptr;
  int last_steps = 0;
  size_t stats_steps = 0;   // rows of `stats` (num_sgd_iter * nb; peer mode may grow it)
};
}  // namespace

struct ddrl_ctx {
  ddrl_cfg cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  Policy pol[DDRL_MAXP];
  RouteArgs route{};
  double *f_n = nullptr, *f_M = nullptr, *f_S = nullptr, *f_normc = nullptr;
  double *f_dn = nullptr, *f_dM = nullptr, *f_dS = nullptr;   // pushes since the last sync
  double* f_part = nullptr;                                     // filter push chunk scratch
  double* pf = nullptr;   // per-policy RLlib MeanStdFilter state [P][PF_STRIDE]
  double* zs = nullptr;   // fp64 column sums of the env-normalized observation [2][D]
  uint8_t* done_tn = nullptr;
  float** stage_tab = nullptr;    // device array of per-policy stage pointers
  int32_t* zero_perm = nullptr;
  unsigned long long* xchg = nullptr;  // norm^2 exchange granules of the update kernel
  unsigned long long* gx = nullptr;    // partial-gradient granules of the row-split update
  unsigned upd_epoch = 0;              // update launches so far (granule tag epochs)
  int update_split = 2;                // workgroups per branch of the fused update (1 or 2)
  int* err = nullptr;                  // device error word (exchange timeout)
  // Placement / rollback (fcnet update): the XCC of every block of the last update launch,
  // the exchange protocol (0: plain stores into the XCD's L2, 1: relaxed agent-scope atomics,
  // chosen by DDRL_XCHG=atomic or after a placement failure), and per policy a snapshot of
  // theta | m | v | beta powers taken before each update, restored when the launch fails.
  int* xcc = nullptr;
  int xchg_atomic = 0;
  int xcc_pending = 0;                 // blocks of an update launch not yet checked (grid size)
  int xcc_ksp = 2;
  int xcc_mask = 0;
  int fail_step = -1;                  // test hook: DDRL_TEST_FAIL_STEP
  float* snap[DDRL_MAXP] = {nullptr};
  int snap_mask = 0;
  float kl_last[DDRL_MAXP] = {0};
  GnnScratch gnn{};               // GraphNet step scratch (per-tile partial gradients, ...)
  // host-variant staging
  float *h_obs = nullptr, *h_eps = nullptr, *h_act = nullptr;
  ncclComm_t comm = nullptr;           // data-parallel learner (ddrl_comm_init)
  float* ddp_chunk = nullptr;          // ddrl_ppo_update_ddp: pre-gathered records of a run of steps
  size_t ddp_chunk_n = 0;
  int32_t* ddp_slots = nullptr;        // ... and the minibatch slot of every step (device copy)
  size_t ddp_slots_n = 0;
  std::vector<int32_t> ddp_slots_host; // source of that copy, alive until the call's final sync
  float *h_fw = nullptr, *h_cfrc = nullptr;
  uint8_t* h_done = nullptr;
  // ddrl_rollout_fragment as one HIP graph (T x (act, reward, filter push, observe) +
  // bootstrap), captured on first use and re-used while the call's buffers are the same
  // (every other kernel argument is fixed at context creation); DDRL_ROLLOUT_GRAPH=0: launches
  int rollout_graph = 1;
  hipGraphExec_t rg_exec = nullptr;
  hipStream_t cap_stream = nullptr;    // capture only (the caller's stream may be the null stream)
  const void* rg_key[6] = {nullptr};
  // peer mode (ddrl_ppo_update_peer): the outboxes shared with the peer context, this context's
  // row half, the launch tags both contexts step in lockstep, the IPC mapping to close, and the
  // per-rank virtual shuffle ([nb][128] row indices, this rank's rows in half peer_rank)
  void* peer_gx = nullptr;
  int peer_rank = -1;
  unsigned peer_epoch = 0;
  unsigned peer_steps = 0;   // steps the attached pair has run (the quads' tag bit and outbox parity)
  int peer_inflight = 0;     // a peer launch is enqueued and not yet checked (check_err)
  void* peer_ipc = nullptr;
  int32_t* peer_vsh = nullptr;
  size_t peer_vsh_n = 0;
  std::vector<void*> allocs;
};

template <class T>
static int dalloc(ddrl_ctx* c, T** p, size_t count) {
  void* ptr = nullptr;
  const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  hipError_t e = hipMalloc(&ptr, bytes);
  if (e != hipSuccess) return fail(std::string("hipMalloc failed: ") + hipGetErrorString(e));
  e = hipMemset(ptr, 0, bytes);
  if (e != hipSuccess) return fail(std::string("hipMemset failed: ") + hipGetErrorString(e));
  c->allocs.push_back(ptr);
  *p = static_cast<T*>(ptr);
  return 0;
}

// a buffer that is replaced by a larger one (the data-parallel loop's chunk and slots): the
// callers run after a stream synchronize, so nothing in flight still reads it
template <class T>
static void dfree(ddrl_ctx* c, T** p) {
  if (!*p) return;
  auto it = std::find(c->allocs.begin(), c->allocs.end(), static_cast<void*>(*p));
  if (it != c->allocs.end()) c->allocs.erase(it);
  (void)hipFree(*p);
  *p = nullptr;
}

static RecLayout make_layout(const ddrl_cfg& cfg, int d) {
  RecLayout L;
  const int A = cfg.act_dim;
  L.obs = 0;
  const int obs_len = cfg.model_kind == DDRL_MODEL_GNN ? 4 * 23 + 1 : d;
  L.act = obs_len;
  L.logit = L.act + A;
  L.logp = L.logit + 2 * A;
  L.vf = L.logp + 1;
  L.adv = L.vf + 1;
  L.vt = L.adv + 1;
  L.rew = L.vt + 1;
  L.cid = cfg.leg_coupling ? L.rew + 1 : -1;   // "cup": the row's leg index (coupling row)
  L.stride = ((cfg.leg_coupling ? L.cid : L.rew) + 1 + 3) & ~3;
  return L;
}

static int validate(const ddrl_cfg& c) {
  if (c.n_envs <= 0 || c.frag_len <= 0) return fail("n_envs and frag_len must be positive");
  if (c.n_policies < 1 || c.n_policies > DDRL_MAXP) return fail("n_policies must be in [1, 4]");
  if (c.n_agents < 1 || c.n_agents > DDRL_MAXAG) return fail("n_agents must be in [1, 4]");
  if (c.act_dim != 2 && c.act_dim != 4 && c.act_dim != 8) return fail("act_dim must be 2, 4 or 8");
  if (c.obs_full_dim < 1 || c.obs_full_dim > DDRL_MAXFULL) return fail("obs_full_dim out of range");
  if (c.sgd_minibatch_size != 128) return fail("sgd_minibatch_size must be 128 (fused kernel tile)");
  if (c.num_sgd_iter < 1) return fail("num_sgd_iter must be >= 1");
  for (int j = 0; j < c.n_agents; ++j)
    if (c.agent_policy[j] < 0 || c.agent_policy[j] >= c.n_policies) return fail("bad agent_policy");
  for (int p = 0; p < c.n_policies; ++p) {
    const int d = c.obs_dim[p];
    if (d < 1 || d > DDRL_MAX_OBS) return fail("obs_dim out of range");
    if (c.model_kind == DDRL_MODEL_FFN && d > 48) return fail("ffn obs_dim must be <= 48");
  }
  if (c.model_kind == DDRL_MODEL_GNN && (c.n_policies != 1 || c.n_agents != 4 || c.obs_dim[0] != 19))
    return fail("gnn requires one shared leg policy, 4 agents and 19 features per node");
  if (c.model_kind == DDRL_MODEL_GNN && c.act_dim != 2) return fail("gnn kernels are built for act_dim 2");
  if (c.gnn_layer < DDRL_GNN_MPNN || c.gnn_layer > DDRL_GNN_GAT1) return fail("gnn_layer must be one of DDRL_GNN_*");
  if (c.leg_coupling && (c.model_kind != DDRL_MODEL_FFN || c.act_dim != 2 || c.n_policies != 1 || c.n_agents != 4 ||
                          c.obs_dim[0] > 20))
    return fail("leg_coupling (\"cup\") requires the fcnet model, one shared leg policy, 4 agents, act_dim 2 and obs_dim <= 20");
  if (c.policy_filter && c.model_kind != DDRL_MODEL_FFN)
    return fail("the per-policy MeanStdFilter is built for fcnet policies (flat observations)");
  for (int j = 0; j < c.n_agents; ++j) {
    const int d = c.obs_dim[c.agent_policy[j]];
    for (int f = 0; f < d; ++f)
      if (c.obs_index[j][f] < -2 || c.obs_index[j][f] >= c.obs_full_dim ||
          (c.model_kind == DDRL_MODEL_GNN && c.obs_index[j][f] < 0))
        return fail("bad obs_index");
      else if (c.policy_filter && c.obs_index[j][f] < 0)
        return fail("constant input columns (LegID) with the per-policy MeanStdFilter are not supported");
    if (c.n_contact[j] < 0 || c.n_contact[j] > 14) return fail("bad n_contact");
    for (int b = 0; b < c.n_contact[j]; ++b)
      if (c.contact_index[j][b] < 0 || c.contact_index[j][b] >= 14) return fail("bad contact_index");
    for (int a = 0; a < c.act_dim; ++a)
      if (c.act_index[j][a] < 0 || c.act_index[j][a] >= 8) return fail("bad act_index");
  }
  return 0;
}

extern "C" {

int ddrl_abi_version(void) { return DDRL_ABI_VERSION; }
const char* ddrl_last_error(void) { return g_err.c_str(); }

int ddrl_ctx_create(const ddrl_cfg* cfg, int device, ddrl_ctx** out) {
  if (!cfg || !out) return fail("null argument");
  if (validate(*cfg)) return -1;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("device index out of range");
  HIPCHK(hipSetDevice(device));
  ddrl_ctx* c = new ddrl_ctx();
  // fused update geometry: DDRL_UPDATE_SPLIT=1 keeps one workgroup per branch (timing / A-B)
  if (const char* e = std::getenv("DDRL_UPDATE_SPLIT")) c->update_split = std::atoi(e) == 1 ? 1 : 2;
  c->cfg = *cfg;
  c->device = device;
  const ddrl_cfg& g = c->cfg;
  const int N = g.n_envs, T = g.frag_len;
  RouteArgs& ra = c->route;
  ra.P = g.n_policies; ra.N = N; ra.A = g.act_dim; ra.full_dim = g.obs_full_dim;
  ra.n_agents = g.n_agents; ra.model = g.model_kind;
  for (int j = 0; j < 4; ++j) ra.leg_angle[j] = g.leg_angle_deg[j];
  int rc = 0;
  for (int p = 0; p < g.n_policies && !rc; ++p) {
    Policy& P = c->pol[p];
    P.d = g.obs_dim[p];
    for (int j = 0; j < g.n_agents; ++j)
      if (g.agent_policy[j] == p) P.agents[P.k++] = j;
    if (P.k == 0) { rc = fail("policy without agents"); break; }
    P.C = N * P.k;
    P.R = T * P.C;
    P.nb = std::max(1, P.R / g.sgd_minibatch_size);
    P.lay = make_layout(g, P.d);
    P.n_params = g.model_kind == DDRL_MODEL_FFN ? ffn_param_count(P.d, g.act_dim) : gnn_param_count(g.act_dim, g.gnn_layer);
    if (g.leg_coupling) P.n_params += 4 * g.act_dim;   // leg_coupling [4][A] after the fcnet variables
    PolicyRoute& pr = ra.pol[p];
    pr.k = P.k; pr.d = P.d;
    for (int s = 0; s < P.k; ++s) {
      pr.agent[s] = P.agents[s];
      for (int f = 0; f < DDRL_MAXD; ++f) pr.obs_index[s][f] = g.obs_index[P.agents[s]][f];
      pr.act_neg[s] = 0;
      for (int a = 0; a < 8; ++a) {
        pr.act_index[s][a] = g.act_index[P.agents[s]][a];
        if (g.act_negate[P.agents[s]][a]) pr.act_neg[s] |= 1 << a;
      }
    }
    const size_t stage_n = g.model_kind == DDRL_MODEL_GNN ? (size_t)N * 4 * 23 : (size_t)P.C * P.d;
    rc = rc || dalloc(c, &P.theta, P.n_params) || dalloc(c, &P.m, P.n_params) ||
         dalloc(c, &P.v, P.n_params) || dalloc(c, &P.beta_pow, 4) || dalloc(c, &P.grad, P.n_params) ||
         dalloc(c, &P.rec, (size_t)P.R * P.lay.stride) || dalloc(c, &P.stage, stage_n) ||
         dalloc(c, &P.last_v, P.C) || dalloc(c, &P.adv_norm, 2) ||
         dalloc(c, &P.partials, (size_t)gae_partials_len(P.C)) ||
         dalloc(c, &P.stats, (size_t)g.num_sgd_iter * P.nb * 8);
    P.stats_steps = (size_t)g.num_sgd_iter * P.nb;
    if (!rc) {
      // beta1^t, beta2^t, then the arrival counter of the multi-workgroup apply kernel (0)
      float bp[4] = {g.adam_beta1, g.adam_beta2, 0.f, 0.f};
      if (hipMemcpy(P.beta_pow, bp, sizeof(bp), hipMemcpyHostToDevice) != hipSuccess) rc = fail("init beta_pow");
      float an[2] = {0.f, 1.f};
      if (hipMemcpy(P.adv_norm, an, sizeof(an), hipMemcpyHostToDevice) != hipSuccess) rc = fail("init adv_norm");
    }
  }
  rc = rc || dalloc(c, &c->f_n, 1) || dalloc(c, &c->f_M, DDRL_MAXFULL) || dalloc(c, &c->f_S, DDRL_MAXFULL) ||
       dalloc(c, &c->f_normc, 2 * DDRL_MAXFULL) || dalloc(c, &c->f_dn, 1) ||
       dalloc(c, &c->f_dM, DDRL_MAXFULL) || dalloc(c, &c->f_dS, DDRL_MAXFULL) ||
       dalloc(c, &c->f_part, filter_part_doubles(N, DDRL_MAXFULL)) ||
       dalloc(c, &c->pf, (size_t)DDRL_MAXP * PF_STRIDE) || dalloc(c, &c->zs, 2 * DDRL_MAXFULL) || dalloc(c, &c->done_tn, (size_t)T * N) ||
       dalloc(c, &c->stage_tab, DDRL_MAXP) || dalloc(c, &c->zero_perm, 4) ||
       dalloc(c, &c->xchg, 8 * DDRL_MAXP) ||
       dalloc(c, &c->gx, gx_bytes(DDRL_MAXP) / sizeof(unsigned long long)) || dalloc(c, &c->err, 1) ||
       dalloc(c, &c->xcc, 32) ||
       dalloc(c, &c->h_obs, (size_t)N * g.obs_full_dim) ||
       dalloc(c, &c->h_eps, (size_t)N * g.n_agents * g.act_dim) || dalloc(c, &c->h_act, (size_t)N * 8) ||
       dalloc(c, &c->h_fw, N) || dalloc(c, &c->h_cfrc, (size_t)N * 14 * 6) || dalloc(c, &c->h_done, N);
  for (int p = 0; p < g.n_policies && !rc; ++p)
    rc = dalloc(c, &c->snap[p], 3 * (size_t)c->pol[p].n_params + 4);
  if (const char* e = std::getenv("DDRL_XCHG")) c->xchg_atomic = std::string(e) == "atomic" ? 1 : 0;
  if (const char* e = std::getenv("DDRL_TEST_FAIL_STEP")) c->fail_step = std::atoi(e);
  if (const char* e = std::getenv("DDRL_ROLLOUT_GRAPH")) c->rollout_graph = std::atoi(e) != 0;
  if (!rc && g.model_kind == DDRL_MODEL_GNN) {
    const int np = c->pol[0].n_params;
    c->gnn.part_stride = (np + 3) & ~3;   // 16-byte aligned tile rows (float4 partial stores)
    c->gnn.grad = c->pol[0].grad;
    rc = dalloc(c, &c->gnn.part, (size_t)(DDRL_MB / 4) * c->gnn.part_stride) || dalloc(c, &c->gnn.statp, 2 * (DDRL_MB / 4) * 8) ||
         dalloc(c, &c->gnn.normp, (np + 255) / 256) || dalloc(c, &c->gnn.bp_cur, 2) || dalloc(c, &c->gnn.flags, 256) ||
         dalloc(c, &c->gnn.gran, 256) || dalloc(c, &c->gnn.plist, np) || dalloc(c, &c->gnn.xcc, 256);
    c->gnn.seq = 0;
    c->gnn.lists = 0;
    c->gnn.err = c->err;
    c->gnn.tail = 1;
    c->gnn.xcc_pending = 0;
    c->gnn.misplace = 0;
    if (const char* e = std::getenv("DDRL_GNN_TAIL")) c->gnn.tail = std::atoi(e) != 0;
    if (const char* e = std::getenv("DDRL_TEST_GNN_MISPLACE")) c->gnn.misplace = std::atoi(e) != 0;
    // the record chunk of the fused update is allocated by the first ddrl_ppo_update (forward-only
    // and data-parallel contexts never need it), sized to the schedule when that is shorter
    c->gnn.chunk = nullptr;
    c->gnn.chunk_steps = std::min(GNN_CHUNK_STEPS, g.num_sgd_iter * c->pol[0].nb);
  }
  if (!rc) {
    float* tab[DDRL_MAXP] = {nullptr};
    for (int p = 0; p < g.n_policies; ++p) tab[p] = c->pol[p].stage;
    if (hipMemcpy(c->stage_tab, tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess) rc = fail("stage table");
  }
  if (!rc && hipDeviceSynchronize() != hipSuccess) rc = fail("device sync after init");
  if (rc) {
    ddrl_ctx_destroy(c);
    return -1;
  }
  *out = c;
  return 0;
}

int ddrl_ctx_destroy(ddrl_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->peer_ipc) (void)hipIpcCloseMemHandle(c->peer_ipc);
  if (c->rg_exec) (void)hipGraphExecDestroy(c->rg_exec);
  if (c->cap_stream) (void)hipStreamDestroy(c->cap_stream);
  for (void* p : c->allocs) (void)hipFree(p);
  delete c;
  return 0;
}

int ddrl_set_stream(ddrl_ctx* c, void* s) {
  CHK_CTX(c);
  c->stream = static_cast<hipStream_t>(s);
  return 0;
}

// Snapshot of the policies an fcnet update launch is about to change (stream-ordered D2D copies:
// theta | m | v | beta powers), restored by check_err when the launch fails.
static int snapshot(ddrl_ctx* c, int mask) {
  for (int p = 0; p < c->cfg.n_policies; ++p) {
    if (!(mask & (1 << p)) || !c->snap[p]) continue;
    Policy& P = c->pol[p];
    const size_t n = (size_t)P.n_params;
    HIPCHK(hipMemcpyAsync(c->snap[p], P.theta, n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->snap[p] + n, P.m, n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->snap[p] + 2 * n, P.v, n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->snap[p] + 3 * n, P.beta_pow, 4 * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  c->snap_mask = mask;
  return 0;
}

static int restore_snapshot(ddrl_ctx* c) {
  for (int p = 0; p < c->cfg.n_policies; ++p) {
    if (!(c->snap_mask & (1 << p)) || !c->snap[p]) continue;
    Policy& P = c->pol[p];
    const size_t n = (size_t)P.n_params;
    HIPCHK(hipMemcpyAsync(P.theta, c->snap[p], n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(P.m, c->snap[p] + n, n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(P.v, c->snap[p] + 2 * n, n * 4, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(P.beta_pow, c->snap[p] + 3 * n, 4 * 4, hipMemcpyDeviceToDevice, c->stream));
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

// The default exchange protocol needs the workgroups of one policy (blocks p, p + 8, ... of the
// launch) on one XCD.  Returns 1 if the last launch's recorded XCC ids (HW_REG_XCC_ID) break that.
static int placement_broken(ddrl_ctx* c) {
  if (!c->xcc_pending) return 0;
  int x[32] = {0};
  if (hipMemcpy(x, c->xcc, sizeof(x), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  const int per = 2 * c->xcc_ksp;   // workgroups per policy
  int bad = 0;
  for (int p = 0; p < 8; ++p) {
    if (!(c->xcc_mask & (1 << p))) continue;
    for (int j = 1; j < per && p + 8 * j < c->xcc_pending; ++j) bad |= x[p + 8 * j] != x[p];
  }
  c->xcc_pending = 0;
  return bad;
}

// The one-launch GNN step needs the 32 tiles of each (net, backward share) combination on one
// XCD (gnn.hip gnn_tail).  Returns 1 if the last such launch's per-tile XCC record breaks that.
static int gnn_placement_broken(ddrl_ctx* c) {
  if (c->cfg.model_kind != DDRL_MODEL_GNN || !c->gnn.xcc_pending) return 0;
  c->gnn.xcc_pending = 0;
  int x[256] = {0};
  if (hipMemcpy(x, c->gnn.xcc, sizeof(x), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  int bad = 0;
  for (int k = 0; k < 8; ++k)
    for (int t = 1; t < DDRL_MB / 4; ++t) bad |= x[32 * k + t] != x[32 * k];
  return bad;
}

// A failed peer launch may have left partly written outboxes on both ranks: the pair must
// re-attach (rank 0's attach clears them) before another peer update, or a retry's tag bit could
// admit the aborted launch's stale quads.  Detaching makes ddrl_ppo_update_peer
// refuse ("no peer") until ddrl_peer_attach runs again.
static void peer_detach(ddrl_ctx* c) {
  c->peer_gx = nullptr;
  c->peer_rank = -1;
  c->peer_inflight = 0;
}

static int check_err(ddrl_ctx* c) {
  int e = 0;
  HIPCHK(hipMemcpy(&e, c->err, sizeof(int), hipMemcpyDeviceToHost));
  const int was_peer = c->peer_inflight;
  c->peer_inflight = 0;
  if (e) {
    (void)hipMemset(c->err, 0, sizeof(int));
    const int bad = placement_broken(c);
    const int gbad = gnn_placement_broken(c);
    if (restore_snapshot(c)) return -1;
    c->snap_mask = 0;
    if (was_peer) {
      peer_detach(c);
      return fail("peer update: an exchange with the peer rank's launch was abandoned (3 s timeout or a failed "
                  "launch).  The weights, Adam state and beta powers are as before the call; this context is "
                  "detached from its peer: both ranks must call ddrl_peer_attach again before a peer update");
    }
    if (c->cfg.model_kind == DDRL_MODEL_GNN) {
      // a one-launch GNN step whose waits were abandoned or refused a flag from another XCD:
      // the context goes on with the three-launch step (no cross-workgroup waits)
      const int was_tail = c->gnn.tail && c->gnn.lists == 1;
      c->gnn.tail = 0;
      if (!was_tail)   // the three-launch step has no waits between workgroups
        return fail("GraphNet update: a launch reported an error (the error word was set).  The weights, Adam "
                    "state and beta powers are as before the call");
      return fail(std::string("GraphNet update: ") +
                  (gbad ? "the workgroups of a (net, backward share) combination ran on different XCDs (placement "
                          "check), so the one-launch step's reduction through the XCD's L2 was refused"
                        : "a wait between workgroups was abandoned (3 s timeout or a failed launch)") +
                  ".  The weights, Adam state and beta powers are as before the call; this context has switched "
                  "to the three-launch step: call the update again");
    }
    if (bad && !c->xchg_atomic) {
      c->xchg_atomic = 1;
      return fail("update kernel: the workgroups of a policy ran on different XCDs (placement check), so the "
                  "default exchange through the XCD's L2 could not complete.  The weights, Adam state and beta "
                  "powers are as before the call; this context has switched to the atomic exchange protocol "
                  "(valid for any placement): call the update again");
    }
    return fail("update kernel: an exchange between the workgroups of a policy was abandoned (3 s timeout or "
                "a failed launch).  The weights, Adam state and beta powers are as before the call");
  }
  // a broken placement whose exchanges still completed (a granule reached the other XCD through
  // memory) gave correct results -- the tags admit only this step's data -- but the next
  // launch might not be so lucky: switch protocols now
  if (placement_broken(c)) c->xchg_atomic = 1;
  // the GNN reducers accept flags only from their own XCD, so a step that completed had its
  // combinations in place; a record that says otherwise still ends the one-launch steps
  if (gnn_placement_broken(c)) c->gnn.tail = 0;
  c->snap_mask = 0;
  return 0;
}

// fcnet update launch with the context's exchange protocol
static void launch_ffn(ddrl_ctx* c, const UpdateArgs* ua, const UpdateHyper& h, int nrows, float inv_n, int d,
                       int stride, int ksp, int mask) {
  c->xcc_pending = ksp == 2 ? 24 + h.P : 8 + h.P;
  c->xcc_ksp = ksp;
  c->xcc_mask = mask;
  // test hook (DDRL_TEST_FAIL_STEP): a fused launch starts with the error word set, as an
  // exchange abandoned in its first step would leave it -- every workgroup runs its steps and
  // none writes back (no per-step cost in the kernel; a compare per step measured 0.18 us)
  if (c->fail_step >= 0 && !ua->grad_out) (void)hipMemsetD32Async((hipDeviceptr_t)c->err, 1, 1, c->stream);
  (c->xchg_atomic ? launch_update_ffn_atomic : launch_update_ffn)(
      c->stream, ua, h, nrows, inv_n, c->cfg.act_dim, d, stride, c->cfg.leg_coupling, c->xchg, c->gx, ksp, c->err,
      &c->upd_epoch, c->xcc, -1, 0u);
}

int ddrl_synchronize(ddrl_ctx* c) {
  CHK_CTX(c);
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipGetLastError());
  return check_err(c);
}

int ddrl_param_count(ddrl_ctx* c, int pid, int64_t* n) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies || !n) return fail("bad policy id");
  *n = c->pol[pid].n_params;
  return 0;
}

int ddrl_record_layout(ddrl_ctx* c, int pid, int32_t* o) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies || !o) return fail("bad policy id");
  const RecLayout& L = c->pol[pid].lay;
  o[0] = L.stride; o[1] = L.obs; o[2] = L.act; o[3] = L.logit; o[4] = L.logp;
  o[5] = L.vf; o[6] = L.adv; o[7] = L.vt; o[8] = L.rew; o[9] = c->pol[pid].C; o[10] = L.cid;
  return 0;
}

static int check_n(ddrl_ctx* c, int pid, size_t n) {
  if (!c) return fail("null context");
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (n != (size_t)c->pol[pid].n_params) return fail("parameter count mismatch");
  return 0;
}

int ddrl_params_set(ddrl_ctx* c, int pid, const float* h, size_t n) {
  if (check_n(c, pid, n)) return -1;
  HIPCHK(hipMemcpyAsync(c->pol[pid].theta, h, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_params_get(ddrl_ctx* c, int pid, float* h, size_t n) {
  if (check_n(c, pid, n)) return -1;
  HIPCHK(hipMemcpyAsync(h, c->pol[pid].theta, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_adam_set(ddrl_ctx* c, int pid, const float* m, const float* v, size_t n, float b1p, float b2p) {
  if (check_n(c, pid, n)) return -1;
  Policy& P = c->pol[pid];
  HIPCHK(hipMemcpyAsync(P.m, m, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(P.v, v, n * 4, hipMemcpyHostToDevice, c->stream));
  float bp[2] = {b1p, b2p};
  HIPCHK(hipMemcpyAsync(P.beta_pow, bp, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_adam_get(ddrl_ctx* c, int pid, float* m, float* v, size_t n, float* b1p, float* b2p) {
  if (check_n(c, pid, n)) return -1;
  Policy& P = c->pol[pid];
  float bp[2];
  HIPCHK(hipMemcpyAsync(m, P.m, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(v, P.v, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(bp, P.beta_pow, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (b1p) *b1p = bp[0];
  if (b2p) *b2p = bp[1];
  return 0;
}

int ddrl_filter_set(ddrl_ctx* c, double n, const double* M, const double* S) {
  CHK_CTX(c);
  const int D = c->cfg.obs_full_dim;
  HIPCHK(hipMemcpyAsync(c->f_n, &n, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->f_M, M, D * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->f_S, S, D * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_filter_get(ddrl_ctx* c, double* n, double* M, double* S) {
  CHK_CTX(c);
  const int D = c->cfg.obs_full_dim;
  HIPCHK(hipMemcpyAsync(n, c->f_n, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(M, c->f_M, D * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(S, c->f_S, D * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_filter_delta_get(ddrl_ctx* c, double* n, double* M, double* S) {
  CHK_CTX(c);
  const int D = c->cfg.obs_full_dim;
  HIPCHK(hipMemcpyAsync(n, c->f_dn, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(M, c->f_dM, D * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(S, c->f_dS, D * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_filter_delta_reset(ddrl_ctx* c) {
  CHK_CTX(c);
  HIPCHK(hipMemsetAsync(c->f_dn, 0, 8, c->stream));
  HIPCHK(hipMemsetAsync(c->f_dM, 0, DDRL_MAXFULL * 8, c->stream));
  HIPCHK(hipMemsetAsync(c->f_dS, 0, DDRL_MAXFULL * 8, c->stream));
  return 0;
}

static int pf_io(ddrl_ctx* c, int pid, double* n, double* M, double* S, bool set, bool delta) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (!n || !M || !S) return fail("null filter buffer");
  const int d = c->pol[pid].d;
  double* P = c->pf + (size_t)pid * PF_STRIDE;
  const int on = delta ? PF_DN : PF_N, om = delta ? PF_DM : PF_M, os = delta ? PF_DS : PF_S;
  const hipMemcpyKind k = set ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
  HIPCHK(hipMemcpyAsync(set ? (void*)(P + on) : (void*)n, set ? (const void*)n : (const void*)(P + on), 8, k, c->stream));
  HIPCHK(hipMemcpyAsync(set ? (void*)(P + om) : (void*)M, set ? (const void*)M : (const void*)(P + om), 8 * d, k, c->stream));
  HIPCHK(hipMemcpyAsync(set ? (void*)(P + os) : (void*)S, set ? (const void*)S : (const void*)(P + os), 8 * d, k, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (set) {   // normalization constants of the restored statistics
    launch_policy_filter(c->stream, c->route, nullptr, c->f_normc, 0.f, c->zs, c->pf, 0);
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  return 0;
}

int ddrl_policy_filter_set(ddrl_ctx* c, int pid, double n, const double* M, const double* S) {
  return pf_io(c, pid, &n, const_cast<double*>(M), const_cast<double*>(S), true, false);
}
int ddrl_policy_filter_get(ddrl_ctx* c, int pid, double* n, double* M, double* S) {
  return pf_io(c, pid, n, M, S, false, false);
}
int ddrl_policy_filter_delta_get(ddrl_ctx* c, int pid, double* n, double* M, double* S) {
  return pf_io(c, pid, n, M, S, false, true);
}
int ddrl_policy_filter_delta_reset(ddrl_ctx* c) {
  CHK_CTX(c);
  for (int p = 0; p < c->cfg.n_policies; ++p) {
    double* P = c->pf + (size_t)p * PF_STRIDE;
    HIPCHK(hipMemsetAsync(P + PF_DN, 0, 8 * (1 + 2 * DDRL_MAXD), c->stream));
  }
  return 0;
}

int ddrl_adv_sums_get(ddrl_ctx* c, int pid, double* host3) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  const Policy& P = c->pol[pid];
  const size_t nblocks = (P.C + 255) / 256;
  HIPCHK(hipMemcpyAsync(host3, P.partials + 2 * nblocks, 3 * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

static int check_range(const ddrl_ctx* c, int e0, int e1) {
  if (e0 < 0 || e1 > c->cfg.n_envs || e0 >= e1) return fail("env range [e0, e1) must lie in [0, n_envs) and be non-empty");
  return 0;
}

// observe / act / reward over the envs [e0, e1) (the whole shard, or one group of a
// pipelined host env plane): the env-side filter pushes the range's rows as one batch.
int ddrl_observe_range(ddrl_ctx* c, const float* obs, int e0, int e1) {
  CHK_CTX(c);
  if (!obs) return fail("null observation buffer");
  if (check_range(c, e0, e1)) return -1;
  const ddrl_cfg& g = c->cfg;
  const int n = e1 - e0;
  const float* obs_r = obs + (size_t)e0 * g.obs_full_dim;
  RouteArgs ra = c->route;
  ra.N = n;
  ra.e0 = e0;
  launch_filter_push(c->stream, obs_r, n, g.obs_full_dim, c->f_n, c->f_M, c->f_S, c->f_normc,
                     g.filter_update, g.filter_enabled, c->f_dn, c->f_dM, c->f_dS, c->f_part);
  const float clip = g.filter_enabled ? g.filter_clip : 0.f;
  if (g.policy_filter) launch_policy_filter(c->stream, ra, obs_r, c->f_normc, clip, c->zs, c->pf, 1);
  const FilterCount fc{c->f_n, c->f_dn, g.filter_enabled && g.filter_update ? n : 0};
  if (g.model_kind == DDRL_MODEL_FFN)
    launch_observe_ffn(c->stream, ra, obs, c->f_normc, clip, c->stage_tab, g.policy_filter ? c->pf : nullptr, fc);
  else
    launch_observe_gnn(c->stream, ra, obs, c->f_normc, g.filter_enabled ? g.filter_clip : 0.f, c->pol[0].stage, fc);
  HIPCHK(hipGetLastError());
  return 0;
}

int ddrl_observe(ddrl_ctx* c, const float* obs) {
  CHK_CTX(c);
  return ddrl_observe_range(c, obs, 0, c->cfg.n_envs);
}

static ActArgs make_act(ddrl_ctx* c, int t, const float* eps, float* actions, int mode) {
  ActArgs aa{};
  for (int p = 0; p < c->cfg.n_policies; ++p) {
    Policy& P = c->pol[p];
    aa.theta[p] = P.theta; aa.stage[p] = P.stage; aa.rec[p] = P.rec; aa.last_v[p] = P.last_v;
    aa.lay[p] = P.lay; aa.C[p] = P.C;
    aa.cup[p] = c->cfg.leg_coupling ? P.theta + ffn_param_count(P.d, c->cfg.act_dim) : nullptr;
  }
  aa.t = t; aa.eps = eps; aa.actions = actions; aa.bootstrap = mode;
  aa.e0 = 0; aa.e1 = c->cfg.n_envs;
  return aa;
}

static int launch_act(ddrl_ctx* c, const ActArgs& aa) {
  if (c->cfg.model_kind == DDRL_MODEL_FFN) launch_act_ffn(c->stream, c->route, aa);
  else launch_act_gnn(c->stream, c->route, aa, c->cfg.gnn_layer);
  HIPCHK(hipGetLastError());
  return 0;
}

int ddrl_act(ddrl_ctx* c, int t, const float* eps, float* actions) {
  CHK_CTX(c);
  if (t < 0 || t >= c->cfg.frag_len) return fail("t out of range");
  if (!eps || !actions) return fail("null eps/actions buffer");
  return launch_act(c, make_act(c, t, eps, actions, 0));
}

int ddrl_act_range(ddrl_ctx* c, int t, int e0, int e1, const float* eps, float* actions) {
  CHK_CTX(c);
  if (t < 0 || t >= c->cfg.frag_len) return fail("t out of range");
  if (!eps || !actions) return fail("null eps/actions buffer");
  if (check_range(c, e0, e1)) return -1;
  ActArgs aa = make_act(c, t, eps, actions, 0);
  aa.e0 = e0;
  aa.e1 = e1;
  return launch_act(c, aa);
}

int ddrl_bootstrap(ddrl_ctx* c) {
  CHK_CTX(c);
  return launch_act(c, make_act(c, 0, nullptr, nullptr, 1));
}

int ddrl_reward(ddrl_ctx* c, int t, const float* fw, const float* cfrc, const float* actions,
                const uint8_t* done) {
  CHK_CTX(c);
  return ddrl_reward_range(c, t, 0, c->cfg.n_envs, fw, cfrc, actions, done);
}

int ddrl_reward_range(ddrl_ctx* c, int t, int e0, int e1, const float* fw, const float* cfrc, const float* actions,
                      const uint8_t* done) {
  CHK_CTX(c);
  if (t < 0 || t >= c->cfg.frag_len) return fail("t out of range");
  if (!fw || !cfrc || !actions) return fail("null reward input");
  if (check_range(c, e0, e1)) return -1;
  const ddrl_cfg& g = c->cfg;
  RewardArgs ra{};
  ra.P = g.n_policies; ra.N = g.n_envs; ra.n_agents = g.n_agents; ra.mode = g.reward_mode;
  ra.e0 = e0; ra.n = e1 - e0;
  ra.ctrl_w = g.ctrl_cost_weight; ra.contact_w = g.contact_cost_weight; ra.t = t;
  for (int p = 0; p < g.n_policies; ++p) {
    ra.k[p] = c->pol[p].k; ra.rec[p] = c->pol[p].rec; ra.lay[p] = c->pol[p].lay;
    for (int s = 0; s < c->pol[p].k; ++s) {
      ra.policy_of_agent[c->pol[p].agents[s]] = p;
      ra.slot_of_agent[c->pol[p].agents[s]] = s;
    }
  }
  for (int j = 0; j < g.n_agents; ++j) {
    ra.n_act[j] = g.act_dim;
    for (int a = 0; a < 8; ++a) ra.act_index[j][a] = g.act_index[j][a];
    ra.n_contact[j] = g.n_contact[j];
    for (int b = 0; b < 14; ++b) {
      ra.contact_index[j][b] = g.contact_index[j][b];
      ra.contact_weight[j][b] = g.contact_weight[j][b];
    }
  }
  launch_reward(c->stream, ra, fw, cfrc, actions, done, c->done_tn);
  HIPCHK(hipGetLastError());
  return 0;
}

static int rollout_launches(ddrl_ctx* c, const float* obs, const float* eps, const float* fw, const float* cfrc,
                            const uint8_t* done, float* actions) {
  const ddrl_cfg& g = c->cfg;
  const size_t N = g.n_envs;
  for (int t = 0; t < g.frag_len; ++t) {
    if (ddrl_act(c, t, eps + (size_t)t * N * g.n_agents * g.act_dim, actions)) return -1;
    if (ddrl_reward(c, t, fw + (size_t)t * N, cfrc + (size_t)t * N * 14 * 6, actions, done ? done + (size_t)t * N : nullptr))
      return -1;
    if (ddrl_observe(c, obs + (size_t)(t + 1) * N * g.obs_full_dim)) return -1;
  }
  return ddrl_bootstrap(c);
}

int ddrl_rollout_fragment(ddrl_ctx* c, const float* obs, const float* eps, const float* fw, const float* cfrc,
                          const uint8_t* done, float* actions) {
  CHK_CTX(c);
  if (!obs || !eps || !fw || !cfrc || !actions) return fail("null rollout buffer");
  if (!c->rollout_graph) return rollout_launches(c, obs, eps, fw, cfrc, done, actions);
  const void* key[6] = {obs, eps, fw, cfrc, done, actions};
  if (!c->rg_exec || !std::equal(key, key + 6, c->rg_key)) {
    if (c->rg_exec) {
      HIPCHK(hipGraphExecDestroy(c->rg_exec));
      c->rg_exec = nullptr;
    }
    // captured on a private stream (a capture records, it does not run), launched on the caller's
    if (!c->cap_stream) HIPCHK(hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking));
    const hipStream_t user = c->stream;
    c->stream = c->cap_stream;
    hipError_t e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
      c->stream = user;
      return fail(std::string("rollout graph capture: ") + hipGetErrorString(e));
    }
    const int rc = rollout_launches(c, obs, eps, fw, cfrc, done, actions);
    hipGraph_t graph = nullptr;
    e = hipStreamEndCapture(c->stream, &graph);
    c->stream = user;
    if (rc) {
      if (graph) (void)hipGraphDestroy(graph);
      return -1;
    }
    if (e != hipSuccess) return fail(std::string("rollout graph capture: ") + hipGetErrorString(e));
    const hipError_t ei = hipGraphInstantiate(&c->rg_exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess) {
      c->rg_exec = nullptr;
      return fail(std::string("rollout graph instantiate: ") + hipGetErrorString(ei));
    }
    std::copy(key, key + 6, c->rg_key);
  }
  HIPCHK(hipGraphLaunch(c->rg_exec, c->stream));
  return 0;
}

int ddrl_step_host(ddrl_ctx* c, int t, const float* obs_h, const float* eps_h, float* act_h) {
  CHK_CTX(c);
  const ddrl_cfg& g = c->cfg;
  HIPCHK(hipMemcpyAsync(c->h_obs, obs_h, (size_t)g.n_envs * g.obs_full_dim * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->h_eps, eps_h, (size_t)g.n_envs * g.n_agents * g.act_dim * 4, hipMemcpyHostToDevice,
                        c->stream));
  if (ddrl_observe(c, c->h_obs)) return -1;
  if (ddrl_act(c, t, c->h_eps, c->h_act)) return -1;
  HIPCHK(hipMemcpyAsync(act_h, c->h_act, (size_t)g.n_envs * 8 * 4, hipMemcpyDeviceToHost, c->stream));
  return 0;
}

int ddrl_act_host(ddrl_ctx* c, int t, const float* eps_h, float* act_h) {
  CHK_CTX(c);
  if (!eps_h || !act_h) return fail("null host buffer");
  const ddrl_cfg& g = c->cfg;
  HIPCHK(hipMemcpyAsync(c->h_eps, eps_h, (size_t)g.n_envs * g.n_agents * g.act_dim * 4, hipMemcpyHostToDevice,
                        c->stream));
  if (ddrl_act(c, t, c->h_eps, c->h_act)) return -1;
  HIPCHK(hipMemcpyAsync(act_h, c->h_act, (size_t)g.n_envs * 8 * 4, hipMemcpyDeviceToHost, c->stream));
  return 0;
}

int ddrl_env_step_host(ddrl_ctx* c, int t, const float* fw_h, const float* cfrc_h, const uint8_t* done_h,
                       const float* obs_h) {
  CHK_CTX(c);
  if (!fw_h || !cfrc_h || !obs_h) return fail("null host buffer");
  const ddrl_cfg& g = c->cfg;
  const size_t N = g.n_envs;
  HIPCHK(hipMemcpyAsync(c->h_fw, fw_h, N * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->h_cfrc, cfrc_h, N * 14 * 6 * 4, hipMemcpyHostToDevice, c->stream));
  if (done_h) HIPCHK(hipMemcpyAsync(c->h_done, done_h, N, hipMemcpyHostToDevice, c->stream));
  // the env actions of step t are still in h_act (act_host / step_host wrote them)
  if (ddrl_reward(c, t, c->h_fw, c->h_cfrc, c->h_act, done_h ? c->h_done : nullptr)) return -1;
  HIPCHK(hipMemcpyAsync(c->h_obs, obs_h, N * g.obs_full_dim * 4, hipMemcpyHostToDevice, c->stream));
  return ddrl_observe(c, c->h_obs);
}

// f1: a fragment with the envs stepped on the host (ddrl_hostenv, hostenv.cpp), pipelined over
// `groups` env groups: while the host threads step group g, the device runs the other groups'
// reward / observe / act and the transfers.  Per step t and group g (envs [e0, e1)):
//   wait for the actions of (t, g) (event) -> host step of [e0, e1) into the pinned buffers ->
//   H2D of the group's fw / cfrc / done / next obs -> reward_range(t) -> observe_range ->
//   act_range(t + 1) -> D2H of the group's actions -> event.
// The call order on the stream is the same as a synchronous loop over the same groups, so the
// records are bit-identical to it (tests/test_gpu_hostenv.py).  reset: 1 = reset every env
// first and observe the reset observations (per group); 0 = continue from the observation
// the context holds.  eps_dev: [T][N][n_agents][A] exploration noise in HBM.  Ends with the
// bootstrap V(s_T) of every env.
int ddrl_rollout_hostenv(ddrl_ctx* c, ddrl_hostenv* env, int groups, const float* eps_dev, int reset) {
  CHK_CTX(c);
  const ddrl_cfg& g = c->cfg;
  if (!env || !eps_dev) return fail("null host env / noise buffer");
  if (env->N != g.n_envs || env->D != g.obs_full_dim) return fail("host env shape differs from the context's");
  if (groups < 1 || groups > 8 || groups > g.n_envs) return fail("groups must be in [1, min(8, n_envs)]");
  const int N = g.n_envs, D = g.obs_full_dim, T = g.frag_len;
  const size_t eps_step = (size_t)N * g.n_agents * g.act_dim;
  std::vector<int> lo(groups + 1);
  for (int k = 0; k <= groups; ++k) lo[k] = (int)((long long)N * k / groups);
  std::vector<hipEvent_t> ev(groups, nullptr);
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  int rc = 0;
  auto h2d = [&](void* dst, const void* src, size_t bytes) {
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream) == hipSuccess ? 0 : fail("H2D copy failed");
  };
  auto d2h_act = [&](int k) {
    const size_t off = (size_t)lo[k] * 8;
    if (hipMemcpyAsync(env->act + off, c->h_act + off, (size_t)(lo[k + 1] - lo[k]) * 8 * 4, hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess || hipEventRecord(ev[k], c->stream) != hipSuccess)
      return fail("D2H copy failed");
    return 0;
  };
  if (reset) env->reset_all();
  for (int k = 0; k < groups && !rc; ++k) {
    const int e0 = lo[k], e1 = lo[k + 1];
    if (reset) rc = h2d(c->h_obs + (size_t)e0 * D, env->obs + (size_t)e0 * D, (size_t)(e1 - e0) * D * 4) ||
                    ddrl_observe_range(c, c->h_obs, e0, e1);
    rc = rc || ddrl_act_range(c, 0, e0, e1, eps_dev, c->h_act) || d2h_act(k);
  }
  for (int t = 0; t < T && !rc; ++t) {
    for (int k = 0; k < groups && !rc; ++k) {
      const int e0 = lo[k], e1 = lo[k + 1], n = e1 - e0;
      if (hipEventSynchronize(ev[k]) != hipSuccess) { rc = fail("event wait failed"); break; }
      env->step(e0, e1);   // host threads; the device meanwhile runs the other groups' work
      rc = h2d(c->h_fw + e0, env->fw + e0, (size_t)n * 4) ||
           h2d(c->h_cfrc + (size_t)e0 * 84, env->cfrc + (size_t)e0 * 84, (size_t)n * 84 * 4) ||
           h2d(c->h_done + e0, env->done + e0, (size_t)n) ||
           h2d(c->h_obs + (size_t)e0 * D, env->obs + (size_t)e0 * D, (size_t)n * D * 4) ||
           ddrl_reward_range(c, t, e0, e1, c->h_fw, c->h_cfrc, c->h_act, c->h_done) ||
           ddrl_observe_range(c, c->h_obs, e0, e1);
      if (!rc && t + 1 < T)
        rc = ddrl_act_range(c, t + 1, e0, e1, eps_dev + (size_t)(t + 1) * eps_step, c->h_act) || d2h_act(k);
    }
  }
  if (!rc) rc = ddrl_bootstrap(c);
  // the pinned buffers are the caller's again only once the stream has consumed them
  if (hipStreamSynchronize(c->stream) != hipSuccess && !rc) rc = fail("stream synchronize failed");
  for (auto& e : ev) (void)hipEventDestroy(e);
  return rc ? -1 : 0;
}

int ddrl_gae(ddrl_ctx* c) {
  CHK_CTX(c);
  const ddrl_cfg& g = c->cfg;
  GaeBatch gb{};
  gb.P = g.n_policies;
  for (int p = 0; p < g.n_policies; ++p) {
    Policy& P = c->pol[p];
    GaeArgs& ga = gb.g[p];
    ga.rec = P.rec; ga.lay = P.lay; ga.C = P.C; ga.T = g.frag_len; ga.N = g.n_envs; ga.k = P.k;
    ga.last_v = P.last_v; ga.done_tn = c->done_tn; ga.gamma = g.gamma; ga.lambda_ = g.lambda_;
    ga.partials = P.partials; ga.adv_norm = P.adv_norm;
  }
  launch_gae(c->stream, gb);
  HIPCHK(hipGetLastError());
  return 0;
}

static UpdateHyper make_hyper(ddrl_ctx* c, int P) {
  const ddrl_cfg& g = c->cfg;
  UpdateHyper h{};
  h.clip = g.clip_param; h.vf_clip = g.vf_clip_param; h.vf_coeff = g.vf_loss_coeff;
  h.ent_coeff = g.entropy_coeff; h.lr = g.lr; h.grad_clip = g.grad_clip; h.b1 = g.adam_beta1;
  h.b2 = g.adam_beta2; h.eps = g.adam_eps; h.vf_mode = g.vf_clip_mode; h.P = P;
  return h;
}

static UpdateArgs make_update(ddrl_ctx* c, int p, const int32_t* shuffle, const int32_t* perm, float kl) {
  Policy& P = c->pol[p];
  UpdateArgs u{};
  u.rec = P.rec; u.lay = P.lay; u.d = P.d; u.A = c->cfg.act_dim; u.R = P.R;
  u.shuffle = shuffle; u.perm = perm; u.nb = P.nb; u.n_epochs = c->cfg.num_sgd_iter;
  u.max_steps = -1; u.step0 = 0;
  u.theta = P.theta; u.m = P.m; u.v = P.v; u.beta_pow = P.beta_pow; u.stats = P.stats;
  u.adv_norm = P.adv_norm; u.grad_out = nullptr; u.gscr = P.grad; u.kl_coeff = kl;
  u.cup = c->cfg.leg_coupling;
  return u;
}

int ddrl_ppo_update(ddrl_ctx* c, int mask, const int32_t* const* shuffle, const int32_t* const* perm,
                    const float* kl, int max_steps) {
  return ddrl_ppo_update_from(c, mask, shuffle, perm, kl, 0, max_steps);
}

int ddrl_ppo_update_from(ddrl_ctx* c, int mask, const int32_t* const* shuffle, const int32_t* const* perm,
                         const float* kl, int step0, int max_steps) {
  CHK_CTX(c);
  if (!shuffle || !perm || !kl) return fail("null update argument");
  if (step0 < 0) return fail("step0 must be >= 0");
  UpdateArgs ua[DDRL_MAXP];
  int n = 0;
  for (int p = 0; p < c->cfg.n_policies; ++p) {
    if (!(mask & (1 << p))) continue;
    if (!shuffle[p] || !perm[p]) return fail("null shuffle/perm for a masked policy");
    // every minibatch is a full slice of the shuffled batch (RLlib's multi-GPU loader refuses
    // a batch smaller than one minibatch too); the kernels read shuffle[0 .. nb * 128)
    if (c->pol[p].R < c->cfg.sgd_minibatch_size)
      return fail("policy " + std::to_string(p) + ": the train batch holds " + std::to_string(c->pol[p].R) +
                  " rows, fewer than one minibatch (sgd_minibatch_size " +
                  std::to_string(c->cfg.sgd_minibatch_size) + ")");
    ua[n] = make_update(c, p, shuffle[p], perm[p], kl[p]);
    c->kl_last[p] = kl[p];
    ua[n].max_steps = max_steps;
    ua[n].step0 = step0;
    const int total = c->cfg.num_sgd_iter * c->pol[p].nb;
    if (step0 > total) return fail("step0 beyond the schedule's " + std::to_string(total) + " steps");
    c->pol[p].last_steps = max_steps >= 0 ? std::min(total - step0, max_steps) : total - step0;
    ++n;
  }
  if (n == 0) return 0;
  int maxd = 0, maxs = 0;  // KS1 instance / staging rows must cover the widest policy
  for (int i = 0; i < n; ++i) maxd = std::max(maxd, ua[i].d), maxs = std::max(maxs, ua[i].lay.stride);
  UpdateHyper h = make_hyper(c, n);
  // the arguments travel by value in the kernel's argument block (no copy from this stack frame)
  if (c->cfg.model_kind == DDRL_MODEL_FFN) {
    if (snapshot(c, mask & ((1 << c->cfg.n_policies) - 1))) return -1;
    launch_ffn(c, ua, h, 128, 1.f / c->cfg.sgd_minibatch_size, maxd, maxs, c->update_split, (1 << n) - 1);
  }
  else if (c->pol[0].last_steps > 0) {   // one shared policy
    const int last = c->pol[0].last_steps;
    if (!c->gnn.chunk && dalloc(c, &c->gnn.chunk, (size_t)c->gnn.chunk_steps * DDRL_MB * c->pol[0].lay.stride))
      return -1;
    if (snapshot(c, 1)) return -1;
    // test hook (DDRL_TEST_FAIL_STEP): the update starts with the error word set, as a failed
    // launch would leave it; the steps run, check_err restores the snapshot
    if (c->fail_step >= 0) (void)hipMemsetD32Async((hipDeviceptr_t)c->err, 1, 1, c->stream);
    const int CH = c->gnn.chunk_steps;
    // the records of each run of GNN_CHUNK_STEPS steps are gathered into one contiguous
    // chunk first (stream order: after the previous run's last step), so every gradient
    // launch reads its minibatch without dependent index loads
    const size_t step_floats = (size_t)DDRL_MB * ua[0].lay.stride;
    for (int step = step0; step < step0 + last; ++step) {
      const int k = (step - step0) % CH;
      if (k == 0) launch_gnn_gather(c->stream, ua[0], step, std::min(CH, step0 + last - step), c->gnn.chunk);
      launch_step_gnn(c->stream, ua[0], h, step, 128, 1.f / c->cfg.sgd_minibatch_size, c->gnn,
                      c->gnn.chunk + k * step_floats, c->cfg.gnn_layer);
    }
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int ddrl_ppo_stats(ddrl_ctx* c, int pid, float* host, size_t n_steps) {
  return ddrl_ppo_stats_range(c, pid, 0, n_steps, host);
}

int ddrl_ppo_stats_range(ddrl_ctx* c, int pid, size_t first, size_t n_steps, float* host) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (!host && n_steps) return fail("null stats buffer");
  const size_t cap = c->pol[pid].stats_steps;
  if (first > cap || n_steps > cap - first) return fail("more stats requested than the schedule holds");
  HIPCHK(hipMemcpyAsync(host, c->pol[pid].stats + first * 8, n_steps * 8 * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (check_err(c)) return -1;
  // the policy / value workgroups each write their own columns; total_loss is their
  // linear combination: mean(-surr) + beta*mean(kl) + vf_coeff*mean(vf) - ent_coeff*mean(H)
  const ddrl_cfg& g = c->cfg;
  const float beta = c->kl_last[pid];
  for (size_t k = 0; k < n_steps; ++k) {
    float* s = host + 8 * k;
    s[0] = s[1] + beta * s[3] + g.vf_loss_coeff * s[2] - g.entropy_coeff * s[4];
  }
  return 0;
}

// Grow policy pid's learner-statistics buffer to at least `rows` rows, keeping its contents.  A
// data-parallel loop in "split" mode runs 128 / (128 / G) = G times the fused schedule's
// minibatches per epoch, which passes the buffer sized at create (num_sgd_iter x R / 128 rows)
// when G > num_sgd_iter (found by the world-4 rehearsal with one epoch, round 6).  Growing waits
// for the context's stream; it happens once per size.
static int stats_reserve(ddrl_ctx* c, int pid, size_t rows) {
  Policy& P = c->pol[pid];
  if (rows <= P.stats_steps) return 0;
  HIPCHK(hipStreamSynchronize(c->stream));
  float* nw = nullptr;
  if (dalloc(c, &nw, rows * 8)) return -1;
  if (P.stats_steps) HIPCHK(hipMemcpy(nw, P.stats, P.stats_steps * 8 * sizeof(float), hipMemcpyDeviceToDevice));
  dfree(c, &P.stats);
  P.stats = nw;
  P.stats_steps = rows;
  return 0;
}

// Workgroups per branch of a gradient-only update launch: the row split of the fused update
// when the rows fill both halves (64 each), else one.  ddrl_ppo_grad and ddrl_ppo_update_ddp
// share this rule, so the two data-parallel loops run the same kernels.
static int grad_split(const ddrl_ctx* c, int n_rows) { return n_rows > 64 ? c->update_split : 1; }

int ddrl_ppo_grad(ddrl_ctx* c, int pid, const int32_t* rows, int n_rows, float kl, float* grad,
                  int stats_step) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (n_rows < 1 || n_rows > 128) return fail("n_rows must be in [1, 128]");
  if (!rows || !grad) return fail("null rows/grad");
  if (stats_step >= 0 && (size_t)stats_step >= c->pol[pid].stats_steps &&
      stats_reserve(c, pid, std::max((size_t)stats_step + 1, 2 * c->pol[pid].stats_steps)))
    return -1;
  UpdateArgs u = make_update(c, pid, rows, c->zero_perm, kl);
  u.nb = 1; u.n_epochs = 1; u.max_steps = 1; u.step0 = 0; u.grad_out = grad;
  c->snap_mask = 0;   // a gradient launch changes no state: the caller's loop keeps its own snapshot
  u.stats = stats_step >= 0 ? c->pol[pid].stats + (size_t)stats_step * 8 : nullptr;
  c->kl_last[pid] = kl;
  UpdateHyper h = make_hyper(c, 1);
  if (c->cfg.model_kind == DDRL_MODEL_FFN)
    launch_ffn(c, &u, h, n_rows, 1.f / c->cfg.sgd_minibatch_size, c->pol[pid].d, c->pol[pid].lay.stride,
               grad_split(c, n_rows), 1);
  else
    launch_step_gnn(c->stream, u, h, 0, n_rows, 1.f / c->cfg.sgd_minibatch_size, c->gnn, nullptr, c->cfg.gnn_layer);
  HIPCHK(hipGetLastError());
  return 0;
}

int ddrl_ppo_apply(ddrl_ctx* c, int pid, const float* grad) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (!grad) return fail("null grad");
  Policy& P = c->pol[pid];
  launch_apply_adam(c->stream, grad, P.n_params, P.theta, P.m, P.v, P.beta_pow, make_hyper(c, 1), 1.f, pid, c->err);
  HIPCHK(hipGetLastError());
  return 0;
}

static_assert(sizeof(ncclUniqueId) == DDRL_COMM_ID_BYTES, "RCCL unique id size");

int ddrl_comm_unique_id(void* out, size_t n) {
  if (!out || n < sizeof(ncclUniqueId)) return fail("unique id buffer too small");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

int ddrl_comm_init(ddrl_ctx* c, const void* id, int rank, int nranks) {
  CHK_CTX(c);
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail("bad communicator arguments");
  if (c->comm) return fail("the context already has a communicator");
  HIPCHK(hipSetDevice(c->device));
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCLCHK(ncclCommInitRank(&c->comm, nranks, uid, rank));
  return 0;
}

int ddrl_comm_allreduce(ddrl_ctx* c, float* buf, size_t n) {
  CHK_CTX(c);
  if (!c->comm) return fail("no communicator (ddrl_comm_init)");
  if (!buf) return fail("null buffer");
  NCCLCHK(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, c->comm, c->stream));
  return 0;
}

int ddrl_ppo_update_ddp(ddrl_ctx* c, int pid, const int32_t* shuffle, const int32_t* perm, int E, int nb,
                        int m, float kl, float gscale) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (!c->comm) return fail("no communicator (ddrl_comm_init)");
  if (!shuffle || !perm || E < 1 || nb < 1) return fail("bad schedule");
  if (m < 1 || m > 128) return fail("rows_per_rank must be in [1, 128]");
  if (stats_reserve(c, pid, (size_t)nb)) return -1;   // the last epoch's rows
  Policy& P = c->pol[pid];
  const int steps = E * nb;
  const UpdateHyper h = make_hyper(c, 1);
  const float inv_n = 1.f / c->cfg.sgd_minibatch_size;
  std::vector<UpdateArgs> ua((size_t)steps);
  for (int e = 0; e < E; ++e)
    for (int b = 0; b < nb; ++b) {
      const int slot = perm[(size_t)e * nb + b];
      if (slot < 0 || (size_t)(slot + 1) * m > (size_t)P.R) return fail("minibatch slot out of range");
      UpdateArgs u = make_update(c, pid, shuffle + (size_t)slot * m, c->zero_perm, kl);
      u.nb = 1; u.n_epochs = 1; u.max_steps = 1; u.step0 = 0; u.grad_out = P.grad;
      u.stats = e == E - 1 ? P.stats + (size_t)b * 8 : nullptr;
      ua[(size_t)e * nb + b] = u;
    }
  const bool ffn = c->cfg.model_kind == DDRL_MODEL_FFN;
  // the records of each run of up to DDP_CHUNK_STEPS steps are gathered into one contiguous
  // chunk first (stream order: after the previous run's last gradient launch), so a one-step
  // gradient launch stages its rows without the dependent perm -> shuffle index loads
  constexpr int DDP_CHUNK_STEPS = 1024;
  const int CH = std::min(DDP_CHUNK_STEPS, steps);
  const int stride = P.lay.stride;
  const size_t need = (size_t)CH * m * stride;
  // grown buffers replace the old ones (the previous call ended with a stream synchronize)
  if (c->ddp_chunk_n < need) {
    dfree(c, &c->ddp_chunk);
    c->ddp_chunk_n = 0;
    if (dalloc(c, &c->ddp_chunk, need)) return -1;
    c->ddp_chunk_n = need;
  }
  if (c->ddp_slots_n < (size_t)steps) {
    dfree(c, &c->ddp_slots);
    c->ddp_slots_n = 0;
    if (dalloc(c, &c->ddp_slots, (size_t)steps)) return -1;
    c->ddp_slots_n = (size_t)steps;
  }
  c->ddp_slots_host.assign(perm, perm + steps);
  HIPCHK(hipMemcpyAsync(c->ddp_slots, c->ddp_slots_host.data(), sizeof(int32_t) * steps, hipMemcpyHostToDevice,
                        c->stream));
  c->kl_last[pid] = kl;
  // restored by check_err if any step fails (the GNN gradient launches of 128 rows per rank
  // reduce in their tail, with bounded waits: ADVICE r4)
  if (snapshot(c, 1 << pid)) return -1;
  for (int s = 0; s < steps; ++s) {
    const int k = s % CH;
    if (k == 0) launch_rows_gather(c->stream, P.rec, stride, shuffle, c->ddp_slots, m, s, std::min(CH, steps - s),
                                   c->ddp_chunk);
    float* rows = c->ddp_chunk + (size_t)k * m * stride;
    // test hook: step s's gradient is lost (its Adam launch and every later one skip)
    if (s == c->fail_step) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)c->err, 1, 1, c->stream));
    if (ffn) {
      ua[s].rec = rows;
      ua[s].shuffle = nullptr;   // rows 0 .. m of the slice
      launch_ffn(c, &ua[s], h, m, inv_n, P.d, stride, grad_split(c, m), 1);
    } else {
      launch_step_gnn(c->stream, ua[s], h, 0, m, inv_n, c->gnn, rows, c->cfg.gnn_layer);
    }
    NCCLCHK(ncclAllReduce(P.grad, P.grad, (size_t)P.n_params, ncclFloat32, ncclSum, c->comm, c->stream));
    launch_apply_adam(c->stream, P.grad, P.n_params, P.theta, P.m, P.v, P.beta_pow, h, gscale, pid, c->err);
  }
  // every rank fails together: a norm-exchange timeout on one rank (whose zeroed gradient has
  // already been summed into every rank's weights) is all-reduced (max) into every rank's
  // error word, so no rank goes on to its next collective while another one raises
  NCCLCHK(ncclAllReduce(c->err, c->err, 1, ncclInt32, ncclMax, c->comm, c->stream));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));   // the error word of every step
  return check_err(c);
}

static_assert(sizeof(hipIpcMemHandle_t) == DDRL_PEER_HANDLE_BYTES, "IPC handle size");

int ddrl_peer_alloc(ddrl_ctx* c, void** gx_out, void* ipc_handle_out) {
  CHK_CTX(c);
  if (!gx_out) return fail("null outbox pointer");
  HIPCHK(hipSetDevice(c->device));
  const size_t bytes = gx_bytes(DDRL_MAXP);
  void* p = nullptr;
  HIPCHK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
  c->allocs.push_back(p);
  HIPCHK(hipMemset(p, 0, bytes));
  if (ipc_handle_out) {
    hipIpcMemHandle_t h;
    HIPCHK(hipIpcGetMemHandle(&h, p));
    std::memcpy(ipc_handle_out, &h, sizeof(h));
  }
  *gx_out = p;
  return 0;
}

int ddrl_peer_open(ddrl_ctx* c, const void* ipc_handle, void** gx_out) {
  CHK_CTX(c);
  if (!ipc_handle || !gx_out) return fail("null IPC handle / outbox pointer");
  if (c->peer_ipc) return fail("the context already maps a peer's outboxes");
  HIPCHK(hipSetDevice(c->device));
  hipIpcMemHandle_t h;
  std::memcpy(&h, ipc_handle, sizeof(h));
  void* p = nullptr;
  HIPCHK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  c->peer_ipc = p;
  *gx_out = p;
  return 0;
}

// Peer-mode buffers for E epochs of nb minibatch slots of policy pid: the statistics rows (the
// union batch has twice this rank's minibatches) and the virtual 128-row shuffle.  Growing them
// frees and allocates, which waits for the whole device -- for a peer context in the same
// process, whose launch waits for this one's, that is a stall until the 3 s bound -- so
// ddrl_peer_attach reserves the configured schedule (num_sgd_iter epochs of R / 64 slots) up front.
static int peer_reserve(ddrl_ctx* c, int pid, size_t E, size_t nb) {
  Policy& P = c->pol[pid];
  if (E * nb > P.stats_steps) {
    HIPCHK(hipStreamSynchronize(c->stream));
    dfree(c, &P.stats);
    P.stats_steps = 0;
    if (dalloc(c, &P.stats, E * nb * 8)) return -1;
    P.stats_steps = E * nb;
  }
  if (c->peer_vsh_n < nb * DDRL_MB) {
    HIPCHK(hipStreamSynchronize(c->stream));
    dfree(c, &c->peer_vsh);
    c->peer_vsh_n = 0;
    if (dalloc(c, &c->peer_vsh, nb * DDRL_MB)) return -1;
    c->peer_vsh_n = nb * DDRL_MB;
  }
  return 0;
}

int ddrl_peer_attach(ddrl_ctx* c, void* gx, int rank, int nranks) {
  CHK_CTX(c);
  if (!gx) return fail("null outboxes");
  if (nranks != 2 || rank < 0 || rank > 1) return fail("peer mode splits the minibatch over exactly two ranks");
  if (c->cfg.model_kind != DDRL_MODEL_FFN) return fail("peer mode is built for fcnet policies");
  if (c->update_split != 2) return fail("peer mode needs the row split (DDRL_UPDATE_SPLIT=2, the default)");
  // rank 0 clears the outboxes (no launch of either rank may be in flight: after a failed update
  // both ranks have synchronized; rank 1 attaches after rank 0); both count launches from here
  if (rank == 0) HIPCHK(hipMemsetAsync(gx, 0, gx_bytes(DDRL_MAXP), c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int p = 0; p < c->cfg.n_policies; ++p)
    if (peer_reserve(c, p, (size_t)c->cfg.num_sgd_iter, (size_t)c->pol[p].R / (DDRL_MB / 2))) return -1;
  c->peer_gx = gx;
  c->peer_rank = rank;
  c->peer_epoch = 0;
  c->peer_steps = 0;
  return 0;
}

int ddrl_ppo_update_peer(ddrl_ctx* c, int pid, const int32_t* shuffle, const int32_t* perm, int E, int nb, float kl,
                         int max_steps) {
  CHK_CTX(c);
  if (!c->peer_gx) return fail("no peer (ddrl_peer_attach)");
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (!shuffle || !perm || E < 1 || nb < 1) return fail("bad schedule");
  Policy& P = c->pol[pid];
  if ((size_t)nb * (DDRL_MB / 2) > (size_t)P.R) return fail("nb x 64 rows exceed this rank's train batch");
  if (peer_reserve(c, pid, (size_t)E, (size_t)nb)) return -1;   // no-op within the attached schedule
  // this rank's rows fill half peer_rank of every 128-row block of the shuffle the kernel indexes
  // (UpdateArgs::shuffle[slot * 128 + row], row half kq = rows 64 kq .. 64 kq + 63)
  constexpr int H = DDRL_MB / 2;
  HIPCHK(hipMemcpy2DAsync(c->peer_vsh + H * c->peer_rank, DDRL_MB * sizeof(int32_t), shuffle, H * sizeof(int32_t),
                          H * sizeof(int32_t), nb, hipMemcpyDeviceToDevice, c->stream));
  UpdateArgs u = make_update(c, pid, c->peer_vsh, perm, kl);
  u.nb = nb;
  u.n_epochs = E;
  u.max_steps = max_steps;
  const int total = E * nb;
  P.last_steps = max_steps >= 0 ? std::min(total, max_steps) : total;
  c->kl_last[pid] = kl;
  if (snapshot(c, 1 << pid)) return -1;
  c->xcc_pending = 0;   // the atomic protocol is valid for any placement
  UpdateHyper h = make_hyper(c, 1);
  launch_update_ffn_peer(c->stream, &u, h, DDRL_MB, 1.f / c->cfg.sgd_minibatch_size, c->cfg.act_dim, P.d,
                         P.lay.stride, c->cfg.leg_coupling, c->xchg, static_cast<unsigned long long*>(c->peer_gx), 2,
                         c->err, &c->peer_epoch, c->xcc, c->peer_rank, c->peer_steps);
  c->peer_steps += (unsigned)P.last_steps;   // the same count on both ranks
  c->peer_inflight = 1;
  const hipError_t le = hipGetLastError();
  if (le != hipSuccess) {
    peer_detach(c);
    return fail(std::string("peer update launch refused: ") + hipGetErrorString(le) +
                "; this context is detached from its peer (both ranks re-attach)");
  }
  return 0;
}

int ddrl_gnn_one_launch(ddrl_ctx* c, int* on) {
  CHK_CTX(c);
  if (!on) return fail("null output");
  *on = c->cfg.model_kind == DDRL_MODEL_GNN && c->gnn.tail && c->gnn.lists == 1;
  return 0;
}

int ddrl_policy_forward(ddrl_ctx* c, int pid, const float* obs, const int32_t* node, int n,
                        float* logits, float* values) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (n < 1 || !obs || !logits || !values) return fail("bad forward arguments");
  if (c->cfg.model_kind == DDRL_MODEL_GNN && !node) return fail("gnn forward needs the node index of every row");
  if (c->cfg.leg_coupling && !node) return fail("the \"cup\" forward needs the leg index of every row");
  Policy& P = c->pol[pid];
  ForwardArgs fa{};
  fa.theta = P.theta; fa.x = obs; fa.node = node; fa.n = n; fa.d = P.d; fa.A = c->cfg.act_dim;
  fa.logits = logits; fa.values = values;
  fa.cup = c->cfg.leg_coupling ? P.theta + ffn_param_count(P.d, c->cfg.act_dim) : nullptr;
  if (c->cfg.model_kind == DDRL_MODEL_FFN) launch_forward_ffn(c->stream, fa);
  else launch_forward_gnn(c->stream, fa, c->cfg.gnn_layer);
  HIPCHK(hipGetLastError());
  return 0;
}

int ddrl_records_get(ddrl_ctx* c, int pid, float* host, size_t n) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  const Policy& P = c->pol[pid];
  if (n != (size_t)P.R * P.lay.stride) return fail("record buffer size mismatch");
  HIPCHK(hipMemcpyAsync(host, P.rec, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_records_set(ddrl_ctx* c, int pid, const float* host, size_t n) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  const Policy& P = c->pol[pid];
  if (n != (size_t)P.R * P.lay.stride) return fail("record buffer size mismatch");
  HIPCHK(hipMemcpyAsync(P.rec, host, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_adv_norm_get(ddrl_ctx* c, int pid, float* host2) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  HIPCHK(hipMemcpyAsync(host2, c->pol[pid].adv_norm, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_adv_norm_set(ddrl_ctx* c, int pid, float mean, float den) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  float a[2] = {mean, den};
  HIPCHK(hipMemcpyAsync(c->pol[pid].adv_norm, a, 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_last_values_get(ddrl_ctx* c, int pid, float* host, size_t n) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (n != (size_t)c->pol[pid].C) return fail("last value count mismatch");
  HIPCHK(hipMemcpyAsync(host, c->pol[pid].last_v, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_last_values_set(ddrl_ctx* c, int pid, const float* host, size_t n) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  if (n != (size_t)c->pol[pid].C) return fail("last value count mismatch");
  HIPCHK(hipMemcpyAsync(c->pol[pid].last_v, host, n * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_done_set(ddrl_ctx* c, const uint8_t* host, size_t n) {
  CHK_CTX(c);
  if (n != (size_t)c->cfg.frag_len * c->cfg.n_envs) return fail("done buffer size mismatch");
  HIPCHK(hipMemcpyAsync(c->done_tn, host, n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

int ddrl_device_buffers(ddrl_ctx* c, int pid, void** records, void** last_v, void** params, void** adv_norm) {
  CHK_CTX(c);
  if (pid < 0 || pid >= c->cfg.n_policies) return fail("bad policy id");
  Policy& P = c->pol[pid];
  if (records) *records = P.rec;
  if (last_v) *last_v = P.last_v;
  if (params) *params = P.theta;
  if (adv_norm) *adv_norm = P.adv_norm;
  return 0;
}

}  // extern "C"
