// a3/a9/a10 + a13-a16 for the GraphNet / MPNN model ("gnn", shared leg policy).
//
// Reference: models/graph_net.py:8-45 (GraphNet: hypernetwork state encoder + MPNN + linear
// out), models/gcn.py:57-94 (MPNN: message = h Wmsg, segment-mean over receivers,
// y = tanh(h Wnode + m)), models/shared_graphnet_glorot_uniform_init.py:14-58 (actor and
// critic are two separate GraphNets on the same graph observation; the agent's own node
// is gathered before linear_out).  Per net and node n of a graph:
//   W_n = tanh(q_n Wenc + benc)  reshaped [19, 64]      (q_n = ego quaternion, 4)
//   h_n = tanh(f_n W_n)                                  (f_n = 19 leg features)
//   m_n = (h_{n-1} Wmsg + h_{n+1} Wmsg) / 2              (ring FL-HL-HR-FR)
//   y_n = tanh(h_n Wnode + m_n);  out = y_sel Wout + bout
//
// Work unit: one workgroup = one TILE of 4 graphs x 4 nodes (16 graph-nodes, the 16 rows
// of a 16x16x4 f32 MFMA) for ONE net (blockIdx.y = 0 actor, 1 critic).  Lane (c, q) of
// every wave owns graph-node row c = 4 g + n; activations live in registers in the
// transposed MFMA layout (row c, features 16 t + 4 q + r), as in the fcnet kernels.
//   hypernet : the 4 waves split the 19 feature rows i of W_n (i = w, w+4, ...); for each
//              (i, 16-column block t) one MFMA (K = 4 quaternion dims, bias in the
//              accumulator), tanh, and f_i * W_n[i] accumulated in registers; the four
//              partial sums meet in LDS (fixed order) -> h.
//   MPNN     : wave w computes output features 16 w .. 16 w + 15 of msg and node from h in
//              registers (A = weights, loaded once per launch into VGPRs); the ring
//              neighbours of a node are the other lanes of its DPP quad (quad_perm).
//   head     : per-wave partial dot over its 16 features, summed across waves in LDS.
//   backward : the reverse of the above; weight gradients of Wmsg / Wnode as 16x16 tiles
//              over the 16 rows (MFMA, LDS images), Wenc / benc / Wout gradients by DPP
//              transpose-reductions over the 16 rows of a DPP row.
// Message-passing layer (template L, model_config "gnn_layer"; models/graph_net.py:20 selects
// one of models/gcn.py's layers, MPNN by default), on the ring where every node has the two
// neighbours n - 1, n + 1 (ring(x)_n = (x_{n-1} + x_{n+1}) / 2, DPP quad moves):
//   MPNN  (gcn.py:57-94)    y = tanh(h Wnode + ring(h Wmsg))
//   GCN   (gcn.py:29-37)    y = tanh(ring(h) W)          (graph_ops.adj_norm: D^-1 A)
//   MPNN2 (gcn.py:113-150)  m = ring(h Wmsg[:64]) + h Wmsg[64:],  y = tanh(h Wnode[:64] + m Wnode[64:])
//   GAT1  (gcn.py:171-206)  z = h Wp, e_sr = leaky_relu(z_s a[:64] + z_r a[64:]) over the ring with
//                           self loops, alpha_sr = exp(e_sr) / sum_s' exp(e_s'r) (softmax over the
//                           senders of r, graph_ops.segment_softmax), y_s = tanh(sum_r alpha_sr z_r)
//                           (the reference's attention @ x aggregates along the sender row)
// Training steps are three launches: per-tile partial gradients (k_gnn<MODE_GRAD>), a
// fixed-order reduction over tiles + squared norm partials (k_gnn_reduce), and
// clip_by_global_norm + tf1 Adam (k_gnn_adam).  A DDP step stops after the reduction.
// (Reduction and Adam fused into one launch behind a grid barrier measured slower: DESIGN §3.)
#include <vector>

#include "common.h"
#include "kernels.h"
#include "ppo_loss.h"
#include "ddrl_hip.h"   // DDRL_GNN_* layer ids

#define GF 19              // leg features per node
#define GHE (GF * 64)      // hypernetwork output width (1216)
#define GNI 5              // feature rows i per wave (ceil(19 / 4))

enum { GNN_ACT = 0, GNN_FWD = 1, GNN_GRAD = 2 };
// the wave index as a scalar and the wave's own h block loaded directly (A/B: -DDDRL_GNN_HW=0)
#ifndef DDRL_GNN_HW
#define DDRL_GNN_HW 1
#endif
// Gradient launches split each tile's backward over GNN_Z workgroups (blockIdx.z): all of
// them run the forward (the backward needs every activation), workgroup z then computes only
// the hypernetwork feature rows k % GNN_Z == z of each wave and its Wnode / Wmsg tile slots
// (gnn_tile_owner); every partial is still written by exactly one workgroup.  Measured at C5
// (2048 envs): Z = 1 / 2 / 4 / 5 -> 25.2 / 24.4 / 21.9 / 24.9 us per step (Z = 5 puts two
// workgroups on some CUs: 320 > 256).
#ifndef DDRL_GNN_Z
#define DDRL_GNN_Z 4
#endif
constexpr int GNN_Z = DDRL_GNN_Z;
static_assert(GNN_Z >= 1 && GNN_Z <= GNI, "split of the gradient backward");
// Owner of the Wnode / Wmsg tile slot k (0..7) of each wave.  With four shares, share 0's
// waves 0-2 also carry the hypernetwork rows 16-18 (19 rows over 16 waves), so its tile
// slots go to shares 1-3 (measured 0.26 us per step shorter at C5 than k % 4).
__device__ __forceinline__ int gnn_tile_owner(int k) {
#ifdef DDRL_GNN_TILE_MOD
  return k % GNN_Z;
#endif
  return GNN_Z == 4 ? 1 + k % 3 : k % GNN_Z;
}
// Owner of the hypernetwork backward's (feature row slot k, 16-column block t) of each wave:
// row slot k % GNN_Z, except that with four shares the last slot (rows 16-18, waves 0-2) is
// dealt by column block, so no wave carries two whole rows.
__device__ __forceinline__ int gnn_hbwd_owner(int k, int t) {
  return (GNN_Z == 4 && k == GNI - 1) ? t : k % GNN_Z;
}

// Layer kernels of a net, in the reference's variable order: "wmsg" holds MPNN msg_transform,
// GCN linear, MPNN2 msg_transform [128][64] or GAT1 pre_att_linear; "wnode" holds MPNN
// node_update, MPNN2 node_update [128][64] or GAT1 att_linear [128][1] (GCN: none).
__host__ __device__ constexpr int gnn_msg_floats(int L) { return L == DDRL_GNN_MPNN2 ? 8192 : 4096; }
__host__ __device__ constexpr int gnn_node_floats(int L) {
  return L == DDRL_GNN_MPNN ? 4096 : (L == DDRL_GNN_MPNN2 ? 8192 : (L == DDRL_GNN_GAT1 ? 128 : 0));
}
// 16 x 16 weight-gradient tiles of the layer per net (16 per 64 x 64 matrix)
__host__ __device__ constexpr int gnn_layer_mats(int L) {
  return L == DDRL_GNN_MPNN ? 2 : (L == DDRL_GNN_MPNN2 ? 4 : 1);
}
struct GnnNetOff { int wenc, benc, wmsg, wnode, wout, bout; };
__host__ __device__ inline GnnNetOff gnn_net_off(int A, int net, int L = DDRL_GNN_MPNN) {
  const int actor = 4 * GHE + GHE + gnn_msg_floats(L) + gnn_node_floats(L) + 64 * 2 * A + 2 * A;
  const int O = net ? 1 : 2 * A;
  GnnNetOff o;
  o.wenc = net ? actor : 0;
  o.benc = o.wenc + 4 * GHE;
  o.wmsg = o.benc + GHE;
  o.wnode = o.wmsg + gnn_msg_floats(L);
  o.wout = o.wnode + gnn_node_floats(L);
  o.bout = o.wout + 64 * O;
  return o;
}

// DPP quad neighbours: lane n of a quad receives lane (n - 1) & 3 / (n + 1) & 3.
__device__ __forceinline__ float quad_prev(float v) { return dpp_mov<0x93>(v); }   // [3,0,1,2]
__device__ __forceinline__ float quad_next(float v) { return dpp_mov<0x39>(v); }   // [1,2,3,0]

// LDS (floats): part [4 waves][16][64] (hypernet partials; later dz exchange), h / du / dm
// images [16][64] swizzled (DDRL_LBLK floats each, common.h), head partials [4][16][4],
// per-graph dout [4][4], stats [4][8].
#define L_PART 0
#define L_H (L_PART + 4096)
#define L_DU (L_H + DDRL_LBLK)
#define L_DM (L_DU + DDRL_LBLK)
#define L_HP (L_DM + DDRL_LBLK)
#define L_DOUT (L_HP + 256)
#define L_ST (L_DOUT + 16)
#define L_SEL (L_ST + 32)
#define L_TP (L_SEL + 8)          // per-wave 2 x 4 x 16x16 transpose tiles of the hypernet backward
#define L_QT (L_TP + 8 * 1024)    // quaternions of the tile's 16 graph-nodes [16][4]
#define L_TOTAL (L_QT + 64)
// inside L_TP (used only by the hypernetwork backward, after every layer tile is done):
#define L_M (L_TP)                      // MPNN2: message image m [16][64] swizzled
#define L_DMR (L_TP + DDRL_LBLK)        // MPNN2: ring(dm) image
#define L_GA (L_TP + 2 * DDRL_LBLK)     // GAT1: cross-wave partial dots [4 waves][16 nodes][4]
static_assert(2 * DDRL_LBLK + 256 <= 8 * 1024, "MPNN2 / GAT1 images inside the hypernet-backward tiles");

// Partial-gradient stores: read once, by the reduction kernel, mostly on other XCDs.
// Nontemporal stores stream them out of the XCD's L2 while the kernel runs instead of
// leaving 3.6 MB of dirty lines for the end-of-kernel write-back (C5: 20.9 -> 20.2 us per step;
// the same for the reduction's and Adam's outputs measured no gain).
// The one-launch step (l2: the partials are read by reducers on the same XCD in the same
// launch, gnn_tail) keeps them in the XCD's L2 with plain stores instead.
// (measured at C5, 2048 envs, one box: plain 18.19 us per step, nontemporal 18.58)
#ifndef DDRL_GNN_L2_PLAIN
#define DDRL_GNN_L2_PLAIN 1
#endif
__device__ __forceinline__ void pst(bool l2, float* p, float v) {
  if (l2 && DDRL_GNN_L2_PLAIN) *p = v;
  else __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void pst4(bool l2, float* p, floatx4 v) {
  if (l2 && DDRL_GNN_L2_PLAIN) *reinterpret_cast<floatx4*>(p) = v;
  else __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(p));
}
__device__ __forceinline__ float leaky02(float x) { return x > 0.f ? x : 0.2f * x; }   // tf.nn.leaky_relu

// Hypernetwork-backward transpose tiles [16 rows][16 columns]: the 4-float chunk q of row c sits
// at chunk q ^ ((c >> 1) & 3) of its row (round 5), so the rows' ds_write_b128 (8-lane groups) and
// the transposed ds_read_b32 (lane c reads column c of a row) are both bank-conflict free; the
// plain [c][4q] layout made the stores 4-way.
__device__ __forceinline__ int tp_w(int c, int q) { return c * 16 + ((q ^ ((c >> 1) & 3)) << 2); }
__device__ __forceinline__ int tp_r(int row, int c) { return row * 16 + (c ^ (((row >> 1) & 3) << 2)); }

// Diagnostic build only (-DDDRL_GNN_STAMPS, tools/diag_gnn_stamps.py): s_memrealtime (100 MHz,
// one clock for the whole chip) at the phase boundaries of the gradient launch, thread 0 of the
// workgroups of tile 0 (both nets, every backward share), and at the start / end of block 0 of
// the reduction and Adam launches; one row per step (plain stores); no stamp executes in the
// real build.
#ifdef DDRL_GNN_STAMPS
#define GST_STEPS 4096
#define GST_K 12
__device__ unsigned long long g_gstamps[GST_STEPS][9][GST_K];   // [step][8 gradient WGs + reduce/adam][k]
// start / end of EVERY workgroup of the three launches: [step][launch][block][start, end]
#define GST_NB 256
__device__ unsigned long long g_gspan[GST_STEPS][3][GST_NB][2];
extern "C" int ddrl_diag_gnn_stamps(unsigned long long* host, unsigned long long* span) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gstamps), sizeof(g_gstamps)) != hipSuccess) return -1;
  return span && hipMemcpyFromSymbol(span, HIP_SYMBOL(g_gspan), sizeof(g_gspan)) != hipSuccess ? -1 : 0;
}
#define SPAN(launch, blk, k)                                                                        \
  do {                                                                                              \
    if (threadIdx.x == 0 && ga.step < GST_STEPS && (blk) < GST_NB)                                  \
      g_gspan[ga.step][launch][blk][k] = __builtin_amdgcn_s_memrealtime();                          \
  } while (0)
#define RSTAMPB(b, k)                                                                               \
  do {                                                                                              \
    if (threadIdx.x == 0 && (b) == 0 && ga.step < GST_STEPS)                                        \
      g_gstamps[ga.step][8][k] = __builtin_amdgcn_s_memrealtime();                                  \
  } while (0)
#define GSTAMP(k)                                                                                   \
  do {                                                                                              \
    if (MODE == GNN_GRAD && threadIdx.x == 0 && tile == 0 && ga.step < GST_STEPS)                   \
      g_gstamps[ga.step][NET * 4 + (zs & 3)][k] = __builtin_amdgcn_s_memrealtime();                \
  } while (0)
#else
#define GSTAMP(k)
#define RSTAMPB(b, k)
#define SPAN(launch, blk, k)
#endif

template <int A, int MODE, int NET, int L>
__device__ __forceinline__ void gnn_tile(const GnnArgs& ga, float* lds, const int tile, const int zs) {
  constexpr int O = NET ? 1 : 2 * A;
#if DDRL_GNN_HW
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, q = lane >> 4,
            w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar index arithmetic
#else
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, q = lane >> 4, w = tid >> 6;
#endif
  const int g = c >> 2, n = c & 3;
  const int graph = 4 * tile + g;
  const bool gvalid = graph < ga.n_graphs;
  const GnnNetOff off = gnn_net_off(A, NET, L);
  const float* __restrict__ th = ga.theta;
  GSTAMP(0);
  if (MODE == GNN_ACT && NET == 0 && ga.bootstrap) return;   // bootstrap: critic only
  if (MODE == GNN_GRAD && ga.only_share >= 0 && zs != ga.only_share) return;   // owner discovery
#ifdef DDRL_ABL_GNN_EMPTY
  if (MODE == GNN_GRAD) return;
#endif

  // ---- locate this lane's graph (X [4][23]) and the selected node ----
  const float* X;
  int sel = 0;
  int ridx = 0;
  constexpr int NPRE = NET ? 2 : 3 * A + 2;
  float pre[NPRE];
#pragma unroll
  for (int j = 0; j < NPRE; ++j) pre[j] = 0.f;
  float adv_m = 0.f, adv_d = 1.f;
  if constexpr (MODE == GNN_ACT) {
    X = ga.x + (size_t)(ga.act_e0 + (gvalid ? graph : 0)) * 92;
  } else if constexpr (MODE == GNN_FWD) {
    X = ga.x + (size_t)(gvalid ? graph : 0) * 92;
    sel = gvalid ? ga.node[graph] : 0;
  } else {
    const UpdateArgs& U = ga.u;
    if (ga.stage) {   // pre-gathered (launch_gnn_gather): no dependent index loads
      X = ga.stage + (size_t)(gvalid ? graph : 0) * U.lay.stride + U.lay.obs;
    } else {
      const int e = ga.step / U.nb, b = ga.step - e * U.nb;
      ridx = gvalid ? U.shuffle[U.perm[e * U.nb + b] * DDRL_MB + graph] : 0;
      X = U.rec + (size_t)ridx * U.lay.stride + U.lay.obs;
    }
    // unconditional load (X is a valid row for every lane), converted where it is used: a
    // conditional one was waited for before any other record or weight load went out
    const float selv = X[92];
    sel = gvalid ? (int)selv : 0;
    // the loss head's record fields (lanes 0-15: node c of graph c / 4), loaded here with the
    // rest of the record: at the head, after the forward, they were one more memory latency on
    // every step's path (an invalid graph reads graph 0's row; the loss masks it)
    if (tid < 16) {
      const float* rp = X - U.lay.obs;
      if constexpr (NET == 0) {
#pragma unroll
        for (int j = 0; j < A; ++j) pre[j] = rp[U.lay.act + j];
#pragma unroll
        for (int j = 0; j < 2 * A; ++j) pre[A + j] = rp[U.lay.logit + j];
        pre[3 * A] = rp[U.lay.logp];
        pre[3 * A + 1] = rp[U.lay.adv];
      } else {
        pre[0] = rp[U.lay.vf];
        pre[1] = rp[U.lay.vt];
      }
    }
    adv_m = U.adv_norm[0];
    adv_d = U.adv_norm[1];
  }
  const float* xr = X + n * 23;
  float fi[GNI];
#pragma unroll
  for (int k = 0; k < GNI; ++k) {
    const int i = w + 4 * k;
    const float xv = xr[i < GF ? i : 0];
    fi[k] = i < GF ? xv : 0.f;
  }
  const float qv = xr[GF + q];   // B operand of the hypernet MFMA: q_row[c][q]

  // ---- weights of this wave into registers (read once per launch) ----
  float we[GNI][4];
  floatx4 be[GNI][4];
#pragma unroll
  for (int k = 0; k < GNI; ++k) {
    const int i = w + 4 * k;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = i * 64 + 16 * t;
      we[k][t] = i < GF ? th[off.wenc + q * GHE + j + c] : 0.f;
      be[k][t] = i < GF ? *reinterpret_cast<const floatx4*>(th + off.benc + j + 4 * q) : splat4(0.f);
    }
  }
  // layer weights of output block w (A operand: W[k = 16 fb + 4 q + r][16 w + c]):
  //   wmf: MPNN msg / GCN linear / MPNN2 msg rows 0-63 / GAT1 pre_att;  wnf: MPNN node / MPNN2
  //   node rows 0-63;  wm2 / wn2: MPNN2 msg / node rows 64-127
  constexpr bool TWO = L == DDRL_GNN_MPNN || L == DDRL_GNN_MPNN2;
  constexpr bool M2 = L == DDRL_GNN_MPNN2;
  float wmf[4][4], wnf[TWO ? 4 : 1][4], wm2[M2 ? 4 : 1][4], wn2[M2 ? 4 : 1][4], wo[4][O];
#pragma unroll
  for (int fb = 0; fb < 4; ++fb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = 16 * fb + 4 * q + r;
      wmf[fb][r] = th[off.wmsg + k * 64 + 16 * w + c];
      if constexpr (TWO) wnf[fb][r] = th[off.wnode + k * 64 + 16 * w + c];
      if constexpr (M2) {
        wm2[fb][r] = th[off.wmsg + (64 + k) * 64 + 16 * w + c];
        wn2[fb][r] = th[off.wnode + (64 + k) * 64 + 16 * w + c];
      }
    }
  // GAT1 attention vector at this lane's output features 16 w + 4 q + r (sender / receiver half)
  float at1[4], at2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    at1[r] = L == DDRL_GNN_GAT1 ? th[off.wnode + 16 * w + 4 * q + r] : 0.f;
    at2[r] = L == DDRL_GNN_GAT1 ? th[off.wnode + 64 + 16 * w + 4 * q + r] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 0; o < O; ++o) wo[r][o] = th[off.wout + (16 * w + 4 * q + r) * O + o];

#ifdef DDRL_GNN_STAMPS
  wait_vmcnt0();   // diagnostic build: the weight / record loads have landed
  GSTAMP(10);
#endif
  // ---- hypernetwork + per-node encoding (partial over this wave's feature rows) ----
  floatx4 hacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) hacc[t] = splat4(0.f);
#pragma unroll
  for (int k = 0; k < GNI; ++k) {
#ifdef DDRL_ABL_GNN_NO_HFWD
    break;
#endif
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const floatx4 pre = mfma4(we[k][t], qv, be[k][t]);
#pragma unroll
      for (int r = 0; r < 4; ++r) hacc[t][r] = fmaf(fi[k], tanh_fast(pre[r]), hacc[t][r]);
    }
  }
  float* part = lds + L_PART;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[w * 1024 + (4 * t + r) * 64 + lane] = hacc[t][r];
  __syncthreads();
  GSTAMP(1);
  float* himg = lds + L_H;
  {
    // wave w finalizes feature block t = w: h = tanh(sum of the four partials, fixed order)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = (4 * w + r) * 64 + lane;
      const float s = ((part[o] + part[1024 + o]) + part[2048 + o]) + part[3072 + o];
      himg[wbase(r) + 16 * w] = tanh_fast(s);
    }
  }
  __syncthreads();
  float h[4][4];
#pragma unroll
  for (int fb = 0; fb < 4; ++fb)
#pragma unroll
    for (int r = 0; r < 4; ++r) h[fb][r] = himg[wbase(r) + 16 * fb];
#if DDRL_GNN_HW
  // this wave's own block h[w] (the backward's dtanh): read here, not indexed out of h[][] with
  // the wave index later (a select chain over every block, ~340 instructions)
  float hw[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) hw[r] = himg[wbase(r) + 16 * w];
#endif
  GSTAMP(2);

  // ---- message-passing layer: output block w of y (lane: node c, features 16 w + 4 q + r) ----
  float y[4];
  float* mimg = lds + L_M;
  float* ga_s = lds + L_GA;
  // GAT1 state kept for the backward: z (block w), attention of this node as sender to its
  // prev / self / next receivers, the per-node score halves and softmax denominators
  floatx4 zf = splat4(0.f);
  float gp = 0.f, gu = 0.f, aSp = 0.f, aSs = 0.f, aSn = 0.f;
  if constexpr (L == DDRL_GNN_MPNN) {
    floatx4 msg = splat4(0.f), nod = splat4(0.f);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        msg = mfma4(wmf[fb][r], h[fb][r], msg);
        nod = mfma4(wnf[fb][r], h[fb][r], nod);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float m = 0.5f * (quad_next(msg[r]) + quad_prev(msg[r]));
      y[r] = tanh_fast(nod[r] + m);
    }
  } else if constexpr (L == DDRL_GNN_GCN) {
    floatx4 msg = splat4(0.f);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) msg = mfma4(wmf[fb][r], h[fb][r], msg);
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = tanh_fast(0.5f * (quad_next(msg[r]) + quad_prev(msg[r])));
  } else if constexpr (L == DDRL_GNN_MPNN2) {
    floatx4 ma = splat4(0.f), mb = splat4(0.f), nod = splat4(0.f);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ma = mfma4(wmf[fb][r], h[fb][r], ma);
        mb = mfma4(wm2[fb][r], h[fb][r], mb);
        nod = mfma4(wnf[fb][r], h[fb][r], nod);
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) mimg[wbase(r) + 16 * w] = 0.5f * (quad_next(ma[r]) + quad_prev(ma[r])) + mb[r];
    __syncthreads();
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) nod = mfma4(wn2[fb][r], mimg[wbase(r) + 16 * fb], nod);
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = tanh_fast(nod[r]);
  } else {   // GAT1
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) zf = mfma4(wmf[fb][r], h[fb][r], zf);
    float pp = 0.f, uu = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) { pp = fmaf(zf[r], at1[r], pp); uu = fmaf(zf[r], at2[r], uu); }
    pp = qsum(pp);
    uu = qsum(uu);
    if (q == 0) { ga_s[(w * 16 + c) * 4] = pp; ga_s[(w * 16 + c) * 4 + 1] = uu; }
    __syncthreads();
    gp = ((ga_s[c * 4] + ga_s[(16 + c) * 4]) + ga_s[(32 + c) * 4]) + ga_s[(48 + c) * 4];
    gu = ((ga_s[c * 4 + 1] + ga_s[(16 + c) * 4 + 1]) + ga_s[(32 + c) * 4 + 1]) + ga_s[(48 + c) * 4 + 1];
    const float up = quad_prev(gu), un = quad_next(gu), pp_ = quad_prev(gp), pn = quad_next(gp);
    // denominator of this node as receiver: its senders n - 1, n, n + 1
    const float S = (__expf(leaky02(pp_ + gu)) + __expf(leaky02(gp + gu))) + __expf(leaky02(pn + gu));
    aSp = __expf(leaky02(gp + up)) / quad_prev(S);
    aSs = __expf(leaky02(gp + gu)) / S;
    aSn = __expf(leaky02(gp + un)) / quad_next(S);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      y[r] = tanh_fast(aSp * quad_prev(zf[r]) + aSs * zf[r] + aSn * quad_next(zf[r]));
  }
  GSTAMP(3);
  // ---- head: partial dot over this wave's 16 features, then across waves ----
  float* hp = lds + L_HP;
#pragma unroll
  for (int o = 0; o < O; ++o) {
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc = fmaf(y[r], wo[r][o], acc);
    acc = qsum(acc);
    if (q == 0) hp[(w * 16 + c) * 4 + o] = acc;
  }
  __syncthreads();

  if constexpr (MODE == GNN_ACT) {
    if (tid < 16) {
      const int cc = tid, gg = cc >> 2, nn = cc & 3, el = 4 * tile + gg, e = ga.act_e0 + el;
      if (el < ga.n_graphs) {
        float out[O];
#pragma unroll
        for (int o = 0; o < O; ++o)
          out[o] = (((hp[cc * 4 + o] + hp[(16 + cc) * 4 + o]) + hp[(32 + cc) * 4 + o]) +
                    hp[(48 + cc) * 4 + o]) + th[off.bout + o];
        const int C = 4 * ga.act_nfull;
        const int row = e * 4 + nn;
        if (NET == 1) {
          if (ga.bootstrap) ga.last_v[row] = out[0];
          else ga.rec[((size_t)ga.t * C + row) * ga.lay.stride + ga.lay.vf] = out[0];
        } else {
          float* rp = ga.rec + ((size_t)ga.t * C + row) * ga.lay.stride;
          float logp = -0.5f * (float)(DDRL_LOG2PI * A);
#pragma unroll
          for (int j = 0; j < A; ++j) {
            const float mu = out[j], ls = out[A + j];
            const float sd = expf(ls);
            const float a = mu + sd * ga.eps[((size_t)e * ga.n_agents + nn) * A + j];
            const float z = (a - mu) / sd;
            logp -= 0.5f * z * z;
            logp -= ls;
            rp[ga.lay.act + j] = a;
            ga.actions[(size_t)e * 8 + ga.act_index[nn][j]] = fminf(fmaxf(a, -1.f), 1.f);
          }
#pragma unroll
          for (int o = 0; o < O; ++o) rp[ga.lay.logit + o] = out[o];
          rp[ga.lay.logp] = logp;
        }
      }
    }
    if (NET == 0 && !ga.bootstrap) {
      // graph observation + node index into the 16 records of the tile
      const int C = 4 * ga.act_nfull;
      for (int idx = tid; idx < 16 * 93; idx += 256) {
        const int rr = idx / 93, f = idx - rr * 93, el = 4 * tile + (rr >> 2), e = ga.act_e0 + el;
        if (el >= ga.n_graphs) continue;
        const float v = f < 92 ? ga.x[(size_t)e * 92 + f] : (float)(rr & 3);
        ga.rec[((size_t)ga.t * C + e * 4 + (rr & 3)) * ga.lay.stride + ga.lay.obs + f] = v;
      }
    }
    return;
  }
  if constexpr (MODE == GNN_FWD) {
    if (tid < 16) {
      const int cc = tid, gg = cc >> 2, nn = cc & 3, r = 4 * tile + gg;
      if (r < ga.n_graphs && nn == ga.node[r]) {
#pragma unroll
        for (int o = 0; o < O; ++o) {
          const float v = (((hp[cc * 4 + o] + hp[(16 + cc) * 4 + o]) + hp[(32 + cc) * 4 + o]) +
                           hp[(48 + cc) * 4 + o]) + th[off.bout + o];
          if (NET == 0) ga.logits[(size_t)r * O + o] = v;
          else ga.values[r] = v;
        }
      }
    }
    return;
  }

  // ===================== GNN_GRAD: loss + backward + partial gradients ==================
  const UpdateArgs& U = ga.u;
  const UpdateHyper& H = ga.h;
  const bool coh = ga.tail;    // one-launch step: partials read by this launch's reducers (pst)
  float* dsh = lds + L_DOUT;   // [4 graphs][4]
  float* sts = lds + L_ST;     // [4 graphs][8]
  if (tid < 16) {
    const int cc = tid, gg = cc >> 2, nn = cc & 3;
    if (nn == sel) {
      const bool ok = gvalid;
      float out[O], dout[O], st[5];
#pragma unroll
      for (int o = 0; o < O; ++o)
        out[o] = (((hp[cc * 4 + o] + hp[(16 + cc) * 4 + o]) + hp[(32 + cc) * 4 + o]) +
                  hp[(48 + cc) * 4 + o]) + th[off.bout + o];
      if constexpr (NET == 0) {
        float act[A], ol[2 * A];
#pragma unroll
        for (int j = 0; j < A; ++j) act[j] = pre[j];
#pragma unroll
        for (int j = 0; j < 2 * A; ++j) ol[j] = pre[A + j];
        const float adv = (pre[3 * A + 1] - adv_m) / adv_d;
        policy_loss_row<A>(out, act, ol, pre[3 * A], adv, U.kl_coeff, 1.f - H.clip, 1.f + H.clip,
                           H.ent_coeff, ga.inv_n, ok, dout, st);
        st[3] = st[4] = 0.f;
      } else {
        value_loss_row(out[0], pre[0], pre[1], H, ga.inv_n, ok, dout, st);
      }
#pragma unroll
      for (int o = 0; o < O; ++o) dsh[gg * 4 + o] = dout[o];
#pragma unroll
      for (int k = 0; k < 5; ++k) sts[gg * 8 + k] = st[k];
    }
  }
  __syncthreads();
  GSTAMP(4);
  // per-tile statistics partial (fixed order over the 4 graphs); zs: backward share of this
  // workgroup (0 .. GNN_Z - 1)
  if (tid < 5 && zs == 0) {
    float s = 0.f;
    for (int gg = 0; gg < 4; ++gg) s += (4 * tile + gg < ga.n_graphs) ? sts[gg * 8 + tid] : 0.f;
    ga.statp[(NET * (DDRL_MB / 4) + tile) * 8 + tid] = s;
  }
  float* P = ga.part + (size_t)tile * ga.part_stride;
#ifdef DDRL_ABL_GNN_FWD_HANDOFF
  // Timing-only cost model (results wrong): one forward per tile shared by
  // its GNN_Z backward shares through the XCD's L2.  Share 0 publishes 16 KB (the size of a net's
  // dz / h / du / dm images for a tile) and a tagged flag in the padding of its partial row; the
  // other shares wait for the flag and read the 16 KB back.  Every share still runs its own
  // forward above: the forward is on the step's critical path either way (the shares wait for
  // share 0's), so this build adds exactly the hand-off.  The payload lands in partial slots that
  // the real partial stores overwrite later.
  if (ga.tail) {
    unsigned* hf = reinterpret_cast<unsigned*>(P + ga.n_params + NET);
    if (zs == 0) {
      for (int i = tid; i < 4096; i += 256) P[i] = lds[i];
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (tid == 0) __hip_atomic_store(hf, ga.tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (tid == 0) {
        const unsigned long long h0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(hf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ga.tag) {
          if (__builtin_amdgcn_s_memrealtime() - h0 > 300000000ull) {
            __hip_atomic_store(ga.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      float acc = 0.f;
      for (int i = tid; i < 4096; i += 256)
        acc += __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(P + i), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT));
      if (acc == 1.2345e-30f) lds[L_ST + 40] = acc;   // keeps the loads
      __syncthreads();
    }
  }
#endif
  const bool is_sel = n == sel;
  float ds[O];
#pragma unroll
  for (int o = 0; o < O; ++o) ds[o] = is_sel ? dsh[g * 4 + o] : 0.f;
  // dWout / dbout
  if (zs != 0) {
  } else if constexpr (O == 4) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 0; o < 4; ++o) v[4 * r + o] = y[r] * ds[o];
    const float s = row16_transpose_sum(v);
    pst(coh, P + off.wout + (16 * w + 4 * q + (c >> 2)) * 4 + (c & 3), s);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = row16_sum(y[r] * ds[0]);
      if (c == 0) pst(coh, P + off.wout + (16 * w + 4 * q + r) * O, v);
    }
  }
  if (tid < O && zs == 0) {
    float s = 0.f;
    for (int gg = 0; gg < 4; ++gg) s += dsh[gg * 4 + tid] * (4 * tile + gg < ga.n_graphs ? 1.f : 0.f);
    pst(coh, P + off.bout + tid, s);
  }
  // dy -> du = dy (1 - y^2): gradient at the layer's pre-activation (lane: node c, block w)
  float du[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float dy = 0.f;
#pragma unroll
    for (int o = 0; o < O; ++o) dy = fmaf(ds[o], wo[r][o], dy);
    du[r] = dy * (1.f - y[r] * y[r]);
  }
  float* duimg = lds + L_DU;
  float* dmimg = lds + L_DM;
  float* dmrimg = lds + L_DMR;
  // A operands of the transposed products: W[16 w + c][16 fb + 4 q + r] of a [64 + 64][64] block
  auto wt = [&](int base, int row0, float (*a)[4]) {
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(th + base + (row0 + 16 * w + c) * 64 + 16 * fb + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) a[fb][r] = v[r];
    }
  };
  // dh (block w) = sum over (W, image) of W . image^T
  auto acc_t = [&](floatx4& acc, float (*a)[4], const float* img) {
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = mfma4(a[fb][r], img[wbase(r) + 16 * fb], acc);
  };
  floatx4 dh = splat4(0.f);
  // weight-gradient tiles of the layer: (A image, B image, parameter base) per matrix
  const float* tA[4];
  const float* tB[4];
  int tP[4];
  if constexpr (L == DDRL_GNN_MPNN) {
    float dm[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) dm[r] = 0.5f * (quad_next(du[r]) + quad_prev(du[r]));
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      duimg[wbase(r) + 16 * w] = du[r];
      dmimg[wbase(r) + 16 * w] = dm[r];
    }
    float wnb[4][4], wmb[4][4];
    wt(off.wnode, 0, wnb);
    wt(off.wmsg, 0, wmb);
    __syncthreads();
    acc_t(dh, wnb, duimg);   // dh = Wnode . du^T + Wmsg . dm^T
    acc_t(dh, wmb, dmimg);
    tA[0] = himg; tB[0] = duimg; tP[0] = off.wnode;
    tA[1] = himg; tB[1] = dmimg; tP[1] = off.wmsg;
  } else if constexpr (L == DDRL_GNN_GCN) {
    // dW = ring(h)^T du = h^T ring(du) (ring symmetric);  dh = W . ring(du)^T
#pragma unroll
    for (int r = 0; r < 4; ++r) dmimg[wbase(r) + 16 * w] = 0.5f * (quad_next(du[r]) + quad_prev(du[r]));
    float wmb[4][4];
    wt(off.wmsg, 0, wmb);
    __syncthreads();
    acc_t(dh, wmb, dmimg);
    tA[0] = himg; tB[0] = dmimg; tP[0] = off.wmsg;
  } else if constexpr (L == DDRL_GNN_MPNN2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) duimg[wbase(r) + 16 * w] = du[r];
    float wa[4][4], wb2[4][4];
    wt(off.wnode, 64, wb2);   // node_update rows 64-127 (the message half)
    wt(off.wnode, 0, wa);     // node_update rows 0-63 (the node's own features)
    __syncthreads();
    floatx4 dm = splat4(0.f);
    acc_t(dm, wb2, duimg);    // dm = Wnode[64:] . du^T
    acc_t(dh, wa, duimg);     // dh = Wnode[:64] . du^T + ...
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dmimg[wbase(r) + 16 * w] = dm[r];
      dmrimg[wbase(r) + 16 * w] = 0.5f * (quad_next(dm[r]) + quad_prev(dm[r]));
    }
    wt(off.wmsg, 0, wa);      // msg_transform rows 0-63 (sender half)
    wt(off.wmsg, 64, wb2);    // msg_transform rows 64-127 (receiver half)
    __syncthreads();
    acc_t(dh, wa, dmrimg);    // ... + Wmsg[:64] . ring(dm)^T + Wmsg[64:] . dm^T
    acc_t(dh, wb2, dmimg);
    tA[0] = himg; tB[0] = duimg; tP[0] = off.wnode;
    tA[1] = mimg; tB[1] = duimg; tP[1] = off.wnode + 4096;
    tA[2] = himg; tB[2] = dmrimg; tP[2] = off.wmsg;
    tA[3] = himg; tB[3] = dmimg; tP[3] = off.wmsg + 4096;
  } else {   // GAT1
    // d alpha_sr = dv_s . z_r for r = prev / self / next (partial over this lane's 4 features)
    float dap = 0.f, das = 0.f, dan = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dap = fmaf(du[r], quad_prev(zf[r]), dap);
      das = fmaf(du[r], zf[r], das);
      dan = fmaf(du[r], quad_next(zf[r]), dan);
    }
    dap = qsum(dap); das = qsum(das); dan = qsum(dan);
    if (q == 0) {
      ga_s[(w * 16 + c) * 4] = dap;
      ga_s[(w * 16 + c) * 4 + 1] = das;
      ga_s[(w * 16 + c) * 4 + 2] = dan;
    }
    __syncthreads();
    auto wsum = [&](int k) {
      return ((ga_s[c * 4 + k] + ga_s[(16 + c) * 4 + k]) + ga_s[(32 + c) * 4 + k]) + ga_s[(48 + c) * 4 + k];
    };
    dap = wsum(0); das = wsum(1); dan = wsum(2);
    // softmax over the senders of each receiver r: sum_s alpha_sr d alpha_sr, at lane r
    const float col = (quad_prev(aSn * dan) + aSs * das) + quad_next(aSp * dap);
    const float up = quad_prev(gu), un = quad_next(gu);
    const float dp_ = aSp * (dap - quad_prev(col)) * (gp + up > 0.f ? 1.f : 0.2f);
    const float ds_ = aSs * (das - col) * (gp + gu > 0.f ? 1.f : 0.2f);
    const float dn_ = aSn * (dan - quad_next(col)) * (gp + un > 0.f ? 1.f : 0.2f);
    const float dps = (dp_ + ds_) + dn_;                                   // d(z_s . a[:64])
    const float dur = (quad_prev(dn_) + ds_) + quad_next(dp_);            // d(z_r . a[64:])
    float dz[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // attention-weighted part: z_r receives alpha_sr dv_s from its senders s = r - 1, r, r + 1
      const float dzz = (quad_prev(aSn) * quad_prev(du[r]) + aSs * du[r]) + quad_next(aSp) * quad_next(du[r]);
      dz[r] = dzz + dps * at1[r] + dur * at2[r];
    }
    // d a[:64] = sum over nodes of dps z, d a[64:] = sum of dur z (this tile's 16 nodes)
    if (zs == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a1 = row16_sum(dps * zf[r]);
        const float a2 = row16_sum(dur * zf[r]);
        if (c == 0) {
          pst(coh, P + off.wnode + 16 * w + 4 * q + r, a1);
          pst(coh, P + off.wnode + 64 + 16 * w + 4 * q + r, a2);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) dmimg[wbase(r) + 16 * w] = dz[r];
    float wpb[4][4];
    wt(off.wmsg, 0, wpb);
    __syncthreads();
    acc_t(dh, wpb, dmimg);   // dh = Wp . dz^T
    tA[0] = himg; tB[0] = dmimg; tP[0] = off.wmsg;
  }
  GSTAMP(5);
  // the hypernet partials are consumed: reuse PART for the dz exchange [block][r][lane]
#pragma unroll
#if DDRL_GNN_HW
  for (int r = 0; r < 4; ++r) part[(4 * w + r) * 64 + lane] = dh[r] * (1.f - hw[r] * hw[r]);
#else
  for (int r = 0; r < 4; ++r) part[(4 * w + r) * 64 + lane] = dh[r] * (1.f - h[w][r] * h[w][r]);
#endif
  // layer weight gradients: 16 tiles of 16x16 per matrix over the 16 rows, 4 per wave and
  // matrix; tile slot k of this wave belongs to this workgroup's share (gnn_tile_owner)
  // (slot k of wave w: tile id w + 4 k -> matrix k / 4, row block k % 4, column block w)
  constexpr int NKT = 4 * gnn_layer_mats(L);
#pragma unroll
  for (int k = 0; k < NKT; ++k) {
    if (gnn_tile_owner(k) != zs) continue;
    const int mat = k >> 2, kb = k & 3, ob = w;
    const floatx4 t = dw_tile<16>(tA[mat], tB[mat], kb, ob);
    const int base = tP[mat] + 16 * ob + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) pst(coh, P + base + (16 * kb + 4 * q + r) * 64, t[r]);
  }
  GSTAMP(6);
  __syncthreads();
  GSTAMP(7);
  float dz[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) dz[t][r] = part[(4 * t + r) * 64 + lane];
#ifdef DDRL_ABL_GNN_NO_HBWD   // ablation build (timing only)
  return;
#endif
  // hypernet backward: recompute W_n column blocks, dpre = f_i dz (1 - W^2); then
  //   [dWenc | dbenc] (block j, qd) = sum over the 16 rows of dpre[row][j] [q_row | 1][qd]
  // as 4 MFMAs per block: dpre goes through a per-wave LDS tile to put rows on the k axis,
  // B = the rows' quaternions with a ones column (bias) at qd = 4.
  // (wave 0's lane (c, q) holds component q of node c's quaternion since the start: qv; a
  // reload from the record here put one memory latency before this barrier on every step)
  float* qt = lds + L_QT;
  if (w == 0) qt[c * 4 + q] = qv;
  __syncthreads();
  float qb[4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) qb[s4] = c < 4 ? qt[(4 * s4 + q) * 4 + c] : (c == 4 ? 1.f : 0.f);
  GSTAMP(8);
  // Software-pipelined over the feature rows i of this wave: the dpre tiles of row k + 1 are
  // computed (MFMA, tanh: VALU) and stored to the other half of a double-buffered LDS tile
  // while the 16 weight-gradient MFMAs of row k run on operands already in registers.
  float* tpb = lds + L_TP + 2048 * w;   // [2][4 column blocks][16 x 16]
  auto dpre_tiles = [&](int k, float* tp) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const floatx4 pre = mfma4(we[k][t], qv, be[k][t]);
      floatx4 dp;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float wn = tanh_fast(pre[r]);
        dp[r] = fi[k] * dz[t][r] * (1.f - wn * wn);
      }
      *reinterpret_cast<floatx4*>(tp + 256 * t + tp_w(c, q)) = dp;   // [row c][j 4q + r]
    }
  };
  constexpr int NK = (GF + 3) / 4;   // feature rows of wave 0 (waves 1..3 have NK or NK - 1)
  static_assert(NK == GNI, "feature rows per wave");
  if constexpr (GNN_Z > 1) {
    // this workgroup's (row k, column block t) pairs (gnn_hbwd_owner), not pipelined
#pragma unroll
    for (int k = 0; k < GNI; ++k) {
      const int i = w + 4 * k;
      bool any = false;
#pragma unroll
      for (int t = 0; t < 4; ++t) any = any || gnn_hbwd_owner(k, t) == zs;
      if (!any || i >= GF) continue;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (gnn_hbwd_owner(k, t) != zs) continue;
        const floatx4 pre = mfma4(we[k][t], qv, be[k][t]);
        floatx4 dp;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float wn = tanh_fast(pre[r]);
          dp[r] = fi[k] * dz[t][r] * (1.f - wn * wn);
        }
        *reinterpret_cast<floatx4*>(tpb + 256 * t + tp_w(c, q)) = dp;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (gnn_hbwd_owner(k, t) != zs) continue;
        floatx4 acc = splat4(0.f);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = mfma4(tpb[256 * t + tp_r(4 * s4 + q, c)], qb[s4], acc);
        const int j = i * 64 + 16 * t + 4 * q;
        if (c < 4) pst4(coh, P + off.wenc + c * GHE + j, acc);
        else if (c == 4) pst4(coh, P + off.benc + j, acc);
      }
    }
    GSTAMP(9);
    return;
  }
  dpre_tiles(0, tpb);
#pragma unroll
  for (int k = 0; k < GNI; ++k) {
    const int i = w + 4 * k;
    if (i >= GF) break;
    const float* tp = tpb + 1024 * (k & 1);
    float a[4][4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int t = 0; t < 4; ++t) a[s4][t] = tp[256 * t + tp_r(4 * s4 + q, c)];
    if (k + 1 < GNI && i + 4 < GF) dpre_tiles(k + 1, tpb + 1024 * ((k + 1) & 1));
    floatx4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = splat4(0.f);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma4(a[s4][t], qb[s4], acc[t]);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int j = i * 64 + 16 * t + 4 * q;                  // acc[r]: column j + r, qd = c
      if (c < 4) pst4(coh, P + off.wenc + c * GHE + j, acc[t]);
      else if (c == 4) pst4(coh, P + off.benc + j, acc[t]);
    }
  }
}

__device__ __forceinline__ void gnn_tail(const GnnArgs& ga, float* lds, int tile, int net, int zs);   // below

template <int A, int MODE, int L>
__global__ void __launch_bounds__(256) k_gnn(GnnArgs ga) {
  __shared__ float lds[L_TOTAL];
  // the one-launch step's 1-D grid groups the workgroups by (net, share) combination k = b mod 8:
  // blocks b = k mod 8 are dealt to one XCD, so a combination's 32 tiles share an L2 (gnn_tail)
  int tile, net, zs;
  if (MODE == GNN_GRAD && ga.xgrid) {
    const int b = blockIdx.x;
    if (ga.xgrid == 2) {   // test hook (DDRL_TEST_GNN_MISPLACE): combination k = b / 32 straddles every XCD
      tile = b & 31; net = (b >> 7) & 1; zs = (b >> 5) & 3;
    } else {
      tile = b >> 3; net = (b >> 2) & 1; zs = b & 3;
    }
  } else {
    tile = blockIdx.x; net = blockIdx.y; zs = blockIdx.z;
  }
  const int blk = blockIdx.x + gridDim.x * (blockIdx.y + 2 * blockIdx.z);
  if (MODE == GNN_GRAD) SPAN(0, blk, 0);
  if (net == 0) gnn_tile<A, MODE, 0, L>(ga, lds, tile, zs);
  else gnn_tile<A, MODE, 1, L>(ga, lds, tile, zs);
  if (MODE == GNN_GRAD) SPAN(0, blk, 1);
  (void)blk;
  if constexpr (MODE == GNN_GRAD)
    if (ga.tail) gnn_tail(ga, lds, tile, net, zs);
}
// k_gnn instance of a layer (MODE fixed)
#define GNN_LAUNCH(MODE, L_, grid, s, ga)                                                            \
  do {                                                                                              \
    switch (L_) {                                                                                   \
      case DDRL_GNN_GCN: hipLaunchKernelGGL((k_gnn<2, MODE, DDRL_GNN_GCN>), grid, dim3(256), 0, s, ga); break;     \
      case DDRL_GNN_MPNN2: hipLaunchKernelGGL((k_gnn<2, MODE, DDRL_GNN_MPNN2>), grid, dim3(256), 0, s, ga); break; \
      case DDRL_GNN_GAT1: hipLaunchKernelGGL((k_gnn<2, MODE, DDRL_GNN_GAT1>), grid, dim3(256), 0, s, ga); break;   \
      default: hipLaunchKernelGGL((k_gnn<2, MODE, DDRL_GNN_MPNN>), grid, dim3(256), 0, s, ga); break;              \
    }                                                                                               \
  } while (0)

// ---- reduction over tiles: grad[p] = sum_t part[t][p] (fixed order) + norm^2 partials ----
// loss statistics of the step: statp [net][tile][8]; lane j < 10 sums (net, stat) j over the
// tiles (independent loads), lane 0 combines
__device__ __forceinline__ void gnn_step_stats(const GnnArgs& ga, int ntiles) {
  __shared__ float sv[10];
  const int j = threadIdx.x, b = j / 5, k = j - 5 * b;
  float sv_t[DDRL_MB / 4];
#pragma unroll
  for (int t = 0; t < DDRL_MB / 4; ++t) sv_t[t] = t < ntiles ? ga.statp[(b * DDRL_MB / 4 + t) * 8 + k] : 0.f;
  float a = 0.f;
#pragma unroll
  for (int t = 0; t < DDRL_MB / 4; ++t) a += sv_t[t];
  sv[j] = a;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const UpdateArgs& U = ga.u;
  if (j == 0) {
    ga.bp_cur[0] = U.beta_pow[0];
    ga.bp_cur[1] = U.beta_pow[1];
    if (U.stats) {
      const float nr = (float)ga.n_graphs;
      float* so = U.stats + (size_t)ga.step * 8;
      so[1] = sv[0] / nr; so[3] = sv[1] / nr; so[4] = sv[2] / nr;
      so[2] = sv[5] / nr;
      const float vy = sv[7] / nr - (sv[6] / nr) * (sv[6] / nr);
      const float vd = sv[9] / nr - (sv[8] / nr) * (sv[8] / nr);
      so[5] = vy > 0.f ? fmaxf(-1.f, 1.f - vd / vy) : 0.f;
    }
  }
}

// ---- reduction over tiles: grad[p] = sum_t part[t][p] (fixed order) + norm^2 partials ----
// Reduction block b (256 parameters): this thread's summed gradient (parameter b * 256 + tid) is
// returned; the block's squared-norm partial goes to normp[b].
__device__ __forceinline__ float gnn_reduce_block(const GnnArgs& ga, int b, int ntiles, int n, bool store_grad) {
  __shared__ float red[4];
  const int p = b * 256 + threadIdx.x;
  // all tile partials of this parameter in flight at once (a runtime-bound loop would wait
  // for each load before the next add), then summed in tile order
  float v[DDRL_MB / 4];
#pragma unroll
  for (int t = 0; t < DDRL_MB / 4; ++t)
    v[t] = (p < n && t < ntiles) ? ga.part[(size_t)t * ga.part_stride + p] : 0.f;
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < DDRL_MB / 4; ++t) s += v[t];
  if (store_grad && p < n) ga.grad[p] = s;
  float ss = wave_sum(s * s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) ga.normp[b] = ((red[0] + red[1]) + red[2]) + red[3];
  return p < n ? s : 0.f;
}

// ---- tf.clip_by_global_norm + tf1 Adam on the 256 parameters of block b ----
// g0, mi, vi, th0: this thread's gradient and state (loaded by the caller, ahead of the norm it
// waits on); b1p, b2p: the step's beta powers.
__device__ __forceinline__ void gnn_adam_block(const GnnArgs& ga, int b, int nred, int n, float g0, float mi,
                                               float vi, float th0, float b1p, float b2p) {
  __shared__ float scale_s;
  const UpdateArgs& U = ga.u;
  const UpdateHyper& h = ga.h;
  const int p = b * 256 + threadIdx.x;
  const bool pv = p < n;
  if (threadIdx.x < 64) {
    // squared-norm partials of the reduction blocks: the same butterfly in every block
    float part = 0.f;
    for (int k = threadIdx.x; k < nred; k += 64) part += ga.normp[k];
    const float tot = wave_sum(part);
    if (threadIdx.x != 0) goto done;
    const float gn = sqrtf(tot);
    scale_s = h.grad_clip * fminf(1.f / gn, 1.f / h.grad_clip);
    if (b == 0) {
      if (U.stats) {
        U.stats[(size_t)ga.step * 8 + 6] = gn;
        U.stats[(size_t)ga.step * 8 + 7] = scale_s;
      }
      U.beta_pow[0] = b1p * h.b1;
      U.beta_pow[1] = b2p * h.b2;
    }
  }
done:
  __syncthreads();
  if (!pv) return;
  const float alpha = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float g = g0 * scale_s;
  mi = mi + (g - mi) * (1.f - h.b1);
  vi = vi + (g * g - vi) * (1.f - h.b2);
  U.m[p] = mi;
  U.v[p] = vi;
  U.theta[p] = th0 - (mi * alpha) / (sqrtf(vi) + h.eps);
}

// Three-launch step: the last block of the reduction grid (one past the parameter blocks) sums
// the step's loss statistics instead, in parallel with the parameter blocks.
__global__ void __launch_bounds__(256) k_gnn_reduce(GnnArgs ga, int ntiles, int n) {
  RSTAMPB(blockIdx.x, 0);
  SPAN(1, blockIdx.x, 0);
  if (blockIdx.x == gridDim.x - 1) {
    if (threadIdx.x < 10) gnn_step_stats(ga, ntiles);
    SPAN(1, blockIdx.x, 1);
    return;
  }
  (void)gnn_reduce_block(ga, blockIdx.x, ntiles, n, true);
  RSTAMPB(blockIdx.x, 1);
  SPAN(1, blockIdx.x, 1);
}

__global__ void __launch_bounds__(256) k_gnn_adam(GnnArgs ga, int nred, int n) {
  RSTAMPB(blockIdx.x, 2);
  SPAN(2, blockIdx.x, 0);
  const UpdateArgs& U = ga.u;
  // this thread's parameter state first: its loads do not depend on the clip scale and
  // overlap the squared-norm reduction
  const int p = blockIdx.x * 256 + threadIdx.x;
  const bool pv = p < n;
  const float g0 = pv ? ga.grad[p] : 0.f;
  const float mi = pv ? U.m[p] : 0.f, vi = pv ? U.v[p] : 0.f;
  const float th0 = pv ? U.theta[p] : 0.f;
  gnn_adam_block(ga, blockIdx.x, nred, n, g0, mi, vi, th0, ga.bp_cur[0], ga.bp_cur[1]);
  RSTAMPB(blockIdx.x, 3);
  SPAN(2, blockIdx.x, 1);
}

// ---- one-launch step: the reduction and Adam run in the gradient launch's tail ----
// The reduction needs every tile's partials and Adam the global norm, so the step used to be
// three launches (two kernel boundaries of ~1.5-2 us each, MI355X_MICROARCH.md "boundary").
// The one-launch step keeps the reduction inside an XCD: the gradient grid is 1-D, block
// b = 8 tile + k with k = 4 net + share, so the 32 tiles of one (net, backward share)
// combination k are blocks b = k mod 8, which the dispatcher deals to one XCD (the fcnet row
// split relies on the same rule, with its placement check).  Every parameter's partials come
// from one share (the owner lists plist, found once per context by gnn_build_owner_lists), so a
// combination's partials are all written -- plain stores into the XCD's L2 -- and read on one
// XCD:
//   * each workgroup, once its partials and loss statistics are in L2 (s_waitcnt), raises its
//     arrival flag (flags[32 k + tile] = this launch's tag and the workgroup's XCC id) and
//     records its XCC for the host's placement check;
//   * tiles r < R_k of combination k are also its reduction blocks: reducer r waits for the 32
//     flags of its combination (one per thread, sc1 polls: they miss the CU's own L1; a flag of
//     this launch from another XCD raises the error word, gnn_wait_flag), sums
//     the 32 partials of 256 owned parameters in tile order with sc1 loads (the three-launch
//     reduction's order, so the gradient is bit-identical) and publishes its norm^2 partial as
//     a tagged granule {value, tag} with a device-scope atomic store (the one value that crosses
//     XCDs);
//   * every reducer waits for all granules, forms the global norm in one fixed order and runs
//     clip + tf1 Adam on its 256 parameters; global reducer 0 writes the norm statistics and the
//     next beta powers (read by every reducer before its granule goes up);
//   * tile R_k of combination (net, 0) sums that net's loss statistics.
// Waits are bounded (the error word, as the fcnet exchanges; the host restores its snapshot and
// the context goes on with three launches).  Measured first with device-wide protocols instead:
// every partial written through to memory + one arrival counter 22.7 us per step (256 arrivals
// on one device-scope atomic serialize, MI355X_MICROARCH.md "fanin"), flags 21.5, release /
// acquire 33.1, against 18.9 for three launches.
// Placement guard: a flag carries its writer's XCC id (HW_REG_XCC_ID)
// below the tag, and a reducer accepts a flag of this launch only from its own XCD.  A flag of
// this launch from another XCD means the combination straddles XCDs, so its partials may still
// sit in the other XCD's L2: the reducer raises the error word instead of summing them (the host
// restores its snapshot and the context goes on with three launches).  A flag that stays in the
// other XCD's L2 is never seen, and the wait ends at its bound the same way.  So no stale partial
// is ever summed, whatever the flag's scope.  The flags are plain (workgroup-scope) stores into
// the XCD's L2: agent scope (written through, seen across XCDs at once) cost 0.2 us per step at C5
// (17.76 vs 17.55 us, profiles/r05/gnn_flag_scope_ab.txt); -DDDRL_GNN_FLAG_AGENT=1 builds it.
#ifndef DDRL_GNN_FLAG_AGENT
#define DDRL_GNN_FLAG_AGENT 0
#endif
// arrival flag of tile t of combination k: the 32 flags of one combination in one 128-B line,
// which a reducer's 32 polling lanes read with one request (measured against the flags spread
// over 8 lines, 4 each: 17.65 / 17.66 vs 17.70 / 17.78 us per step at C5, the same box,
// profiles/r05/gnn_flag_scope_ab.txt)
#ifndef DDRL_GNN_FLAG_PACKED
#define DDRL_GNN_FLAG_PACKED 1
#endif
__device__ __forceinline__ int gnn_flag_idx(int k, int t) { return DDRL_GNN_FLAG_PACKED ? 32 * k + t : 8 * t + k; }
__device__ __forceinline__ unsigned gnn_xcc() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xfu;
}
__device__ __forceinline__ bool gnn_wait_flag(const GnnArgs& ga, const unsigned* flag, unsigned xcc,
                                              unsigned long long t0) {
  for (;;) {
    const unsigned f = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((f >> 4) == ga.tag) {
      if ((f & 0xfu) == xcc) return true;
      __hip_atomic_store(ga.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // misplaced combination
      return false;
    }
    const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
    if ((dt > 20000ull && __hip_atomic_load(ga.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) || dt > 300000000ull) {
      __hip_atomic_store(ga.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ bool gnn_wait_gran(const GnnArgs& ga, const unsigned long long* g, unsigned long long t0,
                                              float& out) {
  for (;;) {
    const unsigned long long v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(v >> 32) == ga.tag) {
      out = __uint_as_float((unsigned)v);
      return true;
    }
    const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
    if ((dt > 20000ull && __hip_atomic_load(ga.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) || dt > 300000000ull) {
      __hip_atomic_store(ga.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ float sc1_ld(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ void gnn_tail(const GnnArgs& ga, float* lds, int tile, int net, int zs) {
  const int k = 4 * net + zs, tid = threadIdx.x;   // combination (net, share)
  const unsigned xcc = gnn_xcc();
  // LDS of the finished tile, reused: [0..3] norm^2 of the waves, [4..5] beta powers,
  // [8..12] loss statistics, [16] clip scale, [17] ok, [64 ..] granule values
  float* T = lds;
  __builtin_amdgcn_s_waitcnt(0);   // this wave's partial / statistics stores are in L2
  __syncthreads();
  // arrival flag of tile `tile` of combination k: this launch's tag and this workgroup's XCC;
  // the placement record for the host check (capi.cpp gnn_placement_broken)
  if (tid == 0) {
    __hip_atomic_store(ga.flags + gnn_flag_idx(k, tile), (ga.tag << 4) | xcc, __ATOMIC_RELAXED,
                       DDRL_GNN_FLAG_AGENT ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_WORKGROUP);
    ga.xcc[32 * k + tile] = (int)xcc;
  }
  const int m = ga.poff[k + 1] - ga.poff[k];
  const int r = tile;   // reducer r of combination k: parameters plist[poff[k] + 256 r ..]
  const int R = (m + 255) / 256;
  const UpdateArgs& U = ga.u;
  // the first tile after the reducers of combination (net, 0) sums that net's loss statistics
  // (the three-launch order), off the reducers' path
  const bool stats = zs == 0 && r == R && U.stats;
  if (r > R || (r == R && !stats)) return;
  const bool adam = U.grad_out == nullptr;
  // this thread's parameter and its state (the loads overlap the flag wait)
  const int e = 256 * r + tid;
  const bool pv = !stats && e < m;
  const int p = pv ? ga.plist[ga.poff[k] + e] : 0;
  const float mi = pv && adam ? U.m[p] : 0.f, vi = pv && adam ? U.v[p] : 0.f;
  const float th0 = pv && adam ? U.theta[p] : 0.f;
  if (tid == 0 && adam && !stats) {
    T[4] = U.beta_pow[0];
    T[5] = U.beta_pow[1];
  }
  // the combination's 32 workgroups have arrived (one flag per thread)
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const bool ok = tid >= ga.ntiles || gnn_wait_flag(ga, ga.flags + gnn_flag_idx(k, tid), xcc, t0);
  if (!__syncthreads_and(ok)) return;
  if (stats) {
    if (tid < 5) {   // all 32 loads in flight (all 32 tiles on this path), then summed in tile order
      float sv[DDRL_MB / 4];
#pragma unroll
      for (int t = 0; t < DDRL_MB / 4; ++t) sv[t] = sc1_ld(ga.statp + (net * (DDRL_MB / 4) + t) * 8 + tid);
      float a = 0.f;
#pragma unroll
      for (int t = 0; t < DDRL_MB / 4; ++t) a += sv[t];
      T[8 + tid] = a;
    }
    __syncthreads();
    if (tid == 0) {
      const float nr = (float)ga.n_graphs;
      float* so = U.stats + (size_t)ga.step * 8;
      if (net == 0) {
        so[1] = T[8] / nr; so[3] = T[9] / nr; so[4] = T[10] / nr;
      } else {
        so[2] = T[8] / nr;
        const float vy = T[10] / nr - (T[9] / nr) * (T[9] / nr);
        const float vd = T[12] / nr - (T[11] / nr) * (T[11] / nr);
        so[5] = vy > 0.f ? fmaxf(-1.f, 1.f - vd / vy) : 0.f;
      }
    }
    return;
  }
  RSTAMPB(ga.rbase[k] + r, 0);
  SPAN(1, ga.rbase[k] + r, 0);
  // the reduction: 32 partials of this thread's parameter (this path runs only with all 32
  // tiles), in tile order.  The loads are unconditional -- a lane without a parameter reads
  // parameter 0's and drops the sum -- so all 32 go out back to back: under a per-load
  // condition the compiler branched around each one and waited for the first before the rest
  float v[DDRL_MB / 4];
  const float* pp = ga.part + (pv ? p : 0);
#pragma unroll
  for (int t = 0; t < DDRL_MB / 4; ++t) v[t] = sc1_ld(pp + (size_t)t * ga.part_stride);
  float g0 = 0.f;
#pragma unroll
  for (int t = 0; t < DDRL_MB / 4; ++t) g0 += v[t];
  if (!pv) g0 = 0.f;
  if (!adam) {   // data-parallel gradient: the all-reduce and Adam follow as launches
    if (pv) ga.grad[p] = g0;
    return;
  }
  const float ss = wave_sum(g0 * g0);
  if ((tid & 63) == 0) T[tid >> 6] = ss;
  __syncthreads();
  const int gi = ga.rbase[k] + r;   // global reducer index
  if (tid == 0) {
    __builtin_amdgcn_s_waitcnt(0);   // the beta powers above have landed before the granule goes up
    const float np = ((T[0] + T[1]) + T[2]) + T[3];
    __hip_atomic_store(ga.gran + gi, ((unsigned long long)ga.tag << 32) | __float_as_uint(np), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  RSTAMPB(gi, 1);
  SPAN(1, gi, 1);
  // every reducer's norm^2 partial (one granule per thread), then the norm in a fixed order
  const int nr_all = ga.rbase[8];
  float gv = 0.f;
#ifdef DDRL_ABL_GNN_LOCAL_NORM
  // timing-only cost model (results wrong): the norm from this XCD's own
  // reducers only -- no granule crosses an XCD
  const bool ok2 = tid < ga.rbase[k] || tid >= ga.rbase[k + 1] || gnn_wait_gran(ga, ga.gran + tid, t0, gv);
#else
  const bool ok2 = tid >= nr_all || gnn_wait_gran(ga, ga.gran + tid, t0, gv);
#endif
  T[64 + tid] = gv;
  if (!__syncthreads_and(ok2)) return;
  RSTAMPB(gi, 2);
  SPAN(2, gi, 0);
  const UpdateHyper& h = ga.h;
  const float b1p = T[4], b2p = T[5];
  if (tid < 64) {
    float part = 0.f;
    for (int j = tid; j < nr_all; j += 64) part += T[64 + j];
    const float tot = wave_sum(part);
    if (tid == 0) {
      const float gn = sqrtf(tot);
      const float scale = h.grad_clip * fminf(1.f / gn, 1.f / h.grad_clip);
      T[16] = scale;
      if (gi == 0) {
        if (U.stats) {
          U.stats[(size_t)ga.step * 8 + 6] = gn;
          U.stats[(size_t)ga.step * 8 + 7] = scale;
        }
        U.beta_pow[0] = b1p * h.b1;
        U.beta_pow[1] = b2p * h.b2;
      }
    }
  }
  __syncthreads();
  if (pv) {
    const float alpha = h.lr * sqrtf(1.f - b2p) / (1.f - b1p);
    const float g = g0 * T[16];
    const float m1 = mi + (g - mi) * (1.f - h.b1);
    const float v1 = vi + (g * g - vi) * (1.f - h.b2);
    U.m[p] = m1;
    U.v[p] = v1;
    U.theta[p] = th0 - (m1 * alpha) / (sqrtf(v1) + h.eps);
  }
  RSTAMPB(gi, 3);
  SPAN(2, gi, 1);
}

// Pre-gather of a run of minibatch steps: dst[k][i][col] = rec[shuffle[perm[e][b] * 128 + i]][col]
// for step0 + k = e * nb + b.  One float per thread (the row index loads hit L2 / MALL: 128
// rows share one perm entry, 'stride' floats share one row index).
__global__ void k_gnn_gather(UpdateArgs u, int step0, size_t n, float* dst) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n) return;
  const int stride = u.lay.stride;
  const size_t rowg = gid / stride;
  const int col = (int)(gid - rowg * stride);
  const int k = (int)(rowg / DDRL_MB), i = (int)(rowg - (size_t)k * DDRL_MB);
  const int s = step0 + k, e = s / u.nb, b = s - e * u.nb;
  const int row = u.shuffle[(size_t)u.perm[e * u.nb + b] * DDRL_MB + i];
  dst[gid] = u.rec[(size_t)row * stride + col];
}

void launch_gnn_gather(hipStream_t s, const UpdateArgs& u, int step0, int n_steps, float* dst) {
  const size_t n = (size_t)n_steps * DDRL_MB * u.lay.stride;
  hipLaunchKernelGGL(k_gnn_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, u, step0, n, dst);
}

int gnn_param_total(int A, int layer) { return gnn_net_off(A, 1, layer).bout + 1; }

static void check_a(int A) {
  if (A != 2) {
    fprintf(stderr, "ddrl: gnn kernels are built for act_dim 2 (got %d)\n", A);
    abort();
  }
}

void launch_act_gnn(hipStream_t s, const RouteArgs& ra, const ActArgs& aa, int layer) {
  check_a(ra.A);
  GnnArgs ga{};
  ga.theta = aa.theta[0];
  ga.n_graphs = aa.e1 - aa.e0;   // the env range [e0, e1) of this call
  ga.act_e0 = aa.e0;
  ga.act_nfull = ra.N;
  ga.x = aa.stage[0];
  ga.rec = aa.rec[0]; ga.lay = aa.lay[0]; ga.t = aa.t; ga.eps = aa.eps; ga.actions = aa.actions;
  ga.n_agents = ra.n_agents; ga.bootstrap = aa.bootstrap; ga.last_v = aa.last_v[0];
  for (int a = 0; a < 4; ++a)
    for (int j = 0; j < 8; ++j) ga.act_index[a][j] = ra.pol[0].act_index[a][j];
  GNN_LAUNCH(GNN_ACT, layer, dim3((ga.n_graphs + 3) / 4, 2), s, ga);
}

void launch_forward_gnn(hipStream_t s, const ForwardArgs& fa, int layer) {
  check_a(fa.A);
  GnnArgs ga{};
  ga.theta = fa.theta; ga.n_graphs = fa.n; ga.x = fa.x; ga.node = fa.node;
  ga.logits = fa.logits; ga.values = fa.values;
  GNN_LAUNCH(GNN_FWD, layer, dim3((fa.n + 3) / 4, 2), s, ga);
}

static GnnArgs grad_args(const UpdateArgs& u, const UpdateHyper& h, int step, int nrows, float inv_n,
                         const GnnScratch& sc, const float* stage, int layer) {
  GnnArgs ga{};
  ga.theta = u.theta; ga.u = u; ga.h = h; ga.step = step; ga.n_graphs = nrows; ga.inv_n = inv_n;
#ifdef DDRL_ABL_GNN_THETA_RO
  // timing-only cost model (results wrong): the tiles read their weights
  // from a buffer no launch writes (the records), as if theta stayed in the reading XCD's L2
  ga.theta = u.rec;
#endif
  ga.part = sc.part; ga.part_stride = sc.part_stride; ga.statp = sc.statp; ga.normp = sc.normp;
  ga.bp_cur = sc.bp_cur; ga.grad = u.grad_out ? u.grad_out : sc.grad;
  ga.stage = stage;
  ga.ntiles = (nrows + 3) / 4;
  ga.n_params = gnn_param_total(u.A, layer);
  ga.nred = (ga.n_params + 255) / 256;
  ga.err = sc.err; ga.flags = sc.flags; ga.gran = sc.gran;
  ga.only_share = -1;
  return ga;
}

// Owner lists of the one-launch step: which backward share writes each parameter's partials
// (the gradient kernel's own store pattern -- gnn_tile_owner, gnn_hbwd_owner, share 0 for the
// head and attention vectors -- observed, not restated): one gradient launch per share with the
// other shares idle, over a partial row pre-filled with a NaN pattern no computed value has.
// Every parameter must be owned by exactly one share, and each (net, share) combination's list
// must fit the reducers its 32 tiles provide; otherwise the context keeps three launches.
// The one-launch step's waits need every workgroup of the 256-block grid resident at once, with
// a combination's 32 workgroups on one XCD: at least 32 blocks per XCD must fit.
static bool gnn_tail_resident(int layer) {
  const void* f = nullptr;
  switch (layer) {
    case DDRL_GNN_GCN: f = reinterpret_cast<const void*>(&k_gnn<2, GNN_GRAD, DDRL_GNN_GCN>); break;
    case DDRL_GNN_MPNN2: f = reinterpret_cast<const void*>(&k_gnn<2, GNN_GRAD, DDRL_GNN_MPNN2>); break;
    case DDRL_GNN_GAT1: f = reinterpret_cast<const void*>(&k_gnn<2, GNN_GRAD, DDRL_GNN_GAT1>); break;
    default: f = reinterpret_cast<const void*>(&k_gnn<2, GNN_GRAD, DDRL_GNN_MPNN>); break;
  }
  int dev = 0, per_cu = 0;
  hipDeviceProp_t pr;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&pr, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 256, 0) != hipSuccess)
    return false;
  return per_cu >= 1 && per_cu * (pr.multiProcessorCount / 8) >= DDRL_MB / 4 && per_cu * pr.multiProcessorCount >= 256;
}

static void gnn_build_owner_lists(hipStream_t s, const UpdateArgs& u, const UpdateHyper& h, float inv_n,
                                  GnnScratch& sc, int layer) {
  sc.lists = -1;
  if (!gnn_tail_resident(layer)) return;
  GnnArgs ga = grad_args(u, h, 0, 4, inv_n, sc, nullptr, layer);
  const int n = ga.n_params;
  const int actor = gnn_net_off(u.A, 1, layer).wenc;   // first critic parameter
  std::vector<int> own(n, -1);
  std::vector<unsigned> row(n);
  for (int z = 0; z < GNN_Z; ++z) {
    if (hipMemsetD32Async((hipDeviceptr_t)sc.part, 0xFFFFFFFFu, (size_t)n, s) != hipSuccess) return;
    ga.only_share = z;
    GNN_LAUNCH(GNN_GRAD, layer, dim3(1, 2, GNN_Z), s, ga);
    if (hipMemcpyAsync(row.data(), sc.part, (size_t)n * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return;
    for (int p = 0; p < n; ++p) {
      if (row[p] == 0xFFFFFFFFu) continue;
      if (own[p] >= 0) return;   // two shares write one parameter
      own[p] = z;
    }
  }
  std::vector<int> lst;
  int poff[9], rbase[9];
  poff[0] = rbase[0] = 0;
  for (int k = 0; k < 8; ++k) {
    const int net = k >> 2, z = k & 3;
    for (int p = 0; p < n; ++p) {
      if (own[p] < 0) return;   // a parameter no share writes
      if ((p >= actor) == (net == 1) && own[p] == z) lst.push_back(p);
    }
    poff[k + 1] = (int)lst.size();
    const int R = (poff[k + 1] - poff[k] + 255) / 256;
    if (R >= DDRL_MB / 4) return;   // the reducers and the statistics tile need R + 1 <= 32 tiles
    rbase[k + 1] = rbase[k] + R;
  }
  if ((int)lst.size() != n || rbase[8] > 256) return;
  if (hipMemcpy(sc.plist, lst.data(), (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) return;
  for (int k = 0; k < 9; ++k) sc.poff[k] = poff[k], sc.rbase[k] = rbase[k];
  sc.lists = 1;
}

void launch_step_gnn(hipStream_t s, const UpdateArgs& u, const UpdateHyper& h, int step, int nrows, float inv_n,
                     GnnScratch& sc, const float* stage, int layer) {
  check_a(u.A);
  GnnArgs ga = grad_args(u, h, step, nrows, inv_n, sc, stage, layer);
  const int ntiles = ga.ntiles, n = ga.n_params, nred = ga.nred;
  // one launch per step for full 128-row minibatches (32 tiles per combination)
  if (sc.tail && sc.lists == 0 && ntiles == DDRL_MB / 4 && GNN_Z == 4) gnn_build_owner_lists(s, u, h, inv_n, sc, layer);
  ga.tail = sc.tail && sc.lists == 1 && ntiles == DDRL_MB / 4 && GNN_Z == 4;
  if (ga.tail) {
    sc.seq = (sc.seq + 1) & 0x0FFFFFFFu;   // 28-bit tags (the flags hold tag << 4 | XCC id)
    if (sc.seq == 0) sc.seq = 1;           // tags never 0 (the buffers start zeroed)
    ga.tag = sc.seq;
    ga.xgrid = sc.misplace ? 2 : 1;
    ga.xcc = sc.xcc;
    sc.xcc_pending = 1;
    ga.plist = sc.plist;
    for (int k = 0; k < 9; ++k) ga.poff[k] = sc.poff[k], ga.rbase[k] = sc.rbase[k];
    GNN_LAUNCH(GNN_GRAD, layer, dim3(ntiles * 8), s, ga);
    return;
  }
  // tiles of the critic write their statistics after the actor's: statp [2][32][8]
  GNN_LAUNCH(GNN_GRAD, layer, dim3(ntiles, 2, GNN_Z), s, ga);
#ifdef DDRL_ABL_GNN_GRAD_ONLY   // ablation build (timing only): no reduction / Adam launches
  return;
#endif
  hipLaunchKernelGGL(k_gnn_reduce, dim3(nred + 1), dim3(256), 0, s, ga, ntiles, n);
  if (!u.grad_out) hipLaunchKernelGGL(k_gnn_adam, dim3(nred), dim3(256), 0, s, ga, nred, n);
}
