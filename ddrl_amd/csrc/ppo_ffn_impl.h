// Fused PPO update kernel for the fcnet model: see ppo_ffn.hip for the design notes.
#pragma once
#include <atomic>
#include "common.h"
#include "kernels.h"
#include "ffn.h"
#include "ppo_loss.h"

// One translation unit per exchange protocol: ppo_ffn.hip builds the default (plain stores into
// the XCD's L2, sc1 polls) as launch_update_ffn, ppo_ffn_atomic.hip the relaxed system-scope
// atomic protocol (valid for any workgroup placement) as launch_update_ffn_atomic, and
// ppo_ffn_peer.hip (DDRL_FFN_AT = 2) peer mode's launch_update_ffn_peer: the LSB-tagged quads of
// the default protocol moved with system-scope buffer accesses (sc0 sc1: written through to
// memory, read past every cache), whose outboxes a peer context's launch shares.  The device
// code has internal linkage, so the instantiations of every kernel never meet at link time.
#ifndef DDRL_FFN_AT
#define DDRL_FFN_AT 0
#endif

// Kernel instances of this TU: 0 all; 2 only the fused row-split kernels (KSP = 2 with the LSB
// quads: ppo_ffn.hip, built with its own scheduling flags; every other launch goes to
// launch_update_ffn_k1); 1 the rest -- KSP = 1 and the gradient-export launches (ppo_ffn_k1.hip,
// default flags: the KSP = 1 kernels spill more under ppo_ffn.hip's)
#ifndef DDRL_FFN_KSP
#define DDRL_FFN_KSP 0
#endif
#if DDRL_FFN_KSP == 1
#define DDRL_FFN_LAUNCH launch_update_ffn_k1
#elif DDRL_FFN_AT == 2
#define DDRL_FFN_LAUNCH launch_update_ffn_peer
#elif DDRL_FFN_AT
#define DDRL_FFN_LAUNCH launch_update_ffn_atomic
#else
#define DDRL_FFN_LAUNCH launch_update_ffn
#endif
#if DDRL_FFN_AT || defined(DDRL_XCHG_ATOMIC)
#define DDRL_XCHG_IS_ATOMIC 1
#else
#define DDRL_XCHG_IS_ATOMIC 0
#endif
// Adam's small-parameter slots past nsb aimed at a sink word instead of masked (A/B: -DDDRL_SINK=0)
#ifndef DDRL_SINK
#define DDRL_SINK 1
#endif
// Per-lane predicates "feature < d" out of the step loop (the inputs of features >= d zeroed
// instead; -DDDRL_PADZERO=0: the predicates, for A/B)
#ifndef DDRL_PADZERO
#define DDRL_PADZERO 1
#endif
// LSB-tagged quads for fused launches (round 4; -DDDRL_LX=0: the {value, tag} pairs everywhere)
#ifndef DDRL_LX
#define DDRL_LX 1
#endif
// the peer TU: atomic granules for the norm exchange and the gradient launches' pairs, quads at
// system scope for the fused launches' partner exchange
#define DDRL_XCHG_LXSYS (DDRL_FFN_AT == 2)
// where the row split issues the next step's record gathers: 0 = behind the partner exchange's
// first poll (vmcnt retires in order), 1 = right after sync #1 (round 6 A/B)
#ifndef DDRL_GATHER_EARLY
#define DDRL_GATHER_EARLY 0
#endif
// DDRL_ABL_PEER4: the timing-only cost model of a four-rank peer mode, in the
// peer TU only: the weight-gradient K of a 32-row share and two more partners' quad reads at
// system scope (the four-way split model of DESIGN.md section 6.2 on the peer protocol)
#if defined(DDRL_ABL_PEER4) && DDRL_FFN_AT == 2
#define DDRL_ABL_HALF_DW
#define DDRL_ABL_XCHG3
#endif
#define DDRL_LX_ON (!DDRL_XCHG_IS_ATOMIC || DDRL_XCHG_LXSYS)

namespace {

// Workgroup geometry: NW waves (8 = two per SIMD with one 16-row tile each; the A = 8
// kernels use 4 waves with two tiles each, their per-wave head partials would not fit LDS).
// Row split (KSP = 2): each branch runs on two workgroups that take 64 rows of the minibatch
// each (one 16-row tile per wave, four waves) and swap their partial gradients every step
// through tagged 8-byte granules; both then hold the same summed gradient and run the same
// clip + Adam, so their weight images stay bit-identical.
typedef float float2v __attribute__((ext_vector_type(2)));

template <int NW, int ROWS>
struct Geo {
  static constexpr int NT = 64 * NW;
  static constexpr int RT = ROWS / (16 * NW);      // 16-row tiles per wave
  static constexpr int NS1 = 16 / NW;              // dW2 tile slots per wave (16 tiles)
  static constexpr int NS2 = (12 + NW - 1) / NW;   // dW1 tile slots per wave (<= 12 tiles)
};
__host__ __device__ constexpr int waves_for(int A, int ksp) { return ksp == 2 ? 4 : (A == 8 ? 4 : 8); }
// value pairs per lane of the partner exchange: small params + stats (padded to a pair),
// then two per owned dW tile
// coupling-table slots ("cup" model, models/coupling_net_glorot_uniform_init.py:11-30) among a
// branch's small parameters: policy branch of the A = 2 kernels
__host__ __device__ constexpr int ncup_slots(int OB, bool pol) { return pol && OB == 4 ? 2 * OB : 0; }
__host__ __device__ constexpr int gx_pairs(int OB, int NW) {
  return ((64 * OB + OB + 128 + ncup_slots(OB, true) + 64 * NW - 1) / (64 * NW) + 2) / 2 + 2 * (16 / NW + (12 + NW - 1) / NW);
}
#define GX_MAX_PAIRS 20

struct UpdateBatch {
  UpdateArgs a[DDRL_MAXP];   // one entry per policy, by value in the kernel argument block
  UpdateHyper h;
  int nrows;             // rows per minibatch handled here (<= 128)
  float inv_n;           // 1 / sgd_minibatch_size (global minibatch)
  unsigned long long* xchg;  // [P][2 branches][KSP][2 parities] tagged norm^2 granules
  unsigned long long* gx;    // [P][2 branches][KSP][2 parities][GX_MAX_PAIRS][256 lanes][2] partial-gradient granules
  int* err;              // set to 1 if an exchange timed out
  int* xcc;              // [grid] XCC id of every block (placement check, capi.cpp)
  unsigned epoch;        // launch counter (12 bits, never 0): high bits of every exchange tag
  unsigned lds_bytes;    // dynamic LDS of the launch (bounds-checked build)
  // -1: every row half runs here.  0 / 1 (peer mode, ddrl_ppo_update_peer): only that half runs
  // in this launch -- the other half is the peer context's launch, which exchanges through the
  // shared outboxes in gx -- and it writes the weights back and the statistics
  int own_kq;
  // peer mode: steps the attached pair has run before this launch.  The quads' tag bit and the
  // outbox parity follow the pair's global step count, so the shared outboxes need no clear
  // between launches (0 otherwise: the outboxes are cleared before each fused launch)
  unsigned lx_base;
};

// Bounds-checked diagnostic build (-DDDRL_BOUNDS, tools/build_diag.py): every staging,
// record, schedule and LDS index the update kernel derives at run time is checked against its
// buffer before use; a violation counts into g_bounds[k] and the access is clamped into range
// (never faults).  k: 0 staging row of a gathered chunk, 1 record row index >= R, 2 schedule
// index (perm / shuffle) out of range, 3 LDS-DMA destination past the launch's LDS, 4 staged
// record read past the staging rows, 5 parameter index past n_params.
#ifdef DDRL_BOUNDS
__device__ unsigned g_bounds[DDRL_NBOUNDS];
__device__ __forceinline__ bool bchk(bool ok, int k) {
  if (!ok) atomicAdd(&g_bounds[k], 1u);
  return ok;
}
}  // namespace
#if !DDRL_FFN_AT
#if DDRL_FFN_KSP == 2
extern "C" int ddrl_diag_bounds_k1(unsigned* host, int reset);
#endif
#if DDRL_FFN_KSP == 1
extern "C" int ddrl_diag_bounds_k1(unsigned* host, int reset) {
#else
extern "C" int ddrl_diag_bounds(unsigned* host, int reset) {
#endif
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bounds), sizeof(g_bounds)) != hipSuccess) return -1;
  if (reset) {
    unsigned z[DDRL_NBOUNDS] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bounds), z, sizeof(z)) != hipSuccess) return -1;
  }
#if DDRL_FFN_KSP == 2   // the KSP = 1 kernels' counters (ppo_ffn_k1.hip) count too
  unsigned k1[DDRL_NBOUNDS];
  if (ddrl_diag_bounds_k1(k1, reset) != 0) return -1;
  for (int i = 0; i < DDRL_NBOUNDS; ++i) host[i] += k1[i];
#endif
  return 0;
}
#endif
namespace {
#define BCHK(cond, k) bchk((cond), (k))
#else
#define BCHK(cond, k) true
#endif
// Exchange tag of a step: the launch epoch above the step count, so a granule line some
// cache still holds from an earlier launch can never carry a tag of this one.
__device__ __forceinline__ unsigned xchg_tag(unsigned epoch, int step) {
  return (epoch << 20) | (((unsigned)step + 1u) & 0xfffffu);
}

// Per-branch view of the flat (Keras-order) parameter vector.
struct BranchOff { int w1, b1, w2, b2, wo, bo, cup; };
__device__ __forceinline__ BranchOff branch_off(const FfnOffsets& o, bool pol) {
  BranchOff b;
  b.cup = o.n;   // "cup" model: the leg-coupling table [4][A] follows the fcnet variables
  b.w1 = pol ? o.w1 : o.vw1; b.b1 = pol ? o.b1 : o.vb1;
  b.w2 = pol ? o.w2 : o.vw2; b.b2 = pol ? o.b2 : o.vb2;
  b.wo = pol ? o.wo : o.vo;  b.bo = pol ? o.bo : o.vbo;
  return b;
}

template <int OB, bool PAD>
__device__ void stage_branch(const float* __restrict__ th, int d, const BranchOff& bo, float* lds,
                             NetLds& W, int ncup) {
  W.w1 = lds; W.w2 = W.w1 + lds_img(48, PAD); W.b1 = W.w2 + lds_img(64, PAD); W.b2 = W.b1 + 64;
  W.wo = W.b2 + 64; W.bo = W.wo + 64 * OB; W.cup = W.bo + OB;   // cup: OB <= 4 (A = 2)
  for (int i = threadIdx.x; i < ncup; i += blockDim.x) W.cup[i] = th[bo.cup + i];
  for (int i = threadIdx.x; i < 48 * 64; i += blockDim.x) {
    const int f = i >> 6;
    W.w1[sidx<PAD>(f, i & 63)] = f < d ? th[bo.w1 + i] : 0.f;
  }
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) W.w2[sidx<PAD>(i >> 6, i & 63)] = th[bo.w2 + i];
  for (int i = threadIdx.x; i < 64; i += blockDim.x) { W.b1[i] = th[bo.b1 + i]; W.b2[i] = th[bo.b2 + i]; }
  for (int i = threadIdx.x; i < 64 * OB; i += blockDim.x) W.wo[i] = th[bo.wo + i];
  for (int i = threadIdx.x; i < OB; i += blockDim.x) W.bo[i] = th[bo.bo + i];
}
// The same image with every weight load of a thread issued before the first LDS store (one
// memory round trip instead of one per loop trip; NT = threads per workgroup, 256 or 512).
template <int OB, int NT, bool PAD>
__device__ __forceinline__ void stage_branch_batched(const float* __restrict__ th, int d, const BranchOff& bo,
                                                     float* lds, NetLds& W, int ncup) {
  static_assert((48 * 64) % NT == 0 && (64 * 64) % NT == 0, "staging split");
  constexpr int N1 = 48 * 64 / NT, N2 = 64 * 64 / NT, NS = (64 * OB + OB + 128 + NT - 1) / NT;
  W.w1 = lds; W.w2 = W.w1 + lds_img(48, PAD); W.b1 = W.w2 + lds_img(64, PAD); W.b2 = W.b1 + 64;
  W.wo = W.b2 + 64; W.bo = W.wo + 64 * OB; W.cup = W.bo + OB;
  const int t = threadIdx.x;
  float a1[N1], a2[N2], as[NS];
#pragma unroll
  for (int k = 0; k < N1; ++k) {
    const int i = t + NT * k;
    a1[k] = (i >> 6) < d ? th[bo.w1 + i] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < N2; ++k) a2[k] = th[bo.w2 + t + NT * k];
#pragma unroll
  for (int k = 0; k < NS; ++k) {   // [wo 64 OB][bo OB][b1 64][b2 64]
    int e = t + NT * k;
    float x = 0.f;
    if (e < 64 * OB) x = th[bo.wo + e];
    else if ((e -= 64 * OB) < OB) x = th[bo.bo + e];
    else if ((e -= OB) < 64) x = th[bo.b1 + e];
    else if ((e -= 64) < 64) x = th[bo.b2 + e];
    as[k] = x;
  }
  float ac = t < ncup ? th[bo.cup + t] : 0.f;   // ncup <= 8 < NT
#pragma unroll
  for (int k = 0; k < N1; ++k) {
    const int i = t + NT * k;
    W.w1[sidx<PAD>(i >> 6, i & 63)] = a1[k];
  }
#pragma unroll
  for (int k = 0; k < N2; ++k) {
    const int i = t + NT * k;
    W.w2[sidx<PAD>(i >> 6, i & 63)] = a2[k];
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    int e = t + NT * k;
    if (e < 64 * OB) W.wo[e] = as[k];
    else if ((e -= 64 * OB) < OB) W.bo[e] = as[k];
    else if ((e -= OB) < 64) W.b1[e] = as[k];
    else if ((e -= 64) < 64) W.b2[e] = as[k];
  }
  if (t < ncup) W.cup[t] = ac;
}
// LDS floats of one branch's weight image (a multiple of 4 floats)
__host__ __device__ constexpr int branch_lds_floats(bool pad) { return lds_img(48, pad) + lds_img(64, pad) + 128 + 64 * 16 + 16; }
// the swizzled image layout of an update kernel (common.h): the padded one, except for the A = 8
// kernel without the row split, whose LDS budget has room only for the compact images
__host__ __device__ constexpr bool update_pad(int A, int ksp) { return kLdsPad && !(A == 8 && ksp == 1); }

// "Small" parameters owned one per thread: [dWo 64*OB][dbo OB][db1 64][db2 64], then the
// policy branch's leg-coupling table [4][A] of the "cup" model
template <int OB>
__device__ __forceinline__ void small_param(int e, const BranchOff& bo, const NetLds& W, int& pidx, float*& lp) {
  if (e < 64 * OB) { pidx = bo.wo + e; lp = W.wo + e; return; }
  e -= 64 * OB;
  if (e < OB) { pidx = bo.bo + e; lp = W.bo + e; return; }
  e -= OB;
  if (e < 64) { pidx = bo.b1 + e; lp = W.b1 + e; return; }
  e -= 64;
  if (e < 64) { pidx = bo.b2 + e; lp = W.b2 + e; return; }
  e -= 64;
  pidx = bo.cup + e; lp = W.cup + e;
}


template <int A, int RT>
struct RowData {
  float x[RT][12];      // this wave's row tiles
  float act[RT][A];
  float ol[RT][2 * A];
  float s0[RT], s1[RT];  // policy: logp_old, adv;  value: vf_old, vt
  int cid[RT];           // "cup": coupling row of the record
};

// The next minibatch's 128 records are gathered by LDS-DMA into stg [128][stride] while the
// current step computes: 16-byte chunk g of the gather is record column 4 (g % cpr) of row
// g / cpr (cpr = stride / 4), and one wave-instruction writes 64 consecutive chunks (the
// lane-linear LDS destination of global_load_lds).  Whole 64-byte record lines instead of
// per-lane dword gathers: 3 line requests per row rather than one per field and lane.
// The staging rows hold cpr_l = cpr | 1 chunks (an odd number: the 16 rows a lane group
// reads then start in 16 different banks); the pad chunk repeats the row's last chunk.
// Issued by waves 0 .. NW-2: the last wave keeps its vector-memory counter free for the
// norm exchange (an early partner poll would otherwise wait for the gathers too).
template <int NW, int ROWS>
__device__ __forceinline__ void issue_rows(const float* rec, int stride, int cpr, int cpr_l, float inv_cpr_l,
                                           const int* idxb, float* stg, int R, unsigned lds_bytes) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
  if (w == NW - 1) return;
  // at most 20 chunks per record (fcnet records: d <= 48, A <= 8 -> stride <= 80 floats), so a
  // wave issues at most MI batches; every staged row index is read from LDS first (one
  // latency for all batches), then the gathers go out back to back
  constexpr int MI = (ROWS * 20 + 64 * (NW - 1) - 1) / (64 * (NW - 1));
  const int nchunk = ROWS * cpr_l;
  int idx[MI], kk[MI];
#pragma unroll
  for (int it = 0; it < MI; ++it) {
    const int g = 64 * w + 64 * (NW - 1) * it + lane;
    int row = (int)(((float)g + 0.5f) * inv_cpr_l);
    kk[it] = min(g - row * cpr_l, cpr - 1);
    idx[it] = 0;
    if (g < nchunk) {
      if (!BCHK(row >= 0 && row < ROWS && kk[it] >= 0, 0)) row = 0;
      idx[it] = idxb[row];
    }
  }
#pragma unroll
  for (int it = 0; it < MI; ++it) {
    const int base = 64 * w + 64 * (NW - 1) * it;          // wave-uniform
    if (base >= nchunk) break;
    const unsigned dst = __builtin_amdgcn_readfirstlane(lds_addr(stg + 4 * base));
    if (base + lane < nchunk) {
      int i = idx[it];
      if (!BCHK(i >= 0 && i < R, 1)) i = 0;
      if (BCHK(dst + 16u * (unsigned)lane + 16u <= lds_bytes, 3))
        glds16(rec + (size_t)i * stride + 4 * kk[it], dst);
    }
  }
  (void)R; (void)lds_bytes;
}

// staging-row chunks for a record of `stride` floats (the A = 8 kernels keep the plain
// stride: their LDS budget has no room for the pad)
__host__ __device__ constexpr int stg_chunks(int stride, int A) { return A == 8 ? stride / 4 : (stride / 4) | 1; }

// This lane's rows from the staged records (padding rows hold record 0; their output
// gradient is zeroed).  Observation columns f >= d are zero (they meet the zero rows of the
// W1 image; their dW1 rows are never stored): the generic KS1 = 12 instance (d of no exact
// instance, e.g. the LegID env's 23) would otherwise read past the record -- past the staging
// buffer for the last row, whatever that LDS holds -- and 0 x NaN is NaN.
template <int A, int KS1, bool POL, int RT>
__device__ __forceinline__ void load_row(const float* stg, int stg_stride, const RecLayout& L, const int* row_l,
                                         int d, RowData<A, RT>& r, unsigned xlast_bits = 0xffffffffu) {
  const int q = (threadIdx.x & 63) >> 4;
#ifdef DDRL_BOUNDS
  {
    // the widest column this lane group reads (the generic KS1 = 12 instance reads columns < d
    // only): it must lie inside the record, i.e. inside this row's staging slot
    int hi = KS1 < 12 ? L.obs + 4 * KS1 - 1 : L.obs + d - 1;
    if (POL) hi = max(max(hi, L.act + A - 1), max(L.logit + 2 * A - 1, max(L.logp, max(L.adv, L.cid))));
    else hi = max(hi, max(L.vf, L.vt));
    for (int t = 0; t < RT; ++t) BCHK(row_l[t] >= 0 && row_l[t] < DDRL_MB && hi < L.stride, 4);
  }
#endif
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    const float* rp = stg + row_l[t] * stg_stride;
#pragma unroll
    for (int s = 0; s < 12; ++s)   // exact instances (KS1 = ceil(d / 4)) stay inside the record
      r.x[t][s] = (s < KS1 && (KS1 < 12 || 4 * s + q < d)) ? rp[L.obs + 4 * s + q] : 0.f;
    // exact instances: the last k-step's features >= d (the record's next columns) -> 0 through
    // a per-lane bit mask (no lane predicate in the step loop), so the dW1 rows >= d are zero
    if (KS1 < 12) r.x[t][KS1 - 1] = __uint_as_float(__float_as_uint(r.x[t][KS1 - 1]) & xlast_bits);
    if (POL) {
#pragma unroll
      for (int j = 0; j < A; ++j) r.act[t][j] = rp[L.act + j];
#pragma unroll
      for (int j = 0; j < 2 * A; ++j) r.ol[t][j] = rp[L.logit + j];
      r.s0[t] = rp[L.logp];
      r.s1[t] = rp[L.adv];
      r.cid[t] = L.cid >= 0 ? min(max((int)rp[L.cid], 0), 3) : 0;
    } else {
      r.cid[t] = 0;
#pragma unroll
      for (int j = 0; j < A; ++j) r.act[t][j] = 0.f;
#pragma unroll
      for (int j = 0; j < 2 * A; ++j) r.ol[t][j] = 0.f;
      r.s0[t] = rp[L.vf];
      r.s1[t] = rp[L.vt];
    }
  }
}

// Per-step learner statistics from the per-wave partial sums red[w * 8 + k]: policy
// workgroup -> policy_loss, kl, entropy; value workgroup -> vf_loss, vf_explained_var.
// inv_n = 1 / rows: x * inv_n is x / n bit for bit when n is a power of two (128 and the
// data-parallel 128 / G), within an ulp otherwise (a caller-chosen ddrl_ppo_grad row count)
template <bool POL, int NSTAT, int NW, int KSP>
__device__ __forceinline__ void write_stats(float* so, const float* red, float inv_n) {
  float sv[NSTAT];
#pragma unroll
  for (int k = 0; k < NSTAT; ++k) {
    if constexpr (KSP == 2) {
      sv[k] = red[96 + k];   // both workgroups' sums, combined at the exchange
    } else {
      sv[k] = 0.f;
      for (int i = 0; i < NW; ++i) sv[k] += red[i * 8 + k];
    }
  }
  if constexpr (POL) {
    gst(so + 1, sv[0] * inv_n); gst(so + 3, sv[1] * inv_n); gst(so + 4, sv[2] * inv_n);
  } else {
    gst(so + 2, sv[0] * inv_n);
    const float vy = sv[2] * inv_n - (sv[1] * inv_n) * (sv[1] * inv_n);
    const float vd = sv[4] * inv_n - (sv[3] * inv_n) * (sv[3] * inv_n);
    gst(so + 5, vy > 0.f ? fmaxf(-1.f, 1.f - vd / vy) : 0.f);
  }
}

__device__ __forceinline__ int row_index(const UpdateArgs& U, int step, int row_l, bool ok) {
  if (!ok) return 0;
  if (!U.shuffle) return row_l;   // pre-gathered rows (data-parallel one-step launches)
  const int e = step / U.nb, b = step - e * U.nb;
#ifdef DDRL_BOUNDS
  if (!BCHK(e >= 0 && e < U.n_epochs, 2)) return 0;
  const int slot = gld(U.perm + e * U.nb + b);
  if (!BCHK(slot >= 0 && slot < U.nb && (slot + 1) * DDRL_MB <= max(U.R, DDRL_MB) && row_l < DDRL_MB, 2)) return 0;
  return gld(U.shuffle + slot * DDRL_MB + row_l);
#else
  return gld(U.shuffle + gld(U.perm + e * U.nb + b) * DDRL_MB + row_l);
#endif
}
// minibatch slot of a step (wave-uniform: perm[e][b])
__device__ __forceinline__ int perm_slot(const UpdateArgs& U, int step) {
  const int e = step / U.nb, b = step - e * U.nb;
  return gld(U.perm + e * U.nb + b);
}

// Diagnostic build only (-DDDRL_STAMPS): per-phase s_memtime cycle counts of wave 0 of each
// workgroup, accumulated over the steps of one launch; no stamp executes in the real build.
#ifdef DDRL_STAMPS
__device__ unsigned long long g_stamps[32][16];
#define STAMP_INIT unsigned long long st_prev = __builtin_amdgcn_s_memtime(), st_acc[16] = {0};
#ifndef DDRL_STAMP_TID   // the stamped thread (lane 0 of a wave): per-wave diagnostic builds
#define DDRL_STAMP_TID 0
#endif
#define STAMP(k) do { if (tid == DDRL_STAMP_TID) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[k] += t_ - st_prev; st_prev = t_; } } while (0)
#define STAMP_DONE do { if (tid == DDRL_STAMP_TID) for (int k_ = 0; k_ < 16; ++k_) g_stamps[blockIdx.x][k_] = st_acc[k_]; } while (0)
}  // namespace
#if !DDRL_FFN_AT && DDRL_FFN_KSP != 1
extern "C" int ddrl_diag_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) == hipSuccess ? 0 : -1;
}
#endif
namespace {
#else
#define STAMP_INIT
#define STAMP(k)
#define STAMP_DONE
#endif

// Partner exchange of the row split: 16-byte granules {value, tag, value, tag} (each 8-byte
// half carries the step tag, so a half is valid exactly when its tag matches: no fence),
// written by one sc1 (write-through) buffer store and read by one sc1 buffer load; the
// outboxes are double buffered by step parity and cleared before each launch.  Pair j of
// lane l sits at box[(j * 256 + l) * 16 bytes] (coalesced per pair).
// Cache policy of the exchange (gfx950 CPol bits: sc0 = 1, nt = 2, sc1 = 16).  The four
// workgroups of a policy share one XCD and hence one L2 (blocks b, b + 8, ... are dealt to
// XCD b mod 8; tools/xchg_bench.hip prints the placement).  Plain stores write through the
// per-CU L1 into that L2 and stay there; the poller's sc1 (device-scope) loads miss its own
// L1.  Measured one-hop latency (tools/xchg_bench.hip, MI355X): plain store / sc1 load
// 0.24 us, sc1 store / sc1 load 0.50 us (the sc1 store writes through to memory), sc0 loads
// never see the partner (they hit the stale L1 line).
#ifndef DDRL_GX_ST
#define DDRL_GX_ST 0
#endif
#ifndef DDRL_GX_LD
#define DDRL_GX_LD 16
#endif
#ifndef DDRL_GX_INV
#define DDRL_GX_INV 0
#endif
__device__ __forceinline__ void xchg_inv_l1() {
#if DDRL_GX_INV
  asm volatile("buffer_inv sc0" ::: "memory");
#endif
}
// Once any exchange has waited this long (100 MHz ticks), the waiter also polls the error
// word, so one timed-out exchange ends every later wait at once instead of each one
// spinning to its own timeout.
#define XCHG_SLOW_TICKS 20000ull        // 200 us
#define XCHG_TIMEOUT_TICKS 300000000ull // 3 s
__device__ __forceinline__ bool xchg_abandon(unsigned long long t0, int* err) {
  const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
  if (dt < XCHG_SLOW_TICKS) return false;
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return true;
  if (dt > XCHG_TIMEOUT_TICKS) { atomicExch(err, 1); return true; }
  return false;
}
// Two builds of the same protocol:
//  * default: plain stores into the XCD's shared L2 and sc1 polls (0.24 us per hop); correct
//    when the workgroups that exchange share an L2.  The dispatcher deals a grid's blocks to
//    the 8 XCDs round robin, from a start XCD that varies between dispatches (measured: a
//    data-parallel gradient launch found block p on XCD != p), so blocks b = p mod 8 -- the
//    workgroups of policy p -- always share one XCD.  Were that ever broken, a poll would
//    never see its partner: the 3 s bound raises the error word and the host names the
//    atomic build.  With coh set the stores are sc1 (device-coherent write-through: the ISA
//    of a relaxed agent-scope atomic store), 0.50 us per hop.
//  * -DDDRL_XCHG_ATOMIC: every granule access is a relaxed 64-bit atomic (__hip_atomic_load /
//    __hip_atomic_store; system scope since round 5, agent before): defined behaviour under the
//    HIP memory model for any placement, each 8-byte {value, tag} half its own atomic.  The bounds-checked
//    diagnostic library is built this way, so the GPU suite runs the update under both.
#if DDRL_XCHG_IS_ATOMIC
// System scope (round 5): the peer mode's outboxes live in fine-grained memory a peer GPU writes
// (ddrl_ppo_update_peer); on one device it orders like agent scope.
#define DDRL_XCHG_SCOPE __HIP_MEMORY_SCOPE_SYSTEM
typedef unsigned long long* gx_box_t;
__device__ __forceinline__ gx_box_t gx_rsrc(unsigned long long* box) { return box; }
__device__ __forceinline__ void gx_put(gx_box_t r, int j, float v0, float v1, unsigned tag, bool) {
  unsigned long long* g = r + 2 * (j * 256 + (int)threadIdx.x);
  __hip_atomic_store(g, ((unsigned long long)tag << 32) | __float_as_uint(v0), __ATOMIC_RELAXED, DDRL_XCHG_SCOPE);
  __hip_atomic_store(g + 1, ((unsigned long long)tag << 32) | __float_as_uint(v1), __ATOMIC_RELAXED,
                     DDRL_XCHG_SCOPE);
}
__device__ __forceinline__ void xchg_store(unsigned long long* g, unsigned long long v, bool) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, DDRL_XCHG_SCOPE);
}
__device__ __forceinline__ unsigned long long xchg_load(unsigned long long* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, DDRL_XCHG_SCOPE);
}
template <int NP, typename F>
__device__ __forceinline__ bool gx_get(gx_box_t r, unsigned tag, float* out, int* err, F&& after_first) {
  bool lost = false;
  unsigned long long g[2 * NP];
  unsigned long long* b = r + 2 * (int)threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool first = true;
  for (;;) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      g[2 * j] = __hip_atomic_load(b + 512 * j, __ATOMIC_RELAXED, DDRL_XCHG_SCOPE);
      g[2 * j + 1] = __hip_atomic_load(b + 512 * j + 1, __ATOMIC_RELAXED, DDRL_XCHG_SCOPE);
    }
    if (first) { after_first(); first = false; }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 2 * NP; ++j) ok = ok && (unsigned)(g[j] >> 32) == tag;
    if (ok) break;
    if (xchg_abandon(t0, err)) {
#pragma unroll
      for (int j = 0; j < 2 * NP; ++j) g[j] = 0ull;
      lost = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int j = 0; j < 2 * NP; ++j) out[j] = __uint_as_float((unsigned)g[j]);
  return lost;
}
#else
typedef __amdgpu_buffer_rsrc_t gx_box_t;
__device__ __forceinline__ gx_box_t gx_rsrc(unsigned long long* box) {
  return __builtin_amdgcn_make_buffer_rsrc(box, 0, GX_MAX_PAIRS * 256 * 16, 0x00020000);
}
__device__ __forceinline__ void gx_put(gx_box_t r, int j, float v0, float v1, unsigned tag, bool coh) {
  const v4u g = {__float_as_uint(v0), tag, __float_as_uint(v1), tag};
  if (coh) __builtin_amdgcn_raw_buffer_store_b128(g, r, (j * 256 + (int)threadIdx.x) * 16, 0, 16);
  else __builtin_amdgcn_raw_buffer_store_b128(g, r, (j * 256 + (int)threadIdx.x) * 16, 0, DDRL_GX_ST);
}
// Norm granule (8 bytes: tag << 32 | value), one 64-bit access each way, same policy.
__device__ __forceinline__ void xchg_store(unsigned long long* g, unsigned long long v, bool coh) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, 8, 0x00020000);
  typedef unsigned v2u_t __attribute__((ext_vector_type(2)));
  const v2u_t x = {(unsigned)v, (unsigned)(v >> 32)};
  if (coh) __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, 16);
  else __builtin_amdgcn_raw_buffer_store_b64(x, r, 0, 0, DDRL_GX_ST);
}
__device__ __forceinline__ unsigned long long xchg_load(unsigned long long* g) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(g, 0, 8, 0x00020000);
  typedef unsigned v2u_t __attribute__((ext_vector_type(2)));
  xchg_inv_l1();
  const v2u_t x = __builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, DDRL_GX_LD);
  return ((unsigned long long)x[1] << 32) | x[0];
}
// The partner's NP pairs of this lane: all loads in flight, re-polled until every tag
// matches; bounded (a timeout flags err and returns zeros).
template <int NP, typename F>
__device__ __forceinline__ bool gx_get(gx_box_t r, unsigned tag, float* out, int* err, F&& after_first) {
  bool lost = false;
  v4u g[NP];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool first = true;
  for (;;) {
    xchg_inv_l1();
#pragma unroll
    for (int j = 0; j < NP; ++j) g[j] = __builtin_amdgcn_raw_buffer_load_b128(r, (j * 256 + (int)threadIdx.x) * 16, 0, DDRL_GX_LD);
    if (first) { after_first(); first = false; }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NP; ++j) ok = ok && g[j][1] == tag && g[j][3] == tag;
    if (ok) break;
    if (xchg_abandon(t0, err)) {
#pragma unroll
      for (int j = 0; j < NP; ++j) g[j] = v4u{0u, 0u, 0u, 0u};
      lost = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    out[2 * j] = __uint_as_float(g[j][0]);
    out[2 * j + 1] = __uint_as_float(g[j][2]);
  }
  return lost;
}
#endif

// Fused-update exchange with the tag in the values themselves (LX, round 4): four values per
// 16-byte granule, each carrying a 1-bit step tag in its mantissa LSB, so the exchanged bytes
// halve against {value, tag, value, tag}.  A value is valid exactly when its LSB is the step's
// tag bit: every 4-byte value is its own single-copy-atomic unit, no 16-byte atomicity is
// assumed.  The bit toggles between the two uses of an outbox (outboxes alternate by step
// parity, the bit is (step >> 1) & 1, inverted), so a value from two steps back carries the other
// bit; one from four steps back cannot reappear, because this lane read the location's
// two-steps-back value and a location's value only moves forward.  The outboxes are cleared
// before every fused launch (zero words fail the first two steps' bit 1).  Both workgroups of a
// branch add the same two LSB-replaced partials, so their sums stay bit-identical; the
// replaced bit is < 1 ulp of each partial.  Data-parallel gradient launches (one step per
// launch) keep the epoch-tagged pairs, which need no clear per launch.
__device__ __forceinline__ unsigned lx_bit(int step) { return ((unsigned)(step >> 1) & 1u) ^ 1u; }
__device__ __forceinline__ float lx_t(float v, unsigned bit) { return __uint_as_float((__float_as_uint(v) & ~1u) | bit); }
#if DDRL_LX_ON
#if DDRL_XCHG_LXSYS
// peer TU: the quads' outboxes as buffer resources, stores and loads at system scope (sc0 sc1)
typedef __amdgpu_buffer_rsrc_t lx_box_t;
__device__ __forceinline__ lx_box_t lx_rsrc(unsigned long long* box) {
  return __builtin_amdgcn_make_buffer_rsrc(box, 0, GX_MAX_PAIRS * 256 * 16, 0x00020000);
}
#define DDRL_LX_ST 17
#define DDRL_LX_LD 17
#else
typedef gx_box_t lx_box_t;
__device__ __forceinline__ lx_box_t lx_rsrc(unsigned long long* box) { return gx_rsrc(box); }
#define DDRL_LX_ST DDRL_GX_ST
#define DDRL_LX_LD DDRL_GX_LD
#endif
__device__ __forceinline__ void gx_put4(lx_box_t r, int j, float a, float b, float c, float d, unsigned bit) {
  const v4u g = {__float_as_uint(lx_t(a, bit)), __float_as_uint(lx_t(b, bit)), __float_as_uint(lx_t(c, bit)),
                 __float_as_uint(lx_t(d, bit))};
  __builtin_amdgcn_raw_buffer_store_b128(g, r, (j * 256 + (int)threadIdx.x) * 16, 0, DDRL_LX_ST);
}
// NX > 0: the timing-only cost-model build of a four-way split; NX more quads (another outbox,
// rx) loaded with every poll and returned unchecked
template <int NQ, int NX = 0, typename F>
__device__ __forceinline__ bool gx_get4(lx_box_t r, unsigned bit, float* out, int* err, F&& after_first,
                                        lx_box_t rx = lx_box_t()) {
  bool lost = false;
  v4u g[NQ + NX];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool first = true;
  for (;;) {
    xchg_inv_l1();
#pragma unroll
    for (int j = 0; j < NQ; ++j) g[j] = __builtin_amdgcn_raw_buffer_load_b128(r, (j * 256 + (int)threadIdx.x) * 16, 0, DDRL_LX_LD);
#pragma unroll
    for (int j = 0; j < NX; ++j) g[NQ + j] = __builtin_amdgcn_raw_buffer_load_b128(rx, (j * 256 + (int)threadIdx.x) * 16, 0, DDRL_LX_LD);
    if (first) { after_first(); first = false; }
    unsigned bad = 0;
#pragma unroll
    for (int j = 0; j < NQ; ++j) bad |= (g[j][0] ^ bit) | (g[j][1] ^ bit) | (g[j][2] ^ bit) | (g[j][3] ^ bit);
    if ((bad & 1u) == 0) break;
    if (xchg_abandon(t0, err)) {
#pragma unroll
      for (int j = 0; j < NQ + NX; ++j) g[j] = v4u{0u, 0u, 0u, 0u};
      lost = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int j = 0; j < NQ + NX; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) out[4 * j + k] = __uint_as_float(g[j][k]);
  return lost;
}
#endif

// dH2^T = Wo . dout^T on the matrix cores (policy head, O = 2A >= 4 outputs): one
// 16x16x4 MFMA per feature block and 4 outputs, A = Wo[f = 16 fb + c][o = 4 kk + q] (LDS),
// B = dout[row c][4 kk + q]; the result lands in the transposed activation layout
// (feature 16 fb + 4q + r of row c) that head_bwd's VALU form produces.
template <int O>
__device__ __forceinline__ void head_bwd_mfma(const NetLds& W, const float* dout, floatx4 dh[4]) {
  static_assert(O % 4 == 0, "policy head: 2A outputs");
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
  float b[O / 4];
#pragma unroll
  for (int kk = 0; kk < O / 4; ++kk)
    b[kk] = q == 0 ? dout[4 * kk] : q == 1 ? dout[4 * kk + 1] : q == 2 ? dout[4 * kk + 2] : dout[4 * kk + 3];
#pragma unroll
  for (int fb = 0; fb < 4; ++fb) {
    floatx4 acc = splat4(0.f);
#pragma unroll
    for (int kk = 0; kk < O / 4; ++kk) acc = mfma4(W.wo[(16 * fb + c) * O + 4 * kk + q], b[kk], acc);
    dh[fb] = acc;
  }
}

// dw_tiles_fm plus one more tile from a second pair of images, interleaved into the same
// MFMA stream (the policy head's dWo = H2^T dout tile of feature block fah, dout image
// rows >= 2A zero): out[i] as dw_tiles_fm, outh[r] = dWo[16 fah + 4q + r][o = c].
template <int NROWS, int NT_, int LD = NROWS + 8>
__device__ __forceinline__ void dw_tiles_fm_head(const float* A, const float* B, const int* fa, int fo, floatx4* out,
                                                 const float* AH, const float* BH, int fah, floatx4& outh) {
  const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < NT_; ++i) out[i] = splat4(0.f);
  outh = splat4(0.f);
  const float* bp = B + (16 * fo + c) * LD + 4 * q;
  const float* bph = BH + c * LD + 4 * q;
  const float* aph = AH + (16 * fah + c) * LD + 4 * q;
  const float* ap[NT_];
#pragma unroll
  for (int i = 0; i < NT_; ++i) ap[i] = A + (16 * fa[i] + c) * LD + 4 * q;
  constexpr int NU = NROWS / 16;
  floatx4 bv[2], av[2][NT_], bhv[2], ahv[2];
  bv[0] = *reinterpret_cast<const floatx4*>(bp);
  bhv[0] = *reinterpret_cast<const floatx4*>(bph);
  ahv[0] = *reinterpret_cast<const floatx4*>(aph);
#pragma unroll
  for (int i = 0; i < NT_; ++i) av[0][i] = *reinterpret_cast<const floatx4*>(ap[i]);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    if (u + 1 < NU) {
      bv[(u + 1) & 1] = *reinterpret_cast<const floatx4*>(bp + 16 * (u + 1));
      bhv[(u + 1) & 1] = *reinterpret_cast<const floatx4*>(bph + 16 * (u + 1));
      ahv[(u + 1) & 1] = *reinterpret_cast<const floatx4*>(aph + 16 * (u + 1));
#pragma unroll
      for (int i = 0; i < NT_; ++i) av[(u + 1) & 1][i] = *reinterpret_cast<const floatx4*>(ap[i] + 16 * (u + 1));
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
#pragma unroll
      for (int i = 0; i < NT_; ++i) out[i] = mfma4(av[u & 1][i][v], bv[u & 1][v], out[i]);
      outh = mfma4(ahv[u & 1][v], bhv[u & 1][v], outh);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int A, int KS1, int OB, bool POL, int NW, int KSP, bool CUP, bool LSBX>
__device__ __forceinline__ void update_loop(const UpdateArgs& U, const UpdateBatch& ub, float* lds, int p, int kq) {
  constexpr int ROWS = DDRL_MB / KSP;
  constexpr int NT = Geo<NW, ROWS>::NT, RT = Geo<NW, ROWS>::RT, NS1 = Geo<NW, ROWS>::NS1, NS2 = Geo<NW, ROWS>::NS2;
  constexpr bool PAD = update_pad(A, KSP);   // layout of the weight images (common.h)
#ifdef DDRL_ABL_NO_MOMENTS
  constexpr bool NOMOM = KSP == 2;
#else
  constexpr bool NOMOM = false;
#endif
  // DDRL_ABL_ADAM_SPLIT: timing-only cost model (round 6) of Adam split over the two row halves
  // -- each half updates half of the parameters, then reads its partner's half of the updated
  // weights (results wrong)
#ifdef DDRL_ABL_ADAM_SPLIT
  constexpr bool ADAM_SPLIT = KSP == 2;
#else
  constexpr bool ADAM_SPLIT = false;
#endif
  const size_t gx_box_n = (size_t)GX_MAX_PAIRS * 256 * 2;   // granules per outbox
  const int wkq = ub.own_kq < 0 ? 0 : ub.own_kq;   // the half that writes back and writes the statistics
  const UpdateHyper& H = ub.h;
  const int d = U.d;
  const FfnOffsets of = ffn_offsets(d, A);
  const BranchOff bo = branch_off(of, POL);
  const int nf1 = (d + 15) >> 4;
  constexpr int NSB0 = 64 * OB + OB + 128;         // small params of this branch
  constexpr int NCUP = CUP ? ncup_slots(OB, POL) : 0;   // + the "cup" coupling table
  constexpr int NSB = NSB0 + NCUP;                  // small params of this branch
  constexpr bool cup = NCUP > 0;
  constexpr int nsb = NSB;
  constexpr int NSLOT = (NSB + NT - 1) / NT;
  constexpr int NSTAT = POL ? 3 : 5;
  constexpr int NTS = NS1 + NS2;
  constexpr int NP0 = (NSLOT + 2) / 2;              // exchange pairs: small params + stats,
  constexpr int NP = NP0 + 2 * NTS;                  // then the owned dW tiles (KSP = 2)
  static_assert(KSP == 1 || (NT == 256 && NP == gx_pairs(OB, NW) && NP <= GX_MAX_PAIRS), "exchange pairs");
  // fused launches (LSBX) sum LSB-replaced partials; the default protocol also exchanges them as
  // LSB-tagged quads (LX: small params + stats, then one quad per owned dW tile), the atomic one
  // keeps its {value, tag} pairs and replaces the bits before the sum -- the same sums
  constexpr bool LX = LSBX && KSP == 2 && DDRL_LX_ON;
  constexpr int NQ0 = (NSLOT + 1 + 3) / 4;
  constexpr int NQ = NQ0 + NTS;
  static_assert(!LX || NQ <= GX_MAX_PAIRS, "exchange quads");

  NetLds W;
  constexpr int LD = ROWS + 8;              // feature-major image stride
  // K (rows) of the weight-gradient tiles; the timing-only cost-model build
  // -DDDRL_ABL_HALF_DW halves it (the weight-gradient work of a four-way row split)
#ifdef DDRL_ABL_HALF_DW
  constexpr int DWR = ROWS / 2;
#else
  constexpr int DWR = ROWS;
#endif
  float* bufA = lds + branch_lds_floats(PAD);    // feature-major [64][LD]: H1, then X
  float* bufB = bufA + 64 * LD;             // feature-major [64][LD]: dZ2, then dZ1
  float* Pb = bufB + 64 * LD;               // [NW][NSB] per-wave partial small grads
  float* red = Pb + NW * NSB;               // [NW][8] row-stat partials, [64..] scalars
  int* idxb = reinterpret_cast<int*>(red + 128);   // [128] record rows of the next step
  // policy branch of the row split: the head gradient dWo = H2^T dout runs on the matrix cores
  // with the dW2 tiles, from feature-major images of H2 and dout (rows >= 2A of the dout
  // image stay zero); the other instances reduce it with DPP transposes (their LDS budget --
  // A = 8, 128-row images -- has no room for the two images)
  constexpr bool HMF = POL && KSP == 2;
  float* bufH = red + 256;                  // HMF: feature-major [64][LD] H2
  float* bufD = bufH + 64 * LD;             // HMF: feature-major [16][LD] dout
  float* stg = red + 256 + (HMF ? 80 * LD : 0);   // [ROWS][stride] records of the next step (16 B aligned)
  const int stride = U.lay.stride, cpr = stride >> 2, cpr_l = stg_chunks(stride, A);
  const float inv_cpr_l = 1.f / (float)cpr_l;

  // w is wave-uniform: readfirstlane keeps it (and the tile indices derived from it) in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, q = lane >> 4,
            w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Store cache policy of the exchange.  A run-time choice here cost 0.3 us per step (the
  // branches around every granule store, measured), so the device-coherent protocol is the
  // separate -DDDRL_XCHG_ATOMIC build and this one always stores plainly into the XCD's L2.
  constexpr bool coh = false;
  int row_l[RT];
  bool row_ok[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    row_l[t] = 16 * RT * w + 16 * t + c;               // row of this workgroup's share
    row_ok[t] = ROWS * kq + row_l[t] < ub.nrows;
  }

  // ---- first step's records (LDS-DMA) in flight while the weights are staged ----
  const int total_steps = U.n_epochs * U.nb;
  const int last = U.max_steps >= 0 ? min(total_steps, U.step0 + U.max_steps) : total_steps;
  // minibatch row of this lane's staging slot (tid < ROWS)
  const int gr = ROWS * kq + tid;
  const bool gok = tid < ROWS && gr < ub.nrows;
  if (tid < ROWS) idxb[tid] = U.step0 < last && gok ? row_index(U, U.step0, gr, true) : 0;
  __syncthreads();
  if (U.step0 < last) issue_rows<NW, ROWS>(U.rec, stride, cpr, cpr_l, inv_cpr_l, idxb, stg, U.R, ub.lds_bytes);
  stage_branch_batched<OB, NT, PAD>(U.theta, d, bo, lds, W, NCUP);
  if constexpr (HMF) {
    // the head tile results go to wave 0's partial row; the other waves' dWo partials stay 0
    for (int i = tid; i < NW * NSB; i += NT) Pb[i] = 0.f;
    for (int i = tid; i < 16 * LD; i += NT) bufD[i] = 0.f;
  }

  // ---- optimizer state of the parameters this lane owns ----
  // tile tt = 4 fa + fo; slots 0..NS1-1: dW2 tiles w + NW i;  then dW1 tiles w + NW i (if < 4 nf1).
  // NW is a multiple of 4, so every tile of a wave has fo = w & 3.
  floatx4 mt[NTS], vt4[NTS];
  bool tv[NTS];
  int tfa[NTS], tfo[NTS];
#pragma unroll
  for (int i = 0; i < NTS; ++i) {
    const int tt = i < NS1 ? w + NW * i : w + NW * (i - NS1);
    tv[i] = i < NS1 ? true : (tt < 4 * nf1);
    tfa[i] = tt >> 2;
    tfo[i] = tt & 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * tfa[i] + 4 * q + r, o = 16 * tfo[i] + c;
      const bool ok = tv[i] && (i < NS1 || f < d) && !U.grad_out;   // gradient-only launches: no Adam
      const int pidx = (i < NS1 ? bo.w2 : bo.w1) + f * 64 + o;
      BCHK(!ok || (pidx >= 0 && pidx < of.n), 5);
      mt[i][r] = ok ? U.m[pidx] : 0.f;
      vt4[i][r] = ok ? U.v[pidx] : 0.f;

    }
  }
  float ms[NSLOT], vs[NSLOT];
  int sp_pidx[NSLOT], sp_lds[NSLOT];   // loop invariants: parameter index and LDS word of each slot
#pragma unroll
  for (int k = 0; k < NSLOT; ++k) {
    const int e = tid + NT * k;
    ms[k] = vs[k] = 0.f;
    sp_pidx[k] = 0;
    // a slot past the small parameters reads and writes a sink word (red[127]: red holds
    // [0, 64) per-wave statistics, [64, 72) norm partials, 80 / 81, [96, 104) the combined
    // statistics, and idxb from 128 on), so Adam's small-parameter LDS accesses need no lane
    // predicate in the step loop
    sp_lds[k] = DDRL_SINK ? (int)(red + 127 - lds) : 0;
    if (e < nsb) {
      int pidx; float* lp;
      small_param<OB>(e, bo, W, pidx, lp);
      BCHK(pidx >= 0 && pidx < of.n + NCUP, 5);
      sp_pidx[k] = pidx;
      sp_lds[k] = (int)(lp - lds);
      if (!U.grad_out) {
        ms[k] = U.m[pidx];
        vs[k] = U.v[pidx];
      }
    }
  }
  int ebase[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) ebase[r] = sidx<PAD>(4 * q + r, 16 * (w & 3) + c);
  float b1p = U.beta_pow[0], b2p = U.beta_pow[1];
  const float adv_mean = U.adv_norm[0], adv_den = U.adv_norm[1];
  const float beta = U.kl_coeff;
  const float lo = 1.f - H.clip, hi = 1.f + H.clip;
  __syncthreads();

  RowData<A, RT> cur;
  // features 4 (KS1 - 1) + q of the last layer-1 k-step: kept below d, zeroed at and above
  const unsigned xlast_bits = (KS1 < 12 && 4 * (KS1 - 1) + q >= d) ? 0u : 0xffffffffu;
  // records of step0 -> stg (issued above), row indices of step0 + 1 -> idxb, of step0 + 2 -> nxt
  wait_vmcnt0();
  __syncthreads();
  if (tid < ROWS) idxb[tid] = U.step0 + 1 < last && gok ? row_index(U, U.step0 + 1, gr, true) : 0;
  int nxt = U.step0 + 2 < last && gok ? row_index(U, U.step0 + 2, gr, true) : 0;
  // partner exchange slots: mine / the other row half of this branch, by step parity
  const size_t gx_branch = ((size_t)p * 2 + (POL ? 0 : 1)) * KSP;
  __syncthreads();

  const float inv_rows = 1.f / (float)ub.nrows;
  STAMP_INIT
  for (int step = U.step0; step < last; ++step) {
    // Adam's step size (tf1: lr sqrt(1 - b2^t) / (1 - b1^t), correctly rounded sqrt and
    // division) early: its latency hides under the forward's MFMAs
    const float alpha = H.lr * sqrtf(1.f - b2p) / (1.f - b1p);
    load_row<A, KS1, POL, RT>(stg, 4 * cpr_l, U.lay, row_l, d, cur, xlast_bits);
    // ---- forward + loss + output gradient (two row tiles) ----
    floatx4 h1[RT][4], h2[RT][4], dz[RT][4];
    float out[RT][OB], dout[RT][OB];
    ffn_fwd_rt<OB, KS1, RT, PAD>(W, cur.x, h1, h2, out);
    // "cup" (coupling_net_glorot_uniform_init.py:22-30): means scaled by the record's leg row
    float pre[RT][A], cf[RT][A];
    if constexpr (cup) {
      {
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int j = 0; j < A; ++j) {
            pre[t][j] = out[t][j];
            cf[t][j] = W.cup[cur.cid[t] * A + j];
            out[t][j] *= cf[t][j];
          }
      }
    }
    STAMP(0);
    float st[NSTAT];
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) st[k] = 0.f;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float st0[NSTAT];
      if constexpr (POL)
        policy_loss_row<A>(out[t], cur.act[t], cur.ol[t], cur.s0[t], (cur.s1[t] - adv_mean) / adv_den,
                           beta, lo, hi, H.ent_coeff, ub.inv_n, row_ok[t], dout[t], st0);
      else
        value_loss_row(out[t][0], cur.s0[t], cur.s1[t], H, ub.inv_n, row_ok[t], dout[t], st0);
#pragma unroll
      for (int k = 0; k < NSTAT; ++k) st[k] += st0[k];
    }
    STAMP(1);
    float* Pw = Pb + w * NSB;
    if constexpr (cup) {
      {
        // d coupling[leg][j] = sum over the leg's rows of dmean_j * pre-coupling mean_j;
        // the fcnet head then sees dmean_j * coupling[leg][j]
#pragma unroll
        for (int lg = 0; lg < 4; ++lg)
#pragma unroll
          for (int j = 0; j < A; ++j) {
            float v = 0.f;
#pragma unroll
            for (int t = 0; t < RT; ++t) v += cur.cid[t] == lg ? dout[t][j] * pre[t][j] : 0.f;
            v = row16_sum(v);
            if (lane == 0) Pw[NSB0 + lg * A + j] = v;
          }
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
          for (int j = 0; j < A; ++j) dout[t][j] *= cf[t][j];
      }
    }
    // head weight / bias partial gradients over this wave's rows: DPP transpose-reduce
    // of the 16 features (fb, r) a lane holds; afterwards lane (c, q) owns feature
    // h = 16 (c >> 2) + 4 q + (c & 3).
    const int h_own = 16 * (c >> 2) + 4 * q + (c & 3);
    if constexpr (HMF) {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        store_act_fm<LD>(bufH, RT * w + t, h2[t]);
        if (q == 0)
#pragma unroll
          for (int o = 0; o < OB; ++o) bufD[o * LD + row_l[t]] = dout[t][o];
      }
    }
#ifndef DDRL_ABL_NO_HEADDPP
#pragma unroll
    for (int o = 0; o < (HMF ? 0 : OB); ++o) {
      float v[16];
#pragma unroll
      for (int fb = 0; fb < 4; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[4 * fb + r] = h2[0][fb][r] * dout[0][o];
#pragma unroll
          for (int t = 1; t < RT; ++t) v[4 * fb + r] += h2[t][fb][r] * dout[t][o];
        }
      Pw[h_own * OB + o] = row16_transpose_sum(v);
    }
#endif
#pragma unroll
    for (int o = 0; o < OB; ++o) {
      float dsum = dout[0][o];
#pragma unroll
      for (int t = 1; t < RT; ++t) dsum += dout[t][o];
      const float s = row16_sum(dsum);
      if (lane == 0) Pw[64 * OB + o] = s;
    }
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) {
      const float s = row16_sum(st[k]);
      if (lane == 0) red[w * 8 + k] = s;
    }
    STAMP(2);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      if constexpr (POL) head_bwd_mfma<OB>(W, dout[t], dz[t]);
      else head_bwd<OB>(W, dout[t], dz[t]);
      dtanh_inplace(dz[t], h2[t]);                       // dz = dZ2
    }
    {
      float v[16];
#pragma unroll
      for (int fb = 0; fb < 4; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[4 * fb + r] = dz[0][fb][r];
#pragma unroll
          for (int t = 1; t < RT; ++t) v[4 * fb + r] += dz[t][fb][r];
        }
      Pw[64 * OB + OB + 64 + h_own] = row16_transpose_sum(v);     // db2
    }
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      store_act_fm<LD>(bufA, RT * w + t, h1[t]);
      store_act_fm<LD>(bufB, RT * w + t, dz[t]);
    }
    STAMP(3);
#ifndef DDRL_ABL_NO_L2BWD
    layer2_bwd_rt<RT, PAD>(W, dz, h2);                   // h2 <- dH1
#endif
#pragma unroll
    for (int t = 0; t < RT; ++t) dtanh_inplace(h2[t], h1[t]);  // h2 = dZ1
    {
      float v[16];
#pragma unroll
      for (int fb = 0; fb < 4; ++fb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[4 * fb + r] = h2[0][fb][r];
#pragma unroll
          for (int t = 1; t < RT; ++t) v[4 * fb + r] += h2[t][fb][r];
        }
      Pw[64 * OB + OB + h_own] = row16_transpose_sum(v);          // db1
    }
    STAMP(4);
    __syncthreads();                                     // #1: H1, dZ2, partials visible
#if DDRL_GATHER_EARLY
    // the row split's prefetch of step + 1's records, issued here: every lane read its rows of
    // this step at the top (load_row), and the gathers now have the rest of the step to land
    if (KSP == 2 && step + 1 < last) issue_rows<NW, ROWS>(U.rec, stride, cpr, cpr_l, inv_cpr_l, idxb, stg, U.R, ub.lds_bytes);
#endif
    STAMP(5);
    const unsigned gtag = xchg_tag(ub.epoch, step);
    const int gstep = step + (int)ub.lx_base;            // outbox parity and quad tag bit
    const unsigned lbit = lx_bit(gstep);
    (void)lbit;
    const size_t gx_box = (size_t)GX_MAX_PAIRS * 256 * 2;   // granules per outbox
    const gx_box_t gx_mine = gx_rsrc(ub.gx + ((gx_branch + kq) * 2 + (gstep & 1)) * gx_box);
    float gs[NSLOT];
    float st_own = 0.f;
    // small-parameter partials and this half's loss statistics into the exchange (KSP = 2):
    // first thing after sync #1, or -- policy branch, whose head tile lands in the partials
    // with the dW2 tiles -- after sync #2 (all pairs are polled together, after the dW1 tiles)
    auto put_small = [&] {
      float v0[2 * NP0];
#pragma unroll
      for (int k = 0; k < 2 * NP0; ++k) v0[k] = 0.f;
#pragma unroll
      for (int k = 0; k < NSLOT; ++k) {
        const int e = tid + NT * k;
        float sm = 0.f;
        if (e < nsb)
          for (int i = 0; i < NW; ++i) sm += Pb[i * NSB + e];
        gs[k] = sm;
        v0[k] = sm;
      }
      if (tid < NSTAT)
        for (int i = 0; i < NW; ++i) st_own += red[i * 8 + tid];
      v0[NSLOT] = st_own;
#if DDRL_LX_ON
      if constexpr (LX) {
        const lx_box_t lx_mine = lx_rsrc(ub.gx + ((gx_branch + kq) * 2 + (gstep & 1)) * gx_box);
        float w0[4 * NQ0];
#pragma unroll
        for (int k = 0; k < 4 * NQ0; ++k) w0[k] = k <= NSLOT ? v0[k] : 0.f;
#pragma unroll
        for (int j = 0; j < NQ0; ++j) gx_put4(lx_mine, j, w0[4 * j], w0[4 * j + 1], w0[4 * j + 2], w0[4 * j + 3], lbit);
        return;
      }
#endif
#pragma unroll
      for (int j = 0; j < NP0; ++j) gx_put(gx_mine, j, v0[2 * j], v0[2 * j + 1], gtag, coh);
    };
    if constexpr (KSP == 2 && !HMF) put_small();
    floatx4 gt[NTS];
#ifndef DDRL_ABL_NO_DW2   // ablation builds (timing only): skip a phase
    if constexpr (HMF) {
      static_assert(NW == 4, "one head tile (16 features) per wave");
      floatx4 gh;
      dw_tiles_fm_head<DWR, NS1, ROWS + 8>(bufA, bufB, tfa, w & 3, gt, bufH, bufD, w, gh);   // dW2 tiles + dWo
      if (c < OB)
#pragma unroll
        for (int r = 0; r < 4; ++r) Pb[(16 * w + 4 * q + r) * OB + c] = gh[r];
    } else {
      dw_tiles_fm<DWR, NS1, ROWS + 8>(bufA, bufB, tfa, w & 3, gt);   // dW2 tiles of this wave
    }
#else
    for (int i = 0; i < NS1; ++i) gt[i] = splat4(0.f);
#endif
    if constexpr (KSP == 2) {
#pragma unroll
      for (int i = 0; i < NS1; ++i) {
#if DDRL_LX_ON
        if constexpr (LX) {
          gx_put4(lx_rsrc(ub.gx + ((gx_branch + kq) * 2 + (gstep & 1)) * gx_box), NQ0 + i, gt[i][0], gt[i][1], gt[i][2],
                  gt[i][3], lbit);
          continue;
        }
#endif
        gx_put(gx_mine, NP0 + 2 * i, gt[i][0], gt[i][1], gtag, coh);
        gx_put(gx_mine, NP0 + 2 * i + 1, gt[i][2], gt[i][3], gtag, coh);
      }
    }
    STAMP(6);
    __syncthreads();                                     // #2: dW2 operands consumed
    if constexpr (HMF) put_small();
    STAMP(7);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      store_act_fm<LD>(bufB, RT * w + t, h2[t]);
#pragma unroll
      for (int s = 0; s < 12; ++s) bufA[(4 * s + q) * LD + row_l[t]] = cur.x[t][s];
    }
    __syncthreads();                                     // #3: X, dZ1 visible
    STAMP(8);
    // ---- prefetch: the records of step + 1 land in stg (LDS-DMA) while the dW1 tiles, the
    //      norm exchange and Adam run; every lane has read its rows of this step (sync #1).
    //      The row split issues them with its partner exchange instead, behind the first
    //      poll's loads: vmcnt retires in order, so the exchange loads would otherwise wait
    //      for the gathers.
#ifndef DDRL_ABL_NO_PREFETCH
    if (KSP == 1 && step + 1 < last) issue_rows<NW, ROWS>(U.rec, stride, cpr, cpr_l, inv_cpr_l, idxb, stg, U.R, ub.lds_bytes);
#endif
    // the exchange lane (wave NW-1, which issued no gathers) polls the partner's granule
    // early: when the other branch is ahead, its norm^2 is already there at the exchange
    const int xlane = 64 * (NW - 1);
    unsigned long long* const xmine = ub.xchg + (((size_t)p * 2 + (POL ? 0 : 1)) * KSP + kq) * 2 + (step & 1);
    unsigned long long* const xother = ub.xchg + (((size_t)p * 2 + (POL ? 1 : 0)) * KSP + kq) * 2 + (step & 1);
    unsigned long long xv = 0;
    if (tid == xlane) xv = xchg_load(xother);
    STAMP(9);
    {
      // dW1 tiles of this wave: the valid slots are a prefix (tiles w + NW i < 4 nf1)
#pragma unroll
      for (int i = NS1; i < NTS; ++i) gt[i] = splat4(0.f);
      int n1 = 0;
#pragma unroll
      for (int i = NS1; i < NTS; ++i) n1 += tv[i] ? 1 : 0;
#ifdef DDRL_ABL_NO_DW1
      n1 = -1;
#endif
      if (n1 == NS2) dw_tiles_fm<DWR, NS2, ROWS + 8>(bufA, bufB, tfa + NS1, w & 3, gt + NS1);
      else if constexpr (NS2 >= 3) {
        if (n1 == 2) dw_tiles_fm<DWR, 2, ROWS + 8>(bufA, bufB, tfa + NS1, w & 3, gt + NS1);
        else if (n1 == 1) dw_tiles_fm<DWR, 1, ROWS + 8>(bufA, bufB, tfa + NS1, w & 3, gt + NS1);
      } else if (n1 == 1) dw_tiles_fm<DWR, 1, ROWS + 8>(bufA, bufB, tfa + NS1, w & 3, gt + NS1);
    }
    STAMP(10);
    if constexpr (KSP == 2) {
      // last share out, then the partner's: value = mine + partner's (commutative, so
      // both workgroups hold the same bits)
#pragma unroll
      for (int i = NS1; i < NTS; ++i) {
#if DDRL_LX_ON
        if constexpr (LX) {
          gx_put4(lx_rsrc(ub.gx + ((gx_branch + kq) * 2 + (gstep & 1)) * gx_box), NQ0 + i, gt[i][0], gt[i][1], gt[i][2],
                  gt[i][3], lbit);
          continue;
        }
#endif
        gx_put(gx_mine, NP0 + 2 * i, gt[i][0], gt[i][1], gtag, coh);
        gx_put(gx_mine, NP0 + 2 * i + 1, gt[i][2], gt[i][3], gtag, coh);
      }
#if DDRL_LX_ON
      if constexpr (LX) {
#ifdef DDRL_ABL_XCHG3P
        // timing-only cost-model build: three partners' outboxes polled at once, every load of
        // the three in flight together, and their sum (here the partner's outbox, checked, and
        // 2 NQ quads of its other-parity outbox, unchecked)
        float o4[12 * NQ];
        gx_get4<NQ, 2 * NQ>(lx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box), lbit, o4, ub.err, [&] {
          if (!DDRL_GATHER_EARLY && step + 1 < last) issue_rows<NW, ROWS>(U.rec, stride, cpr, cpr_l, inv_cpr_l, idxb, stg, U.R, ub.lds_bytes);
        }, lx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + ((gstep + 1) & 1)) * gx_box));
#pragma unroll
        for (int k = 0; k < 4 * NQ; ++k) o4[k] = (o4[k] + o4[4 * NQ + k]) + o4[8 * NQ + k];
#else
        float o4[4 * NQ];
        gx_get4<NQ>(lx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box), lbit, o4, ub.err, [&] {
          if (!DDRL_GATHER_EARLY && step + 1 < last) issue_rows<NW, ROWS>(U.rec, stride, cpr, cpr_l, inv_cpr_l, idxb, stg, U.R, ub.lds_bytes);
        });
#endif
#if defined(DDRL_ABL_XCHG3)
        for (int extra = 0; extra < 2; ++extra) {   // the cost-model build, as below
          float o2[4 * NQ];
          gx_get4<NQ>(lx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box), lbit, o2, ub.err, [] {});
#pragma unroll
          for (int k = 0; k < 4 * NQ; ++k) o4[k] += 0.f * o2[k];
        }
#endif
        // both workgroups add the same two LSB-replaced partials
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) gs[k] = lx_t(gs[k], lbit) + o4[k];
        if (tid < NSTAT) red[96 + tid] = lx_t(st_own, lbit) + o4[NSLOT];
#pragma unroll
        for (int i = 0; i < NTS; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) gt[i][r] = lx_t(gt[i][r], lbit) + o4[4 * (NQ0 + i) + r];
      } else
#endif
      {
      float o[2 * NP];
#ifndef DDRL_ABL_NO_PREFETCH
      // the next step's record gathers go out right behind the first poll's loads (which
      // retire first: vmcnt is in order; a re-poll then waits for them too): 13.0 -> 12.9 us
      // per step against issuing them after the exchange
      gx_get<NP>(gx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box), gtag, o, ub.err, [&] {
        if (!DDRL_GATHER_EARLY && step + 1 < last) issue_rows<NW, ROWS>(U.rec, stride, cpr, cpr_l, inv_cpr_l, idxb, stg, U.R, ub.lds_bytes);
      });
#else
      gx_get<NP>(gx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box), gtag, o, ub.err, [] {});
#endif
#ifdef DDRL_ABL_XCHG3
      // timing-only cost-model build: the two more partner reads of a four-way row split, one
      // after the other (each a poll of the partner's outbox and the transfer of its partials)
      for (int extra = 0; extra < 2; ++extra) {
        float o2[2 * NP];
        gx_get<NP>(gx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box), gtag, o2, ub.err, [] {});
#pragma unroll
        for (int k = 0; k < 2 * NP; ++k) o[k] += 0.f * o2[k];
      }
#endif
      if constexpr (LSBX) {   // the atomic protocol of a fused launch: the quads' sums
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) gs[k] = lx_t(gs[k], lbit) + lx_t(o[k], lbit);
        if (tid < NSTAT) red[96 + tid] = lx_t(st_own, lbit) + lx_t(o[NSLOT], lbit);
#pragma unroll
        for (int i = 0; i < NTS; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) gt[i][r] = lx_t(gt[i][r], lbit) + lx_t(o[2 * NP0 + 4 * i + r], lbit);
      } else {
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) gs[k] += o[k];
        if (tid < NSTAT) red[96 + tid] = st_own + o[NSLOT];
#pragma unroll
        for (int i = 0; i < NTS; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) gt[i][r] += o[2 * NP0 + 4 * i + r];
      }
      }
      STAMP(14);
    } else {
#pragma unroll
      for (int k = 0; k < NSLOT; ++k) {
        const int e = tid + NT * k;
        float sm = 0.f;
        if (e < nsb)
          for (int i = 0; i < NW; ++i) sm += Pb[i * NSB + e];
        gs[k] = sm;
      }
    }
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) ss += gs[k] * gs[k];
#pragma unroll
    for (int i = 0; i < NTS; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 16 * tfa[i] + 4 * q + r;
        // the weights of features >= d: zero gradient (their inputs are zeroed in load_row), so
        // only the uniform tile predicate remains in the loop (the generic KS1 = 12 instance
        // zeroes every feature >= d there too)
        if (tv[i] && (i < NS1 || DDRL_PADZERO || f < d)) ss += gt[i][r] * gt[i][r];
      }

    if (U.grad_out) {   // data-parallel mode: export the raw gradient of this branch
#pragma unroll
      for (int i = 0; i < NTS; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 16 * tfa[i] + 4 * q + r, o = 16 * tfo[i] + c;
          if (tv[i] && (i < NS1 || f < d)) U.grad_out[(i < NS1 ? bo.w2 : bo.w1) + f * 64 + o] = gt[i][r];
        }
#pragma unroll
      for (int k = 0; k < NSLOT; ++k) {
        const int e = tid + NT * k;
        if (e < nsb) U.grad_out[sp_pidx[k]] = gs[k];
      }
      if (U.stats) {
        __syncthreads();   // red[96 ..] (wave 0) / the per-wave red[w * 8 ..] are read by wave 1
        if (tid == 64) write_stats<POL, NSTAT, NW, KSP>(U.stats + (size_t)step * 8, red, inv_rows);
      }
      return;
    }

    // ---- global norm: local reduction, then swap with the other branch's workgroup ----
    ss = wave_sum(ss);
    if (lane == 0) red[64 + w] = ss;
    __syncthreads();                                     // #4
    if (tid == xlane) {
      float local = 0.f;
      for (int i = 0; i < NW; ++i) local += red[64 + i];
      const unsigned tag = xchg_tag(ub.epoch, step);
      xchg_store(xmine, ((unsigned long long)tag << 32) | __float_as_uint(local), coh);
      unsigned long long v = xv;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#ifdef DDRL_ABL_NO_EXCHANGE
      v = ((unsigned long long)tag << 32) | __float_as_uint(local);
#endif
      while ((unsigned)(v >> 32) != tag) {
        v = xchg_load(xother);
        if ((unsigned)(v >> 32) == tag) break;
        if (xchg_abandon(t0, ub.err)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      // A failed exchange (a wait abandoned at its 3 s bound, or the error word seen after
      // 200 us) does not stop the step loop: an early exit checked every step cost 0.5 us per
      // step (measured, 13.24 vs 12.71 us).  Every later wait then ends after 200 us, and no
      // workgroup writes its weights back (the error word is checked before the write-back), so
      // HBM keeps the pre-launch state and the host restores its snapshot for the rest.
      const float partner = __uint_as_float((unsigned)(v & 0xffffffffu));
      const float tot = local + partner;                 // same sum on both workgroups
      // hardware sqrt / reciprocal (<= 1 ulp; tf's are correctly rounded): this lane sits on
      // every step's critical path between syncs #4 and #5, and the IEEE sequences cost
      // 0.08 us per step (measured); on the bench workload the trained state stays bit-identical
      const float gn = __builtin_amdgcn_sqrtf(tot);
      red[80] = gn;
      red[81] = H.grad_clip * fminf(__builtin_amdgcn_rcpf(gn), 1.f / H.grad_clip);
    }
    __syncthreads();                                     // #5
    STAMP(11);
    auto stats_out = [&] {
      write_stats<POL, NSTAT, NW, KSP>(U.stats + (size_t)step * 8, red, inv_rows);
      gst(U.stats + (size_t)step * 8 + 6, red[80]);
      gst(U.stats + (size_t)step * 8 + 7, red[81]);
    };
    // KSP = 1: wave 1, right after the exchange (the per-wave partials red[w * 8 + k] are
    // rewritten by the next step's loss); KSP = 2: after sync #6, off every critical path
    if (KSP == 1 && U.stats && tid == 64 && kq == wkq) stats_out();
    const float scale = red[81];
    const float c1 = 1.f - H.b1, c2 = 1.f - H.b2;

#ifndef DDRL_ABL_NO_ADAM
    // ---- tf1 Adam on owned parameters (m, v in registers, weights in LDS) ----
    // element (f = 16 fa + 4q + r, o = 16 fo + c) sits at ebase[r] + lds_blk(PAD) fa in W1 / W2.
    // All owned weights are read first, then updated, then written (no read-after-write
    // ordering between different parameters' LDS words).
    {
      float th[NTS][4], ts[NSLOT];
#pragma unroll
      for (int i = 0; i < NTS; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          th[i][r] = (i < NS1 ? W.w2 : W.w1)[ebase[r] + lds_blk(PAD) * tfa[i]];
#pragma unroll
      for (int k = 0; k < NSLOT; ++k) {
        const int e = tid + NT * k;
        ts[k] = 0.f;
        ts[k] = (DDRL_SINK || e < nsb) ? lds[sp_lds[k]] : 0.f;
      }
      // two elements per instruction (v_pk_* ops): the same fused operations, element by
      // element, as the scalar form g = gt s; m += (gt s - m) c1; v += (g g - v) c2;
      // theta -= (m alpha) / (sqrt(v) + eps)
#pragma unroll
      for (int i = 0; i < (ADAM_SPLIT ? (NTS + 1) / 2 : NTS); ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float2v gr = {gt[i][2 * h], gt[i][2 * h + 1]};
          // NOMOM: the timing-only cost model of VERDICT r05 item 3 -- the weight tiles' moments
          // not carried across steps, i.e. their 2 x 4 x NTS VGPRs out of the step loop (wrong results)
          float2v m2 = {NOMOM ? 0.f : mt[i][2 * h], NOMOM ? 0.f : mt[i][2 * h + 1]},
                  v2 = {NOMOM ? 0.f : vt4[i][2 * h], NOMOM ? 0.f : vt4[i][2 * h + 1]};
          const float2v sc = {scale, scale}, k1 = {c1, c1}, k2 = {c2, c2}, al = {alpha, alpha};
          const float2v g = gr * sc;
          m2 = __builtin_elementwise_fma(__builtin_elementwise_fma(gr, sc, -m2), k1, m2);
          v2 = __builtin_elementwise_fma(__builtin_elementwise_fma(g, g, -v2), k2, v2);
          float2v den = {__builtin_amdgcn_sqrtf(v2[0]), __builtin_amdgcn_sqrtf(v2[1])};
          den = den + (float2v){H.eps, H.eps};
          const float2v rc = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
          const float2v t2 = __builtin_elementwise_fma(-(m2 * al), rc, (float2v){th[i][2 * h], th[i][2 * h + 1]});
          if constexpr (!NOMOM) {
            mt[i][2 * h] = m2[0]; mt[i][2 * h + 1] = m2[1];
            vt4[i][2 * h] = v2[0]; vt4[i][2 * h + 1] = v2[1];
          }
          th[i][2 * h] = t2[0]; th[i][2 * h + 1] = t2[1];
        }

#pragma unroll
      for (int k = 0; k < (ADAM_SPLIT ? (NSLOT + 1) / 2 : NSLOT); ++k) {
        const float g = gs[k] * scale;
        ms[k] = ms[k] + (g - ms[k]) * c1;
        vs[k] = vs[k] + (g * g - vs[k]) * c2;
        ts[k] = ts[k] - (ms[k] * alpha) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vs[k]) + H.eps);
      }
#pragma unroll
      for (int i = 0; i < NTS; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 16 * tfa[i] + 4 * q + r;
          // (rows >= d of the W1 image: their gradient and moments are zero up to the exchange's
          // tag bits, they meet only zeroed inputs, and the write-back to HBM skips them)
          if (tv[i] && (i < NS1 || DDRL_PADZERO || f < d))
            (i < NS1 ? W.w2 : W.w1)[ebase[r] + lds_blk(PAD) * tfa[i]] = th[i][r];
        }
#pragma unroll
      for (int k = 0; k < NSLOT; ++k) {
        const int e = tid + NT * k;
        if (DDRL_SINK || e < nsb) lds[sp_lds[k]] = ts[k];
      }
    }
#endif
#if DDRL_LX_ON
    if constexpr (ADAM_SPLIT && LX) {
      // the cost model's second hop: the partner's half of the updated weights (half the quads
      // of its outbox, already valid for this step), read before sync #6
      const int gstep = step + (int)ub.lx_base;
      float o2[4 * ((NQ + 1) / 2)];
      gx_get4<(NQ + 1) / 2>(lx_rsrc(ub.gx + ((gx_branch + (kq ^ 1)) * 2 + (gstep & 1)) * gx_box_n), lx_bit(gstep), o2,
                             ub.err, [] {});
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 4 * ((NQ + 1) / 2); ++k) acc += o2[k];
      if (acc == 1.2345e-30f) red[127] = acc;   // keeps the loads
    }
#endif
    b1p = b1p * H.b1;
    b2p = b2p * H.b2;
    STAMP(12);
    wait_vmcnt0();                                       // this wave's record gathers landed
    if (tid < ROWS) idxb[tid] = nxt;                     // row indices of step + 2
    __syncthreads();                                     // #6: weights updated, stg / idxb ready
    if (tid < ROWS) nxt = step + 3 < last && gok ? row_index(U, step + 3, gr, true) : 0;
    // red[80..81] / red[96..] hold until the next step's exchanges (after its sync #1)
    if (KSP == 2 && U.stats && tid == 64 && kq == wkq) stats_out();
    STAMP(13);
  }
  STAMP_DONE;
  if (U.grad_out || kq != wkq) return;   // the row halves hold identical state: one writes it back
  // a failed launch (an exchange abandoned anywhere: the error word) leaves theta / m / v /
  // beta powers in HBM as they were; the host restores its snapshot for the rest
  if (__hip_atomic_load(ub.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;

  // ---- write back weights, optimizer state, beta powers ----
#pragma unroll
  for (int i = 0; i < NTS; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * tfa[i] + 4 * q + r, o = 16 * tfo[i] + c;
      if (!(tv[i] && (i < NS1 || f < d))) continue;
      const int pidx = (i < NS1 ? bo.w2 : bo.w1) + f * 64 + o;
      if constexpr (!NOMOM) {
        U.m[pidx] = mt[i][r];
        U.v[pidx] = vt4[i][r];
      }
    }
#pragma unroll
  for (int k = 0; k < NSLOT; ++k) {
    const int e = tid + NT * k;
    if (e >= nsb) continue;
    int pidx; float* lp;
    small_param<OB>(e, bo, W, pidx, lp);
    U.m[pidx] = ms[k];
    U.v[pidx] = vs[k];
    U.theta[pidx] = *lp;
  }
  for (int i = tid; i < 48 * 64; i += NT) {
    const int f = i >> 6;
    if (f < d) U.theta[bo.w1 + i] = W.w1[sidx<PAD>(f, i & 63)];
  }
  for (int i = tid; i < 64 * 64; i += NT) U.theta[bo.w2 + i] = W.w2[sidx<PAD>(i >> 6, i & 63)];
  if (POL && tid == 0) {
    U.beta_pow[0] = b1p;
    U.beta_pow[1] = b2p;
  }
}

template <int A, int KS1, int KSP, bool CUP, bool LSBX>
__global__ void __launch_bounds__(64 * waves_for(A, KSP)) k_update_ffn(UpdateBatch ub) {
  extern __shared__ float lds[];
  constexpr int NW = waves_for(A, KSP);
  // block b = p + 8 j, j = KSP branch + kq (branch 0 = policy, kq = row half): the blocks of
  // one policy are dealt to the same XCD (b mod 8), so its per-step exchanges stay inside
  // one XCD (speed only; they are agent-scope either way).  Blocks with p >= P have no work.
  const int p = blockIdx.x & 7;
  if (threadIdx.x == 0) {   // placement record: XCC of every block (capi.cpp check_placement)
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    ub.xcc[blockIdx.x] = (int)(x & 0xf);
  }
  if (p >= ub.h.P) return;
  const int j = blockIdx.x >> 3, branch = j / KSP, kq = j - branch * KSP;
  if (ub.own_kq >= 0 && kq != ub.own_kq) return;   // peer mode: the other half runs on the peer context
  const UpdateArgs U = ub.a[p];
  if (branch) update_loop<A, KS1, 1, false, NW, KSP, false, LSBX>(U, ub, lds, p, kq);
  else update_loop<A, KS1, 2 * A, true, NW, KSP, CUP, LSBX>(U, ub, lds, p, kq);
}

// stride: the widest record stride of the launched policies (staging buffer rows)
static size_t update_lds_bytes(int O, int stride, int ksp) {
  const int nsb = 64 * O + O + 128 + ncup_slots(O, true);
  const int nw = waves_for(O / 2, ksp);
  // + the policy head's H2 / dout images of the row split (HMF in update_loop)
  return (size_t)(branch_lds_floats(update_pad(O / 2, ksp)) + 2 * 64 * (DDRL_MB / ksp + 8) + nw * nsb + 256 +
                  (ksp == 2 ? 80 * (DDRL_MB / ksp + 8) : 0) +
                  (DDRL_MB / ksp) * 4 * stg_chunks(stride, O / 2)) * 4;
}

template <int A, int KS1, bool CUP = false>
static void launch_update_t(hipStream_t s, UpdateBatch& ub, int P, int stride, int ksp, bool lx) {
  ub.lds_bytes = (unsigned)update_lds_bytes(2 * A, stride, ksp);
#if DDRL_FFN_KSP != 1
  if (ksp == 2 && lx)
    hipLaunchKernelGGL((k_update_ffn<A, KS1, 2, CUP, true>), dim3(24 + P), dim3(64 * waves_for(A, 2)), ub.lds_bytes, s, ub);
#endif
#if DDRL_FFN_KSP != 2
  if (ksp == 2 && !lx)
    hipLaunchKernelGGL((k_update_ffn<A, KS1, 2, CUP, false>), dim3(24 + P), dim3(64 * waves_for(A, 2)), ub.lds_bytes, s, ub);
  if (ksp == 1)
    hipLaunchKernelGGL((k_update_ffn<A, KS1, 1, CUP, false>), dim3(8 + P), dim3(64 * waves_for(A, 1)), ub.lds_bytes, s, ub);
#endif
}

}  // namespace

void DDRL_FFN_LAUNCH(hipStream_t s, const UpdateArgs* ua, const UpdateHyper& h, int nrows, float inv_n,
                       int A, int d, int stride, int cup, unsigned long long* xchg, unsigned long long* gx, int ksp,
                       int* err, unsigned* epoch_ctr, int* xcc, int own_kq, unsigned lx_base) {
#if DDRL_FFN_KSP == 2
  // only the fused row-split kernels (LSB quads) live here; the KSP = 1 kernels and the
  // gradient-export launches are built in ppo_ffn_k1.hip
  if (!(ksp == 2 && ua[0].grad_out == nullptr && DDRL_LX)) {
    launch_update_ffn_k1(s, ua, h, nrows, inv_n, A, d, stride, cup, xchg, gx, ksp, err, epoch_ctr, xcc, own_kq, lx_base);
    return;
  }
#endif
  UpdateBatch ub;
  for (int p = 0; p < DDRL_MAXP; ++p) ub.a[p] = p < h.P ? ua[p] : UpdateArgs{};
  ub.h = h;
  ub.nrows = nrows;
  ub.inv_n = inv_n;
  ub.xchg = xchg;
  ub.gx = gx;
  ub.err = err;
  ub.xcc = xcc;
  ub.own_kq = own_kq;
  ub.lx_base = lx_base;
  // Every granule tag carries the launch epoch (12 bits, per context). Granules are cleared
  // only when the epoch wraps: between two clears every launch's epoch is larger than that
  // of any granule left in the buffers, so a stale granule can never match.  (A memset per
  // launch costs a fill kernel and a boundary, ~5 us, per data-parallel step.)
  ub.epoch = (*epoch_ctr)++ % 4095u + 1u;
  // fused launches (no gradient export) exchange LSB-tagged quads: their outboxes start cleared
  // in every launch (one fill per iteration); gradient launches keep the epoch-tagged pairs
  const bool lx = ksp == 2 && ua[0].grad_out == nullptr && DDRL_LX;
  if (ub.epoch == 1) (void)hipMemsetAsync(xchg, 0, sizeof(unsigned long long) * 8 * DDRL_MAXP, s);
  // (peer mode: gx is shared with the peer context's launch, which may be running; it is cleared
  // when the peers attach, ddrl_peer_attach, and the quads' tag bits follow the pair's global
  // step count, lx_base, so a value left from an earlier launch never matches)
  if (own_kq < 0 && (ub.epoch == 1 || (lx && DDRL_LX_ON))) {
    // A launch resumed at schedule step s0 (ddrl_ppo_update_from) keeps the quads' tag bits of
    // the global step, so the outbox of each parity must start with the complement of the bit
    // of its first use, s0 or s0 + 1: zero words would pass a first bit of 0.  One byte pattern
    // per parity (0x00: LSB 0, 0x01: LSB 1; the pairs' epoch tags never equal 0x01010101).
    const int s0 = ua[0].step0;
    const unsigned b0 = (((unsigned)s0 >> 1) & 1u) ^ 1u, b1 = (((unsigned)(s0 + 1) >> 1) & 1u) ^ 1u;
    if (!(lx && DDRL_LX_ON) || (b0 && b1)) {
      (void)hipMemsetAsync(gx, 0, gx_bytes(DDRL_MAXP), s);
    } else {
      const size_t box = sizeof(unsigned long long) * (size_t)GX_MAX_PAIRS * 256 * 2;
      const size_t nbox = gx_bytes(DDRL_MAXP) / box;   // box index = 2 * (branch slot) + parity
      for (int q = 0; q < 2; ++q) {
        const unsigned first_bit = (s0 & 1) == q ? b0 : b1;
        (void)hipMemset2DAsync(reinterpret_cast<char*>(gx) + q * box, 2 * box, first_bit ? 0 : 1, box, nbox / 2, s);
      }
    }
  }
  if (cup)   // "cup": one shared leg policy, A = 2, d <= 20 (capi validate)
    launch_update_t<2, 5, true>(s, ub, h.P, stride, ksp, lx);
  else
    DDRL_DISPATCH_A_KS1(A, d, launch_update_t, s, ub, h.P, stride, ksp, lx);
}
