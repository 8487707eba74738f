// mdr_capi.hip — C-ABI host runtime: contexts, launches, graph cache, greedy scratch, RCCL.
//
// The C ABI (include/mdr.h) is what the Python layer (mdr_amd, via ctypes) and any other host
// binds.  It owns only small scratch; every launch goes to the caller's stream.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "mdr_actor.h"
#include "mdr_interp.h"
#include "mdr_obs_dev.h"
#include "mdr_kernels.h"

using namespace mdr;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(MDR_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));            \
  } while (0)

#define RCCL_TRY(expr)                                                                     \
  do {                                                                                     \
    ncclResult_t r_ = (expr);                                                              \
    if (r_ != ncclSuccess) return fail(MDR_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

#define LAUNCH_CHECK(what)                                                                 \
  do {                                                                                     \
    hipError_t e_ = hipGetLastError();                                                     \
    if (e_ != hipSuccess) return fail(MDR_EHIP, std::string(what) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline unsigned blocks(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

struct GraphKey {
  int n_ticks, mode;
  const void* act;
  int64_t act_stride;
  void* rew;
  int64_t rew_stride;
  void* p_out;
  bool operator<(const GraphKey& o) const {
    return std::tie(n_ticks, mode, act, act_stride, rew, rew_stride, p_out) <
           std::tie(o.n_ticks, o.mode, o.act, o.act_stride, o.rew, o.rew_stride, o.p_out);
  }
};

}  // namespace

struct mdr_ctx {
  mdr_config cfg{};
  KParams kp{};
  bool bound = false;
  double* d_tables = nullptr;           // q_on[MDR_MAX_CAP] | p_on[MDR_MAX_CAP]
  unsigned long long* d_slab = nullptr;  // kSlabs x kCountShards x n_cap count slabs (ring of 3 on
                                         // the step path, 4 in the overlapped sharded pipeline)
  int slab_len = 0;
  int ring = 0;                          // slab of the current tick
  bool counts_ready = false;             // current slab filled (phase 1 or previous lookahead)
  double* d_pen_partial = nullptr;       // 2 per block of k_step_t
  double* d_partial2 = nullptr;
  int pen_blocks = 0;
  // ---- options (mdr_set_option; defaults are the measured-fastest exact configuration)
  int tpw = 0;                           // MDR_OPT_STEP_TPW: k_step_pipe tiles per wave (0: k_step_t)
  bool fastdiv = true;                   // MDR_OPT_FASTDIV: shared-reciprocal exact division
  bool win_pipe = true;                  // MDR_OPT_WINDOW_PIPELINE: sharded count-ahead window pipeline
  bool tick_overlap = true;              // MDR_OPT_SHARDED_OVERLAP: per-tick sharded two-stream pipeline
  bool greedy_sort = false;              // MDR_OPT_GREEDY_SORT: the full-sort greedy form only
  bool force_halo = false;               // MDR_OPT_FORCE_HALO: sharded actor halo exchange at world 1
  bool actor_generic = false;            // MDR_OPT_ACTOR_GENERIC: no default-layout k_actor form
  bool actor_fp32_bf16 = false;          // MDR_OPT_ACTOR_FP32_FORM: the three-way bf16 fp32 form (kernel PREC 6)
  bool halo_overlap = true;              // MDR_OPT_HALO_OVERLAP: sharded actor tick, halo beside the interior tiles
  bool halo_in_counts = true;            // MDR_OPT_HALO_IN_COUNTS: the next tick's ring halo rides in the count allreduce
  unsigned long long* d_c5 = nullptr;    // that path's ring of 3 x [count slab | world x halo rows]
  size_t c5_bytes = 0;
  int thermal = MDR_THERMAL_AFFINE;      // MDR_OPT_WINDOW_THERMAL: k_step_window's per-tick update
  int win = kWindowMax;                  // ticks per k_step_window launch (0: one-tick path)
  unsigned long long* d_wslab = nullptr; // 3 window count slots (mdr_kernels.hip K1W: slab | red | rec)
  int wslab_len = 0;
  bool wslab_dirty = true;               // the slots' shard part must be zero when a rollout starts
  uint64_t* d_onb = nullptr;             // per-tick ON lane masks of the next window [tiles][HPT][kWindowMax]
  uint32_t* d_wah = nullptr;             // FSM word at the end of the next window, per house
  uint64_t* d_onb2 = nullptr;            // second set for the count-ahead pipeline (window_launches pipe)
  uint32_t* d_wah2 = nullptr;
  size_t onb_bytes = 0, wah_bytes = 0;
  bool coef_dirty = true;
  int* d_flags = nullptr;                // [0] params_bad
  unsigned* d_tickets = nullptr;         // k_count_window's grid_last_block counters (zero between uses)
  // rollout tick drivers
  TickArgs* d_ticks = nullptr;
  int ticks_cap = 0;
  std::map<GraphKey, std::pair<hipGraphExec_t, int>> graphs;  // exec, ring phase at end
  // greedy scratch
  int64_t g_cap = 0;
  double *g_key = nullptr, *g_key2 = nullptr, *g_ps = nullptr, *g_incl = nullptr;
  int *g_idx = nullptr, *g_idx2 = nullptr;
  uint8_t* g_ls = nullptr;
  void* g_tmp = nullptr;
  size_t g_tmp_bytes = 0;
  int64_t* g_kpos = nullptr;
  int64_t* g_extra = nullptr;
  // histogram-select greedy (k_gq_*): partial min/max, bin histogram, selection, staged window
  double* g_part = nullptr;
  unsigned* g_hist = nullptr;
  GqSel* g_sel = nullptr;
  uint4* g_win = nullptr;                // the candidate window, unordered (k_gq_compact)
  uint32_t* g_map = nullptr;             // the key -> bin map's cells (gq_bin; k_gq_bins writes the next)
  unsigned* g_tickets = nullptr;         // k_gq_select's grid_last_block counters
  double* g_range = nullptr;             // sharded select: this shard's (min, -max) key range (k_gq_range)
  uint4* g_sorted = nullptr;             // the window in (key, house) order (k_gq_select)
  int gq_parts_cap = 0;                  // g_part capacity in (min, max) pairs
  bool gq_keys_ready = false;            // keys + superbin histogram of the current state are in place
  bool gq_hist_dirty = false;            // a producer added counts to g_hist that no select has consumed
  bool gq_slab_zeroed = false;           // the codes' producer zeroed the slab the decisions count into
                                         // (not when its step counted a lookahead there)
  bool gq_band = true;                   // MDR_OPT_GQ_BAND: k_gq_binsc (the predicted band) vs k_gq_bins
  // the fused greedy tick (mdr_greedy_rollout; mdr_kernels.h GqfBufs)
  bool gq_adaptive = true;               // MDR_OPT_GQ_ADAPTIVE: mdr_greedy_rollout skips the band on budget jumps
  bool gq_band_skip = false;             // (set around one mdr_ctrl_greedy call by mdr_greedy_rollout)
  double gq_s1 = NAN, gq_s2 = NAN;       // the last two budgets mdr_greedy_rollout decided for
  bool gq_map_stale = true;              // the state was written since the key maps were last built (k_gq_remap)
  bool gq_fused = false;                 // MDR_OPT_GQ_FUSED (r06: slower than the band form)
  GqfBufs fz{};
  int64_t fz_cap_n = 0;                  // the cluster size fz is allocated for
  int fz_par = 0;                        // the parity the last producer wrote
  bool fz_ready = false;                 // ... for the current state (the last step's GQ = 2 epilogue)
  int gq_nparts = 0;                     //   (from the last step's epilogue: its grid's partials)
  // multi-GPU
  ncclComm_t comm = nullptr;
  struct {                               // mdr_comm_host: the caller's collectives instead of RCCL
    mdr_host_allreduce_fn allreduce = nullptr;
    mdr_host_sendrecv_fn sendrecv = nullptr;
    void* user = nullptr;
  } host;
  int world = 1, rank = 0;
  hipStream_t comm_stream = nullptr;     // per-tick / per-window allreduces of the overlapped pipelines
  hipStream_t cap_stream = nullptr;      // graph capture (graphs are replayed on the caller's stream)
  hipEvent_t ev_k1[kSlabs] = {}, ev_ar[kSlabs] = {}, ev_pc = nullptr;
  hipEvent_t ev[16] = {};
  std::vector<hipEvent_t>* step_events = nullptr;  // mdr_time_step_kernels: events around each step launch
  struct {                               // mdr_rollout_begin: the first window already counted
    bool on = false;
    int n = 0, mode = 0;
    uint64_t tick0 = 0;
    const uint8_t* action = nullptr;
    int64_t act_stride = 0;
    bool sharded = false;                // counts allreduced over the ranks (for mdr_rollout_sharded)
  } begun;
  // MA-PPO actor (row P): packed weight image, per-tick obs scalars of actor rollouts
  unsigned char* d_actor = nullptr;
  size_t actor_cap = 0;
  float* d_actor_raw = nullptr;  // the loaded fp32 weights (w1 b1 w2 b2 w3 b3), packed per obs layout
  size_t actor_raw_cap = 0;
  std::vector<int> actor_key;    // the slot layout + precision d_actor is packed for (empty: stale)
  mdr_actor_spec actor{};                // (the two-hidden-layer view the fused kernel packs from)
  mdr_actor_net net{};                   // the loaded actor: layers, widths, precision
  bool actor_ready = false;
  float* d_chain = nullptr;              // the chain's rows: obs [n][F] | hidden ping-pong 2 x [n][wmax4]
  size_t chain_cap = 0;
  int n_cu = 0;
  double* d_obs_sc = nullptr;  // [ticks_cap][4]
  uint8_t* d_act = nullptr;    // [n_local] actor actions when the caller keeps none
  float* d_halo = nullptr;     // sharded actor rollout: packed edge rows | received ring halo
  double* d_stats = nullptr;   // k_cluster_stats block partials
  size_t halo_bytes = 0;
  std::map<std::vector<int64_t>, hipGraphExec_t> actor_graphs;
  int64_t graph_launches[2] = {0, 0};  // hipGraphLaunch calls: rollout graphs, actor rollout graphs
  int64_t graphs_guarded = 0;            // captured graphs the memset guard walked (graph_memset_guard)
  int64_t graph_nodes_checked = 0;       //   and their nodes
  // interpolated base power (row a10): grid | table | capacities
  double* d_interp = nullptr;
  size_t interp_bytes = 0;
  InterpArgs interp{};
  bool interp_ready = false;
};

namespace {

// the context has a communicator (the library's RCCL one, or the caller's host collectives)
bool has_comm(const mdr_ctx* c) { return c->comm != nullptr || c->host.allreduce != nullptr; }

// in-place allreduce ordered on st (op: the mdr_rccl_allreduce dtype codes; 0 = 64-bit sum, which
// the unsigned count slabs use: the same bits for sums below 2^63)
int comm_allreduce(mdr_ctx* c, void* buf, size_t count, int op, hipStream_t st) {
  if (c->comm) {
    const ncclDataType_t t = op == 0 ? ncclInt64 : op == 3 ? ncclUint32 : ncclFloat64;
    const ncclRedOp_t o = op == 2 ? ncclMax : op == 4 ? ncclMin : ncclSum;
    RCCL_TRY(ncclAllReduce(buf, buf, count, t, o, c->comm, st));
    return MDR_OK;
  }
  if (!c->host.allreduce) return fail(MDR_ESTATE, "no communicator (mdr_rccl_init / mdr_comm_host)");
  HIP_TRY(hipStreamSynchronize(st));
  if (int r = c->host.allreduce(c->host.user, buf, (int64_t)count, op))
    return fail(MDR_ERCCL, "host allreduce callback failed (" + std::to_string(r) + ")");
  return MDR_OK;
}

// the 'neighbours' ring halo of a sharded obs: this shard's last lo rows (mine[hi, hi+lo)) to the
// next rank, its first hi rows to the previous one; recv = [lo rows of prev | hi rows of next]
int comm_halo(mdr_ctx* c, float* mine, float* recv, int lo, int hi, int M, hipStream_t st) {
  const int prev = (c->rank + c->world - 1) % c->world, next = (c->rank + 1) % c->world;
  if (c->comm) {
    RCCL_TRY(ncclGroupStart());
    if (lo) {
      RCCL_TRY(ncclSend(mine + (size_t)hi * M, (size_t)lo * M, ncclFloat32, next, c->comm, st));
      RCCL_TRY(ncclRecv(recv, (size_t)lo * M, ncclFloat32, prev, c->comm, st));
    }
    if (hi) {
      RCCL_TRY(ncclSend(mine, (size_t)hi * M, ncclFloat32, prev, c->comm, st));
      RCCL_TRY(ncclRecv(recv + (size_t)lo * M, (size_t)hi * M, ncclFloat32, next, c->comm, st));
    }
    RCCL_TRY(ncclGroupEnd());
    return MDR_OK;
  }
  if (!c->host.sendrecv) return fail(MDR_ESTATE, "no communicator for the ring halo");
  HIP_TRY(hipStreamSynchronize(st));
  const int64_t b = (int64_t)sizeof(float) * M;
  if (lo)
    if (int r = c->host.sendrecv(c->host.user, mine + (size_t)hi * M, lo * b, next, recv, lo * b, prev, 1))
      return fail(MDR_ERCCL, "host sendrecv callback failed (" + std::to_string(r) + ")");
  if (hi)
    if (int r = c->host.sendrecv(c->host.user, mine, hi * b, prev, recv + (size_t)lo * M, hi * b, next, 2))
      return fail(MDR_ERCCL, "host sendrecv callback failed (" + std::to_string(r) + ")");
  return MDR_OK;
}

unsigned long long* slab_at(mdr_ctx* c, int r) { return c->d_slab + (size_t)((r % 3 + 3) % 3) * c->slab_len; }

// All count slabs to zero with a kernel, never hipMemsetAsync: these launch sequences are captured
// into graphs (mdr_rollout, mdr_actor_rollout), and on ROCm 7.2 a captured memset node wrote
// non-zero words (host stack addresses, 0x7fff....) into the slabs on every replay after the
// first (profiles/r05b_graph_memset_bisect.log: the slab only the memset touches, with every other
// node of the graph removed in turn; tools/graph_memset_repro.hip), which the chained actor's
// rollout read as counts of ~1e14 W in its first two ticks
int zero_slabs(mdr_ctx* c, hipStream_t st) {
  hipLaunchKernelGGL(k_zero_u64, dim3(1), dim3(256), 0, st, c->d_slab, (int64_t)kSlabs * c->slab_len);
  LAUNCH_CHECK("k_zero_u64");
  return MDR_OK;
}

int check_mode(int m) {
  return m == MDR_ACT_BUFFER || m == MDR_ACT_RANDOM || m == MDR_ACT_ALWAYS_ON ||
         m == MDR_ACT_BANGBANG || m == MDR_ACT_DEADBAND_BANGBANG;
}

bool lookahead_ok(int m) { return m != MDR_ACT_BUFFER; }

TickArgs to_tick(const mdr_tick* t) { return TickArgs{t->t_od_prev, t->solar, t->s_prev, t->tick}; }

// k_step_pipe depth measured on MI355X (profiles/r01b_kbench_pipe.log): 2 tiles per wave up to
// ~1.5M houses per shard, 4 above
int default_tpw(int64_t n) { return n <= 1572864 ? 2 : 4; }

// phase 1 into the current slab
int launch_counts(mdr_ctx* c, const uint8_t* action, int mode, uint64_t tick, const TickArgs* tkp,
                  hipStream_t st) {
  int m = mode;
  if (m == MDR_ACT_BANGBANG || m == MDR_ACT_DEADBAND_BANGBANG)
    return fail(MDR_EARG, "phase 1 with a bang-bang action source: use mdr_step lookahead or a BUFFER");
  hipLaunchKernelGGL(k_power_counts, dim3(blocks(c->kp.n, 256 * kPcHouses)), dim3(256), 0, st, c->kp, action, m,
                     tick, tkp, slab_at(c, c->ring));
  LAUNCH_CHECK("k_power_counts");
  return MDR_OK;
}

// parameter-derived state (the fast-division range flag) after a change; called before any
// launch sequence is captured, so graphs never contain it
int refresh_if_dirty(mdr_ctx* c, hipStream_t st) {
  if (!c->coef_dirty) return MDR_OK;
  HIP_TRY(hipMemsetAsync(c->d_flags, 0, sizeof(int), st));
  hipLaunchKernelGGL(k_refresh, dim3(blocks(c->kp.n, 256)), dim3(256), 0, st, c->kp, c->d_flags);
  LAUNCH_CHECK("k_refresh");
  c->coef_dirty = false;
  return MDR_OK;
}

int greedy_scratch(mdr_ctx* c, int64_t n);
int launch_gq_keys(mdr_ctx* c, hipStream_t st, unsigned long long* slab, bool local_map = true);
int gq_hist_produce(mdr_ctx* c, hipStream_t st);
// the histogram select's per-house codes (gq_code, 4 B) live in the sort form's key buffer
uint32_t* gq_codes(mdr_ctx* c) { return reinterpret_cast<uint32_t*>(c->g_key); }

// k_step launch with explicit count slabs; reward_lag: the launch writes the previous tick's
// reward from `cur` (nullptr: none), see k_step_t

int launch_step_on(mdr_ctx* c, const uint8_t* action, int mode, TickArgs tk, const TickArgs* tkp,
                   double* reward, int lookahead, int ctrl, uint8_t* ctrl_out, double* p_out,
                   const unsigned long long* cur, unsigned long long* nxt, unsigned long long* zer,
                   int reward_lag, hipStream_t st) {
  if (int rc = refresh_if_dirty(c, st)) return rc;
  const KParams kp = c->kp;
  const bool gq = ctrl == MDR_CTRL_GREEDY_KEYS;
  if (gq) {
    if (int rc = greedy_scratch(c, kp.n)) return rc;
    ctrl = MDR_CTRL_NONE;
  }
#define MDR_LAUNCH_STEP(F, A, LA)                                                                     \
  hipLaunchKernelGGL((k_step_t<2, F, A, LA>), dim3(blocks(kp.n, 512)), dim3(256), 0, st, kp, action, mode, \
                     tk, tkp, cur, reward, ctrl, ctrl_out, p_out, lookahead, nxt, zer, c->d_pen_partial,    \
                     reward_lag)
  const bool hot_random = mode == MDR_ACT_RANDOM && lookahead == MDR_ACT_RANDOM;
  const bool hot_buffer = mode == MDR_ACT_BUFFER && lookahead == 0;
  // software-pipelined form of the two hot configurations (k_step_pipe): individual_L2, <= 4
  // capacity classes, no controller output, no reward lag, 2-byte aligned action rows
  const bool pipe_ok = c->tpw >= 1 && c->fastdiv && (hot_random || hot_buffer) &&
                       kp.penalty_mode == MDR_PEN_INDIVIDUAL_L2 && kp.n_cap <= kPipeMaxCap &&
                       ctrl == MDR_CTRL_NONE && !reward_lag && (!action || ((uintptr_t)action & 1u) == 0);
  if (pipe_ok) {
    int tpw = c->tpw >= 8 ? 8 : c->tpw >= 4 ? 4 : c->tpw >= 2 ? 2 : 1;
    if (hot_buffer) tpw = tpw >= 4 ? 4 : 2;  // the instantiated buffer variants
    // the greedy controller's keys in the epilogue (buffer actions: the C3 loop; blocks of
    // kStepGqWaves waves), when its partials buffer holds this grid
    const unsigned nbg = blocks(blocks(kp.n, 128), kStepGqWaves * tpw);
    const bool epi = gq && hot_buffer && (int)nbg <= c->gq_parts_cap;
    const int nwv = epi ? kStepGqWaves : 4;
    const unsigned nb = blocks(blocks(kp.n, 128), nwv * tpw);  // every tile covered: ceil(tiles / (waves x tpw))
    const dim3 grid(nb);
    GqOut go{};
    if (epi) {
      if (int rc = gq_hist_produce(c, st)) return rc;
      go = GqOut{nullptr, gq_codes(c), c->g_part, c->g_hist, c->g_sel, c->g_map};
    }
#define MDR_LAUNCH_PIPE(T, A, LA, G)                                                                     \
  hipLaunchKernelGGL((k_step_pipe<T, A, LA, G>), grid, dim3(64 * nwv), 0, st, kp, action, tk, tkp, cur, reward, \
                     p_out, nxt, zer, go, GqfBufs{}, 0)
    if (hot_random) {
      if (tpw == 8) MDR_LAUNCH_PIPE(8, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0);
      else if (tpw == 4) MDR_LAUNCH_PIPE(4, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0);
      else if (tpw == 2) MDR_LAUNCH_PIPE(2, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0);
      else MDR_LAUNCH_PIPE(1, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0);
    } else if (epi) {
      if (tpw >= 4) MDR_LAUNCH_PIPE(4, MDR_ACT_BUFFER, 0, 1);
      else MDR_LAUNCH_PIPE(2, MDR_ACT_BUFFER, 0, 1);
    } else {
      if (tpw >= 4) MDR_LAUNCH_PIPE(4, MDR_ACT_BUFFER, 0, 0);
      else MDR_LAUNCH_PIPE(2, MDR_ACT_BUFFER, 0, 0);
    }
#undef MDR_LAUNCH_PIPE
    LAUNCH_CHECK("k_step_pipe");
    // (a lookahead's counts are in nxt: k_gq_keys leaves them, mdr_ctrl_greedy zeroes the slab)
    if (gq && !epi) return launch_gq_keys(c, st, lookahead ? nullptr : nxt);
    if (epi) {
      c->gq_nparts = (int)nb;
      c->gq_slab_zeroed = true;  // (the GQ epilogue zeroes its next slab; epi implies no lookahead)
    }
    return MDR_OK;
  }
  if (c->fastdiv) {
    if (hot_random) MDR_LAUNCH_STEP(true, MDR_ACT_RANDOM, MDR_ACT_RANDOM);
    else if (hot_buffer) MDR_LAUNCH_STEP(true, MDR_ACT_BUFFER, 0);
    else MDR_LAUNCH_STEP(true, -1, -1);
  } else {
    MDR_LAUNCH_STEP(false, -1, -1);
  }
#undef MDR_LAUNCH_STEP
  LAUNCH_CHECK("k_step");
  if (gq) return launch_gq_keys(c, st, lookahead ? nullptr : nxt);
  return MDR_OK;
}

int launch_step(mdr_ctx* c, const uint8_t* action, int mode, TickArgs tk, const TickArgs* tkp,
                double* reward, int lookahead, int ctrl, uint8_t* ctrl_out, double* p_out,
                hipStream_t st) {
  c->gq_keys_ready = false;
  c->fz_ready = false;
  int rc = launch_step_on(c, action, mode, tk, tkp, reward, lookahead, ctrl, ctrl_out, p_out,
                          slab_at(c, c->ring), slab_at(c, c->ring + 1), slab_at(c, c->ring + 2), 0, st);
  if (rc) return rc;
  c->ring = (c->ring + 1) % 3;
  c->counts_ready = lookahead != 0;
  c->gq_keys_ready = ctrl == MDR_CTRL_GREEDY_KEYS;
  return MDR_OK;
}

}  // namespace

extern "C" {

// an early first-window count (mdr_rollout_begin) is only valid for the mdr_rollout that follows
// it directly: every other entry point that changes the state or uses the slots discards it
static void drop_begun(mdr_ctx* c) {
  if (c && c->begun.on) {
    c->begun.on = false;
    c->wslab_dirty = true;
  }
  if (c) {
    c->gq_keys_ready = false;  // (every such entry point may change the state)
    c->fz_ready = false;
  }
}

#ifndef MDR_SRC_HASH
#define MDR_SRC_HASH "unstamped0000000"
#endif
const char* mdr_build_id(void) { return "MDR_SRC_HASH:" MDR_SRC_HASH; }

int mdr_abi_version(void) { return MDR_ABI_VERSION; }

int mdr_abi_sizes(int64_t* out, int n) {
  const int64_t v[9] = {(int64_t)sizeof(mdr_config), (int64_t)sizeof(mdr_soa), (int64_t)sizeof(mdr_tick),
                        (int64_t)sizeof(mdr_pop_spec), (int64_t)sizeof(mdr_obs_spec),
                        (int64_t)sizeof(mdr_obs_scalars), (int64_t)sizeof(mdr_actor_spec),
                        (int64_t)sizeof(mdr_interp_spec), (int64_t)sizeof(mdr_actor_net)};
  int k = 0;
  for (; out && k < n && k < 9; ++k) out[k] = v[k];
  return k;
}

const char* mdr_last_error(void) { return g_err.c_str(); }

int mdr_graph_info(mdr_ctx* c, int64_t* out, int n) {
  if (!c || !out || n < 0) return fail(MDR_EARG, "mdr_graph_info: bad argument");
  const int64_t v[6] = {(int64_t)c->graphs.size(), (int64_t)c->actor_graphs.size(), c->graph_launches[0],
                        c->graph_launches[1], c->graphs_guarded, c->graph_nodes_checked};
  int k = 0;
  for (; k < n && k < 6; ++k) out[k] = v[k];
  return k;
}

// the parameters of a memset node captured in this library's context, against
// what was passed, and what its replays leave in the slabs.  Captures hipMemsetAsync(d_slab, 0, all
// slabs) exactly as the r04 rollouts did, outside capture_graph (whose guard refuses memset nodes).
// out[0..12] = {nodes, memset nodes, dst == d_slab, value, elementSize, width, height, pitch,
// bytes passed, non-zero 64-bit words after replay 1 (slabs pre-filled with 0xA5), after replay 2
// (re-filled), after replay 3 (not re-filled), non-zero words after a kernel (k_zero_u64) zeroing}
int mdr_graph_memset_probe(mdr_ctx* c, int64_t* out, int n, void* stream) {
  drop_begun(c);
  if (!c || !out || n < 13) return fail(MDR_EARG, "mdr_graph_memset_probe: need out[13]");
  c->counts_ready = false;  // (the slabs are overwritten)
  for (int k = 0; k < n; ++k) out[k] = 0;
  hipStream_t st = S(stream);
  HIP_TRY(hipStreamSynchronize(st));
  if (!c->cap_stream) HIP_TRY(hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking));
  const size_t bytes = (size_t)kSlabs * c->slab_len * sizeof(unsigned long long);
  const size_t words = bytes / 8;
  hipGraph_t g;
  HIP_TRY(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal));
  hipError_t e = hipMemsetAsync(c->d_slab, 0, bytes, c->cap_stream);
  hipError_t e2 = hipStreamEndCapture(c->cap_stream, &g);
  if (e != hipSuccess || e2 != hipSuccess) return fail(MDR_EHIP, "memset probe: capture failed");
  size_t nn = 0;
  hipGraphGetNodes(g, nullptr, &nn);
  std::vector<hipGraphNode_t> nodes(nn);
  if (nn) hipGraphGetNodes(g, nodes.data(), &nn);
  out[0] = (int64_t)nn;
  for (size_t i = 0; i < nn; ++i) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[i], &t) != hipSuccess || t != hipGraphNodeTypeMemset) continue;
    out[1] += 1;
    hipMemsetParams mp{};
    if (hipGraphMemsetNodeGetParams(nodes[i], &mp) == hipSuccess) {
      out[2] = mp.dst == (void*)c->d_slab;
      out[3] = (int64_t)mp.value;
      out[4] = (int64_t)mp.elementSize;
      out[5] = (int64_t)mp.width;
      out[6] = (int64_t)mp.height;
      out[7] = (int64_t)mp.pitch;
    }
  }
  out[8] = (int64_t)bytes;
  hipGraphExec_t ex;
  e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return fail(MDR_EHIP, std::string("memset probe: instantiate: ") + hipGetErrorString(e));
  std::vector<unsigned long long> h(words);
  auto nonzero = [&](int64_t* o) -> int {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(h.data(), c->d_slab, bytes, hipMemcpyDeviceToHost));
    int64_t z = 0;
    for (size_t i = 0; i < words; ++i) z += h[i] != 0ull;
    *o = z;
    return MDR_OK;
  };
  int rc = MDR_OK;
  for (int r = 0; r < 3 && !rc; ++r) {
    if (r < 2) {
      hipMemsetAsync(c->d_slab, 0xA5, bytes, st);
    }
    if (hipGraphLaunch(ex, st) != hipSuccess) rc = fail(MDR_EHIP, "memset probe: launch");
    else rc = nonzero(&out[9 + r]);
  }
  hipGraphExecDestroy(ex);
  if (rc) return rc;
  if ((rc = zero_slabs(c, st))) return rc;
  return nonzero(&out[12]);
}

int mdr_create(mdr_ctx** out, const mdr_config* cfg) {
  if (!out || !cfg) return fail(MDR_EARG, "mdr_create: null argument");
  if (cfg->abi_version != MDR_ABI_VERSION) return fail(MDR_EARG, "mdr_create: ABI version mismatch");
  if (cfg->n_local < 1 || cfg->n_global < cfg->n_local || cfg->global_offset < 0 ||
      cfg->global_offset + cfg->n_local > cfg->n_global)
    return fail(MDR_EARG, "mdr_create: bad shard geometry");
  if (cfg->n_local >= ((int64_t)1 << 29))
    return fail(MDR_EARG, "mdr_create: n_local must be < 2^29 (32-bit byte offsets); shard across GPUs");
  if (cfg->n_cap < 1 || cfg->n_cap > MDR_MAX_CAP) return fail(MDR_EARG, "mdr_create: n_cap out of range");
  if (cfg->dt < 0) return fail(MDR_EARG, "mdr_create: negative dt");
  if (cfg->penalty_mode < 0 || cfg->penalty_mode > 3) return fail(MDR_EARG, "mdr_create: bad penalty mode");
  HIP_TRY(hipSetDevice(cfg->device));
  mdr_ctx* c = new mdr_ctx();
  c->cfg = *cfg;
  KParams& k = c->kp;
  k.n = cfg->n_local;
  k.goff = cfg->global_offset;
  k.n_global = cfg->n_global;
  k.dt = cfg->dt;
  k.L = cfg->lockout_duration;
  k.n_cap = cfg->n_cap;
  k.penalty_mode = cfg->penalty_mode;
  k.deadband = cfg->deadband;
  k.alpha_temp = cfg->alpha_temp;
  k.alpha_sig = cfg->alpha_sig;
  k.norm_temp = cfg->norm_temp;
  k.norm_sig = cfg->norm_sig;
  k.alpha_ind_l2 = cfg->alpha_ind_l2;
  k.alpha_common_l2 = cfg->alpha_common_l2;
  k.alpha_common_max = cfg->alpha_common_max;
  k.seed = cfg->seed;
  // capacity tables with the reference's expressions: hvac.py:94-97 and
  // environment_properties.py:92-98  (-1 * cap / (1 + lcf), cap / cop)
  double tab[2 * MDR_MAX_CAP] = {};
  for (int i = 0; i < cfg->n_cap; ++i) {
    tab[i] = (-1.0 * cfg->cap_table[i]) / (1.0 + cfg->lcf);
    tab[MDR_MAX_CAP + i] = cfg->cap_table[i] / cfg->cop;
  }
  auto cleanup = [&](int rc) { mdr_destroy(c); return rc; };
  if (hipMalloc(&c->d_tables, sizeof(tab)) != hipSuccess) return cleanup(fail(MDR_ENOMEM, "tables"));
  if (hipMemcpy(c->d_tables, tab, sizeof(tab), hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(MDR_EHIP, "tables copy"));
  k.q_on = c->d_tables;
  k.p_on = c->d_tables + MDR_MAX_CAP;
  if (hipMalloc(&c->d_flags, 16) != hipSuccess || hipMemset(c->d_flags, 0, 16) != hipSuccess)
    return cleanup(fail(MDR_ENOMEM, "flags"));  // [0] params_bad, [1..2] the actor's fp16-range counts
  if (hipMalloc(&c->d_tickets, kTicketWords * sizeof(unsigned)) != hipSuccess ||
      hipMemset(c->d_tickets, 0, kTicketWords * sizeof(unsigned)) != hipSuccess)
    return cleanup(fail(MDR_ENOMEM, "tickets"));
  k.params_bad = c->d_flags;
  {
    // the fast division is provably exact for dt < 2^20 s and |q_on| < 2^40 W (mdr_device.h)
    bool ok = cfg->dt < (1 << 20);
    for (int i = 0; i < cfg->n_cap; ++i) ok = ok && fabs(tab[i]) < 1099511627776.0;
    k.fast_tick_ok = ok ? 1 : 0;
  }
  c->slab_len = kCountShards * cfg->n_cap;
  if (hipMalloc(&c->d_slab, kSlabs * c->slab_len * sizeof(unsigned long long)) != hipSuccess)
    return cleanup(fail(MDR_ENOMEM, "count slabs"));
  if (hipMemset(c->d_slab, 0, kSlabs * c->slab_len * sizeof(unsigned long long)) != hipSuccess)
    return cleanup(fail(MDR_EHIP, "count slabs memset"));
  c->tpw = default_tpw(cfg->n_local);
  if (cfg->n_cap <= kWindowCap) {
    // a window count slot: sharded slab | reduced counts (mdr_kernels.hip)
    c->wslab_len = kWindowMax * kCountShards * cfg->n_cap + kWindowMax * cfg->n_cap + kWindowMax * kWindowRec;
    // 64-house lane groups of every wave tile a count / step-window grid launches: the grids round
    // the tiles up to whole blocks (up to kCountWaves tiles per block), and the waves of a ragged
    // last block store and load the mask rows of their (empty) tiles too
    const size_t tiles = ((size_t)cfg->n_local + 64 * kWinHpt - 1) / (64 * kWinHpt);
    const size_t tiles64 = (tiles + kCountWaves) / kCountWaves * kCountWaves * kWinHpt + 1;
    c->onb_bytes = tiles64 * kWindowMax * sizeof(uint64_t);
    c->wah_bytes = ((size_t)cfg->n_local + 1) * sizeof(uint32_t);
    if (hipMalloc(&c->d_wslab, 3 * sizeof(unsigned long long) * c->wslab_len) != hipSuccess ||
        hipMalloc(&c->d_onb, c->onb_bytes) != hipSuccess || hipMalloc(&c->d_wah, c->wah_bytes) != hipSuccess)
      return cleanup(fail(MDR_ENOMEM, "window count slabs"));
  } else {
    c->win = 0;
  }
  c->pen_blocks = (int)blocks(cfg->n_local, 512);  // = k_step_t grid
  if (hipMalloc(&c->d_pen_partial, 2 * sizeof(double) * c->pen_blocks) != hipSuccess ||
      hipMalloc(&c->d_partial2, 2 * sizeof(double)) != hipSuccess)
    return cleanup(fail(MDR_ENOMEM, "penalty partials"));
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return cleanup(fail(MDR_EHIP, "event"));
  for (int i = 0; i < kSlabs; ++i)
    if (hipEventCreateWithFlags(&c->ev_k1[i], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_ar[i], hipEventDisableTiming) != hipSuccess)
      return cleanup(fail(MDR_EHIP, "event"));
  if (hipEventCreateWithFlags(&c->ev_pc, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(MDR_EHIP, "event"));
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess ||
      c->n_cu < 1)
    c->n_cu = 256;
  *out = c;
  return MDR_OK;
}

static void destroy_graphs(mdr_ctx* c) {
  for (auto& g : c->graphs) hipGraphExecDestroy(g.second.first);
  c->graphs.clear();
  for (auto& g : c->actor_graphs) hipGraphExecDestroy(g.second);
  c->actor_graphs.clear();
}

int mdr_destroy(mdr_ctx* c) {
  if (!c) return MDR_OK;
  hipSetDevice(c->cfg.device);
  hipDeviceSynchronize();
  destroy_graphs(c);
  hipFree(c->d_actor);
  hipFree(c->d_actor_raw);
  hipFree(c->d_chain);
  hipFree(c->d_interp);
  hipFree(c->d_act);
  hipFree(c->d_halo);
  hipFree(c->d_stats);
  hipFree(c->d_obs_sc);
  hipFree(c->d_tables);
  hipFree(c->d_flags);
  hipFree(c->d_slab);
  hipFree(c->d_wslab);
  hipFree(c->d_onb);
  hipFree(c->d_wah);
  hipFree(c->d_onb2);
  hipFree(c->d_wah2);
  hipFree(c->d_pen_partial);
  hipFree(c->d_partial2);
  hipFree(c->d_ticks);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  for (int i = 0; i < kSlabs; ++i) {
    if (c->ev_k1[i]) hipEventDestroy(c->ev_k1[i]);
    if (c->ev_ar[i]) hipEventDestroy(c->ev_ar[i]);
  }
  if (c->ev_pc) hipEventDestroy(c->ev_pc);
  if (c->comm_stream) hipStreamDestroy(c->comm_stream);
  if (c->cap_stream) hipStreamDestroy(c->cap_stream);
  hipFree(c->g_key); hipFree(c->g_key2); hipFree(c->g_ps); hipFree(c->g_incl);
  hipFree(c->g_idx); hipFree(c->g_idx2); hipFree(c->g_ls); hipFree(c->g_tmp);
  hipFree(c->g_kpos); hipFree(c->g_extra);
  hipFree(c->g_part); hipFree(c->g_hist); hipFree(c->g_sel); hipFree(c->g_win);
  hipFree(c->g_sorted); hipFree(c->g_map); hipFree(c->g_range); hipFree(c->g_tickets);
  hipFree(c->d_tickets);
  hipFree(c->fz.par[0]); hipFree(c->fz.bkt[0]); hipFree(c->fz.mbkt); hipFree(c->fz.map[0]); hipFree(c->fz.sel);
  hipFree(c->fz.dec);
  hipFree(c->fz.stamps);
  hipFree(c->d_c5);
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
  return MDR_OK;
}

int mdr_set_option(mdr_ctx* c, int option, int64_t value) {
  drop_begun(c);
  if (!c) return fail(MDR_EARG, "mdr_set_option: null ctx");
  switch (option) {
    case MDR_OPT_STEP_TPW:
      if (value < -1 || value > 8) return fail(MDR_EARG, "mdr_set_option: STEP_TPW outside -1..8");
      c->tpw = value < 0 ? default_tpw(c->kp.n) : (int)value;
      break;
    case MDR_OPT_FASTDIV: c->fastdiv = value != 0; break;
    case MDR_OPT_WINDOW_PIPELINE: c->win_pipe = value != 0; break;
    case MDR_OPT_SHARDED_OVERLAP: c->tick_overlap = value != 0; break;
    case MDR_OPT_GREEDY_SORT: c->greedy_sort = value != 0; break;
    case MDR_OPT_FORCE_HALO: c->force_halo = value != 0; break;
    case MDR_OPT_HALO_OVERLAP: c->halo_overlap = value != 0; break;
    case MDR_OPT_HALO_IN_COUNTS: c->halo_in_counts = value != 0; break;
    case MDR_OPT_GQ_BAND: c->gq_band = value != 0; break;
    case MDR_OPT_GQ_FUSED:  // (the other form's key map was last fitted to an older state: re-fit it)
      c->gq_map_stale = c->gq_map_stale || c->gq_fused != (value != 0);
      c->gq_fused = value != 0;
      break;
    case MDR_OPT_GQ_ADAPTIVE: c->gq_adaptive = value != 0; break;
    case MDR_OPT_ACTOR_GENERIC: c->actor_generic = value != 0; break;
    case MDR_OPT_ACTOR_FP32_FORM:
      if (value != MDR_FP32_F16_SPLIT && value != MDR_FP32_BF16_SPLIT3)
        return fail(MDR_EARG, "mdr_set_option: ACTOR_FP32_FORM must be MDR_FP32_F16_SPLIT or MDR_FP32_BF16_SPLIT3");
      c->actor_fp32_bf16 = value == MDR_FP32_BF16_SPLIT3;
      c->actor_key.clear();  // (packed again for the form)
      break;
    case MDR_OPT_WINDOW_THERMAL:
      if (value != MDR_THERMAL_EXACT && value != MDR_THERMAL_AFFINE)
        return fail(MDR_EARG, "mdr_set_option: WINDOW_THERMAL must be MDR_THERMAL_EXACT or _AFFINE");
      c->thermal = (int)value;
      break;
    default: return fail(MDR_EARG, "mdr_set_option: unknown option");
  }
  HIP_TRY(hipDeviceSynchronize());  // cached graphs may be in flight
  destroy_graphs(c);
  return MDR_OK;
}

int mdr_bind(mdr_ctx* c, const mdr_soa* s) {
  drop_begun(c);
  if (!c || !s) return fail(MDR_EARG, "mdr_bind: null argument");
  if (!s->t_air || !s->t_mass || !s->hvac || !s->ua || !s->ca || !s->cm || !s->hm || !s->target ||
      !s->cap_idx)
    return fail(MDR_EARG, "mdr_bind: null array");
  KParams& k = c->kp;
  k.t_air = s->t_air;
  k.t_mass = s->t_mass;
  k.hvac = s->hvac;
  k.ua = s->ua;
  k.ca = s->ca;
  k.cm = s->cm;
  k.hm = s->hm;
  k.target = s->target;
  k.cap_idx = s->cap_idx;
  c->bound = true;
  c->counts_ready = false;
  c->coef_dirty = true;
  c->gq_map_stale = true;
  c->gq_s1 = c->gq_s2 = NAN;
  for (auto& g : c->graphs) hipGraphExecDestroy(g.second.first);
  c->graphs.clear();
  return MDR_OK;
}

int mdr_populate(mdr_ctx* c, const mdr_pop_spec* sp, void* stream) {
  drop_begun(c);
  if (!c || !sp) return fail(MDR_EARG, "mdr_populate: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_populate: context not bound");
  if (sp->n_draw < 0 || sp->n_draw > MDR_MAX_CAP) return fail(MDR_EARG, "mdr_populate: n_draw out of range");
  for (int k = 0; k < sp->n_draw; ++k)
    if (sp->draw_idx[k] >= c->cfg.n_cap) return fail(MDR_EARG, "mdr_populate: draw_idx outside the cap table");
  PopArgs a{sp->target_temp, sp->std_target, sp->thermo_lo, sp->thermo_hi, sp->ca, sp->cm, sp->hm,
            sp->init_air, sp->init_mass, sp->n_draw, {}};
  memcpy(a.draw_idx, sp->draw_idx, sizeof(a.draw_idx));
  hipLaunchKernelGGL(k_populate, dim3(blocks(c->kp.n, 256)), dim3(256), 0, S(stream), c->kp, a);
  LAUNCH_CHECK("k_populate");
  c->counts_ready = false;
  c->coef_dirty = true;
  c->gq_map_stale = true;
  c->gq_s1 = c->gq_s2 = NAN;
  return MDR_OK;
}

int mdr_power_counts(mdr_ctx* c, const uint8_t* action, int mode, uint64_t tick, void* stream) {
  drop_begun(c);
  if (!c) return fail(MDR_EARG, "mdr_power_counts: null ctx");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_power_counts: context not bound");
  if (!check_mode(mode) || (mode == MDR_ACT_BUFFER && !action))
    return fail(MDR_EARG, "mdr_power_counts: bad action source");
  // (re)compute this tick's counts from zero (a previous lookahead may have filled the slab)
  HIP_TRY(hipMemsetAsync(slab_at(c, c->ring), 0, c->slab_len * sizeof(unsigned long long), S(stream)));
  int rc = launch_counts(c, action, mode, tick, nullptr, S(stream));
  if (rc) return rc;
  c->counts_ready = true;
  return MDR_OK;
}

int mdr_counts_buffer(mdr_ctx* c, int64_t** ptr, int* len) {
  if (!c || !ptr || !len) return fail(MDR_EARG, "mdr_counts_buffer: null argument");
  *ptr = reinterpret_cast<int64_t*>(slab_at(c, c->ring));
  *len = c->slab_len;
  return MDR_OK;
}

int mdr_step(mdr_ctx* c, const uint8_t* action, int mode, const mdr_tick* tick, double* reward,
             int lookahead, int ctrl, uint8_t* ctrl_out, double* p_out, void* stream) {
  drop_begun(c);
  if (!c || !tick || !reward) return fail(MDR_EARG, "mdr_step: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_step: context not bound");
  if (!check_mode(mode) || (mode == MDR_ACT_BUFFER && !action))
    return fail(MDR_EARG, "mdr_step: bad action source");
  if (lookahead && (!check_mode(lookahead) || !lookahead_ok(lookahead)))
    return fail(MDR_EARG, "mdr_step: bad lookahead source");
  if (ctrl < MDR_CTRL_NONE || ctrl > MDR_CTRL_GREEDY_KEYS) return fail(MDR_EARG, "mdr_step: bad ctrl");
  if (!c->counts_ready) return fail(MDR_ESTATE, "mdr_step: no cluster-power counts for this tick (call mdr_power_counts)");
  return launch_step(c, action, mode, to_tick(tick), nullptr, reward, lookahead, ctrl, ctrl_out, p_out,
                     S(stream));
}

int mdr_penalty_partials(mdr_ctx* c, void* stream) {
  if (!c) return fail(MDR_EARG, "mdr_penalty_partials: null ctx");
  hipLaunchKernelGGL(k_pen_reduce, dim3(1), dim3(256), 0, S(stream), c->d_pen_partial, c->pen_blocks,
                     c->d_partial2);
  LAUNCH_CHECK("k_pen_reduce");
  return MDR_OK;
}

int mdr_penalty_buffer(mdr_ctx* c, double** ptr) {
  if (!c || !ptr) return fail(MDR_EARG, "mdr_penalty_buffer: null argument");
  *ptr = c->d_partial2;
  return MDR_OK;
}

int mdr_reward_finalize(mdr_ctx* c, const mdr_tick* tick, double* reward, void* stream) {
  if (!c || !tick || !reward) return fail(MDR_EARG, "mdr_reward_finalize: null argument");
  // the tick's counts are in the slab just before the current one
  hipLaunchKernelGGL(k_reward_finalize, dim3(blocks(c->kp.n, 256)), dim3(256), 0, S(stream), c->kp,
                     to_tick(tick), slab_at(c, c->ring - 1), c->d_partial2, reward);
  LAUNCH_CHECK("k_reward_finalize");
  return MDR_OK;
}

// ------------------------------------------------------------------------------------ rollout
// n 32-byte records from host memory into device memory on `st`, through kernel arguments:
// nothing on the host waits for the device, and the host array may be reused on return
static int stage_recs(const void* src, int n, void* dst, hipStream_t st) {
  const Rec32* s = static_cast<const Rec32*>(src);
  Rec32* d = static_cast<Rec32*>(dst);
  for (int off = 0; off < n; off += kStageRecs) {
    const int m = n - off < kStageRecs ? n - off : kStageRecs;
    StagePack pk;
    memcpy(pk.r, s + off, (size_t)m * sizeof(Rec32));
    hipLaunchKernelGGL(k_stage32, dim3(1), dim3(kStageRecs), 0, st, pk, m, d + off);
    LAUNCH_CHECK("k_stage32");
  }
  return MDR_OK;
}

static int ensure_ticks(mdr_ctx* c, int n) {
  if (n > c->ticks_cap) {
    HIP_TRY(hipDeviceSynchronize());  // queued graphs may still read the old buffers
    hipFree(c->d_ticks);
    hipFree(c->d_obs_sc);
    c->d_ticks = nullptr;
    c->d_obs_sc = nullptr;
    int cap = n < 128 ? 128 : n;
    HIP_TRY(hipMalloc(&c->d_ticks, cap * sizeof(TickArgs)));
    HIP_TRY(hipMalloc(&c->d_obs_sc, (size_t)cap * 4 * sizeof(double)));
    c->ticks_cap = cap;
    destroy_graphs(c);
  }
  return MDR_OK;
}

static int stage_ticks(mdr_ctx* c, int n, const mdr_tick* ticks, hipStream_t st) {
  if (int rc = ensure_ticks(c, n)) return rc;
  // stream order: every earlier launch reading d_ticks (a replayed graph) precedes this write
  return stage_recs(ticks, n, c->d_ticks, st);
}

// every node of a captured graph must be a kernel (the launch sequences hold nothing else); a memset
// node fails the capture with MDR_EHIP.  Counts the graphs checked (mdr_graph_info[4]).
static int graph_memset_guard(mdr_ctx* c, hipGraph_t g) {
  size_t nn = 0;
  HIP_TRY(hipGraphGetNodes(g, nullptr, &nn));
  std::vector<hipGraphNode_t> nodes(nn);
  if (nn) HIP_TRY(hipGraphGetNodes(g, nodes.data(), &nn));
  for (size_t i = 0; i < nn; ++i) {
    hipGraphNodeType t;
    HIP_TRY(hipGraphNodeGetType(nodes[i], &t));
    if (t == hipGraphNodeTypeMemset)
      return fail(MDR_EHIP, "capture: graph node " + std::to_string(i) + " of " + std::to_string(nn) +
                                " is a memset (captured launch sequences must zero with kernels)");
  }
  c->graphs_guarded += 1;
  c->graph_nodes_checked += (int64_t)nn;
  return MDR_OK;
}

// Capture a launch sequence into an executable graph on the context's own capture stream (the
// capture executes nothing), so the graph can then be launched on ANY caller stream — the null
// stream included — with no cross-stream synchronisation around each replay.
extern "C++" template <typename F>
static int capture_graph(mdr_ctx* c, F&& launches, hipGraphExec_t* out) {
  if (!c->cap_stream) HIP_TRY(hipStreamCreateWithFlags(&c->cap_stream, hipStreamNonBlocking));
  hipGraph_t g;
  HIP_TRY(hipStreamBeginCapture(c->cap_stream, hipStreamCaptureModeThreadLocal));
  const int rc = launches(c->cap_stream);
  hipError_t e = hipStreamEndCapture(c->cap_stream, &g);
  if (rc) return rc;
  if (e != hipSuccess) return fail(MDR_EHIP, std::string("capture: ") + hipGetErrorString(e));
  // memset guard: a captured hipMemsetAsync node left non-zero words in the count slabs on every
  // replay after the first (zero_slabs) — no captured graph may contain one
  if (int grc = graph_memset_guard(c, g)) {
    hipGraphDestroy(g);
    return grc;
  }
  e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return fail(MDR_EHIP, std::string("instantiate: ") + hipGetErrorString(e));
  // upload the executable graph now (capture time), not on its first replay
  e = hipGraphUpload(*out, c->cap_stream);
  if (e != hipSuccess) return fail(MDR_EHIP, std::string("graph upload: ") + hipGetErrorString(e));
  return MDR_OK;
}

// ---- windowed rollout (k_step_window): open-loop action sources, individual_L2
// SIMPLE = deadband 0, norm_temp 1, and reward weights whose signal / temperature penalties are
// >= +0 (k_step_window forms -(a + s) as (-a) + (-s), exact for such operands)
static bool win_simple(const mdr_ctx* c) {
  return c->kp.deadband == 0.0 && c->kp.norm_temp == 1.0 && c->kp.alpha_temp >= 0.0 && !std::signbit(c->kp.alpha_temp) &&
         c->kp.alpha_sig >= 0.0 && !std::signbit(c->kp.alpha_sig) && c->kp.norm_sig > 0.0;
}

// (the lookahead's FSM runs on unsaturated seconds-since-off in a signed offset form: L <= 2^30 - 1,
// dt <= 2^25, so a saturated value plus 33 ticks of dt and L - 32 dt stay inside int32 —
// mdr_kernels.hip win_run_t)
static bool window_ok(const mdr_ctx* c, int mode) {
  return c->win > 0 && c->d_wslab && c->kp.n_cap <= kWindowCap && c->kp.penalty_mode == MDR_PEN_INDIVIDUAL_L2 &&
         c->kp.L < (1 << 30) && c->kp.dt >= 0 && c->kp.dt <= (1 << 25) &&
         (mode == MDR_ACT_RANDOM || mode == MDR_ACT_ALWAYS_ON || mode == MDR_ACT_BUFFER);
}

// the window slots' shard part is zero between rollouts (k_win_reduce zeroes what it reads);
// after allocation or a failed launch sequence it is cleared once, outside any graph
static int wslab_clean(mdr_ctx* c, hipStream_t st) {
  if (!c->wslab_dirty || !c->d_wslab) return MDR_OK;
  HIP_TRY(hipMemsetAsync(c->d_wslab, 0, 3 * sizeof(unsigned long long) * c->wslab_len, st));
  c->wslab_dirty = false;
  return MDR_OK;
}

static unsigned win_grid(const mdr_ctx* c, int waves = 4) { return blocks(blocks(c->kp.n, 64 * kWinHpt), waves); }  // a tile per wave

extern "C" size_t mdr_window_onb_bytes(int64_t n_local, int waves) {
  if (n_local < 0 || waves < 1) return 0;
  const size_t tiles = ((size_t)n_local + 64 * kWinHpt - 1) / (64 * kWinHpt);
  return (tiles + waves - 1) / waves * waves * kWinHpt * kWindowMax * sizeof(uint64_t);
}

extern "C" int mdr_window_geometry_check(int64_t n_local, size_t onb_bytes, size_t wah_bytes) {
  if (n_local < 1) return fail(MDR_EARG, "window launch: no houses");
  const size_t need = std::max(mdr_window_onb_bytes(n_local, kCountWaves), mdr_window_onb_bytes(n_local, 4));
  if (onb_bytes < need)
    return fail(MDR_EARG, "window launch: ON-mask rows of " + std::to_string(onb_bytes) + " B, the launch geometry touches " +
                              std::to_string(need) + " B");
  if (wah_bytes < (size_t)n_local * sizeof(uint32_t))
    return fail(MDR_EARG, "window launch: end-word buffer shorter than the shard");
  return MDR_OK;
}

// the first window's FSM count: ticks from tk (staged) or tick0 + j (tk == nullptr), from the
// state's FSM words (w_in == nullptr) or from the end words of the previous window
// p_only: the count kernel's last block also does the window's P-only reduce (win_reduce_last),
// for a first window whose drivers ride on the step launch and whose shards need no allreduce
// the reduced per-tick class counts of a window slot (after its kWindowMax x 64 x n_cap shards)
static unsigned long long* win_red_ptr(const mdr_ctx* c, unsigned long long* slot) {
  return slot + (size_t)kWindowMax * kCountShards * c->kp.n_cap;
}

static int launch_count(mdr_ctx* c, int mode, const uint8_t* action, int64_t act_stride, const TickArgs* tk,
                        uint64_t tick0, int K, unsigned long long* slot, uint64_t* onb, uint32_t* wah,
                        const uint32_t* w_in, hipStream_t st, bool p_only = false) {
  if (int rc = mdr_window_geometry_check(c->kp.n, c->onb_bytes, c->wah_bytes)) return rc;
  const unsigned grid = win_grid(c, kCountWaves);
  unsigned* ticket = p_only ? c->d_tickets : nullptr;
#define MDR_COUNT(A)                                                                                  \
  hipLaunchKernelGGL((k_count_window<A, kWinHpt>), dim3(grid), dim3(64 * kCountWaves), 0, st, c->kp, action, act_stride, tk, \
                     tick0, K, slot, onb, wah, w_in, ticket)
  if (mode == MDR_ACT_RANDOM) MDR_COUNT(MDR_ACT_RANDOM);
  else if (mode == MDR_ACT_ALWAYS_ON) MDR_COUNT(MDR_ACT_ALWAYS_ON);
  else MDR_COUNT(MDR_ACT_BUFFER);
#undef MDR_COUNT
  LAUNCH_CHECK("k_count_window");
  return MDR_OK;
}

// one k_step_window launch: the (ACT, SIMPLE, KA, FORM) instantiation for this context; with
// step_events (mdr_time_step_kernels) hipExtLaunchKernel's start / stop events time it
static int launch_step_window(mdr_ctx* c, int mode, bool ka, const uint8_t* action, int64_t act_stride,
                              const TickArgs* tk, int K, int la_K, const double* rec, double* reward,
                              int64_t rew_stride, uint64_t* onb, uint32_t* wah, unsigned long long* next_slot,
                              const WinDrv& dv, hipStream_t st) {
  if (int rc = mdr_window_geometry_check(c->kp.n, c->onb_bytes, c->wah_bytes)) return rc;
  const unsigned grid = win_grid(c);
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (c->step_events) {
    HIP_TRY(hipEventCreate(&t0));
    c->step_events->push_back(t0);
    HIP_TRY(hipEventCreate(&t1));
    c->step_events->push_back(t1);
  }
  const KParams kp = c->kp;
#define MDR_SW_L(A, SI, KA_, FO)                                                                          \
  do {                                                                                                    \
    if (t0)                                                                                               \
      hipExtLaunchKernelGGL((k_step_window<A, kWinHpt, SI, KA_, FO>), dim3(grid), dim3(256), 0, st, t0, t1, 0, kp, \
                            action, act_stride, tk, K, la_K, rec, reward, rew_stride, onb, wah, next_slot, dv); \
    else                                                                                                  \
      hipLaunchKernelGGL((k_step_window<A, kWinHpt, SI, KA_, FO>), dim3(grid), dim3(256), 0, st, kp, action,  \
                         act_stride, tk, K, la_K, rec, reward, rew_stride, onb, wah, next_slot, dv);       \
  } while (0)
#define MDR_SW_F(A, SI, KA_)                                                            \
  do {                                                                                  \
    if (c->thermal == MDR_THERMAL_AFFINE) MDR_SW_L(A, SI, KA_, MDR_THERMAL_AFFINE);     \
    else MDR_SW_L(A, SI, KA_, MDR_THERMAL_EXACT);                                       \
  } while (0)
#define MDR_SW_K(A, SI)                         \
  do {                                          \
    if (ka) MDR_SW_F(A, SI, true);              \
    else MDR_SW_F(A, SI, false);                \
  } while (0)
#define MDR_SW_S(A)                             \
  do {                                          \
    if (win_simple(c)) MDR_SW_K(A, true);       \
    else MDR_SW_K(A, false);                    \
  } while (0)
  if (mode == MDR_ACT_RANDOM) MDR_SW_S(MDR_ACT_RANDOM);
  else if (mode == MDR_ACT_ALWAYS_ON) MDR_SW_S(MDR_ACT_ALWAYS_ON);
  else MDR_SW_S(MDR_ACT_BUFFER);
#undef MDR_SW_S
#undef MDR_SW_K
#undef MDR_SW_F
#undef MDR_SW_L
  LAUNCH_CHECK("k_step_window");
  return MDR_OK;
}

// n ticks as ceil(n / win) windows of near-equal size: a k_count_window for the first window, then
// per window k_win_reduce (shard sums -> counts + tick records; sharded: the shards are allreduced
// first) and one k_step_window (counting the next window's ticks).  Tick drivers come from tk
// (device, staged) for every window.
//
// host_ticks (direct launches, mdr_rollout without a graph; ids consecutive, checked by the caller):
// the first window's count and a P-only reduce (already issued by mdr_rollout_begin when counted)
// need only the tick ids; its step kernel then takes the drivers as kernel arguments
// (k_step_window<..., KA>), and the later windows' drivers are staged into tk behind it (their
// first reader is the first step kernel's lookahead... which reads tick ids only: tick0 + K + j).
//
// pipe (sharded, comm stream present): the count-ahead pipeline.  The FSM of an open-loop source
// needs no thermal state, so window w's count (from the FSM words at the end of window w-1) and
// the allreduce of its counts run on the comm stream, up to two windows ahead of the compute
// stream's reduce + step (which then has no lookahead): the allreduce latency hides behind the
// step kernels.  Two sets of ON-mask / end-word buffers alternate; events order the reuse.
static int window_launches(mdr_ctx* c, int n, const TickArgs* tk, const uint8_t* action, int64_t act_stride,
                           int mode, double* reward, int64_t rew_stride, double* p_out, bool shd,
                           hipStream_t st, bool counted = false, bool pipe = false,
                           const mdr_tick* host_ticks = nullptr, bool ka_red = false) {
  const int nw = (n + c->win - 1) / c->win;
  const int base = n / nw, rem = n % nw;
  auto wsz = [&](int w) { return base + (w < rem ? 1 : 0); };
  auto slot = [&](int w) { return c->d_wslab + (size_t)(w % 3) * c->wslab_len; };
  const KParams kp = c->kp;
  const int ncap = kp.n_cap;
  auto rec = [&](int w) {  // the slot's tick records, after its shards and reduced counts
    return reinterpret_cast<const double*>(slot(w) + (size_t)kWindowMax * kCountShards * ncap + (size_t)kWindowMax * ncap);
  };
  c->wslab_dirty = true;  // until the sequence is fully issued
  if (pipe) {
    hipStream_t cs = c->comm_stream;
    uint64_t* onbs[2] = {c->d_onb, c->d_onb2};
    uint32_t* wahs[2] = {c->d_wah, c->d_wah2};
    HIP_TRY(hipEventRecord(c->ev_pc, st));  // the state and staged ticks, before the first count
    HIP_TRY(hipStreamWaitEvent(cs, c->ev_pc, 0));
    int t0 = 0;
    for (int w = 0; w < nw; ++w) {
      const int K = wsz(w);
      // comm stream: count(w) + allreduce; count(w) reuses the buffers step(w - 2) read
      if (w >= 2) HIP_TRY(hipStreamWaitEvent(cs, c->ev_k1[(w - 2) % kSlabs], 0));
      const uint8_t* a = action ? action + (int64_t)t0 * act_stride : nullptr;
      // (the count kernel's last block sums its shards: one allreduce of K x n_cap totals, <= 1 KiB)
      if (int rc = launch_count(c, mode, a, act_stride, tk + t0, 0, K, slot(w), onbs[w % 2], wahs[w % 2],
                                w == 0 ? nullptr : wahs[(w - 1) % 2], cs, true))
        return rc;
      if (shd)
        if (int rc = comm_allreduce(c, win_red_ptr(c, slot(w)), (size_t)K * ncap, 0, cs)) return rc;
      HIP_TRY(hipEventRecord(c->ev_ar[w % kSlabs], cs));
      // compute stream: the tick records + step (no lookahead)
      HIP_TRY(hipStreamWaitEvent(st, c->ev_ar[w % kSlabs], 0));
      hipLaunchKernelGGL(k_win_records, dim3(1), dim3(kWindowMax), 0, st, kp, slot(w), K, tk + t0,
                         w == nw - 1 ? p_out : nullptr);
      LAUNCH_CHECK("k_win_records");
      if (int rc = launch_step_window(c, mode, false, a, act_stride, tk + t0, K, 0, rec(w),
                                      reward + (int64_t)t0 * rew_stride, rew_stride, onbs[w % 2], wahs[w % 2],
                                      slot(w), WinDrv{}, st))
        return rc;
      HIP_TRY(hipEventRecord(c->ev_k1[w % kSlabs], st));
      t0 += K;
    }
    c->wslab_dirty = false;
    return MDR_OK;
  }
  if (!counted) {  // (counted: mdr_rollout_begin launched the count and its P-only reduce already)
    // host_ticks: the P-only reduce of the first window (the drivers come with the step) — in the
    // count kernel's last block on one GPU, after the shards' allreduce when sharded
    if (int rc = launch_count(c, mode, action, act_stride, host_ticks ? nullptr : tk,
                              host_ticks ? host_ticks[0].tick : 0, wsz(0), slot(0), c->d_onb, c->d_wah, nullptr, st,
                              host_ticks && !shd))
      return rc;
    if (host_ticks && shd)
      if (int rc = comm_allreduce(c, slot(0), (size_t)wsz(0) * kCountShards * ncap, 0, st)) return rc;
    if (host_ticks && shd) {
      hipLaunchKernelGGL(k_win_reduce, dim3(wsz(0)), dim3(64 * ncap), 0, st, kp, slot(0), wsz(0),
                         (const TickArgs*)nullptr, (double*)nullptr);
      LAUNCH_CHECK("k_win_reduce (P only)");
    }
  }
  int t0 = 0;
  for (int w = 0; w < nw; ++w) {
    const int K = wsz(w), la = w + 1 < nw ? wsz(w + 1) : 0;
    const uint8_t* a = action ? action + (int64_t)t0 * act_stride : nullptr;
    if (host_ticks && w == 0) {
      // KA: the drivers ride on the step launch; the later windows' drivers are staged behind it
      WinDrv dv{};
      for (int j = 0; j < K; ++j) {
        const mdr_tick& h = host_ticks[j];
        dv.od_k[j] = h.t_od_prev + 273.0;  // (k_win_reduce's rec[0]: the same IEEE addition)
        dv.solar[j] = h.solar;
        dv.s_prev[j] = h.s_prev;
        if (fabs(h.t_od_prev) < 1048576.0 && fabs(h.solar) < 1099511627776.0) dv.ok |= 1u << j;  // (win_tick_record)
      }
      dv.tick0 = host_ticks[0].tick;
      if (nw == 1) dv.p_out = p_out;
      if (ka_red) dv.red = win_red_ptr(c, slot(0));  // (sharded, begun: P from the allreduced totals)
      if (int rc = launch_step_window(c, mode, true, a, act_stride, tk, K, la, rec(0), reward, rew_stride, c->d_onb,
                                      c->d_wah, slot(1), dv, st))
        return rc;
      if (n > K)
        if (int rc = stage_recs(host_ticks + K, n - K, const_cast<TickArgs*>(tk) + K, st)) return rc;
      t0 += K;
      continue;
    }
    // sharded: every rank's sharded per-tick class counts are summed first (exact integers; the
    // slot's shard part, K x 64 x n_cap values), so one reduce kernel yields the global counts
    if (shd)
      if (int rc = comm_allreduce(c, slot(w), (size_t)K * kCountShards * ncap, 0, st)) return rc;
    hipLaunchKernelGGL(k_win_reduce, dim3(K), dim3(64 * ncap), 0, st, kp, slot(w), K, tk + t0,
                       w == nw - 1 ? p_out : nullptr);
    LAUNCH_CHECK("k_win_reduce");
    if (int rc = launch_step_window(c, mode, false, a, act_stride, tk + t0, K, la, rec(w),
                                    reward + (int64_t)t0 * rew_stride, rew_stride, c->d_onb, c->d_wah, slot(w + 1),
                                    WinDrv{}, st))
      return rc;
    t0 += K;
  }
  c->wslab_dirty = false;
  return MDR_OK;
}

// the second ON-mask / end-word set of the count-ahead pipeline (allocated on first use)
static bool pipe_buffers(mdr_ctx* c) {
  if (c->d_onb2 && c->d_wah2) return true;
  if (hipMalloc(&c->d_onb2, c->onb_bytes) != hipSuccess || hipMalloc(&c->d_wah2, c->wah_bytes) != hipSuccess) {
    (void)hipGetLastError();
    hipFree(c->d_onb2);
    hipFree(c->d_wah2);
    c->d_onb2 = nullptr;
    c->d_wah2 = nullptr;
    return false;
  }
  return true;
}

// The launch sequence of a rollout with staged drivers (d_ticks), so a captured graph is reusable:
// the window sequence, or one step launch per tick (+ phase 1 where no lookahead counts ahead).
static int rollout_launches(mdr_ctx* c, int n, const uint8_t* action, int64_t act_stride, int mode,
                            double* reward, int64_t rew_stride, double* p_out, hipStream_t st) {
  if (window_ok(c, mode))
    return window_launches(c, n, c->d_ticks, action, act_stride, mode, reward, rew_stride, p_out, false, st);
  if (mode == MDR_ACT_BANGBANG || mode == MDR_ACT_DEADBAND_BANGBANG)
    return fail(MDR_EARG, "rollout: bang-bang sources need the per-step API (mdr_step with a lookahead)");
  if (int rc = zero_slabs(c, st)) return rc;
  c->ring = 0;
  const bool la = lookahead_ok(mode);
  for (int t = 0; t < n; ++t) {
    const uint8_t* a = action ? action + (int64_t)t * act_stride : nullptr;
    double* r = reward + (int64_t)t * rew_stride;
    if (!la || t == 0) {
      hipLaunchKernelGGL(k_power_counts, dim3(blocks(c->kp.n, 256 * kPcHouses)), dim3(256), 0, st, c->kp, a, mode,
                         (uint64_t)0, c->d_ticks + t, slab_at(c, c->ring));
      LAUNCH_CHECK("k_power_counts");
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->step_events) {
      HIP_TRY(hipEventCreate(&e0));
      c->step_events->push_back(e0);
      HIP_TRY(hipEventRecord(e0, st));
    }
    int rc = launch_step(c, a, mode, TickArgs{}, c->d_ticks + t, r, la ? mode : 0, MDR_CTRL_NONE,
                         nullptr, t == n - 1 ? p_out : nullptr, st);
    if (rc) return rc;
    if (c->step_events) {
      HIP_TRY(hipEventCreate(&e1));
      c->step_events->push_back(e1);
      HIP_TRY(hipEventRecord(e1, st));
    }
  }
  return MDR_OK;
}

static bool consecutive(const mdr_tick* ticks, int n) {
  for (int i = 1; i < n; ++i)
    if (ticks[i].tick != ticks[0].tick + (uint64_t)i) return false;
  return true;
}

int mdr_rollout(mdr_ctx* c, int n, const mdr_tick* ticks, const uint8_t* action, int64_t act_stride,
                int mode, double* reward, int64_t rew_stride, double* p_out, int use_graph, void* stream) {
  if (!c || !ticks || !reward || n < 1) return fail(MDR_EARG, "mdr_rollout: bad argument");
  c->gq_keys_ready = false;
  c->fz_ready = false;
  if (!c->bound) return fail(MDR_ESTATE, "mdr_rollout: context not bound");
  if (!check_mode(mode) || (mode == MDR_ACT_BUFFER && !action)) return fail(MDR_EARG, "mdr_rollout: bad action source");
  if (c->kp.penalty_mode != MDR_PEN_INDIVIDUAL_L2)
    return fail(MDR_EARG, "mdr_rollout: common penalty modes need the per-step API");
  hipStream_t st = S(stream);
  const bool win = window_ok(c, mode);
  const bool consec = consecutive(ticks, n);
  // the first window counted ahead by mdr_rollout_begin for exactly this call?  (Its count took
  // the ids tick0 + j and its P-only reduce consumed the slot's shards: only the direct sequence
  // with the drivers as kernel arguments can follow it, whatever use_graph asks.)
  const bool counted = c->begun.on && !c->begun.sharded && c->begun.n == n && c->begun.mode == mode &&
                       c->begun.tick0 == ticks[0].tick && c->begun.action == action &&
                       c->begun.act_stride == act_stride && win && consec;
  if (c->begun.on && !counted) c->wslab_dirty = true;  // an unmatched early count: clear its shards
  c->begun.on = false;
  int rc = refresh_if_dirty(c, st);
  if (rc) return rc;
  if (counted || (win && !use_graph && consec)) {
    // direct launches of the windowed path: the first window's drivers travel as kernel arguments
    // of its step kernel (window_launches host_ticks)
    rc = ensure_ticks(c, n);
    if (!rc) rc = wslab_clean(c, st);
    if (!rc)
      rc = window_launches(c, n, c->d_ticks, action, act_stride, mode, reward, rew_stride, p_out, false, st, counted,
                           false, ticks);
    c->counts_ready = false;
    return rc;
  }
  rc = stage_ticks(c, n, ticks, st);
  if (!rc) rc = wslab_clean(c, st);
  if (rc) return rc;
  if (!use_graph) {
    rc = rollout_launches(c, n, action, act_stride, mode, reward, rew_stride, p_out, st);
    c->counts_ready = false;
    return rc;
  }
  GraphKey key{n, mode, action, act_stride, reward, rew_stride, p_out};
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) {
    hipGraphExec_t ex;
    rc = capture_graph(c, [&](hipStream_t cs) {
      return rollout_launches(c, n, action, act_stride, mode, reward, rew_stride, p_out, cs);
    }, &ex);
    if (rc) {
      c->wslab_dirty = true;
      return rc;
    }
    it = c->graphs.emplace(key, std::make_pair(ex, c->ring)).first;
  }
  if (hipGraphLaunch(it->second.first, st) != hipSuccess) {
    c->wslab_dirty = true;
    return fail(MDR_EHIP, "mdr_rollout: hipGraphLaunch");
  }
  ++c->graph_launches[0];
  c->ring = it->second.second;
  c->counts_ready = false;
  return MDR_OK;
}

// The first window's FSM counts (and its cluster power P) of an mdr_rollout of n ticks from tick
// id tick0, launched before the host has the ticks' drivers (they only need the tick ids), so the
// count overlaps the host work.  The next mdr_rollout with the same (n, mode, action, tick0) skips
// them; any other call discards them.  A no-op (returns 0) when the rollout will not take the
// temporally blocked path.
int mdr_rollout_begin(mdr_ctx* c, int n, uint64_t tick0, const uint8_t* action, int64_t act_stride, int mode,
                      void* stream) {
  if (!c || n < 1) return fail(MDR_EARG, "mdr_rollout_begin: bad argument");
  c->gq_keys_ready = false;
  c->fz_ready = false;
  if (!c->bound) return fail(MDR_ESTATE, "mdr_rollout_begin: context not bound");
  if (!check_mode(mode) || (mode == MDR_ACT_BUFFER && !action)) return fail(MDR_EARG, "mdr_rollout_begin: bad action source");
  if (c->begun.on) c->wslab_dirty = true;  // a previous early count that no rollout consumed
  c->begun.on = false;
  if (!window_ok(c, mode)) return MDR_OK;
  // a sharded context (RCCL attached): single-window rollouts only, counts allreduced here, so
  // the matching mdr_rollout_sharded launches just the KA step kernel
  const bool sharded = has_comm(c);
  if (sharded && n > c->win) return MDR_OK;
  hipStream_t st = S(stream);
  int rc = refresh_if_dirty(c, st);
  if (!rc) rc = wslab_clean(c, st);
  if (rc) return rc;
  const int nw = (n + c->win - 1) / c->win;
  const int k0 = n / nw + (n % nw ? 1 : 0);  // window_launches' first window
  c->wslab_dirty = true;
  // the window's P (the counts need no drivers): the matching direct mdr_rollout then launches the
  // step kernel with the drivers as arguments (k_step_window<..., KA>), nothing in between — on one
  // GPU the count kernel's last block reduces; sharded, the reduce follows the counts' allreduce
  rc = launch_count(c, mode, action, act_stride, nullptr, tick0, k0, c->d_wslab, c->d_onb, c->d_wah, nullptr, st,
                    true);
  if (rc) return rc;
  if (sharded) {  // every rank's per-tick class totals (its count kernel's last block), summed
    // (the KA step derives each tick's P from these totals itself: no k_win_records launch, r06)
    if (int rc2 = comm_allreduce(c, win_red_ptr(c, c->d_wslab), (size_t)k0 * c->kp.n_cap, 0, st)) return rc2;
  }
  c->wslab_dirty = false;
  c->begun.sharded = sharded;
  c->begun.on = true;
  c->begun.n = n; c->begun.mode = mode; c->begun.tick0 = tick0;
  c->begun.action = action; c->begun.act_stride = act_stride;
  return MDR_OK;
}

// Measurement: one rollout as direct launches (no graph, drivers staged first) with an event pair
// around every step-kernel launch (k_step_window on the window path, k_step_* per tick otherwise);
// *ms = the summed kernel time, *launches = the number of step launches.  Synchronises on the last
// event.
int mdr_time_step_kernels(mdr_ctx* c, int n, const mdr_tick* ticks, const uint8_t* action, int64_t act_stride,
                          int mode, double* reward, int64_t rew_stride, void* stream, float* ms, int* launches) {
  drop_begun(c);
  if (!c || !ticks || !reward || !ms || !launches || n < 1) return fail(MDR_EARG, "mdr_time_step_kernels: bad argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_time_step_kernels: context not bound");
  if (!check_mode(mode) || (mode == MDR_ACT_BUFFER && !action))
    return fail(MDR_EARG, "mdr_time_step_kernels: bad action source");
  if (c->kp.penalty_mode != MDR_PEN_INDIVIDUAL_L2)
    return fail(MDR_EARG, "mdr_time_step_kernels: common penalty modes need the per-step API");
  hipStream_t st = S(stream);
  int rc = refresh_if_dirty(c, st);
  if (!rc) rc = stage_ticks(c, n, ticks, st);
  if (!rc) rc = wslab_clean(c, st);
  if (rc) return rc;
  std::vector<hipEvent_t> evs;
  c->step_events = &evs;
  rc = rollout_launches(c, n, action, act_stride, mode, reward, rew_stride, nullptr, st);
  c->step_events = nullptr;
  c->counts_ready = false;
  float total = 0.0f;
  if (!rc && !evs.empty() && hipEventSynchronize(evs.back()) != hipSuccess) rc = fail(MDR_EHIP, "event sync");
  for (size_t i = 0; !rc && i + 1 < evs.size(); i += 2) {
    float e = 0.0f;
    if (hipEventElapsedTime(&e, evs[i], evs[i + 1]) != hipSuccess) rc = fail(MDR_EHIP, "event elapsed");
    total += e;
  }
  for (hipEvent_t e : evs) hipEventDestroy(e);
  if (rc) return rc;
  *ms = total;
  *launches = (int)(evs.size() / 2);
  return MDR_OK;
}

// ------------------------------------------------------------------------------------ obs
static ObsArgs obs_args(const mdr_ctx* c, const mdr_obs_spec* sp, const mdr_obs_scalars* sc) {
  ObsArgs o{};
  o.n_feat = sp->n_feat;
  o.msg_w = mdr_msg_width(sp);
  o.n_comm = sp->n_comm;
  o.comm_mode = sp->comm_mode;
  o.hvac_state = sp->hvac_state;
  o.solar_state = sp->solar_state;
  o.thermal_state = sp->thermal_state;
  o.msg_thermal = sp->msg_thermal;
  o.msg_hvac = sp->msg_hvac;
  o.comm_table = sp->comm_table;
  o.halo_msg = sp->halo_msg;
  o.halo_next = nullptr;
  o.msg_all = sp->msg_all;
  o.norm_reg_sig = sp->norm_reg_sig;
  o.cfg_ua = sp->cfg_ua;
  o.cfg_ca = sp->cfg_ca;
  o.cfg_cm = sp->cfg_cm;
  o.cfg_hm = sp->cfg_hm;
  o.cfg_cop = c->cfg.cop;
  o.cfg_lcf = c->cfg.lcf;
  o.cfg_cap = sp->cfg_cap;
  if (sc) { o.p = sc->p; o.s = sc->s; o.solar = sc->solar; o.t_od = sc->t_od; }
  return o;
}

int mdr_msg_width(const mdr_obs_spec* sp) {
  if (!sp) return 0;
  return 4 + (sp->msg_thermal ? 4 : 0) + (sp->msg_hvac ? 3 : 0);
}

static int expected_feat(const mdr_obs_spec* sp) {
  int base = 10 + (sp->hvac_state ? 2 : 0) + (sp->solar_state ? 1 : 0) + (sp->thermal_state ? 5 : 0);
  return base + sp->n_comm * mdr_msg_width(sp);
}

static int check_obs_spec(const mdr_obs_spec* sp, const char* who) {
  if (sp->n_feat != expected_feat(sp)) return fail(MDR_EARG, std::string(who) + ": n_feat does not match the flags");
  if (sp->n_comm < 0 || sp->n_comm > 64) return fail(MDR_EARG, std::string(who) + ": n_comm out of range");
  if (sp->comm_mode == MDR_COMM_TABLE && sp->n_comm > 0 && !sp->comm_table)
    return fail(MDR_EARG, std::string(who) + ": TABLE mode without a table");
  if (sp->comm_mode == MDR_COMM_TABLE && mdr_msg_width(sp) > 16) return fail(MDR_EARG, std::string(who) + ": msg width");
  return MDR_OK;
}

int mdr_obs(mdr_ctx* c, const mdr_obs_spec* sp, const mdr_obs_scalars* sc, const double* p_dev,
            float* obs, void* stream) {
  if (!c || !sp || !sc || !obs) return fail(MDR_EARG, "mdr_obs: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_obs: context not bound");
  if (int rc = check_obs_spec(sp, "mdr_obs")) return rc;
  ObsArgs o = obs_args(c, sp, sc);
  const int lo = sp->n_comm / 2, hi = (sp->n_comm + 1) / 2;
  size_t tile = ((size_t)kObsBlock * sp->n_feat + 3) & ~(size_t)3;
  size_t msg = (size_t)(lo + kObsBlock + hi) * o.msg_w;
  size_t bytes = (tile + msg) * sizeof(float);
  if (bytes > 160 * 1024) return fail(MDR_EARG, "mdr_obs: obs row too wide for one LDS tile");
  hipLaunchKernelGGL(k_obs, dim3(blocks(c->kp.n, kObsBlock)), dim3(kObsBlock), bytes, S(stream), c->kp, o,
                     p_dev, obs);
  LAUNCH_CHECK("k_obs");
  return MDR_OK;
}

int mdr_msg_pack(mdr_ctx* c, const mdr_obs_spec* sp, float* out, void* stream) {
  if (!c || !sp || !out) return fail(MDR_EARG, "mdr_msg_pack: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_msg_pack: context not bound");
  ObsArgs o = obs_args(c, sp, nullptr);
  if (o.msg_w > 16) return fail(MDR_EARG, "mdr_msg_pack: message wider than 16");
  hipLaunchKernelGGL(k_msg_pack, dim3(blocks(c->kp.n, 256)), dim3(256), 0, S(stream), c->kp, o, out);
  LAUNCH_CHECK("k_msg_pack");
  return MDR_OK;
}

int mdr_halo_pack(mdr_ctx* c, const mdr_obs_spec* sp, float* out, void* stream) {
  if (!c || !sp || !out) return fail(MDR_EARG, "mdr_halo_pack: null argument");
  ObsArgs o = obs_args(c, sp, nullptr);
  const int lo = sp->n_comm / 2, hi = (sp->n_comm + 1) / 2;
  if (lo + hi == 0) return MDR_OK;
  hipLaunchKernelGGL(k_halo_pack, dim3(1), dim3(64), 0, S(stream), c->kp, o, lo, hi, out);
  LAUNCH_CHECK("k_halo_pack");
  return MDR_OK;
}

// ------------------------------------------------------------------------------------ greedy
}  // extern "C"

namespace {

// The greedy order: a stable sort of (key, house) pairs (hipCUB / rocprim radix sort; at 2^20
// houses rocprim runs its block merge sort, which measured faster here than forcing Onesweep:
// 212 us vs ~250 us incl. its per-pass lookback resets, profiles/r02g_greedy_kernel_stats.csv)
hipError_t greedy_sort(void* tmp, size_t& bytes, const double* kin, double* kout, const int* vin, int* vout,
                       int64_t n, hipStream_t st) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (int)n, 0, 64, st);
}

int greedy_scratch(mdr_ctx* c, int64_t n) {
  if (c->g_cap >= n) return MDR_OK;
  hipFree(c->g_key); hipFree(c->g_key2); hipFree(c->g_ps); hipFree(c->g_incl);
  hipFree(c->g_idx); hipFree(c->g_idx2); hipFree(c->g_ls); hipFree(c->g_tmp);
  hipFree(c->g_kpos); hipFree(c->g_extra);
  hipFree(c->g_part); hipFree(c->g_hist); hipFree(c->g_sel); hipFree(c->g_win);
  hipFree(c->g_sorted); hipFree(c->g_map); hipFree(c->g_range); hipFree(c->g_tickets);
  c->g_map = nullptr; c->g_range = nullptr; c->g_tickets = nullptr;
  c->g_part = nullptr; c->g_hist = nullptr; c->g_sel = nullptr; c->g_win = nullptr;
  c->g_sorted = nullptr;
  c->gq_keys_ready = false;
  c->fz_ready = false;
  c->gq_hist_dirty = false;
  HIP_TRY(hipMalloc(&c->g_key, n * sizeof(double)));
  HIP_TRY(hipMalloc(&c->g_key2, n * sizeof(double)));
  HIP_TRY(hipMalloc(&c->g_ps, n * sizeof(double)));
  HIP_TRY(hipMalloc(&c->g_incl, n * sizeof(double)));
  HIP_TRY(hipMalloc(&c->g_idx, n * sizeof(int)));
  HIP_TRY(hipMalloc(&c->g_idx2, n * sizeof(int)));
  HIP_TRY(hipMalloc(&c->g_ls, n));
  HIP_TRY(hipMalloc(&c->g_kpos, 2 * sizeof(int64_t)));
  HIP_TRY(hipMalloc(&c->g_extra, 64 * sizeof(int64_t)));
  // (min, max) partials: k_gq_keys' grid, or the grid of the step kernel whose epilogue writes the
  // keys (k_step_pipe: a block per kStepGqWaves x tpw x 128 houses, tpw >= 2)
  c->gq_parts_cap = (int)std::max<int64_t>(kGqParts, (n + 1023) / 1024);
  HIP_TRY(hipMalloc(&c->g_part, 2 * (size_t)c->gq_parts_cap * sizeof(double)));
  HIP_TRY(hipMalloc(&c->g_hist, kGqHistWords * sizeof(unsigned)));
  HIP_TRY(hipMemset(c->g_hist, 0, kGqHistWords * sizeof(unsigned)));  // (the kernels re-zero what they read)
  HIP_TRY(hipMalloc(&c->g_sel, kGqSelBytes));
  HIP_TRY(hipMalloc(&c->g_map, kGqCells * sizeof(uint32_t)));
  {
    unsigned char init[kGqSelBytes] = {};
    uint32_t map[kGqCells];
    gq_sel_init(init, map);
    HIP_TRY(hipMemcpy(c->g_sel, init, kGqSelBytes, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->g_map, map, sizeof(map), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMalloc(&c->g_win, (kGqCap + 1) * sizeof(uint4)));  // (sharded: [0] = the count header)
  HIP_TRY(hipMalloc(&c->g_range, 2 * sizeof(double)));
  HIP_TRY(hipMalloc(&c->g_tickets, kTicketWords * sizeof(unsigned)));
  HIP_TRY(hipMemset(c->g_tickets, 0, kTicketWords * sizeof(unsigned)));
  HIP_TRY(hipMalloc(&c->g_sorted, kGqCap * sizeof(uint4)));
  size_t b1 = 0, b2 = 0;
  HIP_TRY(greedy_sort(nullptr, b1, c->g_key, c->g_key2, c->g_idx, c->g_idx2, n, nullptr));
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, b2, c->g_ps, c->g_incl, (int)n));
  c->g_tmp_bytes = b1 > b2 ? b1 : b2;
  HIP_TRY(hipMalloc(&c->g_tmp, c->g_tmp_bytes));
  c->g_cap = n;
  return MDR_OK;
}

// before a producer (k_gq_keys, the step's GQ epilogue) adds to g_hist: counts an earlier producer
// left unconsumed (two GQ steps with no greedy call between, or keys dropped by a state change)
// are zeroed first, so the select never sees the sum of two states
int gq_hist_produce(mdr_ctx* c, hipStream_t st) {
  if (c->gq_hist_dirty) {
    hipLaunchKernelGGL(k_zero_u64, dim3(64), dim3(256), 0, st, reinterpret_cast<unsigned long long*>(c->g_hist),
                       (int64_t)(kGqHistWords / 2));
    LAUNCH_CHECK("k_zero_u64 (g_hist)");
  }
  c->gq_hist_dirty = true;
  return MDR_OK;
}

// the keys and superbin histogram of the current state (when no step epilogue prepared them);
// slab: zeroed for the decisions' counts (nullptr: none)
int launch_gq_keys(mdr_ctx* c, hipStream_t st, unsigned long long* slab, bool local_map) {
  if (int rc = gq_hist_produce(c, st)) return rc;
  hipLaunchKernelGGL(k_gq_keys, dim3(kGqParts), dim3(kGqThreads), 0, st, c->kp, gq_codes(c), c->g_part, c->g_hist,
                     c->g_sel, c->g_map, slab);
  LAUNCH_CHECK("k_gq_keys");
  // (sharded, local_map = false: every rank's map must stay the one built from the allreduced range)
  if (c->gq_map_stale && local_map) {  // (a written state: cells over its key range, then the codes again)
    unsigned char* sel = reinterpret_cast<unsigned char*>(c->g_sel);
    hipLaunchKernelGGL(k_gq_remap, dim3(1), dim3(256), 0, st, c->kp, (const double*)c->g_part, (int)kGqParts,
                       c->g_hist + kGqBins * 4, c->g_sel, c->g_map,
                       reinterpret_cast<double*>(sel + gq_kmin_offset(-1)), reinterpret_cast<double*>(sel + gq_scale_offset(-1)));
    LAUNCH_CHECK("k_gq_remap");
    hipLaunchKernelGGL(k_gq_keys, dim3(kGqParts), dim3(kGqThreads), 0, st, c->kp, gq_codes(c), c->g_part, c->g_hist,
                       c->g_sel, c->g_map, slab);
    LAUNCH_CHECK("k_gq_keys (remapped)");
    c->gq_map_stale = false;
  }
  c->gq_nparts = kGqParts;
  c->gq_slab_zeroed = slab != nullptr;
  return MDR_OK;
}

}  // namespace

extern "C" {

int mdr_ctrl_greedy(mdr_ctx* c, double budget, uint8_t* action, void* stream) {
  if (!c || !action) return fail(MDR_EARG, "mdr_ctrl_greedy: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_ctrl_greedy: context not bound");
  const bool keys_ready = c->gq_keys_ready && c->g_cap >= c->kp.n;  // (the last step's epilogue wrote them)
  drop_begun(c);
  c->gq_keys_ready = false;  // (the histogram is consumed below)
  c->fz_ready = false;
  int rc = greedy_scratch(c, c->kp.n);
  if (rc) return rc;
  hipStream_t st = S(stream);
  const int n = (int)c->kp.n;
  double pmin = INFINITY;
  for (int k = 0; k < c->cfg.n_cap; ++k) pmin = fmin(pmin, c->cfg.cap_table[k] / c->cfg.cop);
  unsigned long long* slab = slab_at(c, c->ring);  // the counts of the actions decided here
  if (c->kp.n_cap <= 4 && !c->greedy_sort) {
    // histogram select (mdr_kernels.hip k_gq_*): no sort of the whole cluster, no host
    // synchronisation; k_gq_select decides exactly what the candidate window cannot
    if (!keys_ready) {
      if (int rc2 = launch_gq_keys(c, st, slab)) return rc2;
    } else if (!c->gq_slab_zeroed) {
      // the producing step counted a lookahead into this slab: the decisions replace those counts
      hipLaunchKernelGGL(k_zero_u64, dim3(1), dim3(256), 0, st, slab, (int64_t)c->slab_len);
      LAUNCH_CHECK("k_zero_u64 (decision slab)");
    }
    // the slab was zeroed by the codes' producer (k_gq_keys, or the GQ step: its next slab is this)
    const int nstage = (n + kGqStage - 1) / kGqStage;
    if (c->gq_band && !c->gq_band_skip) {
      // the band's two launches: binsc (window from the band and compaction, or the bins), finish
      // (rank + decide, or on a miss window + compaction + decide)
      hipLaunchKernelGGL(k_gq_binsc, dim3(nstage), dim3(kGqThreads), 0, st, c->kp, gq_codes(c), c->g_hist, budget,
                         c->g_sel, c->g_win, action, slab);
      LAUNCH_CHECK("k_gq_binsc");
      hipLaunchKernelGGL(k_gq_finish, dim3(kGqSelBlocks), dim3(1024), 0, st, c->kp, (const uint32_t*)gq_codes(c),
                         c->g_win, c->g_sorted, budget, pmin, c->g_sel, action, slab, c->g_hist, c->g_tickets,
                         (const double*)c->g_part, c->gq_nparts, c->g_map);
      LAUNCH_CHECK("k_gq_finish");
      c->gq_hist_dirty = false;
      c->counts_ready = true;
      return MDR_OK;
    } else {
      hipLaunchKernelGGL(k_gq_bins, dim3(kGqParts), dim3(kGqThreads), 0, st, c->kp, gq_codes(c), c->g_hist, budget,
                         c->g_sel, slab);
      LAUNCH_CHECK("k_gq_bins");
    }
    hipLaunchKernelGGL(k_gq_compact, dim3(nstage), dim3(kGqThreads), 0, st, c->kp, gq_codes(c), c->g_hist, budget,
                       c->g_sel, c->g_win, action, slab);
    LAUNCH_CHECK("k_gq_compact");
    // the window ranked by 256 blocks, the last of them decides (a one-block select measured slower:
    // DESIGN.md §3.3)
    hipLaunchKernelGGL(k_gq_select, dim3(kGqSelBlocks), dim3(1024), 0, st, c->kp, (const uint4*)c->g_win,
                       c->g_sorted, budget, pmin, c->g_sel, action, slab, c->g_hist, (const uint4*)nullptr, 0,
                       c->g_tickets, (const double*)c->g_part, c->gq_nparts, c->g_map);
    LAUNCH_CHECK("k_gq_select");
    c->gq_hist_dirty = false;
    c->counts_ready = true;
    return MDR_OK;
  }
  hipLaunchKernelGGL(k_greedy_keys, dim3(blocks(n, 256)), dim3(256), 0, st, c->kp, c->g_key, c->g_idx);
  LAUNCH_CHECK("k_greedy_keys");
  size_t b = c->g_tmp_bytes;
  HIP_TRY(greedy_sort(c->g_tmp, b, c->g_key, c->g_key2, c->g_idx, c->g_idx2, n, st));
  hipLaunchKernelGGL(k_greedy_gather, dim3(blocks(n, 256)), dim3(256), 0, st, c->kp, c->g_idx2, c->g_ps,
                     c->g_ls);
  LAUNCH_CHECK("k_greedy_gather");
  b = c->g_tmp_bytes;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(c->g_tmp, b, c->g_ps, c->g_incl, n, st));
  hipLaunchKernelGGL(k_greedy_walk, dim3(1), dim3(256), 0, st, (int64_t)n, c->g_incl, c->g_ps, c->g_ls,
                     budget, pmin, c->g_kpos, c->g_extra, 64);
  LAUNCH_CHECK("k_greedy_walk");
  hipLaunchKernelGGL(k_greedy_apply, dim3(blocks(n, 256)), dim3(256), 0, st, (int64_t)n, c->g_idx2,
                     c->g_kpos, c->g_extra, action);
  LAUNCH_CHECK("k_greedy_apply");
  // the counts of these actions, as the histogram form leaves them
  HIP_TRY(hipMemsetAsync(slab, 0, c->slab_len * sizeof(unsigned long long), st));
  if (int rc2 = launch_counts(c, action, MDR_ACT_BUFFER, 0, nullptr, st)) return rc2;
  c->counts_ready = true;
  return MDR_OK;
}

int mdr_greedy_diag(mdr_ctx* c, uint64_t* out) {
  if (!c || !out) return fail(MDR_EARG, "mdr_greedy_diag: null argument");
  for (int k = 0; k < 4; ++k) out[k] = 0;
  if (!c->g_sel) return MDR_OK;
  unsigned char h[kGqSelBytes];
  HIP_TRY(hipMemcpy(h, c->g_sel, kGqSelBytes, hipMemcpyDeviceToHost));
  gq_diag_of(h, out);
  return MDR_OK;
}

int mdr_greedy_state(mdr_ctx* c, uint64_t* out) {
  if (!c || !out) return fail(MDR_EARG, "mdr_greedy_state: null argument");
  for (int k = 0; k < 12; ++k) out[k] = 0;
  if (!c->g_sel) return MDR_OK;
  unsigned char h[kGqSelBytes];
  HIP_TRY(hipMemcpy(h, c->g_sel, kGqSelBytes, hipMemcpyDeviceToHost));
  gq_state_of(h, out);
  return MDR_OK;
}

// config C3's loop in one call: per tick, GreedyMyopic on the current state with the tick's
// pre-step signal as budget (greedy_myopic_controller.py:67-104; the signal the obs carries), then
// the step with those actions (environment.py:86-106), whose epilogue writes the next call's keys
// — Environment.greedy_actions + step_tensor(ctrl='greedy_keys') per tick, without a host round
// trip between them
}  // extern "C"

namespace {
// the fused tick's buffers (mdr_kernels.h GqfBufs), for a cluster of n houses
int gqf_scratch(mdr_ctx* c, int64_t n) {
  if (c->fz_cap_n >= n && c->fz.par[0]) return MDR_OK;
  HIP_TRY(hipDeviceSynchronize());
  hipFree(c->fz.par[0]); hipFree(c->fz.bkt[0]); hipFree(c->fz.mbkt); hipFree(c->fz.map[0]); hipFree(c->fz.sel);
  hipFree(c->fz.dec);
  unsigned long long* keep_stamps = c->fz.stamps;
  c->fz = GqfBufs{};
  c->fz.stamps = keep_stamps;
  c->fz_ready = false;
  // bucket capacity: 4x the houses a (copy, bin) holds on average under an equi-depth map, >= 32
  const int64_t avg = (n + (int64_t)gq_bins_eff(c->kp.n_global) * kGqCopies - 1) / ((int64_t)gq_bins_eff(c->kp.n_global) * kGqCopies);
  const int cap = (int)std::max<int64_t>(32, 4 * avg);
  unsigned* regions = nullptr;
  HIP_TRY(hipMalloc(&regions, (2 * (size_t)kGqfParWords + kGqfMissWords) * sizeof(unsigned)));
  HIP_TRY(hipMemset(regions, 0, (2 * (size_t)kGqfParWords + kGqfMissWords) * sizeof(unsigned)));
  c->fz.par[0] = regions;
  c->fz.par[1] = regions + kGqfParWords;
  c->fz.miss = regions + 2 * kGqfParWords;
  uint4* bk = nullptr;
  const size_t nb = (size_t)kGqCopies * kGqBand * 64 * cap;
  HIP_TRY(hipMalloc(&bk, 2 * nb * sizeof(uint4)));
  c->fz.bkt[0] = bk;
  c->fz.bkt[1] = bk + nb;
  HIP_TRY(hipMalloc(&c->fz.mbkt, (size_t)kGqCopies * 128 * cap * sizeof(uint4)));
  c->fz.cap = cap;
  c->fz.mcap = cap;
  uint32_t* maps = nullptr;
  HIP_TRY(hipMalloc(&maps, 2 * kGqCells * sizeof(uint32_t)));
  c->fz.map[0] = maps;
  c->fz.map[1] = maps + kGqCells;
  HIP_TRY(hipMalloc(&c->fz.sel, kGqSelBytes));
  {
    unsigned char init[kGqSelBytes] = {};
    uint32_t map[kGqCells];
    gqf_sel_init(init, map);
    HIP_TRY(hipMemcpy(c->fz.sel, init, kGqSelBytes, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->fz.map[0], map, sizeof(map), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->fz.map[1], map, sizeof(map), hipMemcpyHostToDevice));
  }
  HIP_TRY(hipMalloc(&c->fz.dec, (size_t)n));
  c->fz_cap_n = n;
  c->fz_par = 0;
  return MDR_OK;
}

// the fused tick's step: k_step_pipe<..., GQ = 2> applying the decision of parity par, producing 1 - par
int launch_step_fused(mdr_ctx* c, const TickArgs& tk, double* reward, uint8_t* act_out, double* p_out, int par,
                      hipStream_t st) {
  const KParams kp = c->kp;
  const int tpw = c->tpw >= 4 ? 4 : 2;
  const unsigned nb = blocks(blocks(kp.n, 128), kStepGqWaves * tpw);
  if ((int)nb > c->gq_parts_cap) return fail(MDR_ESTATE, "fused greedy: the step grid exceeds the partials buffer");
  GqOut go{act_out, nullptr, c->g_part, nullptr, nullptr, nullptr};
  unsigned long long *cur = slab_at(c, c->ring), *nxt = slab_at(c, c->ring + 1), *zer = slab_at(c, c->ring + 2);
  if (tpw >= 4)
    hipLaunchKernelGGL((k_step_pipe<4, MDR_ACT_BUFFER, 0, 2>), dim3(nb), dim3(64 * kStepGqWaves), 0, st, kp,
                       (const uint8_t*)c->fz.dec, tk, (const TickArgs*)nullptr, cur, reward, p_out, nxt, zer, go, c->fz, par);
  else
    hipLaunchKernelGGL((k_step_pipe<2, MDR_ACT_BUFFER, 0, 2>), dim3(nb), dim3(64 * kStepGqWaves), 0, st, kp,
                       (const uint8_t*)c->fz.dec, tk, (const TickArgs*)nullptr, cur, reward, p_out, nxt, zer, go, c->fz, par);
  LAUNCH_CHECK("k_step_pipe (fused greedy)");
  c->gq_nparts = (int)nb;
  c->ring = (c->ring + 1) % 3;
  return MDR_OK;
}
}  // namespace

extern "C" {

// diagnostics: record k_gq_decide2's per-block phase clocks (100 MHz) of the following calls into a
// device buffer of kGqSelBlocks x kGqfStampWords words (n = 0: stop); read it back with mdr_greedy_fused_stamps
int mdr_greedy_fused_stamps(mdr_ctx* c, int on, uint64_t* out) {
  if (!c) return fail(MDR_EARG, "mdr_greedy_fused_stamps: null ctx");
  if (out && c->fz.stamps)
    HIP_TRY(hipMemcpy(out, c->fz.stamps, kGqSelBlocks * kGqfStampWords * sizeof(uint64_t), hipMemcpyDeviceToHost));
  if (on && !c->fz.stamps) {
    HIP_TRY(hipMalloc(&c->fz.stamps, kGqSelBlocks * kGqfStampWords * sizeof(uint64_t)));
    HIP_TRY(hipMemset(c->fz.stamps, 0, kGqSelBlocks * kGqfStampWords * sizeof(uint64_t)));
  }
  if (!on && c->fz.stamps) {
    HIP_TRY(hipDeviceSynchronize());
    hipFree(c->fz.stamps);
    c->fz.stamps = nullptr;
  }
  return MDR_OK;
}

int mdr_greedy_fused_diag(mdr_ctx* c, uint64_t* out) {
  if (!c || !out) return fail(MDR_EARG, "mdr_greedy_fused_diag: null argument");
  for (int k = 0; k < 6; ++k) out[k] = 0;
  if (!c->fz.sel) return MDR_OK;
  unsigned char h[kGqSelBytes];
  HIP_TRY(hipMemcpy(h, c->fz.sel, kGqSelBytes, hipMemcpyDeviceToHost));
  gqf_diag_of(h, out);
  return MDR_OK;
}

int mdr_greedy_rollout(mdr_ctx* c, int n, const mdr_tick* ticks, uint8_t* action, int64_t act_stride,
                       double* reward, int64_t rew_stride, double* p_out, void* stream) {
  if (!c || (n > 0 && (!ticks || !action || !reward))) return fail(MDR_EARG, "mdr_greedy_rollout: null argument");
  if (n < 0 || act_stride < 0 || rew_stride < 0) return fail(MDR_EARG, "mdr_greedy_rollout: negative size");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_greedy_rollout: context not bound");
  if (c->world > 1)  // (a shard-local decision and step would use shard-local counts: per-tick loop)
    return fail(MDR_ESTATE, "mdr_greedy_rollout: single-GPU only (sharded contexts: the per-tick greedy + step loop)");
  hipStream_t st = S(stream);
  // the fused tick (MDR_OPT_GQ_FUSED): individual_L2 on the software-pipelined step, <= 4 classes
  const bool fused = c->gq_fused && !c->greedy_sort && c->kp.n_cap <= 4 && c->tpw >= 1 && c->fastdiv &&
                     c->kp.penalty_mode == MDR_PEN_INDIVIDUAL_L2 && n > 0;
  if (fused) {
    const bool ready = c->fz_ready && c->fz_cap_n >= c->kp.n;  // (the last step produced this state's counts)
    drop_begun(c);
    if (int rc = refresh_if_dirty(c, st)) return rc;
    if (int rc = greedy_scratch(c, c->kp.n)) return rc;  // (the partials, tickets and sorted window)
    if (int rc = gqf_scratch(c, c->kp.n)) return rc;
    double pmin = INFINITY;
    for (int k = 0; k < c->cfg.n_cap; ++k) pmin = fmin(pmin, c->cfg.cap_table[k] / c->cfg.cop);
    int par = c->fz_par;
    if (!ready) {  // the current state's keys: the producer without a step, into parity par
      hipLaunchKernelGGL(k_zero_u64, dim3(64), dim3(256), 0, st, reinterpret_cast<unsigned long long*>(c->fz.par[par]),
                         (int64_t)(kGqfParWords / 2));
      LAUNCH_CHECK("k_zero_u64 (fused producer region)");
      const unsigned g = blocks(c->kp.n, kGqStage);
      hipLaunchKernelGGL(k_gq_keys2, dim3(g), dim3(kGqThreads), 0, st, c->kp, c->fz, par, c->g_part, slab_at(c, c->ring));
      LAUNCH_CHECK("k_gq_keys2");
      if (c->gq_map_stale) {  // (a written state: parity par's cells over its key range, then the producer again)
        unsigned char* fs = reinterpret_cast<unsigned char*>(c->fz.sel);
        hipLaunchKernelGGL(k_gq_remap, dim3(1), dim3(256), 0, st, c->kp, (const double*)c->g_part, (int)g, c->fz.par[par],
                           c->fz.sel, c->fz.map[par], reinterpret_cast<double*>(fs + gq_kmin_offset(par)),
                           reinterpret_cast<double*>(fs + gq_scale_offset(par)));
        LAUNCH_CHECK("k_gq_remap (fused)");
        hipLaunchKernelGGL(k_zero_u64, dim3(64), dim3(256), 0, st, reinterpret_cast<unsigned long long*>(c->fz.par[par]),
                           (int64_t)(kGqfParWords / 2));
        LAUNCH_CHECK("k_zero_u64 (fused producer region, remapped)");
        hipLaunchKernelGGL(k_gq_keys2, dim3(g), dim3(kGqThreads), 0, st, c->kp, c->fz, par, c->g_part, slab_at(c, c->ring));
        LAUNCH_CHECK("k_gq_keys2 (remapped)");
        c->gq_map_stale = false;
      }
      c->gq_nparts = (int)g;
    }
    for (int t = 0; t < n; ++t) {
      hipLaunchKernelGGL(k_gq_decide2, dim3(kGqSelBlocks), dim3(1024), 0, st, c->kp, c->fz, par, ticks[t].s_prev, pmin,
                         slab_at(c, c->ring), c->g_tickets, (const double*)c->g_part, c->gq_nparts);
      LAUNCH_CHECK("k_gq_decide2");
      if (int rc = launch_step_fused(c, to_tick(&ticks[t]), reward + (int64_t)t * rew_stride,
                                     action ? action + (int64_t)t * act_stride : nullptr, p_out, par, st))
        return rc;
      par = 1 - par;
    }
    c->fz_par = par;
    c->fz_ready = true;
    c->counts_ready = false;
    return MDR_OK;
  }
  // the adaptive band (MDR_OPT_GQ_ADAPTIVE): the band is predicted from the crossing's
  // trend, so a budget whose change departs from the last change by more than four superbins' worth of
  // power (a regular-steps edge, the tick after it) would miss it — that tick runs the three-launch
  // form (bins -> compact -> select, cheaper than a band miss), decided on the host from the budgets
  double pavg = 0.0;
  for (int k = 0; k < c->cfg.n_cap; ++k) pavg += c->cfg.cap_table[k] / c->cfg.cop;
  pavg /= c->cfg.n_cap > 0 ? c->cfg.n_cap : 1;
  const double jump = 4.0 * ((double)c->kp.n_global * 64.0 / (double)gq_bins_eff(c->kp.n_global)) * pavg;
  for (int t = 0; t < n; ++t) {
    uint8_t* a = action + (int64_t)t * act_stride;
    double* r = reward + (int64_t)t * rew_stride;
    const double sb = ticks[t].s_prev;
    c->gq_band_skip = c->gq_adaptive && c->gq_s1 == c->gq_s1 && c->gq_s2 == c->gq_s2 &&
                      !(fabs((sb - c->gq_s1) - (c->gq_s1 - c->gq_s2)) <= jump);
    const int rc0 = mdr_ctrl_greedy(c, sb, a, stream);
    c->gq_band_skip = false;
    if (rc0) return rc0;
    c->gq_s2 = c->gq_s1;
    c->gq_s1 = sb;
    if (int rc = launch_step(c, a, MDR_ACT_BUFFER, to_tick(&ticks[t]), nullptr, r, 0, MDR_CTRL_GREEDY_KEYS, nullptr,
                             p_out, st))
      return rc;
    if (c->kp.penalty_mode != MDR_PEN_INDIVIDUAL_L2) {  // (Environment.step_tensor's common-penalty tail)
      if (int rc = mdr_penalty_partials(c, stream)) return rc;
      if (int rc = mdr_reward_finalize(c, &ticks[t], r, stream)) return rc;
    }
  }
  return MDR_OK;
}

int mdr_greedy_band(mdr_ctx* c, uint64_t* out) {
  if (!c || !out) return fail(MDR_EARG, "mdr_greedy_band: null argument");
  for (int k = 0; k < 4; ++k) out[k] = 0;
  if (!c->g_sel) return MDR_OK;
  unsigned char h[kGqSelBytes];
  HIP_TRY(hipMemcpy(h, c->g_sel, kGqSelBytes, hipMemcpyDeviceToHost));
  gq_band_of(h, out);
  return MDR_OK;
}

int mdr_greedy_fallbacks(mdr_ctx* c, uint64_t* count) {
  if (!c || !count) return fail(MDR_EARG, "mdr_greedy_fallbacks: null argument");
  uint64_t d[4];
  if (int rc = mdr_greedy_diag(c, d)) return rc;
  *count = d[0];
  return MDR_OK;
}

// ---- sharded histogram select (the stages between the caller's collectives; mdr.h)
static double greedy_pmin(const mdr_ctx* c) {
  double pmin = INFINITY;
  for (int k = 0; k < c->cfg.n_cap; ++k) pmin = fmin(pmin, c->cfg.cap_table[k] / c->cfg.cop);
  return pmin;
}

int mdr_gq_shard_begin(mdr_ctx* c, void* stream) {
  if (!c) return fail(MDR_EARG, "mdr_gq_shard_begin: null context");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_gq_shard_begin: context not bound");
  if (c->kp.n_cap > 4) return fail(MDR_EARG, "mdr_gq_shard_begin: more than 4 capacity classes (use the all-gather form)");
  const bool keys_ready = c->gq_keys_ready && c->g_cap >= c->kp.n;
  drop_begun(c);
  c->gq_keys_ready = false;
  c->fz_ready = false;
  if (int rc = greedy_scratch(c, c->kp.n)) return rc;
  hipStream_t st = S(stream);
  if (!keys_ready)
    if (int rc = launch_gq_keys(c, st, nullptr, false)) return rc;
  hipLaunchKernelGGL(k_gq_range, dim3(1), dim3(256), 0, st, c->g_part, c->gq_nparts, c->g_range);
  LAUNCH_CHECK("k_gq_range");
  return MDR_OK;
}

int mdr_gq_shard_buffers(mdr_ctx* c, void** super_hist, int64_t* n_super, void** bin_hist, int64_t* n_bin,
                         void** range, void** window, int64_t* window_bytes) {
  if (!c || !super_hist || !n_super || !bin_hist || !n_bin || !range || !window || !window_bytes)
    return fail(MDR_EARG, "mdr_gq_shard_buffers: null argument");
  if (!c->g_sel) return fail(MDR_ESTATE, "mdr_gq_shard_buffers: call mdr_gq_shard_begin first");
  *super_hist = c->g_hist + kGqBins * 4;
  *n_super = (int64_t)kGqCopies * (kGqSuper + 1) * 4;
  *bin_hist = c->g_hist;
  *n_bin = (int64_t)kGqCopies * 512;
  *range = c->g_range;
  *window = c->g_win;
  *window_bytes = (int64_t)(kGqCap + 1) * (int64_t)sizeof(uint4);
  return MDR_OK;
}

int mdr_gq_shard_bins(mdr_ctx* c, double budget, void* stream) {
  if (!c || !c->g_sel) return fail(MDR_ESTATE, "mdr_gq_shard_bins: call mdr_gq_shard_begin first");
  hipLaunchKernelGGL(k_gq_bins, dim3(kGqParts), dim3(kGqThreads), 0, S(stream), c->kp, gq_codes(c), c->g_hist,
                     budget, c->g_sel, (unsigned long long*)nullptr);
  LAUNCH_CHECK("k_gq_bins (sharded)");
  return MDR_OK;
}

int mdr_gq_shard_compact(mdr_ctx* c, double budget, uint8_t* action, void* stream) {
  if (!c || !action) return fail(MDR_EARG, "mdr_gq_shard_compact: null argument");
  if (!c->g_sel) return fail(MDR_ESTATE, "mdr_gq_shard_compact: call mdr_gq_shard_begin first");
  hipStream_t st = S(stream);
  const int nstage = (int)((c->kp.n + kGqStage - 1) / kGqStage);
  hipLaunchKernelGGL(k_gq_compact, dim3(nstage), dim3(kGqThreads), 0, st, c->kp, gq_codes(c), c->g_hist,
                     budget, c->g_sel, c->g_win + 1, action, (unsigned long long*)nullptr);
  LAUNCH_CHECK("k_gq_compact (sharded)");
  // the window's header {count, 0, 0, 0}: the allocator's final count
  HIP_TRY(hipMemsetAsync(c->g_win, 0, sizeof(uint4), st));
  HIP_TRY(hipMemcpyAsync(c->g_win, reinterpret_cast<const unsigned char*>(c->g_sel) + gq_wcount_offset(),
                         sizeof(unsigned), hipMemcpyDeviceToDevice, st));
  return MDR_OK;
}

int mdr_gq_shard_select(mdr_ctx* c, double budget, const void* gathered, int world, uint8_t* action, void* stream) {
  if (!c || !gathered || !action) return fail(MDR_EARG, "mdr_gq_shard_select: null argument");
  if (world < 1 || world > kGqMaxRanks) return fail(MDR_EARG, "mdr_gq_shard_select: 1 <= world <= 64");
  if (!c->g_sel) return fail(MDR_ESTATE, "mdr_gq_shard_select: call mdr_gq_shard_begin first");
  hipLaunchKernelGGL(k_gq_select, dim3(kGqSelBlocks), dim3(1024), 0, S(stream), c->kp, (const uint4*)nullptr,
                     c->g_sorted, budget, greedy_pmin(c), c->g_sel, action, (unsigned long long*)nullptr, c->g_hist,
                     static_cast<const uint4*>(gathered), world, c->g_tickets, (const double*)c->g_range, -1,
                     c->g_map);
  LAUNCH_CHECK("k_gq_select (sharded)");
  c->gq_hist_dirty = false;
  return MDR_OK;
}

int mdr_gq_shard_fallback(mdr_ctx* c, int* need, void* stream) {
  if (!c || !need) return fail(MDR_EARG, "mdr_gq_shard_fallback: null argument");
  if (!c->g_sel) return fail(MDR_ESTATE, "mdr_gq_shard_fallback: call mdr_gq_shard_begin first");
  unsigned v = 0;
  hipStream_t st = S(stream);
  HIP_TRY(hipMemcpyAsync(&v, reinterpret_cast<const unsigned char*>(c->g_sel) + gq_need_fb_offset(), sizeof(v),
                         hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  *need = v ? 1 : 0;
  return MDR_OK;
}

int mdr_rccl_allgather(mdr_ctx* c, const void* send, void* recv, int64_t bytes, void* stream) {
  if (!c || !send || !recv || bytes < 0) return fail(MDR_EARG, "mdr_rccl_allgather: bad argument");
  if (!c->comm) return fail(MDR_ESTATE, "mdr_rccl_allgather: RCCL not initialised");
  RCCL_TRY(ncclAllGather(send, recv, (size_t)bytes, ncclUint8, c->comm, S(stream)));
  return MDR_OK;
}

int mdr_greedy_inputs(mdr_ctx* c, double* key, double* power, uint8_t* lock, void* stream) {
  if (!c || !key || !power || !lock) return fail(MDR_EARG, "mdr_greedy_inputs: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_greedy_inputs: context not bound");
  hipLaunchKernelGGL(k_greedy_inputs, dim3(blocks(c->kp.n, 256)), dim3(256), 0, S(stream), c->kp, key, power, lock);
  LAUNCH_CHECK("k_greedy_inputs");
  return MDR_OK;
}

int mdr_greedy_select(mdr_ctx* c, int64_t n, const double* key, const double* power, const uint8_t* lock,
                      double budget, uint8_t* action, void* stream) {
  if (!c || !key || !power || !lock || !action || n < 1) return fail(MDR_EARG, "mdr_greedy_select: bad argument");
  if (n >= ((int64_t)1 << 31)) return fail(MDR_EARG, "mdr_greedy_select: n must be < 2^31");
  int rc = greedy_scratch(c, n);
  if (rc) return rc;
  hipStream_t st = S(stream);
  hipLaunchKernelGGL(k_greedy_iota, dim3(blocks(n, 256)), dim3(256), 0, st, n, c->g_idx);
  LAUNCH_CHECK("k_greedy_iota");
  size_t b = c->g_tmp_bytes;
  HIP_TRY(greedy_sort(c->g_tmp, b, key, c->g_key2, c->g_idx, c->g_idx2, n, st));
  hipLaunchKernelGGL(k_greedy_gather_rows, dim3(blocks(n, 256)), dim3(256), 0, st, n, c->g_idx2, power, lock,
                     c->g_ps, c->g_ls);
  LAUNCH_CHECK("k_greedy_gather_rows");
  b = c->g_tmp_bytes;
  HIP_TRY(hipcub::DeviceScan::InclusiveSum(c->g_tmp, b, c->g_ps, c->g_incl, (int)n, st));
  double pmin = INFINITY;
  for (int k = 0; k < c->cfg.n_cap; ++k) pmin = fmin(pmin, c->cfg.cap_table[k] / c->cfg.cop);
  hipLaunchKernelGGL(k_greedy_walk, dim3(1), dim3(256), 0, st, n, c->g_incl, c->g_ps, c->g_ls, budget, pmin,
                     c->g_kpos, c->g_extra, 64);
  LAUNCH_CHECK("k_greedy_walk");
  hipLaunchKernelGGL(k_greedy_apply, dim3(blocks(n, 256)), dim3(256), 0, st, n, c->g_idx2, c->g_kpos, c->g_extra,
                     action);
  LAUNCH_CHECK("k_greedy_apply");
  return MDR_OK;
}

// ------------------------------------------------------------------------------------ RCCL
int mdr_rccl_unique_id(uint8_t* id128) {
  if (!id128) return fail(MDR_EARG, "mdr_rccl_unique_id: null");
  ncclUniqueId id;
  RCCL_TRY(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(id128, &id, 128);
  return MDR_OK;
}

int mdr_rccl_init(mdr_ctx* c, const uint8_t* id128, int world, int rank) {
  if (!c || !id128 || world < 1 || rank < 0 || rank >= world) return fail(MDR_EARG, "mdr_rccl_init: bad argument");
  if (c->host.allreduce) return fail(MDR_ESTATE, "mdr_rccl_init: the context already has host collectives");
  HIP_TRY(hipSetDevice(c->cfg.device));
  ncclUniqueId id;
  memcpy(&id, id128, 128);
  RCCL_TRY(ncclCommInitRank(&c->comm, world, id, rank));
  if (!c->comm_stream) HIP_TRY(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
  c->world = world;
  c->rank = rank;
  return MDR_OK;
}

int mdr_comm_host(mdr_ctx* c, int world, int rank, mdr_host_allreduce_fn allreduce, mdr_host_sendrecv_fn sendrecv,
                  void* user) {
  if (!c || !allreduce || !sendrecv || world < 1 || rank < 0 || rank >= world)
    return fail(MDR_EARG, "mdr_comm_host: bad argument");
  if (c->comm) return fail(MDR_ESTATE, "mdr_comm_host: the context already has an RCCL communicator");
  HIP_TRY(hipSetDevice(c->cfg.device));
  if (!c->comm_stream) HIP_TRY(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
  c->host.allreduce = allreduce;
  c->host.sendrecv = sendrecv;
  c->host.user = user;
  c->world = world;
  c->rank = rank;
  return MDR_OK;
}

int mdr_rccl_allreduce(mdr_ctx* c, void* buf, int64_t count, int dtype, void* stream) {
  if (!c || !buf || count < 0) return fail(MDR_EARG, "mdr_rccl_allreduce: bad argument");
  if (!c->comm) return fail(MDR_ESTATE, "mdr_rccl_allreduce: RCCL not initialised");
  ncclDataType_t t = dtype == 0 ? ncclInt64 : dtype == 3 ? ncclUint32 : ncclFloat64;
  ncclRedOp_t op = dtype == 2 ? ncclMax : dtype == 4 ? ncclMin : ncclSum;
  RCCL_TRY(ncclAllReduce(buf, buf, (size_t)count, t, op, c->comm, S(stream)));
  return MDR_OK;
}

}  // extern "C"

namespace {
// Overlapped sharded pipeline (in-kernel action source with lookahead, one reward row per tick).
// The per-tick exchange only feeds the reward's signal term, so the reward of tick t is written
// one launch later (k_step reward_lag; bit-identical, no extra bytes):
//   compute stream  K(t): state of tick t, reward of tick t-1 from the loaded state + allreduced
//                   slab (t-1)%4, lookahead counts of t+1 into slab (t+1)%4, zero slab (t+2)%4
//   comm stream     allreduce(slab t%4) once K(t-1) has filled it — concurrent with K(t)
// K(t+1) waits for allreduce(t); after the loop k_reward_state writes the last tick's reward.
int rollout_sharded_overlap(mdr_ctx* c, const TickArgs* ticks, int n, int mode, double* reward,
                            int64_t rew_stride, double* p_out, hipStream_t st) {
  hipStream_t cs = c->comm_stream;
  auto slab = [&](int t) { return c->d_slab + (size_t)(t % kSlabs) * c->slab_len; };
  HIP_TRY(hipMemsetAsync(c->d_slab, 0, kSlabs * c->slab_len * sizeof(unsigned long long), st));
  hipLaunchKernelGGL(k_power_counts, dim3(blocks(c->kp.n, 256 * kPcHouses)), dim3(256), 0, st, c->kp, nullptr,
                     mode, (uint64_t)0, ticks, slab(0));
  LAUNCH_CHECK("k_power_counts");
  HIP_TRY(hipEventRecord(c->ev_pc, st));
  for (int t = 0; t < n; ++t) {
    // comm stream: counts of tick t are complete once K(t-1) (or phase 1) has finished
    HIP_TRY(hipStreamWaitEvent(cs, t == 0 ? c->ev_pc : c->ev_k1[(t - 1) % kSlabs], 0));
    if (int rc = comm_allreduce(c, slab(t), c->slab_len, 0, cs)) return rc;
    HIP_TRY(hipEventRecord(c->ev_ar[t % kSlabs], cs));
    // compute stream: K(t) needs the allreduced counts of tick t-1 for that tick's reward
    if (t >= 1) HIP_TRY(hipStreamWaitEvent(st, c->ev_ar[(t - 1) % kSlabs], 0));
    int rc = launch_step_on(c, nullptr, mode, TickArgs{}, ticks + t,
                            t >= 1 ? reward + (int64_t)(t - 1) * rew_stride : reward, mode, MDR_CTRL_NONE,
                            nullptr, nullptr, t >= 1 ? slab(t - 1) : nullptr, slab(t + 1), slab(t + 2),
                            1, st);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->ev_k1[t % kSlabs], st));
  }
  HIP_TRY(hipStreamWaitEvent(st, c->ev_ar[(n - 1) % kSlabs], 0));
  hipLaunchKernelGGL(k_reward_state, dim3(blocks(c->kp.n, 256)), dim3(256), 0, st, c->kp,
                     ticks + (n - 1), slab(n - 1), reward + (int64_t)(n - 1) * rew_stride, p_out);
  LAUNCH_CHECK("k_reward_state");
  // leave the step path's invariant (slab ring+1 zero) behind
  HIP_TRY(hipMemsetAsync(c->d_slab, 0, kSlabs * c->slab_len * sizeof(unsigned long long), st));
  c->ring = 0;
  c->counts_ready = false;
  return MDR_OK;
}

// Serial sharded ticks on one stream: [phase 1 if needed] -> allreduce(counts) -> k_step.
int rollout_sharded_serial(mdr_ctx* c, const TickArgs* ticks, int n, const uint8_t* action,
                           int64_t act_stride, int mode, double* reward, int64_t rew_stride,
                           double* p_out, hipStream_t st) {
  HIP_TRY(hipMemsetAsync(c->d_slab, 0, kSlabs * c->slab_len * sizeof(unsigned long long), st));
  c->ring = 0;
  const bool la = lookahead_ok(mode);
  for (int t = 0; t < n; ++t) {
    const uint8_t* a = action ? action + (int64_t)t * act_stride : nullptr;
    if (!la || t == 0) {
      hipLaunchKernelGGL(k_power_counts, dim3(blocks(c->kp.n, 256 * kPcHouses)), dim3(256), 0, st, c->kp, a, mode,
                         (uint64_t)0, ticks + t, slab_at(c, c->ring));
      LAUNCH_CHECK("k_power_counts");
    }
    if (int rc = comm_allreduce(c, slab_at(c, c->ring), c->slab_len, 0, st)) return rc;
    int rc = launch_step(c, a, mode, TickArgs{}, ticks + t, reward + (int64_t)t * rew_stride,
                         la ? mode : 0, MDR_CTRL_NONE, nullptr, t == n - 1 ? p_out : nullptr, st);
    if (rc) return rc;
  }
  c->counts_ready = false;
  return MDR_OK;
}

}  // namespace

extern "C" {

int mdr_rollout_sharded(mdr_ctx* c, int n, const mdr_tick* ticks, const uint8_t* action,
                        int64_t act_stride, int mode, double* reward, int64_t rew_stride, double* p_out,
                        void* stream) {
  if (!c || !ticks || !reward || n < 1) return fail(MDR_EARG, "mdr_rollout_sharded: bad argument");
  // a single window begun by mdr_rollout_begin on this sharded context (count, allreduce, P-only
  // reduce already issued): only the KA step kernel is left, with these drivers as its arguments
  if (c->begun.on && c->begun.sharded && has_comm(c) && c->begun.n == n && c->begun.mode == mode &&
      c->begun.tick0 == ticks[0].tick && c->begun.action == action && c->begun.act_stride == act_stride &&
      window_ok(c, mode) && n <= c->win && consecutive(ticks, n)) {
    c->begun.on = false;
    hipStream_t st = S(stream);
    int rc = ensure_ticks(c, n);
    if (!rc)
      rc = window_launches(c, n, c->d_ticks, action, act_stride, mode, reward, rew_stride, p_out, false, st, true,
                           false, ticks, true);
    c->counts_ready = false;
    return rc;
  }
  drop_begun(c);
  if (!c->bound) return fail(MDR_ESTATE, "mdr_rollout_sharded: context not bound");
  if (!has_comm(c)) return fail(MDR_ESTATE, "mdr_rollout_sharded: no communicator (mdr_rccl_init / mdr_comm_host)");
  if (!check_mode(mode) || (mode == MDR_ACT_BUFFER && !action)) return fail(MDR_EARG, "mdr_rollout_sharded: bad action source");
  if (mode == MDR_ACT_BANGBANG || mode == MDR_ACT_DEADBAND_BANGBANG)
    return fail(MDR_EARG, "mdr_rollout_sharded: bang-bang sources need the per-step API");
  if (c->kp.penalty_mode != MDR_PEN_INDIVIDUAL_L2)
    return fail(MDR_EARG, "mdr_rollout_sharded: common penalty modes need the per-step API");
  hipStream_t st = S(stream);
  int rc = refresh_if_dirty(c, st);
  if (rc) return rc;
  rc = stage_ticks(c, n, ticks, st);
  if (rc) return rc;
  if (window_ok(c, mode)) {
    rc = wslab_clean(c, st);
    if (rc) return rc;
    const bool pipe = c->win_pipe && c->comm_stream && pipe_buffers(c);
    rc = window_launches(c, n, c->d_ticks, action, act_stride, mode, reward, rew_stride, p_out, true, st, false,
                         pipe);
    c->counts_ready = false;
    return rc;
  }
  const bool can_overlap = lookahead_ok(mode) && rew_stride != 0 && c->comm_stream;
  if (can_overlap && c->tick_overlap)
    return rollout_sharded_overlap(c, c->d_ticks, n, mode, reward, rew_stride, p_out, st);
  return rollout_sharded_serial(c, c->d_ticks, n, action, act_stride, mode, reward, rew_stride, p_out, st);
}

int mdr_rollout_sharded_mode(mdr_ctx* c, int* window_pipeline, int* tick_overlap) {
  if (!c || !window_pipeline || !tick_overlap) return fail(MDR_EARG, "mdr_rollout_sharded_mode: null argument");
  *window_pipeline = c->win > 0 && c->win_pipe && c->comm_stream != nullptr;
  *tick_overlap = c->tick_overlap && c->comm_stream != nullptr;
  return MDR_OK;
}

int mdr_set_rollout_window(mdr_ctx* c, int ticks) {
  drop_begun(c);
  if (!c || ticks < 0 || ticks > kWindowMax) return fail(MDR_EARG, "mdr_set_rollout_window: ticks outside 0..32");
  if (ticks > 0 && !c->d_wslab) return fail(MDR_EARG, "mdr_set_rollout_window: more than 4 capacity classes");
  if (ticks != c->win) {
    HIP_TRY(hipDeviceSynchronize());  // cached graphs may be in flight
    destroy_graphs(c);
    c->win = ticks;
  }
  return MDR_OK;
}

int mdr_cluster_stats(mdr_ctx* c, const double* reward, double* out, void* stream) {
  if (!c || !out) return fail(MDR_EARG, "mdr_cluster_stats: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_cluster_stats: context not bound");
  if (!c->d_stats) HIP_TRY(hipMalloc(&c->d_stats, sizeof(double) * kStats * kStatsBlocks));
  const unsigned nb = (unsigned)std::min<int64_t>(kStatsBlocks, (c->kp.n + 255) / 256);
  hipLaunchKernelGGL(k_cluster_stats, dim3(nb), dim3(256), 0, S(stream), c->kp, reward, c->d_stats);
  LAUNCH_CHECK("k_cluster_stats");
  hipLaunchKernelGGL(k_cluster_stats_final, dim3(1), dim3(64), 0, S(stream), c->d_stats, (int)nb, out);
  LAUNCH_CHECK("k_cluster_stats_final");
  return MDR_OK;
}

int mdr_params_changed(mdr_ctx* c) {
  drop_begun(c);
  if (!c) return fail(MDR_EARG, "mdr_params_changed: null ctx");
  c->coef_dirty = true;
  c->gq_map_stale = true;
  c->gq_s1 = c->gq_s2 = NAN;
  return MDR_OK;
}

// ------------------------------------------------------------------------------------ diagnostics
int mdr_probe_stream(mdr_ctx* c, double* reward, void* stream) {
  drop_begun(c);
  if (!c || !reward) return fail(MDR_EARG, "mdr_probe_stream: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_probe_stream: context not bound");
  hipLaunchKernelGGL(k_probe_stream, dim3(blocks(c->kp.n, 512)), dim3(256), 0, S(stream), c->kp, reward);
  LAUNCH_CHECK("k_probe_stream");
  return MDR_OK;
}

int mdr_div_check(const double* a, const double* b, int64_t n, int64_t* mismatches, void* stream) {
  if (!a || !b || !mismatches || n < 0) return fail(MDR_EARG, "mdr_div_check: bad argument");
  HIP_TRY(hipMemsetAsync(mismatches, 0, sizeof(int64_t), S(stream)));
  hipLaunchKernelGGL(k_div_check, dim3(blocks(n, 256)), dim3(256), 0, S(stream), a, b, n,
                     reinterpret_cast<unsigned long long*>(mismatches));
  LAUNCH_CHECK("k_div_check");
  return MDR_OK;
}

// ------------------------------------------------------------------------------------ events
int mdr_event_record(mdr_ctx* c, int slot, void* stream) {
  if (!c || slot < 0 || slot >= 16) return fail(MDR_EARG, "mdr_event_record: bad slot");
  HIP_TRY(hipEventRecord(c->ev[slot], S(stream)));
  return MDR_OK;
}

int mdr_event_elapsed_ms(mdr_ctx* c, int s0, int s1, float* ms) {
  if (!c || !ms || s0 < 0 || s1 < 0 || s0 >= 16 || s1 >= 16) return fail(MDR_EARG, "mdr_event_elapsed_ms: bad slot");
  HIP_TRY(hipEventSynchronize(c->ev[s1]));
  HIP_TRY(hipEventElapsedTime(ms, c->ev[s0], c->ev[s1]));
  return MDR_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------ actor
namespace {

int align16(int x) { return (x + 15) & ~15; }

// Packed-image offsets, the obs row's slot layout and the LDS plan of k_actor for `nw` waves per
// block (mdr_actor.h ActorDims).
// the fused kernel's PREC for the loaded actor: 1 bf16, 3 bf16x3, fp32: 4 (the fp16 split, default) or
// 6 (the three-way bf16 split, MDR_OPT_ACTOR_FP32_FORM)
int actor_kprec(const mdr_ctx* c) {
  const int p = c->actor.precision;
  return p == MDR_PREC_BF16 ? 1 : p == MDR_PREC_FP32 ? (c->actor_fp32_bf16 ? 6 : 4) : 3;
}

ActorDims actor_layout(const mdr_actor_spec& a, const mdr_obs_spec* sp, int nw, int kprec) {
  ActorDims d{};
  d.n_in = a.n_in; d.h1 = a.h1; d.h2 = a.h2; d.n_act = a.n_act;
  const int mbn = (std::max(a.h1, a.h2) + kActorRB - 1) / kActorRB;
  d.mb = mbn <= 7 ? 7 : 8;  // (the kernel's instantiations)
  d.nf = kprec == 6 ? 3 : 2;
  d.f16 = kprec == 4;
  const int K = sp->n_comm, M = mdr_msg_width(sp);
  d.n_comm = K;
  d.msg_w = M;
  d.n_own = a.n_in - K * M;
  d.own4 = (d.n_own + 3) & ~3;
  d.m4 = (M + 3) & ~3;
  d.ring = sp->comm_mode == MDR_COMM_RING && K > 0;
  d.lo = d.ring ? K / 2 : 0;
  d.nslot = d.own4 + K * d.m4;
  d.ks1 = std::max(2, (d.nslot + 31) / 32);  // (the kernel's instantiations: 2, 3, 4; a padding k-step is zero)
  int rs = d.ring ? d.m4 + d.own4 : d.nslot;
  if (((rs / 4) & 1) == 0) rs += 4;  // odd multiple of 16 B: conflict-free ds_read_b128 of 16 rows
  d.rs = rs;
  d.nrows = d.ring ? d.lo + 32 + (K + 1) / 2 : 32;
  d.off_w1 = 0;
  d.off_w2 = d.mb * d.ks1 * d.nf * 1024;
  d.off_tail = d.off_w2 + d.mb * kActorKS2 * d.nf * 1024;
  d.off_end = align16(d.off_tail + kActorTailEnd * 4);
  d.lds_cf = d.off_end;
  d.lds_hist = d.lds_cf + align16(kObsConst * 4);
  d.lds_b1 = d.lds_hist + MDR_MAX_CAP * 4;
  d.lds_wave = d.lds_b1 + (d.f16 ? 2 * kActorRows * 4 + 16 : 0);  // (b1, b2, max of the fp16 split: mdr_actor.hip)

  d.w_zero = align16(d.nrows * rs * 4);
  d.w_hw = d.w_zero + 16;
  d.w_cls = d.w_hw + 32 * 4;
  d.wave_stride = align16(d.w_cls + 32);
  d.lds_total = d.lds_wave + nw * d.wave_stride;
  return d;
}

// the obs layout k_actor<..., DEF = true> fixes at compile time: the reference's defaults (the
// 'neighbours' ring, messages of 4 features, no hvac / solar / thermal state features), <= 64 slots, rows of 20 floats
bool actor_def_layout(const mdr_ctx* c, const mdr_obs_spec* sp, const ActorDims& d) {
  return !c->actor_generic && sp->comm_mode == MDR_COMM_RING && sp->n_comm > 0 && !sp->hvac_state && !sp->solar_state &&
         !sp->thermal_state && !sp->msg_thermal && !sp->msg_hvac && d.ring && d.msg_w == 4 && d.n_own == 10 &&
         d.ks1 == 2 && d.rs == 20;
}

int actor_plan(const mdr_ctx* c, const mdr_obs_spec* sp, ActorDims* d, int* nw) {
  const int prec = actor_kprec(c);
  *d = actor_layout(c->actor, sp, 1, prec);
  if (d->n_own < 0 || d->nslot > kActorMaxSlots)
    return fail(MDR_EARG, "mdr_actor: obs row wider than the actor's 128 feature slots");
  for (int w = actor_max_waves(prec, actor_def_layout(c, sp, *d)); w >= 1; --w) {
    *d = actor_layout(c->actor, sp, w, prec);
    d->w1raw = c->d_actor_raw;
    if (d->lds_total <= 160 * 1024) { *nw = w; return MDR_OK; }
  }
  return fail(MDR_EARG, "mdr_actor: weights + obs rows exceed the 160 KiB LDS of a CU");
}

// the loaded net takes the fused k_actor for this obs layout (two hidden layers <= 128 wide, the obs
// row within 128 slots, weights + rows within the LDS); otherwise the chain runs it
bool actor_fused_ok(const mdr_ctx* c, const mdr_obs_spec* sp) {
  const mdr_actor_net& a = c->net;
  if (a.n_hidden != 2 || a.hidden[0] > kActorRows || a.hidden[1] > kActorRows || a.n_in > kActorMaxIn) return false;
  ActorDims d;
  int nw = 0;
  const std::string keep = g_err;
  const bool ok = actor_plan(c, sp, &d, &nw) == MDR_OK;
  g_err = keep;
  return ok;
}

// offsets of layer l's weights in the loaded fp32 image [w0 b0 w1 b1 ... wL bL]
size_t net_w_off(const mdr_actor_net& a, int l) {
  size_t o = 0;
  int in = a.n_in;
  for (int k = 0; k < l; ++k) {
    const int out = k < a.n_hidden ? a.hidden[k] : a.n_act;
    o += (size_t)out * in + out;
    in = out;
  }
  return o;
}
int net_width(const mdr_actor_net& a) {
  int w = 0;
  for (int l = 0; l < a.n_hidden; ++l) w = std::max(w, a.hidden[l]);
  return w;
}

// the chain's row buffers for n houses and an F-feature obs row (allocated before any capture)
int chain_ensure(mdr_ctx* c, int F, hipStream_t st) {
  const size_t w4 = (size_t)((net_width(c->net) + 3) & ~3);
  const size_t need = ((size_t)F + 2 * w4) * (size_t)c->kp.n * sizeof(float);
  if (need <= c->chain_cap) return MDR_OK;
  HIP_TRY(hipStreamSynchronize(st));
  hipFree(c->d_chain);
  c->d_chain = nullptr;
  HIP_TRY(hipMalloc(&c->d_chain, need));
  c->chain_cap = need;
  for (auto& g : c->actor_graphs) hipGraphExecDestroy(g.second);
  c->actor_graphs.clear();
  return MDR_OK;
}

// The packed weight image for this obs layout (k_actor_pack from the loaded fp32 weights): packed
// again only when the slot layout or the precision changes.  Called by every actor entry point
// before it launches or captures anything.  (The chain needs no packing: its row buffers.)
int actor_ensure_packed(mdr_ctx* c, const mdr_obs_spec* sp, hipStream_t st) {
  if (!actor_fused_ok(c, sp)) return chain_ensure(c, sp->n_feat, st);
  ActorDims d;
  int nw = 0;
  if (int rc = actor_plan(c, sp, &d, &nw)) return rc;
  const std::vector<int> key{d.n_own, d.own4, d.msg_w, d.m4, d.n_comm, d.mb, d.ks1, d.nf, d.ring, d.lo,
                             c->actor.precision, d.f16};
  if (key == c->actor_key) return MDR_OK;
  if ((size_t)d.off_end > c->actor_cap) {
    HIP_TRY(hipStreamSynchronize(st));
    hipFree(c->d_actor);
    c->d_actor = nullptr;
    HIP_TRY(hipMalloc(&c->d_actor, d.off_end));
    c->actor_cap = d.off_end;
    for (auto& g : c->actor_graphs) hipGraphExecDestroy(g.second);
    c->actor_graphs.clear();
  }
  const mdr_actor_spec& a = c->actor;
  const float* w1 = c->d_actor_raw;
  const float* b1 = w1 + (size_t)a.h1 * a.n_in;
  const float* w2 = b1 + a.h1;
  const float* b2 = w2 + (size_t)a.h2 * a.h1;
  const float* w3 = b2 + a.h2;
  const float* b3 = w3 + (size_t)kActorNA * a.h2;
  ActorFold fo{};
  if (d.f16) {  // the folded features (mdr_actor.h ActorFold) and bounds on their values (obs_consts)
    int off[3], mk[3];
    int u = obs_uniform_own(sp->hvac_state, sp->solar_state, sp->thermal_state, fo.feat, fo.cf);
    fo.nu_own = u;
    const int um = obs_uniform_msg(sp->msg_thermal, sp->msg_hvac, off, mk);
    for (int k = 0; k < d.n_comm; ++k)
      for (int j = 0; j < um && u < kActorMaxU; ++j) {
        fo.feat[u] = d.n_own + k * d.msg_w + off[j];
        fo.cf[u++] = mk[j];
      }
    fo.nu = u;
    double pmax = 0.0;
    for (int k = 0; k < c->cfg.n_cap; ++k) pmax = std::max(pmax, fabs(c->cfg.cap_table[k] / c->cfg.cop));
    const double R = sp->norm_reg_sig != 0.0 ? fabs(sp->norm_reg_sig) : 1.0;
    for (int j = 0; j < u; ++j) {
      const int k = fo.cf[j];
      // P / R <= n_global P_on,max / R (every house on); the signal, solar, deadband and OD features
      // are O(1) after norm.py's scaling (64 is a bound for the scale choice only: a value beyond it
      // is still exact, k_actor's range check sends its tile to the fp32 fallback)
      const double b = k == 3 ? (double)c->kp.n_global * pmax / R : k <= 2 ? 1.0 : k == 8 ? fabs(c->cfg.cop)
                       : k == 9 ? fabs(c->cfg.lcf) : k == 10 ? fabs(sp->cfg_cap) : 64.0;
      fo.cfmax[j] = (float)std::min(b, 3.0e38);
    }
  }
  const int nthreads = (d.mb * (d.ks1 + kActorKS2) + 1) * 64;
  hipLaunchKernelGGL(k_actor_pack, dim3(blocks(nthreads, 256)), dim3(256), 0, st, d, fo, w1, b1, w2, b2, w3, b3,
                     c->d_actor);
  LAUNCH_CHECK("k_actor_pack");
  c->actor_key = key;
  return MDR_OK;
}

#define MDR_ACTOR_KERNELS_D(MB, KS, D)                                                                 \
  (const void*)k_actor<1, false, MB, KS, D>, (const void*)k_actor<3, false, MB, KS, D>,                   \
      (const void*)k_actor<4, false, MB, KS, D>, (const void*)k_actor<6, false, MB, KS, D>,               \
      (const void*)k_actor<1, true, MB, KS, D>, (const void*)k_actor<3, true, MB, KS, D>,                 \
      (const void*)k_actor<4, true, MB, KS, D>, (const void*)k_actor<6, true, MB, KS, D>
#define MDR_ACTOR_KERNELS(MB, KS) MDR_ACTOR_KERNELS_D(MB, KS, false)


// The general actor as a chain of launches (mdr_actor.hip "chain"): obs rows (into out.obs when the
// caller keeps them), one k_dense per hidden layer (ping-pong row buffers), k_actor_head.
int launch_actor_chain(mdr_ctx* c, const mdr_obs_spec* sp, const ObsArgs& o, const double* p_dev, uint64_t tick,
                       const TickArgs* tkp, const ActorOut& out, hipStream_t st) {
  if (out.prof) return fail(MDR_EARG, "mdr_actor_profile: the chained actor has no phase profile");
  const mdr_actor_net& a = c->net;
  const int64_t n = c->kp.n;
  const int F = sp->n_feat;
  const int w4 = (net_width(a) + 3) & ~3;
  float* x0 = out.obs ? out.obs : c->d_chain;
  float* hb[2] = {c->d_chain + (size_t)F * n, c->d_chain + ((size_t)F + w4) * n};
  const int lo = sp->n_comm / 2, hi = (sp->n_comm + 1) / 2;
  const size_t tile = ((size_t)kObsBlock * F + 3) & ~(size_t)3;
  const size_t bytes = (tile + (size_t)(lo + kObsBlock + hi) * o.msg_w) * sizeof(float);
  if (bytes > 160 * 1024) return fail(MDR_EARG, "mdr_actor: obs row too wide for one LDS tile");
  hipLaunchKernelGGL(k_obs, dim3(blocks(n, kObsBlock)), dim3(kObsBlock), bytes, st, c->kp, o, p_dev, x0);
  LAUNCH_CHECK("k_obs (actor chain)");
  const float* x = x0;
  int ld = F, K = F;
  const float* raw = c->d_actor_raw;
  const int prec = a.precision;
  for (int l = 0; l < a.n_hidden; ++l) {
    const int out_w = a.hidden[l];
    const float* W = raw + net_w_off(a, l);
    const float* b = W + (size_t)out_w * K;
    float* y = hb[l & 1];
    const dim3 grid(blocks(n, 64), blocks(out_w, 64));
    if (prec == MDR_PREC_BF16) hipLaunchKernelGGL(k_dense<1>, grid, dim3(256), 0, st, x, ld, K, n, W, b, out_w, y, w4, 1);
    else if (prec == MDR_PREC_FP32) hipLaunchKernelGGL(k_dense<6>, grid, dim3(256), 0, st, x, ld, K, n, W, b, out_w, y, w4, 1);
    else hipLaunchKernelGGL(k_dense<3>, grid, dim3(256), 0, st, x, ld, K, n, W, b, out_w, y, w4, 1);
    LAUNCH_CHECK("k_dense");
    x = y;
    ld = w4;
    K = out_w;
  }
  const float* W3 = raw + net_w_off(a, a.n_hidden);
  hipLaunchKernelGGL(k_actor_head, dim3(blocks(n, 256)), dim3(256), 0, st, c->kp, x, ld, K, W3, W3 + (size_t)kActorNA * K,
                     tick, tkp, out);
  LAUNCH_CHECK("k_actor_head");
  return MDR_OK;
}

int launch_actor(mdr_ctx* c, const mdr_obs_spec* sp, const ObsArgs& o, const double* p_dev, uint64_t tick,
                 const TickArgs* tkp, const ActorOut& out_in, hipStream_t st) {
  if (!actor_fused_ok(c, sp)) return launch_actor_chain(c, sp, o, p_dev, tick, tkp, out_in, st);
  ActorOut out = out_in;
  out.ovf = reinterpret_cast<unsigned*>(c->d_flags) + 1;  // (mdr_actor_status; read by the fp16 form only)
  ActorDims d;
  int nw = 0;
  if (int rc = actor_plan(c, sp, &d, &nw)) return rc;
  const int64_t ntile_all = (c->kp.n + 31) / 32;
  const int64_t nv = out.tiles == 1 ? ntile_all - 2 : out.tiles == 2 ? 2 : ntile_all;  // (ActorOut.tiles)
  const int64_t ntile = (nv + nw - 1) / nw;  // blocks with at least one tile per wave
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ntile, (int64_t)c->n_cu));
  static bool lds_attr = false;  // > 64 KiB of dynamic LDS must be opted into per kernel
  if (!lds_attr) {
    for (const void* k : {MDR_ACTOR_KERNELS(7, 2), MDR_ACTOR_KERNELS(7, 3), MDR_ACTOR_KERNELS(7, 4),
                          MDR_ACTOR_KERNELS(8, 2), MDR_ACTOR_KERNELS(8, 3), MDR_ACTOR_KERNELS(8, 4),
                          MDR_ACTOR_KERNELS_D(7, 2, true), MDR_ACTOR_KERNELS_D(8, 2, true)})
      HIP_TRY(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    lds_attr = true;
  }
#define MDR_LAUNCH_ACTOR_S(P, F, MB, KS)                                                                     \
  hipLaunchKernelGGL((k_actor<P, F, MB, KS, false>), dim3(grid), dim3(64 * nw), d.lds_total, st, c->kp, o, d, p_dev, \
                     c->d_actor, out, tick, tkp)
#define MDR_LAUNCH_ACTOR_DEF(P, F, MB)                                                                        \
  hipLaunchKernelGGL((k_actor<P, F, MB, 2, true>), dim3(grid), dim3(64 * nw), d.lds_total, st, c->kp, o, d, p_dev, \
                     c->d_actor, out, tick, tkp)
  const bool def = actor_def_layout(c, sp, d);
#define MDR_LAUNCH_ACTOR(P, F)                                 \
  do {                                                         \
    if (def && d.mb == 7) MDR_LAUNCH_ACTOR_DEF(P, F, 7);         \
    else if (def) MDR_LAUNCH_ACTOR_DEF(P, F, 8);                 \
    else if (d.mb == 7 && d.ks1 == 2) MDR_LAUNCH_ACTOR_S(P, F, 7, 2); \
    else if (d.mb == 7 && d.ks1 == 3) MDR_LAUNCH_ACTOR_S(P, F, 7, 3); \
    else if (d.mb == 7) MDR_LAUNCH_ACTOR_S(P, F, 7, 4);          \
    else if (d.ks1 == 2) MDR_LAUNCH_ACTOR_S(P, F, 8, 2);         \
    else if (d.ks1 == 3) MDR_LAUNCH_ACTOR_S(P, F, 8, 3);         \
    else MDR_LAUNCH_ACTOR_S(P, F, 8, 4);                         \
  } while (0)
  const int prec = actor_kprec(c);
  if (out.prof) {
    if (prec == 1) MDR_LAUNCH_ACTOR(1, true);
    else if (prec == 4) MDR_LAUNCH_ACTOR(4, true);
    else if (prec == 6) MDR_LAUNCH_ACTOR(6, true);
    else MDR_LAUNCH_ACTOR(3, true);
  } else {
    if (prec == 1) MDR_LAUNCH_ACTOR(1, false);
    else if (prec == 4) MDR_LAUNCH_ACTOR(4, false);
    else if (prec == 6) MDR_LAUNCH_ACTOR(6, false);
    else MDR_LAUNCH_ACTOR(3, false);
  }
#undef MDR_LAUNCH_ACTOR
#undef MDR_LAUNCH_ACTOR_S
#undef MDR_LAUNCH_ACTOR_DEF
  LAUNCH_CHECK("k_actor");
  return MDR_OK;
}

// the spec is valid for the loaded actor; the weights are packed for its slot layout (before any
// launch or graph capture of the caller)
int check_actor_obs(mdr_ctx* c, const mdr_obs_spec* sp, const char* who, hipStream_t st) {
  if (!c->actor_ready) return fail(MDR_ESTATE, std::string(who) + ": no actor loaded (mdr_actor_load)");
  if (int rc = check_obs_spec(sp, who)) return rc;
  if (sp->n_feat != c->actor.n_in) return fail(MDR_EARG, std::string(who) + ": obs n_feat != actor n_in");
  return actor_ensure_packed(c, sp, st);
}

}  // namespace

extern "C" {

int mdr_actor_load_net(mdr_ctx* c, const mdr_actor_net* a, const float* const* w, const float* const* b,
                       void* stream) {
  if (!c || !a || !w || !b) return fail(MDR_EARG, "mdr_actor_load_net: null argument");
  if (a->n_in < 1 || a->n_in > 4096 || a->n_hidden < 1 || a->n_hidden > MDR_ACTOR_MAX_LAYERS || a->n_act != kActorNA)
    return fail(MDR_EARG, "mdr_actor_load_net: shape outside 1 <= n_in <= 4096, 1..8 hidden layers, n_act == 2");
  for (int l = 0; l < a->n_hidden; ++l)
    if (a->hidden[l] < 1 || a->hidden[l] > 4096) return fail(MDR_EARG, "mdr_actor_load_net: hidden width outside 1..4096");
  if (a->precision != MDR_PREC_BF16 && a->precision != MDR_PREC_BF16X3 && a->precision != MDR_PREC_FP32)
    return fail(MDR_EARG, "mdr_actor_load_net: bad precision");
  for (int l = 0; l <= a->n_hidden; ++l)
    if (!w[l] || !b[l]) return fail(MDR_EARG, "mdr_actor_load_net: null layer");
  // the fp32 weights, kept on device: the fused kernel's packed image depends on the obs layout, so
  // it is made by the first actor call of each layout (actor_ensure_packed)
  const size_t nraw = net_w_off(*a, a->n_hidden + 1);
  // captured actor graphs hold the chain's weight pointers and the fused / chain choice: they stay
  // valid while the buffer and the net's shape do (a PPO update reloads weights of the same shape)
  const bool same = c->actor_ready && memcmp(&c->net, a, sizeof(mdr_actor_net)) == 0;
  if (!same || nraw * sizeof(float) > c->actor_raw_cap) {
    for (auto& g : c->actor_graphs) hipGraphExecDestroy(g.second);
    c->actor_graphs.clear();
  }
  if (nraw * sizeof(float) > c->actor_raw_cap) {
    HIP_TRY(hipStreamSynchronize(S(stream)));
    hipFree(c->d_actor_raw);
    c->d_actor_raw = nullptr;
    HIP_TRY(hipMalloc(&c->d_actor_raw, nraw * sizeof(float)));
    c->actor_raw_cap = nraw * sizeof(float);
  }
  float* r = c->d_actor_raw;
  int in = a->n_in;
  for (int l = 0; l <= a->n_hidden; ++l) {
    const int out = l < a->n_hidden ? a->hidden[l] : a->n_act;
    HIP_TRY(hipMemcpyAsync(r, w[l], (size_t)out * in * sizeof(float), hipMemcpyDeviceToDevice, S(stream)));
    r += (size_t)out * in;
    HIP_TRY(hipMemcpyAsync(r, b[l], (size_t)out * sizeof(float), hipMemcpyDeviceToDevice, S(stream)));
    r += out;
    in = out;
  }
  c->actor_key.clear();
  c->net = *a;
  c->actor = mdr_actor_spec{a->n_in, a->hidden[0], a->n_hidden > 1 ? a->hidden[1] : 0, a->n_act, a->precision};
  c->actor_ready = true;
  return MDR_OK;
}

int mdr_actor_load(mdr_ctx* c, const mdr_actor_spec* a, const float* w1, const float* b1, const float* w2,
                   const float* b2, const float* w3, const float* b3, void* stream) {
  if (!c || !a || !w1 || !b1 || !w2 || !b2 || !w3 || !b3) return fail(MDR_EARG, "mdr_actor_load: null argument");
  mdr_actor_net net{};
  net.n_in = a->n_in;
  net.n_hidden = 2;
  net.n_act = a->n_act;
  net.precision = a->precision;
  net.hidden[0] = a->h1;
  net.hidden[1] = a->h2;
  const float* w[3] = {w1, w2, w3};
  const float* b[3] = {b1, b2, b3};
  return mdr_actor_load_net(c, &net, w, b, stream);
}

int mdr_actor_status(mdr_ctx* c, int64_t* out, int n, void* stream) {
  if (!c || !out || n < 3) return fail(MDR_EARG, "mdr_actor_status: need out[3]");
  unsigned v[2] = {0u, 0u};
  HIP_TRY(hipStreamSynchronize(S(stream)));
  HIP_TRY(hipMemcpy(v, c->d_flags + 1, sizeof(v), hipMemcpyDeviceToHost));
  const unsigned z[2] = {0u, 0u};
  HIP_TRY(hipMemcpy(c->d_flags + 1, z, sizeof(z), hipMemcpyHostToDevice));
  out[0] = (int64_t)v[0];
  out[1] = c->actor_ready ? actor_kprec(c) : 0;
  out[2] = (int64_t)v[1];
  return MDR_OK;
}

int mdr_actor_fused(mdr_ctx* c, const mdr_obs_spec* sp) {
  if (!c || !sp) return fail(MDR_EARG, "mdr_actor_fused: null argument");
  if (!c->actor_ready) return fail(MDR_ESTATE, "mdr_actor_fused: no actor loaded");
  return actor_fused_ok(c, sp) ? 1 : 0;
}

int mdr_actor_act(mdr_ctx* c, const mdr_obs_spec* sp, const mdr_obs_scalars* sc, const double* p_dev,
                  uint64_t tick, uint8_t* action, float* prob, float* probs, float* obs_out, int count_next,
                  void* stream) {
  drop_begun(c);
  if (!c || !sp || !sc) return fail(MDR_EARG, "mdr_actor_act: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_actor_act: context not bound");
  if (int rc = check_actor_obs(c, sp, "mdr_actor_act", S(stream))) return rc;
  hipStream_t st = S(stream);
  ActorOut out{action, prob, probs, obs_out, nullptr, nullptr};
  if (count_next) {
    // the counts of the tick these actions drive go into the current slab (from zero)
    out.count_next = slab_at(c, c->ring);
    HIP_TRY(hipMemsetAsync(out.count_next, 0, c->slab_len * sizeof(unsigned long long), st));
  }
  if (int rc = launch_actor(c, sp, obs_args(c, sp, sc), p_dev, tick, nullptr, out, st)) return rc;
  if (count_next) c->counts_ready = true;
  return MDR_OK;
}

int mdr_actor_profile(mdr_ctx* c, const mdr_obs_spec* sp, const mdr_obs_scalars* sc, const double* p_dev,
                      double* cycles_out, void* stream) {
  if (!c || !sp || !sc || !cycles_out) return fail(MDR_EARG, "mdr_actor_profile: null argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_actor_profile: context not bound");
  if (int rc = check_actor_obs(c, sp, "mdr_actor_profile", S(stream))) return rc;
  hipStream_t st = S(stream);
  const int nb = c->n_cu * 16;  // waves (at most 16 per block, one block per CU)
  unsigned long long* d = nullptr;
  HIP_TRY(hipMalloc(&d, (size_t)nb * 8 * sizeof(unsigned long long)));
  HIP_TRY(hipMemsetAsync(d, 0, (size_t)nb * 8 * sizeof(unsigned long long), st));
  ActorOut out{nullptr, nullptr, nullptr, nullptr, nullptr, d};
  int rc = launch_actor(c, sp, obs_args(c, sp, sc), p_dev, 0, nullptr, out, st);
  std::vector<unsigned long long> h((size_t)nb * 8);
  if (!rc && hipStreamSynchronize(st) == hipSuccess &&
      hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess) {
    int used = 0;
    for (int k = 0; k < 8; ++k) cycles_out[k] = 0.0;
    for (int b = 0; b < nb; ++b) {
      if (h[b * 8 + 7] == 0) continue;
      ++used;
      for (int k = 0; k < 8; ++k) cycles_out[k] += (double)h[b * 8 + k];
    }
    for (int k = 0; k < 8; ++k) cycles_out[k] /= used ? used : 1;
  } else if (!rc) {
    rc = fail(MDR_EHIP, "mdr_actor_profile: readback");
  }
  hipFree(d);
  return rc;
}

int mdr_actor_rollout(mdr_ctx* c, int n, const mdr_tick* ticks, const mdr_obs_scalars* osc,
                      const mdr_obs_spec* sp, uint8_t* action, int64_t act_stride, float* prob,
                      int64_t prob_stride, double* reward, int64_t rew_stride, double* p_dev, int use_graph,
                      void* stream) {
  drop_begun(c);
  if (!c || !ticks || !osc || !sp || !reward || !p_dev || n < 1) return fail(MDR_EARG, "mdr_actor_rollout: bad argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_actor_rollout: context not bound");
  if (int rc = check_actor_obs(c, sp, "mdr_actor_rollout", S(stream))) return rc;
  if (c->kp.penalty_mode != MDR_PEN_INDIVIDUAL_L2)
    return fail(MDR_EARG, "mdr_actor_rollout: common penalty modes need the per-step API");
  hipStream_t st = S(stream);
  if (int rc = refresh_if_dirty(c, st)) return rc;
  if (int rc = stage_ticks(c, n, ticks, st)) return rc;
  // per-tick obs scalars [s, solar, t_od, -] next to the tick drivers (same capacity)
  if (int rc = stage_recs(osc, n, c->d_obs_sc, st)) return rc;

  ObsArgs o = obs_args(c, sp, &osc[0]);
  auto launches = [&](hipStream_t ls) -> int {
    if (int rc = zero_slabs(c, ls)) return rc;
    c->ring = 0;
    for (int t = 0; t < n; ++t) {
      // the current slab is zero here: the memset above (t = 0), then the previous two steps
      // (each zeroes the slab two ahead and a BUFFER step writes no lookahead)
      ObsArgs ot = o;
      ot.sc_dev = c->d_obs_sc + 4 * t;
      ActorOut out{action ? action + (int64_t)t * act_stride : c->d_act, prob ? prob + (int64_t)t * prob_stride : nullptr,
                   nullptr, nullptr, slab_at(c, c->ring), nullptr};
      if (int rc = launch_actor(c, sp, ot, p_dev, 0, c->d_ticks + t, out, ls)) return rc;
      if (int rc = launch_step(c, out.action, MDR_ACT_BUFFER, TickArgs{}, c->d_ticks + t,
                               reward + (int64_t)t * rew_stride, 0, MDR_CTRL_NONE, nullptr, p_dev, ls))
        return rc;
    }
    return MDR_OK;
  };
  if (!action && !c->d_act) HIP_TRY(hipMalloc(&c->d_act, c->kp.n));  // context-owned action row
  if (!use_graph) {
    const int rc = launches(st);
    c->counts_ready = false;
    return rc;
  }
  std::vector<int64_t> key{n, (int64_t)(uintptr_t)action, act_stride, (int64_t)(uintptr_t)prob, prob_stride,
                           (int64_t)(uintptr_t)reward, rew_stride, (int64_t)(uintptr_t)p_dev,
                           (int64_t)(uintptr_t)sp->comm_table,
                           (int64_t)(uintptr_t)sp->halo_msg, sp->n_feat, (int64_t)(uintptr_t)c->d_actor};
  auto it = c->actor_graphs.find(key);
  if (it == c->actor_graphs.end()) {
    hipGraphExec_t ex;
    if (int rc = capture_graph(c, launches, &ex)) return rc;
    it = c->actor_graphs.emplace(key, ex).first;
  } else {
    c->ring = n % 3;
  }
  HIP_TRY(hipGraphLaunch(it->second, st));
  ++c->graph_launches[1];
  c->counts_ready = false;
  return MDR_OK;
}

// Sharded MA-PPO rollout (config C5): per tick
//   [ring obs across shards] k_halo_pack -> grouped RCCL send/recv of the edge houses' message
//   features with ranks r-1 / r+1 -> k_actor (obs on chip, actions, ON counts of those actions)
//   -> RCCL sum-allreduce of the count slab -> k_step (BUFFER actions, global P)
// Actions are sampled from Philox keyed by (seed, GLOBAL house id, tick) and the counts are exact
// integers, so the sharded run is bit-identical to the single-shard one.
int mdr_actor_rollout_sharded(mdr_ctx* c, int n, const mdr_tick* ticks, const mdr_obs_scalars* osc,
                              const mdr_obs_spec* sp, uint8_t* action, int64_t act_stride, float* prob,
                              int64_t prob_stride, double* reward, int64_t rew_stride, double* p_dev,
                              void* stream) {
  drop_begun(c);
  if (!c || !ticks || !osc || !sp || !reward || !p_dev || n < 1)
    return fail(MDR_EARG, "mdr_actor_rollout_sharded: bad argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_actor_rollout_sharded: context not bound");
  if (!has_comm(c)) return fail(MDR_ESTATE, "mdr_actor_rollout_sharded: no communicator (mdr_rccl_init / mdr_comm_host)");
  if (int rc = check_actor_obs(c, sp, "mdr_actor_rollout_sharded", S(stream))) return rc;
  if (c->kp.penalty_mode != MDR_PEN_INDIVIDUAL_L2)
    return fail(MDR_EARG, "mdr_actor_rollout_sharded: common penalty modes need the per-step API");
  const int K = sp->n_comm, M = mdr_msg_width(sp);
  const int lo = K / 2, hi = (K + 1) / 2;
  // MDR_FORCE_HALO=1 (test hook): exchange the halo even at world 1 (send/recv to self), which
  // must reproduce the local ring wrap-around — the 1-GPU check of the multi-GPU exchange
  const bool halo = (c->world > 1 || c->force_halo) && K > 0;
  if (halo && sp->comm_mode != MDR_COMM_RING)
    return fail(MDR_EARG, "mdr_actor_rollout_sharded: across shards only the 'neighbours' ring obs is supported");
  if (halo && c->kp.n < (lo > hi ? lo : hi))
    return fail(MDR_EARG, "mdr_actor_rollout_sharded: shard smaller than the ring half-width");
  hipStream_t st = S(stream);
  if (int rc = refresh_if_dirty(c, st)) return rc;
  if (int rc = stage_ticks(c, n, ticks, st)) return rc;
  if (int rc = stage_recs(osc, n, c->d_obs_sc, st)) return rc;
  if (!action && !c->d_act) HIP_TRY(hipMalloc(&c->d_act, c->kp.n));
  const size_t hbytes = (size_t)2 * (lo + hi) * M * sizeof(float);
  if (halo && hbytes > c->halo_bytes) {
    HIP_TRY(hipStreamSynchronize(st));
    hipFree(c->d_halo);
    c->d_halo = nullptr;
    HIP_TRY(hipMalloc(&c->d_halo, hbytes));
    c->halo_bytes = hbytes;
  }
  float* mine = c->d_halo;                                    // [hi first | lo last] of this shard
  float* recv = c->d_halo ? c->d_halo + (size_t)(lo + hi) * M : nullptr;  // [lo before | hi after]
  mdr_obs_spec spec = *sp;
  spec.halo_msg = halo ? recv : nullptr;
  const ObsArgs o = obs_args(c, &spec, &osc[0]);
  if (halo && c->halo_in_counts) {
    // ONE collective per tick: the count slab and every rank's post-step edge rows of tick t (the
    // halo of tick t + 1) in one integer sum-allreduce (k_halo_step_pack); tick 0's halo (of the
    // current state) is exchanged once before the loop
    const int W = lo + hi;
    const size_t rows_words = ((size_t)c->world * W * M + 1) / 2;  // floats, two per u64 word
    const size_t words = c->slab_len + rows_words;
    if (3 * words * sizeof(unsigned long long) > c->c5_bytes) {
      HIP_TRY(hipStreamSynchronize(st));
      hipFree(c->d_c5);
      c->d_c5 = nullptr;
      HIP_TRY(hipMalloc(&c->d_c5, 3 * words * sizeof(unsigned long long)));
      c->c5_bytes = 3 * words * sizeof(unsigned long long);
    }
    auto buf = [&](int t) { return c->d_c5 + (size_t)(t % 3) * words; };
    auto rows = [&](int t) { return reinterpret_cast<float*>(buf(t) + c->slab_len); };
    hipLaunchKernelGGL(k_zero_u64, dim3(1), dim3(256), 0, st, c->d_c5, (int64_t)(3 * words));
    LAUNCH_CHECK("k_zero_u64");
    hipLaunchKernelGGL(k_halo_pack, dim3(1), dim3(64), 0, st, c->kp, o, lo, hi, mine);
    LAUNCH_CHECK("k_halo_pack");
    if (int rc = comm_halo(c, mine, recv, lo, hi, M, st)) return rc;
    const int prev = (c->rank + c->world - 1) % c->world, next = (c->rank + 1) % c->world;
    for (int t = 0; t < n; ++t) {
      ObsArgs ot = o;
      ot.sc_dev = c->d_obs_sc + 4 * t;
      if (t > 0) {  // the previous tick's allreduced rows: rank prev's last lo, rank next's first hi
        ot.halo_msg = rows(t - 1) + (size_t)prev * W * M + (size_t)hi * M;
        ot.halo_next = rows(t - 1) + (size_t)next * W * M;
      }
      ActorOut out{action ? action + (int64_t)t * act_stride : c->d_act,
                   prob ? prob + (int64_t)t * prob_stride : nullptr, nullptr, nullptr, buf(t), nullptr};
      if (int rc = launch_actor(c, &spec, ot, p_dev, 0, c->d_ticks + t, out, st)) return rc;
      hipLaunchKernelGGL(k_halo_step_pack, dim3(1), dim3(256), 0, st, c->kp, ot, (const uint8_t*)out.action,
                         (const TickArgs*)(c->d_ticks + t), lo, hi, c->rank, c->world, rows(t));
      LAUNCH_CHECK("k_halo_step_pack");
      if (int rc = comm_allreduce(c, buf(t), words, 0, st)) return rc;
      c->gq_keys_ready = false;
      c->fz_ready = false;
      if (int rc = launch_step_on(c, out.action, MDR_ACT_BUFFER, TickArgs{}, c->d_ticks + t,
                                  reward + (int64_t)t * rew_stride, 0, MDR_CTRL_NONE, nullptr, p_dev, buf(t),
                                  buf(t + 1), buf(t + 2), 0, st))
        return rc;
    }
    c->counts_ready = false;
    return MDR_OK;
  }
  HIP_TRY(hipMemsetAsync(c->d_slab, 0, kSlabs * c->slab_len * sizeof(unsigned long long), st));
  c->ring = 0;
  // overlap (fused actor, >= 4 tiles, a comm stream): per tick the halo is packed and exchanged on the
  // comm stream while the interior tiles' actor runs on the compute stream; the first and last
  // tile follow once it has landed.  They are the only readers of the halo when lo, hi <= 32 and
  // the last tile holds no house whose ring reaches past it: tile ntile-2 reads houses up to
  // 32 (ntile-1) + hi - 1, beyond the shard when the last tile is short, n % 32 in 1 .. hi-1
  const int64_t rag = c->kp.n % 32;
  const bool overlap = halo && c->halo_overlap && c->comm_stream && actor_fused_ok(c, &spec) &&
                       (c->kp.n + 31) / 32 >= 4 && lo <= 32 && hi <= 32 && (rag == 0 || rag >= hi);
  hipStream_t cs = c->comm_stream;
  for (int t = 0; t < n; ++t) {
    ObsArgs ot = o;
    ot.sc_dev = c->d_obs_sc + 4 * t;
    ActorOut out{action ? action + (int64_t)t * act_stride : c->d_act,
                 prob ? prob + (int64_t)t * prob_stride : nullptr, nullptr, nullptr, slab_at(c, c->ring), nullptr};
    if (overlap) {
      HIP_TRY(hipEventRecord(c->ev_pc, st));  // the state after the previous step
      HIP_TRY(hipStreamWaitEvent(cs, c->ev_pc, 0));
      hipLaunchKernelGGL(k_halo_pack, dim3(1), dim3(64), 0, cs, c->kp, o, lo, hi, mine);
      LAUNCH_CHECK("k_halo_pack");
      ActorOut in = out;
      in.tiles = 1;  // (issued before the exchange: host collectives block in comm_halo)
      if (int rc = launch_actor(c, &spec, ot, p_dev, 0, c->d_ticks + t, in, st)) return rc;
      if (int rc = comm_halo(c, mine, recv, lo, hi, M, cs)) return rc;
      HIP_TRY(hipEventRecord(c->ev_ar[0], cs));
      HIP_TRY(hipStreamWaitEvent(st, c->ev_ar[0], 0));
      out.tiles = 2;
    } else if (halo) {
      hipLaunchKernelGGL(k_halo_pack, dim3(1), dim3(64), 0, st, c->kp, o, lo, hi, mine);
      LAUNCH_CHECK("k_halo_pack");
      // the previous rank's last lo houses come first in the halo, the next rank's first hi after
      if (int rc = comm_halo(c, mine, recv, lo, hi, M, st)) return rc;
    }
    if (int rc = launch_actor(c, &spec, ot, p_dev, 0, c->d_ticks + t, out, st)) return rc;
    if (int rc = comm_allreduce(c, slab_at(c, c->ring), c->slab_len, 0, st)) return rc;
    if (int rc = launch_step(c, out.action, MDR_ACT_BUFFER, TickArgs{}, c->d_ticks + t,
                             reward + (int64_t)t * rew_stride, 0, MDR_CTRL_NONE, nullptr, p_dev, st))
      return rc;
  }
  c->counts_ready = false;
  return MDR_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------ interpolation (a10)
extern "C" {

int mdr_interp_load(mdr_ctx* c, const mdr_interp_spec* sp) {
  if (!c || !sp || !sp->grid || !sp->values) return fail(MDR_EARG, "mdr_interp_load: null argument");
  InterpArgs a{};
  int64_t ng = 0, total = 1;
  for (int k = 0; k < kInterpAxes; ++k) {
    const bool linear = !(k < 4 || k == 7);
    if (sp->len[k] < (linear ? 2 : 1) || sp->len[k] > (1 << 16))
      return fail(MDR_EARG, "mdr_interp_load: axis length out of range");
    a.len[k] = sp->len[k];
    a.off[k] = (int)ng;
    double lo = sp->grid[ng], hi = sp->grid[ng];
    for (int i = 0; i < sp->len[k]; ++i) {
      const double g = sp->grid[ng + i];
      if (linear && i > 0 && !(g > sp->grid[ng + i - 1]))
        return fail(MDR_EARG, "mdr_interp_load: a linear axis is not strictly ascending");
      lo = g < lo ? g : lo;
      hi = g > hi ? g : hi;
    }
    a.lo[k] = lo;
    a.hi[k] = hi;
    ng += sp->len[k];
  }
  for (int k = kInterpAxes - 1; k >= 0; --k) {
    a.stride[k] = total;
    total *= sp->len[k];
  }
  const int lin[kInterpLinear] = {4, 5, 6, 8, 9};
  for (int q = 0; q < kInterpLinear; ++q) a.lstride[q] = a.stride[lin[q]];
  a.cfg[0] = sp->cfg_ua; a.cfg[1] = sp->cfg_cm; a.cfg[2] = sp->cfg_ca; a.cfg[3] = sp->cfg_hm;
  const size_t bytes = (size_t)(ng + total + MDR_MAX_CAP) * sizeof(double);
  HIP_TRY(hipSetDevice(c->cfg.device));
  if (bytes > c->interp_bytes) {
    HIP_TRY(hipDeviceSynchronize());  // a previous table may still be read by queued launches
    hipFree(c->d_interp);
    c->d_interp = nullptr;
    c->interp_bytes = 0;
    if (hipMalloc(&c->d_interp, bytes) != hipSuccess) return fail(MDR_ENOMEM, "mdr_interp_load: table");
    c->interp_bytes = bytes;
  } else {
    HIP_TRY(hipDeviceSynchronize());
  }
  HIP_TRY(hipMemcpy(c->d_interp, sp->grid, ng * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_interp + ng, sp->values, total * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_interp + ng + total, c->cfg.cap_table, MDR_MAX_CAP * sizeof(double),
                    hipMemcpyHostToDevice));
  a.grid = c->d_interp;
  a.table = c->d_interp + ng;
  a.cap = c->d_interp + ng + total;
  c->interp = a;
  c->interp_ready = true;
  return MDR_OK;
}

int mdr_interp_values(mdr_ctx* c, const int64_t* ids, int n, double od, double hour, double date, double* vals,
                      void* stream) {
  if (!c || n < 0 || (n > 0 && (!ids || !vals))) return fail(MDR_EARG, "mdr_interp_values: bad argument");
  if (!c->bound) return fail(MDR_ESTATE, "mdr_interp_values: context not bound");
  if (!c->interp_ready) return fail(MDR_ESTATE, "mdr_interp_values: no table (mdr_interp_load)");
  if (n == 0) return MDR_OK;
  hipLaunchKernelGGL(k_interp_values, dim3(blocks(n, 64)), dim3(64), 0, S(stream), c->kp, c->interp, ids, n,
                     od, hour, date, vals);
  LAUNCH_CHECK("k_interp_values");
  return MDR_OK;
}

int mdr_interp_sum(const double* vals, int n, double factor, double* out, void* stream) {
  if (n < 0 || !out || (n > 0 && !vals)) return fail(MDR_EARG, "mdr_interp_sum: bad argument");
  hipLaunchKernelGGL(k_interp_sum, dim3(1), dim3(64), 0, S(stream), vals, n, factor, out);
  LAUNCH_CHECK("k_interp_sum");
  return MDR_OK;
}

}  // extern "C"
