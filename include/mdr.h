/*
 * mdr.h — C ABI of the MI355X-native vectorised environment step (libmdr_hip.so).
 *
 * Drop-in boundary for the reference's per-tick environment step, ALLabMTL/marl-demandresponse
 * v2 (file:line relative to /root/reference):
 *
 *   Environment.step               server/app/core/environment/environment.py:72-108
 *     Cluster.step (house loop)    server/app/core/environment/cluster/cluster.py:73-89
 *       HVAC.step (lockout FSM)    server/app/core/environment/cluster/hvac.py:43-64
 *       Building.update_temperature server/app/core/environment/cluster/building.py:141-222
 *       get_power_consumption      server/app/core/environment/cluster/hvac.py:101-111
 *     RewardsCalculator            server/app/core/environment/rewards_calculator.py:135-203
 *     Cluster.get_obs / messages   server/app/core/environment/cluster/cluster.py:91-121
 *   norm_state_dict (obs vector)   server/app/utils/norm.py:178-218
 *   controllers                    server/app/core/agents/controllers/bangbang_controllers.py:25-89,
 *                                  server/app/core/agents/controllers/greedy_myopic_controller.py:67-104
 *   Environment.reset / noise      server/app/core/environment/environment.py:49-70,161-194
 *   PowerInterpolator (base power) server/app/core/environment/power_grid/interpolation.py:186-264
 *
 * The reference has no FFI: its boundary is a Python object (Environment.reset/step).  The
 * Python layer mdr_amd.Environment keeps that object surface and binds these symbols with ctypes
 * (INTEGRATION.md shows the binding).  Per-tick scalar drivers (outdoor temperature, solar gain,
 * regulation signal, datetime) stay on the host in the reference's own arithmetic and RNG order
 * and are passed in as mdr_tick; everything per house runs on the GPU.
 *
 * Conventions
 *   - All device pointers are caller-owned (PyTorch tensors in mdr_amd); the library owns only
 *     small scratch (per-tick power counts, penalty partials, graph cache).
 *   - Every call is asynchronous on the caller's hipStream_t (passed as void*; NULL = legacy
 *     default stream) and returns 0 on success, a negative MDR_E* code otherwise;
 *     mdr_last_error() gives the text (thread-local).
 *   - A context maps to ONE device and ONE contiguous shard of houses [global_offset,
 *     global_offset + n_local) of a cluster of n_global houses; it is not thread-safe.
 *
 * Per-house state layout (SoA, length n_local):
 *   t_air, t_mass : double   indoor air / mass temperature (Celsius)
 *   hvac          : uint32   bits 0..29 seconds_since_off (saturating), bit 30 lockout, bit 31 on
 *   ua, ca, cm, hm, target : double  (noised per-house parameters)
 *   cap_idx       : uint8    index into the cooling-capacity table (mdr_config.cap_table)
 */
#ifndef MDR_H_
#define MDR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDR_ABI_VERSION 5
#define MDR_MAX_CAP 64

enum {
  MDR_OK = 0,
  MDR_EARG = -1,   /* bad argument / shape / unbound context */
  MDR_EHIP = -2,   /* HIP runtime error */
  MDR_ERCCL = -3,  /* RCCL error */
  MDR_ENOMEM = -4,
  MDR_ESTATE = -5, /* call out of order (e.g. step before bind) */
};

/* penalty modes, rewards_calculator.py:46-133 */
enum { MDR_PEN_INDIVIDUAL_L2 = 0, MDR_PEN_COMMON_L2 = 1, MDR_PEN_COMMON_MAX = 2, MDR_PEN_MIXTURE = 3 };

/* where a tick's actions come from */
enum {
  MDR_ACT_BUFFER = 0,     /* uint8 action[n_local] (non-zero = turn on), the Dict[int,bool] of step() */
  MDR_ACT_RANDOM = 1,     /* Bernoulli(0.5) from Philox4x32-10(seed, global house id, tick) */
  MDR_ACT_ALWAYS_ON = 2,  /* AlwaysOnController, bangbang_controllers.py:7-16 */
  MDR_ACT_BANGBANG = 16,  /* BangBangController on the pre-step state, bangbang_controllers.py:54-65 */
  MDR_ACT_DEADBAND_BANGBANG = 17 /* DeadbandBangBangController, bangbang_controllers.py:25-42 */
};

/* controller evaluated on the post-step state, written as the NEXT tick's action buffer
 * (MDR_CTRL_GREEDY_KEYS: no action buffer — the greedy controller's keys and key histogram of the
 * post-step state are prepared for the next mdr_ctrl_greedy, which then skips its key pass) */
enum { MDR_CTRL_NONE = 0, MDR_CTRL_BANGBANG = 1, MDR_CTRL_DEADBAND_BANGBANG = 2, MDR_CTRL_GREEDY_KEYS = 3 };

/* communication (message) topology, agent_communication_builder.py:36-203 */
enum { MDR_COMM_RING = 0, MDR_COMM_TABLE = 1 };

typedef struct mdr_config {
  int32_t abi_version;      /* = MDR_ABI_VERSION */
  int32_t device;           /* HIP device ordinal */
  int64_t n_local;          /* houses in this shard */
  int64_t global_offset;    /* global id of the shard's first house */
  int64_t n_global;         /* cluster size N (signal penalty, obs normalisation) */
  int32_t dt;               /* time_step.seconds */
  int32_t lockout_duration; /* L (hvac_prop.lockout_duration) */
  double cop;               /* hvac_prop.cop */
  double lcf;               /* hvac_prop.latent_cooling_fraction */
  double deadband;          /* house_prop.deadband */
  int32_t n_cap;            /* entries in cap_table (<= MDR_MAX_CAP) */
  int32_t penalty_mode;     /* MDR_PEN_* */
  double cap_table[MDR_MAX_CAP]; /* cooling capacities (W) the population draws from */
  double alpha_temp, alpha_sig;  /* reward_prop */
  double norm_temp, norm_sig;    /* deadbandL2 normalisers, computed by the caller */
  double alpha_ind_l2, alpha_common_l2, alpha_common_max;
  uint64_t seed;                 /* Philox key for MDR_ACT_RANDOM and synthetic populations */
} mdr_config;

typedef struct mdr_soa {
  double* t_air;
  double* t_mass;
  uint32_t* hvac;
  const double* ua;
  const double* ca;
  const double* cm;
  const double* hm;
  const double* target;
  const uint8_t* cap_idx;
} mdr_soa;

/* host-side per-tick drivers (environment.py:86-106 ordering) */
typedef struct mdr_tick {
  double t_od_prev; /* outdoor temperature BEFORE this step (used by the thermal update) */
  double solar;     /* compute_solar_gain at the NEW datetime, 0 if house_prop.solar_gain is off */
  double s_prev;    /* regulation signal before this step (the reward uses the old signal) */
  uint64_t tick;    /* tick counter (Philox stream for MDR_ACT_RANDOM) */
} mdr_tick;

typedef struct mdr_ctx mdr_ctx;

/* ---- lifecycle ------------------------------------------------------------------------- */
int mdr_abi_version(void);
/* "MDR_SRC_HASH:<16 hex>": sha256 of the sources and build flags the library was built from
 * (build_ext.py src_hash); the Python binding refuses a library whose hash differs from its tree's. */
const char* mdr_build_id(void);
/* sizeof of the ABI structs, for binding checks: out[0..8] = mdr_config, mdr_soa, mdr_tick,
 * mdr_pop_spec, mdr_obs_spec, mdr_obs_scalars, mdr_actor_spec, mdr_interp_spec, mdr_actor_net;
 * returns the number written */
int mdr_abi_sizes(int64_t* out, int n);
const char* mdr_last_error(void);
/* Graph cache diagnostics: out[0..5] = cached rollout graphs, cached actor-rollout graphs,
 * hipGraphLaunch calls of mdr_rollout, of mdr_actor_rollout, captured graphs the memset guard
 * walked (every capture fails with MDR_EHIP on a memset node), their nodes; returns the number
 * written. */
int mdr_graph_info(mdr_ctx* ctx, int64_t* out, int n);
/* Diagnostic (synchronises, overwrites the count slabs): captures hipMemsetAsync of the count slabs
 * to zero in this context and reports out[13] = {nodes, memset nodes, dst == the slabs, value,
 * elementSize, width, height, pitch, bytes passed, non-zero 64-bit words after replays 1..3 (slabs
 * pre-filled with 0xA5 before replays 1 and 2), non-zero words after the kernel zeroing}. */
int mdr_graph_memset_probe(mdr_ctx* ctx, int64_t* out, int n, void* stream);
int mdr_create(mdr_ctx** out, const mdr_config* cfg);
int mdr_destroy(mdr_ctx* ctx);
/* Bind the caller-owned SoA arrays (Environment.reset, environment.py:49-70). */
int mdr_bind(mdr_ctx* ctx, const mdr_soa* soa);

/* The caller rewrote ua/ca/cm/hm (or dt changed): the per-house flag that routes a house outside
 * the exact shared-reciprocal division range to the IEEE operator is recomputed before the next
 * step.  mdr_bind and mdr_populate imply it. */
int mdr_params_changed(mdr_ctx* ctx);

/* ---- options (no reference counterpart) ------------------------------------------------ */
/* Alternative launch forms of the same computation, for verification and measurement; every
 * option has a test that pins it against the default.  Drops cached rollout graphs.
 *   MDR_OPT_STEP_TPW        per-tick step kernel: 1/2/4/8 = k_step_pipe tiles per wave, 0 = the
 *                           one-tile k_step_t, -1 = the measured default (2 up to 1.5M houses, 4)
 *   MDR_OPT_FASTDIV         1 = shared-reciprocal exact division (default), 0 = the IEEE operator
 *                           everywhere (bit-identical results)
 *   MDR_OPT_WINDOW_PIPELINE sharded window rollouts: 1 = count + allreduce on a side stream up to
 *                           two windows ahead (default), 0 = one stream
 *   MDR_OPT_SHARDED_OVERLAP sharded one-tick rollouts: 1 = allreduce of tick t beside the step of
 *                           tick t, rewards written one launch later (default), 0 = serial
 *   MDR_OPT_GREEDY_SORT     1 = mdr_ctrl_greedy always runs the full-sort form
 *   MDR_OPT_FORCE_HALO      1 = mdr_actor_rollout_sharded exchanges the ring halo even at world 1
 *                           (send/recv to self: the one-GPU check of the multi-GPU exchange)
 *   MDR_OPT_HALO_OVERLAP    mdr_actor_rollout_sharded: 1 (default) = each tick's ring halo is packed and
 *                           exchanged on the communicator's side stream while the interior tiles'
 *                           k_actor runs, then the first and last tile; 0 = halo, then one k_actor
 *   MDR_OPT_HALO_IN_COUNTS  mdr_actor_rollout_sharded: 1 (default) = ONE collective per tick: the edge
 *                           houses' post-step message rows (the next tick's ring halo) are computed
 *                           before the step and summed into the count allreduce; 0 = a ring-halo
 *                           send/recv per tick plus the count allreduce (MDR_OPT_HALO_OVERLAP applies)
 *   MDR_OPT_GQ_BAND         mdr_ctrl_greedy: 1 (default) = k_gq_binsc cuts the window from the step
 *                           epilogue's predicted band when it holds the crossing (no bins pass) and
 *                           k_gq_finish ranks and decides; 0 = the bins pass every call (k_gq_bins,
 *                           k_gq_compact, k_gq_select: faster when the budget jumps across the cluster
 *                           every call)
 *   MDR_OPT_GQ_FUSED        mdr_greedy_rollout: 1 = the fused tick, one decision launch per tick
 *                           (k_gq_decide2: the previous step's epilogue counted the keys and the band's
 *                           houses, the step applies the decision from the pre-step keys); 0 (default)
 *                           = the mdr_ctrl_greedy + mdr_step tick (bit-identical; faster at 1M houses,
 *                           DESIGN.md §3.3)
 *   MDR_OPT_GQ_ADAPTIVE     mdr_greedy_rollout with the band form: 1 (default) = a tick whose budget change departs
 *                           from the previous change by more than four superbins' worth of power runs the
 *                           three-launch form (a band miss costs more); 0 = the band form on every tick
 *   MDR_OPT_ACTOR_GENERIC   1 = k_actor runs its generic form for the reference's default obs layout too
 *                           (0, default: that layout runs the form specialised for it, mdr_actor.hip DEF)
 *   MDR_OPT_ACTOR_FP32_FORM the fused actor's MDR_PREC_FP32 arithmetic: MDR_FP32_F16_SPLIT (default) =
 *                           fp16 hi/lo operands on the fp16 MFMA, 3 products per term, power-of-two
 *                           per-layer weight scales (activations must stay inside fp16's range:
 *                           mdr_actor_status counts the tiles that did not); MDR_FP32_BF16_SPLIT3 =
 *                           three-way bf16 operands, 6 products per term, no range limit
 *   MDR_OPT_WINDOW_THERMAL  k_step_window's per-tick thermal update: MDR_THERMAL_AFFINE (default)
 *                           = the reference's update as a per-house affine transition formed once
 *                           per window (4 FMAs per temperature per tick; ~1e-13 K per tick from the
 *                           reference order), MDR_THERMAL_EXACT = the reference's expression in its
 *                           operation order every tick (bit-identical to the one-tick kernels) */
enum { MDR_OPT_STEP_TPW = 1, MDR_OPT_FASTDIV = 2, MDR_OPT_WINDOW_PIPELINE = 3, MDR_OPT_SHARDED_OVERLAP = 4,
       MDR_OPT_GREEDY_SORT = 5, MDR_OPT_FORCE_HALO = 6, MDR_OPT_WINDOW_THERMAL = 7,
       MDR_OPT_HALO_OVERLAP = 9, MDR_OPT_ACTOR_GENERIC = 10, MDR_OPT_HALO_IN_COUNTS = 12,
       MDR_OPT_GQ_BAND = 13, MDR_OPT_ACTOR_FP32_FORM = 14, MDR_OPT_GQ_FUSED = 15, MDR_OPT_GQ_ADAPTIVE = 16 };
enum { MDR_FP32_F16_SPLIT = 0, MDR_FP32_BF16_SPLIT3 = 1 };
/* (8 was MDR_OPT_ACTOR_PINGPONG, a k_actor schedule measured slower and retired in r04: rejected) */
enum { MDR_THERMAL_EXACT = 0, MDR_THERMAL_AFFINE = 1 };
int mdr_set_option(mdr_ctx* ctx, int option, int64_t value);

/* ---- launch geometry (no reference counterpart) ---------------------------------------- */
/* Bytes of the window ON-mask rows ([tiles][HPT][32] u64) that a window launch over n_local houses
 * with `waves` waves per block touches (every wave of a ragged last block stores and loads the rows
 * of its tile): the count launches use the build's kCountWaves, the step launches 4. */
size_t mdr_window_onb_bytes(int64_t n_local, int waves);
/* MDR_OK when ON-mask rows of onb_bytes and end words of wah_bytes cover every count and step
 * window launch over n_local houses; MDR_EARG otherwise.  Every k_count_window / k_step_window
 * launch checks its context's buffers with it, so a new launch geometry cannot overrun them. */
int mdr_window_geometry_check(int64_t n_local, size_t onb_bytes, size_t wah_bytes);

/* ---- population ------------------------------------------------------------------------ */
/* Synthetic population drawn on device from Philox4x32-10(seed, global house id): the reference
 * noise model (building.py:224-267, hvac.py:66-70: target = target_temp + |N(0, std_target)|,
 * Ua = Tri(lo, hi, 1) (the reference ASSIGNS the factor), Cm/Ca/Hm = cfg * Tri(lo, hi, 1), cap =
 * a uniform entry of cooling_capacity_list) with a counter-based RNG instead of MT19937, so a population is
 * identical for any sharding.  Initial state as Building.reset/HVAC.reset: T = init temps, on,
 * no lockout, sso = 0.  Writes every bound array. */
typedef struct mdr_pop_spec {
  double target_temp, std_target;   /* house_prop.target_temp, noise_prop.std_target_temp */
  double thermo_lo, thermo_hi;      /* noise_prop.factor_thermo_low / _high */
  double ca, cm, hm;                /* house_prop.Ca, Cm, Hm */
  double init_air, init_mass;       /* house_prop.init_air_temp, init_mass_temp */
  int32_t n_draw;                   /* cap drawn uniformly over n_draw list entries (random.choices
                                       of noise_prop.cooling_capacity_list, hvac.py:68-70);
                                       0 = uniform over the whole cap_table */
  uint8_t draw_idx[MDR_MAX_CAP];    /* cap_table index of each list entry */
} mdr_pop_spec;
int mdr_populate(mdr_ctx* ctx, const mdr_pop_spec* spec, void* stream);

/* ---- tick: phase 1 (cluster power) ------------------------------------------------------ */
/* Lockout FSM on the current state + this tick's actions -> ON houses per capacity class,
 * accumulated into the context's count slab for this tick (int64[kCountShards * n_cap], sharded
 * to spread atomics).  P = sum_k count_k * cap_k / cop is exact and order independent.  State
 * is not modified.  (cluster.py:82-88)  Not needed when the previous mdr_step ran with a
 * lookahead action source. */
int mdr_power_counts(mdr_ctx* ctx, const uint8_t* action, int action_mode, uint64_t tick,
                     void* stream);
/* Device pointer + element count of the current tick's count slab: the buffer a multi-GPU caller
 * sum-allreduces (int64) between phase 1 and phase 2. */
int mdr_counts_buffer(mdr_ctx* ctx, int64_t** dev_ptr, int* len);

/* ---- tick: phase 2 (fused step) -------------------------------------------------------- */
/* FSM + RC thermal update + per-house reward with this tick's GLOBAL cluster power; updates the
 * state in place and writes reward[n_local] (double).
 *   action_mode : MDR_ACT_* (BUFFER reads action[]), or MDR_ACT_BANGBANG / _DEADBAND_BANGBANG to
 *                 evaluate that controller on the pre-step state (the obs the caller would act on)
 *   lookahead   : 0, or the action source of the NEXT tick (MDR_ACT_RANDOM / _ALWAYS_ON /
 *                 _BANGBANG / _DEADBAND_BANGBANG): its ON counts are accumulated here on the new
 *                 state, so the next tick needs no phase-1 launch
 *   ctrl_out    : if non-NULL, the bang-bang (ctrl = MDR_CTRL_*) decision on the new state
 *   p_out       : if non-NULL, device double receiving the tick's cluster power
 *   ctrl = MDR_CTRL_GREEDY_KEYS: the next mdr_ctrl_greedy's keys (see MDR_CTRL_*)
 * For common penalty modes reward holds the raw penalty until mdr_reward_finalize. */
int mdr_step(mdr_ctx* ctx, const uint8_t* action, int action_mode, const mdr_tick* tick,
             double* reward, int lookahead, int ctrl, uint8_t* ctrl_out, double* p_out,
             void* stream);

/* Common penalty modes (common_L2 / common_max_error / mixture): per-shard {sum pen/N, max pen}
 * into the context's partial buffer (device double[2]; sum-/max-allreduce it on multi-GPU), then
 * the rewards are finalised in place. */
int mdr_penalty_partials(mdr_ctx* ctx, void* stream);
int mdr_penalty_buffer(mdr_ctx* ctx, double** dev_ptr);
int mdr_reward_finalize(mdr_ctx* ctx, const mdr_tick* tick, double* reward, void* stream);

/* ---- several ticks in one call (single GPU) --------------------------------------------- */
/* n_ticks consecutive steps; ticks[] in host memory.  action / reward advance by act_stride /
 * rew_stride elements per tick (0 = reuse one buffer).  With an in-kernel action source
 * (MDR_ACT_RANDOM / _ALWAYS_ON / _BANGBANG / _DEADBAND_BANGBANG) every tick is ONE launch (the
 * counts of tick t+1 come from tick t's lookahead); with MDR_ACT_BUFFER two.  use_graph != 0
 * captures the sequence in a hipGraph (cached per shape) and replays it.  p_out (device scalar,
 * may be NULL) receives the cluster power of the LAST tick, as mdr_step's p_out. */
int mdr_rollout(mdr_ctx* ctx, int n_ticks, const mdr_tick* ticks, const uint8_t* action,
                int64_t act_stride, int action_mode, double* reward, int64_t rew_stride,
                double* p_out, int use_graph, void* stream);

/* Open-loop sources (MDR_ACT_RANDOM / _ALWAYS_ON / _BUFFER) with individual_L2 and <= 4 capacity
 * classes run TEMPORALLY BLOCKED: windows of up to `ticks` steps per launch (k_step_window), the
 * state and parameters read and written once per window, rewards written every tick, each tick's
 * cluster power from counts the previous launch ran ahead (the FSM of an open-loop source does
 * not depend on the thermal state).  Bit-identical to the one-tick path.  ticks in 1..32
 * (default 32), 0 = one launch per tick.  Applies to mdr_rollout and
 * mdr_rollout_sharded; drops cached rollout graphs. */
int mdr_set_rollout_window(mdr_ctx* ctx, int ticks);

/* Optional, before mdr_rollout (no reference counterpart): launch the first window's lockout-FSM
 * count of an n_ticks rollout whose first tick id is tick0, and that window's cluster power — they
 * need the tick ids only, so they run while the host computes the ticks' drivers.  The next
 * mdr_rollout with the same n_ticks, action source, action buffer and first tick id (and
 * consecutive tick ids) uses them and launches the first window's step kernel with the drivers as
 * kernel arguments; any other entry point called in between discards them.  A no-op for rollouts
 * that do not take the temporally blocked path.  On a context with an RCCL communicator it also
 * allreduces the counts (single-window rollouts; the match is mdr_rollout_sharded). */
int mdr_rollout_begin(mdr_ctx* ctx, int n_ticks, uint64_t tick0, const uint8_t* action, int64_t act_stride,
                      int action_mode, void* stream);

/* Measurement (no reference counterpart): mdr_rollout's launch sequence issued directly (no graph)
 * with an event pair around every step-kernel launch; *ms = the summed step-kernel time,
 * *launches = step launches (windows, or ticks on the one-tick path).  Advances the state like
 * mdr_rollout; synchronises the stream. */
int mdr_time_step_kernels(mdr_ctx* ctx, int n_ticks, const mdr_tick* ticks, const uint8_t* action,
                          int64_t act_stride, int action_mode, double* reward, int64_t rew_stride,
                          void* stream, float* ms, int* launches);

/* ---- observation vector (norm_state_dict, norm.py:178-218) ----------------------------- */
typedef struct mdr_obs_spec {
  int32_t n_feat;        /* features per house written (row length of obs) */
  int32_t hvac_state;    /* state_prop.hvac */
  int32_t solar_state;   /* state_prop.solar_gain */
  int32_t thermal_state; /* state_prop.thermal */
  int32_t msg_thermal;   /* message_prop.thermal */
  int32_t msg_hvac;      /* message_prop.hvac */
  int32_t n_comm;        /* messages per house (nb_comm) */
  int32_t comm_mode;     /* MDR_COMM_RING (neighbours, arithmetic) or MDR_COMM_TABLE */
  const int32_t* comm_table; /* TABLE mode: [n_local, n_comm] local house indices */
  const float* halo_msg;     /* RING mode, multi-GPU: [lo + hi][msg_w] message features of the
                                houses before / after the shard (mdr_halo_pack of the neighbours);
                                NULL = single shard, ring wraps around locally */
  double norm_reg_sig;   /* R */
  double cfg_ua, cfg_ca, cfg_cm, cfg_hm; /* house_prop (un-noised) for the thermal ratios */
  double cfg_cap;        /* hvac_prop.cooling_capacity (message hvac feature) */
  const float* msg_all;  /* TABLE mode, multi-GPU: [n_global][msg_w] message features of every house
                            (mdr_msg_pack of each shard, all-gathered); comm_table then holds GLOBAL
                            house ids; NULL = single shard (table ids are local) */
} mdr_obs_spec;

typedef struct mdr_obs_scalars {
  double p;       /* cluster power of the tick (obs cluster_hvac_power) */
  double s;       /* regulation signal after the step (obs reg_signal) */
  double solar;   /* obs solar_gain */
  double t_od;    /* obs OD_temp */
} mdr_obs_scalars;

/* message feature width for a spec (4, +4 thermal, +3 hvac) */
int mdr_msg_width(const mdr_obs_spec* spec);
/* float32 obs[n_local, n_feat].  p_dev, when non-NULL, overrides sc->p with a device scalar
 * (the value mdr_step wrote), so no host round trip is needed. */
int mdr_obs(mdr_ctx* ctx, const mdr_obs_spec* spec, const mdr_obs_scalars* sc,
            const double* p_dev, float* obs, void* stream);
/* message features of this shard's first hi and last lo houses -> out[(hi + lo) * msg_w] floats:
 * rows [0, hi) = first hi houses, rows [hi, hi + lo) = last lo houses. */
/* Message features (Building.message, building.py:79-139) of every local house: out [n_local][msg_w]
 * (sharded table comm modes all-gather these into mdr_obs_spec.msg_all). */
int mdr_msg_pack(mdr_ctx* ctx, const mdr_obs_spec* spec, float* out, void* stream);

int mdr_halo_pack(mdr_ctx* ctx, const mdr_obs_spec* spec, float* out, void* stream);

/* ---- cluster statistics for the server's Metrics / UI summary ----------- */
/* One deterministic reduction over the shard's state (+ reward, may be NULL) into out[12] (device
 * doubles): sum(T - target/N), sum|T - target/N|, max(0, max(T - target/N)), sum (T - target/N)^2,
 * sum reward/N (Metrics.update, metrics_service.py:108-157, its operator precedence kept),
 * sum T, sum (T - target), sum |T - target|, sum T_mass, sum target, #lockout, #on
 * (ClientManagerService, client_manager_service.py:62-111,177-196).  Sharded: sum-allreduce all but
 * out[2] (max-allreduce). */
int mdr_cluster_stats(mdr_ctx* ctx, const double* reward, double* out, void* stream);

/* ---- greedy-myopic controller (greedy_myopic_controller.py:67-104) --------------------- */
/* Next actions for the whole shard (single GPU: shard = cluster) from the current state: order
 * by -(T - target) ascending, then the reference's sequential take rule with budget S.  Also fills
 * the current tick's cluster-power counts with the ON houses those actions produce, so the next
 * mdr_step(action, MDR_ACT_BUFFER) needs no mdr_power_counts.  Asynchronous (no host
 * synchronisation): histogram select on device — only the houses around the budget crossing are
 * ordered; what that window cannot decide (a crossing among NaN keys or inside a bin of > 4,096
 * houses, e.g. identical keys; a walk past the window) the last kernel decides exactly itself.
 * With more than 4 capacity classes (or MDR_OPT_GREEDY_SORT) the full-sort form runs. */
int mdr_ctrl_greedy(mdr_ctx* ctx, double budget, uint8_t* action, void* stream);
/* Diagnostics (synchronises): mdr_ctrl_greedy calls decided by the exact in-kernel fallback;
 * mdr_greedy_diag: out[4] = {fallbacks, histogram-select calls, sum of their candidate-window
 * sizes, the last call's window size}. */
int mdr_greedy_fallbacks(mdr_ctx* ctx, uint64_t* count);
int mdr_greedy_diag(mdr_ctx* ctx, uint64_t* out);
/* The select state after the last stage run (synchronises): out[12] = mdr_greedy_diag's 4 values,
 * then {crossing superbin, crossing bin b*, window end bin, all taken, overflow, houses after the
 * window, window allocator count (zero again once the select has run), sharded need-fallback flag}. */
int mdr_greedy_state(mdr_ctx* ctx, uint64_t* out);
/* Config C3's loop: n ticks of {mdr_ctrl_greedy with budget ticks[t].s_prev (the
 * signal before the tick's step, the one the observation carries) into action + t * act_stride,
 * then mdr_step of those actions with MDR_CTRL_GREEDY_KEYS (reward + t * rew_stride; common
 * penalty modes: + mdr_penalty_partials / mdr_reward_finalize)}; strides 0 = every tick overwrites.
 * Replaces the per-tick Python loop GreedyMyopic.get_action -> Environment.step
 * (greedy_myopic_controller.py:67-104, environment.py:86-106).  Single GPU only: a sharded context
 * (world > 1) returns MDR_ESTATE (its decision needs the caller's collectives: mdr_gq_shard_*). */
int mdr_greedy_rollout(mdr_ctx* ctx, int n, const mdr_tick* ticks, uint8_t* action, int64_t act_stride,
                       double* reward, int64_t rew_stride, double* p_out, void* stream);
/* The predicted band (synchronises): out[4] = {mdr_ctrl_greedy calls that skipped the bins pass
 * (the step epilogue's band held the crossing, or no bins were needed), histogram-select calls,
 * the first superbin of the band the next GQ step counts, the band's width in superbins}.
 * Misses = calls - skips. */
int mdr_greedy_band(mdr_ctx* ctx, uint64_t* out);
/* The fused tick's counters (synchronises): out[6] = {decisions, band hits, misses (the decision's own
 * pass over the cluster), exact decisions (gq_exact), the last decision's mode (0 window, 1 all taken,
 * 2 every house's byte), the last window's houses}. */
int mdr_greedy_fused_diag(mdr_ctx* ctx, uint64_t* out);
/* Diagnostics: on != 0 makes the following fused decisions record each block's phase clocks (the
 * 100 MHz constant clock; [kGqSelBlocks = 256][16] words, slot 10 = 1 in the deciding block); out, when
 * non-NULL, receives the current record (synchronises); on = 0 stops. */
int mdr_greedy_fused_stamps(mdr_ctx* ctx, int on, uint64_t* out);

/* Sharded greedy, histogram form (per-rank work O(N/G + window)): the same
 * select as mdr_ctrl_greedy with the caller's collectives between its stages, every rank deciding
 * the same window:
 *   mdr_gq_shard_begin      this shard's key codes, superbin histogram and (min, -max) key range
 *   [caller] sum-allreduce the superbin histogram (uint32, n_super) and min-allreduce the range (2 f64)
 *   mdr_gq_shard_bins       the crossing superbin, the next key map; this shard's bin counts
 *   [caller] sum-allreduce the bin histogram (uint32, n_bin)
 *   mdr_gq_shard_compact    this shard's actions below the crossing bin and its window houses:
 *                           window = {count, 0, 0, 0} + count 16-B entries (window_bytes in all)
 *   [caller] all-gather the ranks' windows (window_bytes each) in rank order
 *   mdr_gq_shard_select     order the gathered window, decide it, write this shard's window actions
 *   mdr_gq_shard_fallback   (synchronises) 1 = the window could not decide this call (a crossing
 *                           among NaN keys or inside one bin of > 4,096 houses, a walk past the
 *                           window): decide it with the all-gather form below instead.
 * mdr_gq_shard_buffers exposes the device buffers the collectives work on (valid after begin). */
int mdr_gq_shard_begin(mdr_ctx* ctx, void* stream);
int mdr_gq_shard_buffers(mdr_ctx* ctx, void** super_hist, int64_t* n_super, void** bin_hist, int64_t* n_bin,
                         void** range, void** window, int64_t* window_bytes);
int mdr_gq_shard_bins(mdr_ctx* ctx, double budget, void* stream);
int mdr_gq_shard_compact(mdr_ctx* ctx, double budget, uint8_t* action, void* stream);
int mdr_gq_shard_select(mdr_ctx* ctx, double budget, const void* gathered, int world, uint8_t* action, void* stream);
int mdr_gq_shard_fallback(mdr_ctx* ctx, int* need, void* stream);

/* Sharded greedy (the all-gather form): mdr_greedy_inputs writes this shard's
 * rows key = -(T - target), P = cooling capacity / cop, lockout (u8); the caller all-gathers them
 * in global house order, and every rank runs mdr_greedy_select over the n gathered rows — the same
 * sort / sequential take rule as mdr_ctrl_greedy — writing the cluster's actions (u8 [n]), of
 * which it keeps its own slice. */
int mdr_greedy_inputs(mdr_ctx* ctx, double* key, double* power, uint8_t* lock, void* stream);
int mdr_greedy_select(mdr_ctx* ctx, int64_t n, const double* key, const double* power, const uint8_t* lock,
                      double budget, uint8_t* action, void* stream);

/* ---- MA-PPO actor fused with the observation ----------------- */
/* Replaces MAPPO.select_actions (server/app/core/agents/trainables/mappo.py:83-97) over
 * norm_state_dict vectors (server/app/utils/norm.py:178-218) with Actor.forward
 * (server/app/core/agents/trainables/network.py:29-33; actor_layers = [h1, h2], default [100, 100],
 * server/app/core/agents/trainables/ppo.py:23-26): one persistent launch builds every house's obs
 * row on chip, runs both hidden layers on MFMA, softmax + Categorical sampling in fp32. */
enum { MDR_PREC_BF16 = 1,   /* bf16 products, fp32 accumulate (~4e-3 relative) */
       MDR_PREC_BF16X3 = 3, /* split-bf16 (hi*hi + hi*lo + lo*hi), fp32 accumulate (~1e-5) */
       MDR_PREC_FP32 = 6    /* fp32-faithful (~1e-7), the reference Actor's precision: fp16 hi/lo split
                               (22 significand bits, 3 products on the fp16 MFMA) or, with
                               MDR_OPT_ACTOR_FP32_FORM, three-way split-bf16 (24 bits, 6 products);
                               fp32 accumulate.  The layer chain runs the three-way split. */ };

typedef struct mdr_actor_spec {
  int32_t n_in;      /* obs features (= mdr_obs_spec.n_feat) */
  int32_t h1, h2;    /* hidden widths (actor_layers) */
  int32_t n_act;     /* actions (num_action): 2, the on/off decision */
  int32_t precision; /* MDR_PREC_* */
} mdr_actor_spec;

/* Load (or replace, after a PPO update) the actor weights.  Device fp32 tensors in nn.Linear
 * layout: w1 [h1][n_in], b1 [h1], w2 [h2][h1], b2 [h2], w3 [n_act][h2], b3 [n_act] (the
 * reference Actor's fc.0 / fc.1 / fc.2).  They are packed into MFMA fragment order on `stream`. */
int mdr_actor_load(mdr_ctx* ctx, const mdr_actor_spec* spec, const float* w1, const float* b1,
                   const float* w2, const float* b2, const float* w3, const float* b3, void* stream);
/* The general actor: any number of hidden layers (actor_layers, network.py:14-33) of any widths,
 * over any obs row.  w[l] / b[l], l = 0 .. n_hidden: device fp32 nn.Linear weights [out][in] and
 * biases of fc.l (the last one the output layer, [n_act][hidden[n_hidden-1]]).  A net of two
 * hidden layers <= 128 wide whose obs row (<= 128 feature slots) and weight planes fit a CU's LDS
 * runs the fused k_actor; any other runs the chain k_obs -> k_dense per hidden layer ->
 * k_actor_head (the same precisions and sampling stream). */
#define MDR_ACTOR_MAX_LAYERS 8
typedef struct mdr_actor_net {
  int32_t n_in, n_hidden, n_act, precision;
  int32_t hidden[MDR_ACTOR_MAX_LAYERS];
} mdr_actor_net;
int mdr_actor_load_net(mdr_ctx* ctx, const mdr_actor_net* net, const float* const* w, const float* const* b,
                       void* stream);
/* Synchronises; counts since the last call (zeroed by it).  out[0] = 32-house tiles of the fused
 * fp16-split form (MDR_PREC_FP32, MDR_FP32_F16_SPLIT) that met a non-finite logit, out[1] = the fused
 * kernel's arithmetic (1 bf16, 3 bf16x3, 4 the fp16 split, 6 the three-way bf16 split; 0 without an
 * actor), out[2] = tiles of the fp16 split whose values left fp16's range (a hidden activation >= 2^15
 * x the layer's weight scale, or an sso ratio >= 2^15 in the tile's rows) and whose logits were
 * computed in scalar fp32 instead. */
int mdr_actor_status(mdr_ctx* ctx, int64_t* out, int n, void* stream);  /* out[3] */
/* 1 when the loaded actor runs the fused kernel for this obs layout, 0 when it runs the chain. */
int mdr_actor_fused(mdr_ctx* ctx, const mdr_obs_spec* obs);
/* One select_actions over the shard.  Outputs (device, any may be NULL): action u8 [n_local],
 * prob f32 [n_local] (probability of the sampled action, MAPPO.last_probs), probs f32
 * [n_local][n_act], obs_out f32 [n_local][n_in].  Sampling: Philox4x32-10(seed, global house id,
 * tick).  count_next != 0 also fills the cluster-power counts the sampled actions produce, so the
 * next mdr_step(MDR_ACT_BUFFER) needs no mdr_power_counts. */
int mdr_actor_act(mdr_ctx* ctx, const mdr_obs_spec* obs, const mdr_obs_scalars* sc, const double* p_dev,
                  uint64_t tick, uint8_t* action, float* prob, float* probs, float* obs_out,
                  int count_next, void* stream);
/* n_ticks of (select_actions -> env.step) on device, hipGraph-captured when use_graph:
 *   tick t: actor on the state after tick t-1 (obs scalars obs_sc[t]: p ignored — the cluster
 *   power comes from p_dev, which each step rewrites), then the step with those actions.
 * action [n_ticks][n_local] u8 / prob [n_ticks][n_local] f32 (stride 0 = overwrite one row) and
 * reward [n_ticks][n_local] f64 (rew_stride 0 = one row).  p_dev: device double, in/out. */
int mdr_actor_rollout(mdr_ctx* ctx, int n_ticks, const mdr_tick* ticks, const mdr_obs_scalars* obs_sc,
                      const mdr_obs_spec* obs, uint8_t* action, int64_t act_stride, float* prob,
                      int64_t prob_stride, double* reward, int64_t rew_stride, double* p_dev,
                      int use_graph, void* stream);

/* mdr_actor_rollout over a house-sharded cluster (config C5 on N GPUs, RCCL communicator of
 * mdr_rccl_init), no graph: per tick the 'neighbours' ring obs gets the edge houses' message
 * features of ranks r-1 / r+1 (mdr_halo_pack + grouped ncclSend/ncclRecv), then the actor, a
 * sum-allreduce of the ON counts its actions produce, then the step.  obs->halo_msg is ignored
 * (the context owns the halo buffer); TABLE comm modes are single-shard only.  Bit-identical to
 * the single-shard rollout. */
int mdr_actor_rollout_sharded(mdr_ctx* ctx, int n_ticks, const mdr_tick* ticks, const mdr_obs_scalars* obs_sc,
                              const mdr_obs_spec* obs, uint8_t* action, int64_t act_stride, float* prob,
                              int64_t prob_stride, double* reward, int64_t rew_stride, double* p_dev,
                              void* stream);

/* ---- interpolated base power ---------------------------------------- */
/* Replaces PowerInterpolator (server/app/core/environment/power_grid/interpolation.py:24-264) as
 * PowerGrid.power_step calls it every interp_update_period seconds (power_grid.py:149-161): the
 * host draws the sampled house ids (random.choices, interpolation.py:218-224 — the reference's RNG
 * stream) and the per-tick scalars; the per-house clip / nearest / multilinear lookup over the
 * Monte-Carlo table (interpolate_grid_fast, :137-178) reads the device state directly.
 * Axes in interp_dict_keys.csv order: Ua_ratio, Cm_ratio, Ca_ratio, Hm_ratio (nearest), air_temp,
 * mass_temp, OD_temp (linear), HVAC_power (nearest), hour, date (linear). */
#define MDR_INTERP_AXES 10
typedef struct mdr_interp_spec {
  int32_t len[MDR_INTERP_AXES]; /* grid points per axis (linear axes: >= 2, strictly ascending) */
  const double* grid;           /* host: the axis values, concatenated in axis order */
  const double* values;         /* host: the table, prod(len) doubles, C order over the axes */
  double cfg_ua, cfg_cm, cfg_ca, cfg_hm; /* house_prop Ua, Cm, Ca, Hm (the ratio denominators) */
} mdr_interp_spec;
/* Copy the grid + table to the device (synchronous); replaces a previous table. */
int mdr_interp_load(mdr_ctx* ctx, const mdr_interp_spec* spec);
/* vals[s] (device double[n]) = the interpolated power of house ids[s] (device int64 global ids)
 * at outdoor temperature od_temp and the point's hour / date (interpolation.py:204-216); houses
 * outside this shard give +0.0, so a sum-allreduce of vals assembles the cluster's values. */
int mdr_interp_values(mdr_ctx* ctx, const int64_t* ids, int n, double od_temp, double hour, double date,
                      double* vals, void* stream);
/* out[0] (device) = (sum of vals[0..n) in order) * multi_factor — the base power. */
int mdr_interp_sum(const double* vals, int n, double multi_factor, double* out, void* stream);

/* ---- multi-GPU (RCCL over xGMI) --------------------------------------------------------- */
/* ncclUniqueId is 128 bytes; rank 0 creates it, the caller broadcasts it (torch.distributed). */
int mdr_rccl_unique_id(uint8_t* id128);
int mdr_rccl_init(mdr_ctx* ctx, const uint8_t* id128, int world, int rank);
/* in-place allreduce on `stream`: dtype 0 = int64 sum, 1 = double sum, 2 = double max,
 * 3 = uint32 sum, 4 = double min */
int mdr_rccl_allreduce(mdr_ctx* ctx, void* buf, int64_t count, int dtype, void* stream);
/* Host collectives: the same sharded C loops (mdr_rollout_begin / mdr_rollout_sharded /
 * mdr_actor_rollout_sharded) with their exchanges handed to the caller instead of the library
 * RCCL communicator — e.g. torch.distributed over gloo, so several ranks can share one GPU (how the
 * world > 2 sharded paths are tested on a 1-GPU box).  Before each callback the library
 * synchronises the stream the exchange is ordered on; the callback completes the exchange on the
 * device buffers before it returns (0 = OK).  allreduce: in place, `op` = the mdr_rccl_allreduce
 * dtype codes.  sendrecv: `send_bytes` from dev_send to rank dst and `recv_bytes` from rank src
 * into dev_recv, as one paired exchange; `tag` tells the two ring directions apart (1: to the next
 * rank, 2: to the previous).  Replaces SURVEY §8(e)'s RCCL calls one for one (environment.py:72-108
 * exchange points). */
typedef int (*mdr_host_allreduce_fn)(void* user, void* dev_buf, int64_t count, int op);
typedef int (*mdr_host_sendrecv_fn)(void* user, const void* dev_send, int64_t send_bytes, int dst, void* dev_recv,
                                    int64_t recv_bytes, int src, int tag);
int mdr_comm_host(mdr_ctx* ctx, int world, int rank, mdr_host_allreduce_fn allreduce, mdr_host_sendrecv_fn sendrecv,
                  void* user);
/* all-gather of `bytes` per rank into recv (world x bytes, rank order) on `stream` */
int mdr_rccl_allgather(mdr_ctx* ctx, const void* send, void* recv, int64_t bytes, void* stream);
/* sharded multi-tick rollout, RCCL allreduce of the count slab inside the loop:
 * per tick  [phase 1 if BUFFER] -> allreduce(counts) -> phase 2 (with lookahead when possible) */
int mdr_rollout_sharded(mdr_ctx* ctx, int n_ticks, const mdr_tick* ticks, const uint8_t* action,
                        int64_t act_stride, int action_mode, double* reward, int64_t rew_stride,
                        double* p_out, void* stream);
/* Pipelines mdr_rollout_sharded uses (MDR_OPT_WINDOW_PIPELINE / MDR_OPT_SHARDED_OVERLAP with the
 * communicator's side stream present): *window_pipeline = windows counted + allreduced on the side
 * stream ahead of the steps; *tick_overlap = one-tick rollouts with the allreduce of tick t beside
 * the step of tick t (that tick's reward written by the next launch, bit-identical). */
int mdr_rollout_sharded_mode(mdr_ctx* ctx, int* window_pipeline, int* tick_overlap);

/* ---- diagnostics ------------------------------------------------------------------------ */
/* Memory-floor probe: the loads/stores of one mdr_step over the bound arrays with no arithmetic
 * (writes the state back unchanged, garbage into reward).  Roofline calibration only. */
int mdr_probe_stream(mdr_ctx* ctx, double* reward, void* stream);
/* Exact-division self-check: counts (into *mismatches, device int64) the i where the
 * shared-reciprocal division sequence of the step kernels differs bitwise from a[i] / b[i]. */
int mdr_div_check(const double* a, const double* b, int64_t n, int64_t* mismatches, void* stream);

/* Phase profile of one mdr_actor_act launch (no outputs written): shader cycles per phase
 * averaged over the launch's blocks, cycles_out[8] (host): loop-top barrier wait, obs build,
 * prefetch + obs_out, layer 1, layer 2, -, output layer + softmax + stores (+ weight fill), tiles
 * per block.  Synchronises the stream. */
int mdr_actor_profile(mdr_ctx* ctx, const mdr_obs_spec* obs, const mdr_obs_scalars* sc, const double* p_dev,
                      double* cycles_out, void* stream);

/* ---- timing helpers for bench.py (HIP events on the given stream) ---------------------- */
int mdr_event_record(mdr_ctx* ctx, int slot, void* stream);
int mdr_event_elapsed_ms(mdr_ctx* ctx, int slot0, int slot1, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* MDR_H_ */
