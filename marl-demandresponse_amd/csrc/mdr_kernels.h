// mdr_kernels.h — kernel parameter blocks shared by the kernels and the C-ABI host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mdr.h"

namespace mdr {

constexpr int kCountShards = 64;  // atomic shards for the per-class ON counts
constexpr int kWinShards = 16;    // the shards a window count flush uses (the first 16 of kCountShards:
                                  // 128 adds per counter at 2048 blocks, one quarter of the reads to sum)
// waves per k_count_window block (a tile of 64 * kWinHpt houses per wave):
// 16 (512 blocks at 1M houses) against 4: 15.6 vs 17.3 us for 20 ticks, 8.9 vs 14.5 for 1 (r04i)
constexpr int kCountWaves = 16;
constexpr int kTicketGroups = 64; // grid_last_block: group counters (+ 1 top), 32 words apart
constexpr int kTicketWords = 32 * (kTicketGroups + 1);
constexpr int kSlabs = 4;         // count slabs: ring of 3 (step path) / 4 (overlapped pipeline)
constexpr int kObsBlock = 128;    // houses per obs tile
constexpr int kActBangBang = 16;  // internal action modes: controller evaluated on the loaded state
constexpr int kActDeadband = 17;

// Everything per-context a kernel needs, by value (one 256-B kernel argument).
struct KParams {
  int64_t n, goff, n_global;
  int dt, L, n_cap, penalty_mode;
  double deadband, alpha_temp, alpha_sig, norm_temp, norm_sig;
  double alpha_ind_l2, alpha_common_l2, alpha_common_max;
  uint64_t seed;
  double* t_air;
  double* t_mass;
  uint32_t* hvac;
  const double* ua;
  const double* ca;
  const double* cm;
  const double* hm;
  const double* target;
  const uint8_t* cap_idx;
  const double* q_on;  // [n_cap] -cap/(1+lcf)      (device, context-owned)
  const double* p_on;  // [n_cap] cap/cop
  const int* params_bad;  // device flag: some house's parameters are outside the fast-division range
  int fast_tick_ok;       // host-checked: dt and the capacity table are inside that range
};

struct TickArgs {
  double t_od_prev, solar, s_prev;
  uint64_t tick;
};

// Rollout tick drivers / per-tick obs scalars are staged into device memory by a kernel that
// takes them BY VALUE (kernel arguments are copied at launch), so the host never waits for a
// previous copy to finish before rewriting a staging buffer.
struct Rec32 {
  double v[4];
};
constexpr int kStageRecs = 64;  // 2 KiB of records per staging launch
struct StagePack {
  Rec32 r[kStageRecs];
};
static_assert(sizeof(TickArgs) == sizeof(Rec32), "TickArgs is staged as a 32-byte record");

struct PopArgs {
  double target_temp, std_target, lo, hi, ca0, cm0, hm0, init_air, init_mass;
  int n_draw;                     // capacity drawn over n_draw list entries (0: all n_cap)
  uint8_t draw_idx[MDR_MAX_CAP];  // table index of each list entry
};

struct ObsArgs {
  int n_feat, msg_w, n_comm, comm_mode;
  int hvac_state, solar_state, thermal_state, msg_thermal, msg_hvac;
  const int32_t* comm_table;
  const float* halo_msg;  // [lo + hi][msg_w] or null (halo_next set: only the lo rows before the shard)
  const float* halo_next; // the hi rows after the shard when they live apart from the lo rows, or null
  const float* msg_all;   // TABLE, sharded: [n_global][msg_w] (comm_table ids are global) or null
  double norm_reg_sig, cfg_ua, cfg_ca, cfg_cm, cfg_hm, cfg_cop, cfg_lcf, cfg_cap;
  double p, s, solar, t_od;
  const double* sc_dev;  // per-tick device mdr_obs_scalars row {-, s, solar, t_od} overriding the values above, or null
};

__global__ void k_stage32(StagePack pk, int n, Rec32* dst);
__global__ void k_zero_u64(unsigned long long* dst, int64_t n);
constexpr int kPcHouses = 4;  // chunks of 256 houses per k_power_counts block (grid: blocks(n, 256 * kPcHouses))
__global__ void k_power_counts(KParams p, const uint8_t* action, int action_mode, uint64_t tick,
                               const TickArgs* tkp, unsigned long long* slab);
template <int HPT, bool FAST, int ACT, int LA>
__global__ void k_step_t(KParams p, const uint8_t* action, int action_mode, TickArgs tk,
                         const TickArgs* tkp, const unsigned long long* counts, double* reward,
                         int ctrl, uint8_t* ctrl_out, double* p_out, int lookahead,
                         unsigned long long* next_slab, unsigned long long* zero_slab,
                         double* pen_partial, int reward_lag);
struct GqSel;
// the greedy controller's key outputs of a step kernel's epilogue (k_step_pipe GQ; k_gq_keys' outputs)
struct GqOut {
  uint8_t* act_out;  // (the fused tick, GQ = 2) every house's applied action, or null
  uint32_t* code;    // [n] the house's key bin << 2 | capacity class (gq_code)
  double* part;      // [grid][2] per-block (min, max) of the finite keys
  unsigned* hist;    // g_hist (the superbin copies follow its kGqBins * 4 bin words)
  GqSel* sel;        // this call's key map: the cell grid (GqSel.kmin, .scale) ...; the band (band_base, band_valid)
  const uint32_t* map;  // ... and the cells' bin ranges (gq_bin)
};
// waves per block of k_step_pipe with the GQ epilogue (4 without): fewer, larger blocks share one LDS
// superbin histogram, so fewer global flushes
constexpr int kStepGqWaves = 16;
// The fused greedy tick (mdr_greedy_rollout: producer -> k_gq_decide2 -> k_step_pipe<..., 2>).  The
// producer (the previous tick's step epilogue, or k_gq_keys2) writes, under the key map of its parity
// par, into parity region par: the superbin class counts of every house (C) and of the houses that
// can turn on at the next step (A: not locked out, hvac.py:43-64), the class counts (C, A) of the
// predicted band's bins, and the band's houses themselves as window entries in per-(copy, bin)
// buckets.  The decision needs no pass over the cluster when the band holds the crossing; the step
// applies it from the pre-step keys (the same bins under the same map) and the window houses' bytes.
constexpr int kGqfSup = 8 * 257 * 4;             // words: superbin class counts, kGqCopies x kGqSupN x 4
constexpr int kGqfBand = 8 * 8 * 64 * 4;         // words: band bin class counts, kGqCopies x band bins x 4
constexpr int kGqfBandN = 8 * 8 * 64;            // words: band bucket allocators, kGqCopies x band bins
constexpr int kGqfParWords = 2 * kGqfSup + 2 * kGqfBand + kGqfBandN + 64;  // + flags (64 words)
constexpr int kGqfMissC = 8 * 128 * 4;           // miss path: the bins of superbins sb, sb + 1 (C, A)
constexpr int kGqfMissN = 8 * 128;
constexpr int kGqfMissWords = 2 * kGqfMissC + kGqfMissN + 64;
// parity region offsets (words)
// (kGqfOffASum: the A summary, kGqCopies x {A_lo[4], A_all[4]}; the rest of its kGqfSup words unused)
constexpr int kGqfOffASum = kGqfSup, kGqfOffBandC = 2 * kGqfSup, kGqfOffBandA = 2 * kGqfSup + kGqfBand;
// the miss region's A_lo (the houses below the crossing superbin, per class) after its overflow flag
constexpr int kGqfOffMissALo = 2 * kGqfMissC + kGqfMissN + 1;
constexpr int kGqfOffBandN = 2 * kGqfSup + 2 * kGqfBand, kGqfOffFlags = kGqfOffBandN + kGqfBandN;
// decision modes (GqSel.fmode): the band / miss window's bins (take below bs, the window's bytes in
// [bs, be], nothing above), every house taken, every house's byte written (gq_exact)
enum { kGqfBandMode = 0, kGqfAll = 1, kGqfFull = 2 };
constexpr int kGqfList = 1024;  // a GQ = 2 step block's band houses, staged in LDS before their buckets
constexpr int kGqfStampWords = 32;  // phase stamps per block (mdr_greedy_fused_stamps)
struct GqfBufs {
  unsigned* par[2];      // the parity regions (kGqfParWords each)
  unsigned* miss;        // kGqfMissWords
  uint4* bkt[2];         // band buckets per parity: [kGqCopies][band bins][cap] window entries
  uint4* mbkt;           // miss buckets [kGqCopies][128][mcap]
  uint32_t* map[2];      // the key maps of the two parities (gq_bin)
  GqSel* sel;            // the fused path's own select record (fkmin / fscale per parity, the decision)
  uint8_t* dec;          // the decision bytes: window houses (band mode) or every house (full mode)
  int cap, mcap;         // bucket capacities (entries per copy and bin)
  unsigned long long* stamps;  // diagnostics (mdr_greedy_fused_stamps): k_gq_decide2's phase times, or null
};
template <int TPW, int ACT, int LA, int GQ = 0>
__global__ void k_step_pipe(KParams p, const uint8_t* action, TickArgs tk, const TickArgs* tkp,
                            const unsigned long long* counts, double* reward, double* p_out,
                            unsigned long long* next_slab, unsigned long long* zero_slab, GqOut gq,
                            GqfBufs fz, int fpar);
constexpr int kPipeMaxCap = 4;
constexpr int kWindowMax = 32;  // = kWinMax: ticks per k_step_window launch
constexpr int kWindowCap = 4;   // = kWinCap: capacity classes the window kernel supports
constexpr int kWindowRec = 4;   // = kWinRec: doubles per tick record of a window count slot
constexpr int kWinHpt = 2;      // houses per lane of the window kernels (a 128-house tile per wave)
// The first window's drivers as kernel arguments (k_step_window<..., KA = true>): the host computes
// them while the window's count and P-only reduce already run, and launches the step kernel with
// them, so no reduce or staging launch sits between the host's drivers and the thermal loop.
struct WinDrv {
  double od_k[kWindowMax];    // t_od_prev + 273.0 (rc_apply's od_k: the same IEEE addition on the host)
  double solar[kWindowMax];
  double s_prev[kWindowMax];  // the signal the tick's reward compares P with
  uint64_t tick0;             // the window's first tick id (ids are consecutive)
  double* p_out;              // last window: <- P of its last tick
  uint32_t ok;                // bit j: tick j's drivers are in the fast-division ranges
  const unsigned long long* red;  // sharded KA: the allreduced K x n_cap class totals — each lane's P
                                  // from them (win_power), in place of rec (no k_win_records launch)
};
// SIMPLE: deadband 0 and norm_temp 1 (reward without branches / division); FORM: the per-tick
// thermal update, MDR_THERMAL_EXACT (the reference's expression) or MDR_THERMAL_AFFINE (its
// per-window transition coefficients, mdr_kernels.hip K1W)
template <int ACT, int HPT, bool SIMPLE, bool KA, int FORM>
__global__ void k_step_window(KParams p, const uint8_t* action, int64_t act_stride, const TickArgs* tkp, int K,
                              int la_K, const double* rec, double* reward, int64_t rew_stride, uint64_t* onb,
                              uint32_t* wah, unsigned long long* next_slot, WinDrv dv);
__global__ void k_win_reduce(KParams p, unsigned long long* slot, int nt, const TickArgs* tkp, double* p_out);
__global__ void k_win_records(KParams p, unsigned long long* slot, int nt, const TickArgs* tkp, double* p_out);
template <int ACT, int HPT>
__global__ void k_count_window(KParams p, const uint8_t* action, int64_t act_stride, const TickArgs* tkp,
                               uint64_t tick0, int nt, unsigned long long* slot, uint64_t* onb, uint32_t* wah,
                               const uint32_t* w_in, unsigned* ticket);
__global__ void k_probe_stream(KParams p, double* reward);
__global__ void k_refresh(KParams p, int* params_bad);
__global__ void k_div_check(const double* a, const double* b, int64_t n, unsigned long long* mismatches);
__global__ void k_pen_reduce(const double* pen_partial, int nblk, double* partial2);
__global__ void k_reward_finalize(KParams p, TickArgs tk, const unsigned long long* counts,
                                  const double* partial2, double* reward);
__global__ void k_reward_state(KParams p, const TickArgs* tkp, const unsigned long long* counts,
                               double* reward, double* p_out);
__global__ void k_populate(KParams p, PopArgs a);
constexpr int kStats = 12;       // k_cluster_stats outputs (mdr.h mdr_cluster_stats)
constexpr int kStatsBlocks = 512;
__global__ void k_cluster_stats(KParams p, const double* reward, double* partial);
__global__ void k_cluster_stats_final(const double* partial, int nblk, double* out);
__global__ void k_obs(KParams p, ObsArgs o, const double* p_dev, float* obs);
__global__ void k_halo_pack(KParams p, ObsArgs o, int lo, int hi, float* out);
__global__ void k_halo_step_pack(KParams p, ObsArgs o, const uint8_t* action, const TickArgs* tkp, int lo, int hi,
                                 int rank, int world, float* rows);
__global__ void k_msg_pack(KParams p, ObsArgs o, float* out);
__global__ void k_greedy_keys(KParams p, double* key, int* idx);
__global__ void k_greedy_gather(KParams p, const int* perm, double* psorted, uint8_t* lsorted);
__global__ void k_greedy_walk(int64_t n, const double* incl, const double* psorted,
                              const uint8_t* lsorted, double S, double pmin, int64_t* kpos,
                              int64_t* extra, int max_extra);
__global__ void k_greedy_apply(int64_t n, const int* perm, const int64_t* kpos, const int64_t* extra,
                               uint8_t* action);
constexpr int kGqBins = 16384;  // histogram-select greedy: key bins
constexpr int kGqCap = 4096;    // candidate window capacity (LDS, 16 B per house)
constexpr int kGqAfter = 256;   // window houses past the crossing bin (the gap walk's room)
// the fused tick's room: a walk past the window falls back to gq_exact (one block over the cluster,
// ~7 ms at 1M houses, r06); with 256 the walk escaped on ~1 tick in 100 (most houses after the
// crossing locked out), the in-bin ranking costs what the bins hold, not the window
constexpr int kGqfAfter = 1024;
constexpr int kGqStage = 4096;  // houses per k_gq_compact block
constexpr int kGqParts = 256;  // k_gq_keys / k_gq_bins grid (one block per CU)
constexpr int kGqThreads = 1024; // k_gq_keys / k_gq_bins / k_gq_compact block size
constexpr int kGqCopies = 8;  // copies of the global superbin / bin histograms (blockIdx % kGqCopies)
constexpr int kGqUnroll = 4;    // houses per thread per pass of k_gq_keys / k_gq_bins
constexpr int kGqSuper = 256;   // superbins (64 bins each) of the select's first pass (+ 1 for NaN keys)
constexpr int kGqHistWords = kGqBins * 4 + kGqCopies * (kGqSuper + 1) * 4;  // g_hist: bin copies | superbin copies
// the predicted band: the bin class counts of kGqBand superbins around the previous call's crossing,
// counted by the step kernel's GQ epilogue (its kGqCopies copies sit after the bin copies, inside the
// first kGqBins * 4 words of g_hist); a call whose crossing lands inside skips the bins pass
constexpr int kGqBand = 8;
constexpr int kGqBandWords = kGqBand * 64 * 4;
constexpr int kGqBandOff = kGqCopies * 512;
static_assert(kGqBandOff + kGqCopies * kGqBandWords <= kGqBins * 4, "the band copies fit below the superbin copies");
static_assert(kGqHistWords % 2 == 0, "g_hist is zeroed as 64-bit words");
constexpr int kGqCells = 256;   // cells of the key -> bin map (gq_bin)
// bins the key map spreads over for a cluster of n houses: about 8 houses per bin at most, so a
// window of 64 bins holds a few hundred houses however small the cluster (a multiple of 64, >= 1024)
__host__ __device__ __forceinline__ int gq_bins_eff(int64_t n) {
  const int64_t b = (n / 8) & ~(int64_t)63;
  return b >= kGqBins ? kGqBins : (b < 1024 ? 1024 : (int)b);
}
static_assert(kGqfSup == kGqCopies * (kGqSuper + 1) * 4 && kGqfBand == kGqCopies * kGqBandWords &&
              kGqfBandN == kGqCopies * kGqBand * 64 && kGqfMissN == kGqCopies * 128,
              "the fused greedy's region sizes (declared before the histogram constants)");
constexpr int kGqSelBlocks = 256;  // k_gq_select grid, 1024 threads each
constexpr int kGqMaxRanks = 64;   // sharded histogram select: ranks whose windows k_gq_select gathers
struct GqSel;
constexpr int kGqSelBytes = 256;  // g_sel: the GqSel record
void gq_sel_init(void* sel, uint32_t* map);  // host: the first call's key map (uniform over [-32, 32])
void gq_diag_of(const void* sel, uint64_t* out);
void gq_state_of(const void* sel, uint64_t* out);  // gq_diag_of + {sb, bstar, bend, all, overflow, more_after, wcount, need_fb}
size_t gq_wcount_offset();   // host: byte offsets of GqSel.wcount / .need_fb (sharded select)
size_t gq_kmin_offset(int fpar);   // host: GqSel.kmin / .scale (fpar < 0), or the fused parity's fkmin / fscale
size_t gq_scale_offset(int fpar);
size_t gq_need_fb_offset();  // host: [fallbacks, calls, sum of window sizes, last window]
__global__ void k_gq_keys(KParams p, uint32_t* code, double* part, unsigned* hist, GqSel* sel,
                          const uint32_t* map, unsigned long long* slab);
__global__ void k_gq_bins(KParams p, const uint32_t* code, unsigned* hist, double S, GqSel* sel,
                          unsigned long long* slab);
__global__ void k_gq_compact(KParams p, const uint32_t* code, unsigned* hist, double S, GqSel* sel, uint4* win,
                             uint8_t* action, unsigned long long* slab);
__global__ void k_gq_binsc(KParams p, const uint32_t* code, unsigned* hist, double S, GqSel* sel, uint4* win,
                           uint8_t* action, unsigned long long* slab);
void gq_band_of(const void* sel, uint64_t* out);  // host: {calls that skipped the bins pass, calls, band base, band width}
__global__ void k_gq_finish(KParams p, const uint32_t* code, uint4* win, uint4* sorted, double S, double pmin,
                            GqSel* sel, uint8_t* action, unsigned long long* slab, unsigned* hist, unsigned* tickets,
                            const double* part, int nparts, uint32_t* map);
__global__ void k_gq_select(KParams p, const uint4* win, uint4* sorted, double S, double pmin, GqSel* sel,
                            uint8_t* action, unsigned long long* slab, unsigned* hist, const uint4* gathered,
                            int world, unsigned* tickets, const double* part, int nparts, uint32_t* map);
__global__ void k_gq_range(const double* part, int nparts, double* range);
// the fused tick: the producer without a step (the state's first decision), and the decision
__global__ void k_gq_keys2(KParams p, GqfBufs fz, int par, double* part, unsigned long long* slab);
__global__ void k_gq_decide2(KParams p, GqfBufs fz, int par, double S, double pmin, unsigned long long* slab,
                             unsigned* tickets, const double* part, int nparts);
__global__ void k_gq_remap(KParams p, const double* part, int nparts, unsigned* sup, GqSel* sel, uint32_t* map,
                           double* kmin_out, double* scale_out);
void gqf_sel_init(void* sel, uint32_t* map);  // host: the fused record (both parities' cells = gq_sel_init's)
void gqf_diag_of(const void* sel, uint64_t* out);  // host: {calls, band hits, misses, exact, last mode, last window}
__global__ void k_greedy_inputs(KParams p, double* key, double* power, uint8_t* lock);
__global__ void k_greedy_iota(int64_t n, int* idx);
__global__ void k_greedy_gather_rows(int64_t n, const int* perm, const double* power, const uint8_t* lock,
                                     double* psorted, uint8_t* lsorted);

}  // namespace mdr
