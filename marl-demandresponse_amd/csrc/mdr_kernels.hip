// mdr_kernels.hip — house-parallel kernels of the vectorised environment step (gfx950 / CDNA4).
//
// Bandwidth-bound elementwise work: one thread per house, SoA fp64 state/params loaded with
// coalesced 8-B-per-lane accesses, the per-context cooling-capacity tables staged in LDS, the
// cluster power reduced with wave ballots + LDS histogram + sharded global atomics (integer
// counts per capacity class, so the sum is exact and order independent).  No MFMA: there is
// no contraction on this path.
#include "mdr_kernels.h"

#include <type_traits>

#include "mdr_device.h"
#include "mdr_obs_dev.h"

namespace mdr {

// --------------------------------------------------------------------------------------- helpers

// Per-block histogram of ON houses per capacity class, flushed to the sharded slab with at most
// n_cap atomics per block: slab[(blockIdx % kCountShards) * MDR_MAX_CAP + k].
__device__ __forceinline__ void count_on(bool on, int cls, int n_cap, unsigned* hist,
                                         unsigned long long* slab) {
  const int lane = threadIdx.x & 63;
  for (int k = 0; k < n_cap; ++k) {
    const unsigned long long m = __ballot(on && cls == k);
    if (lane == 0 && m) atomicAdd(&hist[k], (unsigned)__popcll(m));
  }
  __syncthreads();
  if ((int)threadIdx.x < n_cap) {
    const unsigned v = hist[threadIdx.x];
    if (v) atomicAdd(&slab[(blockIdx.x % kCountShards) * n_cap + threadIdx.x],
                     (unsigned long long)v);
  }
}

__global__ void k_stage32(StagePack pk, int n, Rec32* __restrict__ dst) {
  const int i = threadIdx.x;
  if (i < n) dst[i] = pk.r[i];
}

// n 64-bit zeros from a kernel (the count slabs inside captured launch sequences: see
// mdr_capi.hip zero_u64)
__global__ void k_zero_u64(unsigned long long* __restrict__ dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = 0ull;
}

// --------------------------------------------------------------------------------------- K0
// Phase 1: FSM only -> ON count per capacity class (cluster.py:82-88).  Reads 6 B per house.
__global__ void __launch_bounds__(256) k_power_counts(KParams p, const uint8_t* __restrict__ action,
                                                      int action_mode, uint64_t tick0,
                                                      const TickArgs* tkp,
                                                      unsigned long long* __restrict__ slab) {
  const uint64_t tick = tkp ? tkp->tick : tick0;
  __shared__ unsigned hist[MDR_MAX_CAP];
  if ((int)threadIdx.x < p.n_cap) hist[threadIdx.x] = 0;
  // kPcHouses chunks of 256 houses per block, every load issued before the first use
  uint32_t hw[kPcHouses];
  int cls[kPcHouses];
  bool a[kPcHouses];
#pragma unroll
  for (int u = 0; u < kPcHouses; ++u) {
    const int64_t c0 = ((int64_t)blockIdx.x * kPcHouses + u) * blockDim.x;
    const int64_t i = c0 + threadIdx.x;
    a[u] = action_mode == MDR_ACT_ALWAYS_ON;
    if (action_mode == MDR_ACT_RANDOM) {
      const WaveRandom wr(p.seed, p.goff + c0 + (threadIdx.x & ~63), tick);  // whole wave, before any divergence
      a[u] = wr.get(p.goff + i, false);
    }
    hw[u] = 0u;
    cls[u] = -1;
    if (i < p.n) {
      if (action_mode == MDR_ACT_BUFFER) a[u] = action[i] != 0;
      hw[u] = p.hvac[i];
      cls[u] = p.cap_idx[i];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < kPcHouses; ++u) {
    const bool on = cls[u] >= 0 && hv_on(hvac_fsm(hw[u], a[u], p.dt, p.L));
    for (int k = 0; k < p.n_cap; ++k) {
      const unsigned long long m = __ballot(on && cls[u] == k);
      if (lane == 0 && m) atomicAdd(&hist[k], (unsigned)__popcll(m));
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < p.n_cap) {
    const unsigned v = hist[threadIdx.x];
    if (v) atomicAdd(&slab[(blockIdx.x % kCountShards) * p.n_cap + threadIdx.x], (unsigned long long)v);
  }
}

// ---- greedy selection state and key-histogram helpers (the k_gq_* kernels below; k_step_pipe
// writes the keys in its GQ epilogue)
struct GqSel {
  double kmin, scale;            // the key map's cell grid: cell = (k - kmin) * scale (gq_code)
  double base_tot;               // P of the houses before the crossing superbin (k_gq_bins; read by every k_gq_compact block)
  double win_tot;                // P of the houses before the window (k_gq_compact block 0 -> k_gq_select; a field of its
                                 // own: overwriting base_tot raced with the compact blocks still reading it)
  unsigned long long base_cnt, total;
  int sb, bstar, bend, all, overflow, more_after, ncand;
  int whole;                     // the cluster fits the window (<= kGqCap houses): every house is a candidate
  unsigned fallbacks;            // calls decided by the exact fallback (gq_exact; diagnostics)
  unsigned wcount;               // k_gq_compact's window allocator (zeroed by gq_decide for the next call; k_gq_bins)
  unsigned calls;                // diagnostics: decisions made, and the sum of their window sizes
  unsigned need_fb;              // sharded: the window could not decide this call (host falls back)
  unsigned long long ncand_sum;
  int band_base;                 // the first superbin of the predicted band the GQ epilogue counts bins of
                                 // (gq_next_map: centred on where this call's crossing lands in the next map)
  unsigned xcnt;                 // the houses before the crossing bin (gq_window block 0 -> gq_next_map)
  unsigned xprev;                // the previous call's xcnt + 1 (0: none), for the band's trend
  int sb_raw;                    // this call's crossing superbin as the last call predicted it (-1: none)
  int sb_bias;                   // the last prediction's error (actual - predicted superbin)
  int band_valid;                // the band copies hold this call's counts (the GQ epilogue sets it)
  int hit;                       // k_gq_binsc compacted from the band (k_gq_finish ranks; reset by its decider)
  unsigned hits;                 // diagnostics: calls whose bins pass was skipped
  // the fused tick (k_gq_decide2; its own record): the cell grids of the two parities' key maps, the
  // decision the step applies, diagnostics
  double fkmin[2], fscale[2];
  int fmode, fbs, fbe;           // kGqfBandMode: take bins < fbs, the bytes of [fbs, fbe]; kGqfAll; kGqfFull
  int fband[2];                  // the band_base of each parity's producer (decide2(par) writes fband[1 - par]:
                                 // a block of the same launch may still read fband[par])
  unsigned fcalls, fhits, fmisses, fexact, fwin;
};
static_assert(sizeof(GqSel) <= kGqSelBytes, "GqSel fits the g_sel buffer");
void gq_sel_init(void* sel, uint32_t* map) {
  GqSel* g = static_cast<GqSel*>(sel);  // (a zeroed host buffer of kGqSelBytes)
  g->kmin = -4.0;                           // the first call: uniform bins over keys in [-4, 4] (K from
  g->scale = (double)kGqCells / 8.0;        // the target; keys outside clamp into the end cells)
  for (int c = 0; c < kGqCells; ++c) map[c] = ((uint32_t)(c * (kGqBins / kGqCells)) << 16) | (uint32_t)(kGqBins / kGqCells);
  g->band_base = kGqSuper / 2 - kGqBand / 2;
  g->sb_raw = -1;
}
void gqf_sel_init(void* sel, uint32_t* map) {
  gq_sel_init(sel, map);
  GqSel* g = static_cast<GqSel*>(sel);
  for (int q = 0; q < 2; ++q) {
    g->fkmin[q] = g->kmin;
    g->fscale[q] = g->scale;
    g->fband[q] = g->band_base;
  }
}
void gqf_diag_of(const void* sel, uint64_t* out) {
  const GqSel* g = static_cast<const GqSel*>(sel);
  out[0] = g->fcalls;
  out[1] = g->fhits;
  out[2] = g->fmisses;
  out[3] = g->fexact;
  out[4] = (uint64_t)(int64_t)g->fmode;
  out[5] = g->fwin;
}
void gq_band_of(const void* sel, uint64_t* out) {
  const GqSel* g = static_cast<const GqSel*>(sel);
  out[0] = g->hits;
  out[1] = g->calls;
  out[2] = (uint64_t)(int64_t)g->band_base;
  out[3] = (uint64_t)kGqBand;
}
size_t gq_wcount_offset() { return offsetof(GqSel, wcount); }
size_t gq_kmin_offset(int fpar) { return fpar < 0 ? offsetof(GqSel, kmin) : offsetof(GqSel, fkmin) + fpar * sizeof(double); }
size_t gq_scale_offset(int fpar) { return fpar < 0 ? offsetof(GqSel, scale) : offsetof(GqSel, fscale) + fpar * sizeof(double); }
size_t gq_need_fb_offset() { return offsetof(GqSel, need_fb); }
void gq_diag_of(const void* sel, uint64_t* out) {
  const GqSel* g = static_cast<const GqSel*>(sel);
  out[0] = g->fallbacks;
  out[1] = g->calls;
  out[2] = g->ncand_sum;
  out[3] = (uint64_t)(int64_t)g->ncand;
}
void gq_state_of(const void* sel, uint64_t* out) {
  const GqSel* g = static_cast<const GqSel*>(sel);
  gq_diag_of(sel, out);
  const int v[8] = {g->sb, g->bstar, g->bend, g->all, g->overflow, g->more_after, (int)g->wcount, (int)g->need_fb};
  for (int k = 0; k < 8; ++k) out[4 + k] = (uint64_t)(int64_t)v[k];
}

constexpr int kGqSupN = kGqSuper + 1;  // superbins + one for NaN keys (sorted last, pandas' na_position)
constexpr int kGqSupStride = kGqSupN * 4;

// okey: -0.0 folded onto +0.0 (value order, numpy's stable argsort), sign-magnitude -> unsigned;
// NaN after every number
__device__ __forceinline__ uint64_t gq_okey(double k) {
  if (k != k) return ~0ull;
  const uint64_t b = (uint64_t)__double_as_longlong(k + 0.0);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
// The key -> bin map (equi-depth, piecewise linear): kGqCells uniform cells over the previous
// call's key range, cell c owning bins [B0_c, B0_c + W_c) (map[c] = B0_c << 16 | W_c, W_c >= 1,
// the W_c summing to kGqBins) in proportion to the houses the previous call had there (k_gq_bins
// builds the next map from this call's superbin histogram), so dense key ranges get many narrow
// bins and the candidate window stays small.  The bin is monotone non-decreasing in k for ANY map,
// range and scale >= 0 (keys outside the range clamp into the end cells), so a stale map only
// costs window size, never exactness.
// In float32: every step (the conversion of k, the subtraction of kmin, the product with the
// positive scale, the truncations) is monotone non-decreasing in k, and a cell's bins end where the
// next cell's begin, so the bin is monotone in the key — all the histogram select needs (the window
// orders its houses by their exact float64 keys; NaN keys never come here).  Every producer of codes
// uses this one function.  (Float64 arithmetic here cost the GQ step kernel's fp64 VALU pipe.)
__device__ __forceinline__ int gq_bin(double k, double kmin, double scale, const uint32_t* map) {
  const float u = ((float)k - (float)kmin) * (float)scale;
  const int c = u >= (float)(kGqCells - 1) ? kGqCells - 1 : (u > 0.0f ? (int)u : 0);
  const uint32_t m = map[c];
  const int w = (int)(m & 0xFFFFu);
  const float f = (u - (float)c) * (float)w;
  return (int)(m >> 16) + (f >= (float)(w - 1) ? w - 1 : (f > 0.0f ? (int)f : 0));
}
// a house's code: its key bin (kGqBins for a NaN key) << 2 | its capacity class; the superbin is
// code >> 8 (kGqBins / kGqSuper = 64 bins each; NaN keys land in superbin kGqSuper)
__device__ __forceinline__ uint32_t gq_code(double k, double kmin, double scale, const uint32_t* map, unsigned cls) {
  return ((uint32_t)(k != k ? kGqBins : gq_bin(k, kmin, scale, map)) << 2) | (cls & 3u);
}
__device__ __forceinline__ double gq_key_of(const KParams& p, int64_t i) {
  return -(p.t_air[i] - p.target[i]);  // greedy_myopic_controller.py:79
}

// the keys' producer side, shared by k_gq_keys and the step kernel's epilogue: a block's houses go
// into ncopy LDS superbin histograms (wave w into copy w % ncopy), then one flush per block (spread
// over kGqCopies global copies) and the block's (min, max) of the finite keys into part[]
__device__ __forceinline__ void gq_flush(const unsigned* s_sh, int ncopy, unsigned* hist, double lo, double hi,
                                         double* part) {
  const int nw = (int)(blockDim.x >> 6);
  __shared__ double s_lo[16], s_hi[16];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
  }
  if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double l = s_lo[0], h = s_hi[0];
    for (int w = 1; w < nw; ++w) { l = fmin(l, s_lo[w]); h = fmax(h, s_hi[w]); }
    part[2 * blockIdx.x] = l;
    part[2 * blockIdx.x + 1] = h;
  }
  for (int e = threadIdx.x; e < kGqSupStride; e += blockDim.x) {
    unsigned v = 0u;
    for (int w = 0; w < ncopy; ++w) v += s_sh[w * kGqSupStride + e];
    if (v) atomicAdd(&hist[kGqBins * 4 + (blockIdx.x % kGqCopies) * kGqSupStride + e], v);
  }
}

// The fused tick's A summary (the houses that can turn on at the next step, per class): of the houses
// below the band's first superbin (A_lo) and of every house (A_all) — the decision's ON counts of the
// houses it takes outside the window (A_lo plus the band's A bins below the window, or A_all when every
// house is taken); per-superbin A counts are not kept (r06: their flush atomics cost ~1.7 us a step).
// Per lane: 16-bit fields (classes 0/1 and 2/3), summed over the wave at the block's end.
struct GqfAcnt {
  uint32_t lo01, lo23, al01, al23;
};
__device__ __forceinline__ void gqf_acount(GqfAcnt& a, bool canon, bool below, unsigned cls) {
  const uint32_t inc = canon ? 1u << (16u * (cls & 1u)) : 0u;
  const uint32_t il = below ? inc : 0u;
  if (cls < 2u) { a.al01 += inc; a.lo01 += il; }
  else { a.al23 += inc; a.lo23 += il; }
}
// the wave's sums into s_acnt[8] (A_lo[4], A_all[4]; LDS, zeroed by the caller before a barrier)
__device__ __forceinline__ void gqf_acount_wave(GqfAcnt a, unsigned* s_acnt) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a.lo01 += __shfl_xor(a.lo01, off);
    a.lo23 += __shfl_xor(a.lo23, off);
    a.al01 += __shfl_xor(a.al01, off);
    a.al23 += __shfl_xor(a.al23, off);
  }
  if ((threadIdx.x & 63) == 0) {
    const uint32_t v[8] = {a.lo01 & 0xFFFFu, a.lo01 >> 16, a.lo23 & 0xFFFFu, a.lo23 >> 16,
                           a.al01 & 0xFFFFu, a.al01 >> 16, a.al23 & 0xFFFFu, a.al23 >> 16};
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (v[k]) atomicAdd(&s_acnt[k], v[k]);
  }
}
// the fused tick's producer flush: the LDS copies of the superbin C counts into the parity region's
// copy blockIdx % kGqCopies, the block's A summary (s_acnt, complete after this function's barrier)
// into the copy's 8 summary words, and the block's (min, max) of the finite keys
__device__ __forceinline__ void gqf_flush(const unsigned* s_sh, int ncopy, unsigned* par, double lo, double hi,
                                          double* part, const unsigned* s_acnt) {
  const int nw = (int)(blockDim.x >> 6);
  __shared__ double s_lo[16], s_hi[16];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
  }
  if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double l = s_lo[0], h = s_hi[0];
    for (int w = 1; w < nw; ++w) { l = fmin(l, s_lo[w]); h = fmax(h, s_hi[w]); }
    part[2 * blockIdx.x] = l;
    part[2 * blockIdx.x + 1] = h;
  }
  const int cp = (int)(blockIdx.x % kGqCopies);
  if (threadIdx.x < 8 && s_acnt[threadIdx.x]) atomicAdd(&par[kGqfOffASum + cp * 8 + threadIdx.x], s_acnt[threadIdx.x]);
  for (int e = threadIdx.x; e < kGqSupStride; e += blockDim.x) {
    unsigned v = 0u;
    for (int w = 0; w < ncopy; ++w) v += s_sh[w * kGqSupStride + e];
    if (v) atomicAdd(&par[cp * kGqSupStride + e], v);
  }
}

// --------------------------------------------------------------------------------------- K1
// Phase 2: fused FSM + RC thermal + reward (environment.py:86-101) for one tick, HPT houses per
// thread (HPT = 2: 16-B-per-lane loads/stores of the fp64 SoA arrays, two independent fp64
// dependency chains per thread).
//   counts    : the tick's GLOBAL per-class ON counts, slab [kCountShards][n_cap]; every wave
//               reduces it itself (lane l reads shard l), so no block barrier precedes the work
//   next_slab : when lookahead != 0, ON counts of tick+1 under the in-kernel action source
//               (random / always-on / bang-bang on the new state) are accumulated here, so the
//               next tick needs no phase-1 launch.

// sum over the 64 lanes; 32-bit partial sums are exact while the cluster has < 2^32 houses
__device__ __forceinline__ unsigned long long wave_sum_counts(unsigned long long v64) {
  unsigned v = (unsigned)v64;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (unsigned)__shfl_xor((int)v, off);
  return v;
}

// cluster power of the tick from the sharded count slab (uniform in the wave)
__device__ __forceinline__ double wave_power(const unsigned long long* __restrict__ counts,
                                             const double* __restrict__ p_on, int n_cap) {
  static_assert(kCountShards == 64, "one shard per lane");
  const int lane = threadIdx.x & 63;
  double P = 0.0;
  for (int k = 0; k < n_cap; ++k) {
    const unsigned long long c = wave_sum_counts(counts[lane * n_cap + k]);
    P += (double)c * p_on[k];
  }
  return P;
}

__device__ __forceinline__ bool pick_action(int mode, const uint8_t* action, uint32_t i, bool rnd,
                                            double T, double tgt, double deadband, uint32_t w0) {
  if (mode == MDR_ACT_BUFFER) return action[i] != 0;
  if (mode == MDR_ACT_RANDOM) return rnd;
  if (mode == MDR_ACT_ALWAYS_ON) return true;
  if (mode == kActBangBang) return ctrl_bangbang(T, tgt);
  return ctrl_deadband(T, tgt, deadband, hv_on(w0));
}

// Loads/stores at an SGPR base + 32-bit VGPR byte offset (computed in 32 bits, so the compiler
// emits the saddr form instead of a 64-bit address add per array).
template <typename V>
__device__ __forceinline__ V ldo(const void* base, uint32_t off) {
  return *reinterpret_cast<const V*>(reinterpret_cast<const char*>(base) + off);
}
template <typename V>
__device__ __forceinline__ void sto(void* base, uint32_t off, V v) {
  *reinterpret_cast<V*>(reinterpret_cast<char*>(base) + off) = v;
}
// reward rows: written once, never re-read by the step kernels — non-temporal stores keep them from
// evicting the state and parameters the next launch reads (the Infinity Cache holds them at 1M houses)
__device__ __forceinline__ void sto_nt(void* base, uint32_t off, double2 v) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(d2{v.x, v.y}, reinterpret_cast<d2*>(reinterpret_cast<char*>(base) + off));
}

template <int HPT, bool FAST, int ACT, int LA>
__global__ void __launch_bounds__(256) k_step_t(KParams p, const uint8_t* __restrict__ action,
                                                int action_mode_rt, TickArgs tk0, const TickArgs* tkp,
                                                const unsigned long long* __restrict__ counts,
                                                double* __restrict__ reward, int ctrl,
                                                uint8_t* __restrict__ ctrl_out, double* p_out,
                                                int lookahead_rt, unsigned long long* next_slab,
                                                unsigned long long* zero_slab,
                                                double* __restrict__ pen_partial, int reward_lag) {
  // ACT / LA >= 0: action source / lookahead fixed at compile time (the hot configurations);
  // -1: taken from the runtime arguments
  const int action_mode = ACT >= 0 ? ACT : action_mode_rt;
  const int lookahead = LA >= 0 ? LA : lookahead_rt;
  __shared__ unsigned hist[MDR_MAX_CAP];
  __shared__ double s_red[2][4];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  if (tid < p.n_cap) hist[tid] = 0;
  if (zero_slab && blockIdx.x == 0)
    for (int j = tid; j < kCountShards * p.n_cap; j += blockDim.x) zero_slab[j] = 0ull;

  // one wave tile of 64*HPT consecutive houses per wave (no grid-stride loop: straight-line code
  // keeps the kernel-argument SGPRs short-lived); 32-bit element indices (n_local < 2^29) so
  // every access is an SGPR base + 32-bit VGPR offset
  const uint32_t tile = blockIdx.x * (blockDim.x >> 6) + (tid >> 6);
  const uint32_t n = (uint32_t)p.n;
  const uint32_t i0 = tile * (64u * HPT) + (uint32_t)lane * HPT;
  bool valid[HPT];
#pragma unroll
  for (int h = 0; h < HPT; ++h) valid[h] = i0 + h < n;

  // ---- all per-house loads first (one round trip)
  uint32_t w0[HPT];
  double T[HPT], Tm[HPT], ua[HPT], ca[HPT], hm[HPT], tg[HPT];
  double cm[HPT];
  int cls[HPT];
  if (HPT == 2 && valid[HPT - 1]) {
    const uint32_t o8 = i0 * 8u;
    auto ld2 = [&](const double* a) { return ldo<double2>(a, o8); };
    const double2 vT = ld2(p.t_air), vTm = ld2(p.t_mass), vua = ld2(p.ua), vca = ld2(p.ca);
    const double2 vhm = ld2(p.hm), vtg = ld2(p.target);
    const uint2 vw = ldo<uint2>(p.hvac, i0 * 4u);
    const unsigned short vc = ldo<unsigned short>(p.cap_idx, i0);
    T[0] = vT.x; T[HPT - 1] = vT.y; Tm[0] = vTm.x; Tm[HPT - 1] = vTm.y;
    ua[0] = vua.x; ua[HPT - 1] = vua.y; ca[0] = vca.x; ca[HPT - 1] = vca.y;
    hm[0] = vhm.x; hm[HPT - 1] = vhm.y;
    tg[0] = vtg.x; tg[HPT - 1] = vtg.y; w0[0] = vw.x; w0[HPT - 1] = vw.y;
    cls[0] = vc & 0xFF; cls[HPT - 1] = vc >> 8;
    const double2 vcm = ld2(p.cm);
    cm[0] = vcm.x; cm[HPT - 1] = vcm.y;
  } else {
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      const uint32_t i = valid[h] ? i0 + h : 0u;
      T[h] = p.t_air[i]; Tm[h] = p.t_mass[i]; ua[h] = p.ua[i]; ca[h] = p.ca[i];
      hm[h] = p.hm[i]; tg[h] = p.target[i]; w0[h] = p.hvac[i]; cls[h] = p.cap_idx[i];
      cm[h] = p.cm[i];
    }
  }
  __syncthreads();  // hist zeroed (the loads above stay in flight across the barrier)

  const TickArgs tk = tkp ? *tkp : tk0;
  // per-tick signal penalty (rewards_calculator.py:183-203), uniform in the wave.
  // reward_lag (overlapped multi-GPU pipeline, tkp required): this launch writes the reward of the
  // PREVIOUS tick — its temperature penalty from the loaded state (= that tick's result) and its
  // signal term from `counts` = that tick's allreduced slab — so the allreduce of tick t runs
  // concurrently with the launch of tick t.  counts == nullptr there (first tick): no reward.
  double sig_term = 0.0;
  const bool write_rew = counts != nullptr;
  if (counts) {
    const double P = wave_power(counts, p.p_on, p.n_cap);
    const double x = (P - (reward_lag ? tkp[-1].s_prev : tk.s_prev)) / (double)p.n_global;
    sig_term = p.alpha_sig * (x * x) / p.norm_sig;
    if (p_out && blockIdx.x == 0 && tid == 0) *p_out = P;
  }

  // random controller bits of this tick (and the next, for the lookahead) for the whole wave
  bool rnd[HPT], rnd1[HPT];
  if (action_mode == MDR_ACT_RANDOM || lookahead == MDR_ACT_RANDOM) {
    const WaveRandom wr(p.seed, p.goff + (uint64_t)tile * (64u * HPT), tk.tick);
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      rnd[h] = wr.get(p.goff + i0 + h, false);
      rnd1[h] = wr.get(p.goff + i0 + h, true);
    }
  } else {
#pragma unroll
    for (int h = 0; h < HPT; ++h) rnd[h] = rnd1[h] = false;
  }

  // shared-reciprocal division only where it is provably the IEEE quotient (mdr_device.h)
  bool house_ok = true;
#pragma unroll
  for (int h = 0; h < HPT; ++h) house_ok = house_ok && fabs(T[h]) < 1048576.0 && fabs(Tm[h]) < 1048576.0;
  const bool tile_fast = FAST && !*p.params_bad && p.fast_tick_ok && fabs(tk.t_od_prev) < 1048576.0 &&
                         fabs(tk.solar) < 1099511627776.0 && __all(house_ok);

  double Tn[HPT], Tmn[HPT], rw[HPT], pen[HPT];
  uint32_t w[HPT];
  bool on[HPT], on1[HPT];
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    const uint32_t i = i0 + h;
    const bool a = valid[h] && pick_action(action_mode, action, i, rnd[h], T[h], tg[h], p.deadband, w0[h]);
    w[h] = hvac_fsm(w0[h], a, p.dt, p.L);
    on[h] = hv_on(w[h]);
    const double q = on[h] ? p.q_on[cls[h]] : 0.0;
    if (tile_fast) {
      const RcCoef kc = rc_coeffs_t<FAST>(ua[h], ca[h], cm[h], hm[h], (double)p.dt);
      rc_apply_t<FAST>(T[h], Tm[h], ua[h], ca[h], hm[h], kc, q, tk.solar, tk.t_od_prev, Tn[h], Tmn[h]);
    } else {
      const RcCoef kc = rc_coeffs_t<false>(ua[h], ca[h], cm[h], hm[h], (double)p.dt);
      rc_apply_t<false>(T[h], Tm[h], ua[h], ca[h], hm[h], kc, q, tk.solar, tk.t_od_prev, Tn[h], Tmn[h]);
    }
    pen[h] = deadband_l2(tg[h], p.deadband, reward_lag ? T[h] : Tn[h]);
    // x / 1.0 == x exactly: the default normaliser (integer target) costs no division
    const double tpen = p.alpha_temp * pen[h];
    rw[h] = p.penalty_mode == MDR_PEN_INDIVIDUAL_L2
                ? -((p.norm_temp == 1.0 ? tpen : tpen / p.norm_temp) + sig_term)
                : pen[h];  // finalised by k_reward_finalize
    on1[h] = false;
    if (lookahead) {
      bool an;
      if (lookahead == MDR_ACT_RANDOM) an = rnd1[h];
      else if (lookahead == MDR_ACT_ALWAYS_ON) an = true;
      else if (lookahead == kActBangBang) an = ctrl_bangbang(Tn[h], tg[h]);
      else an = ctrl_deadband(Tn[h], tg[h], p.deadband, on[h]);
      on1[h] = valid[h] && hv_on(hvac_fsm(w[h], an, p.dt, p.L));
    }
  }

  // ---- stores
  if (HPT == 2 && valid[HPT - 1]) {
    const uint32_t o8 = i0 * 8u;
    sto(p.t_air, o8, make_double2(Tn[0], Tn[HPT - 1]));
    sto(p.t_mass, o8, make_double2(Tmn[0], Tmn[HPT - 1]));
    sto(p.hvac, i0 * 4u, make_uint2(w[0], w[HPT - 1]));
    if (write_rew) sto_nt(reward, o8, make_double2(rw[0], rw[HPT - 1]));
  } else {
#pragma unroll
    for (int h = 0; h < HPT; ++h)
      if (valid[h]) {
        p.t_air[i0 + h] = Tn[h]; p.t_mass[i0 + h] = Tmn[h]; p.hvac[i0 + h] = w[h];
        if (write_rew) __builtin_nontemporal_store(rw[h], reward + i0 + h);
      }
  }
  if (ctrl != MDR_CTRL_NONE && ctrl_out) {
#pragma unroll
    for (int h = 0; h < HPT; ++h)
      if (valid[h]) {
        const bool a1 = ctrl == MDR_CTRL_BANGBANG ? ctrl_bangbang(Tn[h], tg[h])
                                                   : ctrl_deadband(Tn[h], tg[h], p.deadband, on[h]);
        ctrl_out[i0 + h] = a1 ? 1 : 0;
      }
  }

  // ---- cluster reductions for the next launch / the common penalty modes
  if (lookahead) {
    for (int k = 0; k < p.n_cap; ++k) {
      unsigned c = 0;
#pragma unroll
      for (int h = 0; h < HPT; ++h) c += (unsigned)__popcll(__ballot(on1[h] && cls[h] == k));
      if (lane == 0 && c) atomicAdd(&hist[k], c);
    }
    __syncthreads();
    if (tid < p.n_cap && hist[tid])
      atomicAdd(&next_slab[(blockIdx.x % kCountShards) * p.n_cap + tid], (unsigned long long)hist[tid]);
  }
  if (p.penalty_mode != MDR_PEN_INDIVIDUAL_L2) {
    double sacc = 0.0, macc = 0.0;
#pragma unroll
    for (int h = 0; h < HPT; ++h)
      if (valid[h]) { sacc += pen[h] / (double)p.n_global; macc = fmax(macc, pen[h]); }
    for (int off = 32; off > 0; off >>= 1) {
      sacc += __shfl_xor(sacc, off);
      macc = fmax(macc, __shfl_xor(macc, off));
    }
    if (lane == 0) { s_red[0][tid >> 6] = sacc; s_red[1][tid >> 6] = macc; }
    __syncthreads();
    if (tid == 0) {
      double bs = 0.0, bm = 0.0;
      for (int w2 = 0; w2 < (int)(blockDim.x >> 6); ++w2) { bs += s_red[0][w2]; bm = fmax(bm, s_red[1][w2]); }
      pen_partial[2 * blockIdx.x] = bs;
      pen_partial[2 * blockIdx.x + 1] = bm;
    }
  }
}

// --------------------------------------------------------------------------------------- K1'
// Software-pipelined form of the hot step configurations (HPT = 2, shared-reciprocal division,
// individual_L2, <= kPipeCap capacity classes): a wave steps TPW tiles (strided over the grid),
// issuing tile k+1's loads before computing tile k, so the memory stream of one tile overlaps the
// fp64 arithmetic of the previous one.  Straight-line code (TPW and the class loops are unrolled
// at compile time): a loop in the body would make the compiler drain the in-flight loads at its
// header.  Results are bit-identical to k_step_t (same per-house expressions).
constexpr int kPipeCap = 4;

struct Tile2 {
  double2 T, Tm, ua, ca, cm, hm, tg;
  uint2 w;
  unsigned cls;  // two u8 capacity classes
  unsigned act;  // two u8 actions (MDR_ACT_BUFFER)
};

// full: the whole wave tile is inside the shard (wave-uniform), so every lane takes the 16-B path;
// otherwise (the last, ragged tile) each house is loaded on its own from a clamped index (a house
// past the end is computed on a copy of house n-1 and never stored or counted)
template <bool ACT_BUF>
__device__ __forceinline__ void load_tile2(const KParams& p, const uint8_t* action, uint32_t i0, uint32_t n,
                                           bool full, Tile2& t) {
  if (full) {
    const uint32_t o8 = i0 * 8u;
    t.T = ldo<double2>(p.t_air, o8); t.Tm = ldo<double2>(p.t_mass, o8);
    t.ua = ldo<double2>(p.ua, o8); t.ca = ldo<double2>(p.ca, o8); t.cm = ldo<double2>(p.cm, o8);
    t.hm = ldo<double2>(p.hm, o8); t.tg = ldo<double2>(p.target, o8);
    t.w = ldo<uint2>(p.hvac, i0 * 4u);
    t.cls = ldo<unsigned short>(p.cap_idx, i0);
    t.act = ACT_BUF ? (unsigned)ldo<unsigned short>(action, i0) : 0u;
  } else {
    const uint32_t a = i0 < n ? i0 : n - 1u, b = i0 + 1u < n ? i0 + 1u : n - 1u;
    t.T = make_double2(p.t_air[a], p.t_air[b]); t.Tm = make_double2(p.t_mass[a], p.t_mass[b]);
    t.ua = make_double2(p.ua[a], p.ua[b]); t.ca = make_double2(p.ca[a], p.ca[b]);
    t.cm = make_double2(p.cm[a], p.cm[b]); t.hm = make_double2(p.hm[a], p.hm[b]);
    t.tg = make_double2(p.target[a], p.target[b]);
    t.w = make_uint2(p.hvac[a], p.hvac[b]);
    t.cls = (unsigned)p.cap_idx[a] | ((unsigned)p.cap_idx[b] << 8);
    t.act = ACT_BUF ? ((unsigned)action[a] | ((unsigned)action[b] << 8)) : 0u;
  }
}

// GQ = 1: the greedy controller's keys of the post-step state, their superbin histogram and the
// block's key range (k_gq_keys' outputs, gq_flush) as an epilogue, so the next mdr_ctrl_greedy
// skips its key pass; blocks of kStepGqWaves waves (4 LDS histogram copies) instead of 4.
// GQ = 2, the fused tick (mdr_greedy_rollout; mdr_kernels.h GqfBufs): the actions are the decision of
// k_gq_decide2 applied here — the pre-step key's bin under the decision's map (parity fpar: the same
// bin the producer counted) below fbs taken, in [fbs, fbe] the house's byte (action = fz.dec), above
// not — and the epilogue is the producer of the next decision (parity 1 - fpar): superbin C and A
// counts (packed C | A << 16 in the LDS copies), the band's C / A bin counts and its houses as window
// entries in their (copy, bin) buckets; no codes are stored
template <int TPW, int ACT, int LA, int GQ>
__global__ void __launch_bounds__(GQ ? 64 * kStepGqWaves : 256) k_step_pipe(KParams p, const uint8_t* __restrict__ action, TickArgs tk0,
                                                   const TickArgs* tkp, const unsigned long long* __restrict__ counts,
                                                   double* __restrict__ reward, double* p_out,
                                                   unsigned long long* next_slab, unsigned long long* zero_slab,
                                                   GqOut gq, GqfBufs fz, int fpar) {
  constexpr int HPT = 2;
  constexpr bool AB = ACT == MDR_ACT_BUFFER;
  __shared__ unsigned hist[MDR_MAX_CAP];
  __shared__ unsigned s_gq[GQ ? 4 * kGqSupStride : 1];
  __shared__ uint32_t s_map[GQ ? kGqCells : 1];
  __shared__ uint32_t s_mapd[GQ == 2 ? kGqCells : 1];  // (GQ 2) the decision's map
  // (GQ 2) the block's band houses: entries, (bin << 16 | rank in the block's bin), per-bin counts and
  // bucket bases — one returning global atomic per non-empty bin at the block's end, not per house
  __shared__ uint4 s_bl[GQ == 2 ? kGqfList : 1];
  __shared__ uint32_t s_blr[GQ == 2 ? kGqfList : 1];
  __shared__ unsigned s_bcnt[GQ == 2 ? kGqBand * 64 : 1];
  __shared__ unsigned s_blen;
  __shared__ unsigned s_acnt[8];  // (GQ 2) the block's A summary
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  if (tid < p.n_cap) hist[tid] = 0;
  int gq_band0 = 0;  // the band's first bin
  unsigned* gq_band = nullptr;  // this block's copy of the band's class counts
  const int npar = 1 - fpar;    // (GQ 2) the parity this epilogue produces
  unsigned* fz_band_a = nullptr;
  unsigned* fz_band_n = nullptr;
  uint4* fz_bkt = nullptr;
  double d_kmin = 0.0, d_scale = 0.0;
  int f_mode = 0, f_bs = 0, f_be = 0;
  if (GQ == 1) {
    for (int e = tid; e < 4 * kGqSupStride; e += blockDim.x) s_gq[e] = 0u;
    for (int e = tid; e < kGqCells; e += blockDim.x) s_map[e] = gq.map[e];
    gq_band0 = gq.sel->band_base * 64;
    gq_band = gq.hist + kGqBandOff + (blockIdx.x % kGqCopies) * kGqBandWords;
  } else if (GQ == 2) {
    for (int e = tid; e < 4 * kGqSupStride; e += blockDim.x) s_gq[e] = 0u;
    for (int e = tid; e < kGqCells; e += blockDim.x) {
      s_map[e] = fz.map[npar][e];
      s_mapd[e] = fz.map[fpar][e];
    }
    for (int e = tid; e < kGqBand * 64; e += blockDim.x) s_bcnt[e] = 0u;
    if (tid == 0) s_blen = 0u;
    if (tid < 8) s_acnt[tid] = 0u;
    gq_band0 = fz.sel->fband[npar] * 64;
    const int cp = (int)(blockIdx.x % kGqCopies);
    gq_band = fz.par[npar] + kGqfOffBandC + cp * kGqBandWords;
    fz_band_a = fz.par[npar] + kGqfOffBandA + cp * kGqBandWords;
    fz_band_n = fz.par[npar] + kGqfOffBandN + cp * (kGqBand * 64);
    fz_bkt = fz.bkt[npar] + (size_t)cp * (kGqBand * 64) * fz.cap;
    d_kmin = fz.sel->fkmin[fpar];
    d_scale = fz.sel->fscale[fpar];
    f_mode = fz.sel->fmode;
    f_bs = fz.sel->fbs;
    f_be = fz.sel->fbe;
  }
  double gq_lo = INFINITY, gq_hi = -INFINITY;
  GqfAcnt gq_a{0u, 0u, 0u, 0u};
  const double gq_kmin = GQ == 1 ? gq.sel->kmin : GQ == 2 ? fz.sel->fkmin[npar] : 0.0;
  const double gq_scale = GQ == 1 ? gq.sel->scale : GQ == 2 ? fz.sel->fscale[npar] : 0.0;
  if (zero_slab && blockIdx.x == 0)
    for (int j = tid; j < kCountShards * p.n_cap; j += blockDim.x) zero_slab[j] = 0ull;
  // GQ (no lookahead): the greedy call that follows counts its decisions into next_slab, and its
  // one-pass form (k_gq_binsc) cannot zero it itself
  if (GQ && !LA && next_slab && blockIdx.x == 0)
    for (int j = tid; j < kCountShards * p.n_cap; j += blockDim.x) next_slab[j] = 0ull;
  const uint32_t n = (uint32_t)p.n;
  const uint32_t ntiles = (n + 64u * HPT - 1u) / (64u * HPT);
  const uint32_t nwaves = gridDim.x * (blockDim.x >> 6);
  const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + (uint32_t)(tid >> 6);

  // the tick's cluster power: this lane's count-slab shard (issued before the first tile's loads,
  // so waiting for it leaves them in flight)
  unsigned long long cnt[kPipeCap];
#pragma unroll
  for (int k = 0; k < kPipeCap; ++k) cnt[k] = counts ? counts[lane * p.n_cap + (k < p.n_cap ? k : 0)] : 0ull;
  // the cooling-capacity tables as uniform scalars (scalar loads: no vmcnt, so a lookup never
  // drains the in-flight tile loads)
  double q_on[kPipeCap];
#pragma unroll
  for (int k = 0; k < kPipeCap; ++k) q_on[k] = p.q_on[k < p.n_cap ? k : 0];
  auto full_tile = [&](uint32_t t) { return (t + 1u) * (64u * HPT) <= n; };
  Tile2 buf[2];
  if (gw < ntiles) load_tile2<AB>(p, action, gw * (64u * HPT) + (uint32_t)lane * HPT, n, full_tile(gw), buf[0]);
  if (LA || GQ) __syncthreads();  // hist zeroed (a bare s_barrier: the tile loads stay in flight)
  const TickArgs tk = tkp ? *tkp : tk0;
  double sig_term = 0.0;
  if (counts) {
    double P = 0.0;
#pragma unroll
    for (int k = 0; k < kPipeCap; ++k)
      if (k < p.n_cap) P += (double)wave_sum_counts(cnt[k]) * p.p_on[k];
    const double x = (P - tk.s_prev) / (double)p.n_global;
    sig_term = p.alpha_sig * (x * x) / p.norm_sig;
    if (p_out && blockIdx.x == 0 && tid == 0) *p_out = P;
  }
  const bool tick_fast = !*p.params_bad && p.fast_tick_ok && fabs(tk.t_od_prev) < 1048576.0 &&
                         fabs(tk.solar) < 1099511627776.0;
  unsigned la_cnt[kPipeCap] = {0u, 0u, 0u, 0u};

#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const uint32_t tile = gw + (uint32_t)k * nwaves;
    if (tile >= ntiles) break;  // wave-uniform
    if (k + 1 < TPW && tile + nwaves < ntiles)
      load_tile2<AB>(p, action, (tile + nwaves) * (64u * HPT) + (uint32_t)lane * HPT, n,
                     full_tile(tile + nwaves), buf[(k + 1) & 1]);
    const Tile2& in = buf[k & 1];
    const uint32_t i0 = tile * (64u * HPT) + (uint32_t)lane * HPT;
    const double T[2] = {in.T.x, in.T.y}, Tm[2] = {in.Tm.x, in.Tm.y}, ua[2] = {in.ua.x, in.ua.y};
    const double ca[2] = {in.ca.x, in.ca.y}, cm[2] = {in.cm.x, in.cm.y}, hm[2] = {in.hm.x, in.hm.y};
    const double tg[2] = {in.tg.x, in.tg.y};
    const uint32_t w0[2] = {in.w.x, in.w.y};
    const int cls[2] = {(int)(in.cls & 0xFF), (int)((in.cls >> 8) & 0xFF)};
    bool valid[2] = {i0 < n, i0 + 1 < n};

    bool rnd[2] = {false, false}, rnd1[2] = {false, false};
    if (ACT == MDR_ACT_RANDOM || LA == MDR_ACT_RANDOM) {
      const WaveRandom wr(p.seed, p.goff + (uint64_t)tile * (64u * HPT), tk.tick);
#pragma unroll
      for (int h = 0; h < HPT; ++h) {
        rnd[h] = wr.get(p.goff + i0 + h, false);
        rnd1[h] = wr.get(p.goff + i0 + h, true);
      }
    }
    bool house_ok = true;
#pragma unroll
    for (int h = 0; h < HPT; ++h) house_ok = house_ok && fabs(T[h]) < 1048576.0 && fabs(Tm[h]) < 1048576.0;
    const bool tile_fast = tick_fast && __all(house_ok);

    double Tn[2], Tmn[2], rw[2];
    uint32_t w[2];
    bool on1[2], act_ap[2];
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      bool a;
      if (GQ == 2) {  // the fused decision (GqSel.fmode; the byte: fz.dec, loaded as the action row)
        const bool byte = ((in.act >> (8 * h)) & 0xFFu) != 0u;
        if (f_mode == kGqfAll) {
          a = true;
        } else if (f_mode == kGqfFull) {
          a = byte;
        } else {
          const double k = -(T[h] - tg[h]);  // gq_key_of, pre-step: the key the decision ordered
          const int b = k != k ? kGqBins : gq_bin(k, d_kmin, d_scale, s_mapd);
          a = b < f_bs || (b <= f_be && byte);
        }
        a = valid[h] && a;
        act_ap[h] = a;
      } else {
        a = valid[h] && (AB ? ((in.act >> (8 * h)) & 0xFFu) != 0u
                            : pick_action(ACT, action, i0 + h, rnd[h], T[h], tg[h], p.deadband, w0[h]));
      }
      w[h] = hvac_fsm(w0[h], a, p.dt, p.L);
      const bool on = hv_on(w[h]);
      double qc = q_on[0];
#pragma unroll
      for (int c = 1; c < kPipeCap; ++c) qc = cls[h] == c ? q_on[c] : qc;
      const double q = on ? qc : 0.0;
      RcCoef kc;
      if (tile_fast) {
        kc = rc_coeffs_t<true>(ua[h], ca[h], cm[h], hm[h], (double)p.dt);
        rc_apply_t<true>(T[h], Tm[h], ua[h], ca[h], hm[h], kc, q, tk.solar, tk.t_od_prev, Tn[h], Tmn[h]);
      } else {
        kc = rc_coeffs_t<false>(ua[h], ca[h], cm[h], hm[h], (double)p.dt);
        rc_apply_t<false>(T[h], Tm[h], ua[h], ca[h], hm[h], kc, q, tk.solar, tk.t_od_prev, Tn[h], Tmn[h]);
      }
      const double tpen = p.alpha_temp * deadband_l2(tg[h], p.deadband, Tn[h]);
      rw[h] = -((p.norm_temp == 1.0 ? tpen : tpen / p.norm_temp) + sig_term);
      on1[h] = false;
      if (LA) {
        bool an;
        if (LA == MDR_ACT_RANDOM) an = rnd1[h];
        else if (LA == MDR_ACT_ALWAYS_ON) an = true;
        else if (LA == kActBangBang) an = ctrl_bangbang(Tn[h], tg[h]);
        else an = ctrl_deadband(Tn[h], tg[h], p.deadband, on);
        on1[h] = valid[h] && hv_on(hvac_fsm(w[h], an, p.dt, p.L));
      }
    }
    if (GQ == 2 && gq.act_out) {  // (the fused tick: the applied actions, when the caller keeps them)
      if (valid[1] && ((uintptr_t)gq.act_out & 1u) == 0u) {
        sto(gq.act_out, i0, (unsigned short)((act_ap[0] ? 1u : 0u) | (act_ap[1] ? 256u : 0u)));
      } else {  // (an odd row start: per-tick rows of an odd cluster size)
        if (valid[0]) gq.act_out[i0] = act_ap[0] ? 1 : 0;
        if (valid[1]) gq.act_out[i0 + 1] = act_ap[1] ? 1 : 0;
      }
    }
    if (valid[1]) {
      const uint32_t o8 = i0 * 8u;
      sto(p.t_air, o8, make_double2(Tn[0], Tn[1]));
      sto(p.t_mass, o8, make_double2(Tmn[0], Tmn[1]));
      sto(p.hvac, i0 * 4u, make_uint2(w[0], w[1]));
      if (counts) sto_nt(reward, o8, make_double2(rw[0], rw[1]));
    } else if (valid[0]) {
      p.t_air[i0] = Tn[0]; p.t_mass[i0] = Tmn[0]; p.hvac[i0] = w[0];
      if (counts) __builtin_nontemporal_store(rw[0], reward + i0);
    }
    if (GQ == 2) {  // the next decision's producer (gq_key_of of the post-step state)
      const uint32_t Lu = p.L < 0 ? 0u : (uint32_t)p.L;
#pragma unroll
      for (int h = 0; h < HPT; ++h) {
        const double k = -(Tn[h] - tg[h]);
        const uint32_t c = gq_code(k, gq_kmin, gq_scale, s_map, (unsigned)cls[h]);
        if (valid[h] && k == k) {
          gq_lo = fmin(gq_lo, k);
          gq_hi = fmax(gq_hi, k);
        }
        // A: the house can turn on at the next step (hvac_fsm: not locked out)
        const bool canon = hv_on(w[h]) || hv_sso(w[h]) + (uint32_t)p.dt >= Lu;
        if (valid[h]) atomicAdd(&s_gq[((tid >> 6) & 3) * kGqSupStride + (c >> 8) * 4 + (c & 3u)], 1u);
        gqf_acount(gq_a, valid[h] && canon, (c >> 2) < (uint32_t)gq_band0, c & 3u);
        const uint32_t bo = (c >> 2) - (uint32_t)gq_band0;
        const bool inb = valid[h] && bo < (uint32_t)(kGqBand * 64);
        // the list slots: one LDS atomic per wave (same-address LDS atomics serialise), then by lane rank
        const unsigned long long m = __ballot(inb);
        unsigned lbase = 0u;
        if (m) {  // (wave-uniform)
          const int lead = __ffsll((long long)m) - 1;
          if (lane == lead) lbase = atomicAdd(&s_blen, (unsigned)__popcll(m));
          lbase = __shfl(lbase, lead);
        }
        if (inb) {
          atomicAdd(&gq_band[bo * 4 + (c & 3u)], 1u);
          if (canon) atomicAdd(&fz_band_a[bo * 4 + (c & 3u)], 1u);
          const unsigned li = lbase + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
          const unsigned lr = atomicAdd(&s_bcnt[bo], 1u);  // (LDS)
          const uint64_t ok = gq_okey(k);
          if (li < (unsigned)kGqfList) {
            s_bl[li] = make_uint4((uint32_t)ok, (uint32_t)(ok >> 32), (uint32_t)((p.goff + i0 + h) << 2) | (c & 3u), w[h]);
            s_blr[li] = (bo << 16) | lr;
          }
        }
      }
    }
    if (GQ == 1) {  // greedy_myopic_controller.py:79 on the post-step state (gq_key_of)
      const double k0 = -(Tn[0] - tg[0]), k1 = -(Tn[1] - tg[1]);
      const uint32_t c0 = gq_code(k0, gq_kmin, gq_scale, s_map, (unsigned)cls[0]);
      const uint32_t c1 = gq_code(k1, gq_kmin, gq_scale, s_map, (unsigned)cls[1]);
      if (valid[1]) sto(gq.code, i0 * 4u, make_uint2(c0, c1));
      else if (valid[0]) gq.code[i0] = c0;
#pragma unroll
      for (int h = 0; h < HPT; ++h) {
        const double k = h ? k1 : k0;
        if (!valid[h]) continue;
        if (k == k) {
          gq_lo = fmin(gq_lo, k);
          gq_hi = fmax(gq_hi, k);
        }
        const uint32_t c = h ? c1 : c0;
        atomicAdd(&s_gq[((tid >> 6) & 3) * kGqSupStride + (c >> 8) * 4 + (c & 3u)], 1u);
        // the band's houses (~kGqBand / kGqSuper of them) add to the global copy at once: a few lanes
        // per wave-instruction, issued inside the HBM-bound loop instead of a flush at the blocks'
        // common end (NaN keys: bin kGqBins, past any band)
        const uint32_t bo = (c >> 2) - (uint32_t)gq_band0;
        if (bo < (uint32_t)(kGqBand * 64)) atomicAdd(&gq_band[bo * 4 + (c & 3u)], 1u);
      }
    }
    if (LA) {
#pragma unroll
      for (int c = 0; c < kPipeCap; ++c)
        if (c < p.n_cap)
          la_cnt[c] += (unsigned)__popcll(__ballot(on1[0] && cls[0] == c)) +
                       (unsigned)__popcll(__ballot(on1[1] && cls[1] == c));
    }
  }
  if (LA) {
    if (lane == 0) {
#pragma unroll
      for (int c = 0; c < kPipeCap; ++c)
        if (c < p.n_cap && la_cnt[c]) atomicAdd(&hist[c], la_cnt[c]);
    }
    __syncthreads();
    if (tid < p.n_cap && hist[tid])
      atomicAdd(&next_slab[(blockIdx.x % kCountShards) * p.n_cap + tid], (unsigned long long)hist[tid]);
  }
  if (GQ == 1) {
    __syncthreads();
    gq_flush(s_gq, 4, gq.hist, gq_lo, gq_hi, gq.part);
    if (blockIdx.x == 0 && threadIdx.x == 0) gq.sel->band_valid = 1;
  } else if (GQ == 2) {
    gqf_acount_wave(gq_a, s_acnt);
    __syncthreads();
    // the band houses into their buckets: a base per non-empty bin (one returning atomic each, in
    // parallel), then each house at base + its rank in the block's bin
    if (s_blen > (unsigned)kGqfList && tid == 0) atomicOr(&fz.par[npar][kGqfOffFlags], 1u);
    // (the returning atomics' latency overlaps the flush: their values go to LDS after it)
    static_assert(kGqBand * 64 <= 64 * kStepGqWaves, "a thread per band bin");
    unsigned bbase = 0u;
    if (tid < kGqBand * 64 && s_bcnt[tid]) bbase = atomicAdd(&fz_band_n[tid], s_bcnt[tid]);
    gqf_flush(s_gq, 4, fz.par[npar], gq_lo, gq_hi, gq.part, s_acnt);
    unsigned* s_bbase = s_bcnt;  // (in place: each thread owns its bin's entry)
    if (tid < kGqBand * 64) s_bbase[tid] = bbase;
    __syncthreads();
    const unsigned nl = s_blen < (unsigned)kGqfList ? s_blen : (unsigned)kGqfList;
    for (unsigned e = tid; e < nl; e += blockDim.x) {
      const uint32_t br = s_blr[e], bo = br >> 16;
      const unsigned slot = s_bbase[bo] + (br & 0xFFFFu);
      if (slot < (unsigned)fz.cap) fz_bkt[(size_t)bo * fz.cap + slot] = s_bl[e];
      else atomicOr(&fz.par[npar][kGqfOffFlags], 1u);  // (a full bucket: the band is not usable)
    }
  }
}

// --------------------------------------------------------------------------------------- K1W
// Temporally blocked step for OPEN-LOOP action sources (random / always-on / action buffer), the
// rollout path: one launch steps a window of K <= 32 ticks.  Each wave loads its tile's state and
// parameters ONCE, keeps them in registers for the K ticks, and writes the state back once; per
// tick it writes only the reward row.  What makes it exact:
//   * an open-loop source's actions do not depend on the thermal state, so the lockout FSM — and
//     with it every tick's ON set and cluster power P(t) — can be run ahead of the thermal
//     update.  The launch of window w runs the FSM through window w+1 (the "lookahead"): it
//     counts window w+1's per-tick ON houses per capacity class (so each tick's reward has its
//     GLOBAL P(t) when the next launch starts: the same integer counts as the one-tick kernels,
//     bit-identical P), stores the per-tick ON lane masks and the FSM word at the end of window
//     w+1.  The next launch's thermal loop then needs no FSM at all: a tick's heat source is
//     selected by its stored ON mask;
//   * the lookahead keeps the FSM's booleans as wave lane masks (SALU logic) and the random
//     actions as lane masks built from the Philox words of the wave's 64-house groups, so a
//     house-tick of lookahead costs four vector ops;
//   * the parameter-only part of the RC update (roots r1/r2, A3/A4, exp(r dt) and the shared
//     reciprocals of Ca, Ua and r2-r1) is computed once per window, not once per tick — the same
//     expressions in the same order (rc_coeffs_t / recip), so results are bit-identical to the
//     one-tick kernels, which recompute them every tick;
//   * per tick, the record {t_od_prev + 273, solar, signal penalty, range flag} is computed once
//     by k_win_reduce (from the reduced counts) and read by the thermal loop with scalar loads.
// Houses of a wave tile: 64 * HPT consecutive ids, house h of lane l = tile * 64 * HPT + 64 h + l
// (coalesced 8-B accesses; lane l of house slot h is bit l of that slot's lane masks).
constexpr int kWinMax = 32;    // ticks per window launch (and per lookahead)
constexpr int kWinCap = 4;     // capacity classes held in registers
constexpr int kWinRec = 4;     // doubles per tick record

// Per-window thermal constants of one house (FAST path: shared reciprocals).
struct RcWin {
  RcCoef k;
  Recip rCa, rc, rd;  // 1/Ca, 1/Ua (= 1/c), 1/(r2 - r1)
  double UaHm;
};

__device__ __forceinline__ RcWin rc_window(double ua, double ca, double cm, double hm, double dt) {
  RcWin w;
  w.k = rc_coeffs_t<true>(ua, ca, cm, hm, dt);
  w.rCa = recip(ca);
  w.rc = recip(ua);
  w.rd = recip(w.k.r2 - w.k.r1);
  w.UaHm = ua + hm;
  return w;
}

// rc_apply_t<FAST> with the window's reciprocals (identical operations and order); od_k =
// t_od_prev + 273.0 is a per-tick scalar the caller computes once per window lane
template <bool FAST>
__device__ __forceinline__ void rc_apply_win(double T, double Tm, double Ua, double Hm, const RcWin& w,
                                             double q_hvac, double solar, double od_k, double& T_out,
                                             double& Tm_out) {
  const RcCoef& k = w.k;
  const double t_k = T + 273.0;
  const double tm_k = Tm + 273.0;
  const double Qa = q_hvac + solar;
  const double d = Qa + Ua * od_k;
  double dTA0dt, d_c, r2d_c, A1;
  if (FAST) {
    dTA0dt = div_by(Hm * tm_k, w.rCa) - div_by(w.UaHm * t_k, w.rCa) + div_by(Ua * od_k, w.rCa) +
             div_by(Qa, w.rCa);
    d_c = div_by(d, w.rc);
    r2d_c = div_by(k.r2 * d, w.rc);
    A1 = div_by(k.r2 * t_k - dTA0dt - r2d_c, w.rd);
  } else {
    const double Ca = -w.rCa.nb, c = -w.rc.nb;  // (exact negations of the stored -b)
    dTA0dt = Hm * tm_k / Ca - w.UaHm * t_k / Ca + Ua * od_k / Ca + Qa / Ca;
    d_c = d / c;
    r2d_c = k.r2 * d / c;
    A1 = (k.r2 * t_k - dTA0dt - r2d_c) / -w.rd.nb;
  }
  const double A2 = t_k - d_c - A1;
  const double t_new = A1 * k.e1 + A2 * k.e2 + d_c;
  const double tm_new = A1 * k.A3 * k.e1 + A2 * k.A4 * k.e2 + d_c;  // (+ g = 0.0 elided: mdr_device.h)
  T_out = t_new - 273.0;
  Tm_out = tm_new - 273.0;
}

static_assert(kCountShards == 64, "k_win_reduce reduces the shards with one wave");

// Window count slot (u64 units): [slab: kWinMax][kCountShards][n_cap] | [red: kWinMax][n_cap] |
// [rec: kWinMax][kWinRec] (double).  Producers accumulate block histograms into the sharded slab;
// k_win_reduce (the next graph node: the kernel boundary makes every producer atomic visible) sums
// the shards into red, zeroes the shards for the slot's next use, and writes the tick records; the
// first window's P-only reduce runs instead in k_count_window's last block (win_reduce_last: the
// shard adds are 8-B agent-scope atomics, so the hand-off needs no L2 write-back fence).
__device__ __forceinline__ unsigned long long* win_red(unsigned long long* slot, int n_cap) {
  return slot + (size_t)kWinMax * kCountShards * n_cap;
}
__device__ __forceinline__ double* win_rec(unsigned long long* slot, int n_cap) {
  return reinterpret_cast<double*>(win_red(slot, n_cap) + (size_t)kWinMax * n_cap);
}

// tick record j from the tick's global class counts (rewards_calculator.py:183-203 signal part;
// the operations and order of the one-tick kernels); rec[2] is the NEGATED signal penalty (an exact
// negation: the reward is then formed without a sign flip, k_step_window)
// P = sum over classes of count * p_on, in the one-tick kernels' order (cluster.py:73-89)
__device__ __forceinline__ double win_power(const KParams& p, const unsigned long long* cnt, const double* p_on) {
  double P = 0.0;
#pragma unroll
  for (int k = 0; k < kWinCap; ++k)
    if (k < p.n_cap) P += (double)cnt[k] * p_on[k];
  return P;
}

// the negated signal penalty of a tick with cluster power P (rewards_calculator.py:183-203)
__device__ __forceinline__ double win_nsig(const KParams& p, double P, double s_prev) {
  const double x = (P - s_prev) / (double)p.n_global;
  return -(p.alpha_sig * (x * x) / p.norm_sig);
}

__device__ __forceinline__ void win_tick_record(const KParams& p, const unsigned long long* cnt, const TickArgs& tk,
                                                const double* p_on, double* rec, double* p_out) {
  const double P = win_power(p, cnt, p_on);
  rec[0] = tk.t_od_prev + 273.0;  // rc_apply's od_k
  rec[1] = tk.solar;
  rec[2] = win_nsig(p, P, tk.s_prev);
  rec[3] = fabs(tk.t_od_prev) < 1048576.0 && fabs(tk.solar) < 1099511627776.0 ? 1.0 : 0.0;  // fast-division ranges
  if (p_out) *p_out = P;
}

// one block per tick j, one wave per class: sum the 64 shards (sharded rollouts: already summed
// over ranks by the allreduce), zero them, and write the tick record.  tk_j: the tick's drivers,
// read by thread 0 only (win_reduce_body is shared by the two reduce kernels below)
__device__ __forceinline__ void win_reduce_body(const KParams& p, unsigned long long* __restrict__ slot, int nt,
                                                const TickArgs* tk_j, double* p_out) {
  __shared__ unsigned long long s_red[kWinCap];
  const int j = blockIdx.x, c = threadIdx.x >> 6, q = threadIdx.x & 63, ncap = p.n_cap;
  // the record's other inputs are loaded by thread 0 while the shards are read (one memory
  // round trip instead of three dependent ones)
  TickArgs tk{};
  double p_on[kWinCap];
  if (threadIdx.x == 0) {
    if (tk_j) tk = *tk_j;
#pragma unroll
    for (int k = 0; k < kWinCap; ++k) p_on[k] = p.p_on[k < ncap ? k : 0];
  }
  unsigned long long v = 0;
  if (c < ncap) {
    unsigned long long* e = &slot[((size_t)j * kCountShards + q) * ncap + c];
    v = *e;
    *e = 0ull;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if (q == 0 && c < ncap) {
    win_red(slot, ncap)[j * ncap + c] = v;
    s_red[c] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (tk_j) {
      win_tick_record(p, s_red, tk, p_on, win_rec(slot, ncap) + j * kWinRec, j == nt - 1 ? p_out : nullptr);
    } else {  // P only (the drivers come later, as kernel arguments of k_step_window<..., KA>)
      win_rec(slot, ncap)[j * kWinRec] = win_power(p, s_red, p_on);
    }
  }
}

__global__ void __launch_bounds__(256) k_win_reduce(KParams p, unsigned long long* __restrict__ slot, int nt,
                                                    const TickArgs* __restrict__ tkp, double* p_out) {
  win_reduce_body(p, slot, nt, tkp ? tkp + blockIdx.x : nullptr, p_out);
}

// Sharded windows: the tick records from the slot's reduced counts `red` once they hold the
// cluster's totals (every rank's count kernel reduced its own shards in its last block, then one
// sum-allreduce of the K x n_cap totals): thread j writes tick j's record (tkp: the full record;
// null: P only, the drivers come later as kernel arguments).  One block of kWinMax threads.
__global__ void __launch_bounds__(kWinMax) k_win_records(KParams p, unsigned long long* __restrict__ slot, int nt,
                                                         const TickArgs* __restrict__ tkp, double* p_out) {
  const int j = threadIdx.x, ncap = p.n_cap;
  if (j >= nt) return;
  double p_on[kWinCap];
#pragma unroll
  for (int k = 0; k < kWinCap; ++k) p_on[k] = p.p_on[k < ncap ? k : 0];
  const unsigned long long* cnt = win_red(slot, ncap) + j * ncap;
  double* rec = win_rec(slot, ncap) + j * kWinRec;
  if (tkp) win_tick_record(p, cnt, tkp[j], p_on, rec, j == nt - 1 ? p_out : nullptr);
  else rec[0] = win_power(p, cnt, p_on);
}

// LDS written by some lanes of a wave and read by others (the wave's LDS operations execute in
// issue order: a wavefront-scope fence orders the compiler and waits lgkmcnt)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// True in exactly one block of the grid: the last to arrive, after every block's earlier vector
// memory operations have completed (each wave drains them, vmcnt(0), before the workgroup barrier).
// Two-level ticket: block b adds to the counter of group b % G (G = min(grid, kTicketGroups), each
// counter on its own 128-B line), the group's last arrival adds to one top counter, and the top's
// last arrival is the answer; every counter is reset by the block that saw it complete.  (One
// counter for a 2048-block grid serialises 2048 same-address atomics: ~25 us on MI355X.)
// tickets: (kTicketGroups + 1) x 32 words, zero between launches.
__device__ bool grid_last_block(unsigned* __restrict__ tickets) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned G = gridDim.x < (unsigned)kTicketGroups ? gridDim.x : (unsigned)kTicketGroups;
    const unsigned g = blockIdx.x % G;
    const unsigned gsize = (gridDim.x - g + G - 1) / G;
    unsigned last = 0u;
    if (__hip_atomic_fetch_add(&tickets[32 * g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1u) {
      __hip_atomic_store(&tickets[32 * g], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned* top = &tickets[32 * kTicketGroups];
      if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1u) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = 1u;
      }
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0u;
}

// The P-only reduce of a counted window by the count kernel's LAST block, in place of a k_win_reduce
// launch (single GPU: no allreduce sits between the count and the reduce).  Hand-off per
// cdna_hip_programming.md Guideline 16 / MI355X_MICROARCH.md Valid forms ("8-B agent atomics both
// sides"): every block's shard adds (win_flush) are 8-B agent-scope atomics, drained by each wave
// (vmcnt(0)) before the workgroup barrier and the block's agent-scope ticket add (grid_last_block);
// the last block reads the shards only with 8-B agent-scope (sc1) loads.  Thread t takes shard
// t % 16 of entries (tick, class) e = t / 16 + 16 k: every load issued first (one round trip), the
// 16 shards of an entry summed across a 16-lane group (shuffles), the shards zeroed behind.
template <int NTH>
__device__ void win_reduce_last(const KParams& p, unsigned long long* __restrict__ slot, int nt,
                                unsigned* __restrict__ ticket) {
  static_assert(kWinShards == 16, "one 16-lane group per entry");
  constexpr int EPT = kWinMax * kWinCap * kWinShards / NTH;  // loads per thread (blockDim NTH)
  constexpr int EPK = NTH / 16;                               // entries per k
  __shared__ unsigned long long s_red[kWinMax * kWinCap];
  if (!grid_last_block(ticket)) return;  // (block-uniform)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler ordering only: the loads below are sc1)
  const int ncap = p.n_cap, E = nt * ncap, sh = threadIdx.x & 15;
  unsigned long long v[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = (int)(threadIdx.x >> 4) + EPK * k;
    v[k] = 0ull;
    if (e < E) {
      const int j = e / ncap, c = e - j * ncap;
      v[k] = __hip_atomic_load(&slot[((size_t)j * kCountShards + sh) * ncap + c], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int e = (int)(threadIdx.x >> 4) + EPK * k;
    if (e < E) {  // (the slot's next count adds into zeros)
      const int j = e / ncap, c = e - j * ncap;
      __hip_atomic_store(&slot[((size_t)j * kCountShards + sh) * ncap + c], 0ull, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned long long x = v[k];
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if (sh == 0 && e < E) s_red[e] = x;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += blockDim.x) win_red(slot, ncap)[e] = s_red[e];
  if ((int)threadIdx.x < nt) {
    double p_on[kWinCap];
#pragma unroll
    for (int k = 0; k < kWinCap; ++k) p_on[k] = p.p_on[k < ncap ? k : 0];
    win_rec(slot, ncap)[threadIdx.x * kWinRec] = win_power(p, s_red + threadIdx.x * ncap, p_on);
  }
}

// the wave tile: 64 * HPT consecutive houses, house slot h of lane l = i0 + 64 h
template <int HPT>
struct WinTile {
  uint32_t tile, i0;
  uint32_t idx[HPT];  // the lane's house per slot, clamped to n - 1 for loads
  bool v[HPT];
  uint64_t g0;        // first 64-house group of global ids the tile touches
  int sh;             // global id of the tile's first house mod 64 (0 when the shard offset is aligned)
  __device__ __forceinline__ WinTile(const KParams& p) {
    const uint32_t n = (uint32_t)p.n;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    tile = blockIdx.x * (blockDim.x >> 6) + wv;
    i0 = tile * (64u * HPT) + (uint32_t)(threadIdx.x & 63);
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      const uint32_t i = i0 + 64u * h;
      v[h] = i < n;
      idx[h] = v[h] ? i : n - 1u;
    }
    const uint64_t gbase = (uint64_t)p.goff + (uint64_t)tile * (64u * HPT);
    g0 = gbase >> 6;
    sh = (int)(gbase & 63u);
  }
};

__device__ __forceinline__ uint64_t readlane_u64(uint32_t lo, uint32_t hi, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, l) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, l);
}

// lane `lane` of a VGPR set to the wave-uniform val (v_writelane_b32: val in an SGPR, the lane
// select in M0, which does not count against the one-SGPR constant-bus limit of gfx950)
__device__ __forceinline__ uint32_t writelane_u32(uint32_t old, uint32_t val, int lane) {
  uint32_t r;
  asm("v_writelane_b32 %0, %1, m0" : "=v"(r) : "s"(val), "{m0}"(lane), "0"(old));
  return r;
}

// FSM-only run of nt <= kWinMax ticks (HVAC.step, hvac.py:43-64; the transitions of hvac_fsm) from
// the words w[h]; tkp / action: the run's first tick.  The booleans (on, can, action) are wave lane
// masks carried in scalar registers.  The seconds-since-off are carried in a per-house offset form:
// s1_j (the seconds-since-off at tick j after its "if not on: sso += dt") = c + j dt, with c constant
// while the house stays off and c = -(j + 1) dt when it is ON at tick j (so s1_{j+1} = 0).  A tick is
// then one compare of c against the wave-uniform L - j dt (straight into a lane mask) and one select
// of the wave-uniform -(j + 1) dt — no per-house add.  Tick j's ON masks are written into lane j of
// per-wave VGPRs (v_writelane); at the end lane t counts tick t's ON houses per capacity class into
// cnt[t][kWinCap], stores the masks to onb[t][HPT] (this wave's rows, read by the next window's
// thermal loop) and w[h] becomes the FSM word after the run.  Transitions use the unsaturated
// seconds-since-off (window_ok guarantees L < 2^30 and sso + (kWinMax + 1) dt < 2^31, dt < 2^25, so
// c and L - j dt fit a signed 32-bit compare), so saturating once at the end gives the
// per-tick-saturated value; the lock bit comes from the last tick.  SH: the tile starts off a
// 64-house group boundary (sharded runs), so a random action mask is spliced from two words.
template <int ACT, int HPT, bool SH>
__device__ __forceinline__ void win_run_t(const KParams& p, uint32_t* w, const uint64_t (*cm)[kWinCap],
                                          const WinTile<HPT>& t, const TickArgs* tkp, uint64_t tick0, int nt,
                                          const uint8_t* action, int64_t act_stride, unsigned* cnt, uint64_t* onb) {
  const int lane = threadIdx.x & 63;
  const int Li = p.L < 0 ? 0 : p.L, dt = p.dt;
  uint64_t on_m[HPT], can_m[HPT];
  int32_t c[HPT];
  uint32_t mlo[HPT], mhi[HPT];
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    on_m[h] = __ballot((w[h] & kOnBit) != 0);
    const int32_t sso = (int32_t)(w[h] & kSsoMask);
    c[h] = __builtin_amdgcn_inverse_ballot_w64(on_m[h]) ? sso : sso + dt;  // s1_0: if not on, sso += dt
    can_m[h] = 0ull;
    mlo[h] = mhi[h] = 0u;
  }
  // Philox words of the run's ticks (random controller, mdr_device.h philox_words): lane l holds
  // tick (l & 31) of group g0 + (l >> 5); lanes 0..31 of the second pair: group g0 + 2 (a tile of
  // 128 houses off a 64-house boundary spans three groups)
  uint32_t wa_lo = 0, wa_hi = 0, wb_lo = 0, wb_hi = 0;
  constexpr int G = HPT + (SH ? 1 : 0);
  if (ACT == MDR_ACT_RANDOM) {
    const int jj = lane & 31;  // (tick ids: the staged drivers', or consecutive from tick0 before staging)
    const uint64_t tick = tkp ? tkp[jj < nt ? jj : 0].tick : tick0 + (uint64_t)(jj < nt ? jj : 0);
    philox_words(p.seed, t.g0 + (uint64_t)(lane >> 5), tick, wa_lo, wa_hi);
    if constexpr (G > 2) philox_words(p.seed, t.g0 + 2u, tick, wb_lo, wb_hi);
  }
  for (int j = 0; j < nt; ++j) {
    uint64_t W[G];
    if (ACT == MDR_ACT_RANDOM) {
      W[0] = readlane_u64(wa_lo, wa_hi, j);
      if constexpr (G > 1) W[1] = readlane_u64(wa_lo, wa_hi, j + 32);
      if constexpr (G > 2) W[2] = readlane_u64(wb_lo, wb_hi, j);
    }
    const uint8_t* arow = ACT == MDR_ACT_BUFFER ? action + (int64_t)j * act_stride : nullptr;
    const int32_t thr = Li - j * dt;        // s1_j >= L  <=>  c >= L - j dt
    const int32_t c_on = -(j + 1) * dt;     // ON at tick j: s1_{j+1} = 0
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      uint64_t a;  // the actions as a lane mask
      if (ACT == MDR_ACT_RANDOM) a = SH ? (W[h] >> t.sh) | (W[h + 1] << (64 - t.sh)) : W[h];
      else if (ACT == MDR_ACT_ALWAYS_ON) a = ~0ull;
      else a = __ballot(arow[t.idx[h]] != 0);
      can_m[h] = on_m[h] | __ballot(c[h] >= thr);  // not locked
      on_m[h] = can_m[h] & a;
      c[h] = __builtin_amdgcn_inverse_ballot_w64(on_m[h]) ? c_on : c[h];
      mlo[h] = writelane_u32(mlo[h], (uint32_t)on_m[h], j);
      mhi[h] = writelane_u32(mhi[h], (uint32_t)(on_m[h] >> 32), j);
    }
  }
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    // the last tick's lockout (hvac.py:58-63): locked before the decision, or turned off with too
    // little time to finish the lockout (s1_nt = c + nt dt < L); its seconds-since-off: 0 if turned
    // on, else the last tick's s1 = c + (nt - 1) dt
    const bool on = __builtin_amdgcn_inverse_ballot_w64(on_m[h]);
    const uint64_t lock_m = nt > 0 ? ~can_m[h] | (~on_m[h] & __ballot(c[h] < Li - nt * dt)) : 0ull;
    const uint32_t sso = nt > 0 ? (on ? 0u : (uint32_t)(c[h] + (nt - 1) * dt)) : w[h] & kSsoMask;
    const uint32_t s = sso < kSsoMask ? sso : kSsoMask;
    w[h] = s | (__builtin_amdgcn_inverse_ballot_w64(lock_m) ? kLockBit : 0u) | (on ? kOnBit : 0u);
  }
  if (lane < nt) {
    unsigned k[kWinCap] = {};
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      const uint64_t m = ((uint64_t)mhi[h] << 32) | mlo[h];
      onb[lane * HPT + h] = m;
#pragma unroll
      for (int cc = 0; cc < kWinCap; ++cc) k[cc] += (unsigned)__popcll(m & cm[h][cc]);
    }
#pragma unroll
    for (int cc = 0; cc < kWinCap; ++cc) cnt[lane * kWinCap + cc] = k[cc];
  }
}

template <int ACT, int HPT>
__device__ __forceinline__ void win_run(const KParams& p, uint32_t* w, const uint64_t (*cm)[kWinCap],
                                        const WinTile<HPT>& t, const TickArgs* tkp, uint64_t tick0, int nt,
                                        const uint8_t* action, int64_t act_stride, unsigned* cnt, uint64_t* onb) {
  if (ACT == MDR_ACT_RANDOM && t.sh != 0)
    win_run_t<ACT, HPT, true>(p, w, cm, t, tkp, tick0, nt, action, act_stride, cnt, onb);
  else
    win_run_t<ACT, HPT, false>(p, w, cm, t, tkp, tick0, nt, action, act_stride, cnt, onb);
}

// sum the block's per-wave rows cnt[R][kWinMax][kWinCap] and add them to this block's slab shard
template <int R = 4>
__device__ __forceinline__ void win_flush(const KParams& p, int nt, const unsigned (*cnt)[kWinMax * kWinCap],
                                          unsigned long long* slot) {
  const int ncap = p.n_cap;
  for (int e = threadIdx.x; e < nt * ncap; e += blockDim.x) {
    const int j = e / ncap, c = e - j * ncap;
    unsigned v = 0u;
#pragma unroll
    for (int r = 0; r < R; ++r) v += cnt[r][j * kWinCap + c];
    if (v) atomicAdd(&slot[((size_t)j * kCountShards + blockIdx.x % kWinShards) * ncap + c],
                     (unsigned long long)v);
  }
}

// class membership lane masks of the tile (valid houses only)
template <int HPT>
__device__ __forceinline__ void win_classes(const WinTile<HPT>& t, const int* cls, uint64_t (*cm)[kWinCap]) {
#pragma unroll
  for (int h = 0; h < HPT; ++h)
#pragma unroll
    for (int c = 0; c < kWinCap; ++c) cm[h][c] = __ballot(t.v[h] && cls[h] == c);
}



// First window of a rollout: ON counts, ON lane masks and end-of-window FSM words of ticks
// 0 .. nt-1 from the current state (hvac itself is not changed).  Tick ids from the staged drivers,
// or tick0 + t when tkp is null (mdr_rollout_begin: launched before the host computes the drivers).
template <int ACT, int HPT>
__global__ void __launch_bounds__(64 * kCountWaves) k_count_window(KParams p, const uint8_t* __restrict__ action,
                                                      int64_t act_stride, const TickArgs* __restrict__ tkp,
                                                      uint64_t tick0, int nt, unsigned long long* __restrict__ slot,
                                                      uint64_t* __restrict__ onb, uint32_t* __restrict__ wah,
                                                      const uint32_t* __restrict__ w_in, unsigned* __restrict__ ticket) {
  __shared__ unsigned s_cnt[kCountWaves][kWinMax * kWinCap];
  const int wv = threadIdx.x >> 6;
  const WinTile<HPT> t(p);
  uint32_t w[HPT];
  int cls[HPT];
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    w[h] = w_in ? w_in[t.idx[h]] : p.hvac[t.idx[h]];
    cls[h] = p.cap_idx[t.idx[h]];
  }
  uint64_t cm[HPT][kWinCap];
  win_classes<HPT>(t, cls, cm);
  win_run<ACT, HPT>(p, w, cm, t, tkp, tick0, nt, action, act_stride, s_cnt[wv],
                    onb + (size_t)t.tile * HPT * kWinMax);
#pragma unroll
  for (int h = 0; h < HPT; ++h)
    if (t.v[h]) wah[t.i0 + 64u * h] = w[h];
  __syncthreads();
  win_flush<kCountWaves>(p, nt, s_cnt, slot);
  if (ticket) win_reduce_last<64 * kCountWaves>(p, slot, nt, ticket);  // (ticket: the P-only reduce, see win_reduce_last)
}

// Per-window affine transition of one house (FORM = MDR_THERMAL_AFFINE).  The reference's update
// (building.py:141-222) is LINEAR in (t_k, tm_k, Qa, od_k) for fixed parameters: with
// D = r2 - r1, dTA0dt = (Hm tm_k - (Ua+Hm) t_k + Ua od_k + Qa) / Ca and d/c = Qa / Ua + od_k,
//   A1     = a_t t_k + a_m tm_k + a_q Qa + a_o od_k
//            a_t = (r2 + (Ua+Hm)/Ca) / D, a_m = -(Hm/Ca) / D, a_q = -(1/Ca + r2/Ua) / D,
//            a_o = -(Ua/Ca + r2) / D
//   t_new  = A1 (e1 - e2) + e2 t_k + (d/c)(1 - e2)
//   tm_new = A1 (A3 e1 - A4 e2) + A4 e2 t_k + (d/c)(1 - A4 e2)
// so one tick is t_new = tt t_k + tm tm_k + tq Qa + to od_k (and the same for tm_new), four FMAs
// per temperature, with the coefficients formed ONCE per window from the reference's own roots,
// ratios and decay factors (rc_coeffs_t, bit-identical to the exact path's).  Same mathematics,
// another rounding sequence: ~1e-13 K per tick against the reference order, far inside the
// north star's 1e-5 (tests/test_window_gpu.py bounds it over 2,000 ticks).  Heat when ON is folded
// in: qt = tq * q_on(class), so Qa = on ? q_on + solar : solar costs one select.
struct AffWin {
  double tt, tm, tq, to, qt;  // air:  t_new  = tt t_k + tm tm_k + tq solar + to od_k + (on ? qt : 0)
  double mt, mm, mq, mo, qm;  // mass: tm_new = mt t_k + mm tm_k + mq solar + mo od_k + (on ? qm : 0)
};

__device__ __forceinline__ AffWin aff_window(double ua, double ca, double cm, double hm, double dt, double qc,
                                             bool fast) {
  const RcCoef k = fast ? rc_coeffs_t<true>(ua, ca, cm, hm, dt) : rc_coeffs_t<false>(ua, ca, cm, hm, dt);
  const double iD = 1.0 / (k.r2 - k.r1), iCa = 1.0 / ca, iUa = 1.0 / ua;
  const double a_t = (k.r2 + (ua + hm) * iCa) * iD;
  const double a_m = -(hm * iCa) * iD;
  const double a_q = -(iCa + k.r2 * iUa) * iD;
  const double a_o = -(ua * iCa + k.r2) * iD;
  const double E = k.e1 - k.e2, F = k.A3 * k.e1 - k.A4 * k.e2, G = k.A4 * k.e2;
  const double one_e2 = 1.0 - k.e2, one_G = 1.0 - G;
  AffWin w;
  w.tt = a_t * E + k.e2;
  w.tm = a_m * E;
  w.tq = a_q * E + one_e2 * iUa;
  w.to = a_o * E + one_e2;
  w.mt = a_t * F + G;
  w.mm = a_m * F;
  w.mq = a_q * F + one_G * iUa;
  w.mo = a_o * F + one_G;
  w.qt = w.tq * qc;
  w.qm = w.mq * qc;
  return w;
}

// One window of K ticks.  slot: this window's slot (red counts are folded into its tick records);
// onb / wah: the window's ON lane masks and end-of-window FSM words (from k_count_window or the
// previous launch's lookahead), replaced by the next window's when la_K > 0: then the FSM runs on
// through the next la_K ticks (tkp[K..K+la_K), action rows K..) and counts them into next_slot.
// KA (the first window of a directly launched rollout): the tick drivers come as kernel arguments
// (dv) and rec holds only each tick's P (the P-only k_win_reduce); lane j derives tick j's signal
// penalty once (win_nsig, the reduce's expression) and the thermal loop reads it with v_readlane.
// FORM: MDR_THERMAL_EXACT runs the reference's expression per tick (rc_apply_win: bit-identical to
// the one-tick kernels); MDR_THERMAL_AFFINE the per-window transition above (Kelvin state kept in
// registers for the window).
template <int ACT, int HPT, bool SIMPLE, bool KA, int FORM>
__global__ void __launch_bounds__(256) k_step_window(KParams p, const uint8_t* __restrict__ action,
                                                     int64_t act_stride, const TickArgs* __restrict__ tkp, int K,
                                                     int la_K, const double* __restrict__ rec,
                                                     double* __restrict__ reward, int64_t rew_stride,
                                                     uint64_t* __restrict__ onb, uint32_t* __restrict__ wah,
                                                     unsigned long long* __restrict__ next_slot, WinDrv dv) {
  constexpr bool AFF = FORM == MDR_THERMAL_AFFINE;
  __shared__ unsigned s_cnt[4][kWinMax * kWinCap];
  const int wv = threadIdx.x >> 6;
  const WinTile<HPT> t(p);
  uint64_t* onb_w = onb + (size_t)t.tile * HPT * kWinMax;  // this wave's rows [kWinMax][HPT]
  // KA: lane j = tick j's negated signal penalty (its two loads go out first, beside the state's)
  uint32_t ns_lo = 0, ns_hi = 0;
  if (KA) {
    const int l = (int)(threadIdx.x & 63) < K ? (int)(threadIdx.x & 63) : 0;
    double P;
    if (dv.red) {  // (k_win_records' P, in place: the same win_power on the same totals)
      double p_on[kWinCap];
#pragma unroll
      for (int k = 0; k < kWinCap; ++k) p_on[k] = p.p_on[k < p.n_cap ? k : 0];
      P = win_power(p, dv.red + l * p.n_cap, p_on);
      if (dv.p_out && blockIdx.x == 0 && (int)threadIdx.x == K - 1) *dv.p_out = P;
    } else {
      P = rec[l * kWinRec];
      if (dv.p_out && blockIdx.x == 0 && threadIdx.x == 0) *dv.p_out = rec[(K - 1) * kWinRec];  // (last window)
    }
    const double ns = win_nsig(p, P, dv.s_prev[l]);
    ns_lo = (uint32_t)__double_as_longlong(ns);
    ns_hi = (uint32_t)((uint64_t)__double_as_longlong(ns) >> 32);
  }

  // ---- state + parameters, once per window
  double T[HPT], Tm[HPT], ua[HPT], hm[HPT], tg[HPT], ca[HPT], cm[HPT];
  uint32_t w_end[HPT];
  int cls[HPT];
  const bool params_ok = !*p.params_bad && p.fast_tick_ok;
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    const uint32_t i = t.idx[h];
    T[h] = p.t_air[i]; Tm[h] = p.t_mass[i]; ua[h] = p.ua[i]; hm[h] = p.hm[i]; tg[h] = p.target[i];
    ca[h] = p.ca[i]; cm[h] = p.cm[i];
    w_end[h] = wah[i];
    cls[h] = p.cap_idx[i];
  }
  double q_on[kWinCap];
#pragma unroll
  for (int c = 0; c < kWinCap; ++c) q_on[c] = p.q_on[c < p.n_cap ? c : 0];
  double qc[HPT], lo_tg[HPT], hi_tg[HPT];  // heat when ON; deadbandL2 thresholds (utils.py:4-23)
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    qc[h] = q_on[0];
#pragma unroll
    for (int c = 1; c < kWinCap; ++c) qc[h] = cls[h] == c ? q_on[c] : qc[h];
    hi_tg[h] = tg[h] + p.deadband / 2.0;
    lo_tg[h] = tg[h] - p.deadband / 2.0;
  }
  // per-house constants of the form
  RcWin rw[AFF ? 1 : HPT];
  AffWin aw[AFF ? HPT : 1];
  double tk[HPT], tmk[HPT], hk[HPT];  // AFFINE: Kelvin state, Kelvin penalty threshold
  bool win_finite = true;             // AFFINE: every coefficient and temperature finite
#pragma unroll
  for (int h = 0; h < HPT; ++h) {
    if constexpr (AFF) {
      aw[h] = aff_window(ua[h], ca[h], cm[h], hm[h], (double)p.dt, qc[h], params_ok);
      tk[h] = T[h] + 273.0;
      tmk[h] = Tm[h] + 273.0;
      hk[h] = hi_tg[h] + 273.0;
      const AffWin& a = aw[h];
      const double s = a.tt + a.tm + a.tq + a.to + a.qt + a.mt + a.mm + a.mq + a.mo + a.qm + tk[h] + tmk[h] + hk[h];
      win_finite = win_finite && (s - s == 0.0);
    } else if (params_ok) {
      rw[h] = rc_window(ua[h], ca[h], cm[h], hm[h], (double)p.dt);
    } else {  // IEEE division (identical bits; parameters outside the fast-division range)
      rw[h].k = rc_coeffs_t<false>(ua[h], ca[h], cm[h], hm[h], (double)p.dt);
      rw[h].rCa.nb = -ca[h];
      rw[h].rc.nb = -ua[h];
      rw[h].rd.nb = -(rw[h].k.r2 - rw[h].k.r1);
      rw[h].UaHm = ua[h] + hm[h];
    }
  }
  if constexpr (AFF) win_finite = __all(win_finite);

  // ---- the K ticks: heat source from the stored ON masks, thermal update, reward
  // the tick's scalars (record, ON masks) are loaded one tick ahead (scalar loads, no vector work)
  auto lane_nsig = [&](int j) { return __longlong_as_double((long long)readlane_u64(ns_lo, ns_hi, j)); };
  double r_od = KA ? dv.od_k[0] : rec[0], r_sol = KA ? dv.solar[0] : rec[1], r_sig = KA ? lane_nsig(0) : rec[2];
  uint64_t r_ok = KA ? (uint64_t)(dv.ok & 1u) : __double_as_longlong(rec[3]);  // 1.0 or 0.0: compared as bits (scalar unit)
  uint64_t r_on[HPT];
#pragma unroll
  for (int h = 0; h < HPT; ++h) r_on[h] = onb_w[h];
  const uint32_t rb = t.i0 * 8u;  // byte offset of the lane's house in a reward row (n < 2^29)
  const double nalpha = -p.alpha_temp;
  for (int j = 0; j < K; ++j) {
    const double od_k = r_od, solar = r_sol, nsig = r_sig;
    const bool tick_ok = r_ok != 0;
    uint64_t on_m[HPT];
#pragma unroll
    for (int h = 0; h < HPT; ++h) on_m[h] = r_on[h];
    const int jn = j + 1 < K ? j + 1 : j;
    if (KA) {
      r_od = dv.od_k[jn];
      r_sol = dv.solar[jn];
      r_sig = lane_nsig(jn);
      r_ok = (dv.ok >> jn) & 1u;
    } else {
      r_od = rec[jn * kWinRec + 0];
      r_sol = rec[jn * kWinRec + 1];
      r_sig = rec[jn * kWinRec + 2];
      r_ok = __double_as_longlong(rec[jn * kWinRec + 3]);
    }
#pragma unroll
    for (int h = 0; h < HPT; ++h) r_on[h] = onb_w[jn * HPT + h];
    char* rrow = reinterpret_cast<char*>(reward + (int64_t)j * rew_stride);
    // the reward from the new Celsius temperature Tn (Kelvin tkn on the affine path)
    auto reward_of = [&](int h, double Tn, double tkn, auto fast_c) {
      constexpr bool F = decltype(fast_c)::value;
      if (SIMPLE) {  // deadband 0, norm_temp 1 (the defaults): no branches, no division
        // on the fast path Tn is finite, so the reference's two comparisons reduce to x * x (x = 0
        // gives +0 either way); off it a NaN gives 0.  -(a * pen + s) == (-a) * pen + (-s) bit for
        // bit: negation is exact and rounding is symmetric, and with a, s >= +0 (mdr_capi checks
        // the signs for SIMPLE) the only zero sum is +0 + +0, whose negation is -0 either way
        if (AFF && F) {
          const double x = tkn - hk[h];
          return __builtin_fma(nalpha, x * x, nsig);
        }
        const double x = Tn - hi_tg[h];
        const double pen = F ? x * x : deadband_l2_0(hi_tg[h], Tn);
        return nalpha * pen + nsig;
      }
      double pen = 0.0;
      if (hi_tg[h] < Tn) { const double x = Tn - hi_tg[h]; pen = x * x; }
      else if (lo_tg[h] > Tn) { const double x = lo_tg[h] - Tn; pen = x * x; }
      const double tpen = p.alpha_temp * pen;
      return -((p.norm_temp == 1.0 ? tpen : tpen / p.norm_temp) + -nsig);
    };
    if constexpr (AFF) {
      auto houses = [&](auto fast_c) {
        constexpr bool F = decltype(fast_c)::value;
#pragma unroll
        for (int h = 0; h < HPT; ++h) {
          const AffWin& a = aw[h];
          const bool on = __builtin_amdgcn_inverse_ballot_w64(on_m[h]);
          const double ut = __builtin_fma(a.to, od_k, __builtin_fma(a.tq, solar, on ? a.qt : 0.0));
          const double um = __builtin_fma(a.mo, od_k, __builtin_fma(a.mq, solar, on ? a.qm : 0.0));
          const double tkn = __builtin_fma(a.tt, tk[h], __builtin_fma(a.tm, tmk[h], ut));
          const double tmkn = __builtin_fma(a.mt, tk[h], __builtin_fma(a.mm, tmk[h], um));
          tk[h] = tkn;
          tmk[h] = tmkn;
          const double r = reward_of(h, tkn - 273.0, tkn, fast_c);  // (Celsius unused on the SIMPLE fast path)
          if (t.v[h]) __builtin_nontemporal_store(r, reinterpret_cast<double*>(rrow + (rb + 512u * h)));
        }
      };
      if (win_finite && tick_ok) houses(std::true_type());
      else houses(std::false_type());
    } else {
      // all lanes in range: the comparison masks themselves (v_cmp writes a lane mask) against exec
      uint64_t ok_m = ~0ull;
#pragma unroll
      for (int h = 0; h < HPT; ++h)
        ok_m &= __builtin_amdgcn_ballot_w64(fabs(T[h]) < 1048576.0) & __builtin_amdgcn_ballot_w64(fabs(Tm[h]) < 1048576.0);
      const bool fast = params_ok && tick_ok && ok_m == __builtin_amdgcn_read_exec();
      auto houses = [&](auto fast_c) {
        constexpr bool F = decltype(fast_c)::value;
#pragma unroll
        for (int h = 0; h < HPT; ++h) {
          const bool on = __builtin_amdgcn_inverse_ballot_w64(on_m[h]);
          const double q = on ? qc[h] : 0.0;
          double Tn, Tmn;
          rc_apply_win<F>(T[h], Tm[h], ua[h], hm[h], rw[h], q, solar, od_k, Tn, Tmn);
          T[h] = Tn;
          Tm[h] = Tmn;
          const double r = reward_of(h, Tn, 0.0, fast_c);
          if (t.v[h]) __builtin_nontemporal_store(r, reinterpret_cast<double*>(rrow + (rb + 512u * h)));
        }
      };
      if (fast) houses(std::true_type());
      else houses(std::false_type());
    }
  }
  if constexpr (AFF) {
#pragma unroll
    for (int h = 0; h < HPT; ++h) {
      T[h] = tk[h] - 273.0;
      Tm[h] = tmk[h] - 273.0;
    }
  }

  // ---- state back, once per window (the FSM word at the window's end came with the ON masks)
#pragma unroll
  for (int h = 0; h < HPT; ++h)
    if (t.v[h]) {
      const uint32_t i = t.i0 + 64u * h;
      p.t_air[i] = T[h]; p.t_mass[i] = Tm[h]; p.hvac[i] = w_end[h];
    }

  // ---- lookahead: the next window's ON masks, FSM words and class counts
  if (la_K > 0) {
    uint64_t cmk[HPT][kWinCap];
    win_classes<HPT>(t, cls, cmk);
    win_run<ACT, HPT>(p, w_end, cmk, t, KA ? nullptr : tkp + K, KA ? dv.tick0 + (uint64_t)K : 0, la_K,
                      ACT == MDR_ACT_BUFFER ? action + (int64_t)K * act_stride : nullptr, act_stride, s_cnt[wv],
                      onb_w);
#pragma unroll
    for (int h = 0; h < HPT; ++h)
      if (t.v[h]) wah[t.i0 + 64u * h] = w_end[h];
    __syncthreads();
    win_flush(p, la_K, s_cnt, next_slot);
  }
}


#define MDR_INST_WIN_F(A, SI, KA_, FO)                                                                         \
  template __global__ void k_step_window<A, kWinHpt, SI, KA_, FO>(KParams, const uint8_t*, int64_t, const TickArgs*, \
                                                                  int, int, const double*, double*, int64_t,   \
                                                                  uint64_t*, uint32_t*, unsigned long long*, WinDrv);
#define MDR_INST_WIN(A)                                                                                         \
  MDR_INST_WIN_F(A, true, false, MDR_THERMAL_EXACT) MDR_INST_WIN_F(A, false, false, MDR_THERMAL_EXACT)          \
  MDR_INST_WIN_F(A, true, true, MDR_THERMAL_EXACT) MDR_INST_WIN_F(A, false, true, MDR_THERMAL_EXACT)            \
  MDR_INST_WIN_F(A, true, false, MDR_THERMAL_AFFINE) MDR_INST_WIN_F(A, false, false, MDR_THERMAL_AFFINE)        \
  MDR_INST_WIN_F(A, true, true, MDR_THERMAL_AFFINE) MDR_INST_WIN_F(A, false, true, MDR_THERMAL_AFFINE)          \
  template __global__ void k_count_window<A, kWinHpt>(KParams, const uint8_t*, int64_t, const TickArgs*, uint64_t, \
                                                      int, unsigned long long*, uint64_t*, uint32_t*, const uint32_t*, \
                                                      unsigned*);
MDR_INST_WIN(MDR_ACT_RANDOM)
MDR_INST_WIN(MDR_ACT_ALWAYS_ON)
MDR_INST_WIN(MDR_ACT_BUFFER)

#define MDR_INST_PIPE(T, A, LA, G)                                                                    \
  template __global__ void k_step_pipe<T, A, LA, G>(KParams, const uint8_t*, TickArgs, const TickArgs*, \
                                                    const unsigned long long*, double*, double*,         \
                                                    unsigned long long*, unsigned long long*, GqOut, GqfBufs, int);
MDR_INST_PIPE(1, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0)
MDR_INST_PIPE(2, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0)
MDR_INST_PIPE(4, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0)
MDR_INST_PIPE(8, MDR_ACT_RANDOM, MDR_ACT_RANDOM, 0)
MDR_INST_PIPE(2, MDR_ACT_BUFFER, 0, 0)
MDR_INST_PIPE(4, MDR_ACT_BUFFER, 0, 0)
MDR_INST_PIPE(2, MDR_ACT_BUFFER, 0, 1)
MDR_INST_PIPE(4, MDR_ACT_BUFFER, 0, 1)
MDR_INST_PIPE(2, MDR_ACT_BUFFER, 0, 2)
MDR_INST_PIPE(4, MDR_ACT_BUFFER, 0, 2)

#define MDR_INST_STEP(F, A, LA)                                                                  \
  template __global__ void k_step_t<2, F, A, LA>(                                                \
      KParams, const uint8_t*, int, TickArgs, const TickArgs*, const unsigned long long*,        \
      double*, int, uint8_t*, double*, int, unsigned long long*, unsigned long long*, double*, int);
MDR_INST_STEP(false, -1, -1)
MDR_INST_STEP(true, -1, -1)
MDR_INST_STEP(true, MDR_ACT_RANDOM, MDR_ACT_RANDOM)
MDR_INST_STEP(true, MDR_ACT_BUFFER, 0)

// Division self-check: q_fast = shared-reciprocal sequence, q_ieee = the / operator.
__global__ void k_div_check(const double* __restrict__ a, const double* __restrict__ b, int64_t n,
                            unsigned long long* __restrict__ mismatches) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = a[i], y = b[i];
  const double f = div_by(x, recip(y));
  const double q = x / y;
  if (__double_as_longlong(f) != __double_as_longlong(q)) atomicAdd(mismatches, 1ull);
}

// After a parameter change: flag any house whose parameters leave the range in which the
// shared-reciprocal division is provably identical to `/` (Ua in [2^-20, 2^20], Ca/Cm/Hm in
// [2^-10, 2^50]; the step then uses the plain operator).
__device__ __forceinline__ bool in_pow2_range(double x, int lo, int hi) {
  const int e = (int)((__double_as_longlong(x) >> 52) & 0x7FF) - 1023;
  return x > 0.0 && e >= lo && e < hi;
}

__global__ void __launch_bounds__(256) k_refresh(KParams p, int* params_bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const double ua = p.ua[i], ca = p.ca[i], cm = p.cm[i], hm = p.hm[i];
  const bool ok = in_pow2_range(ua, -20, 20) && in_pow2_range(ca, -10, 50) &&
                  in_pow2_range(cm, -10, 50) && in_pow2_range(hm, -10, 50);
  if (!ok) atomicOr(params_bad, 1);
}

// Memory-floor probe for k_step's access pattern: the same loads and stores, trivial arithmetic
// (roofline diagnostics only; never on the product path).
__global__ void __launch_bounds__(256) k_probe_stream(KParams p, double* __restrict__ reward) {
  const int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (i0 + 1 >= p.n) return;
  const double2 vT = *reinterpret_cast<const double2*>(p.t_air + i0);
  const double2 vTm = *reinterpret_cast<const double2*>(p.t_mass + i0);
  const double2 vua = *reinterpret_cast<const double2*>(p.ua + i0);
  const double2 vca = *reinterpret_cast<const double2*>(p.ca + i0);
  const double2 vcm = *reinterpret_cast<const double2*>(p.cm + i0);
  const double2 vhm = *reinterpret_cast<const double2*>(p.hm + i0);
  const double2 vtg = *reinterpret_cast<const double2*>(p.target + i0);
  const uint2 vw = *reinterpret_cast<const uint2*>(p.hvac + i0);
  const unsigned short vc = *reinterpret_cast<const unsigned short*>(p.cap_idx + i0);
  const double s0 = vua.x + vca.x + vcm.x + vhm.x + vtg.x + (double)(vc & 0xFF);
  const double s1 = vua.y + vca.y + vcm.y + vhm.y + vtg.y + (double)(vc >> 8);
  // values depend on every load (0 * s is not foldable: s may be inf/nan), so neither the loads
  // nor the write-backs can be elided
  *reinterpret_cast<double2*>(p.t_air + i0) = make_double2(vT.x + 0.0 * s0, vT.y + 0.0 * s1);
  *reinterpret_cast<double2*>(p.t_mass + i0) = make_double2(vTm.x + 0.0 * s0, vTm.y + 0.0 * s1);
  *reinterpret_cast<uint2*>(p.hvac + i0) = make_uint2(vw.x ^ (vc & 0x100000u), vw.y);
  *reinterpret_cast<double2*>(reward + i0) = make_double2(s0, s1);
}

// Fixed-order reduction of the per-block penalty partials -> partial2 = {sum pen/N, max pen}.
__global__ void __launch_bounds__(256) k_pen_reduce(const double* __restrict__ pen_partial, int nblk,
                                                    double* __restrict__ partial2) {
  __shared__ double ss[256], sm[256];
  double s = 0.0, m = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x) { s += pen_partial[2 * b]; m = fmax(m, pen_partial[2 * b + 1]); }
  ss[threadIdx.x] = s;
  sm[threadIdx.x] = m;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      ss[threadIdx.x] += ss[threadIdx.x + w];
      sm[threadIdx.x] = fmax(sm[threadIdx.x], sm[threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { partial2[0] = ss[0]; partial2[1] = sm[0]; }
}

// rewards for common_L2 / common_max_error / mixture (rewards_calculator.py:46-181)
__global__ void __launch_bounds__(256) k_reward_finalize(KParams p, TickArgs tk,
                                                         const unsigned long long* __restrict__ counts,
                                                         const double* __restrict__ partial2,
                                                         double* __restrict__ reward) {
  const double P = wave_power(counts, p.p_on, p.n_cap);
  const double x = (P - tk.s_prev) / (double)p.n_global;
  const double sig_term = p.alpha_sig * (x * x) / p.norm_sig;
  const double common_l2 = partial2[0], common_max = partial2[1];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const double pen = reward[i];
  double tp;
  if (p.penalty_mode == MDR_PEN_COMMON_L2) tp = common_l2;
  else if (p.penalty_mode == MDR_PEN_COMMON_MAX) tp = common_max;
  else tp = (p.alpha_ind_l2 * pen + p.alpha_common_l2 * common_l2 + p.alpha_common_max * common_max) /
            (p.alpha_ind_l2 + p.alpha_common_l2 + p.alpha_common_max);
  reward[i] = -(p.alpha_temp * tp / p.norm_temp + sig_term);
}

// Reward of the last tick of an overlapped multi-GPU rollout (the k_step launches there write
// the previous tick's reward): temperature penalty from the current state, signal term from the
// tick's allreduced counts (rewards_calculator.py:135-203, individual_L2).
__global__ void __launch_bounds__(256) k_reward_state(KParams p, const TickArgs* __restrict__ tkp,
                                                      const unsigned long long* __restrict__ counts,
                                                      double* __restrict__ reward, double* p_out) {
  const double P = wave_power(counts, p.p_on, p.n_cap);
  const double x = (P - tkp->s_prev) / (double)p.n_global;
  const double sig_term = p.alpha_sig * (x * x) / p.norm_sig;
  if (p_out && blockIdx.x == 0 && threadIdx.x == 0) *p_out = P;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const double tpen = p.alpha_temp * deadband_l2(p.target[i], p.deadband, p.t_air[i]);
  reward[i] = -((p.norm_temp == 1.0 ? tpen : tpen / p.norm_temp) + sig_term);
}

// --------------------------------------------------------------------------------------- stats
// Cluster statistics the server reads after every tick, one pass over the state:
// Metrics.update (metrics_service.py:108-157) and the UI summary / graph data
// (client_manager_service.py:62-111,177-196).  Deterministic two-level reduction (fixed block
// partials, then one block in index order), so a run is reproducible; the reference sums
// sequentially in house order, so floating-point sums agree to rounding (~1e-15 relative).
//   s[0] sum (T - target / N)    (metrics' temp_error, operator precedence as the reference)
//   s[1] sum |T - target / N|    s[2] max(0, max (T - target / N))    s[3] sum (T - target / N)^2
//   s[4] sum reward / N          s[5] sum T     s[6] sum (T - target)   s[7] sum |T - target|
//   s[8] sum T_mass              s[9] sum target   s[10] # lockout     s[11] # on
__global__ void __launch_bounds__(256) k_cluster_stats(KParams p, const double* __restrict__ reward,
                                                       double* __restrict__ partial) {
  __shared__ double sh[kStats][4];
  double a[kStats];
#pragma unroll
  for (int k = 0; k < kStats; ++k) a[k] = 0.0;
  const double N = (double)p.n_global;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += (int64_t)gridDim.x * blockDim.x) {
    const double T = p.t_air[i], tg = p.target[i];
    const double e = T - tg / N;
    const double d = T - tg;
    a[0] += e;
    a[1] += fabs(e);
    a[2] = fmax(a[2], e);
    a[3] += e * e;
    if (reward) a[4] += reward[i] / N;
    a[5] += T;
    a[6] += d;
    a[7] += fabs(d);
    a[8] += p.t_mass[i];
    a[9] += tg;
    const uint32_t w = p.hvac[i];
    a[10] += hv_lock(w) ? 1.0 : 0.0;
    a[11] += hv_on(w) ? 1.0 : 0.0;
  }
#pragma unroll
  for (int k = 0; k < kStats; ++k)
    for (int off = 32; off > 0; off >>= 1) {
      const double o = __shfl_xor(a[k], off);
      a[k] = k == 2 ? fmax(a[k], o) : a[k] + o;
    }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < kStats; ++k) sh[k][wv] = a[k];
  __syncthreads();
  if (threadIdx.x < kStats) {
    const int k = threadIdx.x;
    double v = sh[k][0];
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) v = k == 2 ? fmax(v, sh[k][w]) : v + sh[k][w];
    partial[(size_t)blockIdx.x * kStats + k] = v;
  }
}

__global__ void __launch_bounds__(64) k_cluster_stats_final(const double* __restrict__ partial, int nblk,
                                                            double* __restrict__ out) {
  const int k = threadIdx.x;
  if (k >= kStats) return;
  double v = k == 2 ? 0.0 : partial[k];  // max starts at 0 like the reference's max_temp_error
  for (int b = k == 2 ? 0 : 1; b < nblk; ++b) v = k == 2 ? fmax(v, partial[(size_t)b * kStats + k]) : v + partial[(size_t)b * kStats + k];
  out[k] = v;
}

// --------------------------------------------------------------------------------------- population
// Synthetic population: the reference noise model (building.py:224-267, hvac.py:66-70) drawn
// from Philox4x32-10 keyed by (seed, global house id) — identical for any sharding.
__device__ __forceinline__ double triangular(double u, double lo, double hi, double mode) {
  // random.triangular's inverse CDF
  double c = (mode - lo) / (hi - lo);
  if (u > c) { u = 1.0 - u; c = 1.0 - c; const double t = lo; lo = hi; hi = t; }
  return lo + (hi - lo) * sqrt(u * c);
}

__global__ void __launch_bounds__(256) k_populate(KParams p, PopArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  const uint64_t gid = p.goff + i;
  const u32x4 r0 = philox4x32_10(u32x4{(uint32_t)gid, (uint32_t)(gid >> 32), 0x9090u, 0u},
                                 (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
  const u32x4 r1 = philox4x32_10(u32x4{(uint32_t)gid, (uint32_t)(gid >> 32), 0x9090u, 1u},
                                 (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
  const double g = sqrt(-2.0 * log(u01(r0.x))) * cos(6.283185307179586 * u01(r0.y));
  double* pt = const_cast<double*>(p.target);
  pt[i] = a.target_temp + fabs(g * a.std_target);
  const_cast<double*>(p.ua)[i] = triangular(u01(r0.z), a.lo, a.hi, 1.0);
  const_cast<double*>(p.cm)[i] = a.cm0 * triangular(u01(r0.w), a.lo, a.hi, 1.0);
  const_cast<double*>(p.ca)[i] = a.ca0 * triangular(u01(r1.x), a.lo, a.hi, 1.0);
  const_cast<double*>(p.hm)[i] = a.hm0 * triangular(u01(r1.y), a.lo, a.hi, 1.0);
  if (a.n_draw > 0)  // random.choices(cooling_capacity_list): a uniform list entry
    const_cast<uint8_t*>(p.cap_idx)[i] = a.draw_idx[((uint64_t)r1.z * (uint64_t)a.n_draw) >> 32];
  else
    const_cast<uint8_t*>(p.cap_idx)[i] = (uint8_t)(((uint64_t)r1.z * (uint64_t)p.n_cap) >> 32);
  p.t_air[i] = a.init_air;
  p.t_mass[i] = a.init_mass;
  p.hvac[i] = kOnBit;
}

// --------------------------------------------------------------------------------------- obs
// norm_state_dict (norm.py:178-218) as float32 rows, staged through LDS and flushed with
// 16-B coalesced stores.  Row assembly: mdr_obs_dev.h (shared with the fused actor kernel).
__global__ void __launch_bounds__(kObsBlock) k_obs(KParams p, ObsArgs o, const double* p_dev,
                                                   float* __restrict__ obs) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (o.sc_dev) { o.s = o.sc_dev[1]; o.solar = o.sc_dev[2]; o.t_od = o.sc_dev[3]; }  // (per-tick rows of rollouts)
  const int F = o.n_feat;
  const int64_t b0 = (int64_t)blockIdx.x * kObsBlock;
  const int nb = (int)min((int64_t)kObsBlock, p.n - b0);
  float* tile = smem;                                  // [kObsBlock][F]
  float* msg = smem + ((kObsBlock * F + 3) & ~3);      // [lo + kObsBlock + hi][M]
  __shared__ float cf[kObsConst];
  obs_consts(p, o, p_dev ? *p_dev : o.p, cf, threadIdx.x, kObsBlock);
  __syncthreads();
  const ObsDiv dv = obs_div(p);
  obs_stage_ring(p, o, b0, nb, cf, msg, threadIdx.x, kObsBlock, dv);
  __syncthreads();
  const int t = threadIdx.x;
  if (t < nb) obs_build_row(p, o, b0 + t, t, cf, msg, tile + t * F, dv);
  __syncthreads();
  // coalesced flush of the contiguous tile obs[b0 .. b0+nb) rows
  const int64_t nflt = (int64_t)nb * F;
  float* dst = obs + b0 * F;
  if ((((uintptr_t)dst) & 15) == 0) {
    const int64_t n4 = nflt >> 2;
    for (int64_t q = threadIdx.x; q < n4; q += kObsBlock)
      reinterpret_cast<float4*>(dst)[q] = reinterpret_cast<const float4*>(tile)[q];
    for (int64_t q = (n4 << 2) + threadIdx.x; q < nflt; q += kObsBlock) dst[q] = tile[q];
  } else {
    for (int64_t q = threadIdx.x; q < nflt; q += kObsBlock) dst[q] = tile[q];
  }
}

// message features of the first `lo` (tail) / last `hi` (head) houses of this shard, for the
// neighbouring shards' ring halos: out[0..hi) = first hi houses, out[hi..hi+lo) = last lo houses
__global__ void k_halo_pack(KParams p, ObsArgs o, int lo, int hi, float* out) {
  const int t = threadIdx.x;
  const int M = o.msg_w;
  __shared__ float cf[kObsConst];
  obs_consts(p, o, o.p, cf, t, blockDim.x);  // (the message features use only cf[8..] and P_max/R)
  __syncthreads();
  const ObsDiv dv = obs_div(p);
  if (t < hi) msg_features(p, o, t % p.n, cf, out + t * M, dv);
  else if (t < hi + lo) {
    int64_t j = p.n - lo + (t - hi);
    if (j < 0) j = ((j % p.n) + p.n) % p.n;
    msg_features(p, o, j, cf, out + t * M, dv);
  }
}

// The sharded MA-PPO tick's one collective (mdr_actor_rollout_sharded): the ring halo of tick t + 1
// needs the POST-step message features of this shard's first hi and last lo houses, and those need
// only the houses' own state, the actions just sampled and the tick's drivers — not the cluster
// power — so they are computed here, before the step (the same FSM and one-tick RC expressions as
// the step kernels: bit-identical to the state the step will write), and packed into this rank's
// slot of `rows` [world][hi + lo][msg_w] (rows 0..hi: first hi houses, hi..hi+lo: last lo), every
// other slot zeroed: summed with the count slab in one integer allreduce, the slots become every
// rank's rows (x + 0 is exact on the bit patterns).  One block.
__global__ void k_halo_step_pack(KParams p, ObsArgs o, const uint8_t* __restrict__ action,
                                 const TickArgs* __restrict__ tkp, int lo, int hi, int rank, int world,
                                 float* __restrict__ rows) {
  const int M = o.msg_w, tid = threadIdx.x, slot = (hi + lo) * M;
  __shared__ float cf[kObsConst];
  obs_consts(p, o, o.p, cf, tid, blockDim.x);  // (messages use only cf[8..] and P_max/R)
  for (int e = tid; e < world * slot; e += blockDim.x)
    if (e / slot != rank) rows[e] = 0.f;
  __syncthreads();
  const ObsDiv dv = obs_div(p);
  const TickArgs tk = *tkp;
  for (int t = tid; t < hi + lo; t += blockDim.x) {
    int64_t j = t < hi ? t % p.n : p.n - lo + (t - hi);
    if (j < 0) j = ((j % p.n) + p.n) % p.n;
    HouseRegs r;
    house_load(p, j, true, r);
    r.w = hvac_fsm(r.w, action[j] != 0, p.dt, p.L);
    const double q = hv_on(r.w) ? p.q_on[r.cls] : 0.0;
    const RcCoef kc = rc_coeffs_t<false>(r.ua, r.ca, r.cm, r.hm, (double)p.dt);
    double Tn, Tmn;
    rc_apply_t<false>(r.T, r.Tm, r.ua, r.ca, r.hm, kc, q, tk.solar, tk.t_od_prev, Tn, Tmn);
    r.T = Tn;
    r.Tm = Tmn;
    msg_from_regs(p, o, r, cf, rows + (size_t)rank * slot + (size_t)t * M, dv);
  }
}

// message features of every local house (sharded table comm modes: all-gathered into msg_all)
__global__ void k_msg_pack(KParams p, ObsArgs o, float* out) {
  __shared__ float cf[kObsConst];
  obs_consts(p, o, o.p, cf, threadIdx.x, blockDim.x);  // (messages use only cf[8..] and P_max/R)
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < p.n) msg_features(p, o, i, cf, out + i * o.msg_w, obs_div(p));
}

// --------------------------------------------------------------------------------------- greedy
// GreedyMyopic.get_action (greedy_myopic_controller.py:67-104), device form:
//   key_i = -(T_i - target_i), sorted ascending (stable radix sort; pandas' quicksort tie order
//   is implementation-defined, parity on exact key ties is unpinned).  Then the sequential rule
//   take_j  iff  P_j + tot < S  or  (|P_j + tot - S| < |tot - S| and not lockout_j)
// is evaluated as: a prefix of the sorted order is taken while the inclusive prefix sum of P is
// < S (k = first index where it is not); from k on, with gap g = S - tot, item j is taken iff
// P_j < g or (P_j < 2g and not lockout_j) — gap-dependent, so a single workgroup walks the
// remaining order with 256-wide ballots until g can no longer admit any class (2g <= min P).
__global__ void k_greedy_keys(KParams p, double* __restrict__ key, int* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  key[i] = -(p.t_air[i] - p.target[i]);
  idx[i] = (int)i;
}

__global__ void k_greedy_gather(KParams p, const int* __restrict__ perm, double* __restrict__ psorted,
                                uint8_t* __restrict__ lsorted) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= p.n) return;
  const int i = perm[j];
  psorted[j] = p.p_on[p.cap_idx[i]];
  lsorted[j] = hv_lock(p.hvac[i]) ? 1 : 0;
}

// single workgroup: k from the inclusive prefix sums, then the gap walk; writes the take flag
// for sorted positions >= k into flag_sorted (positions < k are implied) and kpos[0] = k.
__global__ void __launch_bounds__(256) k_greedy_walk(int64_t n, const double* __restrict__ incl,
                                                     const double* __restrict__ psorted,
                                                     const uint8_t* __restrict__ lsorted, double S,
                                                     double pmin, int64_t* kpos,
                                                     int64_t* extra, int max_extra) {
  __shared__ int64_t s_k;
  __shared__ int s_ne;
  __shared__ double s_tot;
  if (threadIdx.x == 0) {
    // first k with incl[k] >= S  (all earlier items satisfy P + tot < S); binary search
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) / 2;
      if (incl[mid] < S) lo = mid + 1; else hi = mid;
    }
    s_k = lo;
    s_tot = lo > 0 ? incl[lo - 1] : 0.0;
    s_ne = 0;
  }
  __syncthreads();
  int64_t pos = s_k;
  while (pos < n) {
    const double tot = s_tot;
    // once tot >= S nothing is taken (P > 0); with gap g = S - tot an item needs P < 2g
    // (conservative margin: the exact predicate below decides)
    if (!(tot < S) || 2.0 * (S - tot) < pmin * (1.0 - 1e-9)) break;
    const int64_t j = pos + threadIdx.x;
    bool take = false;
    if (j < n) {
      const double pj = psorted[j];
      take = (pj + tot < S) || (fabs(pj + tot - S) < fabs(tot - S) && !lsorted[j]);
    }
    __shared__ unsigned long long s_bal[4];
    const unsigned long long b = __ballot(take);
    if ((threadIdx.x & 63) == 0) s_bal[threadIdx.x >> 6] = b;
    __syncthreads();
    int first = -1;
    for (int w = 0; w < 4; ++w)
      if (s_bal[w]) { first = w * 64 + __ffsll((long long)s_bal[w]) - 1; break; }
    __syncthreads();
    if (first < 0) { pos += blockDim.x; continue; }
    if (threadIdx.x == 0) {
      const int64_t jj = pos + first;
      if (s_ne < max_extra) extra[s_ne] = jj;
      s_ne++;
      s_tot = tot + psorted[jj];
    }
    __syncthreads();
    pos += first + 1;
  }
  if (threadIdx.x == 0) { kpos[0] = s_k; kpos[1] = s_ne < max_extra ? s_ne : max_extra; }
}

// ---- histogram-select form (mdr_ctrl_greedy for <= 4 capacity classes; the sort form above
// serves wider capacity tables and the all-gathered sharded rows).
// Only the houses around the budget crossing need an order: houses are binned by a monotone
// linear quantisation of the key over [kmin, kmax] (kGqBins bins, class counts per bin), the bin
// b* where the cumulative P crosses S is found from the bin sums, every house in a lower bin is
// taken, and only the houses of bins [b*, b_end] (at most kGqCap, with >= kGqAfter houses past
// b*) are ordered — by (key value, house), as the stable sort orders them — in LDS, where the exact
// crossing position and the gap walk are evaluated.  Sums of P are exact for integer P (every sum
// of P here is).  What the candidate window cannot decide (a crossing among NaN keys, a crossing
// bin over kGqCap houses — e.g. thousands of identical keys —, a walk that leaves the window) the
// last kernel decides itself, in the same launch, with an exact radix select over the 96-bit
// (key, house) order (gq_exact): no host synchronisation, no sort, every tick.
// The houses travel as 4-B codes (gq_code: key bin << 2 | class) written by the key producer; the
// exact key is re-read from the state (gq_key_of) only for the window's houses.
// The launches of one decision: [codes: k_gq_keys, or the previous step kernel's epilogue] ->
// k_gq_bins -> k_gq_compact -> k_gq_select; compact and select also count the ON houses the
// decided actions produce (the next step's cluster power).
// K1: codes, per-block (min, max) of the finite keys (the next call's range), and the class counts
// per superbin (kGqBins / kGqSuper consecutive bins; NaN keys in their own) under this call's
// quantisation
// (no band counts: band_valid = 0); block 0 zeroes the slab the decisions are counted into
__global__ void __launch_bounds__(kGqThreads) k_gq_keys(KParams p, uint32_t* __restrict__ code, double* __restrict__ part,
                                                        unsigned* __restrict__ hist, GqSel* __restrict__ sel,
                                                        const uint32_t* __restrict__ map, unsigned long long* __restrict__ slab) {
  constexpr int NW = kGqThreads / 64;
  __shared__ unsigned s_sh[NW * kGqSupStride];  // one copy per wave (less atomic contention on hot superbins)
  __shared__ uint32_t s_map[kGqCells];
  for (int e = threadIdx.x; e < NW * kGqSupStride; e += blockDim.x) s_sh[e] = 0u;
  for (int e = threadIdx.x; e < kGqCells; e += blockDim.x) s_map[e] = map[e];
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) sel->band_valid = 0;
    if (slab)
      for (int e = threadIdx.x; e < kCountShards * p.n_cap; e += blockDim.x) slab[e] = 0ull;
  }
  __syncthreads();
  const double kmin = sel->kmin, scale = sel->scale;
  double lo = INFINITY, hi = -INFINITY;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // kGqUnroll houses per thread per pass, every load issued before the first use (the grid is one
  // block per CU: without the batch each pass waits out a full HBM latency)
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < p.n; i0 += kGqUnroll * stride) {
    double ta[kGqUnroll], tg[kGqUnroll];
    unsigned cl[kGqUnroll];
#pragma unroll
    for (int u = 0; u < kGqUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      ta[u] = i < p.n ? p.t_air[i] : 0.0;
      tg[u] = i < p.n ? p.target[i] : 0.0;
      cl[u] = i < p.n ? p.cap_idx[i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kGqUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      if (i >= p.n) break;
      const double k = -(ta[u] - tg[u]);  // gq_key_of
      const uint32_t c = gq_code(k, kmin, scale, s_map, cl[u]);
      code[i] = c;
      if (k == k) {
        lo = fmin(lo, k);
        hi = fmax(hi, k);
      }
      atomicAdd(&s_sh[(threadIdx.x >> 6) * kGqSupStride + (c >> 8) * 4 + (c & 3u)], 1u);
    }
  }
  __syncthreads();
  gq_flush(s_sh, NW, hist, lo, hi, part);
}

// A fresh key map after the state was written (reset, populate, parameter writes): the keys may lie
// far outside the map the last call built, so a code pass under it clamps most houses into its end cells
// and the crossing bin overflows the window (gq_exact: one block over the cluster, ~7 ms at 1M houses).
// From a first pass's per-block key ranges: cells uniform over the cluster's [min, max] (the calls after
// rebuild them equi-depth), the superbin copies that pass counted zeroed, the band prediction reset; the
// caller runs the code pass again.  One block.  map / kmin / scale: the parity's (fused) or the select's.
__global__ void __launch_bounds__(256) k_gq_remap(KParams p, const double* __restrict__ part, int nparts,
                                                  unsigned* __restrict__ sup, GqSel* __restrict__ sel,
                                                  uint32_t* __restrict__ map, double* __restrict__ kmin_out,
                                                  double* __restrict__ scale_out) {
  __shared__ double s_lo[4], s_hi[4], s_rng[2];
  double lo = INFINITY, hi = -INFINITY;
  for (int b = threadIdx.x; b < nparts; b += blockDim.x) { lo = fmin(lo, part[2 * b]); hi = fmax(hi, part[2 * b + 1]); }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
  }
  if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double kmin = s_lo[0], kmax = s_hi[0];
    for (int w = 1; w < 4; ++w) { kmin = fmin(kmin, s_lo[w]); kmax = fmax(kmax, s_hi[w]); }
    const double range = kmax - kmin;
    s_rng[0] = kmin == kmin && kmin < INFINITY ? kmin : 0.0;  // (gq_next_map_core's rules)
    s_rng[1] = range > 0.0 && range < INFINITY ? (double)kGqCells / range : 0.0;
    *kmin_out = s_rng[0];
    *scale_out = s_rng[1];
    sel->band_valid = 0;
    sel->sb_raw = -1;
    sel->xprev = 0u;
  }
  const int NBE = gq_bins_eff(p.n_global);
  for (int c = threadIdx.x; c < kGqCells; c += blockDim.x) {
    const int b0 = c * (NBE / kGqCells), b1 = (c + 1) * (NBE / kGqCells);
    map[c] = ((uint32_t)b0 << 16) | (uint32_t)(b1 - b0);
  }
  for (int e = threadIdx.x; e < kGqCopies * kGqSupStride; e += blockDim.x) sup[e] = 0u;
}

// sharded histogram select: this shard's finite key range from the producer's per-block parts, as
// (min, -max), so ONE min-allreduce gives the cluster's (k_gq_bins with nparts < 0); one block
__global__ void __launch_bounds__(256) k_gq_range(const double* __restrict__ part, int nparts, double* __restrict__ range) {
  __shared__ double s_lo[4], s_hi[4];
  double lo = INFINITY, hi = -INFINITY;
  for (int b = threadIdx.x; b < nparts; b += blockDim.x) { lo = fmin(lo, part[2 * b]); hi = fmax(hi, part[2 * b + 1]); }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
  }
  if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) { lo = fmin(lo, s_lo[w]); hi = fmax(hi, s_hi[w]); }
    lo = fmin(lo, s_lo[0]);
    hi = fmax(hi, s_hi[0]);
    range[0] = lo;
    range[1] = -hi;
  }
}

// a block-wide inclusive scan of (double P, u64 count) over the first n <= blockDim.x threads
// (wave shuffles, then the wave totals through LDS); returns the inclusive values
// (nwd: the waves holding data — the superbin and digit scans fill the first 257 / 256 threads; the
// other waves skip both halves, so the longest serial sum of wave totals is nwd - 1 reads, not 15)
__device__ __forceinline__ void gq_block_scan(double& x, unsigned long long& xc, double* s_w, unsigned long long* s_wc,
                                              int nwd = kGqThreads / 64) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv < nwd) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double y = __shfl_up(x, off);
      const unsigned long long yc = __shfl_up(xc, off);
      if (lane >= off) { x += y; xc += yc; }
    }
    if (lane == 63) { s_w[wv] = x; s_wc[wv] = xc; }
  }
  __syncthreads();
  if (wv < nwd)
    for (int w = 0; w < wv; ++w) { x += s_w[w]; xc += s_wc[w]; }  // (fixed order: the same sums in every block)
}

// relaxed agent-scope (sc1) stores and loads: write-through / L2-served, for data other workgroups of
// the same launch read (MI355X_MICROARCH.md, Valid forms)
template <typename T>
__device__ __forceinline__ void st_sc1(T* d, T v) { __hip_atomic_store(d, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* s) { return __hip_atomic_load(s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// The crossing superbin (k_gq_bins): every block scans the superbin class counts
// itself (the cumulative P where it reaches S; the same arithmetic in every block, so every block
// agrees), block 0 records it and zeroes the current count slab (compact and select fill it) and the
// window allocator.  Returns the superbin, the P and houses before it and the cluster's houses.
struct GqSuper {
  int sb;
  bool whole;  // a cluster of <= kGqCap houses is one window (the select orders all of it, NaN keys included)
  double before;
  unsigned long long before_cnt, total;
};
// the superbin copies of thread tid (< kGqSupN) as loaded values, issued before a caller's other loads
// (gq_super_find's scan then waits only for these: vmcnt counts in issue order)
struct GqSupLoad {
  uint4 v[kGqCopies];
  double pon[kWinCap];  // the classes' P (issued beside the copies: a scalar load waited for after them cost ~1 us)
};
__device__ __forceinline__ void gq_pon_load(const KParams& p, double* pon) {
#pragma unroll
  for (int k = 0; k < kWinCap; ++k) pon[k] = p.p_on[k < p.n_cap ? k : 0];
}
// sup: the superbin copies (kGqCopies x kGqSupStride words; g_hist + kGqBins * 4, or a fused parity's)
__device__ __forceinline__ GqSupLoad gq_super_load_at(const KParams& p, const unsigned* __restrict__ sup) {
  GqSupLoad l;
  gq_pon_load(p, l.pon);
  const int tid = threadIdx.x;
  // (one branch around all the loads: per-load conditions made the compiler wait after every pair)
  const int t = tid < kGqSupN ? tid : 0;
  const uint4* src = reinterpret_cast<const uint4*>(sup + t * 4);
#pragma unroll
  for (int q = 0; q < kGqCopies; ++q) l.v[q] = src[q * (kGqSupStride / 4)];
  return l;  // (threads >= kGqSupN hold superbin 0's counts: gq_super_find ignores them)
}
__device__ __forceinline__ GqSupLoad gq_super_load(const KParams& p, const unsigned* __restrict__ hist) {
  return gq_super_load_at(p, hist + kGqBins * 4);
}
__device__ __forceinline__ GqSuper gq_super_scan(const KParams& p, const GqSupLoad& l, double S, GqSel* __restrict__ sel,
                                 unsigned long long* __restrict__ slab, bool reset_alloc,
                                 unsigned long long* st = nullptr) {
#define GQS_STAMP(k) \
  do { if (st && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
  constexpr int NW = kGqThreads / 64;
  static_assert(kGqSupN <= kGqThreads && kGqCells < kGqThreads, "one superbin / cell edge per thread");
  __shared__ double s_w[NW], s_bt;
  __shared__ unsigned long long s_wc[NW], s_total, s_bc;
  __shared__ int s_first;
  const int tid = threadIdx.x;
  const double* p_on = l.pon;
  unsigned long long c[kWinCap] = {0ull, 0ull, 0ull, 0ull};
  if (tid < kGqSupN)
#pragma unroll
    for (int q = 0; q < kGqCopies; ++q) {
      c[0] += l.v[q].x; c[1] += l.v[q].y; c[2] += l.v[q].z; c[3] += l.v[q].w;
    }
  GQS_STAMP(0);
  const double ps = win_power(p, c, p_on);
  const unsigned long long cs = c[0] + c[1] + c[2] + c[3];
  double x = ps;
  unsigned long long xc = cs;
  if (tid == 0) { s_first = kGqSupN; s_bt = 0.0; s_bc = 0ull; }
  gq_block_scan(x, xc, s_w, s_wc, (kGqSupN + 63) / 64);
  GQS_STAMP(1);
  const double before = x - ps;
  {  // the first non-empty superbin where the P reaches S: one LDS atomic per wave (same-address LDS
     // atomics serialise: one per thread cost ~4 us here, r06 phase stamps)
    const unsigned long long m = __ballot(tid < kGqSupN && cs > 0 && !(before + ps < S));
    if (m && (tid & 63) == 0) atomicMin(&s_first, (tid & ~63) + __ffsll((long long)m) - 1);
  }
  if (tid == kGqSupN - 1) s_total = xc;
  __syncthreads();
  GQS_STAMP(2);
  const int sb = s_first;
  const bool whole = sb < kGqSupN && s_total <= (unsigned long long)kGqCap;
  if (tid == sb) { s_bt = before; s_bc = xc - cs; }
  if (blockIdx.x == 0) {
    if (tid == sb) { sel->base_tot = before; sel->base_cnt = xc - cs; }
    if (tid == kGqSupN - 1) sel->total = xc;
    if (tid == 0) {
      sel->sb = sb;
      sel->all = sb >= kGqSupN;
      sel->overflow = sb == kGqSuper && !whole;  // the crossing among NaN keys: the fallback orders them by house
      sel->whole = whole;
      if (reset_alloc) {  // (k_gq_binsc: other blocks of its launch may already allocate)
        sel->wcount = 0u;
        sel->need_fb = 0u;
      }
    }
    if (slab)
      for (int e = tid; e < kCountShards * p.n_cap; e += blockDim.x) slab[e] = 0ull;
  }
  __syncthreads();
  GQS_STAMP(3);
#undef GQS_STAMP
  return GqSuper{sb, whole, s_bt, s_bc, s_total};
}
__device__ __forceinline__ GqSuper gq_super_find(const KParams& p, const unsigned* __restrict__ hist, double S,
                                                 GqSel* __restrict__ sel, unsigned long long* __restrict__ slab,
                                                 bool reset_alloc = true) {
  return gq_super_scan(p, gq_super_load(p, hist), S, sel, slab, reset_alloc);
}

// The class counts of the bins of superbins sb and sb + 1 (the crossing superbin and the room after
// it) over a block's codes: per-wave LDS copies s_h (NW x 128 bins x 4 classes, zeroed here), then
// one add per non-zero entry into copy blockIdx % kGqCopies of the global bin histograms
constexpr int kGqBinBand = 2 * (kGqBins / kGqSuper);  // bins of two superbins
template <int NC>
__device__ __forceinline__ void gq_bins_add(const uint32_t* cd, int bb, unsigned* s_h) {
  const uint32_t b0 = (uint32_t)bb;
#pragma unroll
  for (int u = 0; u < NC; ++u) {
    const uint32_t b = cd[u] >> 2;  // (NaN keys: kGqBins, past every band; ~0u: no house)
    if (b < (uint32_t)kGqBins && b >= b0 && b < b0 + kGqBinBand)
      atomicAdd(&s_h[(threadIdx.x >> 6) * (kGqBinBand * 4) + (b - b0) * 4 + (cd[u] & 3u)], 1u);
  }
}
__device__ __forceinline__ void gq_bins_flush(const unsigned* s_h, unsigned* __restrict__ hist) {
  constexpr int NW = kGqThreads / 64;
  for (int e = threadIdx.x; e < kGqBinBand * 4; e += blockDim.x) {
    unsigned v = 0u;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += s_h[w * (kGqBinBand * 4) + e];
    if (v) atomicAdd(&hist[(blockIdx.x % kGqCopies) * (kGqBinBand * 4) + e], v);
  }
}

// K2: the crossing superbin (gq_super_find), then the class counts of its bins and the next
// superbin's (gq_bins_add).  The block's codes are loaded first: they stay in flight through the
// scan.  (The next call's key map is k_gq_select's: gq_next_map.)
__global__ void __launch_bounds__(kGqThreads) k_gq_bins(KParams p, const uint32_t* __restrict__ code,
                                                        unsigned* __restrict__ hist, double S, GqSel* __restrict__ sel,
                                                        unsigned long long* __restrict__ slab) {
  constexpr int NW = kGqThreads / 64;
  __shared__ unsigned s_h[NW * kGqBinBand * 4];
  const int tid = threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i00 = (int64_t)blockIdx.x * blockDim.x + tid;
  uint32_t cd[kGqUnroll];
#pragma unroll
  for (int u = 0; u < kGqUnroll; ++u) {
    const int64_t i = i00 + u * stride;
    cd[u] = i < p.n ? code[i] : ~0u;  // (~0u: a bin past kGqBins, never counted)
  }
  const GqSuper g = gq_super_find(p, hist, S, sel, slab);
  if (g.sb >= kGqSuper || g.whole) return;  // everything taken, a NaN crossing, or one window (block-uniform)
  for (int e = tid; e < NW * kGqBinBand * 4; e += blockDim.x) s_h[e] = 0u;
  __syncthreads();
  const int bb = g.sb * (kGqBins / kGqSuper);
  gq_bins_add<kGqUnroll>(cd, bb, s_h);
  for (int64_t i0 = i00 + kGqUnroll * stride; i0 < p.n; i0 += kGqUnroll * stride) {  // (n > one pass)
#pragma unroll
    for (int u = 0; u < kGqUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      cd[u] = i < p.n ? code[i] : ~0u;
    }
    gq_bins_add<kGqUnroll>(cd, bb, s_h);
  }
  __syncthreads();
  gq_bins_flush(s_h, hist);
}

// The next call's key map (gq_bin): cells over this call's finite key range [min, max] (the
// producer's per-block parts, or the allreduced (min, -max) when nparts < 0), each cell's bins in
// proportion to this call's houses there — the superbin CDF (linear inside a superbin) at the cell
// edges, read through this call's map; then the superbin copies are zeroed for the next producer.
// One whole block of kGqThreads (k_gq_select's map block: off the decision's critical path); its
// LDS work areas are carved from `lds` (>= kGqMapLds bytes, free: the caller's window array).
constexpr int kGqMapLds = (3 * (kGqThreads / 64) + 2 + 2 * kGqSuper + kGqCells + 1) * 8 + kGqCells * 4 +
                          (kGqThreads / 64) * 8;
// The core over explicit buffers (the fused tick: the superbin copies and maps of its parities):
// sup = the superbin copies, map_in / (okmin, oscale) the map they were counted under, map_out /
// (*kmin_out, *scale_out) the next map (may alias map_in); zero_sup: zero the copies after
__device__ void gq_next_map_core(const KParams& p, unsigned* __restrict__ sup, const double* __restrict__ part,
                                 int nparts, GqSel* __restrict__ sel, const uint32_t* map_in, double okmin,
                                 double oscale, uint32_t* map_out, double* kmin_out, double* scale_out,
                                 unsigned char* lds, bool zero_sup, int sb_now, unsigned xcnt_now, int* band_out);
__device__ __forceinline__ void gq_next_map(const KParams& p, unsigned* __restrict__ hist, const double* __restrict__ part,
                            int nparts, GqSel* __restrict__ sel, uint32_t* __restrict__ map, unsigned char* lds) {
  // (xcnt: sc1 — k_gq_finish's block 0 may have just written it, past this CU's L1)
  gq_next_map_core(p, hist + kGqBins * 4, part, nparts, sel, map, sel->kmin, sel->scale, map, &sel->kmin, &sel->scale,
                   lds, true, sel->sb, ld_sc1(&sel->xcnt), &sel->band_base);
}
__device__ void gq_next_map_core(const KParams& p, unsigned* __restrict__ sup, const double* __restrict__ part,
                                 int nparts, GqSel* __restrict__ sel, const uint32_t* map_in, double okmin,
                                 double oscale, uint32_t* map_out, double* kmin_out, double* scale_out,
                                 unsigned char* lds, bool zero_sup, int sb_now, unsigned xcnt_now, int* band_out) {
  constexpr int NW = kGqThreads / 64;
  double* s_w = reinterpret_cast<double*>(lds);
  double* s_lo = s_w + NW;
  double* s_hi = s_lo + NW;
  double* s_rng = s_hi + NW;
  double* s_pre = s_rng + 2;
  double* s_cnt = s_pre + kGqSuper;
  double* s_C = s_cnt + kGqSuper;
  unsigned long long* s_wc = reinterpret_cast<unsigned long long*>(s_C + kGqCells + 1);
  uint32_t* s_map = reinterpret_cast<uint32_t*>(s_wc + NW);
  const int tid = threadIdx.x;
  unsigned long long cs = 0ull;  // this superbin's houses (tid < kGqSupN), over the copies
  if (tid < kGqSupN)
#pragma unroll
    for (int q = 0; q < kGqCopies; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(sup + q * kGqSupStride + tid * 4);
      cs += (unsigned long long)v.x + v.y + v.z + v.w;
    }
  double x = 0.0;
  unsigned long long xc = cs;
  gq_block_scan(x, xc, s_w, s_wc, (kGqSupN + 63) / 64);
  if (tid < kGqSuper) { s_pre[tid] = (double)(xc - cs); s_cnt[tid] = (double)cs; }
  if (tid < kGqCells) s_map[tid] = map_in[tid];
  double lo = INFINITY, hi = -INFINITY;
  if (nparts < 0) {  // sharded: the cluster's range, allreduced as (min, -max) (k_gq_range)
    if (tid == 0) { lo = part[0]; hi = -part[1]; }
  } else {
    for (int b = tid; b < nparts; b += blockDim.x) { lo = fmin(lo, part[2 * b]); hi = fmax(hi, part[2 * b + 1]); }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
  }
  if ((tid & 63) == 0) { s_lo[tid >> 6] = lo; s_hi[tid >> 6] = hi; }
  __syncthreads();
  if (tid == 0) {
    double kmin = s_lo[0], kmax = s_hi[0];
    for (int w = 1; w < NW; ++w) { kmin = fmin(kmin, s_lo[w]); kmax = fmax(kmax, s_hi[w]); }
    const double range = kmax - kmin;
    s_rng[0] = kmin == kmin && kmin < INFINITY ? kmin : 0.0;
    s_rng[1] = range > 0.0 && range < INFINITY ? (double)kGqCells / range : 0.0;
  }
  __syncthreads();
  const double nkmin = s_rng[0], nscale = s_rng[1];
  if (tid <= kGqCells) {
    double C = 0.0;
    if (nscale > 0.0) {
      const double u = (nkmin + (double)tid / nscale - okmin) * oscale;  // the edge, in this call's cells
      const int c = u >= (double)(kGqCells - 1) ? kGqCells - 1 : (u > 0.0 ? (int)u : 0);
      const uint32_t m = s_map[c];
      const double f = fmin(fmax(u - (double)c, 0.0), 1.0);
      const double sp = ((double)(m >> 16) + f * (double)(m & 0xFFFFu)) / (double)(kGqBins / kGqSuper);
      const int sc = sp >= (double)(kGqSuper - 1) ? kGqSuper - 1 : (sp > 0.0 ? (int)sp : 0);
      C = s_pre[sc] + fmin(fmax(sp - (double)sc, 0.0), 1.0) * s_cnt[sc];
    }
    s_C[tid] = C;
  }
  __syncthreads();
  if (tid < kGqCells) {  // B0_g = g + floor(K (C_g - C_0) / (C_G - C_0)): non-decreasing in g, so W_g >= 1
    const int NBE = gq_bins_eff(p.n_global), K = NBE - kGqCells;
    const double T = s_C[kGqCells] - s_C[0];
    auto edge = [&](int g) {
      if (g >= kGqCells) return NBE;
      if (!(T > 0.0)) return g * (NBE / kGqCells);  // (no spread seen: uniform cells)
      return g + min(K, (int)((double)K * ((s_C[g] - s_C[0]) / T)));
    };
    const int b0 = edge(tid), b1 = edge(tid + 1);
    map_out[tid] = ((uint32_t)b0 << 16) | (uint32_t)(b1 - b0);
    // the band the next producer counts: centred on the superbin the next call's crossing falls
    // into under the new map if it moves as it did since the last call (xcnt houses before it now,
    // the signal's trend: the sinusoid moves it by up to ~2 superbins a tick, tools/band_probe.py)
    // and shifted by the last prediction's error: the keys move between this call and the next
    // (the taken houses cool, the others warm), which the map of this call's keys cannot see
    // (sb_now / xcnt_now: this call's crossing superbin and the houses before its crossing bin)
    const double X1 = (double)xcnt_now, X0 = sel->xprev ? (double)(sel->xprev - 1u) : X1;
    const double X = fmin(fmax(2.0 * X1 - X0, 0.0), s_C[kGqCells]), c0 = s_C[tid], c1 = s_C[tid + 1];
    if (T > 0.0 && X >= c0 && (X < c1 || tid == kGqCells - 1)) {
      const double f = c1 > c0 ? fmin((X - c0) / (c1 - c0), 1.0) : 0.0;
      const int sbp = (b0 + (int)(f * (double)(b1 - b0))) / (kGqBins / kGqSuper);
      const int sb = sb_now;
      const int bias = sel->sb_raw >= 0 && sb < kGqSuper ? sb - sel->sb_raw : sel->sb_bias;
      sel->sb_bias = bias;
      sel->sb_raw = sbp;
      *band_out = min(max(sbp + bias - (kGqBand / 2 - 1), 0), kGqSuper - kGqBand);
    }
  }
  __syncthreads();  // (every thread has read xprev)
  if (tid == 0) sel->xprev = xcnt_now + 1u;
  if (tid == 0) { *kmin_out = nkmin; *scale_out = nscale; }  // (no later kernel of this call maps keys)
  __syncthreads();  // (every thread has read the superbin copies and the old map)
  if (zero_sup)
    for (int e = tid; e < kGqCopies * kGqSupStride; e += blockDim.x) sup[e] = 0u;
}

// K3: every block finds the crossing bin inside superbin sb (lane l = its bin l) and the candidate
// window [b*, b_end] over the next 64 bins (the same arithmetic in every block; block 0 records it
// and zeroes the superbin histograms); then every house of a bin below b* is taken, the rest start
// as not taken (k_gq_select sets the window's), the window's houses go to win[] as (okey,
// house << 2 | class, FSM word) at slots from one allocator atomic per block (unordered: select
// orders them), and the ON houses of the decided (non-window) houses are counted into the slab
__device__ bool gq_decide(const KParams& p, const uint4* __restrict__ sorted, double S, double pmin,
                          GqSel* __restrict__ sel, uint8_t* __restrict__ action, unsigned long long* __restrict__ slab,
                          uint4* s_e, bool sharded, bool ovf0, bool all, int ncand, double win_tot, bool more_after,
                          bool in_lds, const unsigned* a_add = nullptr, unsigned long long* st = nullptr);
__device__ __forceinline__ void gq_store_sc1(uint4* d, const uint4& v);
__device__ __forceinline__ uint4 gq_load_sc1(const uint4* s);
__device__ __forceinline__ bool gq_less(const uint4& a, const uint4& b);

// The candidate window from the bin counts of the crossing superbin sb and the next (k_gq_compact):
// the crossing bin b*
// (lane l = bin l), the window [b*, b_end] over the next 64 bins, the P and houses before it.  Every
// block runs the same arithmetic; block 0 records it in sel.  ovf: the fallback decides this call
// (a NaN crossing found by gq_super_find, or a crossing bin alone over kGqCap houses).
struct GqWin {
  int bs, be;          // houses of bins < bs are taken, of bins in [bs, be] are candidates
  bool ovf;
  int ncand;
  double win_tot;      // P before the window
  bool more_after;     // houses after the window
  unsigned abelow[4];  // (abins given) the A class counts of superbin sb's bins below bs
  unsigned xcnt;       // the houses before the crossing bin (GqSel.xcnt, the band's prediction)
};
// bins: the class counts of superbin sb's first bin in copy 0 (128 bins x 4 classes follow), the
// other copies at multiples of cstride: gq_bins_flush's (g_hist, 512) or the band's (k_gq_binsc).
// abins (the fused tick): the A class counts in the layout of bins; GqWin.abelow = their sums over
// superbin sb's bins below bs.
// (NC: the copies to sum, 1: counts summed by the caller; AFTER: the houses the window holds past the crossing bin)
template <int NC = kGqCopies, int AFTER = kGqAfter>
__device__ __forceinline__ GqWin gq_window(const KParams& p, const unsigned* __restrict__ bins, int cstride, double S,
                           GqSel* __restrict__ sel, int sb, bool all, bool ovf, bool whole, double base_tot,
                           unsigned long long base_cnt, unsigned long long total,
                           const unsigned* __restrict__ abins = nullptr) {
  static_assert(kGqBins / kGqSuper == 64, "one bin per lane");
  static_assert(kGqCopies * 512 <= kGqBins * 4, "the bin copies fit below the superbin copies");
  __shared__ unsigned s_c[128];
  __shared__ int s_l0, s_le, s_cnt;
  __shared__ double s_base;
  __shared__ unsigned long long s_basec;
  __shared__ unsigned s_ab[4];
  const int tid = threadIdx.x, lane = tid & 63;
  const bool on = !all && !ovf && !whole;
  const int bb = sb * 64;
  if (tid == 0) { s_l0 = 0; s_le = 0; s_cnt = 0; s_base = 0.0; s_basec = 0ull; }
  if (tid < 4) s_ab[tid] = 0u;
  if (on && tid < 128) {
    double p_on[kWinCap];
#pragma unroll
    for (int k = 0; k < kWinCap; ++k) p_on[k] = p.p_on[k < p.n_cap ? k : 0];
    unsigned long long c[kWinCap] = {0ull, 0ull, 0ull, 0ull};
    uint4 v[NC];  // (every copy's load issued before the first sum)
#pragma unroll
    for (int q = 0; q < NC; ++q) v[q] = *reinterpret_cast<const uint4*>(bins + q * cstride + tid * 4);
    uint4 va[NC];
    if (abins && tid < 64)
#pragma unroll
      for (int q = 0; q < NC; ++q) va[q] = *reinterpret_cast<const uint4*>(abins + q * cstride + tid * 4);
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      c[0] += v[q].x; c[1] += v[q].y; c[2] += v[q].z; c[3] += v[q].w;
    }
    s_c[tid] = (unsigned)(c[0] + c[1] + c[2] + c[3]);
    if (tid < 64) {  // wave 0: the crossing bin of superbin sb (it crosses: gq_super_find)
      const double pb = win_power(p, c, p_on);
      const unsigned long long cb = c[0] + c[1] + c[2] + c[3];
      double xb = pb;
      unsigned long long xcb = cb;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const double y = __shfl_up(xb, off);
        const unsigned long long yc = __shfl_up(xcb, off);
        if (lane >= off) { xb += y; xcb += yc; }
      }
      const double bef = base_tot + (xb - pb);
      const unsigned long long befc = base_cnt + (xcb - cb);
      const unsigned long long m = __ballot(cb > 0 && !(bef + pb < S));
      const int l0 = m ? __ffsll((long long)m) - 1 : 63;
      if (lane == l0) { s_l0 = l0; s_base = bef; s_basec = befc; }
      if (abins) {  // the A counts of the bins below the crossing bin
        unsigned a[4] = {0u, 0u, 0u, 0u};
        if (lane < l0)
#pragma unroll
          for (int q = 0; q < NC; ++q) { a[0] += va[q].x; a[1] += va[q].y; a[2] += va[q].z; a[3] += va[q].w; }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) a[k] += __shfl_xor(a[k], off);
        if (lane == 0)
#pragma unroll
          for (int k = 0; k < 4; ++k) s_ab[k] = a[k];
      }
    }
  }
  __syncthreads();
  if (on && tid < 64) {  // the window: bins l0 .. l0 + 63 of the 128 loaded
    const int l0 = s_l0;
    const int li = l0 + lane;
    const bool valid = li < 128 && bb + li < kGqBins;
    const unsigned long long c2 = valid ? s_c[li] : 0ull;
    unsigned long long pre = c2;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long y = __shfl_up(pre, off);
      if (lane >= off) pre += y;
    }
    const unsigned long long c0 = __shfl(c2, 0);
    const unsigned long long fit = __ballot(valid && pre <= (unsigned long long)kGqCap);
    const unsigned long long enough = __ballot(valid && pre >= c0 + AFTER) & fit;
    int le;
    if (!(fit & 1ull)) le = 0;  // the crossing bin alone overflows the window
    else if (enough) le = __ffsll((long long)enough) - 1;
    else le = 63 - __clzll((long long)fit);
    const int cnt = (int)__shfl(pre, le);
    const bool wovf = !(fit & 1ull);
    if (lane == 0) { s_le = wovf ? -1 : le; s_cnt = cnt; }
    if (lane == 0 && blockIdx.x == 0) {
      if (wovf) st_sc1(&sel->overflow, 1);
      st_sc1(&sel->bstar, bb + l0);
      st_sc1(&sel->bend, bb + l0 + le);
      st_sc1(&sel->win_tot, s_base);
      st_sc1(&sel->more_after, s_basec + (unsigned long long)cnt < total ? 1 : 0);
      st_sc1(&sel->ncand, cnt);
      st_sc1(&sel->xcnt, (unsigned)s_basec);
    }
  }
  if (!on && !whole && blockIdx.x == 0 && tid == 0) st_sc1(&sel->xcnt, (unsigned)(all ? total : base_cnt));
  if (whole && blockIdx.x == 0 && tid == 0) {  // every house is in the window
    st_sc1(&sel->bstar, 0);
    st_sc1(&sel->bend, kGqBins);
    st_sc1(&sel->win_tot, 0.0);
    st_sc1(&sel->more_after, 0);
    st_sc1(&sel->ncand, (int)total);
  }
  __syncthreads();
  GqWin w;
  w.ovf = ovf || s_le < 0;
  w.bs = whole ? -1 : bb + s_l0;
  w.be = whole ? kGqBins : bb + s_l0 + s_le;
  w.ncand = whole ? (int)total : s_cnt;
  w.win_tot = whole ? 0.0 : s_base;
  w.more_after = !whole && s_basec + (unsigned long long)s_cnt < total;
#pragma unroll
  for (int k = 0; k < 4; ++k) w.abelow[k] = s_ab[k];
  w.xcnt = (unsigned)(on ? s_basec : (all ? total : base_cnt));
  return w;
}

// A block's houses against the window (k_gq_compact): every house of a bin below bs is
// taken, the rest start as not taken (the select sets the window's), the window's houses go to win[]
// as (okey, house << 2 | class, FSM word) at slots from one allocator atomic per block (unordered:
// the select orders them), and the ON houses of the decided (non-window) houses are counted into the
// slab.  House i = b0 + u * kGqThreads + tid.
template <int U>
__device__ __forceinline__ void gq_compact_houses(const KParams& p, const uint32_t* cd, const uint32_t* hw, int64_t b0,
                                                  bool all, const GqWin& w, GqSel* __restrict__ sel,
                                                  uint4* __restrict__ win, uint8_t* __restrict__ action,
                                                  unsigned long long* __restrict__ slab) {
  constexpr int NW = kGqThreads / 64;
  __shared__ unsigned s_cnt[kWinCap];
  __shared__ unsigned s_wt[NW];
  __shared__ unsigned s_wbase;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < kWinCap) s_cnt[tid] = 0u;
  __syncthreads();
  const int bs = w.bs, be = w.be;
  unsigned oncnt[kWinCap] = {0u, 0u, 0u, 0u};
  bool inw[U];
  unsigned mine = 0u;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b0 + u * kGqThreads + tid;
    const int b = (int)(cd[u] >> 2);
    const unsigned cl = cd[u] & 3u;
    bool dec = false, take = false;  // dec: decided here (outside the window)
    inw[u] = false;
    if (i < p.n) {
      take = all || b < bs;
      action[i] = take ? 1 : 0;
      dec = all || b < bs || b > be;
      inw[u] = !dec;
    }
    mine += inw[u] ? 1u : 0u;
    const bool on1 = dec && hv_on(hvac_fsm(hw[u], take, p.dt, p.L));
#pragma unroll
    for (int c = 0; c < kWinCap; ++c) oncnt[c] += (unsigned)__popcll(__ballot(on1 && cl == (unsigned)c));
  }
  // the window houses' exact keys (issued before the allocator's round trip)
  double kk[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    kk[u] = 0.0;
  // (the loads of every u first, the subtractions after: a use right behind each conditional load
  // made the compiler wait out each pair's round trip in turn)
  double ta[U], tg[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    ta[u] = tg[u] = 0.0;
    if (inw[u]) {
      ta[u] = p.t_air[b0 + u * kGqThreads + tid];
      tg[u] = p.target[b0 + u * kGqThreads + tid];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (inw[u]) kk[u] = -(ta[u] - tg[u]);  // gq_key_of
  unsigned x = mine;  // this lane's slots: a wave prefix, the wave's offset in the block, the block's base
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_wt[wv] = x;
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < kWinCap; ++c)
      if (oncnt[c]) atomicAdd(&s_cnt[c], oncnt[c]);
  __syncthreads();
  if (wv == 0) {  // the waves' offsets by one 16-lane scan (r05: a serial loop in thread 0), the block's base
    const unsigned t = lane < NW ? s_wt[lane] : 0u;
    unsigned y = t;
#pragma unroll
    for (int off = 1; off < NW; off <<= 1) {
      const unsigned z = __shfl_up(y, off);
      if (lane >= off) y += z;
    }
    if (lane < NW) s_wt[lane] = y - t;
    if (lane == NW - 1) s_wbase = y ? atomicAdd(&sel->wcount, y) : 0u;
  }
  __syncthreads();
  unsigned j = s_wbase + s_wt[wv] + (x - mine);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!inw[u]) continue;
    const uint32_t i = (uint32_t)(p.goff + b0 + u * kGqThreads + tid);  // (global id: the order's tie-break)
    const uint64_t ok = gq_okey(kk[u]);
    if (j < (unsigned)kGqCap) gq_store_sc1(win + j, make_uint4((uint32_t)ok, (uint32_t)(ok >> 32), (i << 2) | (cd[u] & 3u), hw[u]));
    ++j;
  }
  if (slab && tid < p.n_cap && s_cnt[tid])
    atomicAdd(&slab[(blockIdx.x % kCountShards) * p.n_cap + tid], (unsigned long long)s_cnt[tid]);
}

__global__ void __launch_bounds__(kGqThreads) k_gq_compact(KParams p, const uint32_t* __restrict__ code,
                                                           unsigned* __restrict__ hist, double S, GqSel* __restrict__ sel,
                                                           uint4* __restrict__ win, uint8_t* __restrict__ action,
                                                           unsigned long long* __restrict__ slab) {
  // this block's houses first (every load before the selection reads: they stay in flight)
  const int64_t b0 = (int64_t)blockIdx.x * kGqStage;
  constexpr int U = kGqStage / kGqThreads;
  uint32_t cd[U], hw[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b0 + u * kGqThreads + threadIdx.x;
    cd[u] = i < p.n ? code[i] : 0u;
    hw[u] = i < p.n ? p.hvac[i] : 0u;
  }
  const bool all = sel->all;
  const GqWin w = gq_window(p, hist, 512, S, sel, sel->sb, all, sel->overflow != 0, sel->whole != 0, sel->base_tot,
                            sel->base_cnt, sel->total);
  if (w.ovf) return;  // the fallback (gq_exact) decides every house (block-uniform)
  gq_compact_houses<U>(p, cd, hw, b0, all, w, sel, win, action, slab);
}

// K2+K3 in one pass when the prediction holds (the single-GPU call, k_gq_compact's grid): every
// block finds the crossing superbin (gq_super_find); when the step epilogue's band holds it and
// the next superbin (band_valid; the band: gq_next_map's prediction), or no bins are needed (all
// taken, a NaN crossing, one window), the block cuts the window from the band and compacts its
// houses at once (GqSel.hit); otherwise it counts its houses' bins of the crossing superbin and
// the next (k_gq_bins' work on this grid) and k_gq_finish cuts the window and compacts.  The slab
// was zeroed by the codes' producer and the allocator by the previous call's gq_decide.
__global__ void __launch_bounds__(kGqThreads) k_gq_binsc(KParams p, const uint32_t* __restrict__ code,
                                                         unsigned* __restrict__ hist, double S, GqSel* __restrict__ sel,
                                                         uint4* __restrict__ win, uint8_t* __restrict__ action,
                                                         unsigned long long* __restrict__ slab) {
  constexpr int NW = kGqThreads / 64;
  constexpr int U = kGqStage / kGqThreads;
  __shared__ unsigned s_h[NW * kGqBinBand * 4];
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kGqStage;
  // the superbin counts and this block's houses, all issued before the scan's first wait (r05: the
  // per-load conditions of the old form made the compiler wait after every pair of superbin loads,
  // four serialised round trips)
  const GqSupLoad sup = gq_super_load(p, hist);
  const int pb = sel->band_base;
  const bool band = sel->band_valid != 0;
  uint32_t cd[U], hw[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // (unconditional, clamped: no branch, nothing waits on them yet)
    const int64_t i = b0 + u * kGqThreads + tid, ic = i < p.n ? i : p.n - 1;
    cd[u] = code[ic];
    hw[u] = p.hvac[ic];
  }
  const GqSuper g = gq_super_scan(p, sup, S, sel, nullptr, false);
#pragma unroll
  for (int u = 0; u < U; ++u)  // (~0u: a bin past kGqBins, never counted; gq_compact_houses checks i)
    if (b0 + u * kGqThreads + tid >= p.n) cd[u] = ~0u;
  const bool all = g.sb >= kGqSupN, ovf = g.sb == kGqSuper && !g.whole;
  const bool inband = band && g.sb >= pb && g.sb + 1 < pb + kGqBand;
  if (all || ovf || g.whole || inband) {  // (block-uniform)
    const unsigned* bins = inband ? hist + kGqBandOff + (g.sb - pb) * 64 * 4 : hist;
    const GqWin w = gq_window(p, bins, kGqBandWords, S, sel, g.sb, all, ovf, g.whole, g.before, g.before_cnt, g.total);
    if (blockIdx.x == 0 && tid == 0) {
      sel->hit = 1;
      atomicAdd(&sel->hits, 1u);  // (no load to wait for: a += stalled block 0 a round trip)
    }
    if (w.ovf) return;  // the fallback (gq_exact) decides every house
    gq_compact_houses<U>(p, cd, hw, b0, all, w, sel, win, action, slab);
    return;
  }
  for (int e = tid; e < NW * kGqBinBand * 4; e += blockDim.x) s_h[e] = 0u;
  __syncthreads();
  gq_bins_add<U>(cd, g.sb * (kGqBins / kGqSuper), s_h);
  __syncthreads();
  gq_bins_flush(s_h, hist);
}

// 16-B window entries handed between workgroups of one launch as two 8-B agent-scope (sc1) accesses
__device__ __forceinline__ void gq_store_sc1(uint4* d, const uint4& v) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(d);
  __hip_atomic_store(q, ((unsigned long long)v.y << 32) | v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, ((unsigned long long)v.w << 32) | v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 gq_load_sc1(const uint4* s) {
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(s);
  const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
}

__device__ __forceinline__ bool gq_less(const uint4& a, const uint4& b) {
  const uint64_t ka = ((uint64_t)a.y << 32) | a.x, kb = ((uint64_t)b.y << 32) | b.x;
  return ka < kb || (ka == kb && a.z < b.z);  // (z = house << 2 | class: house order on equal keys)
}

// the greedy take rule at one house (greedy_myopic_controller.py:93-101)
__device__ __forceinline__ bool gq_take(double pj, double tot, double S, bool lock) {
  return (pj + tot < S) || (fabs(pj + tot - S) < fabs(tot - S) && !lock);
}
// the walk is over once no class can be taken (P > 0: nothing once tot >= S; with gap g = S - tot a
// house needs P < 2g — a conservative margin, the exact rule decides)
__device__ __forceinline__ bool gq_walk_over(double tot, double S, double pmin) {
  return !(tot < S) || 2.0 * (S - tot) < pmin * (1.0 - 1e-9);
}

// 96-bit (okey, house) order for the exact fallback
struct GqKey {
  uint64_t k;
  uint32_t h;
};
__device__ __forceinline__ bool gq_key_less(const GqKey& a, const GqKey& b) {
  return a.k < b.k || (a.k == b.k && a.h < b.h);
}
// digit L (0 = most significant) of the 96-bit key, 8 bits each
__device__ __forceinline__ unsigned gq_digit(const GqKey& c, int L) {
  return L < 8 ? (unsigned)(c.k >> (56 - 8 * L)) & 0xFFu : (c.h >> (24 - 8 * (L - 8))) & 0xFFu;
}
// the top 8L bits of the key equal those of the prefix
__device__ __forceinline__ bool gq_prefix_eq(const GqKey& c, const GqKey& pre, int L) {
  if (L == 0) return true;
  if (L <= 8) {
    const int sh = 64 - 8 * L;
    return sh == 0 ? c.k == pre.k : (c.k >> sh) == (pre.k >> sh);
  }
  const int sh = 32 - 8 * (L - 8);
  return c.k == pre.k && (c.h >> sh) == (pre.h >> sh);
}

// The exact decision of the whole cluster by one workgroup, for what the window cannot decide:
// (1) the crossing house k (the first position where the cumulative P of the (key, house) order
// reaches S) by a radix select over the 96-bit key, 12 passes of 8 bits over all houses with class
// counts (exact P); (2) the gap walk from k: each pass takes the first house after the current one
// that the take rule admits (the houses in between fail it, and a failing house changes nothing),
// until the gap admits no class; (3) every house's action and the ON counts of the decided actions.
// ~15 passes over the keys by one CU: milliseconds, for inputs the window form cannot take (a NaN
// crossing, a crossing bin of more than kGqCap houses, a walk past the window).
__device__ void gq_exact(const KParams& p, double S, double pmin, uint8_t* __restrict__ action,
                         unsigned long long* __restrict__ slab) {
  __shared__ unsigned s_h[256 * 4];
  __shared__ double s_w[16];
  __shared__ unsigned long long s_wc[16];
  __shared__ int s_d;
  __shared__ double s_base;
  __shared__ GqKey s_best[16];
  __shared__ int s_ntake, s_all;
  __shared__ uint32_t s_take[64];
  __shared__ unsigned s_cnt[kWinCap];
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, wv = tid >> 6;
  const int64_t n = p.n;
  double p_on[kWinCap];
#pragma unroll
  for (int k = 0; k < kWinCap; ++k) p_on[k] = p.p_on[k < p.n_cap ? k : 0];
  auto key_of = [&](int64_t i) { return GqKey{gq_okey(gq_key_of(p, i)), (uint32_t)i}; };
  GqKey pre{0ull, 0u};
  double base = 0.0;
  if (tid == 0) { s_all = 0; s_ntake = 0; }
  for (int L = 0; L < 12; ++L) {
    for (int e = tid; e < 256 * 4; e += nth) s_h[e] = 0u;
    __syncthreads();
    for (int64_t i = tid; i < n; i += nth) {
      const GqKey c = key_of(i);
      if (gq_prefix_eq(c, pre, L)) atomicAdd(&s_h[gq_digit(c, L) * 4 + (p.cap_idx[i] & 3u)], 1u);
    }
    __syncthreads();
    unsigned long long c4[kWinCap] = {0ull, 0ull, 0ull, 0ull};
    if (tid < 256)
#pragma unroll
      for (int k = 0; k < kWinCap; ++k) c4[k] = s_h[tid * 4 + k];
    const double pd = win_power(p, c4, p_on);
    const unsigned long long cd = c4[0] + c4[1] + c4[2] + c4[3];
    double x = pd;
    unsigned long long xc = cd;
    if (tid == 0) s_d = 256;
    gq_block_scan(x, xc, s_w, s_wc, 256 / 64);
    {  // (one LDS atomic per wave: same-address LDS atomics serialise)
      const unsigned long long m = __ballot(tid < 256 && cd > 0 && !(base + (x - pd) + pd < S));
      if (m && (tid & 63) == 0) atomicMin(&s_d, (tid & ~63) + __ffsll((long long)m) - 1);
    }
    __syncthreads();
    const int d = s_d;
    if (d >= 256) {  // (L = 0 only: the whole cluster's P stays below S) everything is taken
      if (tid == 0) s_all = 1;
      break;
    }
    if (tid == d) s_base = base + (x - pd);
    __syncthreads();
    base = s_base;
    if (L < 8) pre.k |= (uint64_t)d << (56 - 8 * L);
    else pre.h |= (uint32_t)d << (24 - 8 * (L - 8));
    __syncthreads();  // (s_d / s_base reused by the next level)
  }
  const bool all = s_all != 0;
  // (2) the walk from the crossing house pre (its own take first)
  if (!all) {
    double tot = base;
    GqKey cur = pre;
    bool first = true;
    for (int guard = 0; guard < 64; ++guard) {
      if (gq_walk_over(tot, S, pmin)) break;
      GqKey best{~0ull, ~0u};
      bool found = false;
      if (first) {
        const int64_t i = pre.h;
        found = gq_take(p_on[p.cap_idx[i] & 3u], tot, S, hv_lock(p.hvac[i]));
        best = pre;
      } else {
        for (int64_t i = tid; i < n; i += nth) {
          const GqKey c = key_of(i);
          if (!gq_key_less(cur, c)) continue;
          if (!gq_take(p_on[p.cap_idx[i] & 3u], tot, S, hv_lock(p.hvac[i]))) continue;
          if (gq_key_less(c, best)) best = c;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          const GqKey o{(uint64_t)__shfl_xor((long long)best.k, off), (uint32_t)__shfl_xor((int)best.h, off)};
          if (gq_key_less(o, best)) best = o;
        }
        if (lane == 0) s_best[wv] = best;
        __syncthreads();
        best = s_best[0];
        for (int w = 1; w < (nth >> 6); ++w)
          if (gq_key_less(s_best[w], best)) best = s_best[w];
        __syncthreads();
        found = best.k != ~0ull || best.h != ~0u;
      }
      if (found) {
        if (tid == 0) s_take[s_ntake] = best.h;
        tot += p_on[p.cap_idx[best.h] & 3u];
        __syncthreads();
        if (tid == 0) s_ntake += 1;
        cur = best;
      } else if (!first) {
        break;  // no house after cur is admitted
      }
      first = false;
      __syncthreads();
    }
  }
  // (3) every house's action and the ON counts of the decided actions
  if (tid < kWinCap) s_cnt[tid] = 0u;
  for (int e = tid; e < kCountShards * p.n_cap; e += nth) slab[e] = 0ull;
  __syncthreads();
  const int ntake = s_ntake;
  unsigned oncnt[kWinCap] = {0u, 0u, 0u, 0u};
  for (int64_t i0 = 0; i0 < n; i0 += nth) {
    const int64_t i = i0 + tid;
    bool on1 = false;
    unsigned cl = 0u;
    if (i < n) {
      bool take = all || gq_key_less(key_of(i), pre);
      for (int t = 0; t < ntake; ++t) take = take || s_take[t] == (uint32_t)i;
      action[i] = take ? 1 : 0;
      cl = p.cap_idx[i] & 3u;
      on1 = hv_on(hvac_fsm(p.hvac[i], take, p.dt, p.L));
    }
#pragma unroll
    for (int c = 0; c < kWinCap; ++c) oncnt[c] += (unsigned)__popcll(__ballot(on1 && cl == (unsigned)c));
  }
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < kWinCap; ++c)
      if (oncnt[c]) atomicAdd(&s_cnt[c], oncnt[c]);
  __syncthreads();
  if (tid < p.n_cap) slab[tid] = s_cnt[tid];  // (shard 0; the others stay zero)
}

// The decision on the sorted window (k_gq_select's last block): the window into LDS, the exact
// crossing position from win_tot, the window's prefix taken, then the gap walk (k_greedy_walk's
// rule); the ON counts of the window's decided actions; what the window cannot decide goes to
// gq_exact (sharded: to the host, GqSel.need_fb — one shard cannot order the whole cluster).  The
// window carries global house ids: only this shard's houses are written (offset p.goff).
// a_add (the fused tick): every window house's byte is written (0 or 1: the step reads the window's
// bytes only), and a_add[k] (the ON houses of the decided houses outside the window) joins class k's count
// (returns true when the window could not decide: gq_exact decided, or sharded, the host must)
__device__ bool gq_decide(const KParams& p, const uint4* __restrict__ sorted, double S, double pmin,
                          GqSel* __restrict__ sel, uint8_t* __restrict__ action, unsigned long long* __restrict__ slab,
                          uint4* s_e, bool sharded, bool ovf0, bool all, int ncand, double win_tot, bool more_after,
                          bool in_lds, const unsigned* a_add, unsigned long long* st) {
  __shared__ uint8_t s_tk[kGqCap];
#define GQD_STAMP(k) \
  do { if (st && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
  __shared__ double s_tot;
  __shared__ int s_k, s_ovf;
  __shared__ unsigned s_cnt[kWinCap];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nth = blockDim.x;
  double pon[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) pon[k] = p.p_on[k < p.n_cap ? k : 0];
  auto P_of = [&](uint32_t z) {
    const uint32_t cl = z & 3u;
    return cl == 0u ? pon[0] : cl == 1u ? pon[1] : cl == 2u ? pon[2] : pon[3];
  };
  bool ovf = ovf0;
  if (!all && !ovf) {
    {
      constexpr int U = kGqCap / 1024;  // (blockDim 1024: every load issued before the LDS stores)
      uint4 v[U];
      if (!in_lds) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int e = tid + u * 1024;
          if (e < ncand) v[u] = gq_load_sc1(sorted + e);  // (sc1: written by other workgroups of this launch)
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = tid + u * 1024;
        if (e < ncand) {
          if (!in_lds) s_e[e] = v[u];
          s_tk[e] = 0;
        }
      }
    }
    if (tid < kWinCap) s_cnt[tid] = 0u;
    __syncthreads();
    GQD_STAMP(0);
    // the crossing: the first house whose running P reaches S, by wave 0 alone, 64 houses a wave
    // prefix with the running total carried between them (r04: block-wide prefixes, four barriers a
    // round); sums of integer-valued P are exact in any order
    if (wv == 0) {
      double tot = win_tot;
      int kk = -1;
      for (int c0 = 0; c0 < ncand; c0 += 64) {  // (wave-uniform)
        const int j = c0 + lane;
        const double pj = j < ncand ? P_of(s_e[j].z) : 0.0;
        double x = pj;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const double y = __shfl_up(x, off);
          if (lane >= off) x += y;
        }
        const unsigned long long bl = __ballot(j < ncand && !(tot + x < S));
        if (bl) {
          const int f = __ffsll((long long)bl) - 1;
          kk = c0 + f;
          tot = tot + (__shfl(x, f) - __shfl(pj, f));  // (exclusive: the P before house kk)
          break;
        }
        tot = tot + __shfl(x, 63);  // the round's total (houses past ncand add 0)
      }
      if (lane == 0) {
        s_k = kk;
        s_tot = tot;
      }
    }
    __syncthreads();
    GQD_STAMP(1);
    const int k = s_k;  // >= 0: the crossing lies in bin b*, inside the window
    for (int j = tid; j < (k < 0 ? ncand : k); j += nth) s_tk[j] = 1;
    if (k < 0) {
      if (tid == 0) s_ovf = 1;
    } else {
      // the gap walk from the crossing (k_greedy_walk's rule, in the reference's order): tot changes
      // only at a take, so each step is a search for the first house after the last take that the
      // rule admits — by wave 0 alone, 64 houses a ballot, no block barrier per step (r04: block-wide
      // searches, three barriers a take; r03: one thread stepping house by house).  Every lane
      // carries the same tot: the sums happen in take order.
      if (wv == 0) {
        double tot = s_tot;
        int j0 = k;
        bool over = false;
        for (;;) {
          if (gq_walk_over(tot, S, pmin)) {
            over = true;
            break;
          }
          int f = -1;
          for (int c = j0; c < ncand; c += 64) {  // (wave-uniform)
            const int e = c + lane;
            const bool ok = e < ncand && gq_take(P_of(s_e[e].z), tot, S, hv_lock(s_e[e].w));
            const unsigned long long m = __ballot(ok);
            if (m) {
              f = c + __ffsll((long long)m) - 1;
              break;
            }
          }
          if (f < 0) break;  // no house left in the window: the walk reaches its end
          if (lane == 0) s_tk[f] = 1;
          tot += P_of(s_e[f].z);
          j0 = f + 1;
        }
        if (lane == 0) s_ovf = (!over && more_after && !gq_walk_over(tot, S, pmin)) ? 1 : 0;
      }
    }
    __syncthreads();
    GQD_STAMP(2);
    ovf = s_ovf != 0;
    if (!ovf) {  // the window's actions and the ON counts they produce
      unsigned oncnt[kWinCap] = {0u, 0u, 0u, 0u};
      for (int j0 = 0; j0 < ncand; j0 += nth) {
        const int j = j0 + tid;
        bool on1 = false;
        unsigned cl = 0u;
        if (j < ncand) {
          const uint4 e = s_e[j];
          const bool take = s_tk[j] != 0;
          const int64_t li = (int64_t)(e.z >> 2) - p.goff;
          if ((take || a_add) && li >= 0 && li < p.n) action[li] = take ? 1 : 0;
          cl = e.z & 3u;
          on1 = hv_on(hvac_fsm(e.w, take, p.dt, p.L));
        }
#pragma unroll
        for (int c = 0; c < kWinCap; ++c) oncnt[c] += (unsigned)__popcll(__ballot(on1 && cl == (unsigned)c));
      }
      if (lane == 0)
#pragma unroll
        for (int c = 0; c < kWinCap; ++c)
          if (oncnt[c]) atomicAdd(&s_cnt[c], oncnt[c]);
      __syncthreads();
      const unsigned add = tid < p.n_cap ? s_cnt[tid] + (a_add ? a_add[tid] : 0u) : 0u;
      if (slab && tid < p.n_cap && add) atomicAdd(&slab[tid], (unsigned long long)add);
      GQD_STAMP(3);
    }
  }
#undef GQD_STAMP
  if (ovf && !sharded) gq_exact(p, S, pmin, action, slab);
  if (tid == 0) {  // (counters as atomics: a += would hold the launch's end behind a load's round trip)
    if (ovf) atomicAdd(&sel->fallbacks, 1u);
    if (ovf && sharded) sel->need_fb = 1u;
    sel->overflow = 0;       // (the next call starts clear)
    sel->wcount = 0u;
    atomicAdd(&sel->calls, 1u);
    if (!all && !ovf) atomicAdd(&sel->ncand_sum, (unsigned long long)ncand);
  }
  return ovf;
}




// the bin copies and the band copies after them (read by compact / binsc), a slice per block of
// the launch (a whole-region loop in block 0 made it the ticket's last arrival and delayed the
// decision); only where no block of the launch reads them
__device__ __forceinline__ void gq_zero_bins_sliced(unsigned* __restrict__ hist) {
  static_assert(kGqBandOff == kGqCopies * 512, "the band copies follow the bin copies");
  for (int e = (int)(blockIdx.x * blockDim.x + threadIdx.x); e < kGqBandOff + kGqCopies * kGqBandWords;
       e += (int)(gridDim.x * blockDim.x))
    hist[e] = 0u;
}

// The window's houses ranked by the launch's waves (k_gq_select): wave w of the grid
// takes entries w, w + waves, ... of s_e[0, ncand) (the window in LDS) and counts how many entries
// precede each in (key, house) order, the lanes splitting the comparisons (one LDS read serves all
// of the wave's entries); the entry goes to sorted[rank] (sc1: read by the deciding block)
// Block 0 ranks nothing when the grid has others: it takes its ticket first and builds the next
// call's map beside the decision (as the deciding block it would run the map after the decision).
__device__ void gq_rank(const uint4* s_e, int ncand, uint4* __restrict__ sorted) {
  const int lane = threadIdx.x & 63, wpb = (int)(blockDim.x >> 6);
  const int b0 = gridDim.x > 1 ? 1 : 0;
  if ((int)blockIdx.x < b0) return;
  const int nwv = ((int)gridDim.x - b0) * wpb;
  for (int e = ((int)blockIdx.x - b0) * wpb + (int)(threadIdx.x >> 6); e < ncand; e += nwv) {  // (wave-uniform)
    const uint4 me = s_e[e];
    unsigned r = 0u;
#pragma unroll 2
    for (int f = lane; f < ncand; f += 64) r += gq_less(s_e[f], me) ? 1u : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
    if (lane == 0 && r < (unsigned)kGqCap) gq_store_sc1(sorted + r, me);
  }
}

// K4 (kGqSelBlocks workgroups of 1024): every block loads compact's unordered window win[0, ncand)
// into LDS and ranks kGqCap / (kGqSelBlocks * 16) of its houses per wave (how many window houses
// precede it in (key, house) order, the lanes splitting the comparisons; one LDS read serves all of
// the wave's houses) into sorted[rank]; the last block to take a ticket (sc1 hand-off below: every
// block's sorted[] is visible to it) then decides (gq_decide).  Block 0 zeroes the bin
// histograms (k_gq_compact read them).  Sharded (gathered != null): the window is the ranks'
// all-gathered windows, rank r's at gathered[r * (kGqCap + 1)]: {count, -, -, -} then its entries.
__global__ void __launch_bounds__(1024) k_gq_select(KParams p, const uint4* __restrict__ win, uint4* __restrict__ sorted,
                                                    double S, double pmin, GqSel* __restrict__ sel,
                                                    uint8_t* __restrict__ action, unsigned long long* __restrict__ slab,
                                                    unsigned* __restrict__ hist, const uint4* __restrict__ gathered,
                                                    int world, unsigned* __restrict__ tickets,
                                                    const double* __restrict__ part, int nparts, uint32_t* __restrict__ map) {
  __shared__ uint4 s_e[kGqCap];
  __shared__ int s_off[kGqMaxRanks + 1];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  gq_zero_bins_sliced(hist);
  if (blockIdx.x == 0 && tid == 0) sel->band_valid = 0;
  bool ovf0 = sel->overflow;
  bool live = !sel->all && !ovf0;
  const int ncand = sel->ncand;
  if (gathered) {  // the ranks' window offsets (the counts must add up to the cluster's ncand)
    if (tid == 0) {
      int o = 0;
      for (int r = 0; r < world; ++r) {
        s_off[r] = o;
        o += (int)gathered[(size_t)r * (kGqCap + 1)].x;
      }
      s_off[world] = o;
    }
    __syncthreads();
    if (live && s_off[world] != ncand) {  // (block-uniform; cannot happen with consistent histograms)
      live = false;
      ovf0 = true;  // (decided by the host's fallback)
    }
  }
  if (live) {
    for (int e = tid; e < ncand; e += (int)blockDim.x) {  // (one load per thread up to 1,024 houses)
      if (gathered) {
        int r = 0;
        while (r + 1 < world && s_off[r + 1] <= e) ++r;
        s_e[e] = gathered[(size_t)r * (kGqCap + 1) + 1 + (e - s_off[r])];
      } else {
        s_e[e] = win[e];
      }
    }
    __syncthreads();
    gq_rank(s_e, ncand, sorted);
  }
  // the hand-off to the last block (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md
  // Valid forms): every sorted[] store is sc1 and drained by its wave before the workgroup barrier
  // and the block's agent-scope ticket add (grid_last_block); the last block loads sorted[] only
  // with sc1 loads (gq_decide), so no fence is needed
  if (grid_last_block(tickets)) {  // (block-uniform)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler ordering only)
    gq_decide(p, sorted, S, pmin, sel, action, slab, s_e, gathered != nullptr, ovf0, sel->all != 0, ncand,
              sel->win_tot, sel->more_after != 0, false);
  }
  // the next call's key map, by block 0 (dispatched first, it is rarely the last to take a ticket:
  // the map's ~2 us run beside the decision instead of before it, as they did in k_gq_bins)
  static_assert(kGqMapLds <= (int)sizeof(s_e), "the map's work areas fit the window array");
  if (blockIdx.x == 0) {
    __syncthreads();  // (a decision by this block has finished with s_e)
    gq_next_map(p, hist, part, nparts, sel, map, reinterpret_cast<unsigned char*>(s_e));
  }
}

// The window s_e[0, ncand) sorted in LDS by one block: a bitonic network over the next power of two
// (sentinels past ncand sort last), log2(P)(log2(P)+1)/2 barriers — bounded at any window size, where a
// rank by counting is quadratic in it.  (ncand <= kGqCap; the caller wrote s_e[0, ncand) before.)
__device__ void gq_sort_lds(uint4* s_e, int ncand) {
  const int tid = threadIdx.x;
  int np2 = 1;
  while (np2 < ncand) np2 <<= 1;
  for (int e = ncand + tid; e < np2; e += (int)blockDim.x) s_e[e] = make_uint4(~0u, ~0u, ~0u, ~0u);
  __syncthreads();
  for (int k2 = 2; k2 <= np2; k2 <<= 1)
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < np2; i += (int)blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const uint4 a = s_e[i], b = s_e[l];
          if ((i & k2) == 0 ? gq_less(b, a) : gq_less(a, b)) {
            s_e[i] = b;
            s_e[l] = a;
          }
        }
      }
      __syncthreads();
    }
}

// K3 of the single-GPU call after k_gq_binsc, in place of k_gq_compact + k_gq_select (one launch
// fewer on every call: the host cannot know whether binsc compacted).  GqSel.hit (binsc cut the window
// from the band and compacted): the blocks rank the window as k_gq_select does and the last block
// decides.  Otherwise (a band miss: binsc counted the bins): every block cuts the window from the bin
// copies (gq_window, as k_gq_compact) and compacts its stages blockIdx, blockIdx + grid, ...; the last
// block then ranks the whole window alone (one thread per house against the window in LDS: a miss is
// rare) and decides.  Every block reads hit / the window state before its ticket; only the last block
// (after every ticket) resets them.  Block 0 builds the next call's key map after its ticket.
__global__ void __launch_bounds__(1024) k_gq_finish(KParams p, const uint32_t* __restrict__ code,
                                                    uint4* __restrict__ win, uint4* __restrict__ sorted, double S,
                                                    double pmin, GqSel* __restrict__ sel, uint8_t* __restrict__ action,
                                                    unsigned long long* __restrict__ slab, unsigned* __restrict__ hist,
                                                    unsigned* __restrict__ tickets, const double* __restrict__ part,
                                                    int nparts, uint32_t* __restrict__ map) {
  static_assert(kGqThreads == 1024, "the miss path compacts with gq_compact_houses' block shape");
  __shared__ uint4 s_e[kGqCap];
  const int tid = threadIdx.x;
  // the window's first 1,024 slots are loaded before the window's size is known (beside the GqSel
  // reads: one round trip instead of two; slots past the size are never used)
  const uint4 w0 = win[tid];
  const bool hit = sel->hit != 0;
  const bool all = sel->all != 0;
  bool ovf;
  int ncand;
  double win_tot;
  bool more_after;
  if (hit) {
    gq_zero_bins_sliced(hist);  // (nobody reads the bins or the band on this path)
    ovf = sel->overflow != 0;
    ncand = sel->ncand;
    win_tot = sel->win_tot;
    more_after = sel->more_after != 0;
    if (!all && !ovf) {
      if (tid < ncand) s_e[tid] = w0;
      for (int e = tid + (int)blockDim.x; e < ncand; e += (int)blockDim.x) s_e[e] = win[e];  // (> 1,024)
      __syncthreads();
      gq_rank(s_e, ncand, sorted);
    }
  } else {
    const GqWin w = gq_window(p, hist, 512, S, sel, sel->sb, all, sel->overflow != 0, sel->whole != 0,
                              sel->base_tot, sel->base_cnt, sel->total);
    ovf = w.ovf;
    ncand = w.ncand;
    win_tot = w.win_tot;
    more_after = w.more_after;
    if (!ovf) {
      constexpr int U = kGqStage / kGqThreads;
      const int nstage = (int)((p.n + kGqStage - 1) / kGqStage);
      for (int b = (int)blockIdx.x; b < nstage; b += (int)gridDim.x) {  // (block-uniform)
        const int64_t b0 = (int64_t)b * kGqStage;
        uint32_t cd[U], hw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t i = b0 + u * kGqThreads + tid;
          cd[u] = i < p.n ? code[i] : 0u;
          hw[u] = i < p.n ? p.hvac[i] : 0u;
        }
        gq_compact_houses<U>(p, cd, hw, b0, all, w, sel, win, action, slab);
        __syncthreads();  // (gq_compact_houses' LDS is reused by the next stage)
      }
    }
  }
  // hand-offs to the last block: sorted[] (hit) or win[] (miss), every store sc1 and drained before
  // the ticket (grid_last_block), every load of them there sc1
  if (grid_last_block(tickets)) {  // (block-uniform)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler ordering only)
    if (!hit) {
      if (!all && !ovf) {
        for (int e = tid; e < ncand; e += (int)blockDim.x) s_e[e] = gq_load_sc1(win + e);
        gq_sort_lds(s_e, ncand);
      }
      for (int e = tid; e < kGqBandOff + kGqCopies * kGqBandWords; e += (int)blockDim.x) hist[e] = 0u;
    }
    if (tid == 0) {
      sel->hit = 0;
      sel->band_valid = 0;
    }
    // (a hit's window is in sorted[], ranked by every block; a miss's is in s_e, sorted here)
    gq_decide(p, sorted, S, pmin, sel, action, slab, s_e, false, ovf, all, ncand, win_tot, more_after, !hit);
  }
  if (blockIdx.x == 0) {
    __syncthreads();  // (a decision by this block has finished with s_e)
    gq_next_map(p, hist, part, nparts, sel, map, reinterpret_cast<unsigned char*>(s_e));
  }
}


// ---- the fused greedy tick (mdr_greedy_rollout; mdr_kernels.h GqfBufs)
// A house's window entry: (okey, global id << 2 | class, FSM word) — gq_compact_houses' format.
__device__ __forceinline__ uint4 gqf_entry(double k, int64_t gid, unsigned cls, uint32_t w) {
  const uint64_t ok = gq_okey(k);
  return make_uint4((uint32_t)ok, (uint32_t)(ok >> 32), ((uint32_t)gid << 2) | (cls & 3u), w);
}
// A: the house can turn on at the next step (hvac_fsm: not locked out after "if not on: sso += dt")
__device__ __forceinline__ bool gqf_canon(uint32_t w, const KParams& p) {
  const uint32_t Lu = p.L < 0 ? 0u : (uint32_t)p.L;
  return hv_on(w) || hv_sso(w) + (uint32_t)p.dt >= Lu;
}

// The window's houses from (bin, copy) buckets into s_e[0, total), in (key, house) order: pair q = (bin
// bi0 + q / kGqCopies, copy q % kGqCopies) holds cnt(q) entries at src(q); the pairs' exclusive offsets by
// one block scan, then every thread fetches up to kGqCap / blockDim entries, each located by a binary
// search over the offsets (all loads issued before the LDS stores).  The entries land bin-major, and a
// bin's keys all precede the next bin's (gq_bin is monotone in the key), so each entry's rank is its
// bin's offset plus the entries of its own bin that order before it (~tens of comparisons, not a sort
// of the window); each thread then stores its entries at their ranks.  SC1: entries written by other
// workgroups of this launch.  Returns the total (> kGqCap: nothing ordered, the caller falls back).
template <bool SC1, typename CntF, typename SrcF>
__device__ int gqf_gather(uint4* s_e, int npair, CntF cnt_of, SrcF src_of, unsigned long long* st = nullptr) {
#define GQG_STAMP(k) \
  do { if (st && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
  constexpr int U = kGqCap / 1024;
  __shared__ unsigned s_poff[kGqCopies * 64 + 1];
  __shared__ unsigned s_ws[16];
  const int tid = threadIdx.x, lane = tid & 63;
  const unsigned cnt = tid < npair ? cnt_of(tid) : 0u;
  unsigned x = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_ws[tid >> 6] = x;
  __syncthreads();
  unsigned base = 0u;
  for (int k = 0; k < (tid >> 6); ++k) base += s_ws[k];
  if (tid < npair) s_poff[tid] = base + x - cnt;
  if (tid == npair) s_poff[npair] = base + x - cnt;  // (the total: thread npair holds cnt 0)
  __syncthreads();
  const unsigned total = s_poff[npair];
  GQG_STAMP(0);
  if (st && threadIdx.x == 0) { st[3] = (unsigned long long)npair; st[4] = total; }
  if (total > (unsigned)kGqCap) return (int)total;  // (block-uniform)
  const int nf = (int)total;
  uint4 v[U];
  int q[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * (int)blockDim.x;
    q[u] = 0;
    if (e < nf) {
      int lo = 0, hi = npair - 1;  // the last pair whose offset <= e
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_poff[mid] <= (unsigned)e) lo = mid;
        else hi = mid - 1;
      }
      q[u] = lo;
      const uint4* src = src_of(lo) + (e - (int)s_poff[lo]);
      v[u] = SC1 ? gq_load_sc1(src) : *src;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * (int)blockDim.x;
    if (e < nf) s_e[e] = v[u];
  }
  __syncthreads();
  GQG_STAMP(1);
  unsigned r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * (int)blockDim.x;
    r[u] = 0u;
    if (e < nf) {
      const int b0 = q[u] - q[u] % kGqCopies, b1 = min(b0 + kGqCopies, npair);
      const int lo = (int)s_poff[b0], len = (int)s_poff[b1] - lo;
      // the keys alone first (2 VALU a comparison: wave64 VALU is the bound here, r06 stamps), 8 LDS
      // reads in flight a round, the rounds' tail by clamped re-reads of the bin's last entry counted
      // once below; equal keys (the entry itself, or ties: rare) by house id in a second pass
      uint32_t mx = v[u].x, my = v[u].y, mz = v[u].z;
      asm volatile("" : "+v"(mx), "+v"(my), "+v"(mz));
      const uint64_t mk = ((uint64_t)my << 32) | mx;
      const uint64_t* kb = reinterpret_cast<const uint64_t*>(s_e + lo);  // (the key: the entry's first 8 bytes)
      unsigned lt = 0u, eq = 0u;
      const int full8 = len & ~7;
      for (int f0 = 0; f0 < full8; f0 += 8) {
        uint64_t t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = kb[2 * (f0 + j)];
        __builtin_amdgcn_sched_barrier(0);  // (all 8 reads issued before the first compare waits)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          lt += t[j] < mk ? 1u : 0u;
          eq += t[j] == mk ? 1u : 0u;
        }
      }
      for (int f = full8; f < len; ++f) {
        const uint64_t t = kb[2 * f];
        lt += t < mk ? 1u : 0u;
        eq += t == mk ? 1u : 0u;
      }
      unsigned k = (unsigned)lo + lt;
      if (eq > 1u)  // (ties: the house order among the equal keys)
        for (int f = 0; f < len; ++f) {
          const uint4 t = s_e[lo + f];
          k += (((uint64_t)t.y << 32) | t.x) == mk && t.z < mz ? 1u : 0u;
        }
      r[u] = k;
    }
  }
  GQG_STAMP(5);
  __syncthreads();
  GQG_STAMP(6);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = tid + u * (int)blockDim.x;
    if (e < nf) s_e[r[u]] = v[u];
  }
  __syncthreads();
  GQG_STAMP(2);
#undef GQG_STAMP
  return (int)total;
}

// The producer without a step (a rollout's first decision, or after the state changed): the current
// state's keys under parity par's map into parity region par (zeroed before, k_zero_u64), as the
// GQ = 2 step epilogue writes them.  A block per kGqStage houses (its packed LDS counts < 2^16);
// block 0 zeroes the slab the decision is counted into.
__global__ void __launch_bounds__(kGqThreads) k_gq_keys2(KParams p, GqfBufs fz, int par, double* __restrict__ part,
                                                         unsigned long long* __restrict__ slab) {
  constexpr int U = kGqStage / kGqThreads;
  __shared__ unsigned s_sh[4 * kGqSupStride];
  __shared__ uint32_t s_map[kGqCells];
  __shared__ unsigned s_acnt[8];
  const int tid = threadIdx.x;
  for (int e = tid; e < 4 * kGqSupStride; e += blockDim.x) s_sh[e] = 0u;
  if (tid < 8) s_acnt[tid] = 0u;
  for (int e = tid; e < kGqCells; e += blockDim.x) s_map[e] = fz.map[par][e];
  if (blockIdx.x == 0 && slab)
    for (int e = tid; e < kCountShards * p.n_cap; e += blockDim.x) slab[e] = 0ull;
  __syncthreads();
  const double kmin = fz.sel->fkmin[par], scale = fz.sel->fscale[par];
  const uint32_t band0 = (uint32_t)fz.sel->fband[par] * 64u;
  const int cp = (int)(blockIdx.x % kGqCopies);
  unsigned* R = fz.par[par];
  unsigned* bandC = R + kGqfOffBandC + cp * kGqBandWords;
  unsigned* bandA = R + kGqfOffBandA + cp * kGqBandWords;
  unsigned* bandN = R + kGqfOffBandN + cp * (kGqBand * 64);
  uint4* bkt = fz.bkt[par] + (size_t)cp * (kGqBand * 64) * fz.cap;
  double lo = INFINITY, hi = -INFINITY;
  GqfAcnt acnt{0u, 0u, 0u, 0u};
  const int64_t b0 = (int64_t)blockIdx.x * kGqStage;
  double ta[U], tg[U];
  uint32_t hw[U];
  unsigned cl[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b0 + u * kGqThreads + tid, ic = i < p.n ? i : p.n - 1;
    ta[u] = p.t_air[ic];
    tg[u] = p.target[ic];
    hw[u] = p.hvac[ic];
    cl[u] = p.cap_idx[ic];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = b0 + u * kGqThreads + tid;
    if (i >= p.n) break;
    const double k = -(ta[u] - tg[u]);  // gq_key_of
    const uint32_t c = gq_code(k, kmin, scale, s_map, cl[u]);
    if (k == k) {
      lo = fmin(lo, k);
      hi = fmax(hi, k);
    }
    const bool canon = gqf_canon(hw[u], p);
    atomicAdd(&s_sh[((tid >> 6) & 3) * kGqSupStride + (c >> 8) * 4 + (c & 3u)], 1u);
    gqf_acount(acnt, canon, (c >> 2) < band0, c & 3u);
    const uint32_t bo = (c >> 2) - band0;
    if (bo < (uint32_t)(kGqBand * 64)) {
      atomicAdd(&bandC[bo * 4 + (c & 3u)], 1u);
      if (canon) atomicAdd(&bandA[bo * 4 + (c & 3u)], 1u);
      const unsigned slot = atomicAdd(&bandN[bo], 1u);
      if (slot < (unsigned)fz.cap) bkt[(size_t)bo * fz.cap + slot] = gqf_entry(k, p.goff + i, c, hw[u]);
      else atomicOr(&R[kGqfOffFlags], 1u);
    }
  }
  gqf_acount_wave(acnt, s_acnt);
  __syncthreads();
  gqf_flush(s_sh, 4, R, lo, hi, part, s_acnt);
}

// The fused decision (kGqSelBlocks blocks of 1024): from parity par's counts (its producer: the
// previous step's epilogue or k_gq_keys2) every block finds the crossing superbin (gq_super_scan); then
//  * band hit (the producer's band holds superbins sb and sb + 1, no bucket overflowed): block 0 alone
//    cuts the window from the band's bin counts (gq_window), gathers its houses from the band's buckets
//    into LDS in (key, house) order (gqf_gather) and decides (gq_decide: the window houses' bytes into
//    fz.dec, the ON counts of every decided house into the slab — the A counts below the window, from
//    the A copies it loaded beside the C copies, plus the window's); no hand-off between workgroups;
//  * miss: every block passes over its slice of the cluster, the keys under parity par's map, counting
//    the bins of superbins sb and sb + 1 (C, A) and appending their houses to the miss buckets (sc1:
//    read by the last block of this launch); the last block cuts the window, gathers it in order and
//    decides, then zeroes the miss region;
//  * everything taken (the cluster's P < S): block 0 takes every house, the ON counts = all A counts;
//  * a NaN crossing, a cluster of <= kGqCap houses, a crossing bin over kGqCap houses, a full bucket
//    or a walk past the window: gq_exact decides every house (kGqfFull), in block 0 (the last on a miss).
// The decision (GqSel.fmode, fbs, fbe) is the step's (k_step_pipe GQ = 2).  Every block zeroes its
// slice of the other parity's region (read by the previous call; the step after this call produces
// into it).  The next map (parity 1 - par, its band in fband[1 - par]) is block 1's, beside block 0's
// decision — on a miss the last block's, after the decision (the window's xcnt feeds the band).
__global__ void __launch_bounds__(1024) k_gq_decide2(KParams p, GqfBufs fz, int par, double S, double pmin,
                                                     unsigned long long* __restrict__ slab,
                                                     unsigned* __restrict__ tickets, const double* __restrict__ part,
                                                     int nparts) {
  __shared__ uint4 s_e[kGqCap];
  __shared__ unsigned s_apre[4], s_asum[8];
  __shared__ int s_bad;
  __shared__ uint32_t s_map[kGqCells];
  __shared__ unsigned s_band[2][kGqBand * 64 * 4];  // (blocks 0, 1) the band's C and A bin counts
  static_assert(2 * kGqBand * 64 == 1024 && kGqfBandN == 4 * 1024, "a thread per band bin and kind; 4 bucket counts each");
  const int tid = threadIdx.x, lane = tid & 63;
  GqSel* sel = fz.sel;
  // diagnostics: the constant 100 MHz clock at the phases of this block (fz.stamps[block][kGqfStampWords])
#define GQF_STAMP(k)                                                                              \
  do {                                                                                            \
    if (fz.stamps && tid == 0) fz.stamps[blockIdx.x * kGqfStampWords + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
  GQF_STAMP(0);
  unsigned* R = fz.par[par];
  {  // the other parity's region, for the step after this decision
    unsigned* Z = fz.par[1 - par];
    for (int e = (int)(blockIdx.x * blockDim.x) + tid; e < kGqfParWords; e += (int)(gridDim.x * blockDim.x)) Z[e] = 0u;
  }
  const bool bovf = R[kGqfOffFlags] != 0u;
  const int pb = sel->fband[par];
  // the superbin copies, loaded only by the threads that own a superbin (every thread loading them
  // made 256 blocks x 1024 threads read 33 MB of L2 per call: ~5 us; r06 phase stamps); block 0 (the
  // decider unless the band misses) loads the A summary's copies beside them
  GqSupLoad sup;
  gq_pon_load(p, sup.pon);
#pragma unroll
  for (int q = 0; q < kGqCopies; ++q) sup.v[q] = make_uint4(0u, 0u, 0u, 0u);
  if (tid < kGqSupN)
#pragma unroll
    for (int q = 0; q < kGqCopies; ++q) sup.v[q] = *reinterpret_cast<const uint4*>(R + q * kGqSupStride + tid * 4);
  const unsigned asv = blockIdx.x == 0 && tid < kGqCopies * 8 ? R[kGqfOffASum + tid] : 0u;
  if (tid < 8) s_asum[tid] = 0u;
  // blocks 0 and 1 (they cut the window unless the band misses): the band's C and A bin counts summed
  // over the copies into LDS (a thread per bin and kind), and block 0 the band's bucket counts (into
  // s_e: gqf_gather reads them before it stores an entry) — issued beside the superbin loads, so the
  // window and the gather start without a round trip to memory
  if (blockIdx.x <= 1 && !bovf) {
    const int bn = tid & (kGqBand * 64 - 1), kind = tid / (kGqBand * 64);  // (kind 0: C, 1: A)
    const unsigned* src = R + (kind ? kGqfOffBandA : kGqfOffBandC) + bn * 4;
    uint4 bv[kGqCopies];
#pragma unroll
    for (int q = 0; q < kGqCopies; ++q) bv[q] = *reinterpret_cast<const uint4*>(src + q * kGqBandWords);
    uint4 nv = make_uint4(0u, 0u, 0u, 0u);
    if (blockIdx.x == 0) nv = *reinterpret_cast<const uint4*>(R + kGqfOffBandN + tid * 4);
    uint4 t = bv[0];
#pragma unroll
    for (int q = 1; q < kGqCopies; ++q) { t.x += bv[q].x; t.y += bv[q].y; t.z += bv[q].z; t.w += bv[q].w; }
    *reinterpret_cast<uint4*>(&s_band[kind][bn * 4]) = t;
    if (blockIdx.x == 0) *reinterpret_cast<uint4*>(reinterpret_cast<unsigned*>(s_e) + tid * 4) = nv;
  }
  if (tid < 4) s_apre[tid] = 0u;
  if (fz.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GQF_STAMP(16);
  }
  const GqSuper g = gq_super_scan(p, sup, S, sel, nullptr, false,
                                  fz.stamps ? fz.stamps + blockIdx.x * kGqfStampWords + 27 : nullptr);  // (ends with a block barrier)
  GQF_STAMP(1);
  const bool all = g.sb >= kGqSupN, nanx = g.sb == kGqSuper && !g.whole;
  const bool hit = !all && !nanx && !g.whole && !bovf && g.sb >= pb && g.sb + 1 < pb + kGqBand;
  // 0 band window, 1 miss, 2 everything taken, 3 gq_exact (the same in every block)
  int path = all ? 2 : (nanx || g.whole) ? 3 : hit ? 0 : 1;
  const int path0 = path;
  GqWin w{};
  if (path != 1) {
    if (blockIdx.x > 1) return;  // (block-uniform: blocks 0 and 1 decide and map)
    if (asv) atomicAdd(&s_asum[tid & 7], asv);  // (block 0: A_lo, A_all over the copies; zeroed before the scan's barriers)
    const int off = hit ? (g.sb - pb) * 64 * 4 : 0;
    w = gq_window<1, kGqfAfter>(p, s_band[0] + off, 0, S, sel, g.sb, path != 0, path == 3, g.whole, g.before,
                                g.before_cnt, g.total, s_band[1] + off);
    if (path == 0 && w.ovf) path = 3;  // (a crossing bin over kGqCap houses)
    GQF_STAMP(3);
    if (blockIdx.x == 1) {  // the next map, beside block 0's decision
      gq_next_map_core(p, R, part, nparts, sel, fz.map[par], sel->fkmin[par], sel->fscale[par], fz.map[1 - par],
                       &sel->fkmin[1 - par], &sel->fscale[1 - par], reinterpret_cast<unsigned char*>(s_e), false,
                       g.sb, w.xcnt, &sel->fband[1 - par]);
      GQF_STAMP(8);
      return;
    }
    if (path == 0) {  // the band's A bins of its superbins below the crossing one: a wave sum, one LDS atomic per wave and class
      unsigned a[4] = {0u, 0u, 0u, 0u};
      if (tid < (g.sb - pb) * 64)
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = s_band[1][tid * 4 + k];
      if (tid < (kGqBand - 1) * 64) {  // (wave-uniform bound)
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) a[k] += __shfl_xor(a[k], off);
        if (lane == 0)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (a[k]) atomicAdd(&s_apre[k], a[k]);
      }
    }
  } else {  // the miss pass: this block's slice, the bins of superbins sb and sb + 1, and the A_lo of the houses below them
    for (int e = tid; e < kGqCells; e += blockDim.x) s_map[e] = fz.map[par][e];
    if (tid < 8) s_asum[tid] = 0u;
    __syncthreads();
    const double kmin = sel->fkmin[par], scale = sel->fscale[par];
    const uint32_t bb = (uint32_t)g.sb * 64u;
    const int cp = (int)(blockIdx.x % kGqCopies);
    unsigned* M = fz.miss;
    GqfAcnt acnt{0u, 0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + tid; i < p.n; i += (int64_t)gridDim.x * blockDim.x) {
      const double k = gq_key_of(p, i);
      const uint32_t bin = (uint32_t)(k != k ? kGqBins : gq_bin(k, kmin, scale, s_map)), b = bin - bb;
      const unsigned cls = p.cap_idx[i] & 3u;
      const uint32_t hw = p.hvac[i];
      const bool canon = gqf_canon(hw, p);
      gqf_acount(acnt, canon, bin < bb, cls);
      if (b < 128u) {
        atomicAdd(&M[(cp * 128 + b) * 4 + cls], 1u);
        if (canon) atomicAdd(&M[kGqfMissC + (cp * 128 + b) * 4 + cls], 1u);
        const unsigned slot = atomicAdd(&M[2 * kGqfMissC + cp * 128 + b], 1u);
        if (slot < (unsigned)fz.mcap) gq_store_sc1(fz.mbkt + ((size_t)(cp * 128 + b)) * fz.mcap + slot,
                                                   gqf_entry(k, p.goff + i, cls, hw));
        else atomicOr(&M[2 * kGqfMissC + kGqfMissN], 1u);
      }
    }
    gqf_acount_wave(acnt, s_asum);
    __syncthreads();
    if (tid < 4 && s_asum[tid]) atomicAdd(&M[kGqfOffMissALo + tid], s_asum[tid]);
    // hand-offs to the last block: the miss counts, A_lo and buckets (atomics, sc1 stores)
    const bool last = grid_last_block(tickets);
    GQF_STAMP(6);
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler ordering only)
    if (tid < 4) s_asum[tid] = ld_sc1(&M[kGqfOffMissALo + tid]);  // (the cluster's A_lo below sb, in place of the band's)
  }
  __syncthreads();  // (s_apre, s_asum)
  GQF_STAMP(11);
  // the deciding block (block 0, or the last on a miss)
  int mode = kGqfBandMode, bs = w.bs, be = w.be;
  bool ovf0 = path == 3, more_after = w.more_after;
  int ncand = w.ncand;
  double win_tot = w.win_tot;
  unsigned xcnt = w.xcnt;
  unsigned aadd[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) aadd[k] = s_asum[k] + s_apre[k] + w.abelow[k];
  if (path == 0) {  // the window's houses from the band buckets: (bin, copy) pairs, bin-major
    const int bi0 = w.bs - pb * 64, npair = (w.be - w.bs + 1) * kGqCopies;  // (<= 64 x 8)
    const int np = gqf_gather<false>(
        s_e, npair,
        [&](int q) {  // (prefetched into s_e)
          return reinterpret_cast<const unsigned*>(s_e)[(q % kGqCopies) * (kGqBand * 64) + bi0 + q / kGqCopies];
        },
        [&](int q) { return fz.bkt[par] + ((size_t)(q % kGqCopies) * (kGqBand * 64) + bi0 + q / kGqCopies) * fz.cap; },
        fz.stamps ? fz.stamps + blockIdx.x * kGqfStampWords + 18 : nullptr);
    ovf0 = np != w.ncand;  // (cannot happen: the buckets hold the counted houses)
    GQF_STAMP(4);
  } else if (path == 1) {
    // the miss counts into LDS (sc1: other workgroups' atomics) — C and A behind the window array
    unsigned* lc = reinterpret_cast<unsigned*>(s_e);
    unsigned* M = fz.miss;
    for (int e = tid; e < 2 * kGqfMissC; e += blockDim.x) lc[e] = ld_sc1(&M[e]);
    if (tid == 0) s_bad = ld_sc1(&M[2 * kGqfMissC + kGqfMissN]) != 0u;
    __syncthreads();
    const GqWin wm = gq_window<kGqCopies, kGqfAfter>(p, lc, 512, S, sel, g.sb, false, false, false, g.before,
                                                     g.before_cnt, g.total, lc + kGqfMissC);
    xcnt = wm.xcnt;
    __syncthreads();  // (done with lc: the window goes into s_e)
    ovf0 = wm.ovf || s_bad;
    if (!ovf0) {  // gather [bs, be] of the miss bins (bin-major, copies inside) in order
      const int bi0 = wm.bs - g.sb * 64, npair = (wm.be - wm.bs + 1) * kGqCopies;
      const int np = gqf_gather<true>(
          s_e, npair, [&](int q) { return ld_sc1(&M[2 * kGqfMissC + (q % kGqCopies) * 128 + bi0 + q / kGqCopies]); },
          [&](int q) { return fz.mbkt + ((size_t)(q % kGqCopies) * 128 + bi0 + q / kGqCopies) * fz.mcap; });
      ovf0 = np != wm.ncand;
      ncand = wm.ncand;
      win_tot = wm.win_tot;
      more_after = wm.more_after;
      bs = wm.bs;
      be = wm.be;
#pragma unroll
      for (int k = 0; k < 4; ++k) aadd[k] = s_asum[k] + wm.abelow[k];
    }
    // the miss region back to zero for the next call (this block was its only reader)
    for (int e = tid; e < kGqfMissWords; e += blockDim.x) M[e] = 0u;
  }
  bool full = false;
  if (path == 2) {  // everything taken: the ON counts of every house (shard 0; the rest are zero)
    mode = kGqfAll;
    if (tid < p.n_cap) slab[tid] = s_asum[4 + tid];  // (A_all)
  } else {
    // (a walk past the window, or ovf0: gq_decide's own gq_exact decides every house)
    full = gq_decide(p, nullptr, S, pmin, sel, fz.dec, slab, s_e, false, ovf0, false, ncand, win_tot, more_after,
                     true, aadd, fz.stamps ? fz.stamps + blockIdx.x * kGqfStampWords + 12 : nullptr);
    if (!full && tid == 0) sel->fwin = (unsigned)ncand;
  }
  if (full) mode = kGqfFull;
  if (tid == 0) {
    sel->fmode = mode;
    sel->fbs = bs;
    sel->fbe = be;
    atomicAdd(&sel->fcalls, 1u);
    if (path0 == 0 && path == 0) atomicAdd(&sel->fhits, 1u);
    if (path0 == 1) atomicAdd(&sel->fmisses, 1u);
    if (full) atomicAdd(&sel->fexact, 1u);
    sel->overflow = 0;
  }
  GQF_STAMP(7);
  if (fz.stamps && tid == 0) fz.stamps[blockIdx.x * kGqfStampWords + 10] = 1;  // (the deciding block)
  if (path0 == 1) {  // the next map here, after the miss window's xcnt (see above)
    __syncthreads();
    gq_next_map_core(p, R, part, nparts, sel, fz.map[par], sel->fkmin[par], sel->fscale[par], fz.map[1 - par],
                     &sel->fkmin[1 - par], &sel->fscale[1 - par], reinterpret_cast<unsigned char*>(s_e), false, g.sb,
                     xcnt, &sel->fband[1 - par]);
    GQF_STAMP(8);
  }
  GQF_STAMP(9);
#undef GQF_STAMP
}

// sharded greedy (mdr_greedy_inputs / mdr_greedy_select): this shard's (key, P, lockout) rows, and
// the generic gather / iota for the cluster-wide selection over the gathered rows
__global__ void k_greedy_inputs(KParams p, double* __restrict__ key, double* __restrict__ power,
                                uint8_t* __restrict__ lock) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  key[i] = -(p.t_air[i] - p.target[i]);
  power[i] = p.p_on[p.cap_idx[i]];
  lock[i] = hv_lock(p.hvac[i]) ? 1 : 0;
}

__global__ void k_greedy_iota(int64_t n, int* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) idx[i] = (int)i;
}

__global__ void k_greedy_gather_rows(int64_t n, const int* __restrict__ perm, const double* __restrict__ power,
                                     const uint8_t* __restrict__ lock, double* __restrict__ psorted,
                                     uint8_t* __restrict__ lsorted) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int i = perm[j];
  psorted[j] = power[i];
  lsorted[j] = lock[i];
}

__global__ void k_greedy_apply(int64_t n, const int* __restrict__ perm, const int64_t* kpos,
                               const int64_t* extra, uint8_t* __restrict__ action) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  bool take = j < kpos[0];
  const int64_t ne = kpos[1];
  for (int64_t e = 0; e < ne; ++e) take |= (extra[e] == j);
  action[perm[j]] = take ? 1 : 0;
}

}  // namespace mdr
