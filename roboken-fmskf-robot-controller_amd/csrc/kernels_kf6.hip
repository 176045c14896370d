// kernels_kf6.hip -- the headline 6-state fp32 KF tick (BASELINE.json configs[1], SURVEY.md
// 8(d) cfg 2) for gfx950.
//
// One robot per lane, x (6) and packed P (21) in VGPRs; a tick = measurement frontend
// (yaw, gyro z, 4 wheel rpm -> z, the reference's deg2rad / mecanum FK / rotation,
// VD_vehicle_controller.cpp:21-51) + LDL^T-form update + F P F^T + Q predict, one read and
// one write of every state byte: 232 algorithmic bytes per instance-tick.
//
// Memory-path design (MI355X_MICROARCH.md: s_waitcnt vmcnt is in-order, so any load issued
// after the state loads makes every later wait cover them):
//  * the 2 KiB TABLE512 sine table is staged in LDS (per wave in the single-tick kernel, per
//    block in the loop kernels), so the trig lookups in the middle of the math wait on
//    lgkmcnt only, never behind the state loads;
//  * planes are addressed through buffer descriptors built from kernel arguments (T8) with
//    a 32-bit lane byte offset; when the 21 P planes fit one 4 GiB window (n < 51M, the
//    SMALL instantiation) one descriptor per array plus a per-plane scalar soffset
//    addresses every plane, so the loop needs almost no scalar or vector address math;
//  * whether a validity mask exists is a compile-time choice (no conditional load whose
//    merge would force a full vmcnt(0) drain);
//  * tick_many loads the inputs of tick t+1 before computing tick t.
#include "ens_device.hpp"
#include "kf6_lane.hpp"

#pragma clang fp contract(off)

namespace fmskf {

// copy the sine table to LDS: all global loads first, then the LDS writes, one barrier
template <bool LIBM>
__device__ __forceinline__ void stage_table(float *stab, const float *g) {
  if (!LIBM) {
    const int t = threadIdx.x;
    const float a = g[t], b = g[t + kBlock];
    const float c = t == 0 ? g[2 * kBlock] : 0.f;
    stab[t] = a;
    stab[t + kBlock] = b;
    if (t == 0) stab[2 * kBlock] = c;
    __syncthreads();
  }
}
static_assert(2 * kBlock + 1 == 513, "table staging assumes 256-thread blocks");


// tick_many: T ticks per launch, state in VGPRs throughout; the inputs of the next tick are
// loaded while the current one computes.  Unrolled by two with ping-pong input registers
// (ma / mb) so no input record is copied around the loop; clamped index, no live branch.
template <int WPE, class O>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_kf6(
    KfArgs<MdKF6, Kf6Params> a) {
  __shared__ float stab[O::LIBM ? 1 : 513];
  const uint64_t n = a.n;
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < (uint32_t)n;
  const uint32_t ic = live ? i : (uint32_t)n - 1u;
  const uint32_t T = a.in.n_ticks;
  float x[6], P[21];
  Kf6Lo<O> lo;
  Kf6In ma, mb;
  kf6_load_state<O>(a.x, a.P, a.pitch, ic, x, P);
  kf6_load_lo<O>(a.prm.lo, ic, lo);
  if (O::UPD) ma = kf6_load_in<O>(a.in, n, 0, ic);
  stage_table<O::LIBM>(stab, a.in.sintab);
  for (uint32_t t = 0; t < T; t += 2) {
    if (O::UPD && t + 1 < T) mb = kf6_load_in<O>(a.in, n, t + 1, ic);
    kf6_tick1<O>(ma, stab, a.prm, x, P, lo);
    if (t + 1 >= T) break;
    if (O::UPD && t + 2 < T) ma = kf6_load_in<O>(a.in, n, t + 2, ic);
    kf6_tick1<O>(mb, stab, a.prm, x, P, lo);
  }
  if (live) {
    kf6_store_state<O>(a.x, a.P, a.pitch, i, x, P);
    kf6_store_lo<O>(a.prm.lo, i, lo);
  }
  nan_guard(x, P, a.counters, live);
}

// Single tick, straight line: no tick loop (so no loop-carried register copies) and no
// live/dead branch around the loads: lanes past N load instance N-1 (a clamped index, always
// in bounds), compute on it, and only their stores and NaN count are masked off.
template <int WPE, class O>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_kf6t(
    KfArgs<MdKF6, Kf6Params> a) {
  uint32_t bid = blockIdx.x;
  if constexpr (O::ENS) {
    if (ens_fold_front<6>(a.in, bid)) return;
  }
  const uint64_t n = a.n;
  const uint32_t i = bid * kBlock + threadIdx.x;
  const bool live = i < (uint32_t)n;
  const uint32_t ic = live ? i : (uint32_t)n - 1u;
  float x[6], P[21];
  Kf6In m;
  // wave-private copy of the sine table: its loads are issued first (vmcnt retires in order)
  // and no block barrier couples the four waves' memory phases (~1% over a block-shared copy)
  __shared__ float wtab[O::LIBM ? 1 : kBlock / 64][O::LIBM ? 1 : kWaveTab];
  float *stab = wtab[O::LIBM ? 0 : threadIdx.x >> 6];
  WaveTable<O::LIBM> tv(a.in.sintab);
  Kf6Lo<O> lo;
  kf6_load_state<O>(a.x, a.P, a.pitch, ic, x, P);
  kf6_load_lo<O>(a.prm.lo, ic, lo);
  if (O::UPD) m = kf6_load_in<O>(a.in, n, 0, ic);
  tv.store(stab);
  kf6_tick1<O>(m, stab, a.prm, x, P, lo);
  if (live) {
    kf6_store_state<O>(a.x, a.P, a.pitch, i, x, P);
    kf6_store_lo<O>(a.prm.lo, i, lo);
  }
  nan_guard(x, P, a.counters, live);
  if constexpr (O::ENS) {
    float xs[1][6];
#pragma unroll
    for (int k = 0; k < 6; k++) xs[0][k] = x[k];
    const bool lv[1] = {live};
    ens_epilogue<6, 1>(a.in, xs, lv, bid);
  }
}

// R robots per lane (i, i + G, ..., G = the tick blocks' lane count), the tick inputs of all R
// loaded up front: robot r's inputs (fresh from HBM) arrive while robots 0..r-1 are loaded,
// computed and stored; one register set for the state, 1/R of the grid.
template <int WPE, int R, class O>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_kf6p(
    KfArgs<MdKF6, Kf6Params> a) {
  uint32_t bid = blockIdx.x;
  if constexpr (O::ENS) {
    if (ens_fold_front<6>(a.in, bid)) return;
  }
  const uint64_t n = a.n;
  const uint32_t nn = (uint32_t)n, last = nn - 1u;
  const uint32_t G = (O::ENS ? a.in.ens_grid : gridDim.x) * kBlock;
  const uint32_t i0 = bid * kBlock + threadIdx.x;
  float x[6], P[21];
  __shared__ float wtab[O::LIBM ? 1 : kBlock / 64][O::LIBM ? 1 : kWaveTab];
  float *stab = wtab[O::LIBM ? 0 : threadIdx.x >> 6];
  WaveTable<O::LIBM> tv(a.in.sintab);
  Kf6In m[R];
  float xs[O::ENS ? R : 1][6];
  bool lv[R];
  if (O::UPD) {
#pragma unroll
    for (int r = 0; r < R; r++) m[r] = kf6_load_in<O>(a.in, n, 0, min(i0 + r * G, last));
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t i = i0 + r * G;
    const bool live = i < nn;
    Kf6Lo<O> lo;
    kf6_load_state<O>(a.x, a.P, a.pitch, live ? i : last, x, P);
    kf6_load_lo<O>(a.prm.lo, live ? i : last, lo);
    if (r == 0) tv.store(stab);
    kf6_tick1<O>(m[r], stab, a.prm, x, P, lo);
    if (live) {
      kf6_store_state<O>(a.x, a.P, a.pitch, i, x, P);
      kf6_store_lo<O>(a.prm.lo, i, lo);
    }
    nan_guard(x, P, a.counters, live);
    if constexpr (O::ENS) {
#pragma unroll
      for (int k = 0; k < 6; k++) xs[r][k] = x[k];
    }
    lv[r] = live;
  }
  if constexpr (O::ENS) ens_epilogue<6, R>(a.in, xs, lv, bid);
}

// Variant (FMSKF_KF6_VARIANT, read once) for single-tick launches; default 0:
//   0: k_kf6p with 2 robots per lane while 124 B x N fits the Infinity Cache, else 15
//   15: one instance per lane, grid = N/256, straight-line single-tick kernel (k_kf6t)
//   12: k_kf6p with 2 robots per lane at any N
// (the tests force 12 / 15 at small N to check both kernels).  Measured and removed: 3 or 4
// robots per lane (38.0 us at 2^20 against 37.4-38.6 for 2), the single tick through the
// tick-loop kernel, and persistent double-buffered kernels at 2-8 blocks per CU (5-20% slower).
static int kf6_variant() {
  static int v = [] {
    const char *e = getenv("FMSKF_KF6_VARIANT");
    const int x = e ? atoi(e) : 0;
    return x == 12 || x == 15 ? x : 0;
  }();
  return v;
}

template <class O>
static void launch_o(const KfArgs<MdKF6, Kf6Params> &a, hipStream_t st) {
  const int v = a.in.n_ticks == 1 ? kf6_variant() : 0;
  // state bytes per robot (COMP: + the five low-part rows) and with one tick's 16-byte inputs
  constexpr uint64_t SB = O::COMP ? 128 : 108, RB = SB + 16;
  if (a.in.n_ticks == 1 && v == 12) {
    const unsigned g = (unsigned)((a.n + 2 * kBlock - 1) / (2 * kBlock));
    if constexpr (O::UPD && O::PRED) {
      if (state_nt(a.n * SB)) {
        k_kf6p<4, 2, WithNT<O>><<<g, kBlock, 0, st>>>(a);
        return;
      }
    }
    k_kf6p<4, 2, O><<<g, kBlock, 0, st>>>(a);
  } else if (a.in.n_ticks == 1 && v == 0 && a.n * RB <= (256ull << 20)) {
    // state + one tick's inputs resident in the 256 MiB Infinity Cache: two robots per lane,
    // both robots' inputs loaded up front, one wave round (2^20: 39.7 -> 37.4-38.1 us,
    // 2^21: 75.9 -> 71.5; at 2^24, HBM-bound, it is 3% slower than one robot per lane)
    const unsigned g = (unsigned)((a.n + 2 * kBlock - 1) / (2 * kBlock));
    // 32 KiB of dynamic LDS: at most 5 blocks per CU.  kbench, records, two passes: 2^20
    // 38.2-38.5 -> 37.2-37.3 us (24 KiB 37.6-37.7, 40 KiB 37.4-37.5); 2^21 71.6-71.8 -> 70.5-70.9.
    // Records fed while state + inputs fill at most half the cache (2^20 robots): 48 KiB, 3
    // blocks per CU (round 3, kbench, three alternating passes on one box: 32 KiB 36.99-37.14 us,
    // 48 KiB 36.67-36.93, 64 KiB 36.61-36.97, 80 KiB 44.0, uncapped 38.0).  Plane inputs and
    // 2^21 records stay at 32 KiB (48 KiB: 2^20 planes 37.49 -> 37.72-38.07, 2^21 records
    // 68.3-68.4 -> 69.0, 2^21 planes 69.5-69.7 -> 71.2-71.4)
    const bool rec_half = a.in.rec != nullptr && a.n * RB <= (128ull << 20);
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_KF6P_LDS", true, rec_half ? 48u * 1024u : 32u * 1024u);
    if constexpr (O::UPD && O::PRED) {
      if (state_nt(a.n * SB)) {  // only when forced: this branch's state fits the cache
        k_kf6p<4, 2, WithNT<O>><<<g, kBlock, lds, st>>>(a);
        return;
      }
    }
    k_kf6p<4, 2, O><<<g, kBlock, lds, st>>>(a);
  } else if (a.in.n_ticks == 1 && (v == 0 || v == 15)) {
    // past the Infinity Cache: at most 3 blocks per CU (48 KiB of dynamic LDS).  2^24, records,
    // kbench, one box, two passes: 691-704 us uncapped, 671-684 at 32 KiB, 627-641 at 48 KiB,
    // 626-639 at 64 KiB, 809-826 at 80 KiB (two blocks of 4 waves per CU are too few)
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_KF6_LDS", state_nt(a.n * SB), 48u * 1024u);
    if constexpr (O::UPD && O::PRED) {
      if (state_nt(a.n * SB)) {
        k_kf6t<4, WithNT<O>><<<grid_for(a.n), kBlock, lds, st>>>(a);
        return;
      }
    }
    k_kf6t<4, O><<<grid_for(a.n), kBlock, lds, st>>>(a);
  } else {
    k_kf6<4, O><<<grid_for(a.n), kBlock, 0, st>>>(a);
  }
}

// fused tick + ensemble record (fmskf_tick_ensemble): the kernel launch_o picks by default,
// with the record epilogue (and the carried fold blocks ahead of the tick blocks when
// in.fold_blocks is set); returns the tick grid (= the number of block records).  Four robots
// per lane (half the block reductions per robot) measured slower: K = 1 at 2^20 40.8-41.0 us
// per tick against 38.6-39.0 (kbench, two alternating passes)
template <class O>
static int launch_ens_o(KfArgs<MdKF6, Kf6Params> a, hipStream_t st) {
  using E = WithEns<O>;
  const unsigned carry = a.in.fold_blocks ? (unsigned)EnsRec<6>::LEN : 0u;
  constexpr uint64_t SB = O::COMP ? 128 : 108, RB = SB + 16;
  if (a.n * RB <= (256ull << 20)) {
    const unsigned g = (unsigned)((a.n + 2 * kBlock - 1) / (2 * kBlock));
    a.in.ens_grid = g;
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_KF6P_LDS", true, 32u * 1024u);
    if (state_nt(a.n * SB)) launch_signal(k_kf6p<4, 2, WithNT<E>>, dim3(g + carry), lds, st, a.in.ens_done, a);
    else launch_signal(k_kf6p<4, 2, E>, dim3(g + carry), lds, st, a.in.ens_done, a);
    return (int)g;
  }
  // past the Infinity Cache the record epilogue (fp64 sums and their cross-lane reduction)
  // wants a smaller cap than the plain tick: 2^24, kbench, two passes: 738 us at 48 KiB,
  // 665-670 at 32 KiB, 680-689 at 24 KiB, 722-724 uncapped (the plain tick: 619-628)
  const unsigned g = grid_for(a.n).x;
  a.in.ens_grid = g;
  const unsigned lds = FMSKF_LDS_CAP("FMSKF_KF6E_LDS", state_nt(a.n * SB), 32u * 1024u);
  if (state_nt(a.n * SB)) launch_signal(k_kf6t<4, WithNT<E>>, dim3(g + carry), lds, st, a.in.ens_done, a);
  else launch_signal(k_kf6t<4, E>, dim3(g + carry), lds, st, a.in.ens_done, a);
  return (int)g;
}

template <class O>
static void launch_sel(const KfArgs<MdKF6, Kf6Params> &a, hipStream_t st, int *ens_nb) {
  if constexpr (O::UPD && O::PRED) {
    if (ens_nb) {
      *ens_nb = launch_ens_o<O>(a, st);
      return;
    }
  }
  launch_o<O>(a, st);
}

template <bool LIBM, bool UPD, bool PRED, bool REC>
static void launch_lupr_plain(const KfArgs<MdKF6, Kf6Params> &a, bool small, bool valid, hipStream_t st,
                              int *nb) {
  if (small) {
    if (valid) launch_sel<Opt<LIBM, UPD, PRED, true, true, REC>>(a, st, nb);
    else launch_sel<Opt<LIBM, UPD, PRED, true, false, REC>>(a, st, nb);
  } else {
    if (valid) launch_sel<Opt<LIBM, UPD, PRED, false, true, REC>>(a, st, nb);
    else launch_sel<Opt<LIBM, UPD, PRED, false, false, REC>>(a, st, nb);
  }
}
template <bool LIBM, bool UPD, bool PRED, bool REC>
static void launch_lupr(const KfArgs<MdKF6, Kf6Params> &a, bool small, bool valid, hipStream_t st,
                        int *nb) {
  if (a.prm.lo) {  // FMSKF_CFG_COMP_POS
    if (small) {
      if (valid) launch_sel<Opt<LIBM, UPD, PRED, true, true, REC, false, false, true>>(a, st, nb);
      else launch_sel<Opt<LIBM, UPD, PRED, true, false, REC, false, false, true>>(a, st, nb);
    } else {
      if (valid) launch_sel<Opt<LIBM, UPD, PRED, false, true, REC, false, false, true>>(a, st, nb);
      else launch_sel<Opt<LIBM, UPD, PRED, false, false, REC, false, false, true>>(a, st, nb);
    }
    return;
  }
  launch_lupr_plain<LIBM, UPD, PRED, REC>(a, small, valid, st, nb);
}
template <bool LIBM, bool UPD, bool PRED>
static void launch_lup(const KfArgs<MdKF6, Kf6Params> &a, bool small, bool valid, hipStream_t st,
                       int *nb) {
  if (UPD && a.in.rec) launch_lupr<LIBM, UPD, PRED, UPD>(a, small, valid, st, nb);
  else launch_lupr<LIBM, UPD, PRED, false>(a, small, valid, st, nb);
}

int launch_kf6(const DevState &s, const TickIn &in, const Kf6Params &p, bool libm, bool upd,
               bool pred, hipStream_t st, int *ens_nb) {
  KfArgs<MdKF6, Kf6Params> a{s.n, s.pitch, (float *)s.x, (float *)s.P, in, s.counters, p};
  const bool small = s.pitch * 84 < 0xFFFFFFFFull;
  const bool valid = upd && in.valid != nullptr;
  int *nb = in.ens_blocks && upd && pred && in.n_ticks == 1 ? ens_nb : nullptr;
  if ((in.ens_blocks && !nb) || (in.fold_blocks && !in.ens_blocks)) return (int)hipErrorInvalidValue;
  if (libm) {
    if (upd && pred) launch_lup<true, true, true>(a, small, valid, st, nb);
    else if (upd) launch_lup<true, true, false>(a, small, valid, st, nullptr);
    else launch_lup<true, false, true>(a, small, false, st, nullptr);
  } else {
    if (upd && pred) launch_lup<false, true, true>(a, small, valid, st, nb);
    else if (upd) launch_lup<false, true, false>(a, small, valid, st, nullptr);
    else launch_lup<false, false, true>(a, small, false, st, nullptr);
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf
