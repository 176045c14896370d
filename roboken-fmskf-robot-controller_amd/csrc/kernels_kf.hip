// kernels_kf.hip -- 9-state EKF (fp32) and 12-state KF (fp64) tick kernels for gfx950.
//
// One filter instance per lane; the per-instance state (x and the packed symmetric P)
// lives in VGPRs for the whole launch, so a tick reads and writes each state byte
// exactly once (HBM-bound by design, no MFMA: matrices are <= 12x12 per instance).
// State planes are SoA: lane i of a wave touches consecutive addresses of every plane.
// F / H / Q / R are shared: H and the sparsity of F are compile-time model traits
// (kf_generic.hpp), Q / R / dt ride in the kernarg segment (scalar loads, SGPRs).
// The 6-state headline kernel lives in kernels_kf6.hip.
#include "can_lane.hpp"
#include "ctrl_lane.hpp"
#include "ens_device.hpp"
#include "kf_generic.hpp"

#pragma clang fp contract(off)

namespace fmskf {

// EKF9 z from raw WT901 registers (imu_if_wt901c.cpp:96-99,107-113) + wheel rpm; the heading
// innovation against the compensated heading x[2] + lo
__device__ __forceinline__ void ekf9_innov(const uint4 w, const float (&x)[9], float lo, float (&y)[6]) {
  int16_t a[4], r[4];
  unpack4(make_uint2(w.x, w.y), a);
  unpack4(make_uint2(w.z, w.w), r);
  const float yaw = (float)a[0] / 32768.0f * 180.0f;
  const float gz = (float)a[1] / 32768.0f * 2000.0f;
  const float ax = (float)a[2] / 32768.0f * 16.0f;
  const float ay = -((float)a[3] / 32768.0f * 16.0f);
  float vx, vy, vth;
  mdir_to_vdir(rpm_to_mvel(r[0]), rpm_to_mvel(r[1]), rpm_to_mvel(r[2]), rpm_to_mvel(r[3]), vx, vy,
               vth);
  const float z0 = deg2rad(yaw), z1 = deg2rad(gz), z2 = ax * K::g0, z3 = ay * K::g0;
  const float z4 = vx * 0.001f, z5 = vy * 0.001f;
  y[0] = wrap_innov((z0 - x[2]) - lo);
  y[1] = z1 - (x[5] + x[6]);
  y[2] = z2 - x[7];
  y[3] = z3 - x[8];
  y[4] = z4 - x[3];
  y[5] = z5 - x[4];
}

// one robot's 16-byte raw record of a single tick, read once; NT: non-temporal (gfx950 `nt`).
// Measured (kbench, one box, two passes): 2^20 (two robots per lane) 74.1-74.2 -> 73.0-73.4 us
// with nt; 2^22 (one per lane, HBM) 334.6-335.6 plain vs 337.5-338.3 nt: k_ekf9p uses nt,
// k_ekf9t plain loads
template <bool NT>
__device__ __forceinline__ uint4 ekf9_raw_at(const int16_t *raw, uint64_t i) {
  if constexpr (NT) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(raw) + i);
    return make_uint4(v[0], v[1], v[2], v[3]);
  } else {
    return reinterpret_cast<const uint4 *>(raw)[i];
  }
}

// one EKF9 tick (update with the measurement frontend, then the nonlinear predict)
// SEQ: R is diagonal -> the sequential scalar update (kf_update_seq), else the joint LDL^T one
// lo: the compensated heading's low part (th_add, kf_generic.hpp)
// COMP: FMSKF_CFG_COMP_POS -- px, py, P00, P10, P11 compensated too (cl: their five low parts;
// oracle orc_ekf9_tick_comp)
template <bool LIBM, bool UPD, bool PRED, bool SEQ, bool COMP = false>
__device__ __forceinline__ void ekf9_tick1(const KfArgs<MdEKF9, Ekf9Params> &a, const uint4 raw,
                                           bool have, const float *stab, float (&x)[9],
                                           float (&P)[45], float &lo, float *cl = nullptr) {
  constexpr unsigned CXM = COMP ? kPosCXM : 0u;
  constexpr unsigned long long CPM = COMP ? kPosCPM : 0ull;
  const float dt = a.prm.dt;
  if (UPD && have) {
    float y[6];
    ekf9_innov(raw, x, lo, y);
    if constexpr (SEQ) kf_update_seq<MdEKF9, 2, float, 9, 6, 45, CXM, CPM>(x, P, y, a.prm.r, &lo, cl);
    else kf_update<MdEKF9, 2, float, 9, 6, 45, CXM, CPM>(x, P, y, a.prm.r, &lo, cl);
    th_norm(x[2], lo);
  }
  if (PRED) {
    // f(x): mecanum body velocity rotated into the world frame (the reference's
    // odometry, VD_vehicle_controller.cpp:47-51, generalised) + its Jacobian
    const float rr = normalize_rad_0to2pi(x[2]);
    const float c = cos_p<LIBM>(rr, stab), s = sin_p<LIBM>(rr, stab);
    const float vwx = x[3] * c - x[4] * s;
    const float vwy = x[3] * s + x[4] * c;
    const float f02 = -(vwy * dt), f03 = c * dt, f04 = -(s * dt);
    const float f12 = vwx * dt, f13 = s * dt, f14 = c * dt;
    if constexpr (COMP) {
      th_add(x[0], cl[0], vwx * dt);
      th_add(x[1], cl[1], vwy * dt);
      th_norm(x[0], cl[0]);
      th_norm(x[1], cl[1]);
    } else {
      x[0] = x[0] + vwx * dt;
      x[1] = x[1] + vwy * dt;
    }
    th_add(x[2], lo, x[5] * dt);
    wrap_pi_c(x[2], lo);
    th_norm(x[2], lo);
    x[3] = x[3] + x[7] * dt;
    x[4] = x[4] + x[8] * dt;
    auto fv = [&](int r, int k) -> float {
      if (r == 0) return k == 2 ? f02 : k == 3 ? f03 : f04;
      if (r == 1) return k == 2 ? f12 : k == 3 ? f13 : f14;
      return dt;
    };
    if constexpr (COMP) kf_predict_cov_c<MdEKF9, kPosCXM, kPosCPM>(P, fv, a.prm.q, cl);
    else kf_predict_cov<MdEKF9>(P, fv, a.prm.q);
  }
}

// the COMP low-part rows of one 256-robot chunk (tiled like x, kKf6LoRows rows)
template <bool COMP, int CP>
struct Ekf9Lo {
  float v[COMP ? kKf6LoRows : 1];
  __device__ __forceinline__ void load(const float *clo, uint32_t chunk, uint32_t slot) {
    if constexpr (COMP) {
      const TileRows<float, kKf6LoRows, CP> t(const_cast<float *>(clo), chunk, slot, 0);
#pragma unroll
      for (int k = 0; k < (int)kKf6LoRows; k++) v[k] = t.ld(k);
    }
  }
  __device__ __forceinline__ void store(float *clo, uint32_t chunk, uint32_t slot) const {
    if constexpr (COMP) {
      const TileRows<float, kKf6LoRows, CP> t(clo, chunk, slot, 0);
#pragma unroll
      for (int k = 0; k < (int)kKf6LoRows; k++) t.st(k, v[k]);
    }
  }
};

// tick_many: T ticks per launch, state in VGPRs; the next tick's raw record (16 B) and validity
// byte are loaded while the current tick computes (ping-pong registers, loop unrolled by two)
template <bool LIBM, bool UPD, bool PRED, bool SEQ, bool COMP = false>
__global__ __launch_bounds__(kBlock) void k_ekf9(KfArgs<MdEKF9, Ekf9Params> a) {
  constexpr int N = 9, NP = 45;
  __shared__ float stab[LIBM ? 1 : 513];
  if (!LIBM) {
    for (int k = threadIdx.x; k < 513; k += kBlock) stab[k] = a.in.sintab[k];
    __syncthreads();
  }
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < n;
  const uint64_t ic = live ? i : n - 1;
  const uint32_t T = a.in.n_ticks;
  const uint64_t st = a.in.stride;
  auto raw_at = [&](uint32_t t) -> uint4 {
    return UPD ? reinterpret_cast<const uint4 *>(a.in.raw)[(uint64_t)t * st + ic] : make_uint4(0, 0, 0, 0);
  };
  auto have_at = [&](uint32_t t) -> bool {
    return a.in.valid == nullptr || a.in.valid[(uint64_t)t * st + ic];
  };
  float x[N], P[NP];
  const TileRows<float, N> tx(a.x, tile_slot(n));
  const TileRows<float, NP> tp(a.P, tile_slot(n));
  if constexpr (FMSKF_TILED) {
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = tx.ld(k);
#pragma unroll
    for (int k = 0; k < NP; k++) P[k] = tp.ld(k);
  } else {
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = a.x[k * pp + ic];
#pragma unroll
    for (int k = 0; k < NP; k++) P[k] = a.P[k * pp + ic];
  }
  float lo = a.prm.thlo[ic];
  Ekf9Lo<COMP, 0> cl;
  cl.load(a.prm.clo, blockIdx.x, tile_slot(n));
  uint4 ra = raw_at(0), rb;
  bool ha = have_at(0), hb;
  for (uint32_t t = 0; t < T; t += 2) {
    if (t + 1 < T) {
      rb = raw_at(t + 1);
      hb = have_at(t + 1);
    }
    ekf9_tick1<LIBM, UPD, PRED, SEQ, COMP>(a, ra, ha, stab, x, P, lo, cl.v);
    if (t + 1 >= T) break;
    if (t + 2 < T) {
      ra = raw_at(t + 2);
      ha = have_at(t + 2);
    }
    ekf9_tick1<LIBM, UPD, PRED, SEQ, COMP>(a, rb, hb, stab, x, P, lo, cl.v);
  }
  if (live) {
    a.prm.thlo[i] = lo;
    cl.store(a.prm.clo, blockIdx.x, tile_slot(n));
    if constexpr (FMSKF_TILED) {
#pragma unroll
      for (int k = 0; k < N; k++) tx.st(k, x[k]);
#pragma unroll
      for (int k = 0; k < NP; k++) tp.st(k, P[k]);
    } else {
#pragma unroll
      for (int k = 0; k < N; k++) a.x[k * pp + i] = x[k];
#pragma unroll
      for (int k = 0; k < NP; k++) a.P[k * pp + i] = P[k];
    }
  }
  nan_guard(x, P, a.counters, live);
}

// Single tick, straight line (as k_kf6t): no tick loop, clamped index for lanes past N (only
// their stores and NaN count are masked), every load issued before the table barrier.
// ENS: the record epilogue of fmskf_tick_ensemble (ens_device.hpp)
template <bool LIBM, bool UPD, bool PRED, bool SEQ, int CP = 0, bool ENS = false, bool COMP = false>
__global__ __launch_bounds__(kBlock) void k_ekf9t(KfArgs<MdEKF9, Ekf9Params> a) {
  constexpr int N = 9, NP = 45;
  uint32_t bid = blockIdx.x;  // the tick block (the carried fold blocks come first)
  if constexpr (ENS) {
    if (ens_fold_front<9>(a.in, bid)) return;
  }
  __shared__ float wtab[LIBM ? 1 : kBlock / 64][LIBM ? 1 : kWaveTab];
  float *stab = wtab[LIBM ? 0 : threadIdx.x >> 6];
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t i = (uint64_t)bid * kBlock + threadIdx.x;
  const bool live = i < n;
  const uint64_t ic = live ? i : n - 1;
  float x[N], P[NP];
  WaveTable<LIBM> tv(a.in.sintab);  // wave-private table copy, loads issued first
  const uint32_t sl = tile_slot(n, bid);
  const TileRows<float, N, CP> tx(a.x, bid, sl, 0);
  const TileRows<float, NP, CP> tp(a.P, bid, sl, 0);
  if constexpr (FMSKF_TILED) {
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = tx.ld(k);
#pragma unroll
    for (int k = 0; k < NP; k++) P[k] = tp.ld(k);
  } else {
#pragma unroll
    for (int k = 0; k < N; k++) x[k] = a.x[k * pp + ic];
#pragma unroll
    for (int k = 0; k < NP; k++) P[k] = a.P[k * pp + ic];
  }
  const bool have = a.in.valid == nullptr || a.in.valid[ic];
  const uint4 raw = UPD ? ekf9_raw_at<false>(a.in.raw, ic) : make_uint4(0, 0, 0, 0);
  const uint64_t hb0 = (uint64_t)bid * kBlock;
  float lo = ld_chunk<float, CP>(a.prm.thlo, hb0, n, sl);
  Ekf9Lo<COMP, CP> cl;
  cl.load(a.prm.clo, bid, sl);
  tv.store(stab);
  ekf9_tick1<LIBM, UPD, PRED, SEQ, COMP>(a, raw, have, stab, x, P, lo, cl.v);
  if (live) {
    st_chunk<float, st_pol(CP)>(a.prm.thlo, hb0, n, sl, lo);
    cl.store(a.prm.clo, bid, sl);
    if constexpr (FMSKF_TILED) {
#pragma unroll
      for (int k = 0; k < N; k++) tx.st(k, x[k]);
#pragma unroll
      for (int k = 0; k < NP; k++) tp.st(k, P[k]);
    } else {
#pragma unroll
      for (int k = 0; k < N; k++) a.x[k * pp + i] = x[k];
#pragma unroll
      for (int k = 0; k < NP; k++) a.P[k * pp + i] = P[k];
    }
  }
  nan_guard(x, P, a.counters, live);
  if constexpr (ENS) {
    float xs[1][N];
#pragma unroll
    for (int k = 0; k < N; k++) xs[0][k] = x[k];
    const bool lv[1] = {live};
    ens_epilogue<9, 1>(a.in, xs, lv, bid);
  }
}

// The firmware ISR for the 9-state EKF in one pass (round 5; as k_isr_kf6 for KF6): the EKF9
// tick of k_ekf9t (cached tiled state), then the control half of VEHICLE_CTRL::update on the
// control step's rpm (the caller's plane or the ingested motor state, as fmskf_control reads
// it), then the 0x200 frame; every load of both steps issued before either computes.  One robot
// per lane, the clamped-index form.  Bit-identical to fmskf_tick + fmskf_control +
// fmskf_can_tx.  CPC: the control planes' cache policy.  CAN (fmskf_isr_tick_can): the tick's
// four C610 frames per robot first (can_lane.hpp), their rpm handed to the wheel loops in
// registers instead of read back from the motor state (the EKF9 measurement keeps the raw record).
// CNT: the motor state streamed non-temporal, so that it does not evict the cache-resident EKF9
// state (can_nt; 2^20 robots: 194 -> 155.4-156.2 us per tick against 195.8 for the two calls,
// kbench, two passes)
template <bool LIBM, bool SEQ, int CPC, bool COMP, bool CAN = false, bool CNT = false>
__global__ __launch_bounds__(kBlock) void k_isr_ekf9(KfArgs<MdEKF9, Ekf9Params> a, CtrlDev c, CtrlPrm p,
                                                    uint8_t *frames, const int16_t *rpm, CanArgs can) {
  constexpr int N = 9, NP = 45;
  const uint32_t bid = blockIdx.x;
  __shared__ float wtab[LIBM ? 1 : kBlock / 64][LIBM ? 1 : kWaveTab];
  float *stab = wtab[LIBM ? 0 : threadIdx.x >> 6];
  const uint64_t n = a.n;
  const uint64_t i = (uint64_t)bid * kBlock + threadIdx.x;
  const bool live = i < n;
  const uint64_t ic = live ? i : n - 1;
  Can4Lane<CNT> cl4;
  if constexpr (CAN) cl4.load(can, (uint64_t)bid * kBlock, (uint32_t)(ic - (uint64_t)bid * kBlock));
  float x[N], P[NP];
  WaveTable<LIBM> tv(a.in.sintab);
  const uint32_t sl = tile_slot(n, bid);
  const TileRows<float, N, 0> tx(a.x, bid, sl, 0);
  const TileRows<float, NP, 0> tp(a.P, bid, sl, 0);
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = tx.ld(k);
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = tp.ld(k);
  const bool have = a.in.valid == nullptr || a.in.valid[ic];
  const uint4 raw = ekf9_raw_at<false>(a.in.raw, ic);
  const uint64_t hb0 = (uint64_t)bid * kBlock;
  float lo = ld_chunk<float, 0>(a.prm.thlo, hb0, n, sl);
  Ekf9Lo<COMP, 0> cl;
  cl.load(a.prm.clo, bid, sl);
  uint2 rw;
  if constexpr (!CAN) rw = reinterpret_cast<const uint2 *>(rpm)[ic];
  CtrlLane<true, CPC> L;
  L.load(c, (uint32_t)ic);
  tv.store(stab);
  if constexpr (CAN) rw = cl4.step(can, live);
  ekf9_tick1<LIBM, true, true, SEQ, COMP>(a, raw, have, stab, x, P, lo, cl.v);
  if (live) {
    st_chunk<float, st_pol(0)>(a.prm.thlo, hb0, n, sl, lo);
    cl.store(a.prm.clo, bid, sl);
#pragma unroll
    for (int k = 0; k < N; k++) tx.st(k, x[k]);
#pragma unroll
    for (int k = 0; k < NP; k++) tp.st(k, P[k]);
  }
  nan_guard(x, P, a.counters, live);
  if (live) {
    const uint2 cw = L.step(c, p, (uint32_t)i, rw);
    if (frames) reinterpret_cast<uint2 *>(frames)[i] = tx_frame(cw);
  }
  if constexpr (CAN) cl4.finish(can, live);
}

// Two robots per lane (256-robot chunks b and b + G of the tiled state, G the tick blocks):
// robot B's 54 state loads and its raw record are issued before robot A's update, so they
// stream in while A computes (see launch_ekf9).
template <bool LIBM, bool SEQ, int CP, bool ENS = false, bool COMP = false>
__global__ __launch_bounds__(kBlock) void k_ekf9p(KfArgs<MdEKF9, Ekf9Params> a) {
  constexpr int N = 9, NP = 45;
  uint32_t bid = blockIdx.x;  // the tick block (the carried fold blocks come first)
  if constexpr (ENS) {
    if (ens_fold_front<9>(a.in, bid)) return;
  }
  __shared__ float wtab[LIBM ? 1 : kBlock / 64][LIBM ? 1 : kWaveTab];
  float *stab = wtab[LIBM ? 0 : threadIdx.x >> 6];
  const uint64_t n = a.n;
  const uint32_t ntiles = (uint32_t)((n + kBlock - 1) / kBlock);  // chunks of kBlock instances
  const uint32_t ta = bid, tb0 = bid + (ENS ? a.in.ens_grid : gridDim.x);
  const bool has_b = tb0 < ntiles;  // block-uniform
  const uint32_t tb = has_b ? tb0 : ta;
  const uint32_t t = threadIdx.x;
  auto slot = [&](uint32_t tile) -> uint32_t {
    const uint64_t b0 = (uint64_t)tile * kBlock;
    return b0 + t < n ? t : (uint32_t)(n - 1 - b0);
  };
  const uint64_t ia = (uint64_t)ta * kBlock + t, ib = (uint64_t)tb * kBlock + t;
  const bool live_a = ia < n, live_b = has_b && ib < n;
  const uint64_t iac = live_a ? ia : n - 1, ibc = ib < n ? ib : n - 1;
  WaveTable<LIBM> tv(a.in.sintab);
  const TileRows<float, N, CP> txa(a.x, ta, slot(ta), 0), txb(a.x, tb, slot(tb), 0);
  const TileRows<float, NP, CP> tpa(a.P, ta, slot(ta), 0), tpb(a.P, tb, slot(tb), 0);
  float xa[N], Pa[NP], xb[N], Pb[NP];
#pragma unroll
  for (int k = 0; k < N; k++) xa[k] = txa.ld(k);
#pragma unroll
  for (int k = 0; k < NP; k++) Pa[k] = tpa.ld(k);
  const uint4 ra = ekf9_raw_at<true>(a.in.raw, iac);
  const uint4 rb = ekf9_raw_at<true>(a.in.raw, ibc);
  const bool ha = a.in.valid == nullptr || a.in.valid[iac];
  const bool hb = a.in.valid == nullptr || a.in.valid[ibc];
#pragma unroll
  for (int k = 0; k < N; k++) xb[k] = txb.ld(k);
#pragma unroll
  for (int k = 0; k < NP; k++) Pb[k] = tpb.ld(k);
  float loa = ld_chunk<float, CP>(a.prm.thlo, (uint64_t)ta * kBlock, n, slot(ta));
  float lob = ld_chunk<float, CP>(a.prm.thlo, (uint64_t)tb * kBlock, n, slot(tb));
  Ekf9Lo<COMP, CP> cla, clb;
  cla.load(a.prm.clo, ta, slot(ta));
  clb.load(a.prm.clo, tb, slot(tb));
  tv.store(stab);
  ekf9_tick1<LIBM, true, true, SEQ, COMP>(a, ra, ha, stab, xa, Pa, loa, cla.v);
  if (live_a) {
    st_chunk<float, st_pol(CP)>(a.prm.thlo, (uint64_t)ta * kBlock, n, slot(ta), loa);
    cla.store(a.prm.clo, ta, slot(ta));
#pragma unroll
    for (int k = 0; k < N; k++) txa.st(k, xa[k]);
#pragma unroll
    for (int k = 0; k < NP; k++) tpa.st(k, Pa[k]);
  }
  nan_guard(xa, Pa, a.counters, live_a);
  float xs[ENS ? 2 : 1][N];
  if constexpr (ENS) {
#pragma unroll
    for (int k = 0; k < N; k++) xs[0][k] = xa[k];
  }
  ekf9_tick1<LIBM, true, true, SEQ, COMP>(a, rb, hb, stab, xb, Pb, lob, clb.v);
  if (live_b) {
    st_chunk<float, st_pol(CP)>(a.prm.thlo, (uint64_t)tb * kBlock, n, slot(tb), lob);
    clb.store(a.prm.clo, tb, slot(tb));
#pragma unroll
    for (int k = 0; k < N; k++) txb.st(k, xb[k]);
#pragma unroll
    for (int k = 0; k < NP; k++) tpb.st(k, Pb[k]);
  }
  nan_guard(xb, Pb, a.counters, live_b);
  if constexpr (ENS) {
#pragma unroll
    for (int k = 0; k < N; k++) xs[1][k] = xb[k];
    const bool lv[2] = {live_a, live_b};
    ens_epilogue<9, 2>(a.in, xs, lv, bid);
  }
}

// SEQ: R has no base/tip cross terms -> group-sequential update (base group, then tip group
// with the innovation of the updated state); otherwise the joint 8-measurement update.
template <bool SEQ, bool UPD, bool PRED>
__global__ __launch_bounds__(kBlock) void k_kf12d(KfArgs<MdKF12D, Kf12dParams> a) {
  constexpr int N = 12, NP = 78, M = 8;
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double x[N], P[NP];
  const uint32_t tl = FMSKF_TILED ? tile_w<double>() : 0;
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[st_at(tl, pp, N, k, i)];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[st_at(tl, pp, NP, k, i)];
  const double dt = a.prm.dt;
  const auto fdt = [&](int, int) { return dt; };
  for (uint32_t t = 0; t < a.in.n_ticks; t++) {
    const uint64_t base = (uint64_t)t * a.in.stride * M;
    if (UPD) {
      if (a.in.valid == nullptr || a.in.valid[(uint64_t)t * a.in.stride + i]) {
        if (SEQ) {
          double y[4];
#pragma unroll
          for (int q = 0; q < 4; q++) y[q] = a.in.z[base + q * a.in.stride + i] - x[MdKF12D_G1::h1(q)];
          y[0] = wrap_innov(y[0]);
          kf_update<MdKF12D_G1>(x, P, y, a.prm.r);
#pragma unroll
          for (int q = 0; q < 4; q++)
            y[q] = a.in.z[base + (4 + q) * a.in.stride + i] - x[MdKF12D_G2::h1(q)];
          kf_update<MdKF12D_G2>(x, P, y, a.prm.r2);
        } else {
          double y[M];
#pragma unroll
          for (int q = 0; q < M; q++) y[q] = a.in.z[base + q * a.in.stride + i] - x[MdKF12D::h1(q)];
          y[0] = wrap_innov(y[0]);
          kf_update<MdKF12D>(x, P, y, a.prm.r);
        }
      }
    }
    if (PRED) {
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const int p = q < 3 ? q : q + 3;
        x[p] = dfma(dt, x[p + 3], x[p]);
      }
      x[2] = wrap_pi(x[2]);
      kf_predict_cov<MdKF12D, decltype(fdt), double, 12, 78, true>(P, fdt, a.prm.q);
    }
  }
#pragma unroll
  for (int k = 0; k < N; k++) a.x[st_at(tl, pp, N, k, i)] = x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) a.P[st_at(tl, pp, NP, k, i)] = P[k];
  nan_guard(x, P, a.counters);
}

// ---------------------------------------------------------------------------
// KF12D, R positive definite: decorrelated scalar-sequential update (oracle
// orc_kf12d_decor_update) and the F P F^T + Q predict done per 2x2 (pos, vel) pair block.
// Only one 12-entry HP row is live at a time (the joint / group LDL^T updates hold 8x12 or
// 4x12 update matrices), so x, P and the temporaries fit 256 VGPRs: two waves per SIMD to
// overlap the fp64 arithmetic (~4 cycles per wave64 FMA) with the 1504-byte stream.
// ---------------------------------------------------------------------------
__device__ __forceinline__ constexpr int kf12_pos(int k) { return k < 3 ? k : k + 3; }

// Cinv and Q are 114 wave-uniform doubles (a device buffer, prm.coef).  Loaded all at once
// they exceed the scalar register file and spill through v_writelane / v_readlane; a pointer
// the compiler cannot see through keeps each group's scalar loads at the point of use.
typedef const __attribute__((address_space(4))) double *kparam_ptr;
__device__ __forceinline__ kparam_ptr opaque_param(const double *p) {
  uint64_t v = (uint64_t)p;
  asm volatile("" : "+s"(v));
  return (kparam_ptr)v;
}

// Exact-zero coefficients are skipped (the canonical order of the oracle's
// orc_kf12d_decor_update: a zero C^-1 entry contributes nothing, every sum starts from +0, and
// fma(c, p, +0) = c p up to the sign of a zero).  C^-1 of the default R (diagonal but for the
// two wheel velocities) is mostly exact zeros: 11 of the 20 off-diagonal entries the update
// reads, each a 12-wide dfma row of HP plus the innovation term.  SP (the host checked that
// every C^-1 entry off the diagonal and (3,2), and every Q entry outside the (pos, vel) pair
// blocks, is zero): those terms are dropped at compile time; the entries that may be nonzero
// are added through a select (the same bits as skipping a zero), as every entry is when !SP.
// Measured: runtime branches on the scalar coefficient instead of selects took the kernel to
// 256 VGPRs (1 wave per SIMD) and were not kept.
__device__ __forceinline__ constexpr bool kf12_cinv_sp(int a, int b) { return a == b || (a == 3 && b == 2); }
__device__ __forceinline__ double fma_nz(double c, double p, double acc) {
  const double v = dfma(c, p, acc);
  return c != 0.0 ? v : acc;
}

template <bool BLK, bool SP>
__device__ __forceinline__ void kf12d_decor_update(double (&x)[12], double (&P)[78], double (&y)[8],
                                                   const double *ci) {
#pragma unroll
  for (int a = 0; a < 8; a++) {
    const int b0 = (BLK && a >= 4) ? 4 : 0;
    const kparam_ptr c = opaque_param(ci + a * (a + 1) / 2);
    // the diagonal of C^-1 is 1 / C[a][a] > 0 (R positive definite): a plain fma; the other
    // entries through fma_nz (or, under SP, dropped where the host found them zero)
    auto term = [&](int b, double p, double acc) -> double {
      return b == a ? dfma(c[b], p, acc) : fma_nz(c[b], p, acc);
    };
    // constant trip counts (b over 0..7, filtered): every index stays compile-time after
    // unrolling (a b0..a loop left P indexed at run time, in scratch)
    auto used = [&](int b) { return b >= b0 && b <= a && (!SP || kf12_cinv_sp(a, b)); };
    double hp[12];
#pragma unroll
    for (int j = 0; j < 12; j++) {
      double s = 0.0;
#pragma unroll
      for (int b = 0; b < 8; b++)
        if (used(b)) s = term(b, P[pk(MdKF12D::h1(b), j)], s);
      hp[j] = s;
    }
    double s = 0.0, nu = 0.0;
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (used(b)) s = term(b, hp[MdKF12D::h1(b)], s);
    s = s + 1.0;
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (used(b)) nu = term(b, y[b], nu);
    const double si = 1.0 / s;
    const double g = nu * si;
#pragma unroll
    for (int j = 0; j < 12; j++) x[j] = dfma(hp[j], g, x[j]);
#pragma unroll
    for (int b = 0; b < 8; b++) y[b] = dfma(-hp[MdKF12D::h1(b)], g, y[b]);
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const double t = hp[i] * si;
#pragma unroll
      for (int j = 0; j <= i; j++) P[pk(i, j)] = dfma(-t, hp[j], P[pk(i, j)]);
    }
  }
}

// P <- F P F^T + Q with F = I + dt (pos <- vel): every 2x2 block {p_k, v_k} x {p_l, v_l} maps
// from its own four entries (a b / c d): pp = (a + dt c) + dt (b + dt d), vp = c + dt d,
// pv = b + dt d, vv = d; bit-identical to the generic T = F P, T F^T form (kf_predict_cov).
// Exactly-zero Q entries are not added (kf_predict_cov's SKIPQ); SP: the blocks k != l have
// no Q at all (checked on the host)
template <bool SP>
__device__ __forceinline__ void kf12d_predict_cov(double (&P)[78], double dt, const double *Q) {
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const kparam_ptr q = opaque_param(Q);
#pragma unroll
    for (int l = 0; l <= k; l++) {
      const bool hasq = !SP || k == l;
      auto addq = [&](double v, int e) -> double {
        if (!hasq) return v;
        const double qe = q[e];
        const double w = v + qe;
        return qe != 0.0 ? w : v;
      };
      const int pk_ = kf12_pos(k), vk = pk_ + 3, pl = kf12_pos(l), vl = pl + 3;
      const double a = P[pk(pk_, pl)], b = P[pk(pk_, vl)], c = P[pk(vk, pl)], d = P[pk(vk, vl)];
      const double t01 = dfma(dt, d, b);
      P[pk(pk_, pl)] = addq(dfma(dt, t01, dfma(dt, c, a)), pk(pk_, pl));
      P[pk(vk, pl)] = addq(dfma(dt, d, c), pk(vk, pl));
      if (k != l) P[pk(pk_, vl)] = addq(t01, pk(pk_, vl));
      P[pk(vk, vl)] = addq(d, pk(vk, vl));
    }
  }
}

// Planes through buffer descriptors: a 32-bit lane offset per access and no 64-bit address
// math.  SMALL: the 78 P planes fit one 4 GiB window (pitch < 6.8M), one descriptor per array
// and a scalar plane offset; otherwise one descriptor per plane (n < 2^29 lanes of 8 bytes).
// ENS: the record epilogue of fmskf_tick_ensemble; every lane then stays to the block
// reduction (lanes past N tick instance N-1, a clamped index, and store nothing)
template <bool BLK, bool UPD, bool PRED, bool SMALL, int CP = 0, bool ENS = false, bool SP = false>
__global__ __launch_bounds__(kBlock) void k_kf12s(KfArgs<MdKF12D, Kf12dParams> a) {
  constexpr int N = 12, NP = 78, M = 8;
  uint32_t bid = blockIdx.x;  // the tick block (the carried fold blocks come first)
  if constexpr (ENS) {
    if (ens_fold_front<12>(a.in, bid)) return;
  }
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t i0 = (uint64_t)bid * kBlock + threadIdx.x;
  const bool live = i0 < n;
  if (!ENS && !live) return;
  const uint64_t i = live ? i0 : n - 1;
  double x[N], P[NP];
  const auto rx = rsrc(a.x, pp * 8 * N), rp = rsrc(a.P, pp * 8 * NP);
  const uint32_t vo = (uint32_t)i * 8u;
  uint32_t ps = (uint32_t)pp * 8u;
  auto ld = [&](__amdgpu_buffer_rsrc_t r, const double *base, int k) -> double {
    if constexpr (SMALL) {
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, k * ps, 0));
    } else {  // one descriptor per plane (scalar work only)
      return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc(base + k * pp, pp * 8),
                                                                              vo, 0, 0));
    }
  };
  auto st = [&](__amdgpu_buffer_rsrc_t r, double *base, int k, double v) {
    if constexpr (SMALL) {
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, v), r, vo, k * ps, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, v), rsrc(base + k * pp, pp * 8),
                                            vo, 0, 0);
    }
  };
  // tiled layout (FMSKF_TILED): the block's chunk of its tile through a scalar descriptor (without ENS
  // lanes past N returned above, so a lane's slot is its thread index)
  const uint32_t slot = ENS ? tile_slot(n, bid) : threadIdx.x;
  const TileRows<double, N, CP> tx(a.x, bid, slot, 0);
  const TileRows<double, NP, CP> tp(a.P, bid, slot, 0);
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = FMSKF_TILED ? tx.ld(k) : ld(rx, a.x, k);
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = FMSKF_TILED ? tp.ld(k) : ld(rp, a.P, k);
  const double dt = a.prm.dt;
  for (uint32_t t = 0; t < a.in.n_ticks; t++) {
    if (UPD) {
      if (a.in.valid == nullptr || a.in.valid[(uint64_t)t * a.in.stride + i]) {
        const double *z = a.in.z + (uint64_t)t * a.in.stride * M;
        double y[M];
#pragma unroll
        for (int q = 0; q < M; q++) y[q] = z[q * a.in.stride + i] - x[MdKF12D::h1(q)];
        y[0] = wrap_innov(y[0]);
        kf12d_decor_update<BLK, SP>(x, P, y, a.prm.coef);
      }
    }
    if (PRED) {
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const int p = kf12_pos(q);
        x[p] = dfma(dt, x[p + 3], x[p]);
      }
      x[2] = wrap_pi(x[2]);
      kf12d_predict_cov<SP>(P, dt, a.prm.coef + 36);
    }
  }
  asm volatile("" : "+s"(ps));  // the store offsets are recomputed here, not held from the loads
  if (live) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      if constexpr (FMSKF_TILED) tx.st(k, x[k]);
      else st(rx, a.x, k, x[k]);
    }
#pragma unroll
    for (int k = 0; k < NP; k++) {
      if constexpr (FMSKF_TILED) tp.st(k, P[k]);
      else st(rp, a.P, k, P[k]);
    }
  }
  nan_guard(x, P, a.counters, live);
  if constexpr (ENS) {
    double xs[1][N];
#pragma unroll
    for (int k = 0; k < N; k++) xs[0][k] = x[k];
    const bool lv[1] = {live};
    ens_epilogue<12, 1>(a.in, xs, lv, bid);
  }
}

// fused tick + record (fmskf_tick_ensemble): the default single-tick kernel with the record
// epilogue (and the carried fold blocks past the tick blocks when in.fold_blocks is set);
// returns the tick grid (= the number of block records)
template <bool LIBM, bool SEQ, bool COMP>
static int launch_ekf9_ens(KfArgs<MdEKF9, Ekf9Params> a, const DevState &s, bool nt, hipStream_t st) {
  const unsigned carry = a.in.fold_blocks ? (unsigned)EnsRec<9>::LEN : 0u;
  if (!LIBM && s.n * (COMP ? 240 : 220) <= (256ull << 20)) {
    const uint32_t ntiles = (uint32_t)((s.n + kBlock - 1) / kBlock);
    const unsigned g2 = (ntiles + 1) / 2;
    a.in.ens_grid = g2;
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_EKF9P_LDS", true, 64u * 1024u);
    if (nt) launch_signal(k_ekf9p<false, SEQ, kStateNT, true, COMP>, dim3(g2 + carry), lds, st, a.in.ens_done, a);
    else launch_signal(k_ekf9p<false, SEQ, 0, true, COMP>, dim3(g2 + carry), lds, st, a.in.ens_done, a);
    return (int)g2;
  }
  // past the Infinity Cache the record epilogue (fp64 sums and their cross-lane reduction)
  // wants one more block per CU than the plain tick: 2^22, kbench, two passes: 331-335 us at
  // 64 KiB (2 blocks per CU), 307-308 at 32 KiB (3), 316 uncapped
  const unsigned g = grid_for(s.n).x;
  a.in.ens_grid = g;
  const unsigned lds = LIBM ? 0u : FMSKF_LDS_CAP("FMSKF_EKF9E_LDS", nt, 32u * 1024u);
  if (nt) launch_signal(k_ekf9t<LIBM, true, true, SEQ, kStateNT, true, COMP>, dim3(g + carry), lds, st, a.in.ens_done, a);
  else launch_signal(k_ekf9t<LIBM, true, true, SEQ, 0, true, COMP>, dim3(g + carry), lds, st, a.in.ens_done, a);
  return (int)g;
}

template <bool SEQ, bool COMP>
static int launch_ekf9_s(const KfArgs<MdEKF9, Ekf9Params> &a, const DevState &s, const TickIn &in, bool libm,
                         bool upd, bool pred, bool nt, hipStream_t st, int *ens_nb) {
  const dim3 g = grid_for(s.n);
  if (in.ens_blocks) {
    *ens_nb = libm ? launch_ekf9_ens<true, SEQ, COMP>(a, s, nt, st) : launch_ekf9_ens<false, SEQ, COMP>(a, s, nt, st);
    return (int)hipGetLastError();
  }
  // Single-tick kernel: two robots per lane (k_ekf9p) while the 216-byte state fits the 256 MiB
  // Infinity Cache, else one per lane (k_ekf9t); FMSKF_EKF9_VARIANT (read once) forces one of
  // them, 2 = k_ekf9p, 4 = k_ekf9t (the tests' cross-check at small N).  Measured (kbench, one
  // box, two passes): 2^20 k_ekf9t 74.8-74.9 us, k_ekf9p 71.2-71.9; 2^22 (HBM) k_ekf9t 336-338,
  // k_ekf9p 339.  A raised-priority load phase (s_setprio 3 while issuing the loads) measured
  // 71.2-73.9 at 2^20 and 342-343 at 2^22 and was removed.
  static const int var = [] {
    const char *e = getenv("FMSKF_EKF9_VARIANT");
    return e ? atoi(e) : 0;
  }();
  const int v = var == 2 || var == 4 ? var : (s.n * (COMP ? 240 : 220) <= (256ull << 20) ? 2 : 4);
  if (FMSKF_TILED && in.n_ticks == 1 && upd && pred && !libm && v == 2) {
    const uint32_t ntiles = (uint32_t)((s.n + kBlock - 1) / kBlock);
    const dim3 g2((ntiles + 1) / 2);
    // 64 KiB of dynamic LDS (2 blocks per CU): 2^20 71.2 -> 70.5-70.7 us (two passes)
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_EKF9P_LDS", true, 64u * 1024u);
    if (nt) k_ekf9p<false, SEQ, kStateNT, false, COMP><<<g2, kBlock, lds, st>>>(a);
    else k_ekf9p<false, SEQ, 0, false, COMP><<<g2, kBlock, lds, st>>>(a);
    return (int)hipGetLastError();
  }
  // predict-only launches run no update: one (SEQ = false) instantiation serves both
  if (in.n_ticks == 1) {
    if (libm) {
      if (upd && pred && nt) k_ekf9t<true, true, true, SEQ, kStateNT, false, COMP><<<g, kBlock, 0, st>>>(a);
      else if (upd && pred) k_ekf9t<true, true, true, SEQ, 0, false, COMP><<<g, kBlock, 0, st>>>(a);
      else if (upd) k_ekf9t<true, true, false, SEQ, 0, false, COMP><<<g, kBlock, 0, st>>>(a);
      else k_ekf9t<true, false, true, false, 0, false, COMP><<<g, kBlock, 0, st>>>(a);
    } else {
      // Past the Infinity Cache (non-temporal state) the occupancy is capped at 2 blocks per CU
      // with 64 KiB of dynamic LDS: fewer concurrent tile streams per HBM channel.  2^22:
      // 334.3-338.7 us uncapped, 332 at 32 KiB, 329.7-331.0 at 48 KiB, 326.8-330.9 at 64 KiB,
      // 382-383 at 80 KiB (kbench, two boxes, two passes each); the same-bytes tiled pattern
      // (membench) 299 us.  FMSKF_EKF9_LDS overrides the byte count.
      const unsigned lds = FMSKF_LDS_CAP("FMSKF_EKF9_LDS", nt, 64u * 1024u);
      if (upd && pred && nt) k_ekf9t<false, true, true, SEQ, kStateNT, false, COMP><<<g, kBlock, lds, st>>>(a);
      else if (upd && pred) k_ekf9t<false, true, true, SEQ, 0, false, COMP><<<g, kBlock, lds, st>>>(a);
      else if (upd) k_ekf9t<false, true, false, SEQ, 0, false, COMP><<<g, kBlock, 0, st>>>(a);
      else k_ekf9t<false, false, true, false, 0, false, COMP><<<g, kBlock, 0, st>>>(a);
    }
  } else if (libm) {
    if (upd && pred) k_ekf9<true, true, true, SEQ, COMP><<<g, kBlock, 0, st>>>(a);
    else if (upd) k_ekf9<true, true, false, SEQ, COMP><<<g, kBlock, 0, st>>>(a);
    else k_ekf9<true, false, true, false, COMP><<<g, kBlock, 0, st>>>(a);
  } else {
    if (upd && pred) k_ekf9<false, true, true, SEQ, COMP><<<g, kBlock, 0, st>>>(a);
    else if (upd) k_ekf9<false, true, false, SEQ, COMP><<<g, kBlock, 0, st>>>(a);
    else k_ekf9<false, false, true, false, COMP><<<g, kBlock, 0, st>>>(a);
  }
  return (int)hipGetLastError();
}

int launch_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &p, bool libm, bool upd,
                bool pred, hipStream_t st, int *ens_nb) {
  KfArgs<MdEKF9, Ekf9Params> a{s.n, s.pitch, (float *)s.x, (float *)s.P, in, s.counters, p};
  a.prm.thlo = s.thlo;
  a.prm.clo = s.xlo;  // FMSKF_CFG_COMP_POS
  if (!s.thlo || (s.xlo && !FMSKF_TILED)) return (int)hipErrorInvalidValue;
  const bool nt = FMSKF_TILED && state_nt(s.n * (s.xlo ? 60 : 55) * 4);
  if ((in.ens_blocks && (!FMSKF_TILED || !ens_nb || !upd || !pred || in.n_ticks != 1)) ||
      (in.fold_blocks && !in.ens_blocks))
    return (int)hipErrorInvalidValue;
  // canonical update order (oracle orc_ekf9_tick): sequential scalar updates when R is
  // diagonal, the joint LDL^T update otherwise
  const bool diag = ekf9_r_diagonal(p.r);
  if (s.xlo) return diag ? launch_ekf9_s<true, true>(a, s, in, libm, upd, pred, nt, st, ens_nb)
                         : launch_ekf9_s<false, true>(a, s, in, libm, upd, pred, nt, st, ens_nb);
  return diag ? launch_ekf9_s<true, false>(a, s, in, libm, upd, pred, nt, st, ens_nb)
              : launch_ekf9_s<false, false>(a, s, in, libm, upd, pred, nt, st, ens_nb);
}

template <bool LIBM, bool SEQ, bool COMP, bool CAN, bool CNT>
static int isr_ekf9_w(const KfArgs<MdEKF9, Ekf9Params> &a, const CtrlDev &c, const CtrlPrm &p, uint8_t *frames,
                      const int16_t *rpm, bool nt, hipStream_t st, const CanArgs &can) {
  const dim3 g = grid_for(c.n);
  if (nt) {
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_ISR_LDS", true, 48u * 1024u);
    k_isr_ekf9<LIBM, SEQ, kStateNT, COMP, CAN, CNT><<<g, kBlock, lds, st>>>(a, c, p, frames, rpm, can);
  } else {
    k_isr_ekf9<LIBM, SEQ, 0, COMP, CAN, CNT><<<g, kBlock, 0, st>>>(a, c, p, frames, rpm, can);
  }
  return (int)hipGetLastError();
}

template <bool LIBM, bool SEQ, bool COMP, bool CAN>
static int isr_ekf9_v(const KfArgs<MdEKF9, Ekf9Params> &a, const CtrlDev &c, const CtrlPrm &p, uint8_t *frames,
                      const int16_t *rpm, bool nt, hipStream_t st, const CanArgs &can) {
  if constexpr (CAN) {
    // the EKF9 state and the motor state together past the Infinity Cache: the motor state
    // streams non-temporal and the EKF9 state stays resident
    if (can_nt_flag(can)) return isr_ekf9_w<LIBM, SEQ, COMP, true, true>(a, c, p, frames, rpm, nt, st, can);
  }
  return isr_ekf9_w<LIBM, SEQ, COMP, CAN, false>(a, c, p, frames, rpm, nt, st, can);
}

template <bool SEQ, bool COMP, bool CAN>
static int isr_ekf9_c(const KfArgs<MdEKF9, Ekf9Params> &a, const CtrlDev &c, const CtrlPrm &p, uint8_t *frames,
                      const int16_t *rpm, bool nt, bool libm, hipStream_t st, const CanArgs &can) {
  return libm ? isr_ekf9_v<true, SEQ, COMP, CAN>(a, c, p, frames, rpm, nt, st, can)
              : isr_ekf9_v<false, SEQ, COMP, CAN>(a, c, p, frames, rpm, nt, st, can);
}

template <bool CAN>
static int isr_ekf9_l(const DevState &s, const TickIn &in, const Ekf9Params &prm, bool libm, const CtrlDev &c,
                      const CtrlPrm &p, const int16_t *rpm, uint8_t *frames, hipStream_t st, const CanArgs &can) {
  if (c.n == 0) return 0;
  const uint64_t sb = s.xlo ? 240 : 220;  // state bytes per robot (+ the compensation rows)
  if (!FMSKF_TILED || !s.thlo || in.n_ticks != 1 || !in.raw || (!CAN && !rpm) || state_nt(s.n * sb) ||
      c.pitch * 4 * 3 * kAxF >= 0xFFFFFFFFull)
    return (int)hipErrorNotSupported;
  KfArgs<MdEKF9, Ekf9Params> a{s.n, s.pitch, (float *)s.x, (float *)s.P, in, s.counters, prm};
  a.prm.thlo = s.thlo;
  a.prm.clo = s.xlo;
  const bool nt = state_nt(ctrl_state_bytes(c) + s.n * sb);
  const bool diag = ekf9_r_diagonal(prm.r);
  if (s.xlo) return diag ? isr_ekf9_c<true, true, CAN>(a, c, p, frames, rpm, nt, libm, st, can)
                         : isr_ekf9_c<false, true, CAN>(a, c, p, frames, rpm, nt, libm, st, can);
  return diag ? isr_ekf9_c<true, false, CAN>(a, c, p, frames, rpm, nt, libm, st, can)
              : isr_ekf9_c<false, false, CAN>(a, c, p, frames, rpm, nt, libm, st, can);
}

// fmskf_isr_tick for EKF9 in one kernel where it applies: one tick, the tiled EKF9 state
// cache-resident (past the Infinity Cache the tick kernel streams it non-temporal under its own
// occupancy cap: three kernels, as for KF6), the control planes in one 4 GiB window.
// hipErrorNotSupported otherwise
int launch_isr_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &prm, bool libm, const CtrlDev &c,
                    const CtrlPrm &p, const int16_t *rpm, uint8_t *frames, hipStream_t st) {
  return isr_ekf9_l<false>(s, in, prm, libm, c, p, rpm, frames, st, CanArgs{});
}

// the same with the tick's CAN RX fused in front (fmskf_isr_tick_can: no caller rpm)
int launch_isr_ekf9_can(const DevState &s, const TickIn &in, const Ekf9Params &prm, bool libm, const CtrlDev &c,
                        const CtrlPrm &p, uint8_t *frames, const uint8_t *can_frames, const int16_t *can_stamps,
                        const int8_t dir[4], hipStream_t st) {
  CanArgs ca;
  if (!can_args(s, can_frames, can_stamps, dir, ca)) return (int)hipErrorNotSupported;
  ca.nt = can_nt(s);
  return isr_ekf9_l<true>(s, in, prm, libm, c, p, nullptr, frames, st, ca);
}

int launch_kf12d(const DevState &s, const TickIn &in, const Kf12dParams &p, bool upd, bool pred,
                 hipStream_t st, int *ens_nb) {
  KfArgs<MdKF12D, Kf12dParams> a{s.n, s.pitch, (double *)s.x, (double *)s.P, in, s.counters, p};
  const dim3 g = grid_for(s.n);
  const bool small = FMSKF_TILED || s.pitch * 8 * 78 < 0xFFFFFFFFull;  // tiled: any N
  const bool nt = FMSKF_TILED && state_nt(s.n * 90 * 8);
  const bool sp = p.sparse != 0;
  if (in.fold_blocks && !in.ens_blocks) return (int)hipErrorInvalidValue;
  if (in.ens_blocks) {
    // fused tick + record (fmskf_tick_ensemble): the default kernel (decorrelated update,
    // tiled state) with the record epilogue; one record per tick block
    if (!FMSKF_TILED || !p.decor || !ens_nb || !upd || !pred || in.n_ticks != 1) return (int)hipErrorInvalidValue;
    const bool blk = kf12d_sequential(p.r);
    a.in.ens_grid = g.x;
    const dim3 ge(g.x + (in.fold_blocks ? (unsigned)EnsRec<12>::LEN : 0u));  // + the carried fold
    const hipEvent_t ev = in.ens_done;
    if (sp && nt) launch_signal(k_kf12s<true, true, true, true, kStateNT, true, true>, ge, 0, st, ev, a);
    else if (sp) launch_signal(k_kf12s<true, true, true, true, 0, true, true>, ge, 0, st, ev, a);
    else if (blk && nt) launch_signal(k_kf12s<true, true, true, true, kStateNT, true>, ge, 0, st, ev, a);
    else if (blk) launch_signal(k_kf12s<true, true, true, true, 0, true>, ge, 0, st, ev, a);
    else if (nt) launch_signal(k_kf12s<false, true, true, true, kStateNT, true>, ge, 0, st, ev, a);
    else launch_signal(k_kf12s<false, true, true, true, 0, true>, ge, 0, st, ev, a);
    *ens_nb = (int)g.x;
    return (int)hipGetLastError();
  }
  if (p.decor) {
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_KF12D_LDS", nt, 0u);
    // SP (the default R and Q: sparse C^-1 and Q, checked on the host) implies BLK; tiled
    // state, so SMALL holds for any N
    if (sp && small && upd && pred) {
      if (nt) k_kf12s<true, true, true, true, kStateNT, false, true><<<g, kBlock, lds, st>>>(a);
      else k_kf12s<true, true, true, true, 0, false, true><<<g, kBlock, lds, st>>>(a);
      return (int)hipGetLastError();
    }
    const bool blk = kf12d_sequential(p.r);
#define KF12S(B, S)                                                          \
  if (upd && pred && nt) k_kf12s<B, true, true, S, kStateNT><<<g, kBlock, lds, st>>>(a); \
  else if (upd && pred) k_kf12s<B, true, true, S><<<g, kBlock, lds, st>>>(a); \
  else if (upd) k_kf12s<B, true, false, S><<<g, kBlock, 0, st>>>(a);        \
  else k_kf12s<B, false, true, S><<<g, kBlock, 0, st>>>(a);
    if (blk && small) { KF12S(true, true) }
    else if (blk) { KF12S(true, false) }
    else if (small) { KF12S(false, true) }
    else { KF12S(false, false) }
#undef KF12S
  } else if (kf12d_sequential(p.r)) {
    if (upd && pred) k_kf12d<true, true, true><<<g, kBlock, 0, st>>>(a);
    else if (upd) k_kf12d<true, true, false><<<g, kBlock, 0, st>>>(a);
    else k_kf12d<true, false, true><<<g, kBlock, 0, st>>>(a);
  } else {
    if (upd && pred) k_kf12d<false, true, true><<<g, kBlock, 0, st>>>(a);
    else if (upd) k_kf12d<false, true, false><<<g, kBlock, 0, st>>>(a);
    else k_kf12d<false, false, true><<<g, kBlock, 0, st>>>(a);
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf
