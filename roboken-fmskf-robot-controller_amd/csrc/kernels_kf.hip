// kernels_kf.hip -- 9-state EKF (fp32) and 12-state KF (fp64) tick kernels for gfx950.
//
// One filter instance per lane; the per-instance state (x and the packed symmetric P)
// lives in VGPRs for the whole launch, so a tick reads and writes each state byte
// exactly once (HBM-bound by design, no MFMA: matrices are <= 12x12 per instance).
// State planes are SoA: lane i of a wave touches consecutive addresses of every plane.
// F / H / Q / R are shared: H and the sparsity of F are compile-time model traits
// (kf_generic.hpp), Q / R / dt ride in the kernarg segment (scalar loads, SGPRs).
// The 6-state headline kernel lives in kernels_kf6.hip.
#include "kf_generic.hpp"

#pragma clang fp contract(off)

namespace fmskf {

// EKF9 z from raw WT901 registers (imu_if_wt901c.cpp:96-99,107-113) + wheel rpm
__device__ __forceinline__ void ekf9_innov(const uint4 w, const float (&x)[9], float (&y)[6]) {
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
  y[0] = wrap_innov(z0 - x[2]);
  y[1] = z1 - (x[5] + x[6]);
  y[2] = z2 - x[7];
  y[3] = z3 - x[8];
  y[4] = z4 - x[3];
  y[5] = z5 - x[4];
}

// one EKF9 tick (update with the measurement frontend, then the nonlinear predict)
template <bool LIBM, bool UPD, bool PRED>
__device__ __forceinline__ void ekf9_tick1(const KfArgs<MdEKF9, Ekf9Params> &a, const uint4 raw,
                                           bool have, const float *stab, float (&x)[9],
                                           float (&P)[45]) {
  const float dt = a.prm.dt;
  if (UPD && have) {
    float y[6];
    ekf9_innov(raw, x, y);
    kf_update<MdEKF9>(x, P, y, a.prm.r);
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
    x[0] = x[0] + vwx * dt;
    x[1] = x[1] + vwy * dt;
    x[2] = wrap_pi(x[2] + x[5] * dt);
    x[3] = x[3] + x[7] * dt;
    x[4] = x[4] + x[8] * dt;
    auto fv = [&](int r, int k) -> float {
      if (r == 0) return k == 2 ? f02 : k == 3 ? f03 : f04;
      if (r == 1) return k == 2 ? f12 : k == 3 ? f13 : f14;
      return dt;
    };
    kf_predict_cov<MdEKF9>(P, fv, a.prm.q);
  }
}

// tick_many: T ticks per launch, state in VGPRs; the next tick's raw record (16 B) and validity
// byte are loaded while the current tick computes (ping-pong registers, loop unrolled by two)
template <bool LIBM, bool UPD, bool PRED>
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
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[k * pp + ic];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[k * pp + ic];
  uint4 ra = raw_at(0), rb;
  bool ha = have_at(0), hb;
  for (uint32_t t = 0; t < T; t += 2) {
    if (t + 1 < T) {
      rb = raw_at(t + 1);
      hb = have_at(t + 1);
    }
    ekf9_tick1<LIBM, UPD, PRED>(a, ra, ha, stab, x, P);
    if (t + 1 >= T) break;
    if (t + 2 < T) {
      ra = raw_at(t + 2);
      ha = have_at(t + 2);
    }
    ekf9_tick1<LIBM, UPD, PRED>(a, rb, hb, stab, x, P);
  }
  if (live) {
#pragma unroll
    for (int k = 0; k < N; k++) a.x[k * pp + i] = x[k];
#pragma unroll
    for (int k = 0; k < NP; k++) a.P[k * pp + i] = P[k];
  }
  nan_guard(x, P, a.counters, live);
}

// Single tick, straight line (as k_kf6t): no tick loop, clamped index for lanes past N (only
// their stores and NaN count are masked), every load issued before the table barrier.
template <bool LIBM, bool UPD, bool PRED>
__global__ __launch_bounds__(kBlock) void k_ekf9t(KfArgs<MdEKF9, Ekf9Params> a) {
  constexpr int N = 9, NP = 45;
  __shared__ float wtab[LIBM ? 1 : kBlock / 64][LIBM ? 1 : kWaveTab];
  float *stab = wtab[LIBM ? 0 : threadIdx.x >> 6];
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = i < n;
  const uint64_t ic = live ? i : n - 1;
  float x[N], P[NP];
  WaveTable<LIBM> tv(a.in.sintab);  // wave-private table copy, loads issued first
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[k * pp + ic];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[k * pp + ic];
  const bool have = a.in.valid == nullptr || a.in.valid[ic];
  const uint4 raw = UPD ? reinterpret_cast<const uint4 *>(a.in.raw)[ic] : make_uint4(0, 0, 0, 0);
  tv.store(stab);
  ekf9_tick1<LIBM, UPD, PRED>(a, raw, have, stab, x, P);
  if (live) {
#pragma unroll
    for (int k = 0; k < N; k++) a.x[k * pp + i] = x[k];
#pragma unroll
    for (int k = 0; k < NP; k++) a.P[k * pp + i] = P[k];
  }
  nan_guard(x, P, a.counters, live);
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
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[k * pp + i];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[k * pp + i];
  const double dt = a.prm.dt;
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
      kf_predict_cov<MdKF12D>(P, [&](int, int) { return dt; }, a.prm.q);
    }
  }
#pragma unroll
  for (int k = 0; k < N; k++) a.x[k * pp + i] = x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) a.P[k * pp + i] = P[k];
  nan_guard(x, P, a.counters);
}

int launch_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &p, bool libm, bool upd,
                bool pred, hipStream_t st) {
  KfArgs<MdEKF9, Ekf9Params> a{s.n, s.pitch, (float *)s.x, (float *)s.P, in, s.counters, p};
  const dim3 g = grid_for(s.n);
  if (in.n_ticks == 1) {
    if (libm) {
      if (upd && pred) k_ekf9t<true, true, true><<<g, kBlock, 0, st>>>(a);
      else if (upd) k_ekf9t<true, true, false><<<g, kBlock, 0, st>>>(a);
      else k_ekf9t<true, false, true><<<g, kBlock, 0, st>>>(a);
    } else {
      if (upd && pred) k_ekf9t<false, true, true><<<g, kBlock, 0, st>>>(a);
      else if (upd) k_ekf9t<false, true, false><<<g, kBlock, 0, st>>>(a);
      else k_ekf9t<false, false, true><<<g, kBlock, 0, st>>>(a);
    }
  } else if (libm) {
    if (upd && pred) k_ekf9<true, true, true><<<g, kBlock, 0, st>>>(a);
    else if (upd) k_ekf9<true, true, false><<<g, kBlock, 0, st>>>(a);
    else k_ekf9<true, false, true><<<g, kBlock, 0, st>>>(a);
  } else {
    if (upd && pred) k_ekf9<false, true, true><<<g, kBlock, 0, st>>>(a);
    else if (upd) k_ekf9<false, true, false><<<g, kBlock, 0, st>>>(a);
    else k_ekf9<false, false, true><<<g, kBlock, 0, st>>>(a);
  }
  return (int)hipGetLastError();
}

int launch_kf12d(const DevState &s, const TickIn &in, const Kf12dParams &p, bool upd, bool pred,
                 hipStream_t st) {
  KfArgs<MdKF12D, Kf12dParams> a{s.n, s.pitch, (double *)s.x, (double *)s.P, in, s.counters, p};
  const dim3 g = grid_for(s.n);
  if (kf12d_sequential(p.r)) {
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
