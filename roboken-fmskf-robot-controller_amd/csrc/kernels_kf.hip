// kernels_kf.hip -- batched KF / EKF tick kernels for gfx950 (MI355X).
//
// One filter instance per lane; the whole per-instance state (x and the packed
// symmetric P) lives in VGPRs for the duration of the launch, so a tick reads
// and writes each state byte exactly once (HBM-bound by design, no MFMA: the
// matrices are <= 12x12 per instance).  State planes are SoA, so lane i of a
// wave touches consecutive addresses of every plane (coalesced 256 B per wave
// per plane).  F / H / Q / R are shared by all instances: H and the sparsity of
// F are compile-time model traits, Q / R / dt ride in the kernarg segment and
// are read with scalar loads (SGPRs).
//
// Operation order is the canonical one of oracle/orc_kf_generic.inc (Cholesky
// form of the update, T = F P then T F^T + Q with ascending-k sums), and the
// library is built with -ffp-contract=off, so GPU and oracle agree bit for bit.
#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"

#pragma clang fp contract(off)

namespace fmskf {

// ---------------------------------------------------------------------------
// model traits
// ---------------------------------------------------------------------------
// KF6: x = (px, py, th, vx, vy, w); H selects (th, w, vx, vy); F = [[I, dt I], [0, I]]
struct MdKF6 {
  using T = float;
  static constexpr int N = 6, M = 4;
  __host__ __device__ static constexpr int h1(int a) { return a == 0 ? 2 : a == 1 ? 5 : a == 2 ? 3 : 4; }
  __host__ __device__ static constexpr int h2(int) { return -1; }
  __host__ __device__ static constexpr bool pat(int i, int k) { return i < 3 && k == i + 3; }
};
// EKF9: x = (px, py, th, vbx, vby, w, bw, abx, aby); h(x) = (th, w+bw, abx, aby, vbx, vby)
struct MdEKF9 {
  using T = float;
  static constexpr int N = 9, M = 6;
  __host__ __device__ static constexpr int h1(int a) {
    return a == 0 ? 2 : a == 1 ? 5 : a == 2 ? 7 : a == 3 ? 8 : a == 4 ? 3 : 4;
  }
  __host__ __device__ static constexpr int h2(int a) { return a == 1 ? 6 : -1; }
  __host__ __device__ static constexpr bool pat(int i, int k) {
    return ((i == 0 || i == 1) && (k == 2 || k == 3 || k == 4)) || (i == 2 && k == 5) ||
           (i == 3 && k == 7) || (i == 4 && k == 8);
  }
};
// KF12D: KF6 base + arm tip (tx, ty, tz, tvx, tvy, tvz); H selects (th, w, vx, vy, tx, ty, tz, tvz)
struct MdKF12D {
  using T = double;
  static constexpr int N = 12, M = 8;
  __host__ __device__ static constexpr int h1(int a) {
    return a == 0 ? 2 : a == 1 ? 5 : a == 2 ? 3 : a == 3 ? 4 : a == 4 ? 6 : a == 5 ? 7 : a == 6 ? 8 : 11;
  }
  __host__ __device__ static constexpr int h2(int) { return -1; }
  __host__ __device__ static constexpr bool pat(int i, int k) {
    return (i < 3 || (i >= 6 && i < 9)) && k == i + 3;
  }
};

template <class Md, typename Prm>
struct KfArgs {
  uint64_t n;
  typename Md::T *x;
  typename Md::T *P;
  TickIn in;
  unsigned long long *counters;
  Prm prm;
};

// ---------------------------------------------------------------------------
// generic update / covariance predict (fully unrolled -> registers only)
// ---------------------------------------------------------------------------
template <class Md, typename T = typename Md::T, int N = Md::N, int M = Md::M,
          int NP = Md::N *(Md::N + 1) / 2>
__device__ __forceinline__ void kf_update(T (&x)[N], T (&P)[NP], const T (&y)[M], const T *R) {
  T HP[M][N];
#pragma unroll
  for (int a = 0; a < M; a++) {
#pragma unroll
    for (int j = 0; j < N; j++) {
      T v = P[pk(Md::h1(a), j)];
      if (Md::h2(a) >= 0) v = v + P[pk(Md::h2(a) < 0 ? 0 : Md::h2(a), j)];
      HP[a][j] = v;
    }
  }
  T L[M][M], inv[M];
#pragma unroll
  for (int a = 0; a < M; a++) {
#pragma unroll
    for (int b = 0; b <= a; b++) {
      T s = HP[a][Md::h1(b)];
      if (Md::h2(b) >= 0) s = s + HP[a][Md::h2(b) < 0 ? 0 : Md::h2(b)];
      s = s + R[pk(a, b)];
#pragma unroll
      for (int k = 0; k < b; k++) s = s - L[a][k] * L[b][k];
      if (a == b) {
        L[a][a] = dsqrt<T>(s);
        inv[a] = (T)1 / L[a][a];
      } else {
        L[a][b] = s * inv[b];
      }
    }
  }
  // U = L^-1 HP overwrites HP row by row; w = L^-1 y
  T w[M];
#pragma unroll
  for (int a = 0; a < M; a++) {
#pragma unroll
    for (int j = 0; j < N; j++) {
      T s = HP[a][j];
#pragma unroll
      for (int k = 0; k < a; k++) s = s - L[a][k] * HP[k][j];
      HP[a][j] = s * inv[a];
    }
    T s = y[a];
#pragma unroll
    for (int k = 0; k < a; k++) s = s - L[a][k] * w[k];
    w[a] = s * inv[a];
  }
#pragma unroll
  for (int j = 0; j < N; j++) {
    T t = HP[0][j] * w[0];
#pragma unroll
    for (int a = 1; a < M; a++) t = t + HP[a][j] * w[a];
    x[j] = x[j] + t;
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      T t = HP[0][i] * HP[0][j];
#pragma unroll
      for (int a = 1; a < M; a++) t = t + HP[a][i] * HP[a][j];
      P[pk(i, j)] = P[pk(i, j)] - t;
    }
  }
}

// P <- F P F^T + Q, F = I + Fv(i,k) on the compile-time pattern Md::pat
template <class Md, class FV, typename T = typename Md::T, int N = Md::N,
          int NP = Md::N *(Md::N + 1) / 2>
__device__ __forceinline__ void kf_predict_cov(T (&P)[NP], const FV &fv, const T *Q) {
  T Tm[N][N];
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j < N; j++) {
      T t = P[pk(i, j)];
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(i, k)) t = t + fv(i, k) * P[pk(k, j)];
      Tm[i][j] = t;
    }
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      T t = Tm[i][j];
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(j, k)) t = t + fv(j, k) * Tm[i][k];
      P[pk(i, j)] = t + Q[pk(i, j)];
    }
  }
}

// ---------------------------------------------------------------------------
// per-model measurement frontends and time updates
// ---------------------------------------------------------------------------
__device__ __forceinline__ void unpack4(uint2 r, int16_t (&o)[4]) {
  o[0] = (int16_t)(r.x & 0xFFFFu);
  o[1] = (int16_t)(r.x >> 16);
  o[2] = (int16_t)(r.y & 0xFFFFu);
  o[3] = (int16_t)(r.y >> 16);
}

// KF6 z = (deg2rad(yaw), -deg2rad(gz), wheel velocity rotated by the measured heading)
// (imu_task_main.cpp:102-104, util_mymath.hpp:16, imu_if_wt901c.cpp:113,
//  VD_vehicle_controller.cpp:21-33,47-51)
template <bool LIBM>
__device__ __forceinline__ void kf6_innov(const TickIn &in, uint64_t j, const float (&x)[6],
                                          float (&y)[4]) {
  const float yaw = in.yaw_deg[j];
  const float gz = in.gyro_z[j];
  int16_t r[4];
  unpack4(reinterpret_cast<const uint2 *>(in.rpm)[j], r);
  const float th = deg2rad(yaw);
  const float om = -deg2rad(gz);
  float vx, vy, vth;
  mdir_to_vdir(rpm_to_mvel(r[0]), rpm_to_mvel(r[1]), rpm_to_mvel(r[2]), rpm_to_mvel(r[3]), vx, vy,
               vth);
  const float rr = normalize_rad_0to2pi(th);
  const float c = cos_p<LIBM>(rr, in.sintab), s = sin_p<LIBM>(rr, in.sintab);
  const float z2 = (vx * c - vy * s) * 0.001f;
  const float z3 = (vx * s + vy * c) * 0.001f;
  y[0] = wrap_innov(th - x[2]);
  y[1] = om - x[5];
  y[2] = z2 - x[3];
  y[3] = z3 - x[4];
}

// EKF9 z from raw WT901 registers (imu_if_wt901c.cpp:96-99,107-113) + wheel rpm
__device__ __forceinline__ void ekf9_innov(const TickIn &in, uint64_t j, const float (&x)[9],
                                           float (&y)[6]) {
  const uint4 w = reinterpret_cast<const uint4 *>(in.raw)[j];
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

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
template <typename T, int N, int NP>
__device__ __forceinline__ void nan_guard(const T (&x)[N], const T (&P)[NP],
                                          unsigned long long *counters) {
  T acc = x[0];
#pragma unroll
  for (int k = 1; k < N; k++) acc = acc + x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) acc = acc + P[k];
  const bool bad = !__builtin_isfinite(acc);
  const unsigned long long m = __ballot(bad);
  if (m && (threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(counters, (unsigned long long)__popcll(m));
}

template <bool LIBM, bool UPD, bool PRED>
__global__ __launch_bounds__(kBlock) void k_kf6(KfArgs<MdKF6, Kf6Params> a) {
  constexpr int N = 6, NP = 21;
  const uint64_t n = a.n;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  float x[N], P[NP];
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[k * n + i];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[k * n + i];
  const float dt = a.prm.dt;
  for (uint32_t t = 0; t < a.in.n_ticks; t++) {
    const uint64_t j = (uint64_t)t * a.in.stride + i;
    if (UPD) {
      if (a.in.valid == nullptr || a.in.valid[j]) {
        float y[4];
        kf6_innov<LIBM>(a.in, j, x, y);
        kf_update<MdKF6>(x, P, y, a.prm.r);
      }
    }
    if (PRED) {
      x[0] = x[0] + dt * x[3];
      x[1] = x[1] + dt * x[4];
      x[2] = wrap_pi(x[2] + dt * x[5]);
      kf_predict_cov<MdKF6>(P, [&](int, int) { return dt; }, a.prm.q);
    }
  }
#pragma unroll
  for (int k = 0; k < N; k++) a.x[k * n + i] = x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) a.P[k * n + i] = P[k];
  nan_guard(x, P, a.counters);
}

template <bool LIBM, bool UPD, bool PRED>
__global__ __launch_bounds__(kBlock) void k_ekf9(KfArgs<MdEKF9, Ekf9Params> a) {
  constexpr int N = 9, NP = 45;
  const uint64_t n = a.n;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  float x[N], P[NP];
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[k * n + i];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[k * n + i];
  const float dt = a.prm.dt;
  for (uint32_t t = 0; t < a.in.n_ticks; t++) {
    const uint64_t j = (uint64_t)t * a.in.stride + i;
    if (UPD) {
      if (a.in.valid == nullptr || a.in.valid[j]) {
        float y[6];
        ekf9_innov(a.in, j, x, y);
        kf_update<MdEKF9>(x, P, y, a.prm.r);
      }
    }
    if (PRED) {
      const float rr = normalize_rad_0to2pi(x[2]);
      const float c = cos_p<LIBM>(rr, a.in.sintab), s = sin_p<LIBM>(rr, a.in.sintab);
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
#pragma unroll
  for (int k = 0; k < N; k++) a.x[k * n + i] = x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) a.P[k * n + i] = P[k];
  nan_guard(x, P, a.counters);
}

template <bool UPD, bool PRED>
__global__ __launch_bounds__(kBlock) void k_kf12d(KfArgs<MdKF12D, Kf12dParams> a) {
  constexpr int N = 12, NP = 78, M = 8;
  const uint64_t n = a.n;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  double x[N], P[NP];
#pragma unroll
  for (int k = 0; k < N; k++) x[k] = a.x[k * n + i];
#pragma unroll
  for (int k = 0; k < NP; k++) P[k] = a.P[k * n + i];
  const double dt = a.prm.dt;
  for (uint32_t t = 0; t < a.in.n_ticks; t++) {
    const uint64_t base = (uint64_t)t * a.in.stride * M;
    if (UPD) {
      if (a.in.valid == nullptr || a.in.valid[(uint64_t)t * a.in.stride + i]) {
        double y[M];
#pragma unroll
        for (int q = 0; q < M; q++) y[q] = a.in.z[base + q * a.in.stride + i] - x[MdKF12D::h1(q)];
        y[0] = wrap_innov(y[0]);
        kf_update<MdKF12D>(x, P, y, a.prm.r);
      }
    }
    if (PRED) {
#pragma unroll
      for (int q = 0; q < 6; q++) {
        const int p = q < 3 ? q : q + 3;
        x[p] = x[p] + dt * x[p + 3];
      }
      x[2] = wrap_pi(x[2]);
      kf_predict_cov<MdKF12D>(P, [&](int, int) { return dt; }, a.prm.q);
    }
  }
#pragma unroll
  for (int k = 0; k < N; k++) a.x[k * n + i] = x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) a.P[k * n + i] = P[k];
  nan_guard(x, P, a.counters);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline dim3 grid_for(uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

#define FMSKF_DISPATCH3(K, args, libm, upd, pred)                                   \
  do {                                                                             \
    if (libm) {                                                                    \
      if (upd && pred) K<true, true, true><<<g, kBlock, 0, st>>>(args);            \
      else if (upd) K<true, true, false><<<g, kBlock, 0, st>>>(args);              \
      else K<true, false, true><<<g, kBlock, 0, st>>>(args);                       \
    } else {                                                                       \
      if (upd && pred) K<false, true, true><<<g, kBlock, 0, st>>>(args);           \
      else if (upd) K<false, true, false><<<g, kBlock, 0, st>>>(args);             \
      else K<false, false, true><<<g, kBlock, 0, st>>>(args);                      \
    }                                                                              \
  } while (0)

int launch_kf6(const DevState &s, const TickIn &in, const Kf6Params &p, bool libm, bool upd,
               bool pred, hipStream_t st) {
  KfArgs<MdKF6, Kf6Params> a{s.n, (float *)s.x, (float *)s.P, in, s.counters, p};
  const dim3 g = grid_for(s.n);
  FMSKF_DISPATCH3(k_kf6, a, libm, upd, pred);
  return (int)hipGetLastError();
}

int launch_ekf9(const DevState &s, const TickIn &in, const Ekf9Params &p, bool libm, bool upd,
                bool pred, hipStream_t st) {
  KfArgs<MdEKF9, Ekf9Params> a{s.n, (float *)s.x, (float *)s.P, in, s.counters, p};
  const dim3 g = grid_for(s.n);
  FMSKF_DISPATCH3(k_ekf9, a, libm, upd, pred);
  return (int)hipGetLastError();
}

int launch_kf12d(const DevState &s, const TickIn &in, const Kf12dParams &p, bool upd, bool pred,
                 hipStream_t st) {
  KfArgs<MdKF12D, Kf12dParams> a{s.n, (double *)s.x, (double *)s.P, in, s.counters, p};
  const dim3 g = grid_for(s.n);
  if (upd && pred) k_kf12d<true, true><<<g, kBlock, 0, st>>>(a);
  else if (upd) k_kf12d<true, false><<<g, kBlock, 0, st>>>(a);
  else k_kf12d<false, true><<<g, kBlock, 0, st>>>(a);
  return (int)hipGetLastError();
}

}  // namespace fmskf
