// kf_generic.hpp -- model traits and the generic, fully unrolled KF building blocks
// shared by the tick kernels (one filter per lane, state in VGPRs).
//
// Operation order is the canonical one of oracle/orc_kf_generic.inc (Cholesky form of
// the update, T = F P then T F^T + Q with ascending-k sums); the library is built with
// -ffp-contract=off, so GPU and oracle agree bit for bit.
#pragma once
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

// KF12D measured in two groups: base (th, w, vx, vy) and arm tip (tx, ty, tz, tvz).  When R
// has no cross-group terms the joint update equals the two group updates in sequence
// (canonical order then: group 1, then group 2), which halves the live update matrices.
struct MdKF12D_G1 {
  using T = double;
  static constexpr int N = 12, M = 4;
  __host__ __device__ static constexpr int h1(int a) { return a == 0 ? 2 : a == 1 ? 5 : a == 2 ? 3 : 4; }
  __host__ __device__ static constexpr int h2(int) { return -1; }
};
struct MdKF12D_G2 {
  using T = double;
  static constexpr int N = 12, M = 4;
  __host__ __device__ static constexpr int h1(int a) { return a == 0 ? 6 : a == 1 ? 7 : a == 2 ? 8 : 11; }
  __host__ __device__ static constexpr int h2(int) { return -1; }
};

// Buffer descriptor (MI355X SRD, cdna_hip_programming.md T8) from wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(base), 0, (int)(uint32_t)(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes),
      0x00020000);
}
typedef unsigned int v2u32_t __attribute__((ext_vector_type(2)));
typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));

// One element of a plane at a lane of a 256-robot chunk starting at hb (wave-uniform: the
// wave's first lane rounded down; clamped lanes stay inside the chunk), through a scalar
// descriptor so the access carries the cache policy POL (any N up to the 2^30 cap: the lane
// offset stays below 256 elements).
template <typename T, int POL>
__device__ __forceinline__ T ld_chunk(const T *plane, uint64_t hb, uint64_t n, uint32_t li) {
  const auto r = rsrc(plane + hb, (n - hb) * sizeof(T));
  if constexpr (sizeof(T) == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, li * 8u, 0, POL);
    const uint32_t lo = v[0], hi = v[1];  // element copies (see kf6_load_in)
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, li * 4u, 0, POL));
  }
}
template <typename T, int POL>
__device__ __forceinline__ void st_chunk(T *plane, uint64_t hb, uint64_t n, uint32_t li, T v) {
  const auto r = rsrc(plane + hb, (n - hb) * sizeof(T));
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    v2u32_t w;
    w[0] = (uint32_t)u;
    w[1] = (uint32_t)(u >> 32);
    __builtin_amdgcn_raw_buffer_store_b64(w, r, li * 8u, 0, POL);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, li * 4u, 0, POL);
  }
}

// One descriptor for a whole plane array at a wave-uniform chunk base: the record count is the
// 4 GiB maximum (lanes are clamped, so no access needs the range check), so building it costs
// no clamp of a 64-bit byte count, and every plane of the array is reached through the scalar
// soffset (plane k at k * pitch * sizeof(T) bytes: the caller checks that this stays below
// 4 GiB).  One such descriptor per array replaces one per plane (ld_chunk / st_chunk).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_span(const void *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, -1, 0x00020000);
}
template <typename T, int POL>
__device__ __forceinline__ T ld_span(__amdgpu_buffer_rsrc_t r, uint32_t li, uint32_t soff) {
  if constexpr (sizeof(T) == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, li * 8u, soff, POL);
    const uint32_t lo = v[0], hi = v[1];  // element copies (see kf6_load_in)
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  } else {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, li * 4u, soff, POL));
  }
}
template <typename T, int POL>
__device__ __forceinline__ void st_span(__amdgpu_buffer_rsrc_t r, uint32_t li, uint32_t soff, T v) {
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    v2u32_t w;
    w[0] = (uint32_t)u;
    w[1] = (uint32_t)(u >> 32);
    __builtin_amdgcn_raw_buffer_store_b64(w, r, li * 8u, soff, POL);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, li * 4u, soff, POL);
  }
}

// One tiled state array (ROWS rows, W = tile_w<T>() wide; fmskf_internal.hpp st_at) as one
// chunk of kBlock instances sees it (by default the calling block's own chunk): the chunk's
// base is wave-uniform (a scalar descriptor), rows sit W elements apart (a scalar offset per
// row), the lane offset is t * sizeof(T) with t the lane's slot in the chunk (lanes past N pass
// the last instance's slot).  Any N: the descriptor spans the chunk's columns of one tile.
template <typename T, int ROWS, int CP = 0>
struct TileRows {
  static constexpr uint32_t W = tile_w<T>(), CPT = W / kBlock;
  __amdgpu_buffer_rsrc_t r;
  uint32_t vo;
  static __device__ __forceinline__ T *chunk_base(T *base, uint32_t c) {
    return base + (uint64_t)(c / CPT) * ((uint64_t)ROWS * W) + (uint64_t)(c % CPT) * kBlock;
  }
  static constexpr uint64_t kSpan = ((uint64_t)(ROWS - 1) * W + kBlock) * sizeof(T);
  __device__ __forceinline__ TileRows(T *base, uint32_t t)
      : r(rsrc(chunk_base(base, blockIdx.x), kSpan)), vo(t * (uint32_t)sizeof(T)) {}
  // chunk `chunk` (wave-uniform) instead of the block's own
  __device__ __forceinline__ TileRows(T *base, uint32_t chunk, uint32_t t, int)
      : r(rsrc(chunk_base(base, chunk), kSpan)), vo(t * (uint32_t)sizeof(T)) {}
  __device__ __forceinline__ T ld(int k) const {
    if constexpr (sizeof(T) == 8)
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, vo, k * W * 8, CP));
    else
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, vo, k * W * 4, CP));
  }
  __device__ __forceinline__ void st(int k, T v) const {
    if constexpr (sizeof(T) == 8)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, v), r, vo, k * W * 8, st_pol(CP));
    else
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, k * W * 4, st_pol(CP));
  }
};
// the lane's slot in chunk `bid` (by default its block's); lanes past N take the last
// instance's slot
__device__ __forceinline__ uint32_t tile_slot(uint64_t n, uint32_t bid) {
  const uint64_t b0 = (uint64_t)bid * kBlock;
  return b0 + threadIdx.x < n ? threadIdx.x : (uint32_t)(n - 1 - b0);
}
__device__ __forceinline__ uint32_t tile_slot(uint64_t n) { return tile_slot(n, blockIdx.x); }

template <class Md, typename Prm>
struct KfArgs {
  uint64_t n;
  uint64_t pitch;  // x / P plane pitch (elements)
  typename Md::T *x;
  typename Md::T *P;
  TickIn in;
  unsigned long long *counters;
  Prm prm;
};

// ---------------------------------------------------------------------------
// compensated heading (EKF9): the heading is kept as hi + lo, hi the fp32 state row and lo a
// hidden row of the rounding errors of every addition to it (TwoSum), renormalised once per
// update and once per predict.  The EKF9's rate split is inferred from heading differences over
// dt, so plain fp32 rounding of the heading (up to 2.4e-7 rad) is amplified by 1/dt into the
// omega / gyro-bias split; with the lo row the split stays within 7e-7 of the float64 filter
// (1.3e-5 without) -- tests/test_oracle_kf_long.py.  Canonical order of the oracle's th_add /
// th_norm (oracle/orc_kf_generic.inc).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void th_add(T &hi, T &lo, T d) {
  const T s = hi + d;
  const T bp = s - hi;
  const T e = (hi - (s - bp)) + (d - bp);
  hi = s;
  lo = lo + e;
}
template <typename T>
__device__ __forceinline__ void th_norm(T &hi, T &lo) {
  const T s = hi + lo;
  lo = lo - (s - hi);
  hi = s;
}

// Compensated entries by mask (KF6 with FMSKF_CFG_COMP_POS: CXM = x 0-1, CPM = packed P 0-2):
// lo[] holds the low parts of the states in CXM (ascending), then of the packed P entries in CPM
// (ascending); oracle orc_slot_x / orc_slot_p
__host__ __device__ constexpr int popc_c(unsigned long long v) { return v ? (int)(v & 1ull) + popc_c(v >> 1) : 0; }
template <unsigned CXM>
__host__ __device__ constexpr int slot_x(int j) { return popc_c(CXM & ((1ull << j) - 1ull)); }
template <unsigned CXM, unsigned long long CPM>
__host__ __device__ constexpr int slot_p(int k) { return popc_c(CXM) + popc_c(CPM & ((1ull << k) - 1ull)); }

// FMSKF_CFG_COMP_POS (KF6, EKF9): the compensated entries -- x 0-1 (px, py), packed P 0-2 (P00,
// P10, P11) -- in the kKf6LoRows low-part rows
constexpr unsigned kPosCXM = 3u;
constexpr unsigned long long kPosCPM = 7ull;

// ---------------------------------------------------------------------------
// generic update / covariance predict (fully unrolled -> registers only)
// CI >= 0: state CI is compensated (x[CI] + *lo, th_add instead of the plain addition)
// CXM / CPM: the compensated states / packed P entries (slot_x, slot_p in clo), each added to by
// TwoSum and renormalised after the update (x slots first); oracle orc_kf_update_m
// ---------------------------------------------------------------------------
// every compensated pair renormalised, x slots first (oracle orc_comp_norm)
template <unsigned CXM, unsigned long long CPM, typename T, int N, int NP>
__device__ __forceinline__ void comp_norm(T (&x)[N], T (&P)[NP], T *clo) {
#pragma unroll
  for (int j = 0; j < N; j++)
    if ((CXM >> j) & 1u) th_norm(x[j], clo[slot_x<CXM>(j)]);
#pragma unroll
  for (int k = 0; k < NP; k++)
    if ((CPM >> k) & 1ull) th_norm(P[k], clo[slot_p<CXM, CPM>(k)]);
}

template <class Md, int CI = -1, typename T = typename Md::T, int N = Md::N, int M = Md::M,
          int NP = Md::N *(Md::N + 1) / 2, unsigned CXM = 0, unsigned long long CPM = 0>
__device__ __forceinline__ void kf_update(T (&x)[N], T (&P)[NP], const T (&y)[M], const T *R,
                                          T *lo = nullptr, T *clo = nullptr) {
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
  // S = H P H^T + R = L D L^T (L unit lower, no square roots); E[a][b] = L[a][b] D[b]
  // is the pre-division value of the recurrence
  T L[M][M], E[M][M], dinv[M];
#pragma unroll
  for (int a = 0; a < M; a++) {
#pragma unroll
    for (int b = 0; b <= a; b++) {
      T s = HP[a][Md::h1(b)];
      if (Md::h2(b) >= 0) s = s + HP[a][Md::h2(b) < 0 ? 0 : Md::h2(b)];
      s = s + R[pk(a, b)];
#pragma unroll
      for (int k = 0; k < b; k++) s = dfma<T>(-L[a][k], E[b][k], s);
      if (a == b) {
        dinv[a] = (T)1 / s;
      } else {
        E[a][b] = s;
        L[a][b] = s * dinv[b];
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
      for (int k = 0; k < a; k++) s = dfma<T>(-L[a][k], HP[k][j], s);
      HP[a][j] = s;
    }
    T s = y[a];
#pragma unroll
    for (int k = 0; k < a; k++) s = dfma<T>(-L[a][k], w[k], s);
    w[a] = s;
  }
  // x += U^T (D^-1 w),  P -= U^T (D^-1 U)
  T vw[M], V[M][N];
#pragma unroll
  for (int a = 0; a < M; a++) {
    vw[a] = w[a] * dinv[a];
#pragma unroll
    for (int j = 0; j < N; j++) V[a][j] = HP[a][j] * dinv[a];
  }
#pragma unroll
  for (int j = 0; j < N; j++) {
    T t = HP[0][j] * vw[0];
#pragma unroll
    for (int a = 1; a < M; a++) t = dfma<T>(HP[a][j], vw[a], t);
    if (j == CI) th_add(x[j], *lo, t);
    else if ((CXM >> j) & 1u) th_add(x[j], clo[slot_x<CXM>(j)], t);
    else x[j] = x[j] + t;
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      T t = HP[0][i] * V[0][j];
#pragma unroll
      for (int a = 1; a < M; a++) t = dfma<T>(HP[a][i], V[a][j], t);
      if ((CPM >> pk(i, j)) & 1ull) th_add(P[pk(i, j)], clo[slot_p<CXM, CPM>(pk(i, j))], -t);
      else P[pk(i, j)] = P[pk(i, j)] - t;
    }
  }
  comp_norm<CXM, CPM>(x, P, clo);
}

// Diagonal R: the measurements are independent, so the joint update equals M scalar updates
// in sequence (a = 0 .. M-1, each on the state the previous one left; the innovations of the
// later measurements follow the state: y_b -= H_b K_a y_a).  Per measurement: hp = H_a P (a row
// of P, or the sum of two), s = H_a hp + r_aa, g = y_a / s, x += hp g, P -= (hp / s) hp^T.
// About 2/3 of the LDL^T form's VALU (EKF9: no 6x9 U / V matrices, no forward substitution).
// Canonical order of oracle orc_kf_update_seq.
// CXM / CPM (clo): compensated entries as in kf_update, renormalised after the last measurement
template <class Md, int CI = -1, typename T = typename Md::T, int N = Md::N, int M = Md::M,
          int NP = Md::N *(Md::N + 1) / 2, unsigned CXM = 0, unsigned long long CPM = 0>
__device__ __forceinline__ void kf_update_seq(T (&x)[N], T (&P)[NP], T (&y)[M], const T *R,
                                              T *lo = nullptr, T *clo = nullptr) {
#pragma unroll
  for (int a = 0; a < M; a++) {
    T hp[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
      T v = P[pk(Md::h1(a), j)];
      if (Md::h2(a) >= 0) v = v + P[pk(Md::h2(a) < 0 ? 0 : Md::h2(a), j)];
      hp[j] = v;
    }
    T s = hp[Md::h1(a)];
    if (Md::h2(a) >= 0) s = s + hp[Md::h2(a) < 0 ? 0 : Md::h2(a)];
    s = s + R[pk(a, a)];
    const T si = (T)1 / s;
    const T g = y[a] * si;
#pragma unroll
    for (int j = 0; j < N; j++) {
      if (j == CI) th_add(x[j], *lo, hp[j] * g);
      else if ((CXM >> j) & 1u) th_add(x[j], clo[slot_x<CXM>(j)], hp[j] * g);
      else x[j] = dfma<T>(hp[j], g, x[j]);
    }
#pragma unroll
    for (int b = a + 1; b < M; b++) {
      T h = hp[Md::h1(b)];
      if (Md::h2(b) >= 0) h = h + hp[Md::h2(b) < 0 ? 0 : Md::h2(b)];
      y[b] = dfma<T>(-h, g, y[b]);
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const T t = hp[i] * si;
#pragma unroll
      for (int j = 0; j <= i; j++) {
        if ((CPM >> pk(i, j)) & 1ull) th_add(P[pk(i, j)], clo[slot_p<CXM, CPM>(pk(i, j))], -(t * hp[j]));
        else P[pk(i, j)] = dfma<T>(-t, hp[j], P[pk(i, j)]);
      }
    }
  }
  comp_norm<CXM, CPM>(x, P, clo);
}

// P <- F P F^T + Q, F = I + Fv(i,k) on the compile-time pattern Md::pat
// SKIPQ: an exactly-zero Q entry is not added (a wave-uniform branch on the kernel-argument Q;
// the canonical KF12D order, oracle orc_kf12d_tick: t + 0 only differs from t for t = -0)
template <class Md, class FV, typename T = typename Md::T, int N = Md::N,
          int NP = Md::N *(Md::N + 1) / 2, bool SKIPQ = false>
__device__ __forceinline__ void kf_predict_cov(T (&P)[NP], const FV &fv, const T *Q) {
  T Tm[N][N];
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j < N; j++) {
      T t = P[pk(i, j)];
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(i, k)) t = dfma<T>(fv(i, k), P[pk(k, j)], t);
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
        if (Md::pat(j, k)) t = dfma<T>(fv(j, k), Tm[i][k], t);
      if (!SKIPQ || Q[pk(i, j)] != T(0)) t = t + Q[pk(i, j)];
      P[pk(i, j)] = t;
    }
  }
}

// kf_predict_cov with the packed entries in CPM compensated (lo slots after the CXM states):
// such an entry starts from its old hi / lo pair and takes, by TwoSum, the rounded products
// fv(i,k) P[k][j] (pat(i,k), ascending k), then fv(j,k) T[i][k] (pat(j,k), ascending k), then
// Q, then th_norm; every other entry as kf_predict_cov.  Oracle orc_kf_predict_cov_c.
template <class Md, unsigned CXM, unsigned long long CPM, class FV, typename T = typename Md::T,
          int N = Md::N, int NP = Md::N *(Md::N + 1) / 2>
__device__ __forceinline__ void kf_predict_cov_c(T (&P)[NP], const FV &fv, const T *Q, T *lo) {
  T Tm[N][N];
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j < N; j++) {
      T t = P[pk(i, j)];
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(i, k)) t = dfma<T>(fv(i, k), P[pk(k, j)], t);
      Tm[i][j] = t;
    }
  }
  T hi[NP];
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      if (!((CPM >> pk(i, j)) & 1ull)) continue;
      T h = P[pk(i, j)];
      T &l = lo[slot_p<CXM, CPM>(pk(i, j))];
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(i, k)) th_add(h, l, fv(i, k) * P[pk(k, j)]);
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(j, k)) th_add(h, l, fv(j, k) * Tm[i][k]);
      th_add(h, l, Q[pk(i, j)]);
      th_norm(h, l);
      hi[pk(i, j)] = h;
    }
  }
#pragma unroll
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      if ((CPM >> pk(i, j)) & 1ull) {
        P[pk(i, j)] = hi[pk(i, j)];
        continue;
      }
      T t = Tm[i][j];
#pragma unroll
      for (int k = 0; k < N; k++)
        if (Md::pat(j, k)) t = dfma<T>(fv(j, k), Tm[i][k], t);
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

// Count instances whose state became non-finite (one atomic per wave, rare path).
template <typename T, int N, int NP>
__device__ __forceinline__ void nan_guard(const T (&x)[N], const T (&P)[NP],
                                          unsigned long long *counters, bool live = true) {
  T acc = x[0];
#pragma unroll
  for (int k = 1; k < N; k++) acc = acc + x[k];
#pragma unroll
  for (int k = 0; k < NP; k++) acc = acc + P[k];
  const bool bad = live && !__builtin_isfinite(acc);
  const unsigned long long m = __ballot(bad);
  if (m && (threadIdx.x & 63) == __builtin_ctzll(m))
    atomicAdd(counters, (unsigned long long)__popcll(m));
}

// Per-wave copy of the 513-entry table: the constructor issues the lane's 9 loads, store()
// writes them to the wave's LDS slice (waits only on those loads, the oldest in flight)
constexpr int kWaveTab = 520;
template <bool LIBM>
struct WaveTable {
  float v[LIBM ? 1 : 9];
  __device__ __forceinline__ explicit WaveTable(const float *g) {
    if constexpr (!LIBM) {
      const uint32_t lane = threadIdx.x & 63;
#pragma unroll
      for (int k = 0; k < 9; k++) v[k] = (lane + 64 * k) < 513 ? g[lane + 64 * k] : 0.f;
    }
  }
  __device__ __forceinline__ void store(float *stab) const {
    if constexpr (!LIBM) {
      const uint32_t lane = threadIdx.x & 63;
#pragma unroll
      for (int k = 0; k < 9; k++)
        if (lane + 64 * k < 513) stab[lane + 64 * k] = v[k];
      __builtin_amdgcn_wave_barrier();  // same-wave LDS ops retire in order
    }
  }
};

static inline dim3 grid_for(uint64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }

}  // namespace fmskf
