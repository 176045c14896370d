// kernels_misc.hip -- sin/cos policy evaluation and the ensemble statistics reduction.
//
// Ensemble: mean and covariance of the state x across all instances of a rank, in fp64.
// Each thread accumulates shifted moment sums of its grid-stride instances (no division
// in the streaming loop), waves sum by a fixed xor butterfly, the 4 waves of a block
// through LDS in wave order, and one block folds the per-block sums in block order and
// converts them to the Chan/Golub/LeVeque record {count, mean[n], M2 packed[n(n+1)/2]}
// that ranks all-gather and combine in rank order.  No atomics anywhere: the result is
// bitwise reproducible run to run.
#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"

#pragma clang fp contract(off)

namespace fmskf {

template <bool LIBM>
__global__ __launch_bounds__(kBlock) void k_trig(const float *x, float *sv, float *cv, uint64_t n,
                                                 const float *tab) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  sv[i] = sin_p<LIBM>(x[i], tab);
  cv[i] = cos_p<LIBM>(x[i], tab);
}

int launch_trig(const float *x, float *sv, float *cv, uint64_t n, bool libm, const float *tab,
                hipStream_t st) {
  if (n == 0) return 0;
  const dim3 g((unsigned)((n + kBlock - 1) / kBlock));
  if (libm) k_trig<true><<<g, kBlock, 0, st>>>(x, sv, cv, n, tab);
  else k_trig<false><<<g, kBlock, 0, st>>>(x, sv, cv, n, tab);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// ensemble
// ---------------------------------------------------------------------------
template <int NX>
struct EnsRec {
  static constexpr int NP = NX * (NX + 1) / 2;
  static constexpr int LEN = 1 + NX + NP;
  double v[LEN];
};

// Plain sums of a record {count, S1[n], S2 packed} over the block: butterfly over the wave
// (fixed xor order), then the 4 waves through LDS in wave order.  Deterministic.
template <int LEN>
__device__ __forceinline__ void sum_block(double (&v)[LEN], double *lds) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
    for (int k = 0; k < LEN; k++) v[k] = v[k] + __shfl_xor(v[k], off, 64);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < LEN; k++) lds[wave * LEN + k] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < LEN; k++) {
      double s = lds[k];
      for (int w = 1; w < kBlock / 64; w++) s = s + lds[w * LEN + k];
      v[k] = s;
    }
  }
}

// Shifted moment sums: S1 = sum(x - x0), S2 = sum((x - x0)(x - x0)^T) with the shift x0 =
// instance 0's state (the same for every block), fp64, no division in the streaming loop.
template <int NX, typename T>
__global__ __launch_bounds__(kBlock) void k_ens_partial(const T *x, uint64_t n, double *blocks) {
  constexpr int LEN = EnsRec<NX>::LEN;
  __shared__ double lds[(kBlock / 64) * LEN];
  double sh[NX], v[LEN];
#pragma unroll
  for (int k = 0; k < NX; k++) sh[k] = (double)x[k * n];
#pragma unroll
  for (int k = 0; k < LEN; k++) v[k] = 0.0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    double d[NX];
#pragma unroll
    for (int k = 0; k < NX; k++) {
      d[k] = (double)x[k * n + i] - sh[k];
      v[1 + k] = v[1 + k] + d[k];
    }
#pragma unroll
    for (int p = 0; p < NX; p++)
#pragma unroll
      for (int q = 0; q <= p; q++) v[1 + NX + p * (p + 1) / 2 + q] += d[p] * d[q];
    v[0] = v[0] + 1.0;
  }
  sum_block<LEN>(v, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < LEN; k++) blocks[(uint64_t)blockIdx.x * LEN + k] = v[k];
  }
}

// Sum the block records (thread t: blocks t, t+256, ... in order), then convert the
// shifted sums to the {count, mean, M2} record: mean = x0 + S1/c, M2 = S2 - S1 S1^T / c.
template <int NX, typename T>
__global__ __launch_bounds__(kBlock) void k_ens_fold(const T *x, uint64_t n, const double *blocks,
                                                     int nblocks, double *out) {
  constexpr int LEN = EnsRec<NX>::LEN;
  __shared__ double lds[(kBlock / 64) * LEN];
  double v[LEN];
#pragma unroll
  for (int k = 0; k < LEN; k++) v[k] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock) {
#pragma unroll
    for (int k = 0; k < LEN; k++) v[k] = v[k] + blocks[(uint64_t)b * LEN + k];
  }
  sum_block<LEN>(v, lds);
  if (threadIdx.x == 0) {
    const double c = v[0];
    out[0] = c;
#pragma unroll
    for (int k = 0; k < NX; k++) out[1 + k] = (double)x[k * n] + (c > 0.0 ? v[1 + k] / c : 0.0);
#pragma unroll
    for (int p = 0; p < NX; p++)
#pragma unroll
      for (int q = 0; q <= p; q++) {
        const int k = 1 + NX + p * (p + 1) / 2 + q;
        out[k] = c > 0.0 ? v[k] - v[1 + p] * v[1 + q] / c : 0.0;
      }
  }
}

int ensemble_nblocks(uint64_t n) {
  uint64_t b = (n + kBlock - 1) / kBlock;
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

int launch_ensemble(const DevState &s, int nx, bool f64, double *blocks, double *out,
                    hipStream_t st) {
  const int nb = ensemble_nblocks(s.n);
  if (nx == 6 && !f64) {
    k_ens_partial<6, float><<<nb, kBlock, 0, st>>>((const float *)s.x, s.n, blocks);
    k_ens_fold<6, float><<<1, kBlock, 0, st>>>((const float *)s.x, s.n, blocks, nb, out);
  } else if (nx == 9 && !f64) {
    k_ens_partial<9, float><<<nb, kBlock, 0, st>>>((const float *)s.x, s.n, blocks);
    k_ens_fold<9, float><<<1, kBlock, 0, st>>>((const float *)s.x, s.n, blocks, nb, out);
  } else if (nx == 12 && f64) {
    k_ens_partial<12, double><<<nb, kBlock, 0, st>>>((const double *)s.x, s.n, blocks);
    k_ens_fold<12, double><<<1, kBlock, 0, st>>>((const double *)s.x, s.n, blocks, nb, out);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf

namespace fmskf {

__global__ __launch_bounds__(kBlock) void k_fill64(uint64_t *p, uint64_t bits, uint64_t count) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < count) p[i] = bits;
}

int launch_fill64(void *p, uint64_t bits, uint64_t count, hipStream_t st) {
  if (count == 0) return 0;
  const dim3 g((unsigned)((count + kBlock - 1) / kBlock));
  k_fill64<<<g, kBlock, 0, st>>>((uint64_t *)p, bits, count);
  return (int)hipGetLastError();
}

// Readout in the units of VEHICLE_CTRL::get_vehicle_pos_m_latest (m, m, rad) and
// get_vehicle_vel_mmps_latest (body frame mm/s, mm/s, rad/s).  The KF6 / KF12D state
// carries world-frame velocity in m/s: rotate by -theta (libm sin/cos, readout only).
template <int MODEL>
__global__ __launch_bounds__(kBlock) void k_readout(const void *xv, uint64_t n, float *out) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  if constexpr (MODEL == 0) {  // RS: x = px, py, th, vx, vy, vth (already reference units)
    const float *x = (const float *)xv;
#pragma unroll
    for (int k = 0; k < 6; k++) out[k * n + i] = x[k * n + i];
  } else if constexpr (MODEL == 1 || MODEL == 3) {  // KF6 / KF12D base
    double px, py, th, vx, vy, w;
    if constexpr (MODEL == 1) {
      const float *x = (const float *)xv;
      px = x[i]; py = x[n + i]; th = x[2 * n + i]; vx = x[3 * n + i]; vy = x[4 * n + i]; w = x[5 * n + i];
    } else {
      const double *x = (const double *)xv;
      px = x[i]; py = x[n + i]; th = x[2 * n + i]; vx = x[3 * n + i]; vy = x[4 * n + i]; w = x[5 * n + i];
    }
    const double c = cos(th), s = sin(th);
    out[i] = (float)px;
    out[n + i] = (float)py;
    out[2 * n + i] = (float)th;
    out[3 * n + i] = (float)((vx * c + vy * s) * 1000.0);
    out[4 * n + i] = (float)((-vx * s + vy * c) * 1000.0);
    out[5 * n + i] = (float)w;
  } else {  // EKF9: body-frame velocity already
    const float *x = (const float *)xv;
    out[i] = x[i];
    out[n + i] = x[n + i];
    out[2 * n + i] = x[2 * n + i];
    out[3 * n + i] = x[3 * n + i] * 1000.0f;
    out[4 * n + i] = x[4 * n + i] * 1000.0f;
    out[5 * n + i] = x[5 * n + i];
  }
}

int launch_readout(const DevState &s, float *out, hipStream_t st) {
  const dim3 g((unsigned)((s.n + kBlock - 1) / kBlock));
  switch (s.model) {
    case 0: k_readout<0><<<g, kBlock, 0, st>>>(s.x, s.n, out); break;
    case 1: k_readout<1><<<g, kBlock, 0, st>>>(s.x, s.n, out); break;
    case 2: k_readout<2><<<g, kBlock, 0, st>>>(s.x, s.n, out); break;
    case 3: k_readout<3><<<g, kBlock, 0, st>>>(s.x, s.n, out); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf
