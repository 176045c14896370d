// kernels_misc.hip -- sin/cos policy evaluation and the ensemble statistics reduction.
//
// Ensemble: mean and covariance of the state x across all instances of a rank, in fp64,
// as a Chan/Golub/LeVeque record {count, mean[n], M2 packed[n(n+1)/2]}.  Each thread
// folds its grid-stride instances with Welford updates, the 64 lanes of a wave fold by
// DPP-free shuffles (__shfl_down) in a fixed butterfly order, the 4 waves of a block
// fold through LDS, then one block folds the per-block records in block order.  No
// atomics anywhere: the result is bitwise reproducible run to run, and ranks combine
// their records in rank order after the RCCL all-gather.
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

// Chan et al. pairwise combination a <- a (+) b  (same formula as oracle orc_ens_combine)
template <int NX>
__device__ __forceinline__ void ens_combine(EnsRec<NX> &a, const EnsRec<NX> &b) {
  const double na = a.v[0], nb = b.v[0];
  if (nb == 0.0) return;
  if (na == 0.0) {
    a = b;
    return;
  }
  const double nn = na + nb;
  double d[NX];
#pragma unroll
  for (int k = 0; k < NX; k++) d[k] = b.v[1 + k] - a.v[1 + k];
  const double f = na * nb / nn;
#pragma unroll
  for (int k = 0; k < NX; k++) a.v[1 + k] = a.v[1 + k] + d[k] * (nb / nn);
#pragma unroll
  for (int p = 0; p < NX; p++)
#pragma unroll
    for (int q = 0; q <= p; q++) {
      const int k = p * (p + 1) / 2 + q;
      a.v[1 + NX + k] = a.v[1 + NX + k] + b.v[1 + NX + k] + d[p] * d[q] * f;
    }
  a.v[0] = nn;
}

template <int NX>
__device__ __forceinline__ void ens_block_reduce(EnsRec<NX> &r, double *lds) {
  constexpr int LEN = EnsRec<NX>::LEN;
  // wave: fixed butterfly-down order
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    EnsRec<NX> o;
#pragma unroll
    for (int k = 0; k < LEN; k++) o.v[k] = __shfl_down(r.v[k], off, 64);
    if ((threadIdx.x & 63) < off) ens_combine<NX>(r, o);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < LEN; k++) lds[wave * LEN + k] = r.v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int wv = 1; wv < kBlock / 64; wv++) {
      EnsRec<NX> o;
#pragma unroll
      for (int k = 0; k < LEN; k++) o.v[k] = lds[wv * LEN + k];
      ens_combine<NX>(r, o);
    }
  }
}

template <int NX, typename T>
__global__ __launch_bounds__(kBlock) void k_ens_partial(const T *x, uint64_t n, double *blocks) {
  constexpr int LEN = EnsRec<NX>::LEN;
  __shared__ double lds[(kBlock / 64) * LEN];
  EnsRec<NX> r;
#pragma unroll
  for (int k = 0; k < LEN; k++) r.v[k] = 0.0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    // Welford: count, mean, co-moment update
    double xv[NX], d[NX];
    const double cnt = r.v[0] + 1.0;
#pragma unroll
    for (int k = 0; k < NX; k++) {
      xv[k] = (double)x[k * n + i];
      d[k] = xv[k] - r.v[1 + k];
      r.v[1 + k] = r.v[1 + k] + d[k] / cnt;
    }
#pragma unroll
    for (int p = 0; p < NX; p++)
#pragma unroll
      for (int q = 0; q <= p; q++) {
        const int k = p * (p + 1) / 2 + q;
        r.v[1 + NX + k] = r.v[1 + NX + k] + d[p] * (xv[q] - r.v[1 + q]);
      }
    r.v[0] = cnt;
  }
  ens_block_reduce<NX>(r, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < LEN; k++) blocks[(uint64_t)blockIdx.x * LEN + k] = r.v[k];
  }
}

template <int NX>
__global__ __launch_bounds__(kBlock) void k_ens_fold(const double *blocks, int nblocks, double *out) {
  constexpr int LEN = EnsRec<NX>::LEN;
  __shared__ double lds[(kBlock / 64) * LEN];
  EnsRec<NX> r;
  // thread t folds blocks t, t + 256, ... sequentially (fixed order)
#pragma unroll
  for (int k = 0; k < LEN; k++) r.v[k] = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += kBlock) {
    EnsRec<NX> o;
#pragma unroll
    for (int k = 0; k < LEN; k++) o.v[k] = blocks[(uint64_t)b * LEN + k];
    ens_combine<NX>(r, o);
  }
  ens_block_reduce<NX>(r, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < LEN; k++) out[k] = r.v[k];
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
    k_ens_fold<6><<<1, kBlock, 0, st>>>(blocks, nb, out);
  } else if (nx == 9 && !f64) {
    k_ens_partial<9, float><<<nb, kBlock, 0, st>>>((const float *)s.x, s.n, blocks);
    k_ens_fold<9><<<1, kBlock, 0, st>>>(blocks, nb, out);
  } else if (nx == 12 && f64) {
    k_ens_partial<12, double><<<nb, kBlock, 0, st>>>((const double *)s.x, s.n, blocks);
    k_ens_fold<12><<<1, kBlock, 0, st>>>(blocks, nb, out);
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
