// kernels_misc.hip -- sin/cos policy evaluation and the ensemble statistics reduction.
//
// Ensemble: mean and covariance of the state x across all instances of a rank, in fp64.
// Each thread accumulates shifted moment sums of its grid-stride instances (no division in
// the streaming loop), each block sums its threads through an LDS transpose in a fixed
// order, and a one-block fold sums the per-block records in block order and converts them
// to the Chan/Golub/LeVeque record {count, mean[n], M2 packed[n(n+1)/2]} that ranks
// all-gather and combine in rank order.  No atomics: bitwise reproducible run to run.
// (Single-launch "last block folds" variants measured slower: with plain stores, the
// agent-scope release fence each block needs writes back the XCD's whole L2; with
// write-through (sc1) record stores and sc1 loads in the folding block, 26.4 us against
// 14.3 at 2^20: the one block's serialised record loads outlast the fold launch.)
#include <type_traits>

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
};

constexpr int kEnsPerThread = 8;  // instances per thread at full grid (n = 2^20: 512 blocks)
#ifndef FMSKF_ENS_CH
#define FMSKF_ENS_CH 32
#endif
constexpr int kEnsCh = FMSKF_ENS_CH;   // record elements reduced per LDS pass
constexpr int kEnsSeg = kBlock / kEnsCh;  // threads (column segments) per element
#ifndef FMSKF_ENS_PAD
#define FMSKF_ENS_PAD 8
#endif
// LDS transpose row pitch (doubles).  The segment reads red[e][j*kEnsSeg+seg] put 4 rows e in
// one 32-lane ds_read_b64 group; unpadded rows (2 KiB) land them on the same banks (4-way),
// 8 doubles of padding shift each row by 16 banks (conflict-free).  A/B at 2^20, record
// partial + fold: KF6 12.78 -> 12.58 us, EKF9 29.29 -> 29.18, KF12D 38.37 -> 38.04.
constexpr int kEnsRow = kBlock + FMSKF_ENS_PAD;

// Sum v[LEN] over the 256 threads of the block into tot[LEN] (LDS, visible to all threads
// after return).  Transpose through LDS in chunks of kEnsCh elements: thread t writes column
// t; then kEnsSeg threads per element sum kEnsCh columns each (column j*kEnsSeg+seg, j
// ascending), then one thread per element sums the kEnsSeg segment partials in order.
// Chunks of 32 (64 KiB of LDS) against 16: EKF9 record 35.8 -> 30.4 us at 2^20, KF12D
// 39.4 -> 38.5, KF6 13.9 -> 13.7 (fewer passes and barriers).  Fixed order -> deterministic;
// no cross-lane shuffles (the LDS bandwidth of a shuffle butterfly is ~6x this).
template <int LEN>
__device__ __forceinline__ void block_sum(const double (&v)[LEN], double (*red)[kEnsRow],
                                          double (*part)[kEnsSeg], double *tot) {
  const int t = threadIdx.x;
#pragma unroll
  for (int c = 0; c < LEN; c += kEnsCh) {
#pragma unroll
    for (int e = 0; e < kEnsCh; e++)
      if (c + e < LEN) red[e][t] = v[c + e];
    __syncthreads();
    {
      const int e = t / kEnsSeg, seg = t % kEnsSeg;
      if (c + e < LEN) {
        double s = red[e][seg];
#pragma unroll
        for (int j = 1; j < kEnsCh; j++) s = s + red[e][j * kEnsSeg + seg];
        part[e][seg] = s;
      }
    }
    __syncthreads();
    if (t < kEnsCh && c + t < LEN) {
      double s = part[t][0];
#pragma unroll
      for (int j = 1; j < kEnsSeg; j++) s = s + part[t][j];
      tot[c + t] = s;
    }
    __syncthreads();
  }
}

// Partial: every block accumulates shifted moment sums S1 = sum(x - x0),
// S2 = sum((x - x0)(x - x0)^T) (x0 = instance 0's state, fp64, no division in the streaming
// loop) of its grid-stride instances and writes its record.
// TILED (the EKF9 / KF12D state layout) is a compile-time choice: st_at then divides by the
// constant kTile (shifts), not by a runtime value (a 64-bit division per load)
template <int NX, typename T, bool TILED>
__global__ __launch_bounds__(kBlock) void k_ens_partial(const T *__restrict__ x, uint64_t n,
                                                        uint64_t pp, double *blocks) {
  constexpr uint32_t tile = TILED ? kTile : 0;
  constexpr int LEN = EnsRec<NX>::LEN;
  constexpr int U = 4;
  __shared__ double red[kEnsCh][kEnsRow];
  __shared__ double part[kEnsCh][kEnsSeg];
  __shared__ double tot[LEN];
  double sh[NX], v[LEN];
#pragma unroll
  for (int k = 0; k < NX; k++) sh[k] = (double)x[st_at(tile, pp, NX, k, 0)];
#pragma unroll
  for (int k = 0; k < LEN; k++) v[k] = 0.0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += U * stride) {
    T xv[U][NX];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t i = i0 + u * stride;
#pragma unroll
      for (int k = 0; k < NX; k++) xv[u][k] = i < n ? x[st_at(tile, pp, NX, k, i)] : (T)0;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (i0 + u * stride >= n) break;
      double d[NX];
#pragma unroll
      for (int k = 0; k < NX; k++) {
        d[k] = (double)xv[u][k] - sh[k];
        v[1 + k] = v[1 + k] + d[k];
      }
#pragma unroll
      for (int p = 0; p < NX; p++)
#pragma unroll
        for (int q = 0; q <= p; q++) v[1 + NX + p * (p + 1) / 2 + q] += d[p] * d[q];
      v[0] = v[0] + 1.0;
    }
  }
  block_sum<LEN>(v, red, part, tot);
  // element-major block records ([LEN][gridDim.x]): the fold's loads of one element across
  // consecutive blocks are then one coalesced access
  for (int k = threadIdx.x; k < LEN; k += kBlock) blocks[(uint64_t)k * gridDim.x + blockIdx.x] = tot[k];
}

// Fold (one block): sums the block records (stored element-major, [LEN][nblocks]) in a fixed
// order, then the conversion to {count, mean = x0 + S1/c, M2 = S2 - S1 S1^T / c}.
template <int NX, typename T>
__global__ __launch_bounds__(kBlock) void k_ens_fold(const T *__restrict__ x, uint64_t pp, uint32_t tile,
                                                     const double *__restrict__ blocks,
                                                     int nblocks, double *out) {
  constexpr int LEN = EnsRec<NX>::LEN;
  static_assert(LEN <= kBlock, "one record element per thread in the conversion");
  __shared__ double tot[LEN];
  const int t = threadIdx.x;
  // Records of up to 64 elements (KF6 28, EKF9 55): element-parallel, G threads per record
  // element; thread g of element e sums blocks g, g + G, ... (8 rotating accumulators,
  // combined in order), then the G partials of an element are summed in order: no LEN-wide
  // register record, one barrier.  A/B at 2^20 (partial + fold, 512 blocks): KF6 13.8 ->
  // 12.9 us, EKF9 30.5 -> 29.3.  KF12D's 91 elements would leave 2 threads per element
  // (256 serial loads each): 38.6 -> 40.6 us, so it keeps the register-record fold.
  if constexpr (LEN * 4 <= kBlock) {
    constexpr int G = LEN * 8 <= kBlock ? 8 : 4;
    constexpr int A = 8;
    __shared__ double part[LEN][G];
    {
      const int e = t / G, g = t % G;
      if (e < LEN) {
        const double *row = blocks + (uint64_t)e * nblocks;
        double a[A];
#pragma unroll
        for (int j = 0; j < A; j++) a[j] = 0.0;
        int b = g;
        for (; b + (4 * A - 1) * G < nblocks; b += 4 * A * G) {
          double l[4 * A];
#pragma unroll
          for (int j = 0; j < 4 * A; j++) l[j] = row[b + j * G];
#pragma unroll
          for (int j = 0; j < 4 * A; j++) a[j % A] = a[j % A] + l[j];
        }
        for (int j = 0; b < nblocks; b += G, j++) a[j % A] = a[j % A] + row[b];
        double s = a[0];
#pragma unroll
        for (int j = 1; j < A; j++) s = s + a[j];
        part[e][g] = s;
      }
    }
    __syncthreads();
    if (t < LEN) {
      double s = part[t][0];
#pragma unroll
      for (int j = 1; j < G; j++) s = s + part[t][j];
      tot[t] = s;
    }
    __syncthreads();
  } else {
    __shared__ double red[kEnsCh][kEnsRow];
    __shared__ double part[kEnsCh][kEnsSeg];
    double v[LEN];
#pragma unroll
    for (int k = 0; k < LEN; k++) v[k] = 0.0;
    for (int b = threadIdx.x; b < nblocks; b += kBlock) {
#pragma unroll
      for (int k = 0; k < LEN; k++) v[k] = v[k] + blocks[(uint64_t)k * nblocks + b];
    }
    block_sum<LEN>(v, red, part, tot);
  }
  const double c = tot[0];
  if (t < LEN) {
    const int k = t;
    double r;
    if (k == 0) {
      r = c;
    } else if (k <= NX) {
      r = (double)x[st_at(tile, pp, NX, k - 1, 0)] + (c > 0.0 ? tot[k] / c : 0.0);
    } else {
      int p = 0, q = k - 1 - NX;
      while (q > p) q -= ++p;
      r = c > 0.0 ? tot[k] - tot[1 + p] * tot[1 + q] / c : 0.0;
    }
    out[k] = r;
  }
}

int ensemble_nblocks(uint64_t n) {
  uint64_t b = (n + (uint64_t)kBlock * kEnsPerThread - 1) / ((uint64_t)kBlock * kEnsPerThread);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

template <int NX, typename T>
static void ens_launch(const DevState &s, double *blocks, double *out, hipStream_t st) {
  const int nb = ensemble_nblocks(s.n);
  if (s.tile) k_ens_partial<NX, T, true><<<nb, kBlock, 0, st>>>((const T *)s.x, s.n, s.pitch, blocks);
  else k_ens_partial<NX, T, false><<<nb, kBlock, 0, st>>>((const T *)s.x, s.n, s.pitch, blocks);
  k_ens_fold<NX, T><<<1, kBlock, 0, st>>>((const T *)s.x, s.pitch, s.tile, blocks, nb, out);
}

int launch_ensemble(const DevState &s, int nx, bool f64, double *blocks, double *out,
                    hipStream_t st) {
  if (nx == 6 && !f64) {
    ens_launch<6, float>(s, blocks, out, st);
  } else if (nx == 9 && !f64) {
    ens_launch<9, float>(s, blocks, out, st);
  } else if (nx == 12 && f64) {
    ens_launch<12, double>(s, blocks, out, st);
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

// tiled rows x N arrays (fmskf_internal.hpp st_at): one thread per element of the tiled span
struct RowBits {
  uint64_t v[90];
};
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tiled_fill(T *p, uint32_t rows, uint64_t total, RowBits b) {
  const uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (e >= total) return;
  const uint32_t k = (uint32_t)((e / kTile) % rows);
  p[e] = __builtin_bit_cast(T, (typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type)b.v[k]);
}
template <typename T, bool TO_DENSE>
__global__ __launch_bounds__(kBlock) void k_retile(const T *src, T *dst, uint32_t rows, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;  // instance
  const uint32_t k = blockIdx.y;                                    // row
  if (i >= n) return;
  const uint64_t t = st_at(kTile, 0, rows, k, i), d = (uint64_t)k * n + i;
  if (TO_DENSE) dst[d] = src[t];
  else dst[t] = src[d];
}

int launch_tiled_fill(void *base, uint32_t rows, uint64_t n, const uint64_t *bits, uint32_t elem,
                      hipStream_t st) {
  if (n == 0) return 0;
  if (rows > 90) return (int)hipErrorInvalidValue;
  RowBits b{};
  for (uint32_t k = 0; k < rows; k++) b.v[k] = bits[k];
  const uint64_t total = (n + kTile - 1) / kTile * kTile * rows;
  const dim3 g((unsigned)((total + kBlock - 1) / kBlock));
  if (elem == 8) k_tiled_fill<double><<<g, kBlock, 0, st>>>((double *)base, rows, total, b);
  else k_tiled_fill<float><<<g, kBlock, 0, st>>>((float *)base, rows, total, b);
  return (int)hipGetLastError();
}

int launch_untile(const void *tiled, void *dense, uint32_t rows, uint64_t n, uint32_t elem,
                  hipStream_t st) {
  if (n == 0 || rows == 0) return 0;
  const dim3 g((unsigned)((n + kBlock - 1) / kBlock), rows);
  if (elem == 8) k_retile<double, true><<<g, kBlock, 0, st>>>((const double *)tiled, (double *)dense, rows, n);
  else k_retile<float, true><<<g, kBlock, 0, st>>>((const float *)tiled, (float *)dense, rows, n);
  return (int)hipGetLastError();
}

int launch_tile(const void *dense, void *tiled, uint32_t rows, uint64_t n, uint32_t elem,
                hipStream_t st) {
  if (n == 0 || rows == 0) return 0;
  const dim3 g((unsigned)((n + kBlock - 1) / kBlock), rows);
  if (elem == 8) k_retile<double, false><<<g, kBlock, 0, st>>>((const double *)dense, (double *)tiled, rows, n);
  else k_retile<float, false><<<g, kBlock, 0, st>>>((const float *)dense, (float *)tiled, rows, n);
  return (int)hipGetLastError();
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
__global__ __launch_bounds__(kBlock) void k_readout(const void *xv, uint64_t n, uint64_t pitch, uint32_t tile,
                                                    float *out) {
  const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i0 >= n) return;
  // row k of this instance at [k * pp + i] (planar: pp = pitch, i = i0; tiled: pp = kTile)
  constexpr uint32_t rows = MODEL == 2 ? 9 : MODEL == 3 ? 12 : 6;
  const uint64_t i = tile ? st_at(tile, 0, rows, 0, i0) : i0;
  const uint64_t pp = tile ? tile : pitch;
  if constexpr (MODEL == 0) {  // RS: x = px, py, th, vx, vy, vth (already reference units)
    const float *x = (const float *)xv;
#pragma unroll
    for (int k = 0; k < 6; k++) out[k * n + i0] = x[k * pp + i];
  } else if constexpr (MODEL == 1 || MODEL == 3) {  // KF6 / KF12D base
    double px, py, th, vx, vy, w;
    if constexpr (MODEL == 1) {
      const float *x = (const float *)xv;
      px = x[i]; py = x[pp + i]; th = x[2 * pp + i]; vx = x[3 * pp + i]; vy = x[4 * pp + i]; w = x[5 * pp + i];
    } else {
      const double *x = (const double *)xv;
      px = x[i]; py = x[pp + i]; th = x[2 * pp + i]; vx = x[3 * pp + i]; vy = x[4 * pp + i]; w = x[5 * pp + i];
    }
    const double c = cos(th), s = sin(th);
    out[i0] = (float)px;
    out[n + i0] = (float)py;
    out[2 * n + i0] = (float)th;
    out[3 * n + i0] = (float)((vx * c + vy * s) * 1000.0);
    out[4 * n + i0] = (float)((-vx * s + vy * c) * 1000.0);
    out[5 * n + i0] = (float)w;
  } else {  // EKF9: body-frame velocity already
    const float *x = (const float *)xv;
    out[i0] = x[i];
    out[n + i0] = x[pp + i];
    out[2 * n + i0] = x[2 * pp + i];
    out[3 * n + i0] = x[3 * pp + i] * 1000.0f;
    out[4 * n + i0] = x[4 * pp + i] * 1000.0f;
    out[5 * n + i0] = x[5 * pp + i];
  }
}

int launch_readout(const DevState &s, float *out, hipStream_t st) {
  const dim3 g((unsigned)((s.n + kBlock - 1) / kBlock));
  switch (s.model) {
    case 0: k_readout<0><<<g, kBlock, 0, st>>>(s.x, s.n, s.pitch, s.tile, out); break;
    case 1: k_readout<1><<<g, kBlock, 0, st>>>(s.x, s.n, s.pitch, s.tile, out); break;
    case 2: k_readout<2><<<g, kBlock, 0, st>>>(s.x, s.n, s.pitch, s.tile, out); break;
    case 3: k_readout<3><<<g, kBlock, 0, st>>>(s.x, s.n, s.pitch, s.tile, out); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf
