// kernels_misc.hip -- sin/cos policy evaluation and the ensemble statistics reduction.
//
// Ensemble: mean and covariance of the state x across all instances of a rank, in fp64.
// Each thread accumulates shifted moment sums of its grid-stride instances (no division in
// the streaming loop), each block reduces its lanes with cross-lane swaps and DPP
// (ens_device.hpp), and a fold of one block per record element sums the block records in a
// fixed order and converts them to the Chan/Golub/LeVeque record {count, mean[n],
// M2 packed[n(n+1)/2]} that ranks all-gather and combine in rank order.  No atomics:
// bitwise reproducible run to run.  (Round 1 measured single-launch "last block folds"
// variants slower: the agent-scope release fence each block needs writes back the XCD's
// whole L2.)
#include <type_traits>

#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"
#include "lane_rs.hpp"
#include "ens_device.hpp"

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
// ensemble (ens_device.hpp: record layout, lane accumulation, block reduction)
// ---------------------------------------------------------------------------
// robots per thread per pass (loads of all of them issued before any accumulation; at most 2
// for the fp64 12-state x) and the block cap: 2^20 KF6 robots -> 1024 blocks of 4 robots per
// lane, one pass
template <int NX>
constexpr int ens_r() { return NX >= 12 ? 2 : 8; }
constexpr int kEnsMaxBlocks = 2048;

// robots per lane of the stand-alone partial: sizes the partial's grid, hence the block-record
// count the fold reads: 8 while n <= 2^21 (a small grid: half the block records for the
// fold), else 4.  Measured (rocprof, one box): KF6 2^20 partial + fold 6.35 + 4.42 us with 4
// -> 5.86 + 2.77 with 8; EKF9 2^20 10.66 + 4.30 -> 9.71 + 4.47; at 2^22 8 is neutral (KF6
// 18.9 / 18.7) or slower (EKF9 27.6 -> 31.0)
static int ens_rpl(uint64_t n) { return n <= (2ull << 20) ? 8 : 4; }

int ensemble_nblocks(uint64_t n) {
  const uint64_t per = (uint64_t)kBlock * ens_rpl(n);
  uint64_t b = (n + per - 1) / per;
  if (b > (uint64_t)kEnsMaxBlocks) b = kEnsMaxBlocks;
  if (b < 1) b = 1;
  return (int)b;
}

// Partial: every block accumulates the shifted moment sums of its grid-stride robots and
// writes its block record.  TILED (the EKF9 / KF12D state layout) is a compile-time choice:
// st_at then divides by the constant tile width (shifts), not by a runtime value.
template <int NX, typename T, bool TILED, int R>
__global__ __launch_bounds__(kBlock) void k_ens_partial(const T *__restrict__ x, uint64_t n,
                                                        uint64_t pp, const double *__restrict__ shift,
                                                        double *blocks) {
  constexpr uint32_t tile = TILED ? tile_w<T>() : 0;
  constexpr int LEN4 = EnsRec<NX>::LEN4;
  double sh[NX], v[LEN4];
  ens_load_shift<NX>(shift, sh);
#pragma unroll
  for (int k = 0; k < LEN4; k++) v[k] = 0.0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += R * stride) {
    T xv[R][NX];
#pragma unroll
    for (int u = 0; u < R; u++) {
      const uint64_t i = i0 + u * stride, ic = i < n ? i : n - 1;
#pragma unroll
      for (int k = 0; k < NX; k++) xv[u][k] = x[st_at(tile, pp, NX, k, ic)];
    }
#pragma unroll
    for (int u = 0; u < R; u++)
      if (i0 + u * stride < n) ens_add<NX>(v, xv[u], sh);
  }
  ens_block_write<NX>(v, blocks, gridDim.x, blockIdx.x);
}

// Fold: one block per record element (ens_fold_block: kFoldLanes partial sums, so this kernel
// and the fold blocks a tick kernel carries agree bitwise), LEN blocks in parallel, each one
// load round trip per U passes.  Round 1's one-block fold was 4.2-10 us at 2^20; KF6 record
// at 2^20 (partial + fold back to back) 8.3-8.9 us with 256-1024 threads per block.
template <int NX, int U>
__global__ __launch_bounds__(kBlock) void k_ens_fold(const double *__restrict__ blocks, int nb,
                                                     const double *__restrict__ shift, double *out) {
  ens_fold_block<NX, U>(blocks, (uint32_t)nb, shift, out, blockIdx.x);
}

template <int NX>
static void fold_launch(const double *blocks, int nb, const double *shift, double *out, hipStream_t st) {
  const int per = (nb + (int)kFoldLanes - 1) / (int)kFoldLanes;  // passes of kFoldLanes records
  const dim3 g(EnsRec<NX>::LEN);
  if (per <= 1) k_ens_fold<NX, 1><<<g, kBlock, 0, st>>>(blocks, nb, shift, out);
  else if (per <= 2) k_ens_fold<NX, 2><<<g, kBlock, 0, st>>>(blocks, nb, shift, out);
  else k_ens_fold<NX, 4><<<g, kBlock, 0, st>>>(blocks, nb, shift, out);
}

// the shift vector: robot 0's state
template <int NX, typename T>
__global__ void k_ens_shift(const T *x, uint64_t pp, uint32_t tile, double *shift) {
  const int k = threadIdx.x;
  if (k < NX) shift[k] = (double)x[st_at(tile, pp, NX, k, 0)];
}

// the stand-alone partial (block records of x); then, with `out`, the fold
template <int NX, typename T>
static void ens_launch(const DevState &s, double *blocks, const double *shift, double *out,
                       hipStream_t st) {
  const int nb = ensemble_nblocks(s.n);
  const int r = ens_r<NX>() < ens_rpl(s.n) ? ens_r<NX>() : ens_rpl(s.n);
  auto go = [&](auto tiled, auto rr) {
    k_ens_partial<NX, T, decltype(tiled)::value, decltype(rr)::value>
        <<<nb, kBlock, 0, st>>>((const T *)s.x, s.n, s.pitch, shift, blocks);
  };
  using TT = std::true_type;
  using TF = std::false_type;
  using R2 = std::integral_constant<int, 2>;
  using R4 = std::integral_constant<int, 4>;
  using R8 = std::integral_constant<int, 8>;
  if (s.tile) {
    if (r == 2) go(TT{}, R2{});
    else if (r == 8) go(TT{}, R8{});
    else go(TT{}, R4{});
  } else {
    if (r == 2) go(TF{}, R2{});
    else if (r == 8) go(TF{}, R8{});
    else go(TF{}, R4{});
  }
  if (out) fold_launch<NX>(blocks, nb, shift, out, st);
}

int launch_ensemble(const DevState &s, int nx, bool f64, double *blocks, const double *shift,
                    double *out, hipStream_t st) {
  if (nx == 6 && !f64) ens_launch<6, float>(s, blocks, shift, out, st);
  else if (nx == 9 && !f64) ens_launch<9, float>(s, blocks, shift, out, st);
  else if (nx == 12 && f64) ens_launch<12, double>(s, blocks, shift, out, st);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

int launch_ens_partial(const DevState &s, int nx, bool f64, double *blocks, const double *shift,
                       hipStream_t st, int *nb) {
  *nb = ensemble_nblocks(s.n);
  return launch_ensemble(s, nx, f64, blocks, shift, nullptr, st);
}

int launch_ens_fold(int nx, const double *blocks, int nb, const double *shift, double *out,
                    hipStream_t st) {
  if (nx == 6) fold_launch<6>(blocks, nb, shift, out, st);
  else if (nx == 9) fold_launch<9>(blocks, nb, shift, out, st);
  else if (nx == 12) fold_launch<12>(blocks, nb, shift, out, st);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

int launch_ens_shift(const DevState &s, int nx, bool f64, double *shift, hipStream_t st) {
  if (nx == 6 && !f64) k_ens_shift<6, float><<<1, 64, 0, st>>>((const float *)s.x, s.pitch, s.tile, shift);
  else if (nx == 9 && !f64) k_ens_shift<9, float><<<1, 64, 0, st>>>((const float *)s.x, s.pitch, s.tile, shift);
  else if (nx == 12 && f64) k_ens_shift<12, double><<<1, 64, 0, st>>>((const double *)s.x, s.pitch, s.tile, shift);
  else return (int)hipErrorInvalidValue;
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
// grid-stride: the span can exceed 2^32 elements (KF6 P at 2^28 robots: 5.6e9), more work-items
// than one dispatch's 32-bit grid size holds
template <typename T>
__global__ __launch_bounds__(kBlock) void k_tiled_fill(T *p, uint32_t rows, uint64_t total, RowBits b) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t e = (uint64_t)blockIdx.x * kBlock + threadIdx.x; e < total; e += stride) {
    const uint32_t k = (uint32_t)((e / tile_w<T>()) % rows);
    p[e] = __builtin_bit_cast(T, (typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type)b.v[k]);
  }
}
template <typename T, bool TO_DENSE>
__global__ __launch_bounds__(kBlock) void k_retile(const T *src, T *dst, uint32_t rows, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;  // instance
  const uint32_t k = blockIdx.y;                                    // row
  if (i >= n) return;
  const uint64_t t = st_at(tile_w<T>(), 0, rows, k, i), d = (uint64_t)k * n + i;
  if (TO_DENSE) dst[d] = src[t];
  else dst[t] = src[d];
}

int launch_tiled_fill(void *base, uint32_t rows, uint64_t n, const uint64_t *bits, uint32_t elem,
                      hipStream_t st) {
  if (n == 0) return 0;
  if (rows > 90) return (int)hipErrorInvalidValue;
  RowBits b{};
  for (uint32_t k = 0; k < rows; k++) b.v[k] = bits[k];
  const uint64_t w = tile_w_elem(elem), total = (n + w - 1) / w * w * rows;
  const uint64_t blocks = (total + kBlock - 1) / kBlock;
  const dim3 g((unsigned)(blocks < (1u << 20) ? blocks : (1u << 20)));
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

// RS s64_rawAngleSumPrev in the tick's layout (64-robot tiles of 16-byte wheel pairs,
// lane_rs.hpp rs_prev_at) -> [4][pitch] int64 planes (the ABI's [4][N] readout).  Grid-stride.
__global__ __launch_bounds__(kBlock) void k_prev_out(const int64_t *src, int64_t *dst, uint64_t n, uint64_t pitch) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    const longlong2 a = reinterpret_cast<const longlong2 *>(src)[rs_prev_at(i, 0)];
    const longlong2 b = reinterpret_cast<const longlong2 *>(src)[rs_prev_at(i, 1)];
    dst[i] = a.x;
    dst[pitch + i] = a.y;
    dst[2 * pitch + i] = b.x;
    dst[3 * pitch + i] = b.y;
  }
}
// the motor state's split sums (fmskf_internal.hpp m_sum_lo / m_sum_hi) as whole int64 sums:
// TO_PREV into the RS previous-sum tiles, else into [4][pitch] planes (get_rawAngleSum readout)
template <bool TO_PREV>
__global__ __launch_bounds__(kBlock) void k_motor_sums(const uint32_t *lo, const int32_t *hi, int64_t *dst, uint64_t n,
                                                       uint64_t pitch) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
    int64_t s[4];
    motor_sum_load(lo, hi, i, s);
    if constexpr (TO_PREV) {
      rs_prev_store(dst, i, s);
    } else {
#pragma unroll
      for (int w = 0; w < 4; w++) dst[w * pitch + i] = s[w];
    }
  }
}

static inline dim3 grid_stride(uint64_t n) {
  const uint64_t b = (n + kBlock - 1) / kBlock;
  return dim3((unsigned)(b < (1u << 20) ? b : (1u << 20)));
}

int launch_prev_out(const int64_t *prev, int64_t *dst, uint64_t n, uint64_t pitch, hipStream_t st) {
  if (n == 0) return 0;
  k_prev_out<<<grid_stride(n), kBlock, 0, st>>>(prev, dst, n, pitch);
  return (int)hipGetLastError();
}

int launch_motor_sums(const uint32_t *lo, const int32_t *hi, int64_t *dst, uint64_t n, uint64_t pitch, bool to_prev,
                      hipStream_t st) {
  if (n == 0) return 0;
  if (to_prev) k_motor_sums<true><<<grid_stride(n), kBlock, 0, st>>>(lo, hi, dst, n, pitch);
  else k_motor_sums<false><<<grid_stride(n), kBlock, 0, st>>>(lo, hi, dst, n, pitch);
  return (int)hipGetLastError();
}

int launch_fill64(void *p, uint64_t bits, uint64_t count, hipStream_t st) {
  if (count == 0) return 0;
  const dim3 g((unsigned)((count + kBlock - 1) / kBlock));
  k_fill64<<<g, kBlock, 0, st>>>((uint64_t *)p, bits, count);
  return (int)hipGetLastError();
}

// Status::flt_dltOutAngle_rad of the last frame of every wheel (VD_motor_if_m2006.cpp:64), formed
// at readout from the last two raw angles: the CAN tick keeps the previous angle instead of the
// float, so its bytes stay the decoded ones.  [N][4] int16 in, [N][4] float out.
__global__ __launch_bounds__(kBlock) void k_motor_dlt(const int16_t *angle, const int16_t *prev, float *out,
                                                      uint64_t count) {
  for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < count; g += (uint64_t)gridDim.x * kBlock)
    out[g] = (float)((int32_t)angle[g] - (int32_t)prev[g]) * K::out_rad_per_raw * K::gear_ratio_inv;
}

// the two stamp / angle history slots of every wheel traded (DevState::m_par), one robot per lane
__global__ __launch_bounds__(kBlock) void k_motor_swap(uint2 *m0, uint2 *m1, uint2 *a0, uint2 *a1, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint2 x = m0[i], y = m1[i], p = a0[i], q = a1[i];
  m0[i] = y;
  m1[i] = x;
  a0[i] = q;
  a1[i] = p;
}

int launch_motor_swap(const DevState &s, hipStream_t st) {
  if (s.n == 0 || !s.m_micro) return 0;
  k_motor_swap<<<dim3((unsigned)((s.n + kBlock - 1) / kBlock)), kBlock, 0, st>>>(
      (uint2 *)s.m_micro, (uint2 *)s.m_prev_micro, (uint2 *)s.m_angle, (uint2 *)s.m_prev, s.n);
  return (int)hipGetLastError();
}

int launch_motor_dlt(const int16_t *angle, const int16_t *prev, float *out, uint64_t count, hipStream_t st) {
  if (count == 0) return 0;
  const uint64_t b = (count + kBlock - 1) / kBlock;
  k_motor_dlt<<<dim3((unsigned)(b < (1u << 22) ? b : (1u << 22))), kBlock, 0, st>>>(angle, prev, out, count);
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
  // row k of this instance at [k * pp + i] (planar: pp = pitch, i = i0; tiled: pp = the tile width)
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
