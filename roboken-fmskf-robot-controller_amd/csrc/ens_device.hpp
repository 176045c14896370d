// ens_device.hpp -- device side of the ensemble statistics record: per-lane
// shifted moment sums and their fixed-order block reduction, shared by the stand-alone
// partial kernel (kernels_misc.hip) and the tick kernels that emit the record of the state
// they just wrote (kernels_kf6.hip, fmskf_tick_ensemble).
//
// Record of a set of robots (fp64): {count, S1[n] = sum(x - s), S2 packed = sum((x-s)(x-s)^T)}
// with s the handle's shift vector (robot 0's state when the handle's first record was asked
// for, refreshed by reset / set_state / load_state).  No division in the streaming part.
//
// Block reduction without an LDS transpose (the round-1 design pushed every lane's 28-91
// doubles through LDS: 57 KB per KF6 block).  A wave of 64 lanes reduces its LEN4 = 4Q values
// by recursive halving: v_permlane32_swap pairs value j with value j + 2Q so the lower half
// of the wave sums one and the upper half the other (one swap per dword, no selects), then
// v_permlane16_swap does the same across 16-lane rows, leaving Q values per row; four DPP
// butterfly steps reduce each row.  Row r's lanes then hold elements [rQ, rQ + Q).  LDS holds
// only 4 waves x LEN4 doubles.  Every element goes through the same addition tree (fp add is
// commutative, the pairings are lane-position based), so a value reduced at any position of
// the record gets bitwise the same sum: the parallel fold relies on that.
#pragma once
#include "fmskf_internal.hpp"

namespace fmskf {

template <int NX>
struct EnsRec {
  static constexpr int NP = NX * (NX + 1) / 2;
  static constexpr int LEN = 1 + NX + NP;
  static constexpr int LEN4 = (LEN + 3) & ~3;
  static constexpr int Q = LEN4 / 4;
};

__device__ __forceinline__ uint2 dsplit(double v) { return __builtin_bit_cast(uint2, v); }
__device__ __forceinline__ double djoin(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(double, make_uint2(lo, hi));
}

// lanes 0-31: a(lane) + a(lane + 32); lanes 32-63: b(lane - 32) + b(lane)
__device__ __forceinline__ double halve32(double a, double b) {
  const uint2 ua = dsplit(a), ub = dsplit(b);
  const auto lo = __builtin_amdgcn_permlane32_swap(ua.x, ub.x, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(ua.y, ub.y, false, false);
  return djoin(lo[0], hi[0]) + djoin(lo[1], hi[1]);
}
// within each 32-lane half: rows 0 / 2 sum a over rows (0,1) / (2,3), rows 1 / 3 sum b
__device__ __forceinline__ double halve16(double a, double b) {
  const uint2 ua = dsplit(a), ub = dsplit(b);
  const auto lo = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
  return djoin(lo[0], hi[0]) + djoin(lo[1], hi[1]);
}
template <int CTRL>
__device__ __forceinline__ double dpp_sum(double v) {
  const uint2 u = dsplit(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)u.x, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)u.y, CTRL, 0xF, 0xF, true);
  return v + djoin(lo, hi);
}
// 16-lane row sum, every lane of the row ends with it: xor 1, xor 2 (quad_perm), then
// lane i with 7 - i (row_half_mirror) and with 15 - i (row_mirror)
__device__ __forceinline__ double row_sum(double v) {
  v = dpp_sum<0xB1>(v);   // quad_perm [1,0,3,2]
  v = dpp_sum<0x4E>(v);   // quad_perm [2,3,0,1]
  v = dpp_sum<0x141>(v);  // row_half_mirror
  v = dpp_sum<0x140>(v);  // row_mirror
  return v;
}

// Block barrier ordering LDS only: __syncthreads() is also a workgroup fence for global
// memory, i.e. an s_waitcnt vmcnt(0) that would hold a tick kernel's record epilogue until
// every state store the block issued has drained.  This waits on lgkmcnt only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Sum v[LEN4] over the block's NT lanes; thread t < LEN4 gets element t (returned), the
// other threads get 0.  `red` is LDS of NT / 64 * LEN4 doubles.  Ends with the block's
// threads synchronised on LDS (the caller may reuse nothing of `red` without another barrier).
template <int LEN4, int NT = kBlock>
__device__ __forceinline__ double block_reduce(double (&v)[LEN4], double *red) {
  constexpr int Q = LEN4 / 4;
  double w[2 * Q];
#pragma unroll
  for (int j = 0; j < 2 * Q; j++) w[j] = halve32(v[j], v[j + 2 * Q]);
  double u[Q];
#pragma unroll
  for (int j = 0; j < Q; j++) u[j] = row_sum(halve16(w[j], w[j + Q]));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if ((lane & 15) == 0) {
    const int r = lane >> 4;
#pragma unroll
    for (int j = 0; j < Q; j++) red[wave * LEN4 + r * Q + j] = u[j];
  }
  lds_barrier();
  const int t = threadIdx.x;
  double s = 0.0;
  if (t < LEN4) {
    s = red[t];
#pragma unroll
    for (int wv = 1; wv < NT / 64; wv++) s = s + red[wv * LEN4 + t];
  }
  return s;
}

// Accumulate one robot's shifted moments into v (v[0] count, v[1..NX] S1, then S2 packed).
template <int NX, typename T, int LEN4>
__device__ __forceinline__ void ens_add(double (&v)[LEN4], const T (&x)[NX], const double (&sh)[NX]) {
  double d[NX];
#pragma unroll
  for (int k = 0; k < NX; k++) {
    d[k] = (double)x[k] - sh[k];
    v[1 + k] = v[1 + k] + d[k];
  }
#pragma unroll
  for (int p = 0; p < NX; p++)
#pragma unroll
    for (int q = 0; q <= p; q++) {
      double &a = v[1 + NX + p * (p + 1) / 2 + q];
      a = __builtin_fma(d[p], d[q], a);
    }
  v[0] = v[0] + 1.0;
}

template <int NX>
__device__ __forceinline__ void ens_load_shift(const double *shift, double (&sh)[NX]) {
#pragma unroll
  for (int k = 0; k < NX; k++) sh[k] = shift[k];
}

// Block record (element-major [LEN][nblocks], so the fold reads one element coalesced)
template <int NX>
__device__ __forceinline__ void ens_block_write(double (&v)[EnsRec<NX>::LEN4], double *blocks, uint32_t nblocks,
                                                uint32_t bid) {
  __shared__ double red[4 * EnsRec<NX>::LEN4];
  const double s = block_reduce<EnsRec<NX>::LEN4>(v, red);
  if (threadIdx.x < EnsRec<NX>::LEN)
    blocks[(uint64_t)threadIdx.x * nblocks + bid] = s;
}

// The tick kernels' record epilogue (fmskf_tick_ensemble): the R robots this lane ticked
// (live ones only), reduced over the block into its record of the post-tick state; bid: the
// block's tick block index (its record's column).  Measured and not kept (kbench ens_async, two
// alternating passes, one box): a record per wave (the lane-level tree only, no LDS and no block
// barrier; four times the records for the fold), KF6 2^20 async 39.5-40.1 us per tick against
// 39.0-39.3, EKF9 2^22 323-325 against 305, KF6 2^24 675-676 against 617.
template <int NX, int R, typename T>
__device__ __forceinline__ void ens_epilogue(const TickIn &in, const T (&xs)[R][NX], const bool (&live)[R],
                                             uint32_t bid) {
  double sh[NX], v[EnsRec<NX>::LEN4];
  ens_load_shift<NX>(in.ens_shift, sh);
#pragma unroll
  for (int k = 0; k < EnsRec<NX>::LEN4; k++) v[k] = 0.0;
#pragma unroll
  for (int r = 0; r < R; r++)
    if (live[r]) ens_add<NX>(v, xs[r], sh);
  ens_block_write<NX>(v, in.ens_blocks, in.ens_grid, bid);
}

// Fold of record element k: sum, over the nb block records, the count row, the two S1 rows
// the element needs and its own row, then convert: count; mean = s + S1 / c; M2 = S2 - S1 S1^T
// / c.  The summation order is fixed at kFoldLanes partial sums (lane L adds blocks L,
// L + kFoldLanes, ... ascending, then the block_reduce tree over kFoldLanes / 64 waves), and a
// 256-thread block plays kFoldLanes / 256 lanes per thread, so the stand-alone fold kernel and
// the fold blocks a tick kernel carries (ens_fold_front) give bitwise the same record.  A row
// summed by several elements gets bitwise the same total in each, so the record is
// consistent.  U: passes of kFoldLanes blocks whose loads are in flight together.
constexpr uint32_t kFoldLanes = 1024;
template <int NX, int U>
__device__ __forceinline__ void ens_fold_block(const double *__restrict__ blocks, uint32_t nb,
                                               const double *__restrict__ shift, double *out, uint32_t k) {
  constexpr int J = kFoldLanes / kBlock;
  uint32_t ra = k, rb = k;
  if (k > (uint32_t)NX) {
    uint32_t p = 0, q = k - 1 - NX;
    while (q > p) q -= ++p;
    ra = 1 + p;
    rb = 1 + q;
  }
  const double *rows[4] = {blocks, blocks + (uint64_t)ra * nb, blocks + (uint64_t)rb * nb,
                           blocks + (uint64_t)k * nb};
  double v[J][4];
#pragma unroll
  for (int j = 0; j < J; j++)
#pragma unroll
    for (int c = 0; c < 4; c++) v[j][c] = 0.0;
  for (uint32_t b = threadIdx.x; b < nb; b += U * kFoldLanes) {
    double l[U][J][4];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < J; j++) {
        const uint32_t bi = b + u * kFoldLanes + j * kBlock;
        const uint32_t bc = bi < nb ? bi : b;
#pragma unroll
        for (int c = 0; c < 4; c++) l[u][j][c] = rows[c][bc];
      }
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int j = 0; j < J; j++)
        if (b + u * kFoldLanes + j * kBlock < nb) {
#pragma unroll
          for (int c = 0; c < 4; c++) v[j][c] = v[j][c] + l[u][j][c];
        }
  }
  // block_reduce<4, kFoldLanes>'s tree: lane-level part per played wave, then the waves in order
  __shared__ double red[kFoldLanes / 64 * 4];
  __shared__ double tot[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < J; j++) {
    const double w0 = halve32(v[j][0], v[j][2]), w1 = halve32(v[j][1], v[j][3]);
    const double s = row_sum(halve16(w0, w1));
    if ((lane & 15) == 0) red[(j * (kBlock / 64) + wave) * 4 + (lane >> 4)] = s;
  }
  lds_barrier();
  const int t = threadIdx.x;
  if (t < 4) {
    double s = red[t];
#pragma unroll
    for (int wv = 1; wv < (int)(kFoldLanes / 64); wv++) s = s + red[wv * 4 + t];
    tot[t] = s;
  }
  lds_barrier();
  if (t == 0) {
    const double c = tot[0];
    double r;
    if (k == 0) r = c;
    else if (k <= (uint32_t)NX) r = shift[k - 1] + (c > 0.0 ? tot[3] / c : 0.0);
    else r = c > 0.0 ? tot[3] - tot[1] * tot[2] / c : 0.0;
    // a system-scope store (written through the caches): `out` may be a pinned host slot the
    // host reads behind an event without the system-scope release (api_ctx.hpp kSyncEvent)
    __hip_atomic_store(out + k, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The fold blocks a fused tick kernel carries (fmskf_tick_ensemble_begin): blocks 0 .. LEN - 1
// of its grid fold the PREVIOUS event's block records (complete: that event's kernel ran
// earlier on the stream) into in.fold_out, in the shadow of this tick's blocks instead of a
// launch of their own.  They come FIRST in the grid: dispatched first, their load round trips
// overlap the tick blocks' instead of extending the grid's tail (a fold block makes one pass
// per 1024 records: 64 at 2^24 KF6 robots).  bid: this block's tick block index.
template <int NX>
__device__ __forceinline__ bool ens_fold_front(const TickIn &in, uint32_t &bid) {
  constexpr uint32_t L = EnsRec<NX>::LEN;
  bid = blockIdx.x;
  if (!in.fold_blocks) return false;
  if (blockIdx.x < L) {
    ens_fold_block<NX, 1>(in.fold_blocks, in.fold_nb, in.ens_shift, in.fold_out, blockIdx.x);
    return true;
  }
  bid = blockIdx.x - L;
  return false;
}

}  // namespace fmskf
