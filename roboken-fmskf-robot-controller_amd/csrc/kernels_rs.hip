// kernels_rs.hip -- reference-semantics tick (mode RS) for gfx950.
//
// One robot per lane.  correct = VD_task_main.cpp:368 (theta hard overwrite by the
// IMU yaw), predict = VEHICLE_CTRL::update's velocity + odometry part
// (VD_vehicle_controller.cpp:11-51) with its exact numerics: int64 encoder-sum
// differences scaled in double, narrowed to float, mecanum forward kinematics,
// rotation by the heading through the selected sin/cos policy, mm -> m.
// Built with FP contraction off: bit-identical to the oracle restatement.
//
// Algorithmic bytes per instance-tick: pos 12 B r+w, prev 32 B r+w,
// sums 32 B, yaw 4 B, rpm 8 B, vel 12 B w  -> 12*2 + 32*2 + 32 + 4 + 8 + 12 = 144 B.
#include <type_traits>

#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"
#include "kf_generic.hpp"
#include "lane_rs.hpp"

#pragma clang fp contract(off)

namespace fmskf {

struct RsArgs {
  uint64_t n;
  uint64_t pitch;    // plane pitch of x (elements)
  float *x;          // [6][pitch]: px, py, th, vx, vy, vth
  int64_t *prev;     // 64-robot tiles of 16-byte wheel pairs (lane_rs.hpp rs_prev_at)
  TickIn in;
};

template <bool LIBM, bool CORR, bool PRED>
__global__ __launch_bounds__(kBlock) void k_rs(RsArgs a) {
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  RsLane s;
  s.px = a.x[i];
  s.py = a.x[pp + i];
  s.th = CORR ? 0.f : a.x[2 * pp + i];  // correct overwrites theta before any use
  s.vx = s.vy = s.vth = 0.f;
  if (PRED) rs_prev_load(a.prev, i, s.prev);
  const uint64_t st = a.in.stride;
  for (uint32_t t = 0; t < a.in.n_ticks; t++) {
    const uint64_t j = (uint64_t)t * st + i;
    const float yaw = CORR ? tick_yaw(a.in.imu_words & 1u, reinterpret_cast<const uint32_t *>(a.in.yaw_deg)[j]) : 0.f;
    uint2 r = make_uint2(0u, 0u);
    int64_t sum[4] = {0, 0, 0, 0};
    if (PRED) {
      r = reinterpret_cast<const uint2 *>(a.in.rpm)[j];
      if (a.in.msum_lo) {  // the motor state's sums (single tick; wave-uniform)
        motor_sum_load(a.in.msum_lo, a.in.msum_hi, i, sum);
      } else {
        const int64_t *sp = a.in.angle_sum + (uint64_t)t * st * 4;
#pragma unroll
        for (int w = 0; w < 4; w++) sum[w] = sp[w * a.in.sum_pitch + i];
      }
    }
    rs_tick1<LIBM, CORR, PRED>(s, yaw, r, sum, a.in.sintab);
  }
  if (PRED) {
    a.x[i] = s.px;
    a.x[pp + i] = s.py;
    a.x[3 * pp + i] = s.vx;
    a.x[4 * pp + i] = s.vy;
    a.x[5 * pp + i] = s.vth;
    rs_prev_store(a.prev, i, s.prev);
  }
  if (CORR) a.x[2 * pp + i] = s.th;
}

// Fused correct + predict, one tick, two robots per lane (i and i + G): the tick inputs of
// both robots (yaw, rpm, the four encoder sums: 44 B, fresh every tick) are loaded first, so
// the second robot's arrive while the first one's state is read, stepped and written (the
// input-latency hiding of the KF6 k_kf6p, kernels_kf6.hip).  TABLE512: the sine table as a
// wave-private LDS copy, its loads issued first, as in the KF kernels (global gathers after
// the state arrives measured 26.8-27.7 against 26.5-27.3 us at 2^20).
// Every plane goes through a scalar buffer descriptor at its block chunk (ld_chunk /
// st_chunk, kf_generic.hpp) so the loads and stores carry a cache policy, as in the KF6 tick
// (kf6_lane.hpp): the tick inputs (read once) non-temporal, the state loaded with CP and
// stored with st_pol(CP) (`sc1` while it fits the Infinity Cache, non-temporal past it);
// plain global accesses measured 27.0-27.5 (2^20) and 417 us (2^24) against 26.7 and 398-404.
#ifndef FMSKF_IN_CPOL
#define FMSKF_IN_CPOL 2
#endif
// the cache policy of the motor state's sums in the MS form (-1: the state's, CP)
#ifndef FMSKF_MS_CPOL
#define FMSKF_MS_CPOL 2
#endif
// SO (round 4): one span descriptor per array and robot slot (rsrc_span) with the planes of
// x, prev and the encoder sums reached through soffset, instead of one clamped descriptor per
// plane (16 -> 5 per slot; the launcher checks the 4 GiB span).
// MS: the sums are the motor state's split words (a.in.msum_lo / msum_hi; a compile-time choice:
// a run-time branch between the two load forms slowed both, 25.4 -> 26.4 us on caller sums and
// 20.7 -> 23.5 on the motor state at 2^20)
template <bool LIBM, int CP = 0, bool SO = false, bool MS = false>
__global__ __launch_bounds__(kBlock) void k_rs2(RsArgs a) {
  extern __shared__ double occ_cap[];
  (void)occ_cap;
  constexpr bool WT = !LIBM;
  __shared__ float wtab[WT ? kBlock / 64 : 1][WT ? kWaveTab : 1];
  const uint64_t n = a.n, pp = a.pitch;
  const uint64_t G = (uint64_t)gridDim.x * kBlock;
  const uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  WaveTable<!WT> tv(a.in.sintab);
  const float *tab = WT ? wtab[threadIdx.x >> 6] : a.in.sintab;
  float yaw[2];
  // the yaw plane, or the IMU state's Yaw words (fmskf_device.hpp tick_yaw): one dword either way
  const bool yp = (a.in.imu_words & 1u) != 0;
  const uint32_t *ys = reinterpret_cast<const uint32_t *>(a.in.yaw_deg);
  uint2 rw[2];
  int64_t sum[2][4];
  uint64_t hb[2];
  uint32_t li[2];
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const uint64_t i = i0 + r * G < n ? i0 + r * G : n - 1;
    // the wave's first lane fixes its 256-robot chunk; clamped lanes (n - 1) stay inside it
    hb[r] = __builtin_amdgcn_readfirstlane((uint32_t)i) & ~(uint32_t)(kBlock - 1);
    li[r] = (uint32_t)(i - hb[r]);
    uint64_t rv;
    if constexpr (MS) {  // the motor state's sums: [N][4] low and high words
      yaw[r] = tick_yaw(yp, ld_span<uint32_t, FMSKF_IN_CPOL>(rsrc_span(ys + hb[r]), li[r], 0));
      rv = ld_span<uint64_t, FMSKF_IN_CPOL>(rsrc_span(a.in.rpm + hb[r] * 4), li[r], 0);
      constexpr int MP = FMSKF_MS_CPOL < 0 ? CP : FMSKF_MS_CPOL;
      const auto lw = __builtin_amdgcn_raw_buffer_load_b128(rsrc_span(a.in.msum_lo + hb[r] * 4), li[r] * 16u, 0, MP);
      const auto hw = __builtin_amdgcn_raw_buffer_load_b128(rsrc_span(a.in.msum_hi + hb[r] * 4), li[r] * 16u, 0, MP);
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const uint32_t l = lw[w], h = hw[w];  // element copies (see kf6_load_in)
        sum[r][w] = motor_sum_join((int32_t)h, l);
      }
    } else if constexpr (SO) {
      yaw[r] = tick_yaw(yp, ld_span<uint32_t, FMSKF_IN_CPOL>(rsrc_span(ys + hb[r]), li[r], 0));
      rv = ld_span<uint64_t, FMSKF_IN_CPOL>(rsrc_span(a.in.rpm + hb[r] * 4), li[r], 0);
      const auto rs = rsrc_span(a.in.angle_sum + hb[r]);
#pragma unroll
      for (int w = 0; w < 4; w++)
        sum[r][w] = ld_span<int64_t, FMSKF_IN_CPOL>(rs, li[r], w * (uint32_t)(a.in.sum_pitch * 8));
    } else {
      yaw[r] = tick_yaw(yp, ld_chunk<uint32_t, FMSKF_IN_CPOL>(ys, hb[r], n, li[r]));
      rv = ld_chunk<uint64_t, FMSKF_IN_CPOL>(reinterpret_cast<const uint64_t *>(a.in.rpm), hb[r], n, li[r]);
#pragma unroll
      for (int w = 0; w < 4; w++)
        sum[r][w] = ld_chunk<int64_t, FMSKF_IN_CPOL>(a.in.angle_sum + w * a.in.sum_pitch, hb[r], n, li[r]);
    }
    rw[r] = make_uint2((uint32_t)rv, (uint32_t)(rv >> 32));
  }
  tv.store(wtab[WT ? threadIdx.x >> 6 : 0]);
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const uint64_t i = i0 + r * G;
    if (i >= n) return;
    RsLane s;
    constexpr int SP = st_pol(CP);
    // prev: the chunk's four 64-robot tiles (lane_rs.hpp rs_prev_at), each half of a wave's
    // tile one 1 KiB run (round 6)
    const auto rx = rsrc_span(a.x + hb[r]), rp = rsrc_span(a.prev + hb[r] * 4);
    const uint32_t po = (li[r] & ~63u) * 32u + (li[r] & 63u) * 16u;
    const uint32_t px4 = (uint32_t)(pp * 4);
    if constexpr (SO) {
      s.px = ld_span<float, CP>(rx, li[r], 0);
      s.py = ld_span<float, CP>(rx, li[r], px4);
    } else {
      s.px = ld_chunk<float, CP>(a.x, hb[r], n, li[r]);
      s.py = ld_chunk<float, CP>(a.x + pp, hb[r], n, li[r]);
    }
#pragma unroll
    for (int h2 = 0; h2 < 2; h2++) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, po + 1024u * h2, 0, CP);
      const uint32_t w0 = v[0], w1 = v[1], w2 = v[2], w3 = v[3];  // element copies (see kf6_load_in)
      s.prev[2 * h2] = (int64_t)(((uint64_t)w1 << 32) | w0);
      s.prev[2 * h2 + 1] = (int64_t)(((uint64_t)w3 << 32) | w2);
    }
    s.th = 0.f;
    rs_tick1<LIBM, true, true>(s, yaw[r], rw[r], sum[r], tab);
    const float xs[6] = {s.px, s.py, s.th, s.vx, s.vy, s.vth};
    if constexpr (SO) {
#pragma unroll
      for (int k = 0; k < 6; k++) st_span<float, SP>(rx, li[r], k * px4, xs[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 6; k++) st_chunk<float, SP>(a.x + k * pp, hb[r], n, li[r], xs[k]);
    }
#pragma unroll
    for (int h2 = 0; h2 < 2; h2++) {
      v4u32_t w;
      w[0] = (uint32_t)s.prev[2 * h2];
      w[1] = (uint32_t)((uint64_t)s.prev[2 * h2] >> 32);
      w[2] = (uint32_t)s.prev[2 * h2 + 1];
      w[3] = (uint32_t)((uint64_t)s.prev[2 * h2 + 1] >> 32);
      __builtin_amdgcn_raw_buffer_store_b128(w, rp, po + 1024u * h2, 0, SP);
    }
  }
}

int launch_rs(const DevState &s, const TickIn &in, bool libm, bool correct, bool predict,
              hipStream_t st) {
  RsArgs a{s.n, s.pitch, (float *)s.x, s.prev_sum, in};
  const dim3 g((unsigned)((s.n + kBlock - 1) / kBlock));
  static const bool two = [] {  // A/B switch (FMSKF_RS_TWO=0: one robot per lane)
    const char *e = getenv("FMSKF_RS_TWO");
    return !e || atoi(e) != 0;
  }();
  if (two && correct && predict && in.n_ticks == 1) {
    const dim3 g2((unsigned)((s.n + 2 * kBlock - 1) / (2 * kBlock)));
    // past the Infinity Cache: 2 blocks per CU (64 KiB of dynamic LDS).  2^24, kbench, two
    // passes: 436.7-448.2 us uncapped, 429-430 at 48 KiB, 418.5-424.5 at 64 KiB
    const unsigned lds = FMSKF_LDS_CAP("FMSKF_RS_LDS", state_nt(s.n * 124), 64u * 1024u);
    // FMSKF_RS_VARIANT=0: one clamped descriptor per plane (A/B); the soffset form needs every
    // plane array within 4 GiB of its chunk base
    static const int var = [] {
      const char *e = getenv("FMSKF_RS_VARIANT");
      return e ? atoi(e) : 1;
    }();
    const bool so = var != 0 && 6 * s.pitch * 4 <= 0xFFFFFFFFull && 4 * in.sum_pitch * 8 <= 0xFFFFFFFFull;
    const bool ms = in.msum_lo != nullptr;
    auto go = [&](auto cp, auto so_, auto ms_) {
      constexpr int C = decltype(cp)::value;
      constexpr bool S = decltype(so_)::value, M = decltype(ms_)::value;
      if (libm) k_rs2<true, C, S, M><<<g2, kBlock, lds, st>>>(a);
      else k_rs2<false, C, S, M><<<g2, kBlock, lds, st>>>(a);
    };
    using T = std::true_type;
    using F = std::false_type;
    using NT = std::integral_constant<int, kStateNT>;
    using C0 = std::integral_constant<int, 0>;
    if (state_nt(s.n * 124)) {
      if (ms) go(NT{}, T{}, T{});
      else if (so) go(NT{}, T{}, F{});
      else go(NT{}, F{}, F{});
    } else {
      if (ms) go(C0{}, T{}, T{});
      else if (so) go(C0{}, T{}, F{});
      else go(C0{}, F{}, F{});
    }
    return (int)hipGetLastError();
  }
  if (libm) {
    if (correct && predict) k_rs<true, true, true><<<g, kBlock, 0, st>>>(a);
    else if (correct) k_rs<true, true, false><<<g, kBlock, 0, st>>>(a);
    else k_rs<true, false, true><<<g, kBlock, 0, st>>>(a);
  } else {
    if (correct && predict) k_rs<false, true, true><<<g, kBlock, 0, st>>>(a);
    else if (correct) k_rs<false, true, false><<<g, kBlock, 0, st>>>(a);
    else k_rs<false, false, true><<<g, kBlock, 0, st>>>(a);
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf
