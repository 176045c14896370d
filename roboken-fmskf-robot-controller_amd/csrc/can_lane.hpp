// can_lane.hpp -- MOTOR_IF_M2006::rx_callback (VD_motor_if_m2006.cpp:32-72) as lane functions,
// shared by the CAN RX kernels (kernels_ingest.hip k_can4 / k_can) and the fused firmware tick
// (kernels_ctrl.hip k_isr_kf6 with CAN: the tick's four frames per robot, then the ISR, in one
// kernel).  Cortex-M7 integer semantics: wrapping MUL, SDIV x/0 = 0.
#pragma once
#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"
#include "kf_generic.hpp"
#include "lane_rs.hpp"

#pragma clang fp contract(off)

namespace fmskf {

struct CanArgs {
  uint64_t n;
  const uint8_t *frames;
  const int16_t *stamps;
  const uint8_t *present;
  int8_t dir[4];
  // the newest frame's stamps and angles, and the ones before (DevState::m_par, motor_slots): a
  // frame's stamp and angle go over the older slot (prev_micro / prev), the host flips the order
  int16_t *micro, *angle, *rpm, *curr;
  int16_t *prev;  // [N][4] the angle before this frame (Status::flt_dltOutAngle_rad at readout)
  int16_t *prev_micro;  // [N][4] the stamp before this frame (the IIR1's previous sample, speed_x)
  uint32_t *sum_lo;  // [N][4] s64_rawAngleSum, low 32 bits (fmskf_internal.hpp m_sum_lo)
  int32_t *sum_hi;   // [N][4] high 32 bits (written only when a frame's delta carries)
  float *iir_y;  // [N][4] UTIL::IIR1 output state, also Status::flt_SpeedRadPS
  bool nt;       // host side: the fused kernels' choice of a non-temporal motor state (can_nt)
};
inline bool can_nt_flag(const CanArgs &a) { return a.nt; }

__device__ __forceinline__ int16_t s16_of(uint32_t h, uint32_t l) { return (int16_t)((h << 8) | l); }
__device__ __forceinline__ int32_t mul_wrap(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a * (uint32_t)b);
}
// Cortex-M7 SDIV: x/0 = 0 (CCR.DIV_0_TRP = 0 at reset), INT_MIN/-1 = INT_MIN
// Branch-free: the two special cases divide by 1 and select, so the wave runs one division
// instead of two exec-masked regions per wheel
__device__ __forceinline__ int32_t sdiv_arm(int32_t a, int32_t b) {
  const bool ovf = a == INT32_MIN && b == -1;
  const int32_t q = a / (b == 0 || ovf ? 1 : b);
  return b == 0 ? 0 : q;
}

// one wheel's rx_callback on its 8-byte frame and microsecond stamp (VD_motor_if_m2006.cpp:
// 32-72): the decoded fields, the IIR1 speed state and the wrapped angle step the int64 sum
// takes (:66-69; the caller adds it to the split sum, sum_add).  The Status ring's head
// (:33-34, 71) is not kept: both readers, get_status_latest and get_status_estimate
// (VD_motor_if_m2006.hpp:44-47, .cpp:11-24), read only the newest entry, which is what the
// engine stores, so the head selects nothing that can be observed (round 4: 232 -> 224 B)
struct CanWheel {
  int16_t angle, rpm, curr;
  float iir_y;
  int32_t d;  // s64_rawAngleSum += d (|d| <= 4096)
};
// s64_rawAngleSum += d on the split halves (fmskf_internal.hpp m_sum_lo: sum = hi * 2^32 + the
// low word read as int32): the low word wraps, the carry (-1, 0, +1) goes to the high word.  A
// signed low word carries only where the sum crosses an odd multiple of 2^31, so a wheel that
// turns back and forth around its start (sum near 0) never does; an unsigned one carried at every
// crossing of 0 and measured 8% slower at 2^22 robots on random frames
__device__ __forceinline__ uint32_t sum_add(uint32_t lo, int32_t d, int32_t &carry) {
  const int64_t t = (int64_t)(int32_t)lo + d;
  const int32_t nl = (int32_t)(uint32_t)t;
  carry = (int32_t)((t - nl) >> 32);
  return (uint32_t)nl;
}

// the speed sample rx_callback feeds the IIR1 (VD_motor_if_m2006.cpp:49-63): the wrapped angle
// step over the wrapped microsecond step, with the M7's wrapping MUL and SDIV x/0 = 0
__device__ __forceinline__ float speed_x(int16_t new_angle, int16_t old_angle, int16_t micro, int16_t old_micro) {
  int32_t raw_ang_dlt = new_angle - old_angle;
  int32_t usec_dlt = micro - old_micro;
  if (raw_ang_dlt > (K::raw_per_rot / 2)) raw_ang_dlt = raw_ang_dlt - K::raw_per_rot;
  else if (raw_ang_dlt < -(K::raw_per_rot / 2)) raw_ang_dlt = raw_ang_dlt + K::raw_per_rot;
  if (usec_dlt > 0x7FFF) usec_dlt = usec_dlt - 0x7FFF;
  else if (usec_dlt < -0x7FFF) usec_dlt = usec_dlt + 0x7FFF;
  const int32_t num = mul_wrap(mul_wrap(raw_ang_dlt, 2), 3141593);
  return (float)sdiv_arm(num, usec_dlt) / (float)K::raw_per_rot;
}
// IIR1's state x (prev_X_, util_iir.hpp:39-45) is not stored (round 5): it is the previous
// frame's speed sample, a pure function of that frame's angle / stamp and the ones before it
// (prev_angle / prev_micro, which the engine keeps for Status::flt_dltOutAngle_rad and here), so
// it is formed again from them: 4 B read + 2 B written per wheel instead of a float read and
// written (224 -> 216 B per robot).  All zero after reset gives x = 0 (SDIV 0/0 = 0), the
// zero-initialised filter's prev_X_.
__device__ __forceinline__ CanWheel can_wheel(uint32_t fx, uint32_t fy, int16_t micro, int dir,
                                              int16_t old_micro, int16_t old_angle, int16_t prev_micro,
                                              int16_t prev_angle, float py) {
  const uint32_t b0 = fx & 0xFF, b1 = (fx >> 8) & 0xFF, b2 = (fx >> 16) & 0xFF, b3 = fx >> 24;
  const uint32_t b4 = fy & 0xFF, b5 = (fy >> 8) & 0xFF;
  CanWheel o;
  const int16_t new_angle =
      dir == 1 ? s16_of(b0, b1) : (int16_t)(K::raw_per_rot - s16_of(b0, b1));
  o.angle = new_angle;
  o.rpm = (int16_t)(s16_of(b2, b3) * dir);
  o.curr = (int16_t)(s16_of(b4, b5) * dir);
  const float x = speed_x(new_angle, old_angle, micro, old_micro);
  const float pxv = speed_x(old_angle, prev_angle, old_micro, prev_micro);
  o.iir_y = 0.8f * py + 0.1f * x + 0.1f * pxv;  // UTIL::IIR1::update, util_iir.hpp:39-45
  // Status::flt_dltOutAngle_rad (VD_motor_if_m2006.cpp:64) is formed at readout from this angle and
  // the previous one, which the caller stores (k_motor_dlt)
  int16_t d = (int16_t)(new_angle - old_angle);
  d = (d > 4096) ? (int16_t)(d - 8192) : ((d < -4096) ? (int16_t)(d + 8192) : d);
  o.d = d;
  return o;
}

// One robot per lane, every wheel present: the robot's 32 frame bytes, its four stamps and its
// [N][4] int16 / float / uint32 state in single 8- and 16-byte accesses, every access through a
// scalar descriptor at the block's 256-robot chunk hb (wave-uniform) with the KF6 tick's cache
// policies: the frames and stamps (read once) `nt`, the state stored `sc1` while cache-resident;
// NT: the motor state streams from HBM, `nt` loads and stores.  The angle sums move as their low
// words (one 16-byte row); the high words are read only with FULL (a consumer of the whole new
// sums: the RS odometry on its prev planes) and written only by a wheel whose delta carries.
// load() issues every load; step() computes the four wheels and stores (`live` lanes only: the
// fused ISR runs clamped lanes past N) and returns the new rpm of the four wheels
// (s16_rawSpeedRpm) packed; d[] then holds the four sum deltas and, with FULL, sm[] the new sums
// (get_rawAngleSum).
// the CAN lane's arguments over the handle's motor state; false where the fused form does not
// apply (the motor state past the cached regime or its sum planes past 4 GiB, unaligned frames /
// stamps)
inline bool can_args(const DevState &s, const uint8_t *can_frames, const int16_t *can_stamps, const int8_t dir[4],
                     CanArgs &ca) {
  if (!s.m_sum_lo || state_nt(s.n * 66) || ((uintptr_t)can_frames & 15) != 0 || ((uintptr_t)can_stamps & 7) != 0)
    return false;
  ca = CanArgs{};
  ca.n = s.n;
  ca.frames = can_frames;
  ca.stamps = can_stamps;
  ca.present = nullptr;
  for (int w = 0; w < 4; w++) ca.dir[w] = dir[w];
  const MotorSlots ms = motor_slots(s);
  ca.micro = ms.micro;
  ca.angle = ms.angle;
  ca.prev = ms.prev;
  ca.prev_micro = ms.prev_micro;
  ca.rpm = s.m_rpm;
  ca.curr = s.m_curr;
  ca.sum_lo = s.m_sum_lo;
  ca.sum_hi = s.m_sum_hi;
  ca.iir_y = s.m_iir_y;
  return true;
}


// The motor state non-temporal (k_can4 and the fused kernels alike): once the motor state (66 B
// per robot), the tick's CAN frames and stamps (40 B) and the estimator state together outgrow
// the Infinity Cache, a cached motor state evicts the estimator state the tick reads next.
// Measured (kbench, two passes, profiles/r5_ab.json): ingest_can + isr_tick EKF9 2^20 195 -> 163
// us, KF6 2^21 299 -> 253-263; isr_tick_can KF6 2^21 306-307 -> 248-250, RS 2^21 255-256 ->
// 216-217 (the 40 B of frames count: without them RS 2^21 stayed cached); unchanged where
// everything fits (KF6 / RS 2^20)
inline bool can_nt(const DevState &s) { return state_nt(s.n * (66 + 40 + est_state_bytes(s))); }

template <bool NT, bool FULL = false>
struct Can4Lane {
  static constexpr int LP = NT ? kStateNT : 0, SP = st_pol(LP), IP = 2;  // IP: inputs nt
  uint64_t hb;
  uint32_t li;
  uint4 f01, f23;
  uint32_t iyw[4], slo[4];
  int32_t shi[4];
  uint64_t sv, mv, av, pmv, pav;
  int32_t d[4];   // after step(): the wheels' sum deltas (s64_rawAngleSum += d)
  int64_t sm[4];  // FULL: before step() the stored sums, after it the new ones
  uint32_t cmask; // after step(): wheel w's carry into the high word, 2 bits each (1: +1, 3: -1)

  __device__ __forceinline__ void load(const CanArgs &a, uint64_t hb_, uint32_t li_) {
    hb = hb_;
    li = li_;
    const auto rf = rsrc_span(a.frames + hb * 32);
    const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rf, li * 32u, 0, IP);
    const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rf, li * 32u + 16u, 0, IP);
    f01 = make_uint4(v0[0], v0[1], v0[2], v0[3]);
    f23 = make_uint4(v1[0], v1[1], v1[2], v1[3]);
    const auto iy = __builtin_amdgcn_raw_buffer_load_b128(rsrc_span(a.iir_y + hb * 4), li * 16u, 0, LP);
    // element copies before use (see kf6_load_in: an ext_vector element read through a bit cast
    // miscompiled once)
    iyw[0] = iy[0];
    iyw[1] = iy[1];
    iyw[2] = iy[2];
    iyw[3] = iy[3];
    const auto lw = __builtin_amdgcn_raw_buffer_load_b128(rsrc_span(a.sum_lo + hb * 4), li * 16u, 0, LP);
    slo[0] = lw[0];
    slo[1] = lw[1];
    slo[2] = lw[2];
    slo[3] = lw[3];
    if constexpr (FULL) {
      const auto hw = __builtin_amdgcn_raw_buffer_load_b128(rsrc_span(a.sum_hi + hb * 4), li * 16u, 0, LP);
      shi[0] = (int32_t)hw[0];
      shi[1] = (int32_t)hw[1];
      shi[2] = (int32_t)hw[2];
      shi[3] = (int32_t)hw[3];
#pragma unroll
      for (int w = 0; w < 4; w++) sm[w] = motor_sum_join(shi[w], slo[w]);
    }
    sv = ld_span<uint64_t, IP>(rsrc_span(a.stamps + hb * 4), li, 0);
    mv = ld_span<uint64_t, LP>(rsrc_span(a.micro + hb * 4), li, 0);
    av = ld_span<uint64_t, LP>(rsrc_span(a.angle + hb * 4), li, 0);
    pmv = ld_span<uint64_t, LP>(rsrc_span(a.prev_micro + hb * 4), li, 0);
    pav = ld_span<uint64_t, LP>(rsrc_span(a.prev + hb * 4), li, 0);
  }

  __device__ __forceinline__ uint2 step(const CanArgs &a, bool live) {
    const uint2 st = make_uint2((uint32_t)sv, (uint32_t)(sv >> 32));
    const uint2 om = make_uint2((uint32_t)mv, (uint32_t)(mv >> 32)), oa = make_uint2((uint32_t)av, (uint32_t)(av >> 32));
    const uint32_t fx[4] = {f01.x, f01.z, f23.x, f23.z}, fy[4] = {f01.y, f01.w, f23.y, f23.w};
    const uint32_t sw[2] = {st.x, st.y}, mw[2] = {om.x, om.y}, aw[2] = {oa.x, oa.y};
    const uint32_t pmw[2] = {(uint32_t)pmv, (uint32_t)(pmv >> 32)}, paw[2] = {(uint32_t)pav, (uint32_t)(pav >> 32)};
    uint32_t na[2] = {0, 0}, nr[2] = {0, 0}, nc[2] = {0, 0};
    v4u32_t oy, ol;
    cmask = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const int sh = 16 * (w & 1);
      const CanWheel o = can_wheel(fx[w], fy[w], (int16_t)(sw[w >> 1] >> sh), a.dir[w],
                                   (int16_t)(mw[w >> 1] >> sh), (int16_t)(aw[w >> 1] >> sh),
                                   (int16_t)(pmw[w >> 1] >> sh), (int16_t)(paw[w >> 1] >> sh),
                                   __builtin_bit_cast(float, iyw[w]));
      oy[w] = __builtin_bit_cast(uint32_t, o.iir_y);
      d[w] = o.d;
      int32_t cy;
      ol[w] = sum_add(slo[w], o.d, cy);
      cmask |= ((uint32_t)cy & 3u) << (2 * w);
      if constexpr (FULL) sm[w] += o.d;
      na[w >> 1] |= (uint32_t)(uint16_t)o.angle << sh;
      nr[w >> 1] |= (uint32_t)(uint16_t)o.rpm << sh;
      nc[w >> 1] |= (uint32_t)(uint16_t)o.curr << sh;
    }
    if (live) {
      __builtin_amdgcn_raw_buffer_store_b128(ol, rsrc_span(a.sum_lo + hb * 4), li * 16u, 0, SP);
      __builtin_amdgcn_raw_buffer_store_b128(oy, rsrc_span(a.iir_y + hb * 4), li * 16u, 0, SP);
      const auto pk = [](uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; };
      // the new stamps and angles over the older slots: the current ones become the previous
      // ones where they lie (DevState::m_par)
      st_span<uint64_t, SP>(rsrc_span(a.prev_micro + hb * 4), li, 0, pk(st.x, st.y));
      st_span<uint64_t, SP>(rsrc_span(a.prev + hb * 4), li, 0, pk(na[0], na[1]));
      st_span<uint64_t, SP>(rsrc_span(a.rpm + hb * 4), li, 0, pk(nr[0], nr[1]));
      st_span<uint64_t, SP>(rsrc_span(a.curr + hb * 4), li, 0, pk(nc[0], nc[1]));
    }
    return make_uint2(nr[0], nr[1]);
  }

  // the high word of a wheel whose low word carried (a wheel crossing a multiple of 2^32 counts:
  // rare).  Called last in the kernel: a read-modify-write through a plain pointer that may alias
  // any other array, kept out of the way of the kernel's own loads and stores (issued inside
  // step() it cost the fused EKF9 ISR 40 VGPRs and a spill)
  __device__ __forceinline__ void finish(const CanArgs &a, bool live) {
    if (!live || cmask == 0) return;
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const uint32_t c = (cmask >> (2 * w)) & 3u;
      if (c) {
        int32_t *hp = a.sum_hi + (hb + li) * 4 + w;
        *hp = (FULL ? shi[w] : *hp) + (c == 1u ? 1 : -1);
      }
    }
  }
};

}  // namespace fmskf
