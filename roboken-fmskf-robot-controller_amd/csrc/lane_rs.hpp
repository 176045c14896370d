// lane_rs.hpp -- one robot's reference-semantics tick, shared by the RS tick kernel
// (kernels_rs.hip) and the fused firmware-ISR kernel (kernels_ctrl.hip).
//
// correct = VD_task_main.cpp:368 (theta hard overwrite by the IMU yaw); predict =
// VEHICLE_CTRL::update's velocity + odometry part (VD_vehicle_controller.cpp:11-51): int64
// encoder-sum differences scaled in double and narrowed to float, mecanum forward kinematics,
// rotation by the heading through the selected sin/cos policy, mm -> m.
#pragma once
#include "fmskf_device.hpp"

#pragma clang fp contract(off)

namespace fmskf {

struct RsLane {
  float px, py, th, vx, vy, vth;
  int64_t prev[4];
};

// s64_rawAngleSumPrev (round 6): 16-byte pairs (wheels 0-1, wheels 2-3) in 64-robot tiles,
// [N/64][2][64] x 16 B, so a wave's 64 robots move each half as one 1 KiB run of whole lines:
// two 16-byte accesses per robot instead of one 8-byte access per wheel plane.  (Plain [N][4]
// rows, 32 B per lane, left every line half-written by each store and measured 30% slower with
// the memory-side `sc1` stores of the cache-resident tick: 25.8 -> 33.5 us at 2^20.)
// rs_prev_at: the pair of wheels 2h, 2h + 1 of robot i, in 16-byte units
__host__ __device__ __forceinline__ uint64_t rs_prev_at(uint64_t i, int h) {
  return (i >> 6) * 128 + (uint64_t)h * 64 + (i & 63);
}
__device__ __forceinline__ void rs_prev_load(const int64_t *prev, uint64_t i, int64_t (&pv)[4]) {
  const longlong2 a = reinterpret_cast<const longlong2 *>(prev)[rs_prev_at(i, 0)];
  const longlong2 b = reinterpret_cast<const longlong2 *>(prev)[rs_prev_at(i, 1)];
  pv[0] = a.x;
  pv[1] = a.y;
  pv[2] = b.x;
  pv[3] = b.y;
}
// one s64_rawAngleSum from its split halves: hi * 2^32 + the low word read as int32
// (fmskf_internal.hpp m_sum_lo)
__host__ __device__ __forceinline__ int64_t motor_sum_join(int32_t hi, uint32_t lo) {
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) + (uint64_t)(int64_t)(int32_t)lo);
}
// the motor state's s64_rawAngleSum of robot i from its split halves
__device__ __forceinline__ void motor_sum_load(const uint32_t *lo, const int32_t *hi, uint64_t i, int64_t (&s)[4]) {
  const uint4 l = reinterpret_cast<const uint4 *>(lo)[i];
  const int4 h = reinterpret_cast<const int4 *>(hi)[i];
  s[0] = motor_sum_join(h.x, l.x);
  s[1] = motor_sum_join(h.y, l.y);
  s[2] = motor_sum_join(h.z, l.z);
  s[3] = motor_sum_join(h.w, l.w);
}
__device__ __forceinline__ void rs_prev_store(int64_t *prev, uint64_t i, const int64_t (&pv)[4]) {
  reinterpret_cast<longlong2 *>(prev)[rs_prev_at(i, 0)] = make_longlong2(pv[0], pv[1]);
  reinterpret_cast<longlong2 *>(prev)[rs_prev_at(i, 1)] = make_longlong2(pv[2], pv[3]);
}

template <bool LIBM, bool CORR, bool PRED>
__device__ __forceinline__ void rs_tick1(RsLane &s, float yaw_deg, uint2 rpm, const int64_t (&sum)[4],
                                         const float *tab) {
  if (CORR) s.th = deg2rad(yaw_deg);
  if (PRED) {
    const int16_t r0 = (int16_t)(rpm.x & 0xFFFFu), r1 = (int16_t)(rpm.x >> 16);
    const int16_t r2 = (int16_t)(rpm.y & 0xFFFFu), r3 = (int16_t)(rpm.y >> 16);
    mdir_to_vdir(rpm_to_mvel(r0), rpm_to_mvel(r1), rpm_to_mvel(r2), rpm_to_mvel(r3), s.vx, s.vy,
                 s.vth);
    float mrad[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
      mrad[w] = (float)((double)(sum[w] - s.prev[w]) * (double)K::out_rad_per_raw *
                        (double)K::gear_ratio_inv);
      s.prev[w] = sum[w];
    }
    float lx, ly, lth;
    mdir_to_vdir(mrad[0], mrad[1], mrad[2], mrad[3], lx, ly, lth);
    const float rr = normalize_rad_0to2pi(s.th);
    const float c = cos_p<LIBM>(rr, tab);
    const float sn = sin_p<LIBM>(rr, tab);
    s.px = s.px + (lx * c - ly * sn) * 0.001f;
    s.py = s.py + (lx * sn + ly * c) * 0.001f;
  }
}

}  // namespace fmskf
