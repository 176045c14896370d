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
