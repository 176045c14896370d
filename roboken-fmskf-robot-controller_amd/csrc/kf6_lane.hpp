// kf6_lane.hpp -- one robot's 6-state KF tick as lane functions (inputs, state load / store,
// measurement frontend, update + predict), shared by the KF6 tick kernels (kernels_kf6.hip)
// and the fused firmware ISR (kernels_ctrl.hip k_isr_kf6).  Canonical operation order of the
// oracle (orc_kf6_tick), so every kernel built from these is bit-exact to it.
#pragma once
#include "kf_generic.hpp"

#pragma clang fp contract(off)

namespace fmskf {

// REC: the inputs come as 16-byte fmskf_kf6_record's (one 16-byte load per lane) instead of
// the yaw / gyro / rpm planes (three loads): measured 41.6 -> 39.5 us per tick at 2^20
// NT: the state is loaded and stored non-temporal (fmskf_internal.hpp state_nt)
// ENS: the tick also writes its block's ensemble record of the post-tick state
// (fmskf_tick_ensemble; ens_device.hpp), so the record costs no second pass over x
// COMP: FMSKF_CFG_COMP_POS -- px, py, P00, P10, P11 carried as hi + lo (Kf6Params::lo, 5 tiled
// rows), every addition to them a TwoSum (oracle orc_kf6_tick_comp)
template <bool LIBM_, bool UPD_, bool PRED_, bool SMALL_, bool VALID_, bool REC_ = false, bool NT_ = false,
          bool ENS_ = false, bool COMP_ = false>
struct Opt {
  static constexpr bool LIBM = LIBM_, UPD = UPD_, PRED = PRED_, SMALL = SMALL_, VALID = VALID_,
                        REC = REC_, NT = NT_, ENS = ENS_, COMP = COMP_;
  static constexpr int CP = NT_ ? kStateNT : 0;
};
template <class O>
using WithNT = Opt<O::LIBM, O::UPD, O::PRED, O::SMALL, O::VALID, O::REC, true, O::ENS, O::COMP>;
template <class O>
using WithEns = Opt<O::LIBM, O::UPD, O::PRED, O::SMALL, O::VALID, O::REC, O::NT, true, O::COMP>;
template <class O>
using WithComp = Opt<O::LIBM, O::UPD, O::PRED, O::SMALL, O::VALID, O::REC, O::NT, O::ENS, true>;

// the compensated entries of COMP: x 0-1 (px, py), packed P 0-2 (P00, P10, P11)
constexpr unsigned kKf6CXM = kPosCXM;
constexpr unsigned long long kKf6CPM = kPosCPM;
// the lane's low parts (COMP), one register when unused
template <class O>
struct Kf6Lo {
  float v[O::COMP ? kKf6LoRows : 1];
};

struct Kf6In {
  float yaw, gz;
  uint2 rpm;
  uint32_t valid;
};

template <int CP = 0>
__device__ __forceinline__ float ld_f32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, CP));
}
template <int CP = 0>
__device__ __forceinline__ void st_f32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                       float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, CP);
}

// The per-tick inputs are read exactly once: load them non-temporal (gfx950 `nt`, aux bit 1)
// so the fresh 16 MB per tick at 2^20 displaces less of the state from the caches (measured
// 43.6 -> 42.7 us per tick with a 64-tick input ring).
#ifndef FMSKF_IN_CPOL
#define FMSKF_IN_CPOL 2
#endif
// inputs of one tick; planes of tick t start at t * stride elements
template <class O>
__device__ __forceinline__ Kf6In kf6_load_in(const TickIn &in, uint64_t n, uint64_t t, uint32_t i) {
  const uint64_t tb = t * in.stride;
  // Past the SMALL range (N >= ~51M) descriptors start at the block's first instance hb
  // (wave-uniform: every lane of a block, clamped ones included, lies in [hb, hb + 255]), so the
  // 32-bit lane offsets stay below 4 KiB for any N up to the 2^30 cap (a lane offset of i * 16
  // would wrap past 2^28 robots).  SMALL keeps the array-base form: ~0.2 us per 2^20 tick less.
  const uint32_t hb = O::SMALL ? 0u : __builtin_amdgcn_readfirstlane(i) & ~(uint32_t)(kBlock - 1);
  const uint32_t li = i - hb;
  const uint64_t base = tb + hb, left = n - hb;
  Kf6In m;
  if constexpr (O::REC) {
    const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc(in.rec + base * 4, left * 16), li * 16u, 0,
                                                         FMSKF_IN_CPOL);
    // bit_cast a prvalue copy: on a vector-element lvalue clang's __builtin_bit_cast reads
    // element 0 (measured: r[1] came back as r[0])
    const uint32_t w0 = r[0], w1 = r[1];
    m.yaw = __builtin_bit_cast(float, w0);
    m.gz = __builtin_bit_cast(float, w1);
    m.rpm = make_uint2(r[2], r[3]);
    m.valid = O::VALID ? (uint32_t)in.valid[tb + i] : 1u;
    return m;
  }
  // the yaw / gyro z planes, or for a NULL one the IMU state's Yaw / GZ words (fmskf_device.hpp
  // tick_yaw): one dword per lane either way (with both from the IMU state, the same dword twice)
  const bool yw = (in.imu_words & 1u) != 0, gw = (in.imu_words & 2u) != 0;
  m.yaw = tick_yaw(yw, __builtin_amdgcn_raw_buffer_load_b32(rsrc(in.yaw_deg + base, left * 4), li * 4u, 0,
                                                            FMSKF_IN_CPOL));
  m.gz = tick_gz(gw, __builtin_amdgcn_raw_buffer_load_b32(rsrc(in.gyro_z + base, left * 4), li * 4u, 0,
                                                          FMSKF_IN_CPOL));
  const auto rr = __builtin_amdgcn_raw_buffer_load_b64(rsrc(in.rpm + base * 4, left * 8), li * 8u, 0,
                                                       FMSKF_IN_CPOL);
  m.rpm = make_uint2(rr[0], rr[1]);
  m.valid = O::VALID ? (uint32_t)in.valid[tb + i] : 1u;
  return m;
}

template <class O>
__device__ __forceinline__ void kf6_load_state(const float *xg, const float *Pg, uint64_t pp,
                                               uint32_t i, float (&x)[6], float (&P)[21]) {
  if constexpr (FMSKF_KF6_TILED) {
    // tiled state (fmskf_internal.hpp st_at, 2048 robots per tile row): the tile is
    // wave-uniform (a wave's 64 robots, the clamped ones included, lie in one 256-robot chunk),
    // so each array is one scalar descriptor over its tile and each row a scalar offset
    constexpr uint32_t W = tile_w<float>();
    const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane(i / W);
    const uint32_t c = (i - tl * W) * 4u;
    const auto rx = rsrc(xg + (uint64_t)tl * (6 * W), 6 * W * 4), rp = rsrc(Pg + (uint64_t)tl * (21 * W), 21 * W * 4);
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = ld_f32<O::CP>(rx, c, k * W * 4);
#pragma unroll
    for (int k = 0; k < 21; k++) P[k] = ld_f32<O::CP>(rp, c, k * W * 4);
  } else if constexpr (O::SMALL) {
    const auto rx = rsrc(xg, pp * 24), rp = rsrc(Pg, pp * 84);
    const uint32_t ps = (uint32_t)pp * 4u;
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = ld_f32<O::CP>(rx, i * 4u, k * ps);
#pragma unroll
    for (int k = 0; k < 21; k++) P[k] = ld_f32<O::CP>(rp, i * 4u, k * ps);
  } else {
#pragma unroll
    for (int k = 0; k < 6; k++) x[k] = ld_f32<O::CP>(rsrc(xg + k * pp, pp * 4), i * 4u, 0);
#pragma unroll
    for (int k = 0; k < 21; k++) P[k] = ld_f32<O::CP>(rsrc(Pg + k * pp, pp * 4), i * 4u, 0);
  }
}

template <class O>
__device__ __forceinline__ void kf6_store_state(float *xg, float *Pg, uint64_t pp, uint32_t i,
                                                const float (&x)[6], const float (&P)[21]) {
  if constexpr (FMSKF_KF6_TILED) {
    constexpr uint32_t W = tile_w<float>();
    const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane(i / W);
    const uint32_t c = (i - tl * W) * 4u;
    const auto rx = rsrc(xg + (uint64_t)tl * (6 * W), 6 * W * 4), rp = rsrc(Pg + (uint64_t)tl * (21 * W), 21 * W * 4);
#pragma unroll
    for (int k = 0; k < 6; k++) st_f32<st_pol(O::CP)>(rx, c, k * W * 4, x[k]);
#pragma unroll
    for (int k = 0; k < 21; k++) st_f32<st_pol(O::CP)>(rp, c, k * W * 4, P[k]);
  } else if constexpr (O::SMALL) {
    const auto rx = rsrc(xg, pp * 24), rp = rsrc(Pg, pp * 84);
    const uint32_t ps = (uint32_t)pp * 4u;
#pragma unroll
    for (int k = 0; k < 6; k++) st_f32<st_pol(O::CP)>(rx, i * 4u, k * ps, x[k]);
#pragma unroll
    for (int k = 0; k < 21; k++) st_f32<st_pol(O::CP)>(rp, i * 4u, k * ps, P[k]);
  } else {
#pragma unroll
    for (int k = 0; k < 6; k++) st_f32<st_pol(O::CP)>(rsrc(xg + k * pp, pp * 4), i * 4u, 0, x[k]);
#pragma unroll
    for (int k = 0; k < 21; k++) st_f32<st_pol(O::CP)>(rsrc(Pg + k * pp, pp * 4), i * 4u, 0, P[k]);
  }
}

// the COMP low-part rows, tiled like x ([N/W][5][W], one scalar descriptor per tile)
template <class O>
__device__ __forceinline__ void kf6_load_lo(const float *lg, uint32_t i, Kf6Lo<O> &l) {
  if constexpr (O::COMP) {
    constexpr uint32_t W = tile_w<float>();
    const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane(i / W);
    const uint32_t c = (i - tl * W) * 4u;
    const auto r = rsrc(lg + (uint64_t)tl * (kKf6LoRows * W), kKf6LoRows * W * 4);
#pragma unroll
    for (int k = 0; k < (int)kKf6LoRows; k++) l.v[k] = ld_f32<O::CP>(r, c, k * W * 4);
  }
}
template <class O>
__device__ __forceinline__ void kf6_store_lo(float *lg, uint32_t i, const Kf6Lo<O> &l) {
  if constexpr (O::COMP) {
    constexpr uint32_t W = tile_w<float>();
    const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane(i / W);
    const uint32_t c = (i - tl * W) * 4u;
    const auto r = rsrc(lg + (uint64_t)tl * (kKf6LoRows * W), kKf6LoRows * W * 4);
#pragma unroll
    for (int k = 0; k < (int)kKf6LoRows; k++) st_f32<st_pol(O::CP)>(r, c, k * W * 4, l.v[k]);
  }
}

// z = (deg2rad(yaw), -deg2rad(gz), wheel velocity rotated by the measured heading)
// (imu_task_main.cpp:102-104, util_mymath.hpp:16, imu_if_wt901c.cpp:113,
//  VD_vehicle_controller.cpp:21-33,47-51); y = z - H x with the heading innovation wrapped
template <bool LIBM>
__device__ __forceinline__ void kf6_innov(const Kf6In &m, const float *tab, const float (&x)[6],
                                          float (&y)[4]) {
  int16_t r[4];
  unpack4(m.rpm, r);
  const float th = deg2rad(m.yaw);
  const float om = -deg2rad(m.gz);
  float vx, vy, vth;
  mdir_to_vdir(rpm_to_mvel(r[0]), rpm_to_mvel(r[1]), rpm_to_mvel(r[2]), rpm_to_mvel(r[3]), vx, vy,
               vth);
  // the sin/cos policies reduce any angle themselves (no normalize_rad_0to2pi needed)
  const float c = cos_p<LIBM>(th, tab), s = sin_p<LIBM>(th, tab);
  const float z2 = (vx * c - vy * s) * 0.001f;
  const float z3 = (vx * s + vy * c) * 0.001f;
  y[0] = wrap_innov(th - x[2]);
  y[1] = om - x[5];
  y[2] = z2 - x[3];
  y[3] = z3 - x[4];
}

template <class O>
__device__ __forceinline__ void kf6_tick1(const Kf6In &m, const float *tab, const Kf6Params &prm,
                                          float (&x)[6], float (&P)[21], Kf6Lo<O> &l) {
  if (O::UPD && (!O::VALID || m.valid)) {
    float y[4];
    kf6_innov<O::LIBM>(m, tab, x, y);
    if constexpr (O::COMP) kf_update<MdKF6, -1, float, 6, 4, 21, kKf6CXM, kKf6CPM>(x, P, y, prm.r, nullptr, l.v);
    else kf_update<MdKF6>(x, P, y, prm.r);
  }
  if (O::PRED) {
    const float dt = prm.dt;
    if constexpr (O::COMP) {
      th_add(x[0], l.v[0], dt * x[3]);
      th_add(x[1], l.v[1], dt * x[4]);
      th_norm(x[0], l.v[0]);
      th_norm(x[1], l.v[1]);
      x[2] = wrap_pi(dfma(dt, x[5], x[2]));
      kf_predict_cov_c<MdKF6, kKf6CXM, kKf6CPM>(P, [&](int, int) { return dt; }, prm.q, l.v);
    } else {
      x[0] = dfma(dt, x[3], x[0]);
      x[1] = dfma(dt, x[4], x[1]);
      x[2] = wrap_pi(dfma(dt, x[5], x[2]));
      kf_predict_cov<MdKF6>(P, [&](int, int) { return dt; }, prm.q);
    }
  }
}

}  // namespace fmskf
