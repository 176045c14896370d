// ctrl_lane.hpp -- one robot's vehicle control step as lane functions:
// the VelInterpConstJerk interpolators, conv_Vdir_to_Mdir, the four FF_PI_D wheel loops and
// the C610 current narrowing, over the plane-major control state (fmskf_internal.hpp
// CtrlDev); shared by the control-step kernel and the fused firmware ISR kernels
// (kernels_ctrl.hip).  Reference operation order, bit-identical to oracle/fmskf_oracle.c.
#pragma once
#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"
#include "kf_generic.hpp"

#pragma clang fp contract(off)

namespace fmskf {

enum { IV_TGT, IV_AMAX, IV_JP, IV_JM, IV_DT1, IV_DT2, IV_DT3, IV_VINI, IV_AINI, IV_DT, IV_V, IV_A };
enum { PD_VAL, PD_INTEG, PD_LY, PD_LX, PD_TGT, PD_CTRL };

struct Interp {
  float f[kAxF];
};

// VelInterpConstJerk::set_target_params, util_vel_interp.hpp:55-104 (one active page:
// the reference rewrites every field of the inactive page, then flips)
__device__ __forceinline__ void interp_set(Interp &s, float v_t, float a_m, float jrk) {
  float *f = s.f;
  f[IV_TGT] = v_t;
  f[IV_AMAX] = a_m;
  f[IV_VINI] = f[IV_V];
  f[IV_AINI] = f[IV_A];
  if ((f[IV_TGT] - f[IV_VINI]) < 0) f[IV_AMAX] = -a_m;
  f[IV_JM] = (f[IV_AMAX] >= 0) ? -jrk : jrk;
  const float jm_inv = 1.0f / f[IV_JM];
  f[IV_JP] = (f[IV_AMAX] - f[IV_AINI] >= 0) ? jrk : -jrk;
  const float jp_inv = 1.0f / f[IV_JP];
  f[IV_DT1] = (f[IV_AMAX] - f[IV_AINI]) * jp_inv;
  f[IV_DT3] = f[IV_AMAX] * (-jm_inv);
  f[IV_DT2] = 1.0f / f[IV_AMAX] *
              (f[IV_TGT] - f[IV_VINI] - f[IV_AINI] * f[IV_DT1] * 0.5f -
               f[IV_AMAX] * (f[IV_DT1] + f[IV_DT3]) * 0.5f);
  if (f[IV_DT2] < 0.0f) {
    const float sq_in = (f[IV_AINI] * jp_inv) * (f[IV_AINI] * jp_inv) * 0.5f +
                        (f[IV_TGT] - f[IV_VINI]) * jp_inv;
    const float sq = sq_in >= 0.0f ? __builtin_sqrtf(sq_in) : 0.0f;  // arm_sqrt_f32
    f[IV_DT1] = sq - f[IV_AINI] * jp_inv;
    f[IV_AMAX] = f[IV_AINI] + f[IV_JP] * f[IV_DT1];
    f[IV_DT2] = 0.0f;
    f[IV_DT3] = f[IV_AMAX] * (-jm_inv);
  }
  f[IV_DT1] = (f[IV_DT1] < 0.0f) ? 0.0f : f[IV_DT1];
  f[IV_DT3] = (f[IV_DT3] < 0.0f) ? 0.0f : f[IV_DT3];
  f[IV_DT] = 0.0f;
}

// VelInterpConstJerk::update, util_vel_interp.hpp:106-133
__device__ __forceinline__ float interp_update(Interp &s, float ts) {
  float *f = s.f;
  if (f[IV_DT] <= f[IV_DT1] + ts) {
    f[IV_A] = f[IV_AINI] + f[IV_JP] * f[IV_DT];
    f[IV_V] = f[IV_VINI] + (f[IV_AINI] + f[IV_A]) * f[IV_DT] * 0.5f;
    f[IV_DT] = f[IV_DT] + ts;
  } else if (f[IV_DT] <= f[IV_DT1] + f[IV_DT2] + ts) {
    f[IV_A] = f[IV_AMAX];
    f[IV_V] = f[IV_V] + f[IV_A] * ts;
    f[IV_DT] = f[IV_DT] + ts;
  } else if (f[IV_DT] <= f[IV_DT1] + f[IV_DT2] + f[IV_DT3] + ts) {
    f[IV_A] = f[IV_AMAX] + f[IV_JM] * (f[IV_DT] - f[IV_DT1] - f[IV_DT2]);
    f[IV_V] = f[IV_V] + f[IV_A] * ts;
    f[IV_DT] = f[IV_DT] + ts;
  } else {
    f[IV_A] = 0.0f;
    f[IV_V] = f[IV_TGT];
  }
  return f[IV_V];
}

// conv_Vdir_to_Mdir, VD_vehicle_controller.cpp:113-118 (FL, BL, BR, FR)
__device__ __forceinline__ void vdir_to_mdir(const float v[3], float mt[4]) {
  mt[0] = (v[0] - v[1] - K::sqrtf2 * K::wheel_l * v[2] * 4.0f) / K::wheel_r;
  mt[1] = (v[0] + v[1] - K::sqrtf2 * K::wheel_l * v[2] * 4.0f) / K::wheel_r;
  mt[2] = (v[0] - v[1] + K::sqrtf2 * K::wheel_l * v[2] * 4.0f) / K::wheel_r;
  mt[3] = (v[0] + v[1] + K::sqrtf2 * K::wheel_l * v[2] * 4.0f) / K::wheel_r;
}
// FF_PI_D::update's output (util_controller.hpp:104-120,171-177) from the loop's new target,
// value, integral and LPF output: the step and ctrl_derive form it with these same operations
__device__ __forceinline__ float ffpid_out(const CtrlPrm &p, float tgt, float val, float integ, float ly) {
  const float err = tgt - val;
  float ctrl = p.p_gain * err + integ - p.d_gain * ly;
  float ff = tgt * p.ff_gain;
  ff = (ff >= p.ff_limit) ? p.ff_limit : ((ff <= -p.ff_limit) ? -p.ff_limit : ff);
  return ctrl + ff;
}

// ARM VCVT.S32.F32: truncate, saturate, NaN -> 0 (fmskf_device.hpp)
__device__ __forceinline__ int32_t f2i32_arm(float f) { return cvt_i32_arm(f); }

// set_CurrA_tgt -> set_rawCurr_tgt -> sat_curr (VD_motor_if_m2006.hpp:36-37,59-60)
__device__ __forceinline__ int16_t curr_to_raw(float amp, int dir, int lim) {
  const int16_t raw = (int16_t)(uint16_t)(uint32_t)f2i32_arm(amp * 1000.0f);
  const int16_t t = (int16_t)(uint16_t)(uint32_t)((int)raw * dir);
  return (t > lim) ? (int16_t)lim : ((t < -lim) ? (int16_t)-lim : t);
}

// Plane access for the control state.  Tiled (FMSKF_CTRL_TILED, the default): the interpolator
// and FF_PI_D arrays are [N/W][planes][W] with W = tile_w<float>() (fmskf_internal.hpp st_at),
// one scalar descriptor over robot i's tile (wave-uniform: a wave's robots lie in one
// 256-robot chunk) and a scalar offset per plane.  Planar: SMALL (every array within a 4 GiB
// buffer window) uses buffer descriptors with a 32-bit lane offset and a scalar per-plane
// offset; otherwise plain 64-bit global addressing.
template <bool SMALL, int CP = 0>
struct Planes {
  static constexpr uint32_t W = tile_w<float>();
  __amdgpu_buffer_rsrc_t r;
  float *base;
  uint64_t pp;
  uint32_t vo;
  __device__ __forceinline__ Planes(float *b, uint64_t pitch, int nplanes, uint32_t i)
      : base(b), pp(pitch), vo(i * 4u) {
    if constexpr (FMSKF_CTRL_TILED) {
      const uint32_t tl = (uint32_t)__builtin_amdgcn_readfirstlane(i / W);
      r = rsrc(b + (uint64_t)tl * nplanes * W, (uint64_t)nplanes * W * 4);
      vo = (i - tl * W) * 4u;
    } else if constexpr (SMALL) {
      r = rsrc(b, pitch * 4 * nplanes);
    }
  }
  __device__ __forceinline__ float ld(int plane, uint32_t i) const {
    if constexpr (FMSKF_CTRL_TILED)
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, plane * W * 4, CP));
    else if constexpr (SMALL)
      return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                           r, vo, (uint32_t)(plane * pp * 4), CP));
    else
      return base[plane * pp + i];
  }
  __device__ __forceinline__ void st(int plane, uint32_t i, float v) const {
    if constexpr (FMSKF_CTRL_TILED)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, plane * W * 4,
                                            st_pol(CP));
    else if constexpr (SMALL)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo,
                                            (uint32_t)(plane * pp * 4), st_pol(CP));
    else
      base[plane * pp + i] = v;
  }
};

// One robot's control step, split in its load phase (every load issued up front: vmcnt
// retires in order) and its compute + store phase, so a fused kernel can issue the loads of
// several steps before computing any of them.
template <bool SMALL, int CP = 0>
struct CtrlLane {
  uint8_t on;
  Interp ax[3];
  float pv[4][4];

  __device__ __forceinline__ void load(const CtrlDev &c, uint32_t i) {
    const Planes<SMALL, CP> AX(c.ax, c.pitch, 3 * kAxF, i), PD(c.pid, c.pitch, 4 * kPidF, i);
    on = c.power[i];
    // every interpolator field but acl_now, which update() writes before any use (round 6: 12 B
    // less per robot; only set_target_params reads it, as acl_ini)
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
      for (int k = 0; k < kAxF; k++) ax[a].f[k] = k == IV_A ? 0.0f : AX.ld(a * kAxF + k, i);
    // now_val from the rpm the last step ran on (CtrlDev::rpm_prev), the other loop fields from
    // their planes
    const uint2 rp = reinterpret_cast<const uint2 *>(c.rpm_prev)[i];
    const int16_t r[4] = {(int16_t)(rp.x & 0xFFFFu), (int16_t)(rp.x >> 16), (int16_t)(rp.y & 0xFFFFu),
                          (int16_t)(rp.y >> 16)};
#pragma unroll
    for (int w = 0; w < 4; w++) {
      pv[w][PD_VAL] = rpm_to_mvel(r[w]) * 36.0f;
#pragma unroll
      for (int k = PD_INTEG; k < 4; k++) pv[w][k] = PD.ld(w * kPidF + k, i);
    }
  }

  // rw: the four s16_rawSpeedRpm (FL, BL, BR, FR) packed in 8 bytes.  Returns the packed
  // raw current targets (also stored to c.curr).
  __device__ __forceinline__ uint2 step(const CtrlDev &c, const CtrlPrm &p, uint32_t i, uint2 rw) {
    const uint64_t pp = c.pitch;
    const Planes<SMALL, CP> AX(c.ax, pp, 3 * kAxF, i), PD(c.pid, pp, 4 * kPidF, i);
    float v[3];
#pragma unroll
    for (int a = 0; a < 3; a++) v[a] = interp_update(ax[a], p.ts);
    float mt[4];
    vdir_to_mdir(v, mt);
    const int16_t r[4] = {(int16_t)(rw.x & 0xFFFFu), (int16_t)(rw.x >> 16),
                          (int16_t)(rw.y & 0xFFFFu), (int16_t)(rw.y >> 16)};
    float po[4][kPidF];
    int16_t cur[4];
    if (on) {
#pragma unroll
      for (int w = 0; w < 4; w++) {
        // FF_PI_D::update with now_tgt_ = Mvel_tgt * GEAR_RATIO, _nowval = Mvel * GEAR_RATIO
        const float tgt = mt[w] * 36.0f;
        const float val = rpm_to_mvel(r[w]) * 36.0f;
        const float err = tgt - val;
        const float lx = (val - pv[w][PD_VAL]) * p.freq;
        const float ly = p.a1 * pv[w][PD_LY] + p.b0 * lx + p.b1 * pv[w][PD_LX];
        float integ = pv[w][PD_INTEG] + p.i_gain * p.dt * err;
        integ = (integ >= p.i_limit) ? p.i_limit : ((integ <= -p.i_limit) ? -p.i_limit : integ);
        const float ctrl = ffpid_out(p, tgt, val, integ, ly);
        po[w][PD_VAL] = val;
        po[w][PD_INTEG] = integ;
        po[w][PD_LY] = ly;
        po[w][PD_LX] = lx;
        po[w][PD_TGT] = tgt;
        po[w][PD_CTRL] = ctrl;
        cur[w] = curr_to_raw(ctrl, p.dir[w], p.curr_limit);
      }
    } else {
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int k = 0; k < kAxF; k++) ax[a].f[k] = 0.0f;
#pragma unroll
      for (int w = 0; w < 4; w++) {
#pragma unroll
        for (int k = 0; k < kPidF; k++) po[w][k] = 0.0f;
        cur[w] = curr_to_raw(0.0f, p.dir[w], p.curr_limit);
      }
    }
    // the interpolator fields update() changes; after a reset (power off) all of them
#pragma unroll
    for (int a = 0; a < 3; a++) {
      AX.st(a * kAxF + IV_DT, i, ax[a].f[IV_DT]);
      AX.st(a * kAxF + IV_V, i, ax[a].f[IV_V]);
      AX.st(a * kAxF + IV_A, i, ax[a].f[IV_A]);
    }
    if (!on) {
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int k = 0; k < IV_DT; k++) AX.st(a * kAxF + k, i, 0.0f);
    }
    // the loop state the next step reads; now_tgt, now_ctrl and vel_tgt only where they cannot
    // be formed later from that state (power off: the reset erased the interpolators' output) or
    // when asked to (p.store_derived)
#pragma unroll
    for (int w = 0; w < 4; w++)
#pragma unroll
      for (int k = PD_INTEG; k < PD_TGT; k++) PD.st(w * kPidF + k, i, po[w][k]);
    reinterpret_cast<uint2 *>(c.rpm_prev)[i] = on ? rw : make_uint2(0u, 0u);  // now_val's rpm
    if (p.store_derived) {
#pragma unroll
      for (int w = 0; w < 4; w++) {
        PD.st(w * kPidF + PD_TGT, i, po[w][PD_TGT]);
        PD.st(w * kPidF + PD_CTRL, i, po[w][PD_CTRL]);
      }
    }
    if (!on || p.store_derived) {
#pragma unroll
      for (int a = 0; a < 3; a++) c.vel_tgt[a * pp + i] = v[a];
    }
    const uint2 cw = make_uint2((uint32_t)(uint16_t)cur[0] | ((uint32_t)(uint16_t)cur[1] << 16),
                                (uint32_t)(uint16_t)cur[2] | ((uint32_t)(uint16_t)cur[3] << 16));
    reinterpret_cast<uint2 *>(c.curr)[i] = cw;
    return cw;
  }
};

// now_vhcl_vel_tgt_mmps, FF_PI_D now_tgt and now_ctrl of robot i formed from the state the last
// step left (ctrl_derive_out is the kernel): with the power on, the interpolators' output is the
// stored vel_now and the loops' new value / integral / LPF output are stored, so the same
// operations as the step give the same bits; with it off the step reset everything, stored
// vel_tgt itself, and the loops' target and output are 0.  Valid while the power flags and the
// parameters are those of that step (the host materialises before set_power; p: the step's)
template <bool SMALL>
__device__ __forceinline__ void ctrl_derive_lane(const CtrlDev &c, const CtrlPrm &p, uint32_t i) {
  const Planes<SMALL> AX(c.ax, c.pitch, 3 * kAxF, i), PD(c.pid, c.pitch, 4 * kPidF, i);
  if (!c.power[i]) {
#pragma unroll
    for (int w = 0; w < 4; w++) {
      PD.st(w * kPidF + PD_TGT, i, 0.0f);
      PD.st(w * kPidF + PD_CTRL, i, 0.0f);
    }
    return;
  }
  float v[3], mt[4];
#pragma unroll
  for (int a = 0; a < 3; a++) v[a] = AX.ld(a * kAxF + IV_V, i);
  float pv[4][3];
  const uint2 rp = reinterpret_cast<const uint2 *>(c.rpm_prev)[i];
  const int16_t r[4] = {(int16_t)(rp.x & 0xFFFFu), (int16_t)(rp.x >> 16), (int16_t)(rp.y & 0xFFFFu),
                        (int16_t)(rp.y >> 16)};
#pragma unroll
  for (int w = 0; w < 4; w++) {
    pv[w][PD_VAL] = rpm_to_mvel(r[w]) * 36.0f;  // now_val, as the step formed it
#pragma unroll
    for (int k = PD_INTEG; k < 3; k++) pv[w][k] = PD.ld(w * kPidF + k, i);  // PD_INTEG, PD_LY
  }
  vdir_to_mdir(v, mt);
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const float tgt = mt[w] * 36.0f;
    PD.st(w * kPidF + PD_TGT, i, tgt);
    PD.st(w * kPidF + PD_CTRL, i, ffpid_out(p, tgt, pv[w][PD_VAL], pv[w][PD_INTEG], pv[w][PD_LY]));
  }
#pragma unroll
  for (int a = 0; a < 3; a++) c.vel_tgt[a * c.pitch + i] = v[a];
}

// bytes of the per-robot control state the step streams (interpolators + wheel loops)
inline uint64_t ctrl_state_bytes(const CtrlDev &c) { return c.n * (4ull * (3 * kAxF + 4 * kPidF) + 8ull); }

// C610 0x200 payload of one robot: bytes (hi, lo) per wheel -> swap the bytes of every 16-bit half
__device__ __forceinline__ uint2 tx_frame(uint2 c) {
  auto sw = [](uint32_t v) { return ((v & 0x00FF00FFu) << 8) | ((v >> 8) & 0x00FF00FFu); };
  return make_uint2(sw(c.x), sw(c.y));
}

}  // namespace fmskf
