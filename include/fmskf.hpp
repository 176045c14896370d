// fmskf.hpp -- header-only C++ mirror of the reference's task-level interfaces over the
// C ABI (fmskf.h), batched over N robots.  Names and argument meaning follow the
// reference so a caller of the firmware API finds the same calls:
//
//   reference (one robot)                                   here (N robots, SoA arrays)
//   IMT::IMU_IF_WT901C::update / isError / getDataLatest    fmskf::ImuIfWt901c
//     (src/Imu/imu_if_wt901c.hpp:8-42)
//   IMT::get_status_now_yaw (src/Imu/imu_task_main.cpp:102)  ImuIfWt901c::getYawDate
//   VDT::MOTOR_IF_M2006::rx_callback / get_rawAngleSum        fmskf::MotorIfM2006
//     (src/VehicleDrive/VD_motor_if_m2006.hpp:42,53)
//   VDT::VEHICLE_CTRL::set_now_yaw_world / update /          fmskf::VehicleCtrl
//     get_vehicle_pos_m_latest / get_vehicle_vel_mmps_latest
//     (src/VehicleDrive/VD_vehicle_controller.hpp:52-61)
//   VDT::can_tx_routine_intr (VD_task_main.cpp:366-372)      fmskf::Robots::can_tx_routine
//
// Errors: the reference's calls are void; here a non-OK status throws fmskf::Error
// (host side only -- nothing throws across the C ABI).
#pragma once
#include <stdexcept>
#include <string>

#include "fmskf.h"

namespace fmskf {

struct Error : std::runtime_error {
  int status;
  Error(int s, const std::string &what)
      : std::runtime_error(what + ": " + fmskf_strerror(s) + " (" + fmskf_last_error() + ")"),
        status(s) {}
};

inline void check(int s, const char *what) {
  if (s != FMSKF_OK) throw Error(s, what);
}

// One handle = N robots: IMU, four M2006 wheels and the estimator of each.
class Robots {
 public:
  Robots(uint32_t model, uint64_t n, int device = 0, uint32_t trig = FMSKF_TRIG_TABLE512) {
    fmskf_config cfg;
    check(fmskf_config_init(&cfg, model, n), "fmskf_config_init");
    cfg.device = device;
    cfg.trig = trig;
    check(fmskf_create(&cfg, &h_), "fmskf_create");
    n_ = n;
  }
  explicit Robots(const fmskf_config &cfg) {
    check(fmskf_create(&cfg, &h_), "fmskf_create");
    n_ = cfg.n_instances;
  }
  ~Robots() { fmskf_destroy(h_); }
  Robots(const Robots &) = delete;
  Robots &operator=(const Robots &) = delete;

  fmskf_handle handle() const { return h_; }
  uint64_t size() const { return n_; }
  void set_stream(void *hip_stream) { check(fmskf_set_stream(h_, hip_stream), "fmskf_set_stream"); }
  void sync() { check(fmskf_sync(h_), "fmskf_sync"); }

  // VDT::can_tx_routine_intr: correct with the IMU yaw, then predict from the wheels,
  // reading the device-resident IMU / motor state the ingest calls produced.
  void can_tx_routine() {
    fmskf_tick_inputs in{};
    in.mem = FMSKF_MEM_HOST;
    check(fmskf_tick(h_, &in), "fmskf_tick");
  }

 private:
  fmskf_handle h_ = nullptr;
  uint64_t n_ = 0;
};

// IMT::IMU_IF_WT901C over N robots
class ImuIfWt901c {
 public:
  explicit ImuIfWt901c(Robots &r) : r_(r) {}
  // IMU_IF_WT901C::init: drain until a quaternion frame arrived, latch q_init
  void init(const uint8_t *bytes, uint32_t stride, const uint32_t *len, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_ingest_wt901(r_.handle(), bytes, stride, len, 1, mem), "IMU init");
  }
  // IMU_IF_WT901C::update (one 10 ms poll's UART bytes per robot)
  void update(const uint8_t *bytes, uint32_t stride, const uint32_t *len, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_ingest_wt901(r_.handle(), bytes, stride, len, 0, mem), "IMU update");
  }
  // getDataLatest (Data [16][N]) + isError ([N])
  void getDataLatest(float *data, uint8_t *is_error, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_imu(r_.handle(), data, is_error, mem), "getDataLatest");
  }

 private:
  Robots &r_;
};

// VDT::MOTOR_IF_M2006 x 4 over N robots
class MotorIfM2006 {
 public:
  explicit MotorIfM2006(Robots &r) : r_(r) {}
  // rx_callback for every wheel frame of this tick: frames [N][4][8], stamps [N][4]
  void rx_callback(const uint8_t *frames, const int16_t *stamps, const uint8_t *present = nullptr,
                   uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_ingest_can(r_.handle(), frames, stamps, present, mem), "rx_callback");
  }
  // get_rawAngleSum: [4][N]
  void get_rawAngleSum(int64_t *sum, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_motors(r_.handle(), nullptr, nullptr, nullptr, sum, nullptr, mem), "get_rawAngleSum");
  }

 private:
  Robots &r_;
};

// VDT::VEHICLE_CTRL over N robots
class VehicleCtrl {
 public:
  explicit VehicleCtrl(Robots &r) : r_(r) {}
  // set_now_yaw_world(deg2rad(yaw)) -- the "correct" half of the ISR
  void set_now_yaw_world_deg(const float *yaw_deg, uint32_t mem = FMSKF_MEM_HOST) {
    fmskf_tick_inputs in{};
    in.mem = mem;
    in.yaw_deg = yaw_deg;
    check(fmskf_correct(r_.handle(), &in), "set_now_yaw_world");
  }
  // update(): the odometry / KF time update
  void update(const fmskf_tick_inputs *in = nullptr) {
    fmskf_tick_inputs def{};
    def.mem = FMSKF_MEM_HOST;
    check(fmskf_predict(r_.handle(), in ? in : &def), "update");
  }
  void get_vehicle_pos_m_latest(float *x, float *y, float *th, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_pose(r_.handle(), x, y, th, mem), "get_vehicle_pos_m_latest");
  }
  void get_vehicle_vel_mmps_latest(float *vx, float *vy, float *vth, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_vel(r_.handle(), vx, vy, vth, mem), "get_vehicle_vel_mmps_latest");
  }

 private:
  Robots &r_;
};

}  // namespace fmskf
