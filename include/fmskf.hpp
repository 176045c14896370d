// fmskf.hpp -- header-only C++ mirror of the reference's task-level interfaces over the
// C ABI (fmskf.h), batched over N robots.  Names and argument meaning follow the
// reference so a caller of the firmware API finds the same calls:
//
//   reference (one robot)                                   here (N robots, SoA arrays)
//   IMT::IMU_IF_WT901C::update / isError / getDataLatest    fmskf::ImuIfWt901c
//     (src/Imu/imu_if_wt901c.hpp:8-42)
//   IMT::get_status_now_yaw (src/Imu/imu_task_main.cpp:102)  ImuIfWt901c::getYawDate
//   VDT::MOTOR_IF_M2006::rx_callback / get_rawAngleSum /     fmskf::MotorIfM2006
//     get_status_latest (src/VehicleDrive/VD_motor_if_m2006.hpp:23-30,42,47-50,53)
//   VDT::VEHICLE_CTRL::set_now_yaw_world / update /          fmskf::VehicleCtrl
//     get_vehicle_pos_m_latest / get_vehicle_vel_mmps_latest
//     (src/VehicleDrive/VD_vehicle_controller.hpp:52-61)
//   VDT::can_tx_routine_intr (VD_task_main.cpp:366-372)      fmskf::Robots::can_tx_routine
//   VEHICLE_CTRL::start / stop / set_target_vel /            fmskf::VehicleCtrl
//     get_vehicle_vel_tgt_mmps_latest (VD_vehicle_controller.hpp:54-61)
//   MOTOR_IF_M2006::get_rawCurr_tgt (VD_motor_if_m2006.hpp:52) MotorIfM2006::get_rawCurr_tgt
//   CAN_CTRL::tx_routine (VD_can_controller.hpp:43-55)        Robots::can_tx_routine(frames)
//   RM_task_main routine_ros VehicleInfo publish (:772-823)   fmskf::publish_vehicle_info
//
// Errors: the reference's calls are void; here a non-OK status throws fmskf::Error
// (host side only -- nothing throws across the C ABI).
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

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

  // ensemble mean / covariance over every robot of every rank: the RCCL
  // communicator of this handle (one process per GPU; rank 0 makes the id), then asynchronous
  // records -- the fold and the all-gather run on a side stream behind the ticks, the result is
  // collected later (oldest first)
  static void comm_unique_id(uint8_t id[FMSKF_COMM_ID_BYTES]) {
    check(fmskf_comm_unique_id(id), "fmskf_comm_unique_id");
  }
  void comm_init(const uint8_t id[FMSKF_COMM_ID_BYTES], int rank, int world) {
    check(fmskf_comm_init(h_, id, rank, world), "fmskf_comm_init");
  }
  void ensemble_begin() { check(fmskf_ensemble_begin(h_), "fmskf_ensemble_begin"); }
  void tick_ensemble_begin(const fmskf_tick_inputs *in) {
    check(fmskf_tick_ensemble_begin(h_, in), "fmskf_tick_ensemble_begin");
  }
  void ensemble_end(double *mean, double *cov_packed) {
    check(fmskf_ensemble_end(h_, mean, cov_packed), "fmskf_ensemble_end");
  }
  // the same, with the robots the gathered records count and how many records were folded
  void ensemble_end(double *mean, double *cov_packed, double *count, uint32_t *n_records) {
    check(fmskf_ensemble_end_count(h_, mean, cov_packed, count, n_records), "fmskf_ensemble_end_count");
  }
  // the communicator's size and this rank, as RCCL reports them
  void comm_info(int *world, int *rank) { check(fmskf_comm_info(h_, world, rank), "fmskf_comm_info"); }

  // VDT::can_tx_routine_intr: correct with the IMU yaw, then VEHICLE_CTRL::update (the
  // odometry / estimator time update, then the control half: interpolators, IK, FF_PI_D),
  // then M_CAN.tx_routine -- reading the device-resident IMU / motor state the ingest calls
  // produced.  tx_frames [N][8] receives the 0x200 payloads; NULL skips control and TX
  // (estimation only).
  void can_tx_routine(uint8_t *tx_frames = nullptr, uint32_t mem = FMSKF_MEM_HOST) {
    fmskf_tick_inputs in{};
    in.mem = FMSKF_MEM_HOST;
    if (tx_frames) check(fmskf_isr_tick(h_, &in, tx_frames, mem), "fmskf_isr_tick");
    else check(fmskf_tick(h_, &in), "fmskf_tick");
  }
  // the tick's CAN RX (MOTOR_IF_M2006::rx_callback of every wheel: frames [N][4][8], stamps
  // [N][4]) and can_tx_routine in one call -- one kernel for RS, KF6 and EKF9 (fmskf_isr_tick_can)
  void can_rx_tx_routine(const uint8_t *frames, const int16_t *stamps, uint8_t *tx_frames,
                         uint32_t mem = FMSKF_MEM_HOST) {
    fmskf_tick_inputs in{};
    in.mem = mem;
    check(fmskf_isr_tick_can(h_, frames, stamps, &in, tx_frames, mem), "fmskf_isr_tick_can");
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
  // get_status_latest for every wheel (Status, VD_motor_if_m2006.hpp:23-30): [N][4] each of
  // s16_microsec_id, s16_rawAngle, s16_rawSpeedRpm, s16_rawCurr, flt_dltOutAngle_rad,
  // flt_SpeedRadPS; any pointer may be NULL
  void get_status_latest(int16_t *microsec_id, int16_t *angle, int16_t *rpm, int16_t *curr, float *dlt_out_angle_rad,
                         float *speed_radps, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_motor_status(r_.handle(), microsec_id, angle, rpm, curr, dlt_out_angle_rad, speed_radps, mem),
          "get_status_latest");
  }
  // get_rawCurr_tgt: [N][4] (FL, BL, BR, FR), what tx_routine packs
  void get_rawCurr_tgt(int16_t *curr, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_ctrl(r_.handle(), nullptr, curr, nullptr, nullptr, mem), "get_rawCurr_tgt");
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
  // start / stop (isPowerOn) for every robot, or per robot with on [N]
  void start(const uint8_t *on = nullptr, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_set_power(r_.handle(), on, mem), "start");
  }
  void stop() {
    // power off for all: a zero plane
    std::vector<uint8_t> off(r_.size(), 0);
    check(fmskf_set_power(r_.handle(), off.data(), FMSKF_MEM_HOST), "stop");
  }
  // set_target_vel(vel, acl, jrk): [3][N] planes each (x mm/s, y mm/s, th rad/s)
  void set_target_vel(const float *vel, const float *acl, const float *jrk,
                      const uint8_t *mask = nullptr, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_set_target_vel(r_.handle(), vel, acl, jrk, mask, mem), "set_target_vel");
  }
  // the control half of update() on explicit wheel speeds ([N][4] rpm) or, with NULL, on
  // the device motor state
  void control(const int16_t *rpm = nullptr, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_control(r_.handle(), rpm, mem), "control");
  }
  void get_vehicle_vel_tgt_mmps_latest(float *vel_tgt /*[3][N]*/, uint32_t mem = FMSKF_MEM_HOST) {
    check(fmskf_get_ctrl(r_.handle(), vel_tgt, nullptr, nullptr, nullptr, mem),
          "get_vehicle_vel_tgt_mmps_latest");
  }

 private:
  Robots &r_;
};

// routine_ros (RM_task_main.cpp:772-823): the VehicleInfo message of every robot
inline void publish_vehicle_info(Robots &r, fmskf_vehicle_info *out, const uint8_t *floor = nullptr,
                                 const float *cam_pitch = nullptr, const uint32_t *fault = nullptr,
                                 uint32_t mem = FMSKF_MEM_HOST) {
  check(fmskf_export_vehicle_info(r.handle(), out, floor, cam_pitch, fault, mem), "publish");
}

}  // namespace fmskf
