// fleet_loop.cpp -- the firmware's per-tick call shape, for N robots at once.
//
// Mirrors the task structure of the reference: the IMU task polls the WT901 every
// 10 ms (IMT::main, imu_task_main.cpp:43-82), CAN RX delivers four C610 frames per
// millisecond (VD_can_controller.hpp:65-95), the 1 kHz ISR corrects with the IMU yaw
// and predicts from the wheels, runs the wheel speed loops and sends the 0x200 current
// frame (VD_task_main.cpp:366-372), and the ROS task publishes VehicleInfo at 60 Hz
// (RM_task_main.cpp:772-823).  Synthetic traffic: each robot drives its wheels at a
// constant rpm and is commanded forward at 200 mm/s.  Every 16 ticks the fleet's pose
// mean / covariance is recorded asynchronously (fmskf_ensemble_begin: fold and, across
// processes, the RCCL all-gather on the handle's side stream) and collected two records later.
//
//   fleet_loop [N] [ticks]
//   FLEET_MODEL=kf6 fleet_loop ...    the 6-state KF instead of the reference's RS odometry
//   FLEET_SPLIT_CAN=1 fleet_loop ...  CAN RX and the ISR as two calls (default: one,
//       fmskf_isr_tick_can -- one kernel for RS, KF6 and EKF9)
//   FLEET_WORLD=W FLEET_RANK=r FLEET_ID=/path/id fleet_loop ...   one process per GPU: rank 0
//       writes the communicator id to FLEET_ID, every rank reads it (device = rank, or
//       FLEET_DEVICE)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <string>
#include <thread>
#include <vector>

#include "fmskf.hpp"

static void wt901_frame(uint8_t *o, uint8_t type, int16_t w0, int16_t w1, int16_t w2, int16_t w3) {
  const int16_t w[4] = {w0, w1, w2, w3};
  o[0] = 0x55;
  o[1] = type;
  for (int k = 0; k < 4; k++) {
    o[2 + 2 * k] = (uint8_t)(w[k] & 0xFF);
    o[3 + 2 * k] = (uint8_t)((uint16_t)w[k] >> 8);
  }
  uint8_t s = 0;
  for (int k = 0; k < 10; k++) s += o[k];
  o[10] = s;
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1u << 16);
  const int ticks = argc > 2 ? atoi(argv[2]) : 1000;
  const int world = getenv("FLEET_WORLD") ? atoi(getenv("FLEET_WORLD")) : 1;
  const int rank = getenv("FLEET_RANK") ? atoi(getenv("FLEET_RANK")) : 0;
  try {
    const int device = getenv("FLEET_DEVICE") ? atoi(getenv("FLEET_DEVICE")) : (world > 1 ? rank : 0);
    const bool kf6 = getenv("FLEET_MODEL") && std::string(getenv("FLEET_MODEL")) == "kf6";
    const bool split_can = getenv("FLEET_SPLIT_CAN") && atoi(getenv("FLEET_SPLIT_CAN")) != 0;
    fmskf::Robots robots(kf6 ? FMSKF_MODEL_KF6 : FMSKF_MODEL_RS, n, device);
    if (world > 1) {  // the handle's RCCL communicator, its id passed through a file
      const char *path = getenv("FLEET_ID");
      if (!path) throw std::runtime_error("FLEET_ID must name the id file");
      uint8_t id[FMSKF_COMM_ID_BYTES];
      if (rank == 0) {
        fmskf::Robots::comm_unique_id(id);
        const std::string tmp = std::string(path) + ".tmp";
        FILE *f = fopen(tmp.c_str(), "wb");
        if (!f || fwrite(id, 1, sizeof(id), f) != sizeof(id)) throw std::runtime_error("cannot write FLEET_ID");
        fclose(f);
        rename(tmp.c_str(), path);
      } else {
        FILE *f = nullptr;
        for (int k = 0; k < 600 && !(f = fopen(path, "rb")); k++)
          std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (!f || fread(id, 1, sizeof(id), f) != sizeof(id)) throw std::runtime_error("cannot read FLEET_ID");
        fclose(f);
      }
      robots.comm_init(id, rank, world);
      int cw = 0, cr = -1;
      robots.comm_info(&cw, &cr);  // what RCCL itself reports
      if (cw != world || cr != rank) throw std::runtime_error("communicator size / rank differ from FLEET_*");
    }
    fmskf::ImuIfWt901c imu(robots);
    fmskf::MotorIfM2006 motors(robots);
    fmskf::VehicleCtrl vehicle(robots);

    const uint32_t stride = 48;
    std::vector<uint8_t> bytes(n * stride);
    std::vector<uint32_t> len(n, 44);
    std::vector<uint8_t> frames(n * 32);
    std::vector<int16_t> stamps(n * 4);
    std::vector<int64_t> enc(n * 4, 0);
    std::vector<float> px(n), py(n), pth(n);
    std::vector<uint8_t> tx(n * 8);
    std::vector<fmskf_vehicle_info> info(n);
    const int dir[4] = {1, 1, -1, -1};
    // REQ_MOVE_DIR GO_FORWARD at 200 mm/s with C_ACCEL/JERK_MAX_MOVE (VD_task_main.cpp:29-38,191-198)
    std::vector<float> vel(3 * n, 0.f), acl(3 * n), jrk(3 * n);
    for (uint64_t i = 0; i < n; i++) {
      vel[i] = 200.f;
      acl[i] = acl[n + i] = 1000.f;
      acl[2 * n + i] = 30.f;
      jrk[i] = jrk[n + i] = 10000.f;
      jrk[2 * n + i] = 300.f;
    }
    vehicle.start();
    vehicle.set_target_vel(vel.data(), acl.data(), jrk.data());

    double mean[6], cov[21], counted = 0.0;
    uint32_t folded = 0;
    int pending = 0, records = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < ticks; t++) {
      // CAN RX: wheel i advances (1 + i % 5) counts per tick, all wheels forward
      for (uint64_t i = 0; i < n; i++) {
        for (int w = 0; w < 4; w++) {
          enc[i * 4 + w] += 1 + (int64_t)(i % 5);
          const int32_t sensor = (int32_t)(((enc[i * 4 + w] * dir[w]) % 8192 + 8192) % 8192);
          const int16_t rpm = (int16_t)((1 + i % 5) * 7 * dir[w]);
          uint8_t *f = &frames[(i * 4 + w) * 8];
          f[0] = (uint8_t)(sensor >> 8);
          f[1] = (uint8_t)(sensor & 0xFF);
          f[2] = (uint8_t)((uint16_t)rpm >> 8);
          f[3] = (uint8_t)(rpm & 0xFF);
          f[4] = 0;
          f[5] = 100;
          f[6] = f[7] = 0;
          stamps[i * 4 + w] = (int16_t)(((t + 1) * 1000 + 7 * w) & 0x7FFF);
        }
      }
      if (split_can) motors.rx_callback(frames.data(), stamps.data());
      if (t % 10 == 0) {  // IMU task, 100 Hz: acc, gyro, angle (yaw = 30 deg), quaternion
        for (uint64_t i = 0; i < n; i++) {
          uint8_t *b = &bytes[i * stride];
          wt901_frame(b, 0x51, 0, 0, 2048, 2500);
          wt901_frame(b + 11, 0x52, 0, 0, 0, 0);
          wt901_frame(b + 22, 0x53, 0, 0, (int16_t)(30.0 / 180.0 * 32768.0), 0);
          wt901_frame(b + 33, 0x59, 32767, 0, 0, 0);
        }
        if (t == 0) imu.init(bytes.data(), stride, len.data());
        else imu.update(bytes.data(), stride, len.data());
      }
      // correct + predict + wheel loops + 0x200 frames, device-resident inputs (with the
      // tick's CAN RX in the same call unless split)
      if (split_can) robots.can_tx_routine(tx.data());
      else robots.can_rx_tx_routine(frames.data(), stamps.data(), tx.data());
      if (t % 17 == 16) fmskf::publish_vehicle_info(robots, info.data());  // ~60 Hz
      if (t % 16 == 15) {  // the fleet's ensemble record, collected two records later
        robots.ensemble_begin();
        if (++pending == 3) {
          robots.ensemble_end(mean, cov, &counted, &folded);
          pending--;
          records++;
        }
      }
    }
    while (pending) {
      robots.ensemble_end(mean, cov, &counted, &folded);
      pending--;
      records++;
    }
    robots.sync();
    auto t1 = std::chrono::steady_clock::now();
    vehicle.get_vehicle_pos_m_latest(px.data(), py.data(), pth.data());
    const double s = std::chrono::duration<double>(t1 - t0).count();
    printf("robots=%llu ticks=%d  %.3f s  (host-fed, PCIe-inclusive %.3g robot-ticks/s)\n",
           (unsigned long long)n, ticks, s, (double)n * ticks / s);
    printf("robot 0: x=%.6f m y=%.6f m th=%.6f rad   robot 4: x=%.6f m\n", px[0], py[0], pth[0],
           n > 4 ? px[4] : 0.f);
    printf("robot 0: VehicleInfo pos=(%d, %d) mm imu.fault=%u  tx=[%02x %02x %02x %02x %02x %02x %02x %02x]\n",
           info[0].pos_x, info[0].pos_y, info[0].imu_fault, tx[0], tx[1], tx[2], tx[3], tx[4], tx[5],
           tx[6], tx[7]);
    if (records)
      printf("fleet (%d rank%s): %d ensemble records, last mean x=%.6f m th=%.6f rad, var x=%.3e, %.0f robots in "
             "%u records\n",
             world, world > 1 ? "s" : "", records, mean[0], mean[2], cov[0], counted, folded);
    // MOTOR_IF_M2006::get_status_latest of robot 0's front-left wheel
    std::vector<int16_t> mus(n * 4), ang(n * 4);
    std::vector<float> dlt(n * 4), spd(n * 4);
    motors.get_status_latest(mus.data(), ang.data(), nullptr, nullptr, dlt.data(), spd.data());
    printf("robot 0 FL: microsec_id=%d angle=%d dlt=%.7e rad speed=%.4f rad/s\n", mus[0], ang[0], dlt[0], spd[0]);
  } catch (const std::exception &e) {
    fprintf(stderr, "fleet_loop: %s\n", e.what());
    return 1;
  }
  return 0;
}
