// api_checkpoint.cpp -- fmskf_save_state / fmskf_load_state: every per-robot device array
// of a handle in its device layout, with the layout recorded and a checksum.
#include "api_ctx.hpp"

using namespace fmskf;
using namespace fmskf::capi;

namespace {

// Checkpoint sections: every per-robot device array of the handle in its device layout (planes
// at the handle's pitch, tiles), byte for byte.  Groups: 1 estimator (x, P, RS prev sums,
// counters), 2 IMU ingest, 4 motor ingest, 8 control (state + parameters).
// Format 2 ('FMSKFCK2'): the header records every layout choice a section's bytes depend on
// (estimator pitch / tile / element size, the motor sums' pitch, the control arrays' tiling
// and pitch) and a checksum of everything after the header; a file whose layout differs from
// this build's, or from a format-1 file (which recorded none of the control / motor layout), is
// rejected instead of being loaded into a scrambled state.  Format 3 ('FMSKFCK3'): the motor
// group without the dlt and speed planes (no longer kept).  Format 4 ('FMSKFCK4', ABI 3): the
// motor group with the previous angles (Status::flt_dltOutAngle_rad at readout), the estimator
// group with KF6's position low parts under FMSKF_CFG_COMP_POS, and the config flags in the
// header; format-2 and format-3 files are rejected by name.  Format 5 ('FMSKFCK5', round 5):
// the motor group's IIR1 state as [N][4] rows (k_can4 moves each in one 16-byte access);
// format-4 files, whose IIR state is [4][N] planes, are rejected by name.
constexpr char kCkMagic[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '5'};
constexpr char kCkMagicV4[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '4'};
constexpr char kCkMagicV3[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '3'};
constexpr char kCkMagicV1[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '1'};
constexpr char kCkMagicV2[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '2'};
struct CkHeader {
  char magic[8];
  uint32_t abi, model;
  uint64_t n, pitch;
  uint32_t tile, elem, groups, ctrl_tile;  // ctrl_tile: control arrays' tile width (0 = planar)
  uint64_t m_pitch, ctrl_pitch;            // (round 5: the motor sum planes' pitch), control state's pitch
  uint64_t body_bytes, checksum;           // what follows the header, and its hash
  uint32_t flags;                          // fmskf_config.flags (FMSKF_CFG_*)
  // layout bits of format 5 (0 in round-5 files), so a round-5 file is refused instead of loaded
  // scrambled: bit 0, the RS previous sums in 64-robot tiles of wheel pairs (round 6, lane_rs.hpp
  // rs_prev_at; [4][pitch] planes before); bit 1, the motor group's angle sums as split low /
  // high words (round 6, fmskf_internal.hpp m_sum_lo; int64 [4][pitch] planes before); bit 2, the
  // IMU group's yaw / gyro z as the Yaw / GZ register words (round 6, DevState::imu_yg; two float
  // planes before); bit 3, the control group's rpm of the last step (round 6, CtrlDev::rpm_prev);
  // bit 4, the IMU snapshot as 12-word rows plus the detached magnetometer (round 6, kRowWords)
  uint32_t layout;
};
constexpr uint32_t kCkPrevRows = 1u, kCkSumSplit = 2u, kCkImuYg = 4u, kCkRpmPrev = 8u, kCkImuRow = 16u;
struct CkSection {
  void *dev;
  size_t bytes;
};
std::vector<CkSection> ck_sections(fmskf_ctx *h, uint32_t groups) {
  DevState &s = h->s;
  const uint64_t n = s.n, pp = s.pitch;
  const Dims d = h->d;
  std::vector<CkSection> v;
  if (groups & 1) {
    v.push_back({s.x, (size_t)d.nx * pp * d.elem});
    if (s.P) v.push_back({s.P, (size_t)d.nx * (d.nx + 1) / 2 * pp * d.elem});
    if (s.prev_sum) v.push_back({s.prev_sum, (size_t)4 * pp * 8});
    if (s.thlo) v.push_back({s.thlo, (size_t)n * 4});
    if (s.xlo) v.push_back({s.xlo, (size_t)kKf6LoRows * s.pitch * 4});
    v.push_back({s.counters, 8 * 8});
  }
  if (groups & 2) {
    v.push_back({s.imu_reg, (size_t)0x90 * n * 2});
    v.push_back({s.imu_parser, (size_t)3 * n * 4});
    v.push_back({s.imu_cnt, (size_t)n});
    v.push_back({s.imu_flags, (size_t)n});
    v.push_back({s.imu_err, (size_t)n});
    v.push_back({s.imu_qinit, (size_t)4 * n * 4});
    v.push_back({s.imu_snap, (size_t)kRowWords * n * 2});
    v.push_back({s.imu_mag, (size_t)4 * n * 2});
    v.push_back({s.imu_yg, (size_t)n * 4});
    v.push_back({s.imu_qprev, (size_t)4 * n * 4});
  }
  if (groups & 4) {
    const MotorSlots ms = motor_slots(s);  // newest first, whichever slots hold them (DevState::m_par)
    for (void *p : {(void *)ms.micro, (void *)ms.angle, (void *)ms.prev, (void *)ms.prev_micro,
                    (void *)s.m_rpm, (void *)s.m_curr})
      v.push_back({p, (size_t)4 * n * 2});
    v.push_back({s.m_sum_lo, (size_t)4 * n * 4});
    v.push_back({s.m_sum_hi, (size_t)4 * n * 4});
    v.push_back({s.m_iir_y, (size_t)4 * n * 4});
  }
  if (groups & 8) {
    const CtrlDev &c = h->ctrl;
    v.push_back({c.ax, (size_t)3 * kAxF * c.pitch * 4});
    v.push_back({c.pid, (size_t)4 * kPidF * c.pitch * 4});
    v.push_back({c.vel_tgt, (size_t)3 * c.pitch * 4});
    v.push_back({c.rpm_prev, (size_t)4 * c.n * 2});
    v.push_back({c.curr, (size_t)4 * c.n * 2});
    v.push_back({c.power, (size_t)c.n});
  }
  return v;
}

// the layout fields of a header for this handle (what ensure_motors / ensure_ctrl allocate)
void ck_layout(const fmskf_ctx *h, CkHeader *hd) {
  hd->abi = FMSKF_ABI_VERSION;
  hd->model = h->cfg.model;
  hd->flags = h->cfg.flags;
  hd->n = h->s.n;
  hd->pitch = h->s.pitch;
  hd->tile = h->s.tile;
  hd->elem = h->d.elem;
  hd->ctrl_tile = FMSKF_CTRL_TILED ? tile_w_elem(4) : 0;
  hd->m_pitch = plane_pitch(h->s.n);
  hd->layout = (h->s.prev_sum ? kCkPrevRows : 0u) | kCkSumSplit | kCkImuYg | kCkRpmPrev | kCkImuRow;
  const uint64_t w = tile_w_elem(4);
  hd->ctrl_pitch = FMSKF_CTRL_TILED ? std::max(h->s.pitch, (h->s.n + w - 1) / w * w) : h->s.pitch;
}

// 64-bit multiply-xor hash of a byte stream in 8-byte words (the tail zero-padded); the value
// does not depend on how the stream is split into add() calls
struct CkHash {
  uint64_t h = 0x9E3779B97F4A7C15ull, len = 0;
  unsigned char tail[8] = {};
  size_t nt = 0;
  static uint64_t mix(uint64_t h, uint64_t w) {
    h = (h ^ w) * 0x100000001B3ull;
    return h ^ (h >> 29);
  }
  void add(const char *p, size_t b) {
    len += b;
    while (nt && b) {  // finish a partial word first
      tail[nt++] = (unsigned char)*p++;
      b--;
      if (nt == 8) {
        uint64_t w;
        memcpy(&w, tail, 8);
        h = mix(h, w);
        nt = 0;
      }
    }
    size_t k = 0;
    for (; k + 8 <= b; k += 8) {
      uint64_t w;
      memcpy(&w, p + k, 8);
      h = mix(h, w);
    }
    for (; k < b; k++) tail[nt++] = (unsigned char)p[k];
  }
  uint64_t value() const {
    uint64_t r = h;
    if (nt) {
      uint64_t w = 0;
      memcpy(&w, tail, nt);
      r = mix(r, w);
    }
    return r ^ len;
  }
};

constexpr size_t kCkChunk = (size_t)64 << 20;  // host staging per copy: 64 MiB, a word multiple

struct File {
  FILE *f = nullptr;
  File(const char *path, const char *mode) : f(fopen(path, mode)) {
    if (!f) fail(FMSKF_EINVAL, std::string("cannot open ") + path);
  }
  ~File() {
    if (f) fclose(f);
  }
  void write(const void *p, size_t b) {
    if (fwrite(p, 1, b, f) != b) fail(FMSKF_EINVAL, "checkpoint write failed");
  }
  void read(void *p, size_t b) {
    if (fread(p, 1, b, f) != b) fail(FMSKF_EINVAL, "checkpoint truncated");
  }
  long tell() const { return ftell(f); }
  void seek(long off, int whence) {
    if (fseek(f, off, whence) != 0) fail(FMSKF_EINVAL, "checkpoint seek failed");
  }
};

}  // namespace

extern "C" {

int fmskf_save_state(fmskf_handle h, const char *path) {
  return guarded([&] {
    check_handle(h);
    if (!path) fail(FMSKF_EINVAL, "null path");
    if (h->capturing) fail(FMSKF_EINVAL, "capture open");
    DeviceGuard g(h->cfg.device);
    CkHeader hd{};
    memcpy(hd.magic, kCkMagic, 8);
    ck_layout(h, &hd);
    hd.groups = 1u | (h->s.imu_reg ? 2u : 0u) | (h->s.m_sum_lo ? 4u : 0u) | (h->ctrl_ready ? 8u : 0u);
    rs_prev_materialize(h);  // the file holds the odometry's previous sums in the prev planes
    ctrl_materialize(h);     // and the control step's outputs
    // and the whole WT901 register file in its planes (no row-resident registers)
    launch_check(launch_wt901_regs_sync(h->s, h->stream), "register file sync");
    hip_check(hipStreamSynchronize(h->stream), "save sync");
    File f(path, "wb");
    f.write(&hd, sizeof(hd));  // rewritten with the body size and checksum at the end
    CkHash hash;
    auto put = [&](const void *p, size_t b) {
      f.write(p, b);
      hash.add((const char *)p, b);
    };
    put(&h->cfg, sizeof(h->cfg));
    if (hd.groups & 8) put(&h->cprm, sizeof(h->cprm));
    std::vector<char> buf;
    for (const CkSection &c : ck_sections(h, hd.groups)) {
      const uint64_t b = c.bytes;
      put(&b, 8);
      for (size_t off = 0; off < c.bytes; off += kCkChunk) {  // bounded host memory
        const size_t len = std::min(kCkChunk, c.bytes - off);
        buf.resize(len);
        hip_check(hipMemcpy(buf.data(), (const char *)c.dev + off, len, hipMemcpyDeviceToHost), "save D2H");
        put(buf.data(), len);
      }
    }
    hd.body_bytes = hash.len;
    hd.checksum = hash.value();
    f.seek(0, SEEK_SET);
    f.write(&hd, sizeof(hd));
  });
}

int fmskf_load_state(fmskf_handle h, const char *path) {
  return guarded([&] {
    check_handle(h);
    if (!path) fail(FMSKF_EINVAL, "null path");
    if (h->capturing) fail(FMSKF_EINVAL, "capture open");
    DeviceGuard g(h->cfg.device);
    File f(path, "rb");
    CkHeader hd{};
    f.read(&hd.magic, 8);
    if (memcmp(hd.magic, kCkMagicV1, 8) == 0)
      fail(FMSKF_EINVAL, "format-1 checkpoint (older build): its control / motor layout is not recorded");
    if (memcmp(hd.magic, kCkMagicV2, 8) == 0)
      fail(FMSKF_EINVAL, "format-2 checkpoint (older build): its motor group holds the dlt / speed planes this build no longer keeps");
    if (memcmp(hd.magic, kCkMagicV3, 8) == 0)
      fail(FMSKF_EINVAL, "format-3 checkpoint (older build): its motor group lacks the previous angles");
    if (memcmp(hd.magic, kCkMagicV4, 8) == 0)
      fail(FMSKF_EINVAL, "format-4 checkpoint (older build): it keeps the IMU Data page and [4][N] motor IIR planes, this build the snapshot rows and [N][4] IIR rows");
    if (memcmp(hd.magic, kCkMagic, 8) != 0) fail(FMSKF_EINVAL, "not an fmskf checkpoint");
    f.seek(0, SEEK_SET);
    f.read(&hd, sizeof(hd));
    CkHeader me{};
    ck_layout(h, &me);
    if (hd.abi != me.abi || hd.model != me.model || hd.n != me.n || hd.pitch != me.pitch ||
        hd.tile != me.tile || hd.elem != me.elem || hd.flags != me.flags || (hd.groups & ~15u))
      fail(FMSKF_EINVAL, "checkpoint does not match this handle (ABI, model, flags, N or layout)");
    if ((hd.groups & 4) && hd.m_pitch != me.m_pitch) fail(FMSKF_EINVAL, "checkpoint motor layout differs");
    if (hd.layout != me.layout)
      fail(FMSKF_EINVAL, "checkpoint layout differs (an older file: int64 motor sum planes, RS previous sums as planes, IMU yaw / gyro z floats)");
    if ((hd.groups & 8) && (hd.ctrl_tile != me.ctrl_tile || hd.ctrl_pitch != me.ctrl_pitch))
      fail(FMSKF_EINVAL, "checkpoint control layout differs (tiling / pitch)");
    if (!(hd.groups & 1u)) fail(FMSKF_EINVAL, "checkpoint holds no estimator state");
    // pass 1: the body's length and checksum, read in bounded chunks -- a truncated, extended or
    // corrupted file is rejected before anything of the handle changes
    const long body = f.tell();
    f.seek(0, SEEK_END);
    if ((uint64_t)(f.tell() - body) != hd.body_bytes)
      fail(FMSKF_EINVAL, "checkpoint size mismatch (truncated or trailing bytes)");
    f.seek(body, SEEK_SET);
    std::vector<char> buf;
    {
      CkHash hash;
      for (uint64_t off = 0; off < hd.body_bytes; off += kCkChunk) {
        const size_t len = (size_t)std::min<uint64_t>(kCkChunk, hd.body_bytes - off);
        buf.resize(len);
        f.read(buf.data(), len);
        hash.add(buf.data(), len);
      }
      if (hash.value() != hd.checksum) fail(FMSKF_EINVAL, "checkpoint checksum mismatch");
    }
    f.seek(body, SEEK_SET);
    fmskf_config saved;
    f.read(&saved, sizeof(saved));
    fmskf_ctrl_params cp{};
    if (hd.groups & 8) f.read(&cp, sizeof(cp));
    if (hd.groups & 2) ensure_imu(h);
    if (hd.groups & 4) ensure_motors(h);
    if (hd.groups & 8) ensure_ctrl(h);
    const std::vector<CkSection> secs = ck_sections(h, hd.groups);
    // the section sizes follow from the (validated) layout; check them against the file's
    // before any copy
    const long first = f.tell();
    for (const CkSection &c : secs) {
      uint64_t b = 0;
      f.read(&b, 8);
      if (b != c.bytes) fail(FMSKF_EINVAL, "checkpoint section size mismatch");
      f.seek((long)c.bytes, SEEK_CUR);
    }
    f.seek(first, SEEK_SET);
    // groups the checkpoint does not hold were never used by the saving handle: reset them here
    if (!(hd.groups & 2) && h->s.imu_reg) zero_imu(h);
    if (!(hd.groups & 4) && h->s.m_sum_lo) zero_motors(h);
    if (!(hd.groups & 8) && h->ctrl_ready) zero_ctrl(h);
    h->rs_prev_synced = h->rs_prev_stale = false;  // the prev planes come from the file
    h->ctrl_derived_stale = false;                  // and the control outputs
    hip_check(hipStreamSynchronize(h->stream), "load sync");
    // pass 2: stream each section to the device in bounded chunks
    for (const CkSection &c : secs) {
      uint64_t b = 0;
      f.read(&b, 8);
      for (size_t off = 0; off < c.bytes; off += kCkChunk) {
        const size_t len = std::min(kCkChunk, c.bytes - off);
        buf.resize(len);
        f.read(buf.data(), len);
        hip_check(hipMemcpy((char *)c.dev + off, buf.data(), len, hipMemcpyHostToDevice), "load H2D");
      }
    }
    if (hd.groups & 8) h->cprm = cp;
    h->ens_shift_ok = false;
  });
}

}  // extern "C"
