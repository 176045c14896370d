// kernels_ingest.hip -- device boundary ingest kernels for gfx950.
//
//  k_wt901: one IMU per lane.  The WIT SDK byte state machine (lib/wt901c/wit_c_sdk.c:
//           132-198, NORMAL protocol) with its lazy one-byte-per-arrival resync, the
//           register file sReg (wit_c_sdk.c:13, per instance, SoA int16 planes), the
//           update-flag callback (imu_if_wt901c.cpp:23-48), isComComp (:132-143) and
//           updateData (:91-129).  Integer parts bit exact; the parser window (never
//           more than 11 bytes in NORMAL mode) is held in two 64-bit registers and
//           shifted, so no per-lane dynamic indexing (no scratch).
//  k_can4 / k_can: one robot per lane (every wheel present), or one wheel per lane (a
//           `present` mask).  MOTOR_IF_M2006::rx_callback
//           (VD_motor_if_m2006.cpp:32-72): big-endian decode, reversed motors, 13-bit
//           angle unwrap into the int64 sum, and the speed path with Cortex-M7 integer
//           semantics (wrapping MUL, SDIV x/0 = 0) and its IIR1 low-pass.
#include "fmskf_device.hpp"
#include "fmskf_internal.hpp"
#include "kf_generic.hpp"
#include "can_lane.hpp"

#pragma clang fp contract(off)

namespace fmskf {

// lib/wt901c/REG.h
enum : uint32_t {
  R_VERSION = 0x2e, R_YYMM = 0x30, R_AX = 0x34, R_AZ = 0x36, R_GX = 0x37, R_GZ = 0x39, R_HX = 0x3a,
  R_HZ = 0x3c, R_ROLL = 0x3d, R_YAW = 0x3f, R_TEMP = 0x40, R_D0STATUS = 0x41, R_PRESSUREL = 0x45,
  R_LONL = 0x49, R_GPSHEIGHT = 0x4d, R_Q0 = 0x51, R_Q3 = 0x54, R_SVNUM = 0x55
};
// imu_if_wt901c.cpp:10-15
enum : uint32_t { F_ACC = 0x01, F_GYRO = 0x02, F_ANGLE = 0x04, F_MAG = 0x08, F_QUAT = 0x10, F_READ = 0x80 };
// not a firmware flag (round 6): the robot's row-resident registers -- AX AY AZ GX GY Roll Pitch
// Q0-Q3, the eleven words the snapshot row holds besides the magnetometer's, and GZ and Yaw, the
// two words of its imu_yg dword -- live there, and their sReg planes are behind (the standard
// poll writes them once, into the row and the dword).  Any other poll, fmskf_get_imu_regs and a
// checkpoint write them back first (row_regs_out).
enum : uint32_t { F_ROWREGS = 0x40 };
// not a firmware flag either (round 6): the snapshot's magnetometer words are DevState::imu_mag's,
// since a poll after the last successful one wrote HX-HZ (it saved their earlier values there);
// otherwise they are sReg's (a standard poll carries no magnetometer frame, so its snapshot
// takes the registers as they are, and neither reads nor writes them)
enum : uint32_t { F_MAGDET = 0x20 };
// bit k of a register's row-resident index (AX AY AZ GX GY Roll Pitch Q0-Q3 -> 0..10, GZ 11,
// Yaw 12), or for HX-HZ bits 13-15 (not row-resident: a poll that writes them), or 0
__device__ __forceinline__ uint32_t rowreg_bit(uint32_t r) {
  return r >= R_AX && r < R_GZ ? 1u << (r - R_AX)
         : r == R_ROLL || r == R_ROLL + 1 ? 1u << (5 + r - R_ROLL)
         : r >= R_Q0 && r <= R_Q3 ? 1u << (7 + r - R_Q0)
         : r == R_GZ ? 1u << 11 : r == R_YAW ? 1u << 12
         : r >= R_HX && r <= R_HZ ? 1u << (13 + r - R_HX) : 0u;
}
// the row-resident registers (snapshot-row words 0-10, then the imu_yg dword's GZ and Yaw)
// written back to sReg, except those in `skip` (rowreg_bit mask: registers written since)
__device__ __forceinline__ void row_regs_out(const int16_t *snap, const uint32_t *yg, int16_t *reg, uint64_t n,
                                             uint64_t i, uint32_t skip = 0) {
  uint32_t w[6];  // word k in w[k / 2]
  snap_row_load(snap, i, w);
  // (register, snapshot word) of the eleven, in rowreg_bit order
  constexpr uint32_t kReg[11] = {R_AX, R_AX + 1, R_AX + 2, R_GX, R_GX + 1, R_ROLL, R_ROLL + 1,
                                 R_Q0, R_Q0 + 1, R_Q0 + 2, R_Q0 + 3};
  constexpr int kWord[11] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
#pragma unroll
  for (int k = 0; k < 11; k++) {
    const uint32_t v = w[kWord[k] / 2];
    if (!((skip >> k) & 1u)) reg[kReg[k] * n + i] = (int16_t)(kWord[k] & 1 ? v >> 16 : v & 0xFFFFu);
  }
  const uint32_t g = yg[i];
  if (!((skip >> 11) & 1u)) reg[R_GZ * n + i] = (int16_t)(g >> 16);
  if (!((skip >> 12) & 1u)) reg[R_YAW * n + i] = (int16_t)(g & 0xFFFFu);
}

// SensorDataUpdata for registers [r0, r0 + len)
__device__ __forceinline__ uint32_t flags_of(uint32_t r0, uint32_t len) {
  uint32_t f = 0;
  for (uint32_t k = 0; k < len; k++) {
    const uint32_t r = r0 + k;
    f |= r == R_AZ ? F_ACC : r == R_GZ ? F_GYRO : r == R_HZ ? F_MAG : r == R_YAW ? F_ANGLE
       : r == R_Q3 ? F_QUAT : F_READ;
  }
  return f;
}

struct Wt901Args {
  uint64_t n;
  const uint8_t *bytes;
  uint32_t stride;
  const uint32_t *len;
  int latch_qinit;
  uint32_t read_reg_index;
  int16_t *reg;
  uint32_t *parser;
  uint8_t *cnt;
  uint8_t *flags;
  uint8_t *err;
  float *qinit;
  int16_t *snap;  // [N][12] snapshot rows (fmskf_device.hpp snap_row_load)
  int16_t *mag;   // [N][4] the snapshot's HX-HZ while F_MAGDET
  uint32_t *yg;   // [N] Yaw / GZ words of the snapshot (DevState::imu_yg)
  float *qprev;
};

// One byte through WitSerialDataIn (wit_c_sdk.c:132-198): append to the window, resync by
// one byte on a bad header or checksum, dispatch a complete 11-byte frame to CopeWitData.
struct Wt901Parser {
  uint64_t lo, hi;
  uint32_t cnt, flags;
  uint32_t roww;  // rowreg_bit mask of the row-resident registers this poll's frames wrote
  // CopeWitData on a validated 11-byte window (bytes 0-7 in w0, 8-10 in w1)
  __device__ __forceinline__ void dispatch(uint64_t w0, uint64_t w1, const Wt901Args &a, uint64_t i) {
    const uint64_t n = a.n;
    int16_t *reg = a.reg;
    const uint64_t lo = w0, hi = w1;
    // CopeWitData(type, usData, 4), wit_c_sdk.c:90-130
    const uint32_t type = (uint32_t)(lo >> 8) & 0xFFu;
    const uint32_t d[4] = {(uint32_t)(lo >> 16) & 0xFFFFu, (uint32_t)(lo >> 32) & 0xFFFFu,
                           (uint32_t)(lo >> 48) & 0xFFFFu, (uint32_t)hi & 0xFFFFu};
    uint32_t reg1 = 0, len1 = 4, reg2 = 0, len2 = 0;
    bool known = true;
    switch (type) {
      case 0x51: reg1 = R_AX; len1 = 3; reg2 = R_TEMP; len2 = 1; break;
      case 0x53: reg1 = R_ROLL; len1 = 3; reg2 = R_VERSION; len2 = 1; break;
      case 0x50: reg1 = R_YYMM; break;
      case 0x52: reg1 = R_GX; len1 = 3; break;
      case 0x54: reg1 = R_HX; len1 = 3; break;
      case 0x55: reg1 = R_D0STATUS; break;
      case 0x56: reg1 = R_PRESSUREL; break;
      case 0x57: reg1 = R_LONL; break;
      case 0x58: reg1 = R_GPSHEIGHT; break;
      case 0x59: reg1 = R_Q0; break;
      case 0x5A: reg1 = R_SVNUM; break;
      case 0x5F: reg1 = a.read_reg_index; break;
      default: known = false; break;
    }
    if (known) {
      for (uint32_t k = 0; k < len1; k++) {
        reg[(reg1 + k) * n + i] = (int16_t)d[k];
        roww |= rowreg_bit(reg1 + k);
      }
      flags |= flags_of(reg1, len1);
      if (len2) {
        reg[reg2 * n + i] = (int16_t)d[3];
        flags |= flags_of(reg2, 1);
      }
    }
  }

  __device__ __forceinline__ void byte(uint32_t bv, const Wt901Args &a, uint64_t i) {
    const uint64_t byte = bv;
    // s_ucWitDataBuff[s_uiWitDataCnt++] = ucData  (bytes >= cnt are kept zero)
    if (cnt < 8) lo |= byte << (8 * cnt);
    else hi |= byte << (8 * (cnt - 8));
    cnt++;
    bool drop = (lo & 0xFFu) != 0x55u;  // header check, wit_c_sdk.c:142-147
    if (!drop && cnt >= 11) {
      uint32_t sum = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) sum += (uint32_t)(lo >> (8 * k)) & 0xFFu;
      sum += (uint32_t)hi & 0xFFu;
      sum += (uint32_t)(hi >> 8) & 0xFFu;
      drop = (sum & 0xFFu) != ((uint32_t)(hi >> 16) & 0xFFu);  // __CaliSum, :150-156
      if (!drop) {
        dispatch(lo, hi, a, i);
        cnt = 0;
        lo = 0;
        hi = 0;
        return;
      }
    }
    if (drop) {
      // s_uiWitDataCnt--; memcpy(buf, &buf[1], cnt)
      cnt--;
      lo = (lo >> 8) | (hi << 56);
      hi >>= 8;
    }
  }
};

// VEC: the poll buffer rows are 16-byte aligned and at most 64 bytes (the 44-byte standard
// poll in a 48-byte row): the lane's whole row is fetched with up to four 16-byte loads
// issued before any byte is parsed, instead of one dependent byte load per parser step.
// One IMU per lane.  Measured and not kept (round 3, kbench at 2^20 standard polls, one box
// each): two IMUs per lane with the second one's parser state and poll row loaded before the
// first is parsed (as k_kf6p does), 38.1 us against 34.9; the register file as pair planes
// (registers 2k, 2k + 1 in one dword, so 5 of the poll's 15 register stores become dword
// pairs), 38.7-38.9 against 35-36: the remaining single-register stores then half-fill the
// lines they touch; the magnetometer / q_init loads issued with the poll instead of after the
// parse, neutral.  Round 4 (kbench at 2^20 standard polls, two passes each on one box, against
// 34.9-35.3 us for this kernel): when every lane of a full wave took the standard poll, staging
// its 15 registers and 16 Data-page floats in LDS and storing them transposed (each lane 16
// contiguous bytes of one plane, 7 store instructions per wave instead of 37) measured
// 35.8-35.9 us with a block barrier and 35.4-35.7 with wave-local ordering; fetching the
// wave's poll rows as contiguous 1 KiB runs through LDS as well, 36.9-37.0; forcing 8 waves
// per SIMD (64 VGPRs, 20 B of scratch), 37.2; 24 / 32 KiB occupancy caps, 34.6-36.6.  The
// narrow stores are not what bounds the kernel, and none of these was kept.  Nor the KF6 tick's
// cache policies through buffer descriptors (same box, against 35.4-36.9 plain): `sc1` state
// stores 36.0-36.3; `nt` poll-row loads 41.2-42.0, since a 16-byte load of 48-byte rows uses a
// third of every line it touches and `nt` evicts the line before the next load reads the rest.
// Occupancy (round 5): the kernel that loaded the magnetometer registers after parsing took 67
// VGPRs, 7 waves per SIMD; capped at 64 (8 waves, no spills) it ran 29.2 -> 27.2 us per 2^20
// polls.  With every unconditional load hoisted ahead of the parse (below) it takes 74 VGPRs:
// 6 waves per SIMD, 27.0-27.2 -> 26.2-26.5 us at 2^20, 115.6-116.6 -> 109.9-110.6 at 2^22
// (kbench, three passes, profiles/r5_ab.json); capped at 7 or 8 waves it spills (29.4, 34.8 us).
// Round 6, the bytes read from the chunk registers where used (62 VGPRs, 103 SGPRs: 7 waves per
// SIMD): 6 here (7 waves) against 8 (63 VGPRs, 78 SGPRs, 8 waves) 21.3 / 21.3-21.6 us at 2^20,
// 84.3 / 86.4 at 2^22 (two passes, one box); with the 88-byte poll (54 VGPRs) 17.7-17.8 / 17.9-18.0 us
// at 2^20, 65.0-65.1 / 65.3-65.6 at 2^22 (three passes, profiles/r6_ab.json `wt901_wpe_after_row_split`)
#ifndef FMSKF_WT901_WPE
#define FMSKF_WT901_WPE 6
#endif
template <bool VEC>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FMSKF_WT901_WPE, 8))) void k_wt901(Wt901Args a) {
  const uint64_t n = a.n;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Wt901Parser ps;
  const uint8_t *p = a.bytes + i * (uint64_t)a.stride;
  // Every unconditional load first -- the count, flags, length and the poll row -- so a wave
  // waits for memory once before parsing (the parser words, read only when bytes are pending, and
  // a non-standard poll's register reads come after)
  const uint32_t cnt_in = a.cnt[i];
  const uint32_t flags_in = a.flags[i];
  const uint32_t len_in = a.len[i];
  int16_t *reg = a.reg;
  // the magnetometer registers before this poll: a poll that is not the standard one may write
  // them and fail, and the snapshot must then keep these (F_MAGDET; read before its frames land)
  int16_t rm[3] = {0, 0, 0};
  const auto load_mag = [&] {
#pragma unroll
    for (int k = 0; k < 3; k++) rm[k] = reg[(R_HX + k) * n + i];
  };
  uint4 ch[4];
  if constexpr (VEC) {
    const uint32_t nch = (a.stride + 15) / 16;  // <= 4, wave-uniform
#pragma unroll
    for (int c = 0; c < 4; c++)
      ch[c] = (uint32_t)c < nch ? reinterpret_cast<const uint4 *>(p)[c] : make_uint4(0, 0, 0, 0);
  }
  // The parser window holds exactly cnt bytes and is zero past them, so an empty window (the
  // state every poll of whole frames leaves) is all zero: its three words are read only when
  // bytes are pending, and written only when a window was or is now pending (round 5: the
  // standard poll moves 132 B instead of 157).
  ps.cnt = cnt_in;
  ps.lo = 0;
  ps.hi = 0;
  ps.roww = 0;
  if (cnt_in != 0) {
    ps.lo = (uint64_t)a.parser[i] | ((uint64_t)a.parser[n + i] << 32);
    ps.hi = (uint64_t)a.parser[2 * n + i];
  }
  ps.flags = flags_in & ~(F_ROWREGS | F_MAGDET);  // the firmware's update flags
  const bool row_regs = (flags_in & F_ROWREGS) != 0;
  const uint32_t len = len_in < a.stride ? len_in : a.stride;
  // the standard 10 ms poll (0x51 acc, 0x52 gyro, 0x53 angle, 0x59 quaternion)
  // taken by the fast path: every register updateData reads except the magnetometer's was
  // written by exactly one of its frames, so the Data page is built from the frame words
  // instead of reading the register file back
  bool std4 = false;
  // byte o (a compile-time offset) of the poll row, from the chunk registers
  const auto rb = [&](int o) -> uint32_t {
    if (o >= 64) return 0u;
    const uint4 c = ch[o / 16];
    const uint32_t w = (o % 16) / 4 == 0 ? c.x : (o % 16) / 4 == 1 ? c.y : (o % 16) / 4 == 2 ? c.z : c.w;
    return (w >> (8 * (o % 4))) & 0xFFu;
  };
  // data word k of frame f (CopeWitData's usData[k]: bytes 2 + 2k, 3 + 2k, little-endian)
  const auto fw = [&](int f, int k) -> uint32_t { return rb(f * 11 + 2 + 2 * k) | (rb(f * 11 + 3 + 2 * k) << 8); };
  if constexpr (VEC) {
    // Whole-frame fast path.  With an empty parser window and a poll made of complete frames
    // (0x55 header and a valid checksum every 11 bytes), the byte-serial parser accepts frame
    // k at bytes 11k..11k+10 and never resyncs: dispatch the frames directly (static byte
    // offsets -> register selects).  Anything else takes the byte-serial path from the start.
    // Every byte is taken from the chunk registers where it is used (round 6: the frames were
    // first copied into ten 64-bit window registers; 75 -> 62 VGPRs, 22.4 -> 21.3 us per 2^20
    // standard polls, 90.6 -> 84.3 at 2^22, profiles/r6_ab.json `wt901_chunk_bytes`)
    const uint32_t nfr = len / 11;
    bool fast = ps.cnt == 0 && len == nfr * 11 && len <= 55;
#pragma unroll
    for (int f = 0; f < 5; f++) {
      uint32_t sum = 0;
#pragma unroll
      for (int k = 0; k < 10; k++) sum += rb(f * 11 + k);
      const bool ok = rb(f * 11) == 0x55u && (sum & 0xFFu) == rb(f * 11 + 10);
      if ((uint32_t)f < nfr) fast = fast && ok;
    }
    std4 = fast && nfr == 4 && rb(1) == 0x51u && rb(12) == 0x52u && rb(23) == 0x53u && rb(34) == 0x59u;
    if (!std4) load_mag();
    if (std4) {
      // CopeWitData of the four frames with their register runs known statically.  Round 6: of
      // the 15 registers the four frames write, thirteen are written once (F_ROWREGS): AX AY AZ
      // GX GY Roll Pitch Q0-Q3 into the snapshot row, GZ and Yaw into the imu_yg dword (below);
      // TEMP and VERSION go to sReg
      int16_t *reg = a.reg;
      reg[R_TEMP * n + i] = (int16_t)fw(0, 3);
      reg[R_VERSION * n + i] = (int16_t)fw(2, 3);
      ps.flags |= flags_of(R_AX, 3) | flags_of(R_TEMP, 1) | flags_of(R_GX, 3) | flags_of(R_ROLL, 3) |
                  flags_of(R_VERSION, 1) | flags_of(R_Q0, 4);
    } else if (fast) {
#pragma unroll
      for (int f = 0; f < 5; f++)
        if ((uint32_t)f < nfr) {
          uint64_t w0 = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) w0 |= (uint64_t)rb(f * 11 + k) << (8 * k);
          const uint64_t w1 = (uint64_t)rb(f * 11 + 8) | ((uint64_t)rb(f * 11 + 9) << 8) | ((uint64_t)rb(f * 11 + 10) << 16);
          ps.dispatch(w0, w1, a, i);
        }
    } else {
    // one parser body: the next chunk's bytes are consumed from the bottom of a 128-bit
    // shift register
#pragma unroll 1
    for (uint32_t c = 0; c * 16 < len; c++) {
      uint4 cur = ch[0];  // chunks advance by register moves, never a dynamic index
      ch[0] = ch[1];
      ch[1] = ch[2];
      ch[2] = ch[3];
      const uint32_t lim = len - c * 16 < 16 ? len - c * 16 : 16;
#pragma unroll 1
      for (uint32_t j = 0; j < lim; j++) {
        ps.byte(cur.x & 0xFFu, a, i);
        cur.x = (cur.x >> 8) | (cur.y << 24);
        cur.y = (cur.y >> 8) | (cur.z << 24);
        cur.z = (cur.z >> 8) | (cur.w << 24);
        cur.w >>= 8;
      }
    }
    }
  } else {
    load_mag();
    for (uint32_t b = 0; b < len; b++) ps.byte(p[b], a, i);
  }
  // any other poll worked on the register file itself: the row-resident registers its frames did
  // not write are brought back from the row now (after the parse, when the poll row's registers
  // are dead; frames only write registers, so the order is immaterial).  Rare: a damaged or
  // non-standard poll
  if (!std4 && row_regs) row_regs_out(a.snap, a.yg, a.reg, n, i, ps.roww);
  uint64_t lo = ps.lo, hi = ps.hi;
  uint32_t cnt = ps.cnt, flags = ps.flags;
  // isComComp / update, imu_if_wt901c.cpp:83-89,132-143
  const bool ok = (flags & F_QUAT) != 0;
  if (ok) flags = 0;
  a.err[i] = ok ? 0 : 1;
  // the standard poll (always a successful one) leaves its row-resident registers in the row
  if (std4) flags |= F_ROWREGS;
  // a successful poll's snapshot takes the magnetometer registers as they are (F_MAGDET clear);
  // after a failed one that wrote them the snapshot's are the ones before, kept in imu_mag (once:
  // if they were detached already, imu_mag holds the snapshot's)
  if (!ok) {
    if (flags_in & F_MAGDET) {
      flags |= F_MAGDET;
    } else if ((ps.roww >> 13) & 7u) {
      reinterpret_cast<uint2 *>(a.mag)[i] = make_uint2((uint32_t)(uint16_t)rm[0] | ((uint32_t)(uint16_t)rm[1] << 16),
                                                       (uint32_t)(uint16_t)rm[2]);
      flags |= F_MAGDET;
    }
  }
  if (cnt_in != 0 || cnt != 0) {
    a.parser[i] = (uint32_t)lo;
    a.parser[n + i] = (uint32_t)(lo >> 32);
    a.parser[2 * n + i] = (uint32_t)hi;
    a.cnt[i] = (uint8_t)cnt;
  }
  a.flags[i] = (uint8_t)flags;
  if (!ok) return;
  // updateData, imu_if_wt901c.cpp:91-129: the page is not formed here.  Its 16 words are kept
  // (the snapshot row: 24 bytes, three 8-byte stores -- round 6: the magnetometer's stay in sReg --
  // and the Yaw / GZ words the tick reads);
  // fmskf_get_imu and VehicleInfo form the page from them (imu_data_page), so a poll moves 157 B
  // instead of 197 (the 64-byte page written, q_init read; 132 B with the empty-window rule above).  Only a latching poll reads q_init,
  // to keep it (qprev) for the page of that very poll, which used the old one.
  int16_t ra[3], rg[3], rr[3], rq[4];
  if (std4) {  // (VEC only: the chunk registers still hold the poll)
#pragma unroll
    for (int k = 0; k < 3; k++) {
      ra[k] = (int16_t)fw(0, k);
      rg[k] = (int16_t)fw(1, k);
      rr[k] = (int16_t)fw(2, k);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) rq[k] = (int16_t)fw(3, k);
  } else {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      ra[k] = reg[(R_AX + k) * n + i];
      rg[k] = reg[(R_GX + k) * n + i];
      rr[k] = reg[(R_ROLL + k) * n + i];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) rq[k] = reg[(R_Q0 + k) * n + i];
  }
  // Data.angle[2] / Data.gyro[2] as their register words (fmskf_device.hpp imu_yaw_deg)
  a.yg[i] = (uint32_t)(uint16_t)rr[2] | ((uint32_t)(uint16_t)rg[2] << 16);
  uint32_t snapf = kSnapValid;
  if (a.latch_qinit) {
    snapf |= kSnapLatched;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      a.qprev[k * n + i] = a.qinit[k * n + i];
      a.qinit[k * n + i] = (float)rq[k] / 32768.0f;
    }
  }
  const auto u = [](int16_t lo, int16_t hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); };
  uint2 *row = reinterpret_cast<uint2 *>(a.snap + (uint64_t)kRowWords * i);  // fmskf_device.hpp snap_row_load
  row[0] = make_uint2(u(ra[0], ra[1]), u(ra[2], rg[0]));
  row[1] = make_uint2(u(rg[1], rr[0]), u(rr[1], rq[0]));
  row[2] = make_uint2(u(rq[1], rq[2]), u(rq[3], (int16_t)snapf));
}

// the register file made whole (fmskf_get_imu_regs, a checkpoint): robots whose row-resident
// registers live in their snapshot row (F_ROWREGS) get them written back into sReg
__global__ __launch_bounds__(kBlock) void k_wt901_regs_sync(const int16_t *snap, const uint32_t *yg, int16_t *reg,
                                                            uint8_t *flags, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = flags[i];
  if (!(f & F_ROWREGS)) return;
  row_regs_out(snap, yg, reg, n, i);
  flags[i] = (uint8_t)(f & ~F_ROWREGS);
}

int launch_wt901_regs_sync(const DevState &s, hipStream_t st) {
  if (s.n == 0 || !s.imu_reg) return 0;
  k_wt901_regs_sync<<<dim3((unsigned)((s.n + kBlock - 1) / kBlock)), kBlock, 0, st>>>(s.imu_snap, s.imu_yg,
                                                                                      s.imu_reg, s.imu_flags, s.n);
  return (int)hipGetLastError();
}

// IMU_IF::Data [16][N] of every robot from its snapshot (fmskf_get_imu): zeros until the first
// successful poll, like the firmware's zero-initialised page
__global__ __launch_bounds__(kBlock) void k_imu_data(const int16_t *snap, const int16_t *mag, const int16_t *reg,
                                                     const uint8_t *flags, const uint32_t *yg, const float *qinit,
                                                     const float *qprev, uint64_t n, float *out) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint32_t rw[6];
  snap_row_load(snap, i, rw);
  // the snapshot's magnetometer: sReg's, or the ones a later failed poll displaced (F_MAGDET)
  int16_t hm[3];
  if (flags[i] & F_MAGDET) {
    const uint2 m = reinterpret_cast<const uint2 *>(mag)[i];
    hm[0] = (int16_t)(m.x & 0xFFFFu);
    hm[1] = (int16_t)(m.x >> 16);
    hm[2] = (int16_t)(m.y & 0xFFFFu);
  } else {
#pragma unroll
    for (int k = 0; k < 3; k++) hm[k] = reg[(R_HX + k) * n + i];
  }
  int16_t w[kSnapWords];
  snap_page_words(rw, hm[0], hm[1], hm[2], w);
  float d[16];
  if (w[14] & kSnapValid) {
    const float *q = (w[14] & kSnapLatched) ? qprev : qinit;
    const float qi[4] = {q[i], q[n + i], q[2 * n + i], q[3 * n + i]};
    const uint32_t g = yg[i];
    imu_data_page(w, imu_yaw_deg(g), imu_gz_dps(g), qi, d);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = 0.0f;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) out[k * n + i] = d[k];
}

int launch_imu_data(const DevState &s, float *out, hipStream_t st) {
  if (s.n == 0) return 0;
  k_imu_data<<<dim3((unsigned)((s.n + kBlock - 1) / kBlock)), kBlock, 0, st>>>(s.imu_snap, s.imu_mag, s.imu_reg,
                                                                                s.imu_flags, s.imu_yg, s.imu_qinit,
                                                                                s.imu_qprev, s.n, out);
  return (int)hipGetLastError();
}

int launch_wt901(const DevState &s, const uint8_t *bytes, uint32_t stride, const uint32_t *len,
                 int latch_qinit, uint32_t read_reg_index, hipStream_t st) {
  Wt901Args a{s.n,       bytes,      stride,   len,        latch_qinit,  read_reg_index, s.imu_reg,
              s.imu_parser, s.imu_cnt, s.imu_flags, s.imu_err, s.imu_qinit, s.imu_snap, s.imu_mag,
              s.imu_yg,    s.imu_qprev};
  const dim3 g((unsigned)((s.n + kBlock - 1) / kBlock));
  const bool vec = stride % 16 == 0 && stride <= 64 && ((uintptr_t)bytes & 15) == 0;
  if (vec) k_wt901<true><<<g, kBlock, 0, st>>>(a);
  else k_wt901<false><<<g, kBlock, 0, st>>>(a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// CAN: MOTOR_IF_M2006::rx_callback
// ---------------------------------------------------------------------------
__device__ __forceinline__ void can_lane(const CanArgs &a, uint64_t n, uint64_t g) {
  const uint64_t i = g >> 2;
  const int w = (int)(g & 3);
  if (a.present && !((a.present[i] >> w) & 1)) {
    // no frame: the wheel's state stays, so its two history slots trade places with the order
    // the host flips for every wheel (DevState::m_par)
    const int16_t m0 = a.micro[g], m1 = a.prev_micro[g], a0 = a.angle[g], a1 = a.prev[g];
    a.micro[g] = m1;
    a.prev_micro[g] = m0;
    a.angle[g] = a1;
    a.prev[g] = a0;
    return;
  }
  const uint2 f = reinterpret_cast<const uint2 *>(a.frames)[g];
  const CanWheel o = can_wheel(f.x, f.y, a.stamps[g], a.dir[w], a.micro[g], a.angle[g], a.prev_micro[g],
                               a.prev[g], a.iir_y[g]);
  a.iir_y[g] = o.iir_y;
  int32_t cy;
  a.sum_lo[g] = sum_add(a.sum_lo[g], o.d, cy);
  if (cy != 0) a.sum_hi[g] += cy;
  a.prev_micro[g] = a.stamps[g];  // over the older slots (DevState::m_par)
  a.prev[g] = o.angle;
  a.rpm[g] = o.rpm;
  a.curr[g] = o.curr;
}

// one wheel per lane: any `present` mask (absent wheels keep their state).  Grid-stride: 4 N
// lanes reach 2^32 at the 2^30-robot cap, past one dispatch's 32-bit grid size
__global__ __launch_bounds__(kBlock) void k_can(CanArgs a) {
  const uint64_t n = a.n;
  for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g < 4 * n;
       g += (uint64_t)gridDim.x * kBlock)  // (instance, wheel)
    can_lane(a, n, g);
}

// one robot per lane, every wheel present (no mask): the robot's 32 frame bytes, its four
// stamps and its [N][4] int16 / float / uint32 state in single 16- and 8-byte accesses (the
// per-wheel kernel moves 64 B half-lines: 2^20 57.4-57.7 -> 42.1-44.1 us, 2^22 232-239 -> 211).  Every access goes through a scalar
// descriptor at the block's 256-robot chunk with the KF6 tick's cache policies: the frames and
// stamps (read once) `nt`, the state stored `sc1` while cache-resident; NT: the motor state
// streams from HBM (past the Infinity Cache), `nt` loads and stores.  Plain global accesses
// measured 43.4-44.6 (2^20) and 191-195 us (2^22) against 43.0-43.1 and 185-189.
// Round 5: the IIR1 output state y of the four wheels as [N][4] floats, one 16-byte access (the
// [4][N] planes took 4 dword loads and stores per array: measured neutral, 39.3-41.0 against
// 40.0-40.1 us at 2^20, profiles/r5_kb_can_iir_ab.jsonl, issue-wait 0.78 either way), and the
// IIR1 state x formed again from the previous frame (can_wheel): 224 -> 216 B per robot.
// Round 6: the angle sums as their low words (one 16-byte access each way; the high words only on
// a carry): 216 -> 184 B per robot.
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_can4(CanArgs a) {
  extern __shared__ double occ_cap[];
  (void)occ_cap;
  const uint64_t n = a.n;
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint64_t hb = (uint64_t)(__builtin_amdgcn_readfirstlane((uint32_t)i) & ~(uint32_t)(kBlock - 1));
  Can4Lane<NT> L;
  L.load(a, hb, (uint32_t)(i - hb));
  (void)L.step(a, true);
  L.finish(a, true);
}

int launch_can(const DevState &s, const uint8_t *frames, const int16_t *stamps,
               const uint8_t *present, const int8_t dir[4], hipStream_t st) {
  CanArgs a{};
  a.n = s.n;
  a.frames = frames;
  a.stamps = stamps;
  a.present = present;
  for (int w = 0; w < 4; w++) a.dir[w] = dir[w];
  const MotorSlots ms = motor_slots(s);
  a.micro = ms.micro;
  a.angle = ms.angle;
  a.prev = ms.prev;
  a.rpm = s.m_rpm;
  a.curr = s.m_curr;
  a.sum_lo = s.m_sum_lo;
  a.sum_hi = s.m_sum_hi;
  a.iir_y = s.m_iir_y;
  a.prev_micro = ms.prev_micro;
  // every wheel present and the caller's frames / stamps aligned for the wide loads: one robot
  // per lane; a `present` mask or unaligned buffers: one wheel per lane
  if (!present && ((uintptr_t)frames & 15) == 0 && ((uintptr_t)stamps & 7) == 0) {
    const dim3 g((unsigned)((s.n + kBlock - 1) / kBlock));
    // 132 B of motor state per robot.  Non-temporal with 2 blocks per CU once it is well past
    // the Infinity Cache; measured (kbench, two passes): 2^22 plain 191.6-192.8 us, nt
    // 183.9-187.2, nt + 64 KiB cap 176.7-179.8; at 2^21 (277 MB) plain 83.3-85.1, nt 87.5-87.9
    // non-temporal once the motor state, the frames and the estimator state together outgrow
    // the Infinity Cache (can_nt, can_lane.hpp)
    if (can_nt(s)) {
      const unsigned lds = FMSKF_LDS_CAP("FMSKF_CAN_LDS", true, 64u * 1024u);
      k_can4<true><<<g, kBlock, lds, st>>>(a);
    } else {
      const unsigned lds = FMSKF_LDS_CAP("FMSKF_CAN_LDS", false, 0u);
      k_can4<false><<<g, kBlock, lds, st>>>(a);
    }
  } else {
    const uint64_t blocks = (4 * s.n + kBlock - 1) / kBlock;
    k_can<<<dim3((unsigned)(blocks < (1u << 22) ? blocks : (1u << 22))), kBlock, 0, st>>>(a);
  }
  return (int)hipGetLastError();
}

}  // namespace fmskf
