// fmskf_api.cpp -- the C ABI (include/fmskf.h) over the HIP kernels.
//
// Owns the device SoA state of a handle, resolves NULL input planes to the
// device-resident ingest state (full pipeline), stages host inputs with async
// copies on the handle's stream, validates shapes, and converts every failure to
// a status code (no exception crosses the ABI).  No CPU fallback exists: every
// compute entry point launches a HIP kernel or fails with FMSKF_EDEVICE.
#include "../../include/fmskf.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "fmskf_internal.hpp"

using namespace fmskf;

namespace {

thread_local std::string g_last_error;

struct ApiError {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string &msg) { throw ApiError{code, msg}; }

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) fail(FMSKF_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
void launch_check(int e, const char *what) { hip_check((hipError_t)e, what); }

// The events the library records only to order its own work or to tell the host that the GPU
// is done with a pinned host buffer: no system-scope release.  That release writes back and
// invalidates the L2 behind each recorded event before the next kernel starts; the host reads
// nothing behind these events but pinned host memory that kernels and copies write over PCIe.
constexpr unsigned kSyncEvent = hipEventDisableTiming | hipEventDisableSystemFence;

template <class F>
int guarded(F &&f) {
  try {
    g_last_error.clear();
    f();
    return FMSKF_OK;
  } catch (const ApiError &e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::bad_alloc &) {
    g_last_error = "host allocation failed";
    return FMSKF_ENOMEM;
  } catch (...) {
    g_last_error = "unexpected exception";
    return FMSKF_EDEVICE;
  }
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

struct Dims {
  uint32_t nx, m, elem;
};

Dims dims_of(uint32_t model) {
  switch (model) {
    case FMSKF_MODEL_RS: return {6, 0, 4};
    case FMSKF_MODEL_KF6: return {6, 4, 4};
    case FMSKF_MODEL_EKF9: return {9, 6, 4};
    case FMSKF_MODEL_KF12D: return {12, 8, 8};
    default: fail(FMSKF_EINVAL, "unknown model");
  }
}

}  // namespace

struct fmskf_ctx {
  fmskf_config cfg{};
  Dims d{};
  DevState s{};
  hipStream_t stream = nullptr;
  std::vector<void *> allocs;
  // staging for host-resident inputs
  void *stage = nullptr;
  size_t stage_bytes = 0;
  // pinned host slots for small host-resident inputs and outputs: the planes of one call are
  // packed into a slot by the CPU and cross PCIe as one DMA (instead of one pageable copy per
  // plane); two input slots, each reused only after its event (the DMA that read it) completed
  static constexpr size_t kPinned = (size_t)1 << 20;
  void *pin_in[2] = {nullptr, nullptr};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  bool pin_open[2] = {false, false};
  int pin_slot = 0;
  void *pin_out = nullptr;
  // ensemble scratch: block records [LEN][blocks], the record, the shift vector (robot 0's
  // state when the first record after create / reset / set_state / load_state was asked for)
  double *ens_blocks = nullptr;
  double *ens_out = nullptr;
  double *ens_shift = nullptr;
  bool ens_shift_ok = false;
  size_t ens_gather_cap = 0;
  // readout scratch [6][N] float
  float *readout = nullptr;
  // output scratch for host-destined results of the control / export entry points
  void *oscratch = nullptr;
  size_t oscratch_bytes = 0;
  // captured per-tick sequence (fmskf_graph_*)
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  bool capturing = false;
  // RCCL communicator (fmskf_comm_init) and the all-gather buffer [world][record]
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
  double *ens_gather = nullptr;
  // asynchronous ensemble (fmskf_tick_ensemble_begin / fmskf_ensemble_begin / _end): up to
  // kEnsSlots events in flight, each slot with its own block records, record, gather buffer and
  // pinned host copy.  A slot is reused only after fmskf_ensemble_end consumed it (its `done`
  // event, behind the fold, was waited for), so the tick that rewrites a slot's block records
  // needs no stream wait.  Event k's fold rides in the next event's tick kernel (extra blocks
  // ahead of its tick blocks: ens_fold_front), or runs stand-alone when a plain tick or a result
  // request comes first (ens_flush); with a communicator the side stream `ens_stream`
  // all-gathers it while the tick stream runs on.
  static constexpr int kEnsSlots = 4;
  struct EnsSlot {
    double *blocks = nullptr, *rec = nullptr, *gather = nullptr;
    double *host = nullptr;  // pinned [ranks][len]
    double *host_dev = nullptr;  // the device's address of `host` (the fold writes it over PCIe)
    size_t cap = 0;          // ranks the gather / host buffers hold
    hipEvent_t done = nullptr;
    int nb = 0;              // the event's block records
    int ranks = 1;
  } eslot[kEnsSlots];
  hipEvent_t ens_ticked = nullptr;  // the tick stream's point the side stream waits for
  hipStream_t ens_stream = nullptr;
  int ens_head = 0, ens_pending = 0;
  int ens_carry = -1;  // the newest event's slot while its fold is not queued yet
  // vehicle control state (allocated on first use) and its parameters
  CtrlDev ctrl{};
  fmskf_ctrl_params cprm{};
  bool ctrl_ready = false;
  // model parameters (fp32 / fp64 copies of cfg)
  Kf6Params kf6{};
  Ekf9Params ekf9{};
  Kf12dParams kf12{};
  bool timing = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // pooled per-launch events (fmskf_kernel_time_total)
  std::vector<hipEvent_t> tpool;
  size_t tcount = 0;
  static constexpr size_t kMaxTimed = 65536;

  void time_begin() {
    if (!timing) return;
    if (tcount < kMaxTimed) {
      while (tpool.size() < 2 * (tcount + 1)) {
        hipEvent_t e;
        hip_check(hipEventCreate(&e), "hipEventCreate");
        tpool.push_back(e);
      }
      hip_check(hipEventRecord(tpool[2 * tcount], stream), "hipEventRecord");
    }
    hip_check(hipEventRecord(ev0, stream), "hipEventRecord");
  }
  void time_end() {
    if (!timing) return;
    hip_check(hipEventRecord(ev1, stream), "hipEventRecord");
    if (tcount < kMaxTimed) {
      hip_check(hipEventRecord(tpool[2 * tcount + 1], stream), "hipEventRecord");
      tcount++;
    }
  }

  template <typename T>
  T *alloc(size_t count) {
    void *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e != hipSuccess) fail(FMSKF_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    allocs.push_back(p);
    return (T *)p;
  }
  // free one allocation made by alloc() (after the stream has drained)
  void release(void *p) {
    if (!p) return;
    for (size_t i = 0; i < allocs.size(); i++)
      if (allocs[i] == p) {
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        (void)hipFree(p);
        allocs.erase(allocs.begin() + (long)i);
        return;
      }
  }
  void *stage_for(size_t bytes) {
    if (bytes > stage_bytes) {
      if (stage) {
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        hip_check(hipFree(stage), "hipFree");
        stage = nullptr;
        stage_bytes = 0;  // a failed hipMalloc below must not leave a stale capacity
      }
      hipError_t e = hipMalloc(&stage, bytes);
      if (e != hipSuccess) fail(FMSKF_ENOMEM, "staging hipMalloc failed");
      stage_bytes = bytes;
    }
    return stage;
  }
  // the next pinned input slot.  The slot the previous staging call used gets its event now,
  // behind everything that call queued (its DMA, or the kernels that read the slot in place);
  // a slot is rewritten only once the event recorded after its last use has completed
  char *pinned_in() {
    const int prev = pin_slot ^ 1, slot = pin_slot;
    if (pin_open[prev]) {
      hip_check(hipEventRecord(pin_ev[prev], stream), "hipEventRecord");
      pin_open[prev] = false;
    }
    pin_slot ^= 1;
    if (!pin_in[slot]) {
      hip_check(hipHostMalloc(&pin_in[slot], kPinned, hipHostMallocDefault), "hipHostMalloc");
      hip_check(hipEventCreateWithFlags(&pin_ev[slot], kSyncEvent), "hipEventCreate");
    } else {
      hip_check(hipEventSynchronize(pin_ev[slot]), "hipEventSynchronize");
    }
    pin_open[slot] = true;
    return (char *)pin_in[slot];
  }
  char *pinned_out() {
    if (!pin_out) hip_check(hipHostMalloc(&pin_out, kPinned, hipHostMallocDefault), "hipHostMalloc");
    return (char *)pin_out;
  }
  // the device's address of a pinned host slot (kernels read / write it over PCIe)
  static void *dev_ptr(void *host) {
    void *d = nullptr;
    hip_check(hipHostGetDevicePointer(&d, host, 0), "hipHostGetDevicePointer");
    return d;
  }
  void destroy_comm();
  void *out_for(size_t bytes) {
    if (bytes > oscratch_bytes) {
      if (oscratch) {
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        hip_check(hipFree(oscratch), "hipFree");
        oscratch = nullptr;
        oscratch_bytes = 0;
      }
      hipError_t e = hipMalloc(&oscratch, bytes);
      if (e != hipSuccess) fail(FMSKF_ENOMEM, "output scratch hipMalloc failed");
      oscratch_bytes = bytes;
    }
    return oscratch;
  }
  ~fmskf_ctx() {
    if (ens_stream) (void)hipStreamSynchronize(ens_stream);
    if (stream) (void)hipStreamSynchronize(stream);
    else (void)hipDeviceSynchronize();
    for (void *p : allocs) (void)hipFree(p);
    if (stage) (void)hipFree(stage);
    if (oscratch) (void)hipFree(oscratch);
    for (int k = 0; k < 2; k++) {
      if (pin_in[k]) (void)hipHostFree(pin_in[k]);
      if (pin_ev[k]) (void)hipEventDestroy(pin_ev[k]);
    }
    if (pin_out) (void)hipHostFree(pin_out);
    for (EnsSlot &e : eslot) {
      if (e.host) (void)hipHostFree(e.host);
      if (e.done) (void)hipEventDestroy(e.done);
    }
    if (ens_ticked) (void)hipEventDestroy(ens_ticked);
    if (ens_stream) (void)hipStreamDestroy(ens_stream);
    destroy_comm();
    if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
    if (graph) (void)hipGraphDestroy(graph);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    for (hipEvent_t e : tpool) (void)hipEventDestroy(e);
  }
};

namespace {

void check_handle(fmskf_handle h) {
  if (!h) fail(FMSKF_EINVAL, "null handle");
}

// Small host-resident inputs / outputs (<= 1 MiB per call) are zero-copy: the CPU packs the
// call's planes into a pinned slot, the kernels read them from there and write their
// host-destined result into the pinned output slot over PCIe, with no DMA at all.  Measured
// against one pageable copy per plane and against a packed slot moved by one DMA (DESIGN.md
// section 5): KF6 isr_tick at 4096 robots 60.6-63.6 / 51.5-55.1 / 31.7-34.7 us.

// Host->device staging of a set of planes; returns device pointers.
struct Stager {
  fmskf_ctx *h;
  bool host;
  std::vector<std::pair<const void **, size_t>> items;
  Stager(fmskf_ctx *hh, uint32_t mem) : h(hh), host(mem == FMSKF_MEM_HOST) {
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
  }
  void add(const void **p, size_t bytes) {
    if (*p && host) items.push_back({p, bytes});
  }
  void run() {
    if (!host || items.empty()) return;
    size_t total = 0;
    for (auto &it : items) total += (it.second + 255) & ~size_t(255);
    size_t off = 0;
    if (total <= fmskf_ctx::kPinned && !h->capturing) {  // pack into a pinned slot, zero-copy
      char *pin = h->pinned_in();
      char *base = (char *)fmskf_ctx::dev_ptr(pin);
      for (auto &it : items) {
        memcpy(pin + off, *it.first, it.second);
        *it.first = base + off;
        off += (it.second + 255) & ~size_t(255);
      }
      return;
    }
    char *base = (char *)h->stage_for(total);
    for (auto &it : items) {
      hip_check(hipMemcpyAsync(base + off, *it.first, it.second, hipMemcpyHostToDevice, h->stream),
                "stage H2D");
      *it.first = base + off;
      off += (it.second + 255) & ~size_t(255);
    }
  }
};

void apply_defaults(fmskf_config *c, uint32_t model, uint64_t n) {
  memset(c, 0, sizeof(*c));
  c->abi_version = FMSKF_ABI_VERSION;
  c->model = model;
  c->n_instances = n;
  c->device = 0;
  c->trig = FMSKF_TRIG_TABLE512;
  c->dt = 0.001;
  c->motor_dir[0] = 1;   // FL  (VD_task_main.cpp:75)
  c->motor_dir[1] = 1;   // BL  (:76)
  c->motor_dir[2] = -1;  // BR  (:77)
  c->motor_dir[3] = -1;  // FR  (:78)
  c->imu_read_reg = 0x51;  // q0: IMU_IF_WT901C::init -> WitReadReg(q0, 4)
  const double dt = c->dt;
  auto setq = [&](int i, int j, double v) { c->q[i * (i + 1) / 2 + j] = v; };
  auto setr = [&](int i, int j, double v) { c->r[i * (i + 1) / 2 + j] = v; };
  auto setp = [&](int i, double v) { c->p0[i * (i + 1) / 2 + i] = v; };
  // discretised white-noise-acceleration blocks for a (pos, vel) pair with density qc
  auto cv_block = [&](int p, int v, double qc) {
    setq(p, p, qc * dt * dt * dt / 3.0);
    setq(v, p, qc * dt * dt / 2.0);
    setq(v, v, qc * dt);
  };
  switch (model) {
    case FMSKF_MODEL_KF6:
      cv_block(0, 3, 4.0);
      cv_block(1, 4, 4.0);
      cv_block(2, 5, 100.0);
      setr(0, 0, 2.5e-5);  // yaw (5 mrad)^2
      setr(1, 1, 2.5e-3);  // gyro (0.05 rad/s)^2
      setr(2, 2, 4e-4);    // wheel velocity (2 cm/s)^2
      setr(3, 3, 4e-4);
      setr(3, 2, 1e-5);
      for (int i = 0; i < 6; i++) setp(i, i < 3 ? 1.0 : 0.25);
      break;
    case FMSKF_MODEL_EKF9: {
      const double qd[9] = {1e-10, 1e-10, 1e-10, 4e-3 * dt, 4e-3 * dt, 100.0 * dt, 1e-12, 2500.0 * dt, 2500.0 * dt};
      for (int i = 0; i < 9; i++) setq(i, i, qd[i]);
      const double rd[6] = {2.5e-5, 2.5e-3, 0.25, 0.25, 4e-4, 4e-4};
      for (int i = 0; i < 6; i++) setr(i, i, rd[i]);
      for (int i = 0; i < 9; i++) setp(i, i < 3 ? 1.0 : (i == 6 ? 1e-2 : 0.25));
      break;
    }
    case FMSKF_MODEL_KF12D: {
      cv_block(0, 3, 4.0);
      cv_block(1, 4, 4.0);
      cv_block(2, 5, 100.0);
      cv_block(6, 9, 1.0);
      cv_block(7, 10, 1.0);
      cv_block(8, 11, 1.0);
      const double rd[8] = {2.5e-5, 2.5e-3, 4e-4, 4e-4, 1e-6, 1e-6, 1e-6, 1e-4};
      for (int i = 0; i < 8; i++) setr(i, i, rd[i]);
      setr(3, 2, 1e-5);
      for (int i = 0; i < 12; i++) setp(i, (i % 6) < 3 ? 1.0 : 0.25);
      break;
    }
    default: break;
  }
}

void convert_params(fmskf_ctx *h) {
  const fmskf_config &c = h->cfg;
  h->kf6.dt = (float)c.dt;
  for (int k = 0; k < 21; k++) h->kf6.q[k] = (float)c.q[k];
  for (int k = 0; k < 10; k++) h->kf6.r[k] = (float)c.r[k];
  h->ekf9.dt = (float)c.dt;
  for (int k = 0; k < 45; k++) h->ekf9.q[k] = (float)c.q[k];
  for (int k = 0; k < 21; k++) h->ekf9.r[k] = (float)c.r[k];
  h->kf12.dt = c.dt;
  for (int k = 0; k < 78; k++) h->kf12.q[k] = c.q[k];
  for (int k = 0; k < 36; k++) h->kf12.r[k] = c.r[k];
  for (int a = 0; a < 4; a++)
    for (int b = 0; b <= a; b++) h->kf12.r2[a * (a + 1) / 2 + b] = c.r[(a + 4) * (a + 5) / 2 + (b + 4)];
  h->kf12.decor = kf12d_cinv(h->kf12.r, h->kf12.cinv) ? 1 : 0;
  h->kf12.sparse = h->kf12.decor && kf12d_sparse(h->kf12.cinv, h->kf12.q) ? 1 : 0;
}

// WT901 / IMU_IF state and M2006 motor state, allocated on first use (an ingest call, a NULL
// input plane that reads them, a readout of them, or a graph capture) and zero-initialised like
// the firmware's static objects
void zero_imu(fmskf_ctx *h) {
  DevState &s = h->s;
  const uint64_t n = s.n;
  hipStream_t st = h->stream;
  hip_check(hipMemsetAsync(s.imu_reg, 0, 0x90 * n * 2, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_parser, 0, 3 * n * 4, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_cnt, 0, n, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_flags, 0, n, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_err, 0, n, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_qinit, 0, 4 * n * 4, st), "reset imu");
  hip_check(hipMemsetAsync(s.imu_data, 0, 16 * n * 4, st), "reset imu");
}
void zero_motors(fmskf_ctx *h) {
  DevState &s = h->s;
  const uint64_t n = s.n;
  hipStream_t st = h->stream;
  hip_check(hipMemsetAsync(s.m_micro, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_angle, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_prev, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_rpm, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_curr, 0, 4 * n * 2, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_sum, 0, 4 * s.m_pitch * 8, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_iir_y, 0, 4 * n * 4, st), "reset motors");
  hip_check(hipMemsetAsync(s.m_iir_x, 0, 4 * n * 4, st), "reset motors");
}
// ---- asynchronous ensemble: queueing a slot's fold ----------------------------------------
// The fold of slot S is queued on the handle's stream (carried by a tick kernel, or
// stand-alone): with a communicator the side stream all-gathers the record over xGMI and copies
// the gathered records into the slot's pinned buffer behind it; on one GPU the fold wrote the
// pinned buffer itself.  Then the slot's `done` event.
double *ens_fold_dst(const fmskf_ctx *h, const fmskf_ctx::EnsSlot &S) { return h->comm ? S.rec : S.host_dev; }
void ens_gather_async(fmskf_ctx *h, fmskf_ctx::EnsSlot &S);  // with the RCCL entry points below
// One GPU: the event behind the fold (the fold stored the record into the pinned slot with
// system-scope stores, ens_fold_block).  Waiting on the pinned slot itself instead of an event
// (a signalling-NaN sentinel polled by fmskf_ensemble_end) measured slower: K = 1 at 2^20
// 41.8-41.9 us per tick against 40.0-40.2 (kbench ens_async, two passes each, one box).
void ens_fold_queued(fmskf_ctx *h, fmskf_ctx::EnsSlot &S) {
  if (h->comm) ens_gather_async(h, S);
  else hip_check(hipEventRecord(S.done, h->stream), "hipEventRecord");
  h->ens_carry = -1;
}
// the stand-alone fold of the newest event, when no tick kernel carried it
void ens_flush(fmskf_ctx *h) {
  if (h->ens_carry < 0) return;
  fmskf_ctx::EnsSlot &S = h->eslot[h->ens_carry];
  launch_check(launch_ens_fold((int)h->d.nx, S.blocks, S.nb, h->ens_shift, ens_fold_dst(h, S), h->stream),
               "ensemble fold launch");
  ens_fold_queued(h, S);
}

// the ensemble shift vector: robot 0's state, taken once per create / reset / set_state /
// load_state, so successive records of one state are bitwise identical
void ensure_shift(fmskf_ctx *h) {
  if (h->ens_shift_ok) return;
  // a launch inside a capture is only recorded: the flag would claim a shift that no run wrote
  // (fmskf_graph_begin takes it before capturing)
  if (h->capturing) fail(FMSKF_EINVAL, "ensemble shift first taken inside a graph capture");
  // a pending fold reads the shift its event's records were taken against: queue it first
  // (stream order then keeps it ahead of the rewrite)
  ens_flush(h);
  launch_check(launch_ens_shift(h->s, (int)h->d.nx, h->d.elem == 8, h->ens_shift, h->stream),
               "ensemble shift launch");
  h->ens_shift_ok = true;
}

// the models whose tick kernel writes the ensemble block records of the state it stores
bool fused_record(const fmskf_ctx *h) {
  return h->cfg.model == FMSKF_MODEL_KF6 || (h->cfg.model == FMSKF_MODEL_EKF9 && h->s.tile) ||
         (h->cfg.model == FMSKF_MODEL_KF12D && h->s.tile && h->kf12.decor);
}

void ensure_imu(fmskf_ctx *h) {
  DevState &s = h->s;
  if (s.imu_reg) return;
  if (h->capturing) fail(FMSKF_EINVAL, "IMU state first used inside a graph capture");
  const uint64_t n = s.n;
  s.imu_reg = h->alloc<int16_t>(0x90 * n);
  s.imu_parser = h->alloc<uint32_t>(3 * n);
  s.imu_cnt = h->alloc<uint8_t>(n);
  s.imu_flags = h->alloc<uint8_t>(n);
  s.imu_err = h->alloc<uint8_t>(n);
  s.imu_qinit = h->alloc<float>(4 * n);
  s.imu_data = h->alloc<float>(16 * n);
  zero_imu(h);
}
void ensure_motors(fmskf_ctx *h) {
  DevState &s = h->s;
  if (s.m_sum) return;
  if (h->capturing) fail(FMSKF_EINVAL, "motor state first used inside a graph capture");
  const uint64_t n = s.n;
  s.m_micro = h->alloc<int16_t>(4 * n);
  s.m_angle = h->alloc<int16_t>(4 * n);
  s.m_prev = h->alloc<int16_t>(4 * n);
  s.m_rpm = h->alloc<int16_t>(4 * n);
  s.m_curr = h->alloc<int16_t>(4 * n);
  s.m_pitch = plane_pitch(n);
  s.m_sum = h->alloc<int64_t>(4 * s.m_pitch);
  s.m_iir_y = h->alloc<float>(4 * n);
  s.m_iir_x = h->alloc<float>(4 * n);
  zero_motors(h);
}
void ensure_ctrl(fmskf_ctx *h);
void zero_ctrl(fmskf_ctx *h);

void do_reset(fmskf_ctx *h) {
  DevState &s = h->s;
  const uint64_t n = s.n;
  const Dims d = h->d;
  const uint32_t np = d.nx * (d.nx + 1) / 2;
  hipStream_t st = h->stream;
  const uint64_t pp = s.pitch;
  hip_check(hipMemsetAsync(s.x, 0, (size_t)d.nx * pp * d.elem, st), "reset x");
  if (d.m > 0 && s.tile) {  // tiled P: every row filled with its P0 entry in one pass
    std::vector<uint64_t> bits(np);
    for (uint32_t k = 0; k < np; k++) {
      const double v = h->cfg.p0[k];
      if (d.elem == 4) {
        const float f = (float)v;
        uint32_t b;
        memcpy(&b, &f, 4);
        bits[k] = b;
      } else {
        memcpy(&bits[k], &v, 8);
      }
    }
    launch_check(launch_tiled_fill(s.P, np, n, bits.data(), d.elem, st), "reset P0");
  } else if (d.m > 0) {
    hip_check(hipMemsetAsync(s.P, 0, (size_t)np * pp * d.elem, st), "reset P");
    for (uint32_t i = 0; i < d.nx; i++) {
      for (uint32_t j = 0; j <= i; j++) {
        const double v = h->cfg.p0[i * (i + 1) / 2 + j];
        if (v == 0.0) continue;
        const size_t k = i * (i + 1) / 2 + j;
        if (d.elem == 4) {
          float f = (float)v;
          uint32_t bits;
          memcpy(&bits, &f, 4);
          hip_check(hipMemsetD32Async((hipDeviceptr_t)((float *)s.P + k * pp), bits, n, st), "reset P0");
        } else {
          uint64_t bits;
          memcpy(&bits, &v, 8);
          launch_check(launch_fill64((double *)s.P + k * pp, bits, n, st), "reset P0");
        }
      }
    }
  }
  if (s.prev_sum) hip_check(hipMemsetAsync(s.prev_sum, 0, 4 * pp * 8, st), "reset prev");
  if (s.thlo) hip_check(hipMemsetAsync(s.thlo, 0, n * 4, st), "reset heading low part");
  if (s.xlo) hip_check(hipMemsetAsync(s.xlo, 0, (size_t)kKf6LoRows * pp * 4, st), "reset position low parts");
  if (s.imu_reg) zero_imu(h);
  if (s.m_sum) zero_motors(h);
  if (h->ctrl_ready) {  // the control objects are static in the firmware too: zero, power off
    const CtrlDev &c = h->ctrl;
    hip_check(hipMemsetAsync(c.ax, 0, (size_t)3 * kAxF * c.pitch * 4, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.pid, 0, (size_t)4 * kPidF * c.pitch * 4, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.vel_tgt, 0, (size_t)3 * c.pitch * 4, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.curr, 0, (size_t)4 * c.n * 2, st), "reset ctrl");
    hip_check(hipMemsetAsync(c.power, 0, (size_t)c.n, st), "reset ctrl");
  }
  hip_check(hipMemsetAsync(s.counters, 0, 8 * 8, st), "reset counters");
  h->ens_shift_ok = false;
}

// Resolve the tick inputs of a call (NULL -> device-resident ingest state), stage host
// planes and validate what the model needs.
TickIn resolve_inputs(fmskf_ctx *h, const fmskf_tick_inputs *in, bool need_upd, bool need_pred,
                      uint32_t n_ticks, uint64_t stride) {
  if (!in) fail(FMSKF_EINVAL, "null inputs");
  DevState &s = h->s;
  const uint64_t n = s.n;
  if (stride < n) fail(FMSKF_EINVAL, "tick_stride < N");
  if (n_ticks == 0) fail(FMSKF_EINVAL, "n_ticks == 0");
  TickIn t{};
  t.yaw_deg = in->yaw_deg;
  t.gyro_z = in->gyro_z_dps;
  t.rpm = in->rpm;
  t.angle_sum = in->angle_sum;
  t.raw = in->raw;
  t.z = in->z;
  t.valid = in->valid;
  t.rec = (const uint32_t *)in->kf6_rec;
  t.sintab = s.sintab;
  t.stride = stride;
  t.sum_pitch = stride;
  t.n_ticks = n_ticks;
  if (t.rec && h->cfg.model != FMSKF_MODEL_KF6) fail(FMSKF_EINVAL, "kf6_rec is a KF6 input");
  if (t.rec && (t.yaw_deg || t.gyro_z || t.rpm))
    fail(FMSKF_EINVAL, "kf6_rec replaces yaw_deg / gyro_z_dps / rpm: pass one or the other");
  if (in->angle_sum_pitch) {
    if (n_ticks != 1 || stride != n) fail(FMSKF_EINVAL, "angle_sum_pitch is for single-tick calls (tick_many: tick_stride)");
    if (in->angle_sum_pitch < n) fail(FMSKF_EINVAL, "angle_sum_pitch < N");
    t.sum_pitch = in->angle_sum_pitch;
  }
  const uint64_t span = (uint64_t)(n_ticks - 1) * stride + n;  // elements per [N] plane
  Stager sg(h, in->mem);
  sg.add((const void **)&t.yaw_deg, span * 4);
  sg.add((const void **)&t.gyro_z, span * 4);
  sg.add((const void **)&t.rpm, span * 8);
  sg.add((const void **)&t.angle_sum, ((uint64_t)(n_ticks - 1) * stride * 4 + 3 * t.sum_pitch + n) * 8);
  sg.add((const void **)&t.raw, span * 16);
  sg.add((const void **)&t.z, ((uint64_t)(n_ticks - 1) * stride * 8 + 7 * stride + n) * 8);
  sg.add((const void **)&t.valid, span);
  sg.add((const void **)&t.rec, span * 16);
  sg.run();
  const bool many = n_ticks > 1 || stride != n;
  auto dev_default = [&](const void *p, const char *name) {
    if (!p && many) fail(FMSKF_EINVAL, std::string("tick_many needs explicit plane ") + name);
  };
  switch (h->cfg.model) {
    case FMSKF_MODEL_RS:
      if (need_upd) {
        dev_default(t.yaw_deg, "yaw_deg");
        if (!t.yaw_deg) {
          ensure_imu(h);
          t.yaw_deg = s.imu_data + 11 * n;  // IMT::get_status_now_yaw
        }
      }
      if (need_pred) {
        dev_default(t.rpm, "rpm");
        dev_default(t.angle_sum, "angle_sum");
        if (!t.rpm || !t.angle_sum) ensure_motors(h);
        if (!t.rpm) t.rpm = s.m_rpm;
        if (!t.angle_sum) {
          t.angle_sum = s.m_sum;
          t.sum_pitch = s.m_pitch;
        }
      }
      break;
    case FMSKF_MODEL_KF6:
      if (need_upd && !t.rec) {
        dev_default(t.yaw_deg, "yaw_deg");
        dev_default(t.gyro_z, "gyro_z_dps");
        dev_default(t.rpm, "rpm");
        if (!t.yaw_deg || !t.gyro_z) ensure_imu(h);
        if (!t.rpm) ensure_motors(h);
        if (!t.yaw_deg) t.yaw_deg = s.imu_data + 11 * n;
        if (!t.gyro_z) t.gyro_z = s.imu_data + 5 * n;
        if (!t.rpm) t.rpm = s.m_rpm;
      }
      break;
    case FMSKF_MODEL_EKF9:
      if (need_upd && !t.raw) fail(FMSKF_EINVAL, "EKF9 needs raw words");
      break;
    case FMSKF_MODEL_KF12D:
      if (need_upd && !t.z) fail(FMSKF_EINVAL, "KF12D needs z");
      break;
  }
  return t;
}

void run_tick(fmskf_ctx *h, const fmskf_tick_inputs *in, bool upd, bool pred, uint32_t n_ticks,
              uint64_t stride) {
  check_handle(h);
  DeviceGuard g(h->cfg.device);
  TickIn t = resolve_inputs(h, in, upd, pred, n_ticks, stride);
  // a plain tick after an asynchronous ensemble event: the event's fold runs stand-alone
  // ahead of it (a record every K > 1 ticks gets its result one fold after its tick; only the
  // next ensemble tick's kernel carries it).  Not inside a capture: the replay would fold
  // whatever the slot holds then
  if (!h->capturing) ens_flush(h);
  const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
  h->time_begin();
  int e = 0;
  switch (h->cfg.model) {
    case FMSKF_MODEL_RS: e = launch_rs(h->s, t, libm, upd, pred, h->stream); break;
    case FMSKF_MODEL_KF6: e = launch_kf6(h->s, t, h->kf6, libm, upd, pred, h->stream); break;
    case FMSKF_MODEL_EKF9: e = launch_ekf9(h->s, t, h->ekf9, libm, upd, pred, h->stream); break;
    case FMSKF_MODEL_KF12D: e = launch_kf12d(h->s, t, h->kf12, upd, pred, h->stream); break;
  }
  launch_check(e, "tick kernel launch");
  h->time_end();
}

void copy_out(fmskf_ctx *h, void *dst, const void *src, size_t bytes, uint32_t mem) {
  if (!dst) return;
  if (mem == FMSKF_MEM_HOST) {
    hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
  } else if (mem == FMSKF_MEM_DEVICE) {
    hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, h->stream), "D2D");
  } else {
    fail(FMSKF_EINVAL, "bad mem flag");
  }
}
// `planes` planes of `row` bytes: device planes at `dev_pitch` bytes <-> dense user planes
void copy_planes_out(fmskf_ctx *h, void *dst, const void *src, size_t row, size_t dev_pitch,
                     size_t planes, uint32_t mem) {
  if (!dst) return;
  if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
  const hipMemcpyKind k = mem == FMSKF_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
  hip_check(hipMemcpy2DAsync(dst, row, src, dev_pitch, row, planes, k, h->stream), "copy planes");
}
void copy_planes_in(fmskf_ctx *h, void *dst, const void *src, size_t row, size_t dev_pitch,
                    size_t planes, uint32_t mem) {
  if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
  const hipMemcpyKind k = mem == FMSKF_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  hip_check(hipMemcpy2DAsync(dst, dev_pitch, src, row, row, planes, k, h->stream), "copy planes");
}
void finish_out(fmskf_ctx *h, uint32_t mem) {
  if (mem == FMSKF_MEM_HOST) hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
}
// where a kernel writes a result of `bytes` bound for the caller's host memory: the pinned
// output slot itself under zero-copy staging, else device scratch
void *host_result(fmskf_ctx *h, size_t bytes) {
  if (bytes <= fmskf_ctx::kPinned && !h->capturing) return fmskf_ctx::dev_ptr(h->pinned_out());
  return h->out_for(bytes);
}
// one device buffer to the caller's host (or device) buffer, complete on return: a small host
// result goes through the pinned slot (written there by the kernel under zero-copy staging, or
// one DMA), then a CPU copy
void copy_out_sync(fmskf_ctx *h, void *dst, const void *src, size_t bytes, uint32_t mem) {
  if (mem == FMSKF_MEM_HOST && h->pin_out && src == fmskf_ctx::dev_ptr(h->pin_out)) {
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    memcpy(dst, h->pin_out, bytes);
    return;
  }
  if (mem == FMSKF_MEM_HOST && bytes <= fmskf_ctx::kPinned && !h->capturing) {
    char *pin = h->pinned_out();
    hip_check(hipMemcpyAsync(pin, src, bytes, hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    memcpy(dst, pin, bytes);
    return;
  }
  if (mem == FMSKF_MEM_HOST) copy_out(h, dst, src, bytes, mem);
  finish_out(h, mem);
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int fmskf_abi_version(void) { return (int)FMSKF_ABI_VERSION; }

const char *fmskf_strerror(int status) {
  switch (status) {
    case FMSKF_OK: return "ok";
    case FMSKF_EINVAL: return "invalid argument";
    case FMSKF_ENOMEM: return "out of memory";
    case FMSKF_EDEVICE: return "device error";
    case FMSKF_ERCCL: return "collective error";
    case FMSKF_ENOTSUP: return "not supported for this model";
    default: return "unknown status";
  }
}

const char *fmskf_last_error(void) { return g_last_error.c_str(); }

int fmskf_model_dims(uint32_t model, uint32_t *n, uint32_t *m, uint32_t *elem_bytes) {
  return guarded([&] {
    Dims d = dims_of(model);
    if (n) *n = d.nx;
    if (m) *m = d.m;
    if (elem_bytes) *elem_bytes = d.elem;
  });
}

int fmskf_config_init(fmskf_config *cfg, uint32_t model, uint64_t n) {
  return guarded([&] {
    if (!cfg) fail(FMSKF_EINVAL, "null config");
    (void)dims_of(model);
    apply_defaults(cfg, model, n);
  });
}

int fmskf_create(const fmskf_config *cfg, fmskf_handle *out) {
  return guarded([&] {
    if (!cfg || !out) fail(FMSKF_EINVAL, "null argument");
    *out = nullptr;
    if (cfg->abi_version != FMSKF_ABI_VERSION) fail(FMSKF_EINVAL, "ABI version mismatch");
    const Dims d = dims_of(cfg->model);
    if (cfg->n_instances == 0) fail(FMSKF_EINVAL, "n_instances == 0");
    if (cfg->n_instances > (1ull << 30)) fail(FMSKF_EINVAL, "n_instances > 2^30 per handle");
    if (cfg->trig > FMSKF_TRIG_LIBM) fail(FMSKF_EINVAL, "bad trig policy");
    if (!(cfg->dt > 0.0) || !isfinite(cfg->dt)) fail(FMSKF_EINVAL, "dt must be > 0");
    if (cfg->imu_read_reg + 4 > 0x90) fail(FMSKF_EINVAL, "imu_read_reg out of range");
    if ((cfg->flags & ~FMSKF_CFG_COMP_POS) || cfg->reserved) fail(FMSKF_EINVAL, "unknown config flags");
    if ((cfg->flags & FMSKF_CFG_COMP_POS) && cfg->model != FMSKF_MODEL_KF6 && cfg->model != FMSKF_MODEL_EKF9)
      fail(FMSKF_ENOTSUP, "FMSKF_CFG_COMP_POS is a KF6 / EKF9 mode");
    for (int w = 0; w < 4; w++)
      if (cfg->motor_dir[w] != 1 && cfg->motor_dir[w] != -1) fail(FMSKF_EINVAL, "motor_dir must be +-1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail(FMSKF_EDEVICE, "no HIP device");
    if (cfg->device < 0 || cfg->device >= ndev) fail(FMSKF_EINVAL, "bad device ordinal");
    DeviceGuard g(cfg->device);
    fmskf_ctx *h = new fmskf_ctx();
    try {
      h->cfg = *cfg;
      h->d = d;
      const uint64_t n = cfg->n_instances;
      DevState &s = h->s;
      s.n = n;
      s.model = cfg->model;
      const uint32_t np = d.nx * (d.nx + 1) / 2;
      s.tile = (FMSKF_TILED && (cfg->model == FMSKF_MODEL_EKF9 || cfg->model == FMSKF_MODEL_KF12D)) ||
                       (FMSKF_KF6_TILED && cfg->model == FMSKF_MODEL_KF6)
                   ? tile_w_elem(d.elem) : 0;
      // a tiled array's rows x pitch elements cover ceil(N / tile) whole tiles
      s.pitch = s.tile ? std::max(plane_pitch(n), (n + s.tile - 1) / s.tile * s.tile) : plane_pitch(n);
      s.x = h->alloc<char>((size_t)d.nx * s.pitch * d.elem);
      s.P = d.m ? h->alloc<char>((size_t)np * s.pitch * d.elem) : nullptr;
      s.prev_sum = cfg->model == FMSKF_MODEL_RS ? h->alloc<int64_t>(4 * s.pitch) : nullptr;
      // EKF9: the compensated heading's hidden low part (kf_generic.hpp th_add), one float a robot
      s.thlo = cfg->model == FMSKF_MODEL_EKF9 ? h->alloc<float>(n) : nullptr;
      // KF6 / EKF9 with FMSKF_CFG_COMP_POS: the position low parts, tiled like x and P
      s.xlo = (cfg->flags & FMSKF_CFG_COMP_POS) ? h->alloc<float>((size_t)kKf6LoRows * s.pitch) : nullptr;
      h->kf6.lo = s.xlo;
      // the WT901 / motor ingest state (~470 B per robot) is allocated on first use
      // (ensure_imu / ensure_motors): a handle fed tick inputs by the caller holds only x, P
      s.counters = h->alloc<unsigned long long>(8);
      s.sintab = h->alloc<float>(513);
      {
        // the fused KF6 tick + record (fmskf_tick_ensemble) writes one record per tick block
        const size_t len = 1 + d.nx + np;
        size_t nb = (size_t)ensemble_nblocks(n);
        if (cfg->model == FMSKF_MODEL_KF6 || cfg->model == FMSKF_MODEL_EKF9 || cfg->model == FMSKF_MODEL_KF12D)
          nb = std::max(nb, (size_t)((n + kBlock - 1) / kBlock));
        h->ens_blocks = h->alloc<double>(nb * len);
        h->ens_out = h->alloc<double>(91);
        h->ens_shift = h->alloc<double>(12);
      }
      h->readout = h->alloc<float>(6 * n);
      // TABLE512: CMSIS-DSP's sinTable_f32 as its published 8-decimal literals (arm_common_tables.c;
      // the firmware's arm_sin_f32 / arm_cos_f32, util_mymath.hpp:44-45), cmsis_sintab.inc
      static const float tab[513] = {
#include "cmsis_sintab.inc"
      };
      hip_check(hipMemcpy(s.sintab, tab, sizeof(tab), hipMemcpyHostToDevice), "sintab upload");
      hip_check(hipEventCreate(&h->ev0), "hipEventCreate");
      hip_check(hipEventCreate(&h->ev1), "hipEventCreate");
      convert_params(h);
      {
        double *coef = h->alloc<double>(36 + 78);
        hip_check(hipMemcpy(coef, h->kf12.cinv, 36 * sizeof(double), hipMemcpyHostToDevice), "coef upload");
        hip_check(hipMemcpy(coef + 36, h->kf12.q, 78 * sizeof(double), hipMemcpyHostToDevice), "coef upload");
        h->kf12.coef = coef;
      }
      do_reset(h);
      hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int fmskf_destroy(fmskf_handle h) {
  return guarded([&] {
    if (!h) return;
    DeviceGuard g(h->cfg.device);
    delete h;
  });
}

int fmskf_reset(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    do_reset(h);
  });
}

int fmskf_set_stream(fmskf_handle h, void *stream) {
  return guarded([&] {
    check_handle(h);
    // work queued on the old stream (staging buffers, pinned slots) completes before the new
    // stream can reuse what it reads
    if (h->stream != (hipStream_t)stream && !h->capturing)
      hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    h->stream = (hipStream_t)stream;
  });
}

int fmskf_graph_begin(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    if (!h->stream) fail(FMSKF_EINVAL, "graph capture needs a stream (fmskf_set_stream)");
    if (h->capturing) fail(FMSKF_EINVAL, "capture already open");
    if (h->timing) fail(FMSKF_EINVAL, "disable per-launch timing before capturing");
    DeviceGuard g(h->cfg.device);
    // state that is allocated on first use must exist before the capture starts
    ensure_imu(h);
    ensure_motors(h);
    ensure_ctrl(h);
    ensure_shift(h);
    hip_check(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal),
              "hipStreamBeginCapture");
    h->capturing = true;
  });
}

int fmskf_graph_end(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    if (!h->capturing) fail(FMSKF_EINVAL, "no capture open");
    DeviceGuard g(h->cfg.device);
    h->capturing = false;
    hipGraph_t gnew = nullptr;
    hip_check(hipStreamEndCapture(h->stream, &gnew), "hipStreamEndCapture");
    if (h->graph_exec) hip_check(hipGraphExecDestroy(h->graph_exec), "hipGraphExecDestroy");
    if (h->graph) hip_check(hipGraphDestroy(h->graph), "hipGraphDestroy");
    h->graph_exec = nullptr;
    h->graph = gnew;
    hip_check(hipGraphInstantiate(&h->graph_exec, h->graph, nullptr, nullptr, 0),
              "hipGraphInstantiate");
  });
}

int fmskf_graph_launch(fmskf_handle h, uint32_t times) {
  return guarded([&] {
    check_handle(h);
    if (!h->graph_exec) fail(FMSKF_EINVAL, "no graph captured");
    if (h->capturing) fail(FMSKF_EINVAL, "capture still open");
    DeviceGuard g(h->cfg.device);
    for (uint32_t k = 0; k < times; k++)
      hip_check(hipGraphLaunch(h->graph_exec, h->stream), "hipGraphLaunch");
  });
}

int fmskf_sync(fmskf_handle h) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
  });
}

int fmskf_get_config(fmskf_handle h, fmskf_config *out) {
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    *out = h->cfg;
  });
}

int fmskf_ingest_wt901(fmskf_handle h, const uint8_t *bytes, uint32_t stride, const uint32_t *len,
                       int latch_qinit, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!bytes || !len) fail(FMSKF_EINVAL, "null bytes/len");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    if (mem == FMSKF_MEM_HOST) {
      for (uint64_t i = 0; i < n; i++)
        if (len[i] > stride) fail(FMSKF_EINVAL, "len[i] > stride");
    }
    ensure_imu(h);
    Stager sg(h, mem);
    const void *b = bytes, *l = len;
    sg.add(&b, (size_t)stride * n);
    sg.add(&l, n * 4);
    sg.run();
    launch_check(launch_wt901(h->s, (const uint8_t *)b, stride, (const uint32_t *)l, latch_qinit,
                              h->cfg.imu_read_reg, h->stream),
                 "wt901 launch");
  });
}

int fmskf_ingest_can(fmskf_handle h, const uint8_t *frames, const int16_t *stamps,
                     const uint8_t *present, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!frames || !stamps) fail(FMSKF_EINVAL, "null frames/stamps");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_motors(h);
    Stager sg(h, mem);
    const void *f = frames, *s = stamps, *p = present;
    sg.add(&f, n * 32);
    sg.add(&s, n * 8);
    sg.add(&p, n);
    sg.run();
    launch_check(launch_can(h->s, (const uint8_t *)f, (const int16_t *)s, (const uint8_t *)p,
                            h->cfg.motor_dir, h->stream),
                 "can launch");
  });
}

int fmskf_correct(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] { run_tick(h, in, true, false, 1, h ? h->s.n : 0); });
}

int fmskf_predict(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] { run_tick(h, in, false, true, 1, h ? h->s.n : 0); });
}

int fmskf_tick(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] { run_tick(h, in, true, true, 1, h ? h->s.n : 0); });
}

int fmskf_tick_many(fmskf_handle h, const fmskf_tick_inputs *in, uint32_t n_ticks,
                    uint64_t tick_stride) {
  return guarded([&] { run_tick(h, in, true, true, n_ticks, tick_stride); });
}

int fmskf_get_pose(fmskf_handle h, float *x, float *y, float *th, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    launch_check(launch_readout(h->s, h->readout, h->stream), "readout");
    copy_out(h, x, h->readout, n * 4, mem);
    copy_out(h, y, h->readout + n, n * 4, mem);
    copy_out(h, th, h->readout + 2 * n, n * 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_vel(fmskf_handle h, float *vx, float *vy, float *vth, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    launch_check(launch_readout(h->s, h->readout, h->stream), "readout");
    copy_out(h, vx, h->readout + 3 * n, n * 4, mem);
    copy_out(h, vy, h->readout + 4 * n, n * 4, mem);
    copy_out(h, vth, h->readout + 5 * n, n * 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_state(fmskf_handle h, void *x, void *p_packed, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const Dims d = h->d;
    const size_t row = (size_t)n * d.elem, pb = (size_t)h->s.pitch * d.elem;
    const uint32_t np = d.nx * (d.nx + 1) / 2;
    if (p_packed && !d.m) fail(FMSKF_ENOTSUP, "RS model has no covariance");
    if (h->s.tile) {  // tiled state: gather into dense planes (device), then copy
      if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
      auto out = [&](void *dst, const void *src, uint32_t rows) {
        if (!dst) return;
        void *dense = mem == FMSKF_MEM_DEVICE ? dst : h->out_for(row * rows);
        launch_check(launch_untile(src, dense, rows, n, d.elem, h->stream), "untile");
        if (mem == FMSKF_MEM_HOST) {
          copy_out(h, dst, dense, row * rows, mem);
          hip_check(hipStreamSynchronize(h->stream), "get_state sync");  // scratch reused next
        }
      };
      out(x, h->s.x, d.nx);
      if (p_packed) out(p_packed, h->s.P, np);
    } else {
      copy_planes_out(h, x, h->s.x, row, pb, d.nx, mem);
      if (p_packed) copy_planes_out(h, p_packed, h->s.P, row, pb, np, mem);
    }
    finish_out(h, mem);
  });
}

int fmskf_set_state(fmskf_handle h, const void *x, const void *p_packed, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const Dims d = h->d;
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    const size_t row = (size_t)n * d.elem, pb = (size_t)h->s.pitch * d.elem;
    const uint32_t np = d.nx * (d.nx + 1) / 2;
    if (p_packed && !d.m) fail(FMSKF_ENOTSUP, "RS model has no covariance");
    if (h->s.tile) {  // dense planes (staged to the device when on the host) -> tiled state
      auto in = [&](void *dst, const void *src, uint32_t rows) {
        if (!src) return;
        const void *dense = src;
        if (mem == FMSKF_MEM_HOST) {
          void *stg = h->stage_for(row * rows);
          hip_check(hipMemcpyAsync(stg, src, row * rows, hipMemcpyHostToDevice, h->stream), "stage H2D");
          dense = stg;
        }
        launch_check(launch_tile(dense, dst, rows, n, d.elem, h->stream), "tile");
        if (mem == FMSKF_MEM_HOST) hip_check(hipStreamSynchronize(h->stream), "set_state sync");
      };
      in(h->s.x, x, d.nx);
      if (p_packed) in(h->s.P, p_packed, np);
    } else {
      if (x) copy_planes_in(h, h->s.x, x, row, pb, d.nx, mem);
      if (p_packed) copy_planes_in(h, h->s.P, p_packed, row, pb, np, mem);
    }
    if (x) h->ens_shift_ok = false;
    // a heading set from outside is exact as given: its compensation term restarts at zero
    if (x && h->s.thlo) hip_check(hipMemsetAsync(h->s.thlo, 0, n * 4, h->stream), "heading low part");
    // compensated positions: a state set from outside restarts every low part (x and P)
    if ((x || p_packed) && h->s.xlo)
      hip_check(hipMemsetAsync(h->s.xlo, 0, (size_t)kKf6LoRows * h->s.pitch * 4, h->stream), "position low parts");
    finish_out(h, mem);
  });
}

}  // extern "C"

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
// header; format-2 and format-3 files are rejected by name.
constexpr char kCkMagic[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '4'};
constexpr char kCkMagicV3[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '3'};
constexpr char kCkMagicV1[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '1'};
constexpr char kCkMagicV2[8] = {'F', 'M', 'S', 'K', 'F', 'C', 'K', '2'};
struct CkHeader {
  char magic[8];
  uint32_t abi, model;
  uint64_t n, pitch;
  uint32_t tile, elem, groups, ctrl_tile;  // ctrl_tile: control arrays' tile width (0 = planar)
  uint64_t m_pitch, ctrl_pitch;            // motor sum planes' pitch, control state's pitch
  uint64_t body_bytes, checksum;           // what follows the header, and its hash
  uint32_t flags, reserved;                // fmskf_config.flags (FMSKF_CFG_*)
};
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
    v.push_back({s.imu_data, (size_t)16 * n * 4});
  }
  if (groups & 4) {
    for (void *p : {(void *)s.m_micro, (void *)s.m_angle, (void *)s.m_prev, (void *)s.m_rpm, (void *)s.m_curr})
      v.push_back({p, (size_t)4 * n * 2});
    v.push_back({s.m_sum, (size_t)4 * s.m_pitch * 8});
    for (void *p : {(void *)s.m_iir_y, (void *)s.m_iir_x})
      v.push_back({p, (size_t)4 * n * 4});
  }
  if (groups & 8) {
    const CtrlDev &c = h->ctrl;
    v.push_back({c.ax, (size_t)3 * kAxF * c.pitch * 4});
    v.push_back({c.pid, (size_t)4 * kPidF * c.pitch * 4});
    v.push_back({c.vel_tgt, (size_t)3 * c.pitch * 4});
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
    hd.groups = 1u | (h->s.imu_reg ? 2u : 0u) | (h->s.m_sum ? 4u : 0u) | (h->ctrl_ready ? 8u : 0u);
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
    if (memcmp(hd.magic, kCkMagic, 8) != 0) fail(FMSKF_EINVAL, "not an fmskf checkpoint");
    f.seek(0, SEEK_SET);
    f.read(&hd, sizeof(hd));
    CkHeader me{};
    ck_layout(h, &me);
    if (hd.abi != me.abi || hd.model != me.model || hd.n != me.n || hd.pitch != me.pitch ||
        hd.tile != me.tile || hd.elem != me.elem || hd.flags != me.flags || (hd.groups & ~15u))
      fail(FMSKF_EINVAL, "checkpoint does not match this handle (ABI, model, flags, N or layout)");
    if ((hd.groups & 4) && hd.m_pitch != me.m_pitch) fail(FMSKF_EINVAL, "checkpoint motor layout differs");
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
    if (!(hd.groups & 4) && h->s.m_sum) zero_motors(h);
    if (!(hd.groups & 8) && h->ctrl_ready) zero_ctrl(h);
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

int fmskf_get_prev_sum(fmskf_handle h, int64_t *prev, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!h->s.prev_sum) fail(FMSKF_ENOTSUP, "prev_sum exists in the RS model only");
    DeviceGuard g(h->cfg.device);
    copy_planes_out(h, prev, h->s.prev_sum, h->s.n * 8, h->s.pitch * 8, 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_imu(fmskf_handle h, float *data, uint8_t *is_error, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_imu(h);
    copy_out(h, data, h->s.imu_data, 16 * h->s.n * 4, mem);
    copy_out(h, is_error, h->s.imu_err, h->s.n, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_imu_regs(fmskf_handle h, int16_t *regs, uint8_t *pending, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_imu(h);
    copy_out(h, regs, h->s.imu_reg, 0x90 * h->s.n * 2, mem);
    copy_out(h, pending, h->s.imu_cnt, h->s.n, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_motors(fmskf_handle h, int16_t *angle, int16_t *rpm, int16_t *curr,
                     int64_t *angle_sum, float *speed_radps, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_motors(h);
    copy_out(h, angle, h->s.m_angle, 4 * n * 2, mem);
    copy_out(h, rpm, h->s.m_rpm, 4 * n * 2, mem);
    copy_out(h, curr, h->s.m_curr, 4 * n * 2, mem);
    copy_planes_out(h, angle_sum, h->s.m_sum, n * 8, h->s.m_pitch * 8, 4, mem);
    // Status::flt_SpeedRadPS is the IIR1 output, i.e. its state y (VD_motor_if_m2006.cpp:63)
    copy_out(h, speed_radps, h->s.m_iir_y, 4 * n * 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_get_motor_status(fmskf_handle h, int16_t *microsec_id, int16_t *angle, int16_t *rpm,
                           int16_t *curr, float *dlt_out_angle_rad, float *speed_radps, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_motors(h);
    copy_out(h, microsec_id, h->s.m_micro, 4 * n * 2, mem);
    copy_out(h, angle, h->s.m_angle, 4 * n * 2, mem);
    copy_out(h, rpm, h->s.m_rpm, 4 * n * 2, mem);
    copy_out(h, curr, h->s.m_curr, 4 * n * 2, mem);
    if (dlt_out_angle_rad) {
      float *dst = mem == FMSKF_MEM_DEVICE ? dlt_out_angle_rad : (float *)h->out_for(4 * n * 4);
      launch_check(launch_motor_dlt(h->s.m_angle, h->s.m_prev, dst, 4 * n, h->stream), "motor dlt");
      if (mem == FMSKF_MEM_HOST) copy_out(h, dlt_out_angle_rad, dst, 4 * n * 4, mem);
    }
    // Status::flt_SpeedRadPS [N][4] from the IIR1 output planes [4][N]
    if (speed_radps) {
      if (mem == FMSKF_MEM_HOST) {
        std::vector<float> pl(4 * n);
        copy_out(h, pl.data(), h->s.m_iir_y, 4 * n * 4, mem);
        hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
        for (uint64_t i = 0; i < n; i++)
          for (int w = 0; w < 4; w++) speed_radps[4 * i + w] = pl[(size_t)w * n + i];
      } else {  // one strided copy per wheel: plane w -> column w
        for (int w = 0; w < 4; w++)
          hip_check(hipMemcpy2DAsync(speed_radps + w, 16, h->s.m_iir_y + (size_t)w * n, 4, 4, n,
                                     hipMemcpyDeviceToDevice, h->stream),
                    "speed transpose");
      }
    }
    finish_out(h, mem);
  });
}

int fmskf_get_state_lo(fmskf_handle h, float *lo, uint32_t *rows, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const uint32_t rh = h->s.thlo ? 1u : 0u, rx = h->s.xlo ? kKf6LoRows : 0u;
    if (rows) *rows = rh + rx;
    if (!lo || !(rh + rx)) return;
    if (rh) copy_out(h, lo, h->s.thlo, n * 4, mem);
    if (rx) {
      float *dst = lo + (size_t)rh * n;
      void *dense = mem == FMSKF_MEM_DEVICE ? (void *)dst : h->out_for((size_t)rx * n * 4);
      launch_check(launch_untile(h->s.xlo, dense, rx, n, 4, h->stream), "untile");
      if (mem == FMSKF_MEM_HOST) copy_out(h, dst, dense, (size_t)rx * n * 4, mem);
    }
    finish_out(h, mem);
  });
}

int fmskf_set_state_lo(fmskf_handle h, const float *lo, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    if (!lo) fail(FMSKF_EINVAL, "null lo");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    const uint32_t rh = h->s.thlo ? 1u : 0u, rx = h->s.xlo ? kKf6LoRows : 0u, r = rh + rx;
    if (!r) fail(FMSKF_ENOTSUP, "this model keeps no low-part rows");
    const float *src = lo;
    if (mem == FMSKF_MEM_HOST) {
      void *stg = h->stage_for((size_t)r * n * 4);
      hip_check(hipMemcpyAsync(stg, lo, (size_t)r * n * 4, hipMemcpyHostToDevice, h->stream), "stage H2D");
      src = (const float *)stg;
    }
    if (rh) hip_check(hipMemcpyAsync(h->s.thlo, src, n * 4, hipMemcpyDeviceToDevice, h->stream), "lo");
    if (rx) launch_check(launch_tile(src + (size_t)rh * n, h->s.xlo, rx, n, 4, h->stream), "tile");
    h->ens_shift_ok = false;
    finish_out(h, FMSKF_MEM_HOST);
  });
}

int fmskf_get_counters(fmskf_handle h, uint64_t *counters, uint32_t n_counters) {
  return guarded([&] {
    check_handle(h);
    if (!counters || n_counters == 0) return;
    DeviceGuard g(h->cfg.device);
    unsigned long long tmp[8];
    hip_check(hipMemcpyAsync(tmp, h->s.counters, sizeof(tmp), hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipStreamSynchronize(h->stream), "sync");
    for (uint32_t k = 0; k < n_counters && k < 8; k++) counters[k] = tmp[k];
  });
}

int fmskf_ensemble_record_len(fmskf_handle h, uint32_t *len) {
  return guarded([&] {
    check_handle(h);
    if (!len) fail(FMSKF_EINVAL, "null len");
    const uint32_t nx = h->d.nx;
    *len = 1 + nx + nx * (nx + 1) / 2;
  });
}

int fmskf_ensemble_partial(fmskf_handle h, double *out, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    DeviceGuard g(h->cfg.device);
    const uint32_t nx = h->d.nx;
    const uint32_t len = 1 + nx + nx * (nx + 1) / 2;
    double *dst = mem == FMSKF_MEM_DEVICE ? out : h->ens_out;
    ensure_shift(h);
    launch_check(launch_ensemble(h->s, (int)nx, h->d.elem == 8, h->ens_blocks, h->ens_shift, dst,
                                 h->stream),
                 "ensemble launch");
    if (mem == FMSKF_MEM_HOST) {
      copy_out(h, out, h->ens_out, len * 8, mem);
      finish_out(h, mem);
    } else if (mem != FMSKF_MEM_DEVICE) {
      fail(FMSKF_EINVAL, "bad mem flag");
    }
  });
}

int fmskf_tick_ensemble(fmskf_handle h, const fmskf_tick_inputs *in, double *out, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    const uint32_t nx = h->d.nx;
    const uint32_t len = 1 + nx + nx * (nx + 1) / 2;
    double *dst = mem == FMSKF_MEM_DEVICE ? out : h->ens_out;
    ensure_shift(h);
    if (fused_record(h)) {
      // one kernel: the tick writes each block's record of the state it just stored (no
      // second pass over x), then the fold
      TickIn t = resolve_inputs(h, in, true, true, 1, h->s.n);
      t.ens_blocks = h->ens_blocks;
      t.ens_shift = h->ens_shift;
      int nb = 0;
      const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
      h->time_begin();
      if (h->cfg.model == FMSKF_MODEL_KF6)
        launch_check(launch_kf6(h->s, t, h->kf6, libm, true, true, h->stream, &nb), "tick kernel launch");
      else if (h->cfg.model == FMSKF_MODEL_EKF9)
        launch_check(launch_ekf9(h->s, t, h->ekf9, libm, true, true, h->stream, &nb), "tick kernel launch");
      else
        launch_check(launch_kf12d(h->s, t, h->kf12, true, true, h->stream, &nb), "tick kernel launch");
      h->time_end();
      launch_check(launch_ens_fold((int)nx, h->ens_blocks, nb, h->ens_shift, dst, h->stream),
                   "ensemble fold launch");
    } else {
      run_tick(h, in, true, true, 1, h->s.n);
      launch_check(launch_ensemble(h->s, (int)nx, h->d.elem == 8, h->ens_blocks, h->ens_shift, dst,
                                   h->stream),
                   "ensemble launch");
    }
    if (mem == FMSKF_MEM_HOST) {
      copy_out(h, out, h->ens_out, len * 8, mem);
      finish_out(h, mem);
    }
  });
}

int fmskf_ensemble_combine(uint32_t n_state, const double *records, uint32_t n_records,
                           double *mean, double *cov_packed) {
  return guarded([&] {
    if (n_state == 0 || n_state > 12 || !records) fail(FMSKF_EINVAL, "bad arguments");
    const uint32_t nx = n_state, np = nx * (nx + 1) / 2, len = 1 + nx + np;
    std::vector<double> acc(len, 0.0);
    for (uint32_t r = 0; r < n_records; r++) {  // fixed rank order: deterministic
      const double *b = records + (size_t)r * len;
      const double na = acc[0], nb = b[0];
      if (nb == 0.0) continue;
      if (na == 0.0) {
        acc.assign(b, b + len);
        continue;
      }
      const double nn = na + nb;
      double d[12];
      for (uint32_t k = 0; k < nx; k++) d[k] = b[1 + k] - acc[1 + k];
      const double f = na * nb / nn;
      for (uint32_t k = 0; k < nx; k++) acc[1 + k] = acc[1 + k] + d[k] * (nb / nn);
      for (uint32_t p = 0; p < nx; p++)
        for (uint32_t q = 0; q <= p; q++) {
          const uint32_t k = p * (p + 1) / 2 + q;
          acc[1 + nx + k] = acc[1 + nx + k] + b[1 + nx + k] + d[p] * d[q] * f;
        }
      acc[0] = nn;
    }
    if (mean)
      for (uint32_t k = 0; k < nx; k++) mean[k] = acc[1 + k];
    if (cov_packed)
      for (uint32_t k = 0; k < np; k++) cov_packed[k] = acc[0] > 1.0 ? acc[1 + nx + k] / (acc[0] - 1.0) : 0.0;
  });
}

}  // extern "C"

// ============================================================================
// native multi-GPU ensemble over RCCL
// ============================================================================
namespace {

// RCCL entry points, resolved once from librccl.so.1 (the copy torch already loaded, if any)
struct RcclApi {
  bool ok = false;
  std::string why;
  std::string path;  // the file the entry points came from (dladdr)
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int *) = nullptr;
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int *) = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};

const RcclApi &rccl() {
  static RcclApi api = [] {
    RcclApi a;
    // FMSKF_RCCL_LIBRARY names the tests' one-GPU loopback stand-in (tests/native/
    // loopback_rccl.cpp), used alone, without falling back.  Only a library that exports the
    // stand-in's marker symbol is accepted, so the environment cannot swap a deployed
    // controller's collective for another implementation.
    const char *alt = getenv("FMSKF_RCCL_LIBRARY");
    void *lib = nullptr;
    if (alt && *alt) {
      lib = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
      if (lib && !dlsym(lib, "fmskf_rccl_stand_in")) {
        dlclose(lib);
        a.why = std::string("FMSKF_RCCL_LIBRARY=") + alt + " is not the test stand-in (no fmskf_rccl_stand_in)";
        return a;
      }
    } else {
      lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (!lib) {
      a.why = std::string("cannot load librccl.so.1: ") + dlerror();
      return a;
    }
    a.get_unique_id = (decltype(a.get_unique_id))dlsym(lib, "ncclGetUniqueId");
    a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(lib, "ncclCommInitRank");
    a.comm_destroy = (decltype(a.comm_destroy))dlsym(lib, "ncclCommDestroy");
    a.all_gather = (decltype(a.all_gather))dlsym(lib, "ncclAllGather");
    a.comm_count = (decltype(a.comm_count))dlsym(lib, "ncclCommCount");
    a.comm_user_rank = (decltype(a.comm_user_rank))dlsym(lib, "ncclCommUserRank");
    a.error_string = (decltype(a.error_string))dlsym(lib, "ncclGetErrorString");
    a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_gather && a.comm_count &&
           a.comm_user_rank && a.error_string;
    if (!a.ok) a.why = "librccl.so.1 lacks an entry point";
    Dl_info di{};
    if (a.all_gather && dladdr((void *)a.all_gather, &di) && di.dli_fname) a.path = di.dli_fname;
    return a;
  }();
  return api;
}

const RcclApi &need_rccl() {
  const RcclApi &a = rccl();
  if (!a.ok) fail(FMSKF_ERCCL, a.why);
  return a;
}

void nccl_check(ncclResult_t r, const char *what) {
  if (r != ncclSuccess) fail(FMSKF_ERCCL, std::string(what) + ": " + rccl().error_string(r));
}

// behind the fold queued on the tick stream, on the side stream: ncclAllGather of the slot's
// record over the handle's communicator, one D2H of the gathered records, the slot's event
void ens_gather_async(fmskf_ctx *h, fmskf_ctx::EnsSlot &S) {
  if (!h->ens_stream) {
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&h->ens_stream, hipStreamNonBlocking, hi), "hipStreamCreate");
    hip_check(hipEventCreateWithFlags(&h->ens_ticked, kSyncEvent), "hipEventCreate");
  }
  const uint32_t nx = h->d.nx, len = 1 + nx + nx * (nx + 1) / 2;
  hip_check(hipEventRecord(h->ens_ticked, h->stream), "hipEventRecord");
  hip_check(hipStreamWaitEvent(h->ens_stream, h->ens_ticked, 0), "hipStreamWaitEvent");
  nccl_check(need_rccl().all_gather(S.rec, S.gather, len, ncclFloat64, h->comm, h->ens_stream),
             "ncclAllGather");
  hip_check(hipMemcpyAsync(S.host, S.gather, (size_t)S.ranks * len * 8, hipMemcpyDeviceToHost, h->ens_stream),
            "D2H");
  hip_check(hipEventRecord(S.done, h->ens_stream), "hipEventRecord");
}

}  // namespace

void fmskf_ctx::destroy_comm() {
  if (comm) {
    (void)rccl().comm_destroy(comm);
    comm = nullptr;
  }
}

extern "C" {

int fmskf_comm_unique_id(uint8_t id[FMSKF_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == FMSKF_COMM_ID_BYTES, "RCCL unique id size");
  return guarded([&] {
    if (!id) fail(FMSKF_EINVAL, "null id");
    ncclUniqueId u;
    nccl_check(need_rccl().get_unique_id(&u), "ncclGetUniqueId");
    memcpy(id, &u, sizeof(u));
  });
}

int fmskf_comm_init(fmskf_handle h, const uint8_t id[FMSKF_COMM_ID_BYTES], int rank, int world) {
  return guarded([&] {
    check_handle(h);
    if (!id || world < 1 || rank < 0 || rank >= world) fail(FMSKF_EINVAL, "bad rank / world / id");
    // a pending asynchronous result may still be gathered over the old communicator
    if (h->ens_pending) fail(FMSKF_EINVAL, "collect the pending ensemble results (fmskf_ensemble_end) first");
    const RcclApi &a = need_rccl();
    DeviceGuard g(h->cfg.device);
    h->destroy_comm();
    h->rank = 0;
    h->world = 1;
    // the gather buffer is reused while the new world fits it (re-initialising does not leak)
    if ((size_t)world > h->ens_gather_cap) {
      double *buf = h->alloc<double>((size_t)world * 91);
      h->release(h->ens_gather);
      h->ens_gather = buf;
      h->ens_gather_cap = (size_t)world;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    nccl_check(a.comm_init_rank(&c, world, u, rank), "ncclCommInitRank");
    h->comm = c;
    h->rank = rank;
    h->world = world;
  });
}

int fmskf_comm_info(fmskf_handle h, int *world, int *rank) {
  return guarded([&] {
    check_handle(h);
    if (!h->comm) fail(FMSKF_EINVAL, "the handle has no communicator (fmskf_comm_init)");
    const RcclApi &a = need_rccl();
    int w = 0, r = -1;
    nccl_check(a.comm_count(h->comm, &w), "ncclCommCount");
    nccl_check(a.comm_user_rank(h->comm, &r), "ncclCommUserRank");
    if (world) *world = w;
    if (rank) *rank = r;
  });
}

const char *fmskf_rccl_library(void) {
  static std::string path;
  try {
    path = rccl().path;
  } catch (...) {
    path.clear();
  }
  return path.c_str();
}

int fmskf_ensemble_stats(fmskf_handle h, double *mean, double *cov_packed) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    const uint32_t nx = h->d.nx, len = 1 + nx + nx * (nx + 1) / 2;
    ensure_shift(h);
    launch_check(launch_ensemble(h->s, (int)nx, h->d.elem == 8, h->ens_blocks, h->ens_shift, h->ens_out,
                                 h->stream),
                 "ensemble launch");
    const double *src = h->ens_out;
    int ranks = 1;
    if (h->comm) {
      nccl_check(need_rccl().all_gather(h->ens_out, h->ens_gather, len, ncclFloat64, h->comm,
                                        h->stream),
                 "ncclAllGather");
      src = h->ens_gather;
      ranks = h->world;
    }
    std::vector<double> recs((size_t)ranks * len);
    hip_check(hipMemcpyAsync(recs.data(), src, recs.size() * 8, hipMemcpyDeviceToHost, h->stream),
              "D2H");
    hip_check(hipStreamSynchronize(h->stream), "hipStreamSynchronize");
    const int rc = fmskf_ensemble_combine(nx, recs.data(), (uint32_t)ranks, mean, cov_packed);
    if (rc != FMSKF_OK) fail(rc, "ensemble combine");
  });
}

}  // extern "C"

namespace {

// One asynchronous ensemble event (the record fused into the tick, the fold
// and the gather off the tick's critical path).  On the handle's stream: the tick whose kernel
// writes the slot's block records and, in LEN blocks ahead of its tick blocks, folds the
// PREVIOUS event's records (ens_fold_front) | the stand-alone partial.  The previous event's fold is
// then queued: its `done` event (one GPU: the fold wrote the pinned host slot itself) or, with
// a communicator, the all-gather and D2H on the side stream.  This event's own fold waits for
// the next event's tick kernel, or runs stand-alone ahead of a plain tick, at
// fmskf_ensemble_end or before a shift rewrite (ens_flush).
// Nothing waits on the host.

void ens_async_begin(fmskf_ctx *h, const fmskf_tick_inputs *in) {
  check_handle(h);
  if (h->capturing) fail(FMSKF_EINVAL, "asynchronous ensemble inside a graph capture");
  if (h->ens_pending == fmskf_ctx::kEnsSlots)
    fail(FMSKF_EINVAL, "four ensemble results pending: call fmskf_ensemble_end first");
  DeviceGuard g(h->cfg.device);
  const uint32_t nx = h->d.nx, len = 1 + nx + nx * (nx + 1) / 2;
  const int ranks = h->comm ? h->world : 1;
  const int si = (h->ens_head + h->ens_pending) % fmskf_ctx::kEnsSlots;
  fmskf_ctx::EnsSlot &S = h->eslot[si];
  if (!S.blocks) {
    size_t nb = (size_t)ensemble_nblocks(h->s.n);
    nb = std::max(nb, (size_t)((h->s.n + kBlock - 1) / kBlock));
    S.blocks = h->alloc<double>(nb * len);
    S.rec = h->alloc<double>(91);
    hip_check(hipEventCreateWithFlags(&S.done, kSyncEvent), "hipEventCreate");
  }
  if ((size_t)ranks > S.cap) {  // the slot's previous result was consumed (or never existed)
    double *gbuf = h->alloc<double>((size_t)ranks * 91);
    if (S.gather) h->release(S.gather);
    S.gather = gbuf;
    if (S.host) hip_check(hipHostFree(S.host), "hipHostFree");
    S.host = nullptr;
    // coherent (fine-grained): the fold's stores to it are not held in the GPU's L2
    hip_check(hipHostMalloc((void **)&S.host, (size_t)ranks * 91 * 8, hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc");
    S.host_dev = (double *)fmskf_ctx::dev_ptr(S.host);
    S.cap = (size_t)ranks;
  }
  ensure_shift(h);  // queues the previous event's fold first if it rewrites the shift
  int nb = 0;
  if (in && fused_record(h)) {
    TickIn t = resolve_inputs(h, in, true, true, 1, h->s.n);
    t.ens_blocks = S.blocks;
    t.ens_shift = h->ens_shift;
    fmskf_ctx::EnsSlot *C = h->ens_carry >= 0 ? &h->eslot[h->ens_carry] : nullptr;
    if (C) {
      t.fold_blocks = C->blocks;
      t.fold_nb = (uint32_t)C->nb;
      t.fold_out = ens_fold_dst(h, *C);
      // one GPU, untimed: the carrying kernel's own completion records C's event
      if (!h->comm && !h->timing) t.ens_done = C->done;
    }
    const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
    h->time_begin();
    int e = 0;
    if (h->cfg.model == FMSKF_MODEL_KF6) e = launch_kf6(h->s, t, h->kf6, libm, true, true, h->stream, &nb);
    else if (h->cfg.model == FMSKF_MODEL_EKF9) e = launch_ekf9(h->s, t, h->ekf9, libm, true, true, h->stream, &nb);
    else e = launch_kf12d(h->s, t, h->kf12, true, true, h->stream, &nb);
    launch_check(e, "tick kernel launch");
    h->time_end();
    if (C) {
      if (t.ens_done) h->ens_carry = -1;  // recorded by the kernel's completion signal
      else ens_fold_queued(h, *C);
    }
  } else {
    ens_flush(h);
    if (in) run_tick(h, in, true, true, 1, h->s.n);
    launch_check(launch_ens_partial(h->s, (int)nx, h->d.elem == 8, S.blocks, h->ens_shift, h->stream, &nb),
                 "ensemble partial launch");
  }
  S.nb = nb;
  S.ranks = ranks;
  h->ens_carry = si;
  h->ens_pending++;
}

}  // namespace

extern "C" {

int fmskf_tick_ensemble_begin(fmskf_handle h, const fmskf_tick_inputs *in) {
  return guarded([&] {
    if (!in) fail(FMSKF_EINVAL, "null inputs");
    ens_async_begin(h, in);
  });
}

int fmskf_ensemble_begin(fmskf_handle h) {
  return guarded([&] { ens_async_begin(h, nullptr); });
}

int fmskf_ensemble_end(fmskf_handle h, double *mean, double *cov_packed) {
  return fmskf_ensemble_end_count(h, mean, cov_packed, nullptr, nullptr);
}

int fmskf_ensemble_end_count(fmskf_handle h, double *mean, double *cov_packed, double *count,
                             uint32_t *n_records) {
  return guarded([&] {
    check_handle(h);
    if (h->ens_pending == 0) fail(FMSKF_EINVAL, "no ensemble pending (fmskf_*ensemble_begin)");
    DeviceGuard g(h->cfg.device);
    fmskf_ctx::EnsSlot &S = h->eslot[h->ens_head];
    if (h->ens_carry == h->ens_head) {  // no later tick kernel carried its fold: queue it now
      if (h->capturing) fail(FMSKF_EINVAL, "the newest ensemble result collected inside a graph capture");
      ens_flush(h);
    }
    hip_check(hipEventSynchronize(S.done), "hipEventSynchronize");
    h->ens_head = (h->ens_head + 1) % fmskf_ctx::kEnsSlots;
    h->ens_pending--;
    const int rc = fmskf_ensemble_combine(h->d.nx, S.host, (uint32_t)S.ranks, mean, cov_packed);
    if (rc != FMSKF_OK) fail(rc, "ensemble combine");
    // what the gathered records themselves count: every rank's robots, once each
    const uint32_t len = 1 + h->d.nx + h->d.nx * (h->d.nx + 1) / 2;
    double c = 0.0;
    for (int r = 0; r < S.ranks; r++) c += S.host[(size_t)r * len];
    if (count) *count = c;
    if (n_records) *n_records = (uint32_t)S.ranks;
  });
}

}  // extern "C"

// ============================================================================
// vehicle control step, CAN TX, VehicleInfo export
// ============================================================================
namespace {

void ctrl_params_defaults(fmskf_ctrl_params *p) {
  memset(p, 0, sizeof(*p));
  p->ctrl_freq_hz = 100.0f;  // U32_VD_TASK_CTRL_FREQ_HZ (VD_task_main.cpp:23,86-89)
  p->ff_gain = 0.0075f;
  p->p_gain = 0.02f;
  p->i_gain = 0.01f;
  p->d_gain = 0.0f;
  p->i_limit = 0.5f;
  p->lpf_freq_hz = 10.0f;
  p->ff_limit = 1.0f;                            // VD_task_main.cpp:157-160
  p->interp_ts = 1.0f / (float)1000;             // VD_task_main.cpp:95-97
  p->curr_limit_raw = 3000;                      // VD_motor_if_m2006.hpp:62
}

// the device parameter block, computed like the reference's constructors
// (util_controller.hpp:10,96-101: dt_ = 1.0f / freq, the IIR1 coefficients in float)
CtrlPrm make_ctrl_prm(const fmskf_ctx *h) {
  const fmskf_ctrl_params &c = h->cprm;
  CtrlPrm p{};
  p.freq = c.ctrl_freq_hz;
  p.dt = 1.0f / c.ctrl_freq_hz;
  p.ff_gain = c.ff_gain;
  p.p_gain = c.p_gain;
  p.i_gain = c.i_gain;
  p.d_gain = c.d_gain;
  p.i_limit = c.i_limit;
  p.ff_limit = c.ff_limit;
  p.a1 = (2.0f * c.ctrl_freq_hz - c.lpf_freq_hz) / (2.0f * c.ctrl_freq_hz + c.lpf_freq_hz);
  p.b0 = c.lpf_freq_hz / (2.0f * c.ctrl_freq_hz + c.lpf_freq_hz);
  p.b1 = c.lpf_freq_hz / (2.0f * c.ctrl_freq_hz + c.lpf_freq_hz);
  p.ts = c.interp_ts;
  p.curr_limit = c.curr_limit_raw;
  for (int w = 0; w < 4; w++) p.dir[w] = h->cfg.motor_dir[w];
  return p;
}

void zero_ctrl(fmskf_ctx *h) {
  CtrlDev &c = h->ctrl;
  hip_check(hipMemsetAsync(c.ax, 0, (size_t)3 * kAxF * c.pitch * 4, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.pid, 0, (size_t)4 * kPidF * c.pitch * 4, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.vel_tgt, 0, (size_t)3 * c.pitch * 4, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.curr, 0, (size_t)4 * c.n * 2, h->stream), "ctrl init");
  hip_check(hipMemsetAsync(c.power, 0, (size_t)c.n, h->stream), "ctrl init");
  ctrl_params_defaults(&h->cprm);
}

void ensure_ctrl(fmskf_ctx *h) {
  if (h->ctrl_ready) return;
  CtrlDev &c = h->ctrl;
  c.n = h->s.n;
  // tiled interpolator / FF_PI_D arrays cover ceil(N / W) whole tiles (ctrl_lane.hpp Planes)
  const uint64_t w = tile_w_elem(4);
  c.pitch = FMSKF_CTRL_TILED ? std::max(h->s.pitch, (c.n + w - 1) / w * w) : h->s.pitch;
  c.ax = h->alloc<float>((size_t)3 * kAxF * c.pitch);
  c.pid = h->alloc<float>((size_t)4 * kPidF * c.pitch);
  c.vel_tgt = h->alloc<float>((size_t)3 * c.pitch);
  c.curr = h->alloc<int16_t>((size_t)4 * c.n);
  c.power = h->alloc<uint8_t>((size_t)c.n);
  zero_ctrl(h);
  h->ctrl_ready = true;
}

}  // namespace

extern "C" {

int fmskf_ctrl_params_init(fmskf_ctrl_params *p) {
  return guarded([&] {
    if (!p) fail(FMSKF_EINVAL, "null params");
    ctrl_params_defaults(p);
  });
}

int fmskf_set_ctrl_params(fmskf_handle h, const fmskf_ctrl_params *p) {
  return guarded([&] {
    check_handle(h);
    if (!p) fail(FMSKF_EINVAL, "null params");
    if (!(p->ctrl_freq_hz > 0.0f) || !(p->interp_ts > 0.0f) || p->curr_limit_raw < 0)
      fail(FMSKF_EINVAL, "ctrl params: freq and ts must be > 0, current limit >= 0");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    h->cprm = *p;
  });
}

int fmskf_set_power(fmskf_handle h, const uint8_t *on, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const uint64_t n = h->s.n;
    if (!on) {
      hip_check(hipMemsetAsync(h->ctrl.power, 1, n, h->stream), "power");
      return;
    }
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    hip_check(hipMemcpyAsync(h->ctrl.power, on, n,
                             mem == FMSKF_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                             h->stream),
              "power");
    finish_out(h, mem);  // the caller's host buffer may be reused on return
  });
}

int fmskf_set_target_vel(fmskf_handle h, const float *vel, const float *acl, const float *jrk,
                         const uint8_t *mask, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!vel || !acl || !jrk) fail(FMSKF_EINVAL, "null vel/acl/jrk");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const uint64_t n = h->s.n;
    Stager sg(h, mem);
    const void *v = vel, *a = acl, *j = jrk, *m = mask;
    sg.add(&v, 3 * n * 4);
    sg.add(&a, 3 * n * 4);
    sg.add(&j, 3 * n * 4);
    sg.add(&m, n);
    sg.run();
    launch_check(launch_ctrl_set_target(h->ctrl, (const float *)v, (const float *)a,
                                        (const float *)j, (const uint8_t *)m, h->stream),
                 "set_target_vel launch");
  });
}

int fmskf_control(fmskf_handle h, const int16_t *rpm, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const void *r = rpm;
    if (r) {
      Stager sg(h, mem);
      sg.add(&r, h->s.n * 8);
      sg.run();
    } else {
      ensure_motors(h);
      r = h->s.m_rpm;
    }
    h->time_begin();
    launch_check(launch_ctrl_step(h->ctrl, make_ctrl_prm(h), (const int16_t *)r, 1, h->stream),
                 "control launch");
    h->time_end();
  });
}

int fmskf_can_tx(fmskf_handle h, uint8_t *frames, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!frames) fail(FMSKF_EINVAL, "null frames");
    if (mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const size_t bytes = h->s.n * 8;
    uint8_t *dst = mem == FMSKF_MEM_DEVICE ? frames : (uint8_t *)host_result(h, bytes);
    launch_check(launch_can_tx(h->ctrl, dst, h->stream), "can_tx launch");
    copy_out_sync(h, frames, dst, bytes, mem);
  });
}

// FMSKF_ISR_FUSED=0: the KF6 ISR as three kernels (A/B, and the tests' cross-check)
static bool isr_kf6_fused() {
  static const bool v = [] {
    const char *e = getenv("FMSKF_ISR_FUSED");
    return !e || atoi(e) != 0;
  }();
  return v;
}

int fmskf_isr_tick(fmskf_handle h, const fmskf_tick_inputs *in, uint8_t *frames, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (frames && mem != FMSKF_MEM_HOST && mem != FMSKF_MEM_DEVICE) fail(FMSKF_EINVAL, "bad mem flag");
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const uint64_t n = h->s.n;
    TickIn t = resolve_inputs(h, in, true, true, 1, n);
    const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
    const size_t bytes = n * 8;
    uint8_t *dst = !frames ? nullptr : mem == FMSKF_MEM_DEVICE ? frames : (uint8_t *)host_result(h, bytes);
    const CtrlPrm p = make_ctrl_prm(h);
    h->time_begin();
    int fused = (int)hipErrorNotSupported;
    if (h->cfg.model == FMSKF_MODEL_KF6 && isr_kf6_fused()) {
      if (!t.rec && !t.rpm) ensure_motors(h);
      fused = launch_isr_kf6(h->s, t, h->kf6, libm, h->ctrl, p, dst, h->stream);
      if (fused != (int)hipErrorNotSupported) launch_check(fused, "isr launch");
    }
    if (h->cfg.model == FMSKF_MODEL_RS) {
      launch_check(launch_isr_rs(h->s, t, libm, h->ctrl, p, dst, h->stream), "isr launch");
    } else if (fused == (int)hipErrorNotSupported) {  // estimator tick, then the control step and the frame (three launches)
      int e = 0;
      switch (h->cfg.model) {
        case FMSKF_MODEL_KF6: e = launch_kf6(h->s, t, h->kf6, libm, true, true, h->stream); break;
        case FMSKF_MODEL_EKF9: e = launch_ekf9(h->s, t, h->ekf9, libm, true, true, h->stream); break;
        case FMSKF_MODEL_KF12D: e = launch_kf12d(h->s, t, h->kf12, true, true, h->stream); break;
      }
      launch_check(e, "tick kernel launch");
      if (!t.rec && !t.rpm) ensure_motors(h);
      const int16_t *rpm = t.rec ? (const int16_t *)(t.rec + 2) : t.rpm ? t.rpm : h->s.m_rpm;
      launch_check(launch_ctrl_step(h->ctrl, p, rpm, t.rec ? 2 : 1, h->stream), "control launch");
      if (dst) launch_check(launch_can_tx(h->ctrl, dst, h->stream), "can_tx launch");
    }
    h->time_end();
    if (frames) copy_out_sync(h, frames, dst, bytes, mem);
  });
}

int fmskf_get_ctrl(fmskf_handle h, float *vel_tgt, int16_t *curr_raw, float *wheel_tgt,
                   float *wheel_ctrl, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    DeviceGuard g(h->cfg.device);
    ensure_ctrl(h);
    const CtrlDev &c = h->ctrl;
    const size_t row = c.n * 4, pb = c.pitch * 4;
    copy_planes_out(h, vel_tgt, c.vel_tgt, row, pb, 3, mem);
    copy_out(h, curr_raw, c.curr, c.n * 8, mem);
    // wheel w's field k is plane w*kPidF + k: planes of one field are kPidF planes apart
    const float *pid = c.pid;
    size_t ppb = pb;
    if (FMSKF_CTRL_TILED && (wheel_tgt || wheel_ctrl)) {  // dense [4 * kPidF][N] copy first
      float *dense = (float *)h->stage_for((size_t)4 * kPidF * row);
      launch_check(launch_untile(c.pid, dense, 4 * kPidF, c.n, 4, h->stream), "untile pid");
      pid = dense;
      ppb = row;
    }
    copy_planes_out(h, wheel_tgt, pid + 4 * (ppb / 4), row, ppb * kPidF, 4, mem);
    copy_planes_out(h, wheel_ctrl, pid + 5 * (ppb / 4), row, ppb * kPidF, 4, mem);
    finish_out(h, mem);
  });
}

int fmskf_export_vehicle_info(fmskf_handle h, fmskf_vehicle_info *out, const uint8_t *floor,
                              const float *cam_pitch, const uint32_t *fault, uint32_t mem) {
  static_assert(sizeof(fmskf_vehicle_info) == 84, "VehicleInfo record layout");
  return guarded([&] {
    check_handle(h);
    if (!out) fail(FMSKF_EINVAL, "null out");
    DeviceGuard g(h->cfg.device);
    const uint64_t n = h->s.n;
    ensure_imu(h);
    Stager sg(h, mem);
    const void *f = floor, *c = cam_pitch, *u = fault;
    sg.add(&f, n * 8);
    sg.add(&c, n * 4);
    sg.add(&u, n * 4);
    sg.run();
    launch_check(launch_readout(h->s, h->readout, h->stream), "readout");
    const size_t bytes = n * sizeof(fmskf_vehicle_info);
    void *dst = mem == FMSKF_MEM_DEVICE ? (void *)out : host_result(h, bytes);
    launch_check(launch_vehicle_info(h->s, h->readout, dst, (const uint8_t *)f, (const float *)c,
                                     (const uint32_t *)u, h->stream),
                 "vehicle_info launch");
    copy_out_sync(h, out, dst, bytes, mem);
  });
}

int fmskf_eval_trig(fmskf_handle h, const float *x, float *s, float *c, uint64_t n, uint32_t mem) {
  return guarded([&] {
    check_handle(h);
    if (!x || !s || !c) fail(FMSKF_EINVAL, "null argument");
    DeviceGuard g(h->cfg.device);
    const bool libm = h->cfg.trig == FMSKF_TRIG_LIBM;
    if (mem == FMSKF_MEM_DEVICE) {
      launch_check(launch_trig(x, s, c, n, libm, h->s.sintab, h->stream), "trig launch");
      return;
    }
    if (mem != FMSKF_MEM_HOST) fail(FMSKF_EINVAL, "bad mem flag");
    if (n == 0) return;
    char *buf = (char *)h->stage_for(3 * n * 4);
    float *dx = (float *)buf, *ds = dx + n, *dc = ds + n;
    hip_check(hipMemcpyAsync(dx, x, n * 4, hipMemcpyHostToDevice, h->stream), "H2D");
    launch_check(launch_trig(dx, ds, dc, n, libm, h->s.sintab, h->stream), "trig launch");
    hip_check(hipMemcpyAsync(s, ds, n * 4, hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipMemcpyAsync(c, dc, n * 4, hipMemcpyDeviceToHost, h->stream), "D2H");
    hip_check(hipStreamSynchronize(h->stream), "sync");
  });
}

int fmskf_set_timing(fmskf_handle h, int enable) {
  return guarded([&] {
    check_handle(h);
    h->timing = enable != 0;
    h->tcount = 0;
  });
}

int fmskf_kernel_time_total(fmskf_handle h, double *total_ms, uint32_t *count) {
  return guarded([&] {
    check_handle(h);
    if (!total_ms || !count) fail(FMSKF_EINVAL, "null argument");
    DeviceGuard g(h->cfg.device);
    double sum = 0.0;
    if (h->tcount) hip_check(hipEventSynchronize(h->tpool[2 * h->tcount - 1]), "hipEventSynchronize");
    for (size_t k = 0; k < h->tcount; k++) {
      float ms = 0.f;
      hip_check(hipEventElapsedTime(&ms, h->tpool[2 * k], h->tpool[2 * k + 1]), "hipEventElapsedTime");
      sum += ms;
    }
    *total_ms = sum;
    *count = (uint32_t)h->tcount;
  });
}

int fmskf_last_kernel_ms(fmskf_handle h, float *ms) {
  return guarded([&] {
    check_handle(h);
    if (!ms) fail(FMSKF_EINVAL, "null ms");
    if (!h->timing) fail(FMSKF_EINVAL, "timing not enabled");
    DeviceGuard g(h->cfg.device);
    hip_check(hipEventSynchronize(h->ev1), "hipEventSynchronize");
    hip_check(hipEventElapsedTime(ms, h->ev0, h->ev1), "hipEventElapsedTime");
  });
}

}  // extern "C"
