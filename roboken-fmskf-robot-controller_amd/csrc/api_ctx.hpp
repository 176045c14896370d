// api_ctx.hpp -- the C-ABI layer's shared internals: the handle (struct fmskf_ctx), error
// plumbing (every failure becomes a status code, no exception crosses the ABI), host staging,
// and the helpers the api_*.cpp translation units share.  Not part of the public ABI.
//   api_handle.cpp      lifecycle, staging, ingest, tick entry points, state get / set
//   api_checkpoint.cpp  fmskf_save_state / fmskf_load_state
//   api_readout.cpp     readouts of the ingest state, counters, synchronous ensemble records
//   api_comm.cpp        RCCL (dlopen), the communicator, the asynchronous ensemble exchange
//   api_ctrl.cpp        control step, CAN TX, the fused ISR, VehicleInfo, timing
#pragma once
#include "../../include/fmskf.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "fmskf_internal.hpp"

namespace fmskf {
namespace capi {

extern thread_local std::string g_last_error;

struct ApiError {
  int code;
  std::string msg;
};

[[noreturn]] inline void fail(int code, const std::string &msg) { throw ApiError{code, msg}; }

inline void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) fail(FMSKF_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
inline void launch_check(int e, const char *what) { hip_check((hipError_t)e, what); }
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

inline Dims dims_of(uint32_t model) {
  switch (model) {
    case FMSKF_MODEL_RS: return {6, 0, 4};
    case FMSKF_MODEL_KF6: return {6, 4, 4};
    case FMSKF_MODEL_EKF9: return {9, 6, 4};
    case FMSKF_MODEL_KF12D: return {12, 8, 8};
    default: fail(FMSKF_EINVAL, "unknown model");
  }
}

}  // namespace capi
}  // namespace fmskf


struct fmskf_ctx {
  fmskf_config cfg{};
  fmskf::capi::Dims d{};
  fmskf::DevState s{};
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
    // timing events around the side stream's all-gather + copy-out (fmskf_ensemble_exchange_ms)
    hipEvent_t x0 = nullptr, x1 = nullptr;
    bool exchanged = false;  // the pending result went through the side stream
    int nb = 0;              // the event's block records
    int ranks = 1;
  } eslot[kEnsSlots];
  hipEvent_t ens_ticked = nullptr;  // the tick stream's point the side stream waits for
  hipStream_t ens_stream = nullptr;
  int ens_head = 0, ens_pending = 0;
  int ens_carry = -1;  // the newest event's slot while its fold is not queued yet
  float ens_xms = -1.f;  // the last collected result's exchange time (fmskf_ensemble_exchange_ms)
  // vehicle control state (allocated on first use) and its parameters
  fmskf::CtrlDev ctrl{};
  fmskf_ctrl_params cprm{};
  bool ctrl_ready = false;
  // model parameters (fp32 / fp64 copies of cfg)
  fmskf::Kf6Params kf6{};
  fmskf::Ekf9Params ekf9{};
  fmskf::Kf12dParams kf12{};
  // which launch form the firmware-ISR calls took (fmskf_get_counters [1], [2]): calls of
  // fmskf_isr_tick_can that ran the CAN RX as its own kernel before the ISR, and ISRs (of either
  // call) that ran as the tick, control-step and frame kernels instead of one fused kernel
  uint64_t isr_can_split = 0, isr_ctrl_split = 0;
  // RS: where the odometry's previous encoder sums (s64_rawAngleSumPrev) are.  rs_prev_synced:
  // they equal the motor state's sums (the last predict read those, and nothing changed them
  // since); rs_prev_stale: the prev planes are behind, the fused RS CAN ISR took the previous sums
  // from the motor state and wrote no prev (k_isr_rs PS).  stale implies synced.  Every reader of
  // the prev planes and every writer of the motor sums calls rs_prev_materialize first.
  bool rs_prev_synced = false, rs_prev_stale = false;
  // The control step's outputs nothing reads back (vel_tgt, FF_PI_D now_tgt / now_ctrl) are
  // formed on demand (round 6, ctrl_lane.hpp ctrl_derive_lane): ctrl_derived_stale says the last
  // step left them to be formed, with its parameters ctrl_prm_last.  fmskf_get_ctrl and a
  // checkpoint form them first (ctrl_materialize), and so does fmskf_set_power, since the forming
  // reads the power flags the step ran with.  Inside a graph capture the step stores them itself
  // (the host cannot follow the replays): graph_has_ctrl marks a captured sequence with a step.
  bool ctrl_derived_stale = false, graph_has_ctrl = false;
  // the motor history order (DevState::m_par) at the start and the end of the captured sequence
  uint32_t graph_par0 = 0, graph_par_end = 0;
  fmskf::CtrlPrm ctrl_prm_last{};
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
        fmskf::capi::hip_check(hipEventCreate(&e), "hipEventCreate");
        tpool.push_back(e);
      }
      fmskf::capi::hip_check(hipEventRecord(tpool[2 * tcount], stream), "hipEventRecord");
    }
    fmskf::capi::hip_check(hipEventRecord(ev0, stream), "hipEventRecord");
  }
  void time_end() {
    if (!timing) return;
    fmskf::capi::hip_check(hipEventRecord(ev1, stream), "hipEventRecord");
    if (tcount < kMaxTimed) {
      fmskf::capi::hip_check(hipEventRecord(tpool[2 * tcount + 1], stream), "hipEventRecord");
      tcount++;
    }
  }

  template <typename T>
  T *alloc(size_t count) {
    void *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(&p, count * sizeof(T));
    if (e != hipSuccess) fmskf::capi::fail(FMSKF_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    allocs.push_back(p);
    return (T *)p;
  }
  // free one allocation made by alloc() (after the stream has drained)
  void release(void *p) {
    if (!p) return;
    for (size_t i = 0; i < allocs.size(); i++)
      if (allocs[i] == p) {
        fmskf::capi::hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        (void)hipFree(p);
        allocs.erase(allocs.begin() + (long)i);
        return;
      }
  }
  void *stage_for(size_t bytes) {
    if (bytes > stage_bytes) {
      if (stage) {
        fmskf::capi::hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        fmskf::capi::hip_check(hipFree(stage), "hipFree");
        stage = nullptr;
        stage_bytes = 0;  // a failed hipMalloc below must not leave a stale capacity
      }
      hipError_t e = hipMalloc(&stage, bytes);
      if (e != hipSuccess) fmskf::capi::fail(FMSKF_ENOMEM, "staging hipMalloc failed");
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
      fmskf::capi::hip_check(hipEventRecord(pin_ev[prev], stream), "hipEventRecord");
      pin_open[prev] = false;
    }
    pin_slot ^= 1;
    if (!pin_in[slot]) {
      fmskf::capi::hip_check(hipHostMalloc(&pin_in[slot], kPinned, hipHostMallocDefault), "hipHostMalloc");
      fmskf::capi::hip_check(hipEventCreateWithFlags(&pin_ev[slot], fmskf::capi::kSyncEvent), "hipEventCreate");
    } else {
      fmskf::capi::hip_check(hipEventSynchronize(pin_ev[slot]), "hipEventSynchronize");
    }
    pin_open[slot] = true;
    return (char *)pin_in[slot];
  }
  char *pinned_out() {
    if (!pin_out) fmskf::capi::hip_check(hipHostMalloc(&pin_out, kPinned, hipHostMallocDefault), "hipHostMalloc");
    return (char *)pin_out;
  }
  // the device's address of a pinned host slot (kernels read / write it over PCIe)
  static void *dev_ptr(void *host) {
    void *d = nullptr;
    fmskf::capi::hip_check(hipHostGetDevicePointer(&d, host, 0), "hipHostGetDevicePointer");
    return d;
  }
  void destroy_comm();
  void *out_for(size_t bytes) {
    if (bytes > oscratch_bytes) {
      if (oscratch) {
        fmskf::capi::hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        fmskf::capi::hip_check(hipFree(oscratch), "hipFree");
        oscratch = nullptr;
        oscratch_bytes = 0;
      }
      hipError_t e = hipMalloc(&oscratch, bytes);
      if (e != hipSuccess) fmskf::capi::fail(FMSKF_ENOMEM, "output scratch hipMalloc failed");
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
      if (e.x0) (void)hipEventDestroy(e.x0);
      if (e.x1) (void)hipEventDestroy(e.x1);
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

namespace fmskf {
namespace capi {

inline void check_handle(fmskf_handle h) {
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

// api_handle.cpp
void zero_imu(fmskf_ctx *h);
void zero_motors(fmskf_ctx *h);
void ensure_imu(fmskf_ctx *h);
void ensure_motors(fmskf_ctx *h);
// RS: copy the motor state's sums into the prev planes if they are behind (rs_prev_stale)
void rs_prev_materialize(fmskf_ctx *h);
// extra: more host planes of the same call staged together with the tick inputs (one pinned
// slot per call: two staging rounds in one call would release the first slot before the
// kernel that reads it is queued); they must share in->mem
TickIn resolve_inputs(fmskf_ctx *h, const fmskf_tick_inputs *in, bool need_upd, bool need_pred,
                      uint32_t n_ticks, uint64_t stride,
                      const std::vector<std::pair<const void **, size_t>> *extra = nullptr);
void run_tick(fmskf_ctx *h, const fmskf_tick_inputs *in, bool upd, bool pred, uint32_t n_ticks,
              uint64_t stride);
void copy_out(fmskf_ctx *h, void *dst, const void *src, size_t bytes, uint32_t mem);
void copy_planes_out(fmskf_ctx *h, void *dst, const void *src, size_t row, size_t dev_pitch,
                     size_t planes, uint32_t mem);
void copy_planes_in(fmskf_ctx *h, void *dst, const void *src, size_t row, size_t dev_pitch,
                    size_t planes, uint32_t mem);
void finish_out(fmskf_ctx *h, uint32_t mem);
void *host_result(fmskf_ctx *h, size_t bytes);
void copy_out_sync(fmskf_ctx *h, void *dst, const void *src, size_t bytes, uint32_t mem);
// api_comm.cpp
double *ens_fold_dst(const fmskf_ctx *h, const fmskf_ctx::EnsSlot &S);
void ens_fold_queued(fmskf_ctx *h, fmskf_ctx::EnsSlot &S);
void ens_flush(fmskf_ctx *h);
void ensure_shift(fmskf_ctx *h);
bool fused_record(const fmskf_ctx *h);
// api_ctrl.cpp
void ensure_ctrl(fmskf_ctx *h);
void zero_ctrl(fmskf_ctx *h);
// form the control step's derived outputs if the last step left them (ctrl_derived_stale)
void ctrl_materialize(fmskf_ctx *h);

}  // namespace capi
}  // namespace fmskf
