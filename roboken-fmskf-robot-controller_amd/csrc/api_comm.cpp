// api_comm.cpp -- the ensemble exchange: queueing a slot's fold, RCCL resolved at run time
// (dlopen), the handle's communicator, and the asynchronous ensemble events.
#include <dlfcn.h>
#include <elf.h>

#include <atomic>

#include "api_ctx.hpp"

using namespace fmskf;
using namespace fmskf::capi;

namespace fmskf {
namespace capi {

// ---- asynchronous ensemble: queueing a slot's fold ----------------------------------------
// The fold of slot S is queued on the handle's stream (carried by a tick kernel, or
// stand-alone): with a communicator the side stream all-gathers the record over xGMI and copies
// the gathered records into the slot's pinned buffer behind it; on one GPU the fold wrote the
// pinned buffer itself.  Then the slot's `done` event.
// A communicator of one rank exchanges nothing: the all-gather of one record is that record.  So
// the side stream runs only with world > 1; at world 1 the fold writes the pinned slot as on a
// handle without a communicator.  Round 6, kbench ens_async (K = 1, 2^20 KF6, one box): the
// side-stream RCCL copy + D2H took the per-tick time from 39.2 to 82.6-91.7 us on the null
// stream (the bench line's own stream: 46.2 against 39.1 in round 5).
bool ens_exchanges(const fmskf_ctx *h) { return h->comm && h->world > 1; }
double *ens_fold_dst(const fmskf_ctx *h, const fmskf_ctx::EnsSlot &S) { return ens_exchanges(h) ? S.rec : S.host_dev; }
void ens_gather_async(fmskf_ctx *h, fmskf_ctx::EnsSlot &S);  // with the RCCL entry points below
// One GPU: the event behind the fold (the fold stored the record into the pinned slot with
// system-scope stores, ens_fold_block).  Waiting on the pinned slot itself instead of an event
// (a signalling-NaN sentinel polled by fmskf_ensemble_end) measured slower: K = 1 at 2^20
// 41.8-41.9 us per tick against 40.0-40.2 (kbench ens_async, two passes each, one box).
void ens_fold_queued(fmskf_ctx *h, fmskf_ctx::EnsSlot &S) {
  if (ens_exchanges(h)) ens_gather_async(h, S);
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

}  // namespace capi
}  // namespace fmskf

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

// Does the ELF shared object at `path` export `name` in its dynamic symbol table?  Read from the
// file, so a library that does not is refused before dlopen runs any of its constructors.
bool elf_exports(const char *path, const char *name) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  std::vector<unsigned char> img;
  unsigned char buf[1 << 16];
  size_t got;
  while ((got = fread(buf, 1, sizeof(buf), f)) > 0 && img.size() < ((size_t)256 << 20)) img.insert(img.end(), buf, buf + got);
  fclose(f);
  if (img.size() < sizeof(Elf64_Ehdr) || memcmp(img.data(), ELFMAG, SELFMAG) != 0 || img[EI_CLASS] != ELFCLASS64)
    return false;
  Elf64_Ehdr eh;
  memcpy(&eh, img.data(), sizeof(eh));
  // every extent is checked field by field against the image, never as a sum that could wrap
  // past 2^64 (a header with e_shoff or sh_offset near 2^64 is refused, not read out of bounds)
  const uint64_t size = img.size();
  auto within = [size](uint64_t off, uint64_t len) { return off <= size && len <= size - off; };
  if (eh.e_shentsize != sizeof(Elf64_Shdr) || eh.e_shoff > size ||
      eh.e_shnum > (size - eh.e_shoff) / sizeof(Elf64_Shdr))
    return false;
  auto shdr = [&](uint32_t k) {
    Elf64_Shdr sh;
    memcpy(&sh, img.data() + eh.e_shoff + (uint64_t)k * sizeof(Elf64_Shdr), sizeof(sh));
    return sh;
  };
  const size_t nlen = strlen(name);
  for (uint32_t k = 0; k < eh.e_shnum; k++) {
    const Elf64_Shdr sy = shdr(k);
    if (sy.sh_type != SHT_DYNSYM || sy.sh_link >= eh.e_shnum || !within(sy.sh_offset, sy.sh_size)) continue;
    const Elf64_Shdr st = shdr(sy.sh_link);
    if (!within(st.sh_offset, st.sh_size)) continue;
    for (uint64_t o = 0; o + sizeof(Elf64_Sym) <= sy.sh_size; o += sizeof(Elf64_Sym)) {
      Elf64_Sym sym;
      memcpy(&sym, img.data() + sy.sh_offset + o, sizeof(sym));
      if (sym.st_shndx == SHN_UNDEF || sym.st_name >= st.sh_size || nlen >= st.sh_size - sym.st_name) continue;
      if (memcmp(img.data() + st.sh_offset + sym.st_name, name, nlen + 1) == 0) return true;
    }
  }
  return false;
}

// set once rccl() has resolved the entry points (fmskf_rccl_library reads it without loading)
std::atomic<const RcclApi *> g_rccl_loaded{nullptr};

const RcclApi &rccl() {
  static RcclApi api = [] {
    RcclApi a;
    // FMSKF_RCCL_LIBRARY names the tests' one-GPU loopback stand-in (tests/native/
    // loopback_rccl.cpp), used alone, without falling back.  Only a file whose dynamic symbol
    // table exports the stand-in's marker is loaded (checked before dlopen), so an RCCL build
    // or another collective library named there by mistake is refused without running its
    // constructors.  Not a defence against a hostile library (it can export the marker too).
    const char *alt = getenv("FMSKF_RCCL_LIBRARY");
    void *lib = nullptr;
    if (alt && *alt) {
      if (!elf_exports(alt, "fmskf_rccl_stand_in")) {
        a.why = std::string("FMSKF_RCCL_LIBRARY=") + alt + " is not the test stand-in (no fmskf_rccl_stand_in)";
        return a;
      }
      lib = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
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
  g_rccl_loaded.store(&api, std::memory_order_release);
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

}  // namespace

// behind the fold queued on the tick stream, on the side stream: ncclAllGather of the slot's
// record over the handle's communicator, one D2H of the gathered records, the slot's event
void fmskf::capi::ens_gather_async(fmskf_ctx *h, fmskf_ctx::EnsSlot &S) {
  if (!h->ens_stream) {
    int lo = 0, hi = 0;
    hip_check(hipDeviceGetStreamPriorityRange(&lo, &hi), "hipDeviceGetStreamPriorityRange");
    hip_check(hipStreamCreateWithPriority(&h->ens_stream, hipStreamNonBlocking, hi), "hipStreamCreate");
    hip_check(hipEventCreateWithFlags(&h->ens_ticked, kSyncEvent), "hipEventCreate");
  }
  const uint32_t nx = h->d.nx, len = 1 + nx + nx * (nx + 1) / 2;
  // FMSKF_ENS_XTIME=0: no timing events around the exchange (A/B of their cost; then
  // fmskf_ensemble_exchange_ms reports -1)
  static const bool xtime = [] {
    const char *e = getenv("FMSKF_ENS_XTIME");
    return !e || atoi(e) != 0;
  }();
  if (xtime && !S.x0) {  // timing events on the side stream only (the tick stream records none)
    hip_check(hipEventCreate(&S.x0), "hipEventCreate");
    hip_check(hipEventCreate(&S.x1), "hipEventCreate");
  }
  hip_check(hipEventRecord(h->ens_ticked, h->stream), "hipEventRecord");
  hip_check(hipStreamWaitEvent(h->ens_stream, h->ens_ticked, 0), "hipStreamWaitEvent");
  if (xtime) hip_check(hipEventRecord(S.x0, h->ens_stream), "hipEventRecord");
  nccl_check(need_rccl().all_gather(S.rec, S.gather, len, ncclFloat64, h->comm, h->ens_stream),
             "ncclAllGather");
  hip_check(hipMemcpyAsync(S.host, S.gather, (size_t)S.ranks * len * 8, hipMemcpyDeviceToHost, h->ens_stream),
            "D2H");
  if (xtime) hip_check(hipEventRecord(S.x1, h->ens_stream), "hipEventRecord");
  hip_check(hipEventRecord(S.done, h->ens_stream), "hipEventRecord");
  S.exchanged = xtime;
}


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
  // never loads RCCL; RcclApi::path is immutable once rccl() has returned
  const RcclApi *a = g_rccl_loaded.load(std::memory_order_acquire);
  return a ? a->path.c_str() : "";
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
  const int ranks = ens_exchanges(h) ? h->world : 1;
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
      if (!ens_exchanges(h) && !h->timing) t.ens_done = C->done;
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
  S.exchanged = false;  // set when its fold is queued to the side stream (ens_gather_async)
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
    h->ens_xms = -1.f;
    if (S.exchanged) {
      hip_check(hipEventElapsedTime(&h->ens_xms, S.x0, S.x1), "hipEventElapsedTime");
      S.exchanged = false;
    }
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

int fmskf_ensemble_exchange_ms(fmskf_handle h, float *ms) {
  return guarded([&] {
    check_handle(h);
    if (!ms) fail(FMSKF_EINVAL, "null ms");
    *ms = h->ens_xms;
  });
}

}  // extern "C"
