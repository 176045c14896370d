// loopback_rccl.cpp -- test infrastructure: the seven RCCL entry points libfmskf resolves
// (ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclAllGather, ncclCommCount,
// ncclCommUserRank, ncclGetErrorString), implemented by staging every rank's buffer through a
// shared directory.  It exports `fmskf_rccl_stand_in`, the marker libfmskf requires of any
// library FMSKF_RCCL_LIBRARY names.
//
// RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so a one-GPU box cannot run
// libfmskf's communicator at world > 1.  Loaded through FMSKF_RCCL_LIBRARY, this library
// lets several processes on that one GPU run the library's multi-rank code unchanged: slot
// sizing by world, the all-gather's rank order, the pinned copy-out and the host fold of
// `world` records.  It is no collective: ncclAllGather synchronises the stream it is given,
// copies the send buffer to the host, publishes it as <dir>/<seq>.<rank>, waits for every
// rank's file of the same call and copies the concatenation into the receive buffer.
// LOOPBACK_RCCL_MODE=callback instead enqueues the exchange on the stream: a copy of the send
// buffer into pinned memory, a host function (hipLaunchHostFunc) that publishes it and waits for
// the other ranks' files, and a copy of the concatenation into the receive buffer -- so the call
// returns at once and libfmskf's side-stream ordering (gather behind the fold, copy-out behind
// the gather, the slot's event behind the copy-out) is exercised without the host blocking.
// Never part of the product; built by the package Makefile into build/.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

extern "C" {

typedef int ncclResult_t;  // ncclSuccess 0, ncclSystemError 2, ncclInvalidArgument 4
typedef struct {
  char internal[128];
} ncclUniqueId;
typedef int ncclDataType_t;

int fmskf_rccl_stand_in(void) { return 1; }

struct LoopComm {
  std::string dir;
  int rank, world;
  unsigned long seq;
  std::vector<struct Exchange *> pending;  // callback mode: freed at ncclCommDestroy
};

// one enqueued exchange (callback mode): the pinned [world][bytes] buffer and what the host
// function needs to fill it
struct Exchange {
  LoopComm *comm;
  unsigned long seq;
  size_t bytes;
  char *host;  // pinned
  hipEvent_t done;  // behind the exchange's last copy: the buffer may be freed once it completed
};
typedef LoopComm *ncclComm_t;

static size_t type_bytes(ncclDataType_t t) {
  switch (t) {  // RCCL's numbering
    case 0: case 1: return 1;
    case 2: case 3: case 7: return 4;
    case 4: case 5: case 8: return 8;
    case 6: case 9: return 2;
    default: return 0;
  }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
  if (!id) return 4;
  const char *base = getenv("LOOPBACK_RCCL_DIR");
  std::string tmpl = std::string(base ? base : "/tmp") + "/loopback_rccl.XXXXXX";
  if (tmpl.size() >= sizeof(id->internal)) return 4;
  std::vector<char> buf(tmpl.begin(), tmpl.end());
  buf.push_back('\0');
  if (!mkdtemp(buf.data())) return 2;
  memset(id->internal, 0, sizeof(id->internal));
  memcpy(id->internal, buf.data(), strlen(buf.data()));
  return 0;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return 4;
  char dir[129];
  memcpy(dir, id.internal, 128);
  dir[128] = '\0';
  if (access(dir, W_OK) != 0) return 2;
  *comm = new LoopComm{dir, rank, nranks, 0, {}};
  return 0;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return 4;
  for (Exchange *x : comm->pending) {
    (void)hipEventSynchronize(x->done);
    (void)hipEventDestroy(x->done);
    (void)hipHostFree(x->host);
    delete x;
  }
  delete comm;
  return 0;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int *count) {
  if (!comm || !count) return 4;
  *count = comm->world;
  return 0;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int *rank) {
  if (!comm || !rank) return 4;
  *rank = comm->rank;
  return 0;
}

static std::string slot_name(const LoopComm *c, unsigned long seq, int r) {
  return c->dir + "/" + std::to_string(seq) + "." + std::to_string(r);
}

// publish this rank's part of host[] as <dir>/<seq>.<rank>, then read every other rank's part
static int exchange(const LoopComm *c, unsigned long seq, char *host, size_t bytes) {
  const std::string mine = slot_name(c, seq, c->rank), tmp = mine + ".tmp";
  FILE *f = fopen(tmp.c_str(), "wb");
  if (!f) return 2;
  const bool wrote = fwrite(host + bytes * c->rank, 1, bytes, f) == bytes;
  if (fclose(f) != 0 || !wrote || rename(tmp.c_str(), mine.c_str()) != 0) return 2;
  const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(60);
  for (int r = 0; r < c->world; r++) {
    if (r == c->rank) continue;
    FILE *g = nullptr;
    while (!(g = fopen(slot_name(c, seq, r).c_str(), "rb"))) {
      if (std::chrono::steady_clock::now() > until) {
        fprintf(stderr, "loopback_rccl: rank %d timed out waiting for %s\n", c->rank, slot_name(c, seq, r).c_str());
        return 2;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    const bool ok = fread(host + bytes * r, 1, bytes, g) == bytes;
    fclose(g);
    if (!ok) return 2;
  }
  return 0;
}

// the host function of callback mode: runs in stream order, calls no HIP API.  ncclAllGather
// returned success long ago, so a failed exchange cannot be reported through it: the process
// aborts instead of leaving the receive buffer with stale bytes (test infrastructure only)
static void exchange_cb(void *arg) {
  Exchange *x = (Exchange *)arg;
  if (exchange(x->comm, x->seq, x->host, x->bytes) != 0) {
    fprintf(stderr, "loopback_rccl: callback exchange %lu failed: aborting\n", x->seq);
    abort();
  }
}

// free the pinned buffers of exchanges whose stream work has completed
static void reap(LoopComm *c) {
  size_t k = 0;
  for (Exchange *x : c->pending) {
    if (hipEventQuery(x->done) == hipSuccess) {
      (void)hipEventDestroy(x->done);
      (void)hipHostFree(x->host);
      delete x;
    } else {
      c->pending[k++] = x;
    }
  }
  c->pending.resize(k);
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t type, ncclComm_t comm,
                           hipStream_t stream) {
  const size_t tb = type_bytes(type);
  if (!comm || !tb) return 4;
  const size_t bytes = count * tb;
  const unsigned long seq = comm->seq++;
  const char *mode = getenv("LOOPBACK_RCCL_MODE");
  if (mode && strcmp(mode, "callback") == 0) {
    reap(comm);
    Exchange *x = new Exchange{comm, seq, bytes, nullptr, nullptr};
    if (hipHostMalloc((void **)&x->host, bytes * comm->world, hipHostMallocDefault) != hipSuccess) {
      delete x;
      return 2;
    }
    if (hipEventCreateWithFlags(&x->done, hipEventDisableTiming) != hipSuccess) {
      (void)hipHostFree(x->host);
      delete x;
      return 2;
    }
    comm->pending.push_back(x);
    if (hipMemcpyAsync(x->host + bytes * comm->rank, send, bytes, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipLaunchHostFunc(stream, exchange_cb, x) != hipSuccess ||
        hipMemcpyAsync(recv, x->host, bytes * comm->world, hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipEventRecord(x->done, stream) != hipSuccess)
      return 2;
    return 0;
  }
  std::vector<char> host(bytes * comm->world);
  if (hipStreamSynchronize(stream) != hipSuccess) return 2;
  if (hipMemcpy(host.data() + bytes * comm->rank, send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  if (exchange(comm, seq, host.data(), bytes) != 0) return 2;
  if (hipMemcpyAsync(recv, host.data(), host.size(), hipMemcpyHostToDevice, stream) != hipSuccess) return 2;
  if (hipStreamSynchronize(stream) != hipSuccess) return 2;
  return 0;
}

const char *ncclGetErrorString(ncclResult_t r) {
  return r == 0 ? "no error" : r == 4 ? "invalid argument" : "loopback staging failed";
}

}  // extern "C"
