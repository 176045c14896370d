// loopback_rccl.cpp -- test infrastructure: the five RCCL entry points libfmskf resolves
// (ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclAllGather, ncclGetErrorString),
// implemented by staging every rank's buffer through a shared directory.
//
// RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so a one-GPU box cannot run
// libfmskf's communicator at world > 1.  Loaded through FMSKF_RCCL_LIBRARY, this library
// lets several processes on that one GPU run the library's multi-rank code unchanged: slot
// sizing by world, the all-gather's rank order, the pinned copy-out and the host fold of
// `world` records.  It is no collective: ncclAllGather synchronises the stream it is given,
// copies the send buffer to the host, publishes it as <dir>/<seq>.<rank>, waits for every
// rank's file of the same call and copies the concatenation into the receive buffer.
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

struct LoopComm {
  std::string dir;
  int rank, world;
  unsigned long seq;
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
  *comm = new LoopComm{dir, rank, nranks, 0};
  return 0;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return 0;
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t type, ncclComm_t comm,
                           hipStream_t stream) {
  const size_t tb = type_bytes(type);
  if (!comm || !tb) return 4;
  const size_t bytes = count * tb;
  const unsigned long seq = comm->seq++;
  std::vector<char> host(bytes * comm->world);
  if (hipStreamSynchronize(stream) != hipSuccess) return 2;
  if (hipMemcpy(host.data() + bytes * comm->rank, send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 2;
  auto name = [&](int r) { return comm->dir + "/" + std::to_string(seq) + "." + std::to_string(r); };
  const std::string mine = name(comm->rank), tmp = mine + ".tmp";
  FILE *f = fopen(tmp.c_str(), "wb");
  if (!f) return 2;
  const bool wrote = fwrite(host.data() + bytes * comm->rank, 1, bytes, f) == bytes;
  if (fclose(f) != 0 || !wrote || rename(tmp.c_str(), mine.c_str()) != 0) return 2;
  const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(60);
  for (int r = 0; r < comm->world; r++) {
    if (r == comm->rank) continue;
    FILE *g = nullptr;
    while (!(g = fopen(name(r).c_str(), "rb"))) {
      if (std::chrono::steady_clock::now() > until) {
        fprintf(stderr, "loopback_rccl: rank %d timed out waiting for %s\n", comm->rank, name(r).c_str());
        return 2;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    const bool ok = fread(host.data() + bytes * r, 1, bytes, g) == bytes;
    fclose(g);
    if (!ok) return 2;
  }
  if (hipMemcpyAsync(recv, host.data(), host.size(), hipMemcpyHostToDevice, stream) != hipSuccess) return 2;
  if (hipStreamSynchronize(stream) != hipSuccess) return 2;
  return 0;
}

const char *ncclGetErrorString(ncclResult_t r) {
  return r == 0 ? "no error" : r == 4 ? "invalid argument" : "loopback staging failed";
}

}  // extern "C"
