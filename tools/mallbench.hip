// mallbench.hip -- does the tick's fresh-input stream evict the state from the Infinity Cache,
// and does the input buffer's allocation type change that?
//
// The KF6 access pattern (27 pitched state planes read + written, yaw / gyro / rpm read; no
// math) at N = 2^20, with the inputs taken from a ring of R ticks (R = 1: cache resident;
// R = 64: fresh every tick, as bench.py) allocated with hipMalloc, or hipExtMallocWithFlags
// (fine-grained / uncached).  Prints us per tick and GB/s of algorithmic bytes.
//   hipcc --offload-arch=gfx950 -O3 tools/mallbench.hip -o build/mallbench && build/mallbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

template <int CPOL>
__global__ __launch_bounds__(256) void k_pat(float *st, const float *yaw, const float *gz,
                                             const uint2 *rpm, uint64_t n, uint64_t pitch, float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = st[k * pitch + v];
  float a, b;
  uint2 r;
  if constexpr (CPOL == 0) {
    a = yaw[v];
    b = gz[v];
    r = rpm[v];
  } else {
    a = __builtin_nontemporal_load(yaw + v);
    b = __builtin_nontemporal_load(gz + v);
    r.x = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(rpm + v));
    r.y = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(rpm + v) + 1);
  }
  const float m = sink * a * b * (float)(r.x & 1);
#pragma unroll
  for (int k = 0; k < 27; k++) st[k * pitch + v] = s[k] + m;
}

int main(int argc, char **argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 20;
  const uint64_t n = 1ull << lg, pitch = n + 256;
  float *st;
  CK(hipMalloc(&st, 27 * pitch * 4));
  CK(hipMemset(st, 0, 27 * pitch * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *kinds[] = {"hipMalloc", "finegrained", "uncached"};
  const unsigned flags[] = {hipDeviceMallocDefault, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  for (int kind = 0; kind < 3; kind++) {
    for (int R : {1, 8, 16, 64}) {
      for (int cpol = 0; cpol < 2; cpol++) {
        float *yaw, *gz;
        uint2 *rpm;
        CK(hipExtMallocWithFlags((void **)&yaw, R * n * 4, flags[kind]));
        CK(hipExtMallocWithFlags((void **)&gz, R * n * 4, flags[kind]));
        CK(hipExtMallocWithFlags((void **)&rpm, R * n * 8, flags[kind]));
        CK(hipMemset(yaw, 0, R * n * 4));
        CK(hipMemset(gz, 0, R * n * 4));
        CK(hipMemset(rpm, 0, R * n * 8));
        const int iters = 256;
        auto launch = [&](int it) {
          const uint64_t o = (uint64_t)(it % R) * n;
          if (cpol == 0)
            k_pat<0><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw + o, gz + o, rpm + o, n, pitch, 0.f);
          else
            k_pat<1><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw + o, gz + o, rpm + o, n, pitch, 0.f);
        };
        for (int w = 0; w < 2 * R; w++) launch(w);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int it = 0; it < iters; it++) launch(it);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / iters;
        printf("{\"n\": %llu, \"inputs\": \"%s\", \"ring\": %d, \"nontemporal\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
               (unsigned long long)n, kinds[kind], R, cpol, us, 232.0 * n / (us * 1e-6) / 1e9);
        fflush(stdout);
        CK(hipFree(yaw));
        CK(hipFree(gz));
        CK(hipFree(rpm));
      }
    }
  }
  return 0;
}
