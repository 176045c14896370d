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

// variants isolating what the inputs cost: MODE 0 no inputs, 1 global loads, 2 buffer loads
// (as k_kf6t), 3 buffer loads + a 2 KiB LDS table staged behind a barrier (as k_kf6t)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void *base, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)(uint32_t)bytes, 0x00020000);
}
// MODE 4: the three input streams interleaved into one 16-byte record per robot
template <int MODE>
__global__ __launch_bounds__(256) void k_pat2(float *st, const float *yaw, const float *gz,
                                              const uint2 *rpm, const float *tab, uint64_t n,
                                              uint64_t pitch, float sink) {
  __shared__ float stab[513];
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const bool live = v < n;
  const uint64_t vc = live ? v : n - 1;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = st[k * pitch + vc];
  float m = sink;
  if constexpr (MODE == 4) {
    const uint32_t i = (uint32_t)vc;
    const auto r = __builtin_amdgcn_raw_buffer_load_b128(mk_rsrc(yaw, n * 16), i * 16u, 0, 2);
    const uint32_t w0 = r[0], w1 = r[1];  // bit_cast of a vector-element lvalue reads element 0
    m = m * __builtin_bit_cast(float, w0) * __builtin_bit_cast(float, w1) * (float)(r[2] & 1);
  } else if constexpr (MODE == 1) {
    m = m * yaw[vc] * gz[vc] * (float)(rpm[vc].x & 1);
  } else if constexpr (MODE >= 2) {
    const uint32_t i = (uint32_t)vc;
    const float a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mk_rsrc(yaw, n * 4), i * 4u, 0, 2));
    const float b = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(mk_rsrc(gz, n * 4), i * 4u, 0, 2));
    const auto r = __builtin_amdgcn_raw_buffer_load_b64(mk_rsrc(rpm, n * 8), i * 8u, 0, 2);
    m = m * a * b * (float)(r[0] & 1);
  }
  if constexpr (MODE == 3) {
    const int t = threadIdx.x;
    const float ta = tab[t], tb = tab[t + 256];
    stab[t] = ta;
    stab[t + 256] = tb;
    if (t == 0) stab[512] = tab[512];
    __syncthreads();
    m = m * stab[((uint32_t)(m * 100.f)) & 511];
  }
  if (live) {
#pragma unroll
    for (int k = 0; k < 27; k++) st[k * pitch + v] = s[k] + m;
  }
}

__global__ void k_fill_rand(uint32_t *p, uint64_t words, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (x & 0x007FFFFFu) | 0x3F800000u;  // floats in [1, 2): nonzero, finite
  }
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
  {
    const int R = argc > 2 ? atoi(argv[2]) : 64;
    float *yaw, *gz, *tab;
    uint2 *rpm;
    CK(hipMalloc(&yaw, R * n * 16));
    CK(hipMalloc(&gz, R * n * 4));
    CK(hipMalloc(&rpm, R * n * 8));
    CK(hipMalloc(&tab, 513 * 4));
    CK(hipMemset(yaw, 0, R * n * 4));
    CK(hipMemset(gz, 0, R * n * 4));
    CK(hipMemset(rpm, 0, R * n * 8));
    CK(hipMemset(tab, 0, 513 * 4));
    if (argc > 4) {  // random (nonzero) contents for inputs and state
      k_fill_rand<<<4096, 256>>>((uint32_t *)yaw, R * n * 4, 1);
      k_fill_rand<<<4096, 256>>>((uint32_t *)gz, R * n, 2);
      k_fill_rand<<<4096, 256>>>((uint32_t *)rpm, R * n * 2, 3);
      k_fill_rand<<<4096, 256>>>((uint32_t *)st, 27 * pitch, 4);
      CK(hipDeviceSynchronize());
    }
    const char *names[] = {"no_inputs", "inputs_global", "inputs_buffer_nt", "inputs_buffer_nt+lds_table",
                           "inputs_packed16_nt"};
    for (int mode = 0; mode < 5; mode++) {
      auto launch = [&](int it) {
        const uint64_t o = (uint64_t)(it % R) * n;
        const dim3 g((unsigned)((n + 255) / 256));
        if (mode == 0) k_pat2<0><<<g, 256>>>(st, yaw + o, gz + o, rpm + o, tab, n, pitch, 0.f);
        if (mode == 1) k_pat2<1><<<g, 256>>>(st, yaw + o, gz + o, rpm + o, tab, n, pitch, 0.f);
        if (mode == 2) k_pat2<2><<<g, 256>>>(st, yaw + o, gz + o, rpm + o, tab, n, pitch, 0.f);
        if (mode == 3) k_pat2<3><<<g, 256>>>(st, yaw + o, gz + o, rpm + o, tab, n, pitch, 0.f);
        if (mode == 4) k_pat2<4><<<g, 256>>>(st, yaw + 4 * o, gz + o, rpm + o, tab, n, pitch, 0.f);
      };
      for (int w = 0; w < 2 * R; w++) launch(w);
      CK(hipDeviceSynchronize());
      const int iters = 512;
      CK(hipEventRecord(e0));
      for (int it = 0; it < iters; it++) launch(it);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"n\": %llu, \"variant\": \"%s\", \"ring\": %d, \"us\": %.2f}\n",
             (unsigned long long)n, names[mode], R, ms * 1e3 / iters);
      fflush(stdout);
    }
    CK(hipFree(yaw));
    CK(hipFree(gz));
    CK(hipFree(rpm));
    if (argc > 3) return 0;
  }
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
