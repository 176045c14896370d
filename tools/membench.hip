// membench.hip -- bandwidth ceilings for the KF6 tick's access pattern on MI355X.
//
// Streams exactly the bytes of one KF6 tick (27 fp32 state planes read + written,
// yaw/gyro planes and the [N][4] int16 rpm plane read = 232 B per instance) with no
// arithmetic, at 1, 2 and 4 instances per lane (dword / dwordx2 / dwordx4 accesses),
// plus a plain float4 copy of the same byte count.  Prints GB/s of algorithmic bytes.
//   hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build/membench && build/membench [log2N] [0=zeros]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int IPL>
struct Vec;
template <>
struct Vec<1> {
  using F = float;
  using R = uint2;
};
template <>
struct Vec<2> {
  using F = float2;
  using R = uint4;
};

template <int IPL>
__global__ __launch_bounds__(256) void k_pattern(float *st, const float *yaw, const float *gz,
                                                 const uint2 *rpm, uint64_t n, float sink) {
  using F = typename Vec<IPL>::F;
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // vector index
  const uint64_t nv = n / IPL;
  if (v >= nv) return;
  F s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = reinterpret_cast<const F *>(st + k * n)[v];
  const F a = reinterpret_cast<const F *>(yaw)[v];
  const F b = reinterpret_cast<const F *>(gz)[v];
  uint2 r[IPL];
#pragma unroll
  for (int q = 0; q < IPL; q++) r[q] = rpm[v * IPL + q];
  float m = sink;
  if constexpr (IPL == 1) {
    m = m * a * b * (float)(r[0].x & 1);
  } else {
    m = m * a.x * b.y * (float)(r[0].x & r[1].y & 1);
  }
#pragma unroll
  for (int k = 0; k < 27; k++) {
    F t = s[k];
    if constexpr (IPL == 1) t = t + m;
    else {
      t.x = t.x + m;
      t.y = t.y + m;
    }
    reinterpret_cast<F *>(st + k * n)[v] = t;
  }
}

__global__ __launch_bounds__(256) void k_pattern4(float *st, const float *yaw, const float *gz,
                                                  const uint4 *rpm, uint64_t n, float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n / 4) return;
  float4 s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = reinterpret_cast<const float4 *>(st + k * n)[v];
  const float4 a = reinterpret_cast<const float4 *>(yaw)[v];
  const float4 b = reinterpret_cast<const float4 *>(gz)[v];
  const uint4 r0 = rpm[2 * v], r1 = rpm[2 * v + 1];
  const float m = sink * a.x * b.w * (float)(r0.x & r1.w & 1);
#pragma unroll
  for (int k = 0; k < 27; k++) {
    float4 t = s[k];
    t.x += m;
    t.y += m;
    t.z += m;
    t.w += m;
    reinterpret_cast<float4 *>(st + k * n)[v] = t;
  }
}

// plane pitch != n (padding), and tiled SoA ("AoSoA": [N/T][27][T], a wave's 27 state
// rows are one contiguous 27*T*4-byte span) variants of the ipl1 pattern
__global__ __launch_bounds__(256) void k_pattern_pitch(float *st, const float *yaw, const float *gz,
                                                       const uint2 *rpm, uint64_t n, uint64_t pitch,
                                                       float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = st[k * pitch + v];
  const float m = sink * yaw[v] * gz[v] * (float)(rpm[v].x & 1);
#pragma unroll
  for (int k = 0; k < 27; k++) st[k * pitch + v] = s[k] + m;
}

template <int T>
__global__ __launch_bounds__(256) void k_pattern_tiled(float *st, const float *yaw, const float *gz,
                                                       const uint2 *rpm, uint64_t n, float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float *tile = st + (v / T) * (27 * T) + (v % T);
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = tile[k * T];
  const float m = sink * yaw[v] * gz[v] * (float)(rpm[v].x & 1);
#pragma unroll
  for (int k = 0; k < 27; k++) tile[k * T] = s[k] + m;
}

// the ipl1 pattern (pitched) with ITERS x 27 FMAs between the loads and the stores: how
// much arithmetic the memory phases hide
template <int ITERS>
__global__ __launch_bounds__(256) void k_pattern_delay(float *st, const float *yaw, const float *gz,
                                                       const uint2 *rpm, uint64_t n, uint64_t pitch,
                                                       float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = st[k * pitch + v];
  const float a = yaw[v], b = gz[v] * (float)(rpm[v].x & 1);
#pragma unroll
  for (int it = 0; it < ITERS; it++)
#pragma unroll
    for (int k = 0; k < 27; k++) s[k] = __builtin_fmaf(s[k], a, b);
#pragma unroll
  for (int k = 0; k < 27; k++) st[k * pitch + v] = s[k] + sink;
}

// the same with ONE dependent chain of ITERS FMAs (the KF update's shape: serial, low ILP)
template <int ITERS>
__global__ __launch_bounds__(256) void k_pattern_chain(float *st, const float *yaw, const float *gz,
                                                       const uint2 *rpm, uint64_t n, uint64_t pitch,
                                                       float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++) s[k] = st[k * pitch + v];
  const float a = yaw[v], b = gz[v] * (float)(rpm[v].x & 1);
  float t = b;
#pragma unroll
  for (int it = 0; it < ITERS; it++) t = __builtin_fmaf(t, a, s[it % 27]);
#pragma unroll
  for (int k = 0; k < 27; k++) st[k * pitch + v] = s[k] + t * sink;
}

// the EKF9 (54 fp32 state planes + a 16-byte raw record) and KF12D (90 fp64 state planes +
// 8 fp64 measurement planes) access patterns, pitched like the engine's planes
template <typename T, int NS, int NIN>
__global__ __launch_bounds__(256) void k_model_pattern(T *st, const T *in, uint64_t n, uint64_t pitch,
                                                       T sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  T s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = st[k * pitch + v];
  T m = sink;
#pragma unroll
  for (int k = 0; k < NIN; k++) m = m * in[k * n + v];
#pragma unroll
  for (int k = 0; k < NS; k++) st[k * pitch + v] = s[k] + m;
}
// the same bytes streamed CH planes at a time (few registers, full occupancy)
template <typename T, int NS, int NIN, int CH>
__global__ __launch_bounds__(256) void k_model_stream(T *st, const T *in, uint64_t n, uint64_t pitch,
                                                      T sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  T m = sink;
#pragma unroll
  for (int k = 0; k < NIN; k++) m = m * in[k * n + v];
#pragma unroll 1
  for (int c = 0; c < NS; c += CH) {
    T s[CH];
#pragma unroll
    for (int k = 0; k < CH; k++) s[k] = st[(c + k) * pitch + v];
#pragma unroll
    for (int k = 0; k < CH; k++) st[(c + k) * pitch + v] = s[k] + m;
  }
}
__global__ __launch_bounds__(256) void k_ekf9_pattern(float *st, const uint4 *raw, uint64_t n,
                                                      uint64_t pitch, float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float s[54];
#pragma unroll
  for (int k = 0; k < 54; k++) s[k] = st[k * pitch + v];
  const uint4 r = raw[v];
  const float m = sink * (float)(r.x & r.y & r.z & r.w & 1);
#pragma unroll
  for (int k = 0; k < 54; k++) st[k * pitch + v] = s[k] + m;
}

// tiled ("AoSoA") state: [N/T][NS][T] -- a wave's NS rows are one contiguous NS*T*sizeof(T) span
template <typename TT, int NS, int T>
__global__ __launch_bounds__(256) void k_model_tiled(TT *st, const uint4 *raw, uint64_t n, TT sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  TT *tile = st + (v / T) * ((uint64_t)NS * T) + (v % T);
  TT s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = tile[k * T];
  const uint4 r = raw[v];
  const TT m = sink * (TT)(r.x & r.y & r.z & r.w & 1);
#pragma unroll
  for (int k = 0; k < NS; k++) tile[k * T] = s[k] + m;
}

// tiled with 4 rows per lane access: [N/T][NS4][T] float4 (row 4q..4q+3 of robot i are one
// 16-byte word), so one wave instruction covers 1 KB contiguous instead of 256 B
template <int NS4, int T>
__global__ __launch_bounds__(256) void k_model_tiled4(float4 *st, const uint4 *raw, uint64_t n, float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float4 *tile = st + (v / T) * ((uint64_t)NS4 * T) + (v % T);
  float4 s[NS4];
#pragma unroll
  for (int k = 0; k < NS4; k++) s[k] = tile[k * T];
  const uint4 r = raw[v];
  const float m = sink * (float)(r.x & r.y & r.z & r.w & 1);
#pragma unroll
  for (int k = 0; k < NS4; k++) {
    float4 t = s[k];
    t.x += m;
    t.y += m;
    t.z += m;
    t.w += m;
    tile[k * T] = t;
  }
}

// HBM-regime probes of the tiled pattern. MODE 0: loads only (one 4-byte store per lane);
// 1: stores only; 2: non-temporal loads and stores; 3: non-temporal stores only
template <int NS, int T, int MODE, typename TT = float>
__global__ __launch_bounds__(256) void k_tiled_probe(TT *st, const uint4 *raw, uint64_t n, TT sink) {
  extern __shared__ double occ_cap[];  // dynamic LDS only limits the blocks per CU
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  TT *tile = st + (v / T) * ((uint64_t)NS * T) + (v % T);
  const uint4 r = raw[v];
  const TT m = sink * (TT)(r.x & r.y & r.z & r.w & 1);
  if (MODE == 1) {
#pragma unroll
    for (int k = 0; k < NS; k++) tile[k * T] = m + (TT)k;
    return;
  }
  TT s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = MODE == 2 ? __builtin_nontemporal_load(tile + k * T) : tile[k * T];
  if (MODE == 0) {
    TT acc = m;
#pragma unroll
    for (int k = 0; k < NS; k++) acc += s[k];
    if (acc == 12345.f) occ_cap[threadIdx.x] = acc, tile[0] = occ_cap[threadIdx.x ^ 1];
    return;
  }
#pragma unroll
  for (int k = 0; k < NS; k++) {
    if (MODE >= 2) __builtin_nontemporal_store(s[k] + m, tile + k * T);
    else tile[k * T] = s[k] + m;
  }
}

// the non-temporal tiled pattern with FMAS fp32 FMAs (8 independent chains over every loaded
// row) between the loads and the stores: the tick kernels' compute phase without their math
// the KF12D shape: NS non-temporal fp64 rows per robot, FMAS fp64 FMAs (8 chains) between
// the loads and the stores, VG extra live doubles to hold the kernel's occupancy (2 waves/SIMD)
template <int NS, int FMAS, int T = 256>
__global__ __launch_bounds__(256) void k_tiled_delay64(double *st, const uint4 *raw, uint64_t n, double sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  double *tile = st + (v / T) * ((uint64_t)NS * T) + (v % T);
  const uint4 r = raw[v];
  double s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = __builtin_nontemporal_load(tile + k * T);
  const double a = (double)(r.x & 0xFF) * sink + 1.0;
  double c[8];
#pragma unroll
  for (int j = 0; j < 8; j++) c[j] = s[j];
#pragma unroll
  for (int it = 0; it < FMAS / 8; it++)
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = __builtin_fma(c[j], a, s[(it * 8 + j) % NS]);
  double m = c[0];
#pragma unroll
  for (int j = 1; j < 8; j++) m += c[j];
#pragma unroll
  for (int k = 0; k < NS; k++) __builtin_nontemporal_store(s[k] + m * sink, tile + k * T);
}

template <int NS, int FMAS, int T = 256>
__global__ __launch_bounds__(256) void k_tiled_delay(float *st, const uint4 *raw, uint64_t n, float sink) {
  extern __shared__ double occ_cap[];
  (void)occ_cap;
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float *tile = st + (v / T) * ((uint64_t)NS * T) + (v % T);
  const uint4 r = raw[v];
  float s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = __builtin_nontemporal_load(tile + k * T);
  const float a = __builtin_bit_cast(float, r.x | 0x3F800000u) * sink;
  float c[8];
#pragma unroll
  for (int j = 0; j < 8; j++) c[j] = s[j];
#pragma unroll
  for (int it = 0; it < FMAS / 8; it++)
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = __builtin_fmaf(c[j], a, s[(it * 8 + j) % NS]);
  float m = c[0];
#pragma unroll
  for (int j = 1; j < 8; j++) m += c[j];
#pragma unroll
  for (int k = 0; k < NS; k++) __builtin_nontemporal_store(s[k] + m * sink, tile + k * T);
}

// the same pattern out of place: the tile is read from src and written to dst (a ping-pong
// state pair), fp32 (EKF9 shape) or fp64 (KF12D shape)
template <int NS, int FMAS, class T>
__global__ __launch_bounds__(256) void k_tiled_oop(const T *src, T *dst, const uint4 *raw, uint64_t n, T sink) {
  extern __shared__ double occ_cap[];
  (void)occ_cap;
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  const uint64_t off = (v / 256) * ((uint64_t)NS * 256) + (v % 256);
  const uint4 r = raw[v];
  T s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = __builtin_nontemporal_load(src + off + k * 256);
  const T a = (T)(r.x & 0xFF) * sink + (T)1;
  T c[8];
#pragma unroll
  for (int j = 0; j < 8; j++) c[j] = s[j];
#pragma unroll
  for (int it = 0; it < FMAS / 8; it++)
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if constexpr (sizeof(T) == 4) c[j] = __builtin_fmaf(c[j], a, s[(it * 8 + j) % NS]);
      else c[j] = __builtin_fma(c[j], a, s[(it * 8 + j) % NS]);
    }
  T m = c[0];
#pragma unroll
  for (int j = 1; j < 8; j++) m += c[j];
#pragma unroll
  for (int k = 0; k < NS; k++) __builtin_nontemporal_store(s[k] + m * sink, dst + off + k * 256);
}

// the same non-temporal tiled pattern with its compute phase, persistent: block b walks tiles
// b, b + G, ... with two register sets, the next tile's loads issued before the current tile's
// compute and stores (software pipelining across tiles; a wave's memory phases overlap its
// own compute)
template <int NS, int FMAS>
__device__ __forceinline__ void tile_ld(const float *st, uint64_t t, float (&s)[NS], uint4 &r,
                                        const uint4 *raw) {
  const float *tile = st + t * ((uint64_t)NS * 256) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = __builtin_nontemporal_load(tile + k * 256);
  r = raw[t * 256 + threadIdx.x];
}
template <int NS, int FMAS>
__device__ __forceinline__ void tile_cs(float *st, uint64_t t, const float (&s)[NS], uint4 r, float sink) {
  const float a = __builtin_bit_cast(float, r.x | 0x3F800000u) * sink;
  float c[8];
#pragma unroll
  for (int j = 0; j < 8; j++) c[j] = s[j];
#pragma unroll
  for (int it = 0; it < FMAS / 8; it++)
#pragma unroll
    for (int j = 0; j < 8; j++) c[j] = __builtin_fmaf(c[j], a, s[(it * 8 + j) % NS]);
  float m = c[0];
#pragma unroll
  for (int j = 1; j < 8; j++) m += c[j];
  float *tile = st + t * ((uint64_t)NS * 256) + threadIdx.x;
#pragma unroll
  for (int k = 0; k < NS; k++) __builtin_nontemporal_store(s[k] + m * sink, tile + k * 256);
}
template <int NS, int FMAS, bool PIPE>
__global__ __launch_bounds__(256) void k_tiled_persist(float *st, const uint4 *raw, uint64_t n, float sink) {
  const uint64_t ntiles = n / 256, G = gridDim.x;
  uint64_t t = blockIdx.x;
  if (t >= ntiles) return;
  float sa[NS], sb[NS];
  uint4 ra, rb;
  tile_ld<NS, FMAS>(st, t, sa, ra, raw);
  for (;;) {
    const uint64_t tb = t + G;
    if (PIPE && tb < ntiles) tile_ld<NS, FMAS>(st, tb, sb, rb, raw);
    tile_cs<NS, FMAS>(st, t, sa, ra, sink);
    if (tb >= ntiles) break;
    if (!PIPE) tile_ld<NS, FMAS>(st, tb, sb, rb, raw);
    const uint64_t ta = tb + G;
    if (PIPE && ta < ntiles) tile_ld<NS, FMAS>(st, ta, sa, ra, raw);
    tile_cs<NS, FMAS>(st, tb, sb, rb, sink);
    if (ta >= ntiles) break;
    if (!PIPE) tile_ld<NS, FMAS>(st, ta, sa, ra, raw);
    t = ta;
  }
}

// the pitched KF6 pattern (27 state planes + a 16-byte record) through buffer descriptors with
// explicit cache-policy bits on the state loads (LAUX) and stores (SAUX): gfx950 sc0 = 1,
// nt = 2, sc1 = 16
template <int LAUX, int SAUX>
__global__ __launch_bounds__(256) void k_pitch_pol(float *st, const uint4 *raw, uint64_t n, uint64_t pitch,
                                                   float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  const auto r = __builtin_amdgcn_make_buffer_rsrc(st, 0, (int)(uint32_t)(pitch * 27 * 4), 0x00020000);
  const uint32_t vo = (uint32_t)v * 4u, ps = (uint32_t)pitch * 4u;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++)
    s[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, k * ps, LAUX));
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(raw) + v);
  const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const float m = sink * (float)(q0 & q1 & q2 & q3 & 1);
#pragma unroll
  for (int k = 0; k < 27; k++)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, s[k] + m), r, vo, k * ps, SAUX);
}

// the KF6 pattern over tiled state (27 rows of T robots per tile), policy bits as k_pitch_pol
template <int T, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void k_tiled_pol(float *st, const uint4 *raw, uint64_t n, float sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  const uint64_t b = (uint64_t)blockIdx.x;
  float *base = st + (b / (T / 256)) * (27ull * T) + (b % (T / 256)) * 256;
  const auto r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(26u * T * 4 + 1024), 0x00020000);
  const uint32_t vo = threadIdx.x * 4u;
  float s[27];
#pragma unroll
  for (int k = 0; k < 27; k++)
    s[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, k * T * 4, LAUX));
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(raw) + v);
  const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const float m = sink * (float)(q0 & q1 & q2 & q3 & 1);
#pragma unroll
  for (int k = 0; k < 27; k++)
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, s[k] + m), r, vo, k * T * 4, SAUX);
}

// L2 pinning across launches: blocks b with b / 8 < pinb (the first pinb blocks of each XCD,
// with blocks dealt round-robin to the 8 XCDs) load / store their state with policies PL / PS,
// the others with SL / SS: can a state subset written back with plain stores stay in its
// XCD's L2 for the next launch while the rest streams past it (nt = evict first)?
template <int PL, int PS, int SL, int SS>
__global__ __launch_bounds__(256) void k_pitch_pin(float *st, const uint4 *raw, uint64_t n, uint64_t pitch,
                                                   float sink, uint32_t pinb) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  const auto r = __builtin_amdgcn_make_buffer_rsrc(st, 0, (int)(uint32_t)(pitch * 27 * 4), 0x00020000);
  const uint32_t vo = (uint32_t)v * 4u, ps = (uint32_t)pitch * 4u;
  const bool pin = (blockIdx.x >> 3) < pinb;
  float s[27];
  if (pin) {
#pragma unroll
    for (int k = 0; k < 27; k++)
      s[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, k * ps, PL));
  } else {
#pragma unroll
    for (int k = 0; k < 27; k++)
      s[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, k * ps, SL));
  }
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(raw) + v);
  const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
  const float m = sink * (float)(q0 & q1 & q2 & q3 & 1);
  if (pin) {
#pragma unroll
    for (int k = 0; k < 27; k++)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, s[k] + m), r, vo, k * ps, PS);
  } else {
#pragma unroll
    for (int k = 0; k < 27; k++)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, s[k] + m), r, vo, k * ps, SS);
  }
}

// the pitched (planar) KF6 pattern with non-temporal state loads and stores and a 16-byte record
template <int NS>
__global__ __launch_bounds__(256) void k_pitch_nt(float *st, const uint4 *raw, uint64_t n, uint64_t pitch,
                                                  float sink) {
  extern __shared__ double occ_cap[];  // dynamic LDS only limits the blocks per CU
  (void)occ_cap;
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  float s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = __builtin_nontemporal_load(st + k * pitch + v);
  const uint4 r = raw[v];
  const float m = sink * (float)(r.x & r.y & r.z & r.w & 1);
#pragma unroll
  for (int k = 0; k < NS; k++) __builtin_nontemporal_store(s[k] + m, st + k * pitch + v);
}

// the tiled pattern, read from one state buffer and written to another (ping-pong state)
template <typename TT, int NS, int T>
__global__ __launch_bounds__(256) void k_model_tiled_pp(const TT *src, TT *dst, const uint4 *raw, uint64_t n,
                                                        TT sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  const uint64_t o = (v / T) * ((uint64_t)NS * T) + (v % T);
  TT s[NS];
#pragma unroll
  for (int k = 0; k < NS; k++) s[k] = src[o + k * T];
  const uint4 r = raw[v];
  const TT m = sink * (TT)(r.x & r.y & r.z & r.w & 1);
#pragma unroll
  for (int k = 0; k < NS; k++) dst[o + k * T] = s[k] + m;
}

// a path row's byte mix with no arithmetic (membench LG 1 mix): RI dword planes of tick inputs
// read from a ring of 16 tick slots (as tools/kbench.py feeds the kernels: fresh inputs every
// tick), RW state planes read and written, WO state planes only written, V robots per lane
// (dword / dwordx2 accesses), planar at a padded pitch (plane_pitch: n rounded to 512 + 256;
// an exact power-of-two stride aliases) -- the streaming ceiling of a kernel moving those bytes
// in the same cache regime.  W > 0: the state tiled instead ([n/W][planes][W], V == 1).
template <int RI, int RW, int WO, int V, int W = 0>
__global__ __launch_bounds__(256) void k_mix(uint32_t *st, const uint32_t *in, uint64_t n, uint64_t pitch,
                                             uint32_t sink) {
  using T = typename std::conditional<V == 1, uint32_t, uint2>::type;
  uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n / V) return;
  uint32_t m = sink;
#pragma unroll
  for (int k = 0; k < RI; k++) {
    const T r = reinterpret_cast<const T *>(in + k * pitch)[v];
    if constexpr (V == 1) m ^= r;
    else m ^= r.x ^ r.y;
  }
  uint64_t sp = pitch;
  if constexpr (W > 0) {  // plane k of robot v at tile base + k * W
    st += (v / W) * (uint64_t)(RW + WO) * W;
    v %= W;
    sp = W;
  }
  T s[RW + 1];
#pragma unroll
  for (int k = 0; k < RW; k++) s[k] = reinterpret_cast<const T *>(st + k * sp)[v];
#pragma unroll
  for (int k = 0; k < RW; k++) {
    T t = s[k];
    if constexpr (V == 1) t ^= (m & 1);
    else {
      t.x ^= (m & 1);
      t.y ^= (m & 1);
    }
    reinterpret_cast<T *>(st + k * sp)[v] = t;
  }
#pragma unroll
  for (int k = 0; k < WO; k++) {
    T t;
    if constexpr (V == 1) t = m + k;
    else t = make_uint2(m + k, m - k);
    reinterpret_cast<T *>(st + (RW + k) * sp)[v] = t;
  }
}

// the same with the planes' access widths of the real kernels: dword (A4) and qword (A8) planes
// of ring-fed inputs (RI), state read and written (RW) and state written (WO), one robot per lane
template <int RI4, int RI8, int RW4, int RW8, int WO4, int WO8>
__global__ __launch_bounds__(256) void k_mixw(uint32_t *st, const uint32_t *in, uint64_t n, uint64_t pitch,
                                              uint32_t sink) {
  const uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= n) return;
  uint32_t m = sink;
#pragma unroll
  for (int k = 0; k < RI4; k++) m ^= in[k * pitch + v];
#pragma unroll
  for (int k = 0; k < RI8; k++) {
    const uint2 r = reinterpret_cast<const uint2 *>(in + (RI4 + 2 * k) * pitch)[v];
    m ^= r.x ^ r.y;
  }
  uint32_t a[RW4 + 1];
  uint2 b[RW8 + 1];
#pragma unroll
  for (int k = 0; k < RW4; k++) a[k] = st[k * pitch + v];
#pragma unroll
  for (int k = 0; k < RW8; k++) b[k] = reinterpret_cast<const uint2 *>(st + (RW4 + 2 * k) * pitch)[v];
#pragma unroll
  for (int k = 0; k < RW4; k++) st[k * pitch + v] = a[k] ^ (m & 1);
#pragma unroll
  for (int k = 0; k < RW8; k++)
    reinterpret_cast<uint2 *>(st + (RW4 + 2 * k) * pitch)[v] = make_uint2(b[k].x ^ (m & 1), b[k].y);
  constexpr int B = RW4 + 2 * RW8;
#pragma unroll
  for (int k = 0; k < WO4; k++) st[(B + k) * pitch + v] = m + k;
#pragma unroll
  for (int k = 0; k < WO8; k++)
    reinterpret_cast<uint2 *>(st + (B + WO4 + 2 * k) * pitch)[v] = make_uint2(m + k, m - k);
}

// the WT901 poll's exact accesses with no parsing (membench LG 1 mix): the lane's 48-byte poll
// row as three 16-byte loads and its length (ring-fed), the parser window (3 dword planes), the
// count / flags / error byte planes, 3 magnetometer and 15 written int16 register planes of a
// [0x90][n] register file, 4 q_init and 16 Data-page dword planes.  PACK: count, flags and
// error in one dword plane instead of three byte planes
template <bool PACK>
__global__ __launch_bounds__(256) void k_mix_wt901(const uint4 *rows, const uint32_t *len, uint32_t *parser,
                                                   uint8_t *cnt, uint8_t *flg, uint8_t *err, uint32_t *packed,
                                                   int16_t *reg, const float *qinit, float *data, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4 a = rows[3 * i], b = rows[3 * i + 1], c = rows[3 * i + 2];
  uint32_t m = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ len[i];
  const uint32_t p0 = parser[i], p1 = parser[n + i], p2 = parser[2 * n + i];
  uint32_t st;
  if constexpr (PACK) st = packed[i];
  else st = cnt[i] | ((uint32_t)flg[i] << 8);
  m ^= p0 ^ p1 ^ p2 ^ st;
  const int16_t h0 = reg[0x3a * n + i], h1 = reg[0x3b * n + i], h2 = reg[0x3c * n + i];
  float q[4];
#pragma unroll
  for (int k = 0; k < 4; k++) q[k] = qinit[k * n + i];
  m ^= (uint32_t)(h0 ^ h1 ^ h2);
  parser[i] = p0 ^ m;
  parser[n + i] = p1;
  parser[2 * n + i] = p2;
  if constexpr (PACK) packed[i] = st ^ (m & 0xFF0000u);
  else {
    cnt[i] = (uint8_t)st;
    flg[i] = (uint8_t)(st >> 8);
    err[i] = (uint8_t)m;
  }
  const uint32_t rk[15] = {0x34, 0x35, 0x36, 0x40, 0x37, 0x38, 0x39, 0x3d, 0x3e, 0x3f, 0x2e, 0x51, 0x52, 0x53, 0x54};
#pragma unroll
  for (int k = 0; k < 15; k++) reg[rk[k] * n + i] = (int16_t)(m >> k);
#pragma unroll
  for (int k = 0; k < 16; k++) data[k * n + i] = q[k & 3] + (float)(m & 7) * (float)k;
}

// the same planes with two adjacent IMUs per lane: every int16 register access a dword, every
// dword plane a dwordx2, the byte planes 2 bytes, the two 48-byte rows six 16-byte loads
__global__ __launch_bounds__(256) void k_mix_wt901_pair(const uint4 *rows, const uint32_t *len, uint32_t *parser,
                                                        uint8_t *cnt, uint8_t *flg, uint8_t *err, int16_t *reg,
                                                        const float *qinit, float *data, uint64_t n) {
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // IMUs 2j, 2j + 1
  if (2 * j >= n) return;
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const uint4 a = rows[6 * j + k];
    m ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  const uint2 l = reinterpret_cast<const uint2 *>(len)[j];
  m ^= l.x ^ l.y;
  uint2 pw[3];
#pragma unroll
  for (int k = 0; k < 3; k++) pw[k] = reinterpret_cast<const uint2 *>(parser + k * n)[j];
  const uint16_t c2 = reinterpret_cast<const uint16_t *>(cnt)[j], f2 = reinterpret_cast<const uint16_t *>(flg)[j];
  m ^= pw[0].x ^ pw[1].y ^ pw[2].x ^ c2 ^ f2;
#pragma unroll
  for (int k = 0; k < 3; k++) m ^= reinterpret_cast<const uint32_t *>(reg + (0x3a + k) * n)[j];
  float2 q[4];
#pragma unroll
  for (int k = 0; k < 4; k++) q[k] = reinterpret_cast<const float2 *>(qinit + k * n)[j];
#pragma unroll
  for (int k = 0; k < 3; k++) reinterpret_cast<uint2 *>(parser + k * n)[j] = make_uint2(pw[k].x ^ m, pw[k].y);
  reinterpret_cast<uint16_t *>(cnt)[j] = (uint16_t)(c2 ^ m);
  reinterpret_cast<uint16_t *>(flg)[j] = (uint16_t)(f2 ^ (m >> 3));
  reinterpret_cast<uint16_t *>(err)[j] = (uint16_t)(m >> 5);
  const uint32_t rk[15] = {0x34, 0x35, 0x36, 0x40, 0x37, 0x38, 0x39, 0x3d, 0x3e, 0x3f, 0x2e, 0x51, 0x52, 0x53, 0x54};
#pragma unroll
  for (int k = 0; k < 15; k++) reinterpret_cast<uint32_t *>(reg + rk[k] * n)[j] = m >> k;
#pragma unroll
  for (int k = 0; k < 16; k++)
    reinterpret_cast<float2 *>(data + k * n)[j] = make_float2(q[k & 3].x + (float)(m & 7) * (float)k, q[k & 3].y);
}

// round 6 probes (membench LG 1 r6): the RS tick and CAN RX byte mixes at the kernels' exact
// access widths, with the int64 encoder sums / previous sums as [4][pitch] planes (8-byte
// accesses, one per wheel) against [N][4] rows (two 16-byte accesses per robot).  RS: yaw f32,
// rpm u64 and the four sums from a 16-slot ring (SUMROWS: rows; else planes at sum pitch sp);
// px, py read, six state floats written, prev (PREVROWS: rows) read and written.  140 B.
template <bool SUMROWS, bool PREVROWS>
__global__ __launch_bounds__(256) void k_rsmix(float *x, int64_t *prev, const float *yaw, const uint64_t *rpm,
                                               const int64_t *sums, uint64_t n, uint64_t pp, uint64_t sp) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int64_t sm[4], pv[4];
  if constexpr (SUMROWS) {
    const longlong2 a = reinterpret_cast<const longlong2 *>(sums)[2 * i], b = reinterpret_cast<const longlong2 *>(sums)[2 * i + 1];
    sm[0] = a.x, sm[1] = a.y, sm[2] = b.x, sm[3] = b.y;
  } else {
#pragma unroll
    for (int w = 0; w < 4; w++) sm[w] = __builtin_nontemporal_load(sums + w * sp + i);
  }
  const float y = __builtin_nontemporal_load(yaw + i);
  const uint64_t r = __builtin_nontemporal_load(rpm + i);
  const float px = x[i], py = x[pp + i];
  if constexpr (PREVROWS) {
    const longlong2 a = reinterpret_cast<const longlong2 *>(prev)[2 * i], b = reinterpret_cast<const longlong2 *>(prev)[2 * i + 1];
    pv[0] = a.x, pv[1] = a.y, pv[2] = b.x, pv[3] = b.y;
  } else {
#pragma unroll
    for (int w = 0; w < 4; w++) pv[w] = prev[w * pp + i];
  }
  float d = y + (float)(r & 7);
#pragma unroll
  for (int w = 0; w < 4; w++) d += (float)(sm[w] - pv[w]);
  x[i] = px + d;
  x[pp + i] = py - d;
#pragma unroll
  for (int k = 2; k < 6; k++) x[k * pp + i] = d * (float)k;
  if constexpr (PREVROWS) {
    reinterpret_cast<longlong2 *>(prev)[2 * i] = make_longlong2(sm[0], sm[1]);
    reinterpret_cast<longlong2 *>(prev)[2 * i + 1] = make_longlong2(sm[2], sm[3]);
  } else {
#pragma unroll
    for (int w = 0; w < 4; w++) prev[w * pp + i] = sm[w];
  }
}

// CAN RX (k_can4's accesses, 216 B): the robot's 32 frame bytes (two 16-byte loads) and four
// stamps (8 B) from a 16-slot ring; micro, angle, previous angle, previous micro ([N][4] int16,
// 8 B each) and the IIR output ([N][4] f32, 16 B) read and written; the four int64 sums read
// and written (SUMROWS: two 16-byte accesses each way, else four [4][pp] planes); rpm and curr
// ([N][4] int16) written
template <bool SUMROWS>
__global__ __launch_bounds__(256) void k_canmix(const uint4 *frames, const uint64_t *stamps, uint64_t *st16,
                                                uint4 *iir, int64_t *sums, uint64_t n, uint64_t pp) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint4 f0 = frames[2 * i], f1 = frames[2 * i + 1];
  const uint64_t stp = __builtin_nontemporal_load(stamps + i);
  uint64_t v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = st16[k * n + i];
  uint4 y = iir[i];
  int64_t sm[4];
  if constexpr (SUMROWS) {
    const longlong2 a = reinterpret_cast<const longlong2 *>(sums)[2 * i], b = reinterpret_cast<const longlong2 *>(sums)[2 * i + 1];
    sm[0] = a.x, sm[1] = a.y, sm[2] = b.x, sm[3] = b.y;
  } else {
#pragma unroll
    for (int w = 0; w < 4; w++) sm[w] = sums[w * pp + i];
  }
  const uint32_t m = f0.x ^ f0.y ^ f0.z ^ f0.w ^ f1.x ^ f1.y ^ f1.z ^ f1.w ^ (uint32_t)stp;
#pragma unroll
  for (int w = 0; w < 4; w++) sm[w] += (int16_t)(m >> (4 * w));
  y.x ^= m;
  iir[i] = y;
#pragma unroll
  for (int k = 0; k < 4; k++) st16[k * n + i] = v[k] ^ (uint64_t)m;
  st16[4 * n + i] = (uint64_t)m * 3u;
  st16[5 * n + i] = (uint64_t)m * 5u;
  if constexpr (SUMROWS) {
    reinterpret_cast<longlong2 *>(sums)[2 * i] = make_longlong2(sm[0], sm[1]);
    reinterpret_cast<longlong2 *>(sums)[2 * i + 1] = make_longlong2(sm[2], sm[3]);
  } else {
#pragma unroll
    for (int w = 0; w < 4; w++) sums[w * pp + i] = sm[w];
  }
}

// the round-6 standard WT901 poll's exact accesses with no parsing (membench LG 1 w6, 110 B):
// the 48-byte poll row (three 16-byte loads) and its length from a 16-slot ring; the count and
// flags byte planes read; the three magnetometer int16 registers read (MAG); GZ, Yaw, TEMP and
// VERSION int16 registers written; the error and flags bytes written; the yaw / gyro z floats
// written (FLT 1: two float planes; 2: one [N][2] float plane; 3: instead of the floats and the GZ
// / Yaw registers, their raw words as one dword plane: 102 B); the 32-byte snapshot row written as
// two 16-byte stores.  PACK: count, flags and error in one dword plane read and written (114 B)
template <bool MAG, int FLT, bool PACK>
__global__ __launch_bounds__(256) void k_wt901mix6(const uint4 *rows, const uint32_t *len, uint8_t *cnt, uint8_t *flg,
                                                   uint8_t *err, uint32_t *packed, int16_t *reg, float *yaw,
                                                   float *gz, uint4 *snap, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t st;
  if constexpr (PACK) st = packed[i];
  else st = cnt[i] | ((uint32_t)flg[i] << 8);
  const uint32_t l = len[i];
  int16_t h[3] = {0, 0, 0};
  if constexpr (MAG) {
#pragma unroll
    for (int k = 0; k < 3; k++) h[k] = reg[(0x3a + k) * n + i];
  }
  const uint4 a = rows[3 * i], b = rows[3 * i + 1], c = rows[3 * i + 2];
  const uint32_t m = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ l ^ st;
  if constexpr (FLT != 3) {
    reg[0x39 * n + i] = (int16_t)m;
    reg[0x3f * n + i] = (int16_t)(m >> 3);
  }
  reg[0x40 * n + i] = (int16_t)(m >> 5);
  reg[0x2e * n + i] = (int16_t)(m >> 7);
  if constexpr (PACK) packed[i] = (st & 0xFF00FFu) ^ (m & 0xFF0000u);
  else {
    err[i] = (uint8_t)m;
    flg[i] = (uint8_t)(st >> 8);
  }
  const float fy = (float)(int16_t)(a.y >> 16) / 32768.0f * 180.0f;
  const float fg = (float)(int16_t)(b.x >> 8) / 32768.0f * 2000.0f;
  if constexpr (FLT == 1) {
    yaw[i] = fy;
    gz[i] = fg;
  } else if constexpr (FLT == 2) {
    reinterpret_cast<float2 *>(yaw)[i] = make_float2(fy, fg);
  } else if constexpr (FLT == 3) {
    reinterpret_cast<uint32_t *>(yaw)[i] = (a.y >> 16) | (b.x << 16);
  }
  snap[2 * i] = make_uint4(a.x ^ m, b.y, (uint32_t)(uint16_t)h[0] | (c.x << 16), (uint32_t)(uint16_t)h[1] | ((uint32_t)(uint16_t)h[2] << 16));
  snap[2 * i + 1] = make_uint4(c.y, c.z ^ m, a.w, 1u);
}

__global__ __launch_bounds__(256) void k_copy4(const float4 *a, float4 *b, uint64_t nv) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * 256)
    b[i] = a[i];
}

// fill with nonzero pseudo-random floats in [1, 2): memory traffic of all-zero buffers is
// measurably cheaper on MI355X (tools/mallbench.hip), so ceilings are measured on real-looking data
__global__ void k_fill_rand(uint32_t *p, uint64_t words, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (uint64_t)gridDim.x * 256) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (x & 0x007FFFFFu) | 0x3F800000u;
  }
}

int main(int argc, char **argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 20;
  const uint64_t n = 1ull << lg;
  float *st, *yaw, *gz, *ca, *cb;
  uint2 *rpm;
  const uint64_t pad = 4096;  // elements of padding per plane for the pitch variants
  CK(hipMalloc(&st, 27 * (n + 4 * pad) * 4));
  CK(hipMalloc(&yaw, n * 4));
  CK(hipMalloc(&gz, n * 4));
  CK(hipMalloc(&rpm, n * 8));
  CK(hipMemset(st, 0, 27 * n * 4));
  CK(hipMemset(yaw, 0, n * 4));
  CK(hipMemset(gz, 0, n * 4));
  CK(hipMemset(rpm, 0, n * 8));
  const uint64_t bytes = 232 * n;
  CK(hipMalloc(&ca, bytes / 2));
  CK(hipMalloc(&cb, bytes / 2));
  CK(hipMemset(ca, 0, bytes / 2));
  const bool zeros = argc > 2 && atoi(argv[2]) == 0;  // membench LG 0 -> all-zero buffers
  if (argc > 3 && argv[3][0] == 'w' && argv[3][1] == '6') {
    // membench LG 1 w6: the round-6 standard WT901 poll's byte mix (k_wt901mix6) and what each
    // of its parts costs -- two passes, random data, rows and lengths from a 16-slot ring
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    constexpr int kRing = 16;
    uint8_t *ring, *b3;
    uint32_t *pk;
    int16_t *rg;
    float *yw, *gzz;
    uint4 *sn;
    const size_t slot = (size_t)52 * n;  // [n][48] rows + [n] lengths
    CK(hipMalloc(&ring, kRing * slot));
    CK(hipMalloc(&b3, 3 * n));
    CK(hipMalloc(&pk, 4 * n));
    CK(hipMalloc(&rg, (size_t)0x41 * n * 2));
    CK(hipMalloc(&yw, 8 * n));
    CK(hipMalloc(&gzz, 4 * n));
    CK(hipMalloc(&sn, 32 * n));
    k_fill_rand<<<4096, 256>>>((uint32_t *)ring, kRing * slot / 4, 1);
    k_fill_rand<<<4096, 256>>>((uint32_t *)rg, (uint64_t)0x41 * n / 2, 2);
    k_fill_rand<<<4096, 256>>>((uint32_t *)sn, 8 * n, 3);
    k_fill_rand<<<4096, 256>>>(pk, n, 4);
    CK(hipMemset(b3, 0, 3 * n));
    CK(hipDeviceSynchronize());
    int tick = 0;
    const unsigned g1 = (unsigned)((n + 255) / 256);
    auto tm = [&](const char *name, int bpr, auto kern) {
      auto launch = [&] {
        const uint8_t *in = ring + (size_t)(tick++ % kRing) * slot;
        kern<<<g1, 256>>>((const uint4 *)in, (const uint32_t *)(in + 48 * n), b3, b3 + n, b3 + 2 * n, pk, rg, yw,
                          gzz, sn, n);
      };
      for (int w = 0; w < 2 * kRing; w++) launch();
      for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(f0));
        for (int it = 0; it < 64; it++) launch();
        CK(hipEventRecord(f1));
        CK(hipEventSynchronize(f1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, f0, f1));
        const double us = ms * 1e3 / 64;
        printf("{\"n\": %llu, \"mix\": \"%s\", \"bytes_per_robot\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
               (unsigned long long)n, name, bpr, us, (double)bpr * n / (us * 1e-6) / 1e9);
      }
    };
    for (int rep = 0; rep < 2; rep++) {
      tm("wt901_r6_exact", 110, k_wt901mix6<true, 1, false>);
      tm("wt901_r6_no_mag", 104, k_wt901mix6<false, 1, false>);
      tm("wt901_r6_no_floats", 102, k_wt901mix6<true, 0, false>);
      tm("wt901_r6_packed_bytes", 114, k_wt901mix6<true, 1, true>);
      tm("wt901_r6_no_mag_no_floats", 96, k_wt901mix6<false, 0, false>);
      tm("wt901_r6_float2_plane", 110, k_wt901mix6<true, 2, false>);
      tm("wt901_r6_raw_gz_yaw_dword", 102, k_wt901mix6<true, 3, false>);
    }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'r' && argv[3][1] == '6') {
    // membench LG 1 r6: the RS tick and CAN RX mixes with int64 sum planes against [N][4] rows
    // (k_rsmix, k_canmix), and the KF6 2^24-shape tiled pattern fed a ring of 16-byte records
    // (`kf6ring`: 1, 4 and 16 ticks of records at LG + 4) -- two passes, random data
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t pp = ((n + 511) / 512) * 512 + 256;
    constexpr int kRing = 16;
    float *xs;
    int64_t *pv, *sm;
    uint8_t *ring;
    uint64_t *st16;
    uint4 *iir;
    CK(hipMalloc(&xs, 6 * pp * 4));
    CK(hipMalloc(&pv, 4 * pp * 8));
    CK(hipMalloc(&sm, 4 * pp * 8));
    CK(hipMalloc(&st16, 6 * n * 8));
    CK(hipMalloc(&iir, n * 16));
    const size_t slot = (size_t)48 * pp;  // RS: yaw 4 + rpm 8 + sums 32 (planes at pitch pp or n); CAN: 40
    CK(hipMalloc(&ring, kRing * slot));
    k_fill_rand<<<4096, 256>>>((uint32_t *)xs, 6 * pp, 1);
    k_fill_rand<<<4096, 256>>>((uint32_t *)pv, 8 * pp, 2);
    k_fill_rand<<<4096, 256>>>((uint32_t *)sm, 8 * pp, 3);
    k_fill_rand<<<4096, 256>>>((uint32_t *)st16, 12 * n, 4);
    k_fill_rand<<<4096, 256>>>((uint32_t *)iir, 4 * n, 5);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ring, kRing * slot / 4, 6);
    CK(hipDeviceSynchronize());
    int tick = 0;
    auto tm = [&](const char *name, int bpr, auto launch) {
      for (int w = 0; w < 2 * kRing; w++) launch(ring + (size_t)(tick++ % kRing) * slot);
      for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(f0));
        for (int it = 0; it < 64; it++) launch(ring + (size_t)(tick++ % kRing) * slot);
        CK(hipEventRecord(f1));
        CK(hipEventSynchronize(f1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, f0, f1));
        const double us = ms * 1e3 / 64;
        printf("{\"n\": %llu, \"mix\": \"%s\", \"bytes_per_robot\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
               (unsigned long long)n, name, bpr, us, (double)bpr * n / (us * 1e-6) / 1e9);
      }
    };
    const unsigned g1 = (unsigned)((n + 255) / 256);
    auto rs = [&](auto kern, uint64_t sp) {
      return [=](uint8_t *in) {
        kern<<<g1, 256>>>(xs, pv, (const float *)in, (const uint64_t *)(in + 4 * pp), (const int64_t *)(in + 12 * pp),
                          n, pp, sp);
      };
    };
    for (int rep = 0; rep < 2; rep++) {
      tm("rs_sums_planes_dense_prev_planes", 140, rs(k_rsmix<false, false>, n));
      tm("rs_sums_planes_padded_prev_planes", 140, rs(k_rsmix<false, false>, pp));
      tm("rs_sums_planes_dense_prev_rows", 140, rs(k_rsmix<false, true>, n));
      tm("rs_sums_planes_padded_prev_rows", 140, rs(k_rsmix<false, true>, pp));
      tm("rs_sums_rows_prev_planes", 140, rs(k_rsmix<true, false>, n));
      tm("rs_sums_rows_prev_rows", 140, rs(k_rsmix<true, true>, n));
      tm("can_sums_planes", 216, [&](uint8_t *in) {
        k_canmix<false><<<g1, 256>>>((const uint4 *)in, (const uint64_t *)(in + 32 * pp), st16, iir, sm, n, pp);
      });
      tm("can_sums_rows", 216, [&](uint8_t *in) {
        k_canmix<true><<<g1, 256>>>((const uint4 *)in, (const uint64_t *)(in + 32 * pp), st16, iir, sm, n, pp);
      });
    }
    CK(hipFree(xs));
    CK(hipFree(pv));
    CK(hipFree(sm));
    CK(hipFree(st16));
    CK(hipFree(iir));
    CK(hipFree(ring));
    // the KF6 tick's 2^24 pattern (27 tiled non-temporal rows, 2048-wide tiles, 448 FMAs, the
    // 48 KiB cap) with its 16-byte records taken from a ring of R ticks, as the bench feeds it
    const uint64_t n6 = n << 4;
    float *sb;
    uint4 *rb;
    CK(hipMalloc(&sb, (size_t)27 * n6 * 4));
    CK(hipMalloc(&rb, (size_t)16 * n6 * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, (uint64_t)27 * n6, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)rb, (uint64_t)16 * n6 * 4, 8);
    CK(hipDeviceSynchronize());
    const unsigned g6 = (unsigned)(n6 / 256);
    for (int rep = 0; rep < 2; rep++)
      for (int R : {1, 4, 16}) {
        int k = 0;
        auto launch = [&] { k_tiled_delay<27, 448, 2048><<<g6, 256, 48 * 1024>>>(sb, rb + (size_t)(k++ % R) * n6, n6, 0.f); };
        for (int w = 0; w < 3; w++) launch();
        CK(hipEventRecord(f0));
        for (int it = 0; it < 16; it++) launch();
        CK(hipEventRecord(f1));
        CK(hipEventSynchronize(f1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, f0, f1));
        const double us = ms * 1e3 / 16;
        printf("{\"n\": %llu, \"kernel\": \"kf6ring_t2048_fma448_lds48\", \"ring\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
               (unsigned long long)n6, R, us, 232.0 * n6 / (us * 1e-6) / 1e9);
      }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'd') {
    // membench LG 1 d: the KF12D-shaped pattern (90 fp64 rows, non-temporal) with fp64 compute
    // phases of increasing length, at 2 blocks per CU (the kernel's 2 waves per SIMD) and uncapped
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    double *sb;
    uint4 *ib;
    CK(hipMalloc(&sb, (size_t)90 * n * 8));
    CK(hipMalloc(&ib, (size_t)n * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, (uint64_t)180 * n, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, (uint64_t)n * 4, 8);
    CK(hipDeviceSynchronize());
    auto tm = [&](const char *name, int par, auto launch) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipEventRecord(f0));
      for (int it = 0; it < 20; it++) launch();
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 20;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"lds_KiB\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)n, name, par, us, 1504.0 * n / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)(n / 256);
    for (int rep = 0; rep < 2; rep++)
      for (int kb : {64, 0}) {
        const size_t L = (size_t)kb * 1024;
        tm("kf12d_nt_fma0", kb, [&] { k_tiled_delay64<90, 0><<<g, 256, L>>>(sb, ib, n, 0.0); });
        tm("kf12d_nt_fma512", kb, [&] { k_tiled_delay64<90, 512><<<g, 256, L>>>(sb, ib, n, 0.0); });
        tm("kf12d_nt_fma1024", kb, [&] { k_tiled_delay64<90, 1024><<<g, 256, L>>>(sb, ib, n, 0.0); });
        tm("kf12d_nt_fma1280", kb, [&] { k_tiled_delay64<90, 1280><<<g, 256, L>>>(sb, ib, n, 0.0); });
        tm("kf12d_nt_fma1536", kb, [&] { k_tiled_delay64<90, 1536><<<g, 256, L>>>(sb, ib, n, 0.0); });
        tm("kf12d_nt_fma2048", kb, [&] { k_tiled_delay64<90, 2048><<<g, 256, L>>>(sb, ib, n, 0.0); });
      }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'm') {
    // membench LG 1 mix: the path rows' byte mixes (bench.py PATH_BYTES, pmc_traffic.py PATHS),
    // tick inputs from a 16-slot ring / state read+written / state written, in dwords per robot:
    //   KF6 record tick 4 / 27 / 0 (124 r, 108 w); RS tick 11 / 10 / 4 (84, 56);
    //   CAN RX 10 / 21 / 6 (124, 108); WT901 standard poll 13 / 9 / 18 (88, 108)
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t pp = ((n + 511) / 512) * 512 + 256;
    constexpr int kRing = 16;
    uint32_t *mb, *ib;
    CK(hipMalloc(&mb, (size_t)64 * pp * 4));
    CK(hipMalloc(&ib, (size_t)kRing * 16 * pp * 4));
    k_fill_rand<<<4096, 256>>>(mb, (uint64_t)64 * pp, 5);
    k_fill_rand<<<4096, 256>>>(ib, (uint64_t)kRing * 16 * pp, 6);
    CK(hipDeviceSynchronize());
    int tick = 0;
    auto tm = [&](const char *name, int bpr, auto launch) {
      for (int w = 0; w < 2 * kRing; w++) launch(ib + (size_t)(tick++ % kRing) * 16 * pp);
      for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(f0));
        for (int it = 0; it < 64; it++) launch(ib + (size_t)(tick++ % kRing) * 16 * pp);
        CK(hipEventRecord(f1));
        CK(hipEventSynchronize(f1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, f0, f1));
        const double us = ms * 1e3 / 64;
        printf("{\"n\": %llu, \"mix\": \"%s\", \"bytes_per_robot\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
               (unsigned long long)n, name, bpr, us, (double)bpr * n / (us * 1e-6) / 1e9);
      }
    };
    const unsigned g1 = (unsigned)((n + 255) / 256), g2 = (unsigned)((n / 2 + 255) / 256);
    tm("kf6_in16_rw108", 232, [&](const uint32_t *in) { k_mix<4, 27, 0, 1><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("kf6_in16_rw108_tiled2048", 232, [&](const uint32_t *in) { k_mix<4, 27, 0, 1, 2048><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("rs_in44_rw40_w16", 140, [&](const uint32_t *in) { k_mix<11, 10, 4, 1><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("rs_in44_rw40_w16_x2", 140, [&](const uint32_t *in) { k_mix<11, 10, 4, 2><<<g2, 256>>>(mb, in, n, pp, 0); });
    tm("rs_in44_rw40_w16_tiled2048", 140, [&](const uint32_t *in) { k_mix<11, 10, 4, 1, 2048><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("can_in40_rw84_w24", 232, [&](const uint32_t *in) { k_mix<10, 21, 6, 1><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("can_in40_rw84_w24_x2", 232, [&](const uint32_t *in) { k_mix<10, 21, 6, 2><<<g2, 256>>>(mb, in, n, pp, 0); });
    tm("can_in40_rw84_w24_tiled2048", 232, [&](const uint32_t *in) { k_mix<10, 21, 6, 1, 2048><<<g1, 256>>>(mb, in, n, pp, 0); });
    // the real kernels' access widths: RS yaw / rpm + 4 sums, px py / 4 prev, th vx vy vth;
    // CAN 40 B of frame + stamps as 5 qwords, head + 8 IIR / micro angle + 4 sums, prev rpm curr
    tm("rs_widths_q", 140, [&](const uint32_t *in) { k_mixw<1, 5, 2, 4, 4, 0><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("rs_widths_d", 140, [&](const uint32_t *in) { k_mixw<11, 0, 10, 0, 4, 0><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("can_widths_q", 232, [&](const uint32_t *in) { k_mixw<0, 5, 9, 6, 0, 3><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("can_widths_d", 232, [&](const uint32_t *in) { k_mixw<10, 0, 21, 0, 6, 0><<<g1, 256>>>(mb, in, n, pp, 0); });
    {
      // the WT901 poll's exact planes (k_mix_wt901); rows from a 16-slot ring of [n][48 B]
      uint8_t *wb;
      const size_t rowb = (size_t)n * 48, regb = (size_t)0x90 * n * 2;
      const size_t tot = kRing * rowb + kRing * n * 4 + 3 * n * 4 + 3 * n + n * 4 + regb + 4 * n * 4 + 16 * n * 4;
      CK(hipMalloc(&wb, tot));
      k_fill_rand<<<4096, 256>>>((uint32_t *)wb, tot / 4, 11);
      CK(hipDeviceSynchronize());
      uint8_t *q = wb + kRing * rowb;
      uint32_t *lens = (uint32_t *)q;
      q += kRing * n * 4;
      uint32_t *par = (uint32_t *)q;
      q += 3 * n * 4;
      uint8_t *cn = q, *fl = q + n, *er = q + 2 * n;
      q += 3 * n;
      uint32_t *pk = (uint32_t *)((uintptr_t)(q + 3) & ~(uintptr_t)3);
      q += n * 4;
      int16_t *rg = (int16_t *)q;
      q += regb;
      float *qi = (float *)q, *dt = (float *)(q + 4 * n * 4);
      int slot = 0;
      auto w = [&](bool pack) {
        const int s = slot++ % kRing;
        const uint4 *rows = (const uint4 *)(wb + s * rowb);
        if (pack) k_mix_wt901<true><<<g1, 256>>>(rows, lens + s * n, par, cn, fl, er, pk, rg, qi, dt, n);
        else k_mix_wt901<false><<<g1, 256>>>(rows, lens + s * n, par, cn, fl, er, pk, rg, qi, dt, n);
      };
      tm("wt901_exact_planes", 197, [&](const uint32_t *) { w(false); });
      tm("wt901_exact_planes_packed_bytes", 197, [&](const uint32_t *) { w(true); });
      const unsigned gp = (unsigned)((n / 2 + 255) / 256);
      tm("wt901_exact_planes_two_per_lane", 197, [&](const uint32_t *) {
        const int s = slot++ % kRing;
        k_mix_wt901_pair<<<gp, 256>>>((const uint4 *)(wb + s * rowb), lens + s * n, par, cn, fl, er, rg, qi, dt, n);
      });
      CK(hipFree(wb));
    }
    tm("wt901_in52_rw36_w72", 196, [&](const uint32_t *in) { k_mix<13, 9, 18, 1><<<g1, 256>>>(mb, in, n, pp, 0); });
    tm("wt901_in52_rw36_w72_tiled2048", 196, [&](const uint32_t *in) { k_mix<13, 9, 18, 1, 2048><<<g1, 256>>>(mb, in, n, pp, 0); });
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'o') {
    // membench LG 1 oop: in-place read-modify-write of the tiled state against a ping-pong pair
    // (read one buffer, write the other, swap per launch); EKF9 shape at LG, KF12D at LG - 2
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t nk = n >> 2;
    float *sa, *sb;
    uint4 *ib;
    CK(hipMalloc(&sa, (size_t)54 * n * 4));
    CK(hipMalloc(&sb, (size_t)54 * n * 4));
    CK(hipMalloc(&ib, (size_t)n * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sa, (uint64_t)54 * n, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, (uint64_t)54 * n, 9);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, (uint64_t)n * 4, 8);
    CK(hipDeviceSynchronize());
    int flip = 0;
    auto tm = [&](const char *name, int kb, uint64_t nn, double bpi, auto launch) {
      for (int w = 0; w < 4; w++) launch(flip++ & 1);
      CK(hipEventRecord(f0));
      for (int it = 0; it < 20; it++) launch(flip++ & 1);
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 20;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"lds_KiB\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)nn, name, kb, us, bpi * nn / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)(n / 256), gk = (unsigned)(nk / 256);
    double *da = (double *)sa, *db = (double *)sb;  // 90 doubles x n/4 fit 54 floats x n
    for (int rep = 0; rep < 2; rep++)
      for (int kb : {0, 64}) {
        const size_t L = (size_t)kb * 1024;
        tm("ekf9_inplace_fma0", kb, n, 448, [&](int) { k_tiled_oop<54, 0, float><<<g, 256, L>>>(sa, sa, ib, n, 0.f); });
        tm("ekf9_pingpong_fma0", kb, n, 448, [&](int f) {
          k_tiled_oop<54, 0, float><<<g, 256, L>>>(f ? sb : sa, f ? sa : sb, ib, n, 0.f);
        });
        tm("ekf9_inplace_fma864", kb, n, 448, [&](int) { k_tiled_oop<54, 864, float><<<g, 256, L>>>(sa, sa, ib, n, 0.f); });
        tm("ekf9_pingpong_fma864", kb, n, 448, [&](int f) {
          k_tiled_oop<54, 864, float><<<g, 256, L>>>(f ? sb : sa, f ? sa : sb, ib, n, 0.f);
        });
        tm("kf12d_inplace_fma1280", kb, nk, 1504, [&](int) {
          k_tiled_oop<90, 1280, double><<<gk, 256, L>>>(da, da, ib, nk, 0.0);
        });
        tm("kf12d_pingpong_fma1280", kb, nk, 1504, [&](int f) {
          k_tiled_oop<90, 1280, double><<<gk, 256, L>>>(f ? db : da, f ? da : db, ib, nk, 0.0);
        });
      }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'k') {
    // membench LG 1 kf6tiles: the KF6 state (27 fp32 rows, non-temporal) at LG, planar planes at
    // the engine's pitch against tiles of width T, with and without a 448-FMA compute phase
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t pitch = ((n + 511) / 512) * 512 + 256;
    float *sb;
    uint4 *ib;
    CK(hipMalloc(&sb, (size_t)27 * (pitch > n + 4096 ? pitch : n + 4096) * 4));
    CK(hipMalloc(&ib, (size_t)n * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, (uint64_t)27 * n, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, (uint64_t)n * 4, 8);
    CK(hipDeviceSynchronize());
    auto tm = [&](const char *name, int kb, auto launch) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipEventRecord(f0));
      for (int it = 0; it < 10; it++) launch();
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 10;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"lds_KiB\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)n, name, kb, us, 232.0 * n / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)(n / 256);
    for (int rep = 0; rep < 2; rep++)
      for (int kb : {48, 0}) {
        const size_t L = (size_t)kb * 1024;
        tm("kf6_pitch_nt", kb, [&] { k_pitch_nt<27><<<g, 256, L>>>(sb, ib, n, pitch, 0.f); });
        tm("kf6_t256_nt", kb, [&] { k_tiled_probe<27, 256, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf6_t2048_nt", kb, [&] { k_tiled_probe<27, 2048, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf6_t4096_nt", kb, [&] { k_tiled_probe<27, 4096, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf6_t256_fma448", kb, [&] { k_tiled_delay<27, 448, 256><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf6_t2048_fma448", kb, [&] { k_tiled_delay<27, 448, 2048><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf6_t4096_fma448", kb, [&] { k_tiled_delay<27, 448, 4096><<<g, 256, L>>>(sb, ib, n, 0.f); });
      }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 't') {
    // membench LG 1 tiles: the EKF9 non-temporal pattern at LG (and KF12D's at LG - 2) with
    // tile widths T = 64 ... 2048 robots (a tile is NS rows of T contiguous elements), at full
    // occupancy and at the kernels' 64 KiB cap
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t nk = n >> 2;
    float *sb;
    uint4 *ib;
    CK(hipMalloc(&sb, (size_t)54 * n * 4));
    CK(hipMalloc(&ib, (size_t)n * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, (uint64_t)54 * n, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, (uint64_t)n * 4, 8);
    CK(hipDeviceSynchronize());
    auto tm = [&](const char *name, int kb, uint64_t nn, double bpi, auto launch) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipEventRecord(f0));
      for (int it = 0; it < 20; it++) launch();
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 20;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"lds_KiB\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)nn, name, kb, us, bpi * nn / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)(n / 256), gk = (unsigned)(nk / 256);
    double *db = (double *)sb;
    for (int rep = 0; rep < 2; rep++)
      for (int kb : {0, 64}) {
        const size_t L = (size_t)kb * 1024;
        tm("ekf9_t64", kb, n, 448, [&] { k_tiled_probe<54, 64, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t128", kb, n, 448, [&] { k_tiled_probe<54, 128, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t256", kb, n, 448, [&] { k_tiled_probe<54, 256, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t512", kb, n, 448, [&] { k_tiled_probe<54, 512, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t2048", kb, n, 448, [&] { k_tiled_probe<54, 2048, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf12d_t256_fma1280", kb, nk, 1504, [&] { k_tiled_delay64<90, 1280, 256><<<gk, 256, L>>>(db, ib, nk, 0.0); });
        tm("kf12d_t1024_fma1280", kb, nk, 1504, [&] { k_tiled_delay64<90, 1280, 1024><<<gk, 256, L>>>(db, ib, nk, 0.0); });
        tm("kf12d_t2048_fma1280", kb, nk, 1504, [&] { k_tiled_delay64<90, 1280, 2048><<<gk, 256, L>>>(db, ib, nk, 0.0); });
        tm("kf12d_t4096_fma1280", kb, nk, 1504, [&] { k_tiled_delay64<90, 1280, 4096><<<gk, 256, L>>>(db, ib, nk, 0.0); });
        tm("ekf9_t1024_fma864", kb, n, 448, [&] { k_tiled_delay<54, 864, 1024><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t256_fma864", kb, n, 448, [&] { k_tiled_delay<54, 864, 256><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t512_fma864", kb, n, 448, [&] { k_tiled_delay<54, 864, 512><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t2048_fma864", kb, n, 448, [&] { k_tiled_delay<54, 864, 2048><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t4096_fma864", kb, n, 448, [&] { k_tiled_delay<54, 864, 4096><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("ekf9_t4096", kb, n, 448, [&] { k_tiled_probe<54, 4096, 2><<<g, 256, L>>>(sb, ib, n, 0.f); });
        tm("kf12d_t64", kb, nk, 1504, [&] { k_tiled_probe<90, 64, 2, double><<<gk, 256, L>>>(db, ib, nk, 0.0); });
        tm("kf12d_t256", kb, nk, 1504, [&] { k_tiled_probe<90, 256, 2, double><<<gk, 256, L>>>(db, ib, nk, 0.0); });
        tm("kf12d_t1024", kb, nk, 1504, [&] { k_tiled_probe<90, 1024, 2, double><<<gk, 256, L>>>(db, ib, nk, 0.0); });
      }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'x') {
    // membench LG 1 x: the EKF9-shaped tiled pattern (54 non-temporal rows, a compute phase of
    // 864 FMAs) one tile per block against persistent blocks that pipeline tiles (PIPE) or not
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    float *sb;
    uint4 *ib;
    CK(hipMalloc(&sb, (size_t)54 * n * 4));
    CK(hipMalloc(&ib, (size_t)n * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, (uint64_t)54 * n, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, (uint64_t)n * 4, 8);
    CK(hipDeviceSynchronize());
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto tm = [&](const char *name, int par, auto launch) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipEventRecord(f0));
      for (int it = 0; it < 20; it++) launch();
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 20;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"param\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)n, name, par, us, 448.0 * n / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)(n / 256);
    for (int rep = 0; rep < 2; rep++) {
      for (int kb : {0, 64})
        tm("delay864_one_tile_per_block", kb, [&] {
          k_tiled_delay<54, 864><<<g, 256, (size_t)kb * 1024>>>(sb, ib, n, 0.f);
        });
      for (int bpc : {1, 2, 3, 4}) {
        const unsigned gp = (unsigned)(cus * bpc) < g ? (unsigned)(cus * bpc) : g;
        tm("persist_pipe_blocks_per_cu", bpc, [&] { k_tiled_persist<54, 864, true><<<gp, 256>>>(sb, ib, n, 0.f); });
        tm("persist_nopipe_blocks_per_cu", bpc, [&] { k_tiled_persist<54, 864, false><<<gp, 256>>>(sb, ib, n, 0.f); });
      }
    }
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'p') {
    // membench LG 1 pol: the KF6 pattern (pitched planes, a 64-tick ring of 16-byte records)
    // under each load / store cache policy, at LG (2^20: the state resident in the Infinity Cache)
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t pitch = ((n + 511) / 512) * 512 + 256;
    float *sb;
    uint4 *ib;
    const int ring = 64;
    CK(hipMalloc(&sb, 27 * pitch * 4));
    CK(hipMalloc(&ib, (size_t)ring * n * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, 27 * pitch, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, (uint64_t)ring * n * 4, 8);
    CK(hipDeviceSynchronize());
    const unsigned g = (unsigned)((n + 255) / 256);
    int tick = 0;
    auto tm = [&](const char *name, auto launch) {
      for (int w = 0; w < 5; w++) launch(ib + (size_t)(tick++ % ring) * n);
      CK(hipEventRecord(f0));
      for (int it = 0; it < 100; it++) launch(ib + (size_t)(tick++ % ring) * n);
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 100;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}\n", (unsigned long long)n, name, us,
             232.0 * n / (us * 1e-6) / 1e9);
    };
    if (argv[3][1] == 'l') {  // membench LG 1 planes-vs-tiles: KF6 pattern, planar vs tiled
      for (int rep = 0; rep < 2; rep++) {
        tm("planar_ld_plain_st_sc1", [&](const uint4 *in) { k_pitch_pol<0, 16><<<g, 256>>>(sb, in, n, pitch, 0.f); });
        tm("t256_ld_plain_st_sc1", [&](const uint4 *in) { k_tiled_pol<256, 0, 16><<<g, 256>>>(sb, in, n, 0.f); });
        tm("t2048_ld_plain_st_sc1", [&](const uint4 *in) { k_tiled_pol<2048, 0, 16><<<g, 256>>>(sb, in, n, 0.f); });
        tm("t4096_ld_plain_st_sc1", [&](const uint4 *in) { k_tiled_pol<4096, 0, 16><<<g, 256>>>(sb, in, n, 0.f); });
        tm("planar_ld_nt_st_nt", [&](const uint4 *in) { k_pitch_pol<2, 2><<<g, 256>>>(sb, in, n, pitch, 0.f); });
        tm("t2048_ld_nt_st_nt", [&](const uint4 *in) { k_tiled_pol<2048, 2, 2><<<g, 256>>>(sb, in, n, 0.f); });
      }
      return 0;
    }
    if (argv[3][1] == 'i') {  // membench LG 1 pin: the L2-pinning sweep
      for (int rep = 0; rep < 2; rep++)
        for (unsigned pb : {0u, 32u, 64u, 96u, 128u}) {
          char nm[96];
          snprintf(nm, sizeof nm, "pin%u_plain_plain__stream_plain_sc1", pb);
          tm(nm, [&](const uint4 *in) { k_pitch_pin<0, 0, 0, 16><<<g, 256>>>(sb, in, n, pitch, 0.f, pb); });
          snprintf(nm, sizeof nm, "pin%u_plain_plain__stream_nt_sc1", pb);
          tm(nm, [&](const uint4 *in) { k_pitch_pin<0, 0, 2, 16><<<g, 256>>>(sb, in, n, pitch, 0.f, pb); });
          snprintf(nm, sizeof nm, "pin%u_plain_plain__stream_nt_nt", pb);
          tm(nm, [&](const uint4 *in) { k_pitch_pin<0, 0, 2, 2><<<g, 256>>>(sb, in, n, pitch, 0.f, pb); });
        }
      return 0;
    }
#define POL(L, S, NAME) tm(NAME, [&](const uint4 *in) { k_pitch_pol<L, S><<<g, 256>>>(sb, in, n, pitch, 0.f); })
    for (int rep = 0; rep < 2; rep++) {
      POL(0, 0, "ld_plain_st_plain");
      POL(0, 2, "ld_plain_st_nt");
      POL(0, 16, "ld_plain_st_sc1");
      POL(0, 17, "ld_plain_st_sc0sc1");
      POL(0, 1, "ld_plain_st_sc0");
      POL(16, 0, "ld_sc1_st_plain");
      POL(1, 0, "ld_sc0_st_plain");
      POL(2, 0, "ld_nt_st_plain");
      POL(16, 16, "ld_sc1_st_sc1");
      POL(2, 2, "ld_nt_st_nt");
      POL(2, 16, "ld_nt_st_sc1");
      POL(17, 16, "ld_sc0sc1_st_sc1");
      POL(1, 16, "ld_sc0_st_sc1");
    }
#undef POL
    return 0;
  }
  if (argc > 3 && argv[3][0] == 'c') {
    // membench LG 1 caps: the HBM-regime patterns (non-temporal state) under the occupancy cap
    // (dynamic LDS per block -> blocks per CU), tiled against planar; LG sizes the EKF9 case,
    // KF12D runs at LG - 2 and KF6 at LG + 2 (the configs' ratios: 2^22 / 2^20 / 2^24)
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t nk = n >> 2, n6 = n << 2;
    const uint64_t pitch = ((n + 511) / 512) * 512 + 256, pitch6 = ((n6 + 511) / 512) * 512 + 256;
    uint64_t words = 54 * pitch > 27 * pitch6 ? 54 * pitch : 27 * pitch6;
    if (words < 112 * n) words = 112 * n;  // the copy reads 224 n bytes and writes the next 224 n
    if (words < 45 * n) words = 45 * n;    // KF12D tiles: 90 doubles x n / 4
    void *sb, *ib;
    CK(hipMalloc(&sb, words * 4));
    CK(hipMalloc(&ib, n6 * 16));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, words, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, n6 * 4, 8);
    CK(hipDeviceSynchronize());
    auto tm = [&](const char *name, int kb, uint64_t nn, double bpi, auto launch) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipEventRecord(f0));
      for (int it = 0; it < 20; it++) launch();
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 20;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"lds_KiB\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)nn, name, kb, us, bpi * nn / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)((n + 255) / 256), gk = (unsigned)((nk + 255) / 256),
                   g6 = (unsigned)((n6 + 255) / 256);
    for (int kb : {0, 32, 48, 64, 80}) {
      const size_t L = (size_t)kb * 1024;
      tm("ekf9_t256_nt", kb, n, 448, [&] { k_tiled_probe<54, 256, 2><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_pitch_nt", kb, n, 448, [&] { k_pitch_nt<54><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, pitch, 0.f); });
      tm("kf12d_t256_nt", kb, nk, 1504, [&] {
        k_tiled_probe<90, 256, 2, double><<<gk, 256, L>>>((double *)sb, (const uint4 *)ib, nk, 0.0);
      });
      tm("kf6_pitch_nt", kb, n6, 232, [&] { k_pitch_nt<27><<<g6, 256, L>>>((float *)sb, (const uint4 *)ib, n6, pitch6, 0.f); });
      tm("kf6_t256_nt", kb, n6, 232, [&] { k_tiled_probe<27, 256, 2><<<g6, 256, L>>>((float *)sb, (const uint4 *)ib, n6, 0.f); });
    }
    tm("copy_float4_448B_fullgrid", 0, n, 448, [&] {
      k_copy4<<<(unsigned)(224 * n / 16 / 256), 256>>>((const float4 *)sb, (float4 *)((char *)sb + 224 * n),
                                                      224 * n / 16);
    });
    // compute between the loads and the stores (EKF9 tick: ~860 VALU per robot), at the
    // EKF9 kernel's occupancy cap (64 KiB: 2 blocks per CU) and uncapped
    for (int kb : {0, 64, 48, 64}) {
      const size_t L = (size_t)kb * 1024;
      tm("ekf9_t256_nt_fma0", kb, n, 448, [&] { k_tiled_delay<54, 0><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma1024", kb, n, 448, [&] { k_tiled_delay<54, 1024><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma1536", kb, n, 448, [&] { k_tiled_delay<54, 1536><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma2048", kb, n, 448, [&] { k_tiled_delay<54, 2048><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma256", kb, n, 448, [&] { k_tiled_delay<54, 256><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma512", kb, n, 448, [&] { k_tiled_delay<54, 512><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma864", kb, n, 448, [&] { k_tiled_delay<54, 864><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
      tm("ekf9_t256_nt_fma1280", kb, n, 448, [&] { k_tiled_delay<54, 1280><<<g, 256, L>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    }
    return 0;
  }
  if (argc > 3) {  // membench LG 1 models: the EKF9 and KF12D patterns only
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0));
    CK(hipEventCreate(&f1));
    const uint64_t pitch = ((n + 511) / 512) * 512 + 256;
    void *sb, *ib;
    CK(hipMalloc(&sb, 90 * pitch * 8));
    CK(hipMalloc(&ib, 8 * n * 8));
    k_fill_rand<<<4096, 256>>>((uint32_t *)sb, 90 * pitch * 2, 7);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ib, 8 * n * 2, 8);
    CK(hipDeviceSynchronize());
    auto tm = [&](const char *name, double bpi, auto launch) {
      for (int w = 0; w < 3; w++) launch();
      CK(hipEventRecord(f0));
      for (int it = 0; it < 20; it++) launch();
      CK(hipEventRecord(f1));
      CK(hipEventSynchronize(f1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, f0, f1));
      const double us = ms * 1e3 / 20;
      printf("{\"n\": %llu, \"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}\n",
             (unsigned long long)n, name, us, bpi * n / (us * 1e-6) / 1e9);
    };
    const unsigned g = (unsigned)((n + 255) / 256);
    tm("ekf9_pattern_448B", 448, [&] { k_ekf9_pattern<<<g, 256>>>((float *)sb, (const uint4 *)ib, n, pitch, 0.f); });
    tm("ekf9_tiled64_448B", 448, [&] { k_model_tiled<float, 54, 64><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("ekf9_tiled256_448B", 448, [&] { k_model_tiled<float, 54, 256><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_tiled256_232B", 232, [&] { k_model_tiled<float, 27, 256><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    {
      void *sb2;
      CK(hipMalloc(&sb2, 90 * pitch * 8));
      k_fill_rand<<<4096, 256>>>((uint32_t *)sb2, 90 * pitch * 2, 9);
      CK(hipDeviceSynchronize());
      int flip = 0;
      tm("ekf9_tiled256_pingpong_448B", 448, [&] {
        float *a = (float *)(flip ? sb2 : sb), *b = (float *)(flip ? sb : sb2);
        flip ^= 1;
        k_model_tiled_pp<float, 54, 256><<<g, 256>>>(a, b, (const uint4 *)ib, n, 0.f);
      });
      tm("kf6_tiled256_pingpong_232B", 232, [&] {
        float *a = (float *)(flip ? sb2 : sb), *b = (float *)(flip ? sb : sb2);
        flip ^= 1;
        k_model_tiled_pp<float, 27, 256><<<g, 256>>>(a, b, (const uint4 *)ib, n, 0.f);
      });
      CK(hipFree(sb2));
    }
    tm("ekf9_tiled4x256_464B_as448", 448, [&] { k_model_tiled4<14, 256><<<g, 256>>>((float4 *)sb, (const uint4 *)ib, n, 0.f); });
    tm("ekf9_tiled4x64_464B_as448", 448, [&] { k_model_tiled4<14, 64><<<g, 256>>>((float4 *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_tiled4x256_240B_as232", 232, [&] { k_model_tiled4<7, 256><<<g, 256>>>((float4 *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_tiled4x64_240B_as232", 232, [&] { k_model_tiled4<7, 64><<<g, 256>>>((float4 *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_t256_loads_only_as232", 232, [&] { k_tiled_probe<27, 256, 0><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_t256_stores_only_as232", 232, [&] { k_tiled_probe<27, 256, 1><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_t256_nt_ldst", 232, [&] { k_tiled_probe<27, 256, 2><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_t256_nt_st", 232, [&] { k_tiled_probe<27, 256, 3><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_t256_plain", 232, [&] { k_tiled_probe<27, 256, 4><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    for (int kb : {16, 32, 48, 80})
      tm(kb == 16 ? "kf6_t256_lds16K" : kb == 32 ? "kf6_t256_lds32K" : kb == 48 ? "kf6_t256_lds48K" : "kf6_t256_lds80K", 232,
         [&] { k_tiled_probe<27, 256, 4><<<g, 256, kb * 1024>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("ekf9_t256_nt_st", 448, [&] { k_tiled_probe<54, 256, 3><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("ekf9_t256_nt_ldst", 448, [&] { k_tiled_probe<54, 256, 2><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    for (int kb : {16, 32, 48})
      tm(kb == 16 ? "ekf9_t256_lds16K" : kb == 32 ? "ekf9_t256_lds32K" : "ekf9_t256_lds48K", 448,
         [&] { k_tiled_probe<54, 256, 4><<<g, 256, kb * 1024>>>((float *)sb, (const uint4 *)ib, n, 0.f); });
    tm("kf6_pitch_nt_232B", 232, [&] { k_pitch_nt<27><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, pitch, 0.f); });
    tm("ekf9_pitch_nt_448B", 448, [&] { k_pitch_nt<54><<<g, 256>>>((float *)sb, (const uint4 *)ib, n, pitch, 0.f); });
    tm("kf12d_t256_1504B", 1504, [&] { k_tiled_probe<90, 256, 4, double><<<g, 256>>>((double *)sb, (const uint4 *)ib, n, 0.0); });
    tm("kf12d_t256_nt_ldst_1504B", 1504, [&] { k_tiled_probe<90, 256, 2, double><<<g, 256>>>((double *)sb, (const uint4 *)ib, n, 0.0); });
    // HBM-scale copy ceilings at the model's byte count (half read, half written)
    tm("copy_float4_448B", 448, [&] {
      k_copy4<<<2048, 256>>>((const float4 *)sb, (float4 *)((char *)sb + 224 * n), 224 * n / 16);
    });
    tm("copy_float4_448B_fullgrid", 448, [&] {
      k_copy4<<<(unsigned)(224 * n / 16 / 256), 256>>>((const float4 *)sb, (float4 *)((char *)sb + 224 * n),
                                                      224 * n / 16);
    });
    tm("kf12d_tiled64_1504B", 1504, [&] { k_model_tiled<double, 90, 64><<<g, 256>>>((double *)sb, (const uint4 *)ib, n, 0.0); });
    tm("kf12d_pattern_1504B", 1504, [&] {
      k_model_pattern<double, 90, 8><<<g, 256>>>((double *)sb, (const double *)ib, n, pitch, 0.0);
    });
    tm("kf12d_stream10_1504B", 1504, [&] {
      k_model_stream<double, 90, 8, 10><<<g, 256>>>((double *)sb, (const double *)ib, n, pitch, 0.0);
    });
    tm("kf12d_stream30_1504B", 1504, [&] {
      k_model_stream<double, 90, 8, 30><<<g, 256>>>((double *)sb, (const double *)ib, n, pitch, 0.0);
    });
    return 0;
  }
  if (!zeros) {
    k_fill_rand<<<4096, 256>>>((uint32_t *)st, 27 * (n + 4 * pad), 1);
    k_fill_rand<<<4096, 256>>>((uint32_t *)yaw, n, 2);
    k_fill_rand<<<4096, 256>>>((uint32_t *)gz, n, 3);
    k_fill_rand<<<4096, 256>>>((uint32_t *)rpm, 2 * n, 4);
    k_fill_rand<<<4096, 256>>>((uint32_t *)ca, bytes / 8, 5);
    CK(hipDeviceSynchronize());
  }
  printf("{\"data\": \"%s\"}\n", zeros ? "zeros" : "random");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 100;
  auto timeit = [&](const char *name, auto launch) {
    for (int w = 0; w < 5; w++) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int it = 0; it < iters; it++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf("{\"n\": %llu, \"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}\n", (unsigned long long)n,
           name, us, bytes / (us * 1e-6) / 1e9);
  };
  timeit("pattern_ipl1_dword", [&] {
    k_pattern<1><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, 0.f);
  });
  timeit("pattern_ipl2_dwordx2", [&] {
    k_pattern<2><<<(unsigned)((n / 2 + 255) / 256), 256>>>(st, yaw, gz, rpm, n, 0.f);
  });
  timeit("pattern_ipl4_dwordx4", [&] {
    k_pattern4<<<(unsigned)((n / 4 + 255) / 256), 256>>>(st, yaw, gz, (const uint4 *)rpm, n, 0.f);
  });
  for (uint64_t pp : {(uint64_t)64, (uint64_t)256, (uint64_t)1024, (uint64_t)4096, (uint64_t)16384 / 4}) {
    char name[64];
    snprintf(name, sizeof(name), "pattern_pitch_n+%llu", (unsigned long long)pp);
    timeit(name, [&] {
      k_pattern_pitch<<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + pp, 0.f);
    });
  }
  timeit("pattern_delay_0", [&] {
    k_pattern_delay<0><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_delay_108fma", [&] {
    k_pattern_delay<4><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_delay_216fma", [&] {
    k_pattern_delay<8><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_delay_432fma", [&] {
    k_pattern_delay<16><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_delay_864fma", [&] {
    k_pattern_delay<32><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_chain_0", [&] {
    k_pattern_chain<0><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_chain_200", [&] {
    k_pattern_chain<200><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_chain_400", [&] {
    k_pattern_chain<400><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_chain_800", [&] {
    k_pattern_chain<800><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, n + 256, 0.f);
  });
  timeit("pattern_tiled64", [&] {
    k_pattern_tiled<64><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, 0.f);
  });
  timeit("pattern_tiled256", [&] {
    k_pattern_tiled<256><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, 0.f);
  });
  timeit("pattern_tiled1024", [&] {
    k_pattern_tiled<1024><<<(unsigned)((n + 255) / 256), 256>>>(st, yaw, gz, rpm, n, 0.f);
  });
  timeit("copy_float4_same_bytes", [&] {
    k_copy4<<<2048, 256>>>((const float4 *)ca, (float4 *)cb, bytes / 2 / 16);
  });
  return 0;
}
