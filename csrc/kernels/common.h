// Shared device helpers for the gfx950 (CDNA4) kernel library.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes.
//   * bf16 is carried as raw `uint16_t` bits; all global traffic is
//     vectorised to 16 B per lane (8 bf16) -- hipcc does not auto-vectorise
//     bf16 scalar loads (cdna_hip_programming.md Guideline 13).
//   * every launch entry point is `extern "C"` with raw pointers and a
//     hipStream_t so Python can bind it with ctypes without pulling in torch
//     headers, and so the launches are hipGraph-capturable (no malloc/sync).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define KCA_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Bounds/invariant checks of the debug kernel library (tools/build_ext.py
// --debug -> libkca_kernels_debug.so, loaded when KCA_DEBUG=1):
// a violated check prints the site and the offending block/thread and traps,
// so the fault is reported at the kernel that caused it. Compiled out of the
// release library.
#ifdef KCA_DEBUG
#define KCA_DASSERT(cond)                                                                                  \
  do {                                                                                                     \
    if (!(cond)) {                                                                                         \
      printf("KCA_DASSERT failed %s:%d: %s (block %d,%d,%d thread %d)\n", __FILE__, __LINE__, #cond,         \
             (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)threadIdx.x);                         \
      __builtin_trap();                                                                                    \
    }                                                                                                      \
  } while (0)
#else
#define KCA_DASSERT(cond) ((void)0)
#endif

struct alignas(16) U16x8 { uint16_t v[8]; };
struct alignas(8) U16x4 { uint16_t v[4]; };

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// Round-to-nearest-even; plain cast lowers to v_cvt_pk_bf16_f32 on gfx950 and
// keeps NaN a NaN (MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(uint16_t, h);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ void load8(const bf16_t* p, float (&x)[8]) {
  U16x8 u = *reinterpret_cast<const U16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = bf2f(u.v[i]);
}

__device__ __forceinline__ void store8(bf16_t* p, const float (&x)[8]) {
  U16x8 u;
#pragma unroll
  for (int i = 0; i < 8; ++i) u.v[i] = f2bf(x[i]);
  *reinterpret_cast<U16x8*>(p) = u;
}

__device__ __forceinline__ void load8f(const float* p, float (&x)[8]) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
  x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
}

__device__ __forceinline__ void store8f(float* p, const float (&x)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
}

// Element type of the 16-bit serving kernels: DT 0 = bf16, 1 = fp16 (FasterTransformer / DS-Inference
// serve fp16). DT 0 is exactly bf2f / f2bf.
template <int DT>
__device__ __forceinline__ float e2f(uint32_t u16) {
  if constexpr (DT == 0) return __uint_as_float(u16 << 16);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)u16);
}
template <int DT>
__device__ __forceinline__ uint32_t f2e(float f) {
  if constexpr (DT == 0) return (uint32_t)f2bf(f);
  else return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f);
}
template <int DT>
__device__ __forceinline__ void load8_t(const uint16_t* p, float (&x)[8]) {
  U16x8 u = *reinterpret_cast<const U16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = e2f<DT>(u.v[i]);
}
template <int DT>
__device__ __forceinline__ void store8_t(uint16_t* p, const float (&x)[8]) {
  U16x8 u;
#pragma unroll
  for (int i = 0; i < 8; ++i) u.v[i] = (uint16_t)f2e<DT>(x[i]);
  *reinterpret_cast<U16x8*>(p) = u;
}

// The two elements of a packed 32-bit pair (low / high half), and acc + w.lo * x.lo + w.hi * x.hi of
// two pairs -- the GEMV inner step: one v_dot2c_f32_bf16 / v_dot2_f32_f16 (fp32 accumulation) instead of
// two unpacks and two FMAs per pair (KCA_BF16_FMA_GEMV: the FMA form, for A/B).
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
template <int DT>
__device__ __forceinline__ float lo2f(uint32_t q) {
  if constexpr (DT == 0) return __uint_as_float(q << 16);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)(q & 0xffffu));
}
template <int DT>
__device__ __forceinline__ float hi2f(uint32_t q) {
  if constexpr (DT == 0) return __uint_as_float(q & 0xffff0000u);
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)(q >> 16));
}
template <int DT>
__device__ __forceinline__ float dot2_acc(uint32_t w, uint32_t x, float acc) {
  if constexpr (DT == 0) {
#ifdef KCA_BF16_FMA_GEMV
    acc = fmaf(lo2f<0>(w), lo2f<0>(x), acc);
    return fmaf(hi2f<0>(w), hi2f<0>(x), acc);
#else
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, w), __builtin_bit_cast(bf16x2_t, x), acc,
                                           false);
#endif
  } else {
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2, w), __builtin_bit_cast(f16x2, x), acc, false);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `red` must hold
// blockDim.x/64 floats. Result broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Grid size for memory-bound grid-stride kernels: enough blocks to fill 256 CUs
// several times over, capped (cdna_hip_programming.md Guideline 11).
static inline int kca_grid(long long work_items, int per_block, int cap = 2048) {
  long long g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// tanh(u) = 1 - 2 / (exp(2u) + 1) on v_exp_f32 + v_rcp_f32: ~1e-7 absolute
// error, saturates correctly (exp -> inf gives 1, exp -> 0 gives -1), and a
// fraction of libm tanhf's instructions and registers -- the activation kernels
// stay memory-bound at full occupancy.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = fast_tanh(u);
  float du = k0 * (1.f + 3.f * k1 * x2);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * du;
}

// XCD-aware workgroup remap (cdna_hip_programming.md §5.5 T1). The dispatcher
// hands linear workgroup id i to XCD i % 8, and each XCD has its own 4 MiB L2.
// Kernels whose neighbouring logical tiles share operands (the q-blocks of one
// attention head share its K/V) call this so that logical ids
// [x*n/8, (x+1)*n/8) all run on XCD x: the shared stream is fetched into one
// L2 instead of eight. Ids past the last multiple of 8 map to themselves.
__device__ __forceinline__ int xcd_remap(int bid, int n) {
  const int full = n & ~7;
  if (bid >= full) return bid;
  return (bid & 7) * (full >> 3) + (bid >> 3);
}
