// Fused decode tail shared by decode.hip (the out-projection / fc_out GEMV launches) and
// csrc/comm/xgmi_allreduce.hip (the tensor-parallel all-reduce that closes a row-parallel projection):
// every workgroup publishes its part of y, the last one to arrive adds bias + residual, rounds the new
// residual stream to bf16 and normalises it for the next projection(s) -- no LayerNorm launch.
#pragma once
#include "common.h"

// Partials that another workgroup of the same launch combines: write-through (sc1) stores, so a
// drain (vmcnt(0)) + barrier + counter add publishes them across XCDs without a release fence
// (cdna_hip_programming.md Guideline 16, recipe R1).
__device__ __forceinline__ void st_pub(float* a, float v) {
  __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bf16 results handed to the tail the same way: one element (2 B) or eight (16 B, as two 8-B stores)
__device__ __forceinline__ void st_pub_bf16(bf16_t* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned short*>(p), f2bf(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_pub_bf16x8(bf16_t* p, const float (&v)[8]) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  const unsigned long long lo = (unsigned long long)pack_bf16x2(v[0], v[1]) |
                                ((unsigned long long)pack_bf16x2(v[2], v[3]) << 32);
  const unsigned long long hi = (unsigned long long)pack_bf16x2(v[4], v[5]) |
                                ((unsigned long long)pack_bf16x2(v[6], v[7]) << 32);
  __hip_atomic_store(q, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// either element type (DT, common.h)
template <int DT>
__device__ __forceinline__ void st_pub_e(bf16_t* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned short*>(p), (unsigned short)f2e<DT>(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
template <int DT>
__device__ __forceinline__ void st_pub_x8(bf16_t* p, const float (&v)[8]) {
  unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
  uint32_t w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = f2e<DT>(v[2 * j]) | (f2e<DT>(v[2 * j + 1]) << 16);
  __hip_atomic_store(q, (unsigned long long)w[0] | ((unsigned long long)w[1] << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, (unsigned long long)w[2] | ((unsigned long long)w[3] << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kDualSub = 64;  // sub-counters of gemv_dual_ln_kernel's arrival (cnt: 32 * (1 + 64) uints)

struct DualLn {
  const bf16_t* x1;    // [K1] (attention output)
  const bf16_t* w1;    // [N, K1]
  const bf16_t* x2;    // [K2] (GELU(fc_in)); nullable: one GEMV (sequential-residual layers)
  const bf16_t* w2;    // [N, K2]
  const bf16_t* bias;  // [N] (nullable)
  float* ypart;        // unused (kept in the C ABI)
  unsigned int* cnt;   // arrival counters, zero before the first launch, re-armed by the last workgroup
  const bf16_t* h;     // [N] residual stream in
  bf16_t* h_out;       // [N] h' = bf16(h + y + bias), written write-through by the workgroup that owns
                       // the rows (st_pub_bf16); the finishing workgroup reads it back
  const bf16_t* gamma; // next LayerNorm
  const bf16_t* beta;
  float eps;
  bf16_t* xn_out;      // [N] LN(h + y)
  const bf16_t* gamma2;  // nullable: a second LayerNorm of the same h + y (GPT-NeoX's ln_2: parallel
  const bf16_t* beta2;   // residual with two norms), sharing the statistics
  bf16_t* xn2_out;
  int N, K1, K2;
};

template <int PER, int DT = 0>
__device__ void dual_ln_finish(const DualLn& a);

// Arrival of the work of a fused decode tail launch, then -- in the last arrival -- the LayerNorm(s) of
// h' (DualLn), which the arriving workgroups have already written for their own rows into h_out.
// Two-level counting: thousands of arrivals on ONE address serialise at the memory side (~7 ns each:
// 5120 arrivals were +38 us per layer), so an arrival adds `n` items to sub-counter `sub` (of
// kDualSub, 128 B apart; `members` items in all arrive there) and the arrival that completes a
// sub-counter counts into the top one (cnt[0]; `nsub` sub-counters receive items). Default: one item per
// workgroup, sub = blockIdx % 64. 256-thread workgroups; PER: 2048-column slices (N <= 256 * 8 * PER).
template <int PER, int DT = 0>
__device__ void dual_ln_arrive(const DualLn& a, int sub, unsigned members, int nsub, unsigned n) {
  __shared__ int s_last;
  const int tid = threadIdx.x;
  // publish (cdna_hip_programming.md Guideline 16, R1): write-through stores drained, barrier, one
  // agent-scope arrival; the last arrival re-arms the counters and acquires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    unsigned* sc = a.cnt + 32 * (1 + sub);
    int last = 0;
    if (__hip_atomic_fetch_add(sc, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + n == members) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      last = __hip_atomic_fetch_add(a.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nsub - 1;
    }
    if (last) {
      __hip_atomic_store(a.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  const int last = s_last;
  __syncthreads();  // (s_last is rewritten by this workgroup's next arrival)
  if (last) dual_ln_finish<PER, DT>(a);
}

template <int PER, int DT = 0>
__device__ void dual_ln_arrive_tail(const DualLn& a) {
  constexpr int NSUB = kDualSub;
  const int G = gridDim.x, sub = blockIdx.x % NSUB;
  dual_ln_arrive<PER, DT>(a, sub, (unsigned)((G - sub + NSUB - 1) / NSUB), G < NSUB ? G : NSUB, 1u);
}

// The LayerNorm(s) of h' (h_out, complete and visible to this workgroup), written to xn_out (and
// xn2_out).
template <int PER, int DT>
__device__ void dual_ln_finish(const DualLn& a) {
  __shared__ float red[16];
  const int tid = threadIdx.x;
  // LN(h') -- the ln_rows_kernel math (statistics over the bf16-rounded sum). h' stays in registers
  // as packed bf16 (4 VGPRs per 8 columns) and gamma / beta are read in the last pass: this tail is
  // inlined into every workgroup of the launch, and its register peak sets the whole kernel's
  // occupancy (fp32 h' + prefetched gamma / beta + the partial sums' loads: 186 VGPRs, 2 waves per
  // SIMD at N > 8192).
  uint4 hp[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    hp[i] = make_uint4(0u, 0u, 0u, 0u);
    if (k < a.N) hp[i] = *reinterpret_cast<const uint4*>(a.h_out + k);
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const uint32_t q4[4] = {hp[i].x, hp[i].y, hp[i].z, hp[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) s += lo2f<DT>(q4[j]) + hi2f<DT>(q4[j]);
  }
  const float mean = block_sum(s, red) / a.N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if ((i * 256 + tid) * 8 >= a.N) continue;
    const uint32_t q4[4] = {hp[i].x, hp[i].y, hp[i].z, hp[i].w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = lo2f<DT>(q4[j]) - mean, hi = hi2f<DT>(q4[j]) - mean;
      q += lo * lo + hi * hi;
    }
  }
  const float rstd = rsqrtf(block_sum(q, red + 8) / a.N + a.eps);
  // normalise: h' re-read (this workgroup's L1 / L2 holds it) with gamma / beta, two slices in flight
  // at a time -- the packed copy above is dead here, so the peak stays at the first passes'
#pragma unroll 2
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k >= a.N) continue;
    float xh[8], gm[8], bt[8], o[8];
    load8_t<DT>(a.h_out + k, xh);
    load8_t<DT>(a.gamma + k, gm);
    if (a.beta) load8_t<DT>(a.beta + k, bt);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) bt[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xh[j] = (xh[j] - mean) * rstd;
      o[j] = xh[j] * gm[j] + bt[j];
    }
    store8_t<DT>(a.xn_out + k, o);
    if (a.xn2_out) {
      load8_t<DT>(a.gamma2 + k, gm);
      if (a.beta2) load8_t<DT>(a.beta2 + k, bt);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bt[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = xh[j] * gm[j] + bt[j];
      store8_t<DT>(a.xn2_out + k, o);
    }
  }
}

