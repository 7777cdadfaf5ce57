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

constexpr int kDualSub = 64;  // sub-counters of gemv_dual_ln_kernel's arrival (cnt: 32 * (1 + 64) uints)

struct DualLn {
  const bf16_t* x1;    // [K1] (attention output)
  const bf16_t* w1;    // [N, K1]
  const bf16_t* x2;    // [K2] (GELU(fc_in)); nullable: one GEMV (sequential-residual layers)
  const bf16_t* w2;    // [N, K2]
  const bf16_t* bias;  // [N] (nullable)
  float* ypart;        // [N] fp32 row results (write-through: the finishing workgroup reads them)
  unsigned int* cnt;   // arrival counters, zero before the first launch, re-armed by the last workgroup
  const bf16_t* h;     // [N] residual stream in
  bf16_t* h_out;       // [N] h + y (bf16)
  const bf16_t* gamma; // next LayerNorm
  const bf16_t* beta;
  float eps;
  bf16_t* xn_out;      // [N] LN(h + y)
  const bf16_t* gamma2;  // nullable: a second LayerNorm of the same h + y (GPT-NeoX's ln_2: parallel
  const bf16_t* beta2;   // residual with two norms), sharing the statistics
  bf16_t* xn2_out;
  int N, K1, K2;
};

// Arrival of every workgroup of a fused decode tail launch, then -- in the last one -- h' = bf16(h + y
// + bias) and its LayerNorm(s) (DualLn). ypart holds y. 256-thread workgroups; PER: h' register slices
// of 2048 columns (N <= 256 * 8 * PER).
template <int PER>
__device__ void dual_ln_arrive_tail(const DualLn& a) {
  __shared__ float red[16];
  __shared__ int s_last;
  const int tid = threadIdx.x;
  // publish (cdna_hip_programming.md Guideline 16, R1): write-through stores drained, barrier, one
  // agent-scope arrival; the last workgroup re-arms the counter and acquires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // two-level arrival: thousands of workgroups adding to ONE address serialise at the memory side
  // (~7 ns each: 5120 arrivals were +38 us per layer), so workgroup b counts into sub-counter b % 64
  // (128 B apart) and each sub-counter's last arrival counts into the top one (cnt[0])
  if (tid == 0) {
    constexpr int NSUB = kDualSub;
    const int G = gridDim.x, sub = blockIdx.x % NSUB;
    const int nsub = G < NSUB ? G : NSUB;
    const unsigned members = (unsigned)((G - sub + NSUB - 1) / NSUB);
    unsigned* sc = a.cnt + 32 * (1 + sub);
    int last = 0;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
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
  if (!s_last) return;
  // h' = bf16(h + y + b), LN(h') -- the ln_rows_kernel math (statistics over the bf16-rounded sum);
  // gamma / beta requested in the same memory round trip as the partials (they do not depend on them)
  float hv[PER][8];
  U16x8 gr[PER], br[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k < a.N) {
      gr[i] = *reinterpret_cast<const U16x8*>(a.gamma + k);
      if (a.beta) br[i] = *reinterpret_cast<const U16x8*>(a.beta + k);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k < a.N) {
      float y8[8], b8[8];
      load8f(a.ypart + k, y8);
      if (a.bias) {
        load8(a.bias + k, b8);
#pragma unroll
        for (int j = 0; j < 8; ++j) y8[j] += b8[j];
      }
      load8(a.h + k, hv[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        hv[i][j] = bf2f(f2bf(hv[i][j] + y8[j]));
        s += hv[i][j];
      }
      store8(a.h_out + k, hv[i]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[i][j] = 0.f;
    }
  }
  const float mean = block_sum(s, red) / a.N;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if ((i * 256 + tid) * 8 >= a.N) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) q += (hv[i][j] - mean) * (hv[i][j] - mean);
  }
  const float rstd = rsqrtf(block_sum(q, red + 8) / a.N + a.eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k >= a.N) continue;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) hv[i][j] = (hv[i][j] - mean) * rstd;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = hv[i][j] * bf2f(gr[i].v[j]) + (a.beta ? bf2f(br[i].v[j]) : 0.f);
    store8(a.xn_out + k, o);
    if (a.xn2_out) {
      float gm[8], bt[8];
      load8(a.gamma2 + k, gm);
      if (a.beta2) load8(a.beta2 + k, bt);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bt[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = hv[i][j] * gm[j] + bt[j];
      store8(a.xn2_out + k, o);
    }
  }
}

