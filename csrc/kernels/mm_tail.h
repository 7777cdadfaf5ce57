// Row-statistics tail of the batched decode layer (M = 2..64 rows), shared by skinny_mfma.hip (the
// out-projection / fc_out GEMMs that close a residual branch) and csrc/comm/xgmi_allreduce.hip (the
// tensor-parallel all-reduce that closes a row-parallel projection).
//
// The batch-1 tail (decode_tail.h) normalises the whole new residual row in the last-arriving
// workgroup. At M rows that is M x N elements through one workgroup (BLOOM B=32: 917 KB), so here
// the producer only publishes statistics: every `tw`-column slice of every row contributes its own
// (mean, M2) -- exact two-pass over 16 values, merged up to the slice inside the producing workgroup --
// and the last arriver merges them (Chan's parallel variance: all slices hold tw values, so
// mean = avg(mean_t), M2 = sum(M2_t) + tw sum (mean_t - mean)^2) into (mean, rstd) per row. The
// consumer GEMM (next QKV / fc_in / LM head) normalises its activation fragments on load
// (skinny_mfma.hip, LN-on-load), so no LayerNorm launch and no normalised-row round trip exists in
// the layer loop.
#pragma once
#include "decode_tail.h"

struct RowStats {
  float* part;     // [M][N/tw][2] per-slice (mean, M2), published with st_pub
  float* stats;    // [M][2] (mean, rstd) -- written by the last arriver
  unsigned* cnt;   // 32 * (1 + 64) arrival counters, zero before the first launch, re-armed every launch
  int M, N;        // N % tw == 0
  float eps;
  int tw;          // columns per published partial
};

// Publish one slice's partial (called by one thread per (row, slice)).
__device__ __forceinline__ void rs_publish(const RowStats& s, int m, int slice, float mean_t, float m2_t) {
  float* p = s.part + ((long long)m * (s.N / s.tw) + slice) * 2;
  st_pub(p, mean_t);
  st_pub(p + 1, m2_t);
}

// Chan merge of n equal-count groups' (mean, M2) (count c each)
template <int n>
__device__ __forceinline__ void chan_merge(const float (&mean)[n], const float (&m2)[n], float c, float& mo,
                                           float& m2o) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < n; ++i) s += mean[i];
  mo = s * (1.f / n);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < n; ++i) q += m2[i] + c * (mean[i] - mo) * (mean[i] - mo);
  m2o = q;
}

// (mean, M2) of 16 values spread as 4 per lane over the 4 lanes {l, l^16, l^32, l^48} (the
// mfma_f32_16x16x32 C layout: one output column per lane & 15, four rows per lane >> 4).
__device__ __forceinline__ void rs_tile16(const float (&v)[4], float& mean_t, float& m2_t) {
  float s = v[0] + v[1] + v[2] + v[3];
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  mean_t = s * (1.f / 16.f);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) q += (v[i] - mean_t) * (v[i] - mean_t);
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  m2_t = q;
}

// The last arriver: merge the slices of every row. One wave per group of RG rows, lanes over slices,
// every load of the group issued before any is used (a row-at-a-time loop was a chain of dependent L2
// round trips: +100-200 us per step at B = 32, profiles/decode_suite_r6_v1_batched.jsonl).
__device__ __forceinline__ void rs_merge(const RowStats& s) {
  constexpr int RG = 4, PL = 4;  // rows per group, slices per lane (NT <= 256)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int NT = s.N / s.tw;
  for (int m0 = wv * RG; m0 < s.M; m0 += nw * RG) {
    float mt[RG][PL], qt[RG][PL];
#pragma unroll
    for (int r = 0; r < RG; ++r)
#pragma unroll
      for (int i = 0; i < PL; ++i) {
        const int t = lane + 64 * i, m = m0 + r;
        mt[r][i] = 0.f;
        qt[r][i] = 0.f;
        if (m < s.M && t < NT) {
          const float2 v = *reinterpret_cast<const float2*>(s.part + ((long long)m * NT + t) * 2);
          mt[r][i] = v.x;
          qt[r][i] = v.y;
        }
      }
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < PL; ++i) sm += mt[r][i];
      const float mean = wave_sum(sm) / NT;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < PL; ++i)
        if (lane + 64 * i < NT) q += qt[r][i] + s.tw * (mt[r][i] - mean) * (mt[r][i] - mean);
      const float var = wave_sum(q) / s.N;
      if (lane == 0 && m0 + r < s.M) {
        s.stats[2 * (m0 + r)] = mean;
        s.stats[2 * (m0 + r) + 1] = rsqrtf(var + s.eps);
      }
    }
  }
}

// Arrival of one workgroup (every thread calls it): the decode_tail.h protocol -- write-through
// partials drained, barrier, a two-level agent-scope count (sub-counter `sub` of 64, `members`
// arrivals there; `nsub` sub-counters in use), the last arrival re-arms the counters, acquires, and
// merges. `seq` (the all-reduce close, xgmi_allreduce.hip): the last arrival also advances the
// all-reduce's sequence word to `call` -- every workgroup has read it by then -- so that kernel needs
// no finished-block count of its own.
__device__ __forceinline__ void rs_arrive(const RowStats& s, int sub, unsigned members, int nsub,
                                          uint32_t* seq = nullptr, uint32_t call = 0) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* sc = s.cnt + 32 * (1 + sub);
    int last = 0;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == members) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(s.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nsub - 1;
    }
    if (last) {
      __hip_atomic_store(s.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (seq) __hip_atomic_store(seq, call, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  const int last = s_last;
  __syncthreads();
  if (last) rs_merge(s);
}

// Arrival of workgroup `b` of `G` taking part in one tail.
__device__ __forceinline__ void rs_arrive_of(const RowStats& s, int b, int G, uint32_t* seq = nullptr,
                                             uint32_t call = 0) {
  constexpr int NSUB = kDualSub;
  const int sub = b % NSUB;
  rs_arrive(s, sub, (unsigned)((G - sub + NSUB - 1) / NSUB), G < NSUB ? G : NSUB, seq, call);
}
