// Single-row (decode batch 1) weight-streaming pieces shared by gemv.hip (the skinny GEMM / GEMV
// kernels) and decode.hip (the fused decode-layer kernels). DT: element type (common.h e2f).
#pragma once
#include "common.h"

struct LnArgs {
  const bf16_t* r1;     // residual adds (nullable): h = x (+ r1) (+ r2)
  const bf16_t* r2;
  bf16_t* h_out;        // updated residual stream, written by workgroup 0 (nullable)
  long long ldh;        // row stride of r1 / r2 / h_out
  const bf16_t* gamma;  // [K]
  const bf16_t* beta;   // [K] (nullable)
  float eps;
  bf16_t* xn_out;       // normalised rows [M][K], written by workgroup 0 (nullable): GPT-J's shared LN
                        // feeds the fc_in GEMV too, which then skips its own prologue
};

// Weight stream loads: every weight byte of a decode GEMV is read once, by one workgroup, so
// they are non-temporal (global_load_dwordx4 ... nt): they do not displace the L2 / MALL lines the
// latency-bound attention chain and the activations re-read (MI355X_MICROARCH.md, nt-weights:
// decode layers 5-10 % faster with nt weight streams).
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_w16(const bf16_t* p) {
  const u32x4_nt v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// acc[r] += W[n0 + r, :K] . x[:K] for the lane's K slice (K-split over the 256 threads: lane (wave
// w, lane l) owns positions i*2048 + w*512 + l*8), R weight rows, 16 / R slabs of loads in flight --
// the gemv1_kernel<R, false, 1> loop (gemv.hip) as a device function, so that a fused kernel can
// run it on a subset of its workgroups. Not reduced across lanes: call gemv_m1_finish.
template <int R, int UO = 0, int DT = 0>
__device__ __forceinline__ void gemv_m1_accum(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, int N,
                                              int K, int n0, float (&acc)[R], long long ldw = -1) {
  if (ldw < 0) ldw = K;  // row stride of w (a K-chunk of a wider matrix: the full row length)
  // 16 weight loads in flight per lane, any R (UO: another slab count)
  constexpr int U = UO > 0 ? UO : (R >= 16 ? 1 : (R >= 8 ? 2 : 4));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kl = wid * 512 + lane * 8;
  const bf16_t* wr[R];
  bool rv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    rv[r] = n0 + r < N;
    wr[r] = w + (long long)(rv[r] ? n0 + r : 0) * ldw;
  }
  const int NI = (K + 2047) / 2048;
  for (int i0 = 0; i0 < NI; i0 += U) {
    uint4 wv[U][R];
    uint4 xr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (i0 + u) * 2048 + kl;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        wv[u][r] = make_uint4(0u, 0u, 0u, 0u);
        if (k < K && rv[r]) wv[u][r] = ld_w16(wr[r] + k);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (i0 + u) * 2048 + kl;
      xr[u] = make_uint4(0u, 0u, 0u, 0u);
      if (k < K) xr[u] = *reinterpret_cast<const uint4*>(x + k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if ((i0 + u) * 2048 + kl >= K) continue;
      const uint32_t xq[4] = {xr[u].x, xr[u].y, xr[u].z, xr[u].w};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t q[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r] = dot2_acc<DT>(q[j], xq[j], acc[r]);
      }
    }
  }
}

// Reduce the R per-lane partial dots over the workgroup (waves in LDS `part` [4][R]) and apply
// bias + activation (0 none, 1 GELU tanh, 2 GELU erf). Returns the value for row n0 + tid in
// threads tid < R (valid iff n0 + tid < N); callers store it.
template <int R, int DT = 0>
__device__ __forceinline__ float gemv_m1_finish(float (&acc)[R], float (*part)[R], const bf16_t* __restrict__ bias,
                                                int n0, int N, int act) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) part[wid][r] = acc[r];
  }
  __syncthreads();
  float v = 0.f;
  if (tid < R && n0 + tid < N) {
    v = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    v += bias ? e2f<DT>(bias[n0 + tid]) : 0.f;
    if (act == 1) v = gelu_tanh(v);
    else if (act == 2) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  }
  return v;
}
