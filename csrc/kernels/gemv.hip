// Skinny GEMM for decode: y[M, N] = act(x[M, K] . W[N, K]^T + b), M <= 16.
//
// Decode GEMMs are weight-streaming bound (BLOOM-176B TP=8: ~44 GB of weights
// per token per GPU; GPT-J: 12 GB), so the kernel is built to read W exactly
// once at HBM speed: every lane streams 16-byte chunks of R weight rows with
// 4 K-steps unrolled (R*4 independent 16 B loads in flight per lane), the M
// activation rows are staged once per workgroup in LDS (K-chunked so M*Kc
// fits in 64 KB) and read with conflict-free ds_read_b128, fp32 accumulation,
// one wave-reduction per (row, m) at the end. Bias and GELU (tanh or erf) are
// fused into the store, replacing the separate bias/GELU kernels of the
// FT / DS-Inference decoders (SURVEY K1/K5 decode shapes).
#include "common.h"

template <int M, int R>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(
    const bf16_t* __restrict__ x, long long ldx, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ bias, bf16_t* __restrict__ y, long long ldy, int N, int K,
    int kc, int act, int mv) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];  // [M][kc]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  float acc[R][M];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
  const bf16_t* wr[R];
  bool rv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    rv[r] = n0 + r < N;
    wr[r] = w + (long long)(rv[r] ? n0 + r : 0) * K;
  }
  for (int k0 = 0; k0 < K; k0 += kc) {
    const int kn = min(kc, K - k0);
    __syncthreads();
    for (int i = tid * 8; i < M * kn; i += 256 * 8) {
      const int m = i / kn, kk = i % kn;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);  // rows >= mv (padding of M) stay zero
      if (m < mv) v = *reinterpret_cast<const uint4*>(x + m * ldx + k0 + kk);
      *reinterpret_cast<uint4*>(xs + m * kc + kk) = v;
    }
    __syncthreads();
    // 4 K-steps of 512 elements per iteration: R*4 independent 16 B loads per lane
    for (int kb = lane * 8; kb < kn; kb += 4 * 512) {
      uint4 wv[4][R];  // raw bf16 (4 VGPRs per 8 weights), widened at use
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + u * 512;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          wv[u][r] = make_uint4(0u, 0u, 0u, 0u);
          if (k < kn && rv[r]) wv[u][r] = *reinterpret_cast<const uint4*>(wr[r] + k0 + k);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + u * 512;
        if (k < kn) {
#pragma unroll
          for (int m = 0; m < M; ++m) {
            float xv[8];
            load8(xs + m * kc + k, xv);
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const uint32_t q[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                acc[r][m] = fmaf(__uint_as_float(q[j] << 16), xv[2 * j], acc[r][m]);
                acc[r][m] = fmaf(__uint_as_float(q[j] & 0xffff0000u), xv[2 * j + 1], acc[r][m]);
              }
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = wave_sum(acc[r][m]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!rv[r]) continue;
      const float b = bias ? bf2f(bias[n0 + r]) : 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (m >= mv) break;
        float v = acc[r][m] + b;
        if (act == 1) v = gelu_tanh(v);
        else if (act == 2) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        y[m * ldy + n0 + r] = f2bf(v);
      }
    }
  }
}

template <int M>
static void launch_skinny(const bf16_t* x, long long ldx, const bf16_t* w, const bf16_t* bias,
                          bf16_t* y, long long ldy, int mv, int N, int K, int act, hipStream_t s) {
  constexpr int R = (M <= 4) ? 4 : 2;
  int kc = (32768 / M) / 512 * 512;  // M*kc*2 B <= 64 KB of LDS
  if (kc < 512) kc = 512;
  if (kc > K) kc = (K + 7) / 8 * 8;
  const int rows_per_block = 4 * R;
  const dim3 grid((N + rows_per_block - 1) / rows_per_block);
  hipLaunchKernelGGL((skinny_gemm_kernel<M, R>), grid, dim3(256), (size_t)M * kc * sizeof(bf16_t), s,
                     x, ldx, w, bias, y, ldy, N, K, kc, act, mv);
}

KCA_API int kca_skinny_gemm(const void* x, long long ldx, const void* w, const void* bias, void* y,
                            long long ldy, int M, int N, int K, int act, hipStream_t stream) {
  if (M < 1 || M > 16 || K % 8 || ldx % 8 || N < 1) return 1;
  if (((uintptr_t)x | (uintptr_t)w) & 15) return 2;
  const bf16_t* xp = (const bf16_t*)x;
  const bf16_t* wp = (const bf16_t*)w;
  const bf16_t* bp = (const bf16_t*)bias;
  bf16_t* yp = (bf16_t*)y;
  // one launch, M padded up to the next instantiated row count (W is read once)
  if (M == 1) launch_skinny<1>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else if (M == 2) launch_skinny<2>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else if (M <= 4) launch_skinny<4>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else if (M <= 8) launch_skinny<8>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else launch_skinny<16>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  return 0;
}
