// GroupNorm(32) (+ fused SiLU) forward / backward for the UNet and VAE ResNet
// blocks (K14 in SURVEY §2.4; sd-finetuner/finetuner.py:470-500 and the
// txt2img predictor run these through diffusers' nn.GroupNorm + F.silu).
//
// Layout NCHW, bf16 in/out, fp32 statistics. A (n, c) plane of HW elements is
// contiguous, and a group is C/G consecutive planes, so:
//   fwd  1) plane_stats : one workgroup per plane -> Welford (mean, M2)
//        2) gn_apply    : one workgroup per plane, merges its group's C/G plane
//                         partials (Chan's parallel Welford; exact, no
//                         E[x^2]-E[x]^2 cancellation), normalises, affine, SiLU,
//                         and the group's first plane records (mean, rstd)
//   bwd  1) plane_grads : per plane  sum(g*dyp), sum(g*dyp*xhat), and the
//                         per-(n,c) dgamma/dbeta partials (dyp = dy * silu')
//        2) gn_dx       : per plane, merges the group sums -> dx
//        3) dgamma/dbeta: sum the N plane partials per channel
// Every pass streams the plane with 16-B loads; no atomics (deterministic).
#include "common.h"

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = 1.f / (1.f + __expf(-x));
  return s * (1.f + x * (1.f - s));
}

// Block-wide Welford merge of per-thread (n, mean, M2).
__device__ void block_welford(float& n, float& mean, float& m2, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float n2 = __shfl_xor(n, o, 64), mu2 = __shfl_xor(mean, o, 64), q2 = __shfl_xor(m2, o, 64);
    const float nt = n + n2;
    if (nt > 0.f) {
      const float d = mu2 - mean;
      mean += d * n2 / nt;
      m2 += q2 + d * d * n * n2 / nt;
      n = nt;
    }
  }
  __syncthreads();
  if (lane == 0) { red[wid * 3] = n; red[wid * 3 + 1] = mean; red[wid * 3 + 2] = m2; }
  __syncthreads();
  n = 0.f; mean = 0.f; m2 = 0.f;
  for (int w = 0; w < nw; ++w) {
    const float n2 = red[w * 3], mu2 = red[w * 3 + 1], q2 = red[w * 3 + 2];
    const float nt = n + n2;
    if (nt > 0.f) {
      const float d = mu2 - mean;
      mean += d * n2 / nt;
      m2 += q2 + d * d * n * n2 / nt;
      n = nt;
    }
  }
}

__global__ void __launch_bounds__(256) gn_plane_stats(const bf16_t* __restrict__ x, int hw,
                                                      float* __restrict__ part) {
  __shared__ float red[48];
  const long long plane = blockIdx.x;
  const bf16_t* p = x + plane * hw;
  // shifted sums per thread (shift = first element: no catastrophic cancellation
  // for offset-heavy activations), then an exact Welford merge across threads
  const float K = bf2f(p[0]);
  float cnt = 0.f, s1 = 0.f, s2 = 0.f;
  if ((hw % 8) == 0) {
    for (int i = threadIdx.x; i < hw / 8; i += blockDim.x) {
      float v[8];
      load8(p + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - K;
        s1 += d;
        s2 += d * d;
      }
      cnt += 8.f;
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += blockDim.x) {
      const float d = bf2f(p[i]) - K;
      s1 += d;
      s2 += d * d;
      cnt += 1.f;
    }
  }
  float n = cnt, mean = 0.f, m2 = 0.f;
  if (cnt > 0.f) {
    mean = K + s1 / cnt;
    m2 = fmaxf(s2 - s1 * s1 / cnt, 0.f);
  }
  block_welford(n, mean, m2, red);
  if (threadIdx.x == 0) {
    part[plane * 2] = mean;
    part[plane * 2 + 1] = m2;
  }
}

__device__ __forceinline__ void group_stats(const float* part, long long plane0, int cpg, int hw,
                                            float eps, float& mean, float& rstd) {
  float n = 0.f, mu = 0.f, m2 = 0.f;
  for (int c = 0; c < cpg; ++c) {
    const float n2 = (float)hw, mu2 = part[(plane0 + c) * 2], q2 = part[(plane0 + c) * 2 + 1];
    const float nt = n + n2;
    const float d = mu2 - mu;
    mu += d * n2 / nt;
    m2 += q2 + d * d * n * n2 / nt;
    n = nt;
  }
  mean = mu;
  rstd = rsqrtf(m2 / n + eps);
}

__global__ void __launch_bounds__(256) gn_apply(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                const float* __restrict__ part, float* __restrict__ mean_out,
                                                float* __restrict__ rstd_out, int C, int hw, int G,
                                                float eps, int silu) {
  const long long plane = blockIdx.x;
  const int c = plane % C;
  const long long n = plane / C;
  const int cpg = C / G, g = c / cpg;
  const long long plane0 = n * C + (long long)g * cpg;
  float mean, rstd;
  group_stats(part, plane0, cpg, hw, eps, mean, rstd);
  if (threadIdx.x == 0 && c % cpg == 0) {
    mean_out[n * G + g] = mean;
    rstd_out[n * G + g] = rstd;
  }
  const float gw = bf2f(w[c]) * rstd;
  const float gb = (b ? bf2f(b[c]) : 0.f) - mean * gw;
  const bf16_t* p = x + plane * hw;
  bf16_t* q = y + plane * hw;
  if ((hw % 8) == 0) {
    for (int i = threadIdx.x; i < hw / 8; i += blockDim.x) {
      float v[8];
      load8(p + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = v[j] * gw + gb;
        if (silu) v[j] = silu_f(v[j]);
      }
      store8(q + i * 8, v);
    }
  } else {
    for (int i = threadIdx.x; i < hw; i += blockDim.x) {
      float v = bf2f(p[i]) * gw + gb;
      q[i] = f2bf(silu ? silu_f(v) : v);
    }
  }
}

// per plane: s1 = sum(gam*dyp), s2 = sum(gam*dyp*xhat), dgp = sum(dyp*xhat), dbp = sum(dyp)
__global__ void __launch_bounds__(256) gn_plane_grads(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                      const float* __restrict__ mean_g,
                                                      const float* __restrict__ rstd_g, int C, int hw, int G,
                                                      int silu, float* __restrict__ ws) {
  __shared__ float red[16];
  const long long plane = blockIdx.x;
  const int c = plane % C;
  const long long n = plane / C;
  const int g = c / (C / G);
  const float mean = mean_g[n * G + g], rstd = rstd_g[n * G + g];
  const float gam = bf2f(w[c]), bet = b ? bf2f(b[c]) : 0.f;
  const bf16_t* px = x + plane * hw;
  const bf16_t* pd = dy + plane * hw;
  float a_dy = 0.f, a_dyx = 0.f;
  for (int i = threadIdx.x; i < hw; i += blockDim.x) {
    const float xh = (bf2f(px[i]) - mean) * rstd;
    float d = bf2f(pd[i]);
    if (silu) d *= silu_grad(xh * gam + bet);
    a_dy += d;
    a_dyx += d * xh;
  }
  const float s_dy = block_sum(a_dy, red);
  const float s_dyx = block_sum(a_dyx, red + 8);
  if (threadIdx.x == 0) {
    ws[plane * 4 + 0] = gam * s_dy;
    ws[plane * 4 + 1] = gam * s_dyx;
    ws[plane * 4 + 2] = s_dyx;  // dgamma partial
    ws[plane * 4 + 3] = s_dy;   // dbeta partial
  }
}

__global__ void __launch_bounds__(256) gn_dx(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                             const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                             const float* __restrict__ mean_g, const float* __restrict__ rstd_g,
                                             const float* __restrict__ ws, int C, int hw, int G, int silu,
                                             bf16_t* __restrict__ dx) {
  const long long plane = blockIdx.x;
  const int c = plane % C;
  const long long n = plane / C;
  const int cpg = C / G, g = c / cpg;
  const float mean = mean_g[n * G + g], rstd = rstd_g[n * G + g];
  float A = 0.f, Bv = 0.f;
  for (int k = 0; k < cpg; ++k) {
    const long long pl = n * C + (long long)g * cpg + k;
    A += ws[pl * 4];
    Bv += ws[pl * 4 + 1];
  }
  const float M = (float)cpg * hw;
  A /= M;
  Bv /= M;
  const float gam = bf2f(w[c]), bet = b ? bf2f(b[c]) : 0.f;
  const bf16_t* px = x + plane * hw;
  const bf16_t* pd = dy + plane * hw;
  bf16_t* po = dx + plane * hw;
  for (int i = threadIdx.x; i < hw; i += blockDim.x) {
    const float xh = (bf2f(px[i]) - mean) * rstd;
    float d = bf2f(pd[i]);
    if (silu) d *= silu_grad(xh * gam + bet);
    po[i] = f2bf(rstd * (gam * d - A - xh * Bv));
  }
}

__global__ void gn_param_grads(const float* __restrict__ ws, int N, int C, bf16_t* __restrict__ dw,
                               bf16_t* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float sg = 0.f, sb = 0.f;
  for (int n = 0; n < N; ++n) {
    sg += ws[((long long)n * C + c) * 4 + 2];
    sb += ws[((long long)n * C + c) * 4 + 3];
  }
  dw[c] = f2bf(sg);
  if (db) db[c] = f2bf(sb);
}

// part: >= N*C*2 floats scratch (caller-owned: no allocation in the launch path)
KCA_API int kca_groupnorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                              float* part, int N, int C, int hw, int G, float eps, int silu,
                              hipStream_t stream) {
  if (C % G) return 1;
  const int planes = N * C;
  const int th = hw >= 2048 ? 256 : (hw >= 512 ? 128 : 64);
  hipLaunchKernelGGL(gn_plane_stats, dim3(planes), dim3(th), 0, stream, (const bf16_t*)x, hw, part);
  hipLaunchKernelGGL(gn_apply, dim3(planes), dim3(th), 0, stream, (const bf16_t*)x, (const bf16_t*)w,
                     (const bf16_t*)b, (bf16_t*)y, part, mean, rstd, C, hw, G, eps, silu);
  return 0;
}

// ws: >= 4*N*C floats scratch
KCA_API int kca_groupnorm_bwd(const void* dy, const void* x, const void* w, const void* b, const float* mean,
                              const float* rstd, void* dx, void* dw, void* db, float* ws, int N, int C,
                              int hw, int G, int silu, hipStream_t stream) {
  if (C % G) return 1;
  const int planes = N * C;
  const int th = hw >= 2048 ? 256 : (hw >= 512 ? 128 : 64);
  hipLaunchKernelGGL(gn_plane_grads, dim3(planes), dim3(th), 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                     (const bf16_t*)w, (const bf16_t*)b, mean, rstd, C, hw, G, silu, ws);
  hipLaunchKernelGGL(gn_dx, dim3(planes), dim3(th), 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                     (const bf16_t*)w, (const bf16_t*)b, mean, rstd, ws, C, hw, G, silu, (bf16_t*)dx);
  hipLaunchKernelGGL(gn_param_grads, dim3((C + 255) / 256), dim3(256), 0, stream, ws, N, C, (bf16_t*)dw,
                     (bf16_t*)db);
  return 0;
}
