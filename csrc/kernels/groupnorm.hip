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

#include <algorithm>

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


// ------------------------------------------------------------ forward, sliced
// The per-plane kernels above launch one workgroup per (n, c) plane: at the
// UNet's 8x8..64x64 planes that is thousands of 64..4096-element workgroups
// plus a serial cpg-way partial merge in each. The sliced form works on the
// group instead: a group (n, g) is cpg*hw CONTIGUOUS elements (its channels'
// planes are adjacent in NCHW), cut into S slices of SL elements chosen so the
// grid holds ~2048 workgroups of >= 8K elements (S <= cpg keeps the partials
// inside the caller's 2*N*C scratch). Stats: shifted sums + Welford per slice.
// Apply: merge the S slice partials (exact Chan merge), stage the group's
// per-channel scale/shift in LDS, normalise the slice with 16-B accesses.
__global__ void __launch_bounds__(256) gn_slice_stats(const bf16_t* __restrict__ x, long long Lg, long long SL,
                                                      int S, float* __restrict__ part) {
  __shared__ float red[48];
  const long long grp = blockIdx.x / S;
  const long long a = (long long)(blockIdx.x % S) * SL, e = min(a + SL, Lg);
  const bf16_t* p = x + grp * Lg;
  const float K = bf2f(p[a]);
  float cnt = 0.f, s1 = 0.f, s2 = 0.f;
  if ((SL % 8) == 0 && (Lg % 8) == 0) {
    for (long long i = a / 8 + threadIdx.x; i < e / 8; i += blockDim.x) {
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
    for (long long i = a + threadIdx.x; i < e; i += blockDim.x) {
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
    part[blockIdx.x * 2] = mean;
    part[blockIdx.x * 2 + 1] = m2;
  }
}

__global__ void __launch_bounds__(256) gn_slice_apply(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                      const float* __restrict__ part, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out, int C, int hw, int G,
                                                      long long Lg, long long SL, int S, float eps, int silu) {
  constexpr int MAXC = 128;
  __shared__ float sgw[MAXC], sgb[MAXC];
  const long long grp = blockIdx.x / S;
  const int s = blockIdx.x % S;
  const int g = (int)(grp % G), cpg = C / G;
  float nn = 0.f, mu = 0.f, m2 = 0.f;
  for (int k = 0; k < S; ++k) {
    const float n2 = (float)min(SL, Lg - (long long)k * SL);
    const float mu2 = part[(grp * S + k) * 2], q2 = part[(grp * S + k) * 2 + 1];
    const float nt = nn + n2;
    const float d = mu2 - mu;
    mu += d * n2 / nt;
    m2 += q2 + d * d * nn * n2 / nt;
    nn = nt;
  }
  const float rstd = rsqrtf(m2 / nn + eps);
  if (threadIdx.x == 0 && s == 0) {
    mean_out[grp] = mu;
    rstd_out[grp] = rstd;
  }
  const bool staged = cpg <= MAXC;
  if (staged) {
    for (int c = threadIdx.x; c < cpg; c += blockDim.x) {
      const int cc = g * cpg + c;
      const float gw = bf2f(w[cc]) * rstd;
      sgw[c] = gw;
      sgb[c] = (b ? bf2f(b[cc]) : 0.f) - mu * gw;
    }
    __syncthreads();
  }
  const long long a = (long long)s * SL, e = min(a + SL, Lg);
  const bf16_t* p = x + grp * Lg;
  bf16_t* q = y + grp * Lg;
  if ((SL % 8) == 0 && (hw % 8) == 0) {
    for (long long i = a / 8 + threadIdx.x; i < e / 8; i += blockDim.x) {
      const int cl = (int)((i * 8) / hw);
      float gw, gb;
      if (staged) { gw = sgw[cl]; gb = sgb[cl]; }
      else { gw = bf2f(w[g * cpg + cl]) * rstd; gb = (b ? bf2f(b[g * cpg + cl]) : 0.f) - mu * gw; }
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
    for (long long i = a + threadIdx.x; i < e; i += blockDim.x) {
      const int cl = (int)(i / hw);
      float gw, gb;
      if (staged) { gw = sgw[cl]; gb = sgb[cl]; }
      else { gw = bf2f(w[g * cpg + cl]) * rstd; gb = (b ? bf2f(b[g * cpg + cl]) : 0.f) - mu * gw; }
      const float v = bf2f(p[i]) * gw + gb;
      q[i] = f2bf(silu ? silu_f(v) : v);
    }
  }
}

// ------------------------------------------------------- backward, vectorised
// Same per-plane partials as gn_plane_grads / gn_dx, but TPP threads per plane
// (one wave for planes under 2K elements, four planes per workgroup) and 16-B
// loads: the scalar per-plane loops above issued one 2-byte load per element.
template <int TPP>
__global__ void __launch_bounds__(256) gn_plane_grads_v(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                        const float* __restrict__ mean_g,
                                                        const float* __restrict__ rstd_g, int C, int hw, int G,
                                                        int silu, long long planes, float* __restrict__ ws) {
  __shared__ float red[16];
  constexpr int PPB = 256 / TPP;
  const long long plane = (long long)blockIdx.x * PPB + threadIdx.x / TPP;
  const int t = threadIdx.x % TPP;
  float a_dy = 0.f, a_dyx = 0.f;
  float gam = 0.f;
  if (plane < planes) {
    const int c = (int)(plane % C);
    const long long n = plane / C;
    const int g = c / (C / G);
    const float mean = mean_g[n * G + g], rstd = rstd_g[n * G + g];
    gam = bf2f(w[c]);
    const float bet = b ? bf2f(b[c]) : 0.f;
    const bf16_t* px = x + plane * hw;
    const bf16_t* pd = dy + plane * hw;
    for (int i = t; i < hw / 8; i += TPP) {
      float xv[8], dv[8];
      load8(px + i * 8, xv);
      load8(pd + i * 8, dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (xv[j] - mean) * rstd;
        float d = dv[j];
        if (silu) d *= silu_grad(xh * gam + bet);
        a_dy += d;
        a_dyx += d * xh;
      }
    }
  }
  float s_dy, s_dyx;
  if (TPP == 64) {
    s_dy = wave_sum(a_dy);
    s_dyx = wave_sum(a_dyx);
  } else {
    s_dy = block_sum(a_dy, red);
    s_dyx = block_sum(a_dyx, red + 8);
  }
  if (t == 0 && plane < planes) {
    ws[plane * 4 + 0] = gam * s_dy;
    ws[plane * 4 + 1] = gam * s_dyx;
    ws[plane * 4 + 2] = s_dyx;
    ws[plane * 4 + 3] = s_dy;
  }
}

template <int TPP>
__global__ void __launch_bounds__(256) gn_dx_v(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                               const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                               const float* __restrict__ mean_g, const float* __restrict__ rstd_g,
                                               const float* __restrict__ ws, int C, int hw, int G, int silu,
                                               long long planes, bf16_t* __restrict__ dx) {
  constexpr int PPB = 256 / TPP;
  const long long plane = (long long)blockIdx.x * PPB + threadIdx.x / TPP;
  if (plane >= planes) return;
  const int t = threadIdx.x % TPP;
  const int c = (int)(plane % C);
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
  for (int i = t; i < hw / 8; i += TPP) {
    float xv[8], dv[8], o[8];
    load8(px + i * 8, xv);
    load8(pd + i * 8, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (xv[j] - mean) * rstd;
      float d = dv[j];
      if (silu) d *= silu_grad(xh * gam + bet);
      o[j] = rstd * (gam * d - A - xh * Bv);
    }
    store8(po + i * 8, o);
  }
}

// part: >= N*C*2 floats scratch (caller-owned: no allocation in the launch path)
KCA_API int kca_groupnorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                              float* part, int N, int C, int hw, int G, float eps, int silu,
                              hipStream_t stream) {
  if (C % G) return 1;
  const int cpg = C / G;
  const long long NG = (long long)N * G, Lg = (long long)cpg * hw;
  long long S = (2048 + NG - 1) / NG;           // ~2048 workgroups
  S = std::min<long long>(S, cpg);              // partials fit the 2*N*C scratch
  S = std::min<long long>(S, std::max<long long>(1, Lg / 8192));  // >= 8K elements per slice
  if (S < 1) S = 1;
  long long SL = (Lg + S - 1) / S;
  if (hw % 8 == 0) SL = (SL + 7) / 8 * 8;
  S = (Lg + SL - 1) / SL;
  hipLaunchKernelGGL(gn_slice_stats, dim3((unsigned)(NG * S)), dim3(256), 0, stream, (const bf16_t*)x, Lg, SL,
                     (int)S, part);
  hipLaunchKernelGGL(gn_slice_apply, dim3((unsigned)(NG * S)), dim3(256), 0, stream, (const bf16_t*)x,
                     (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, part, mean, rstd, C, hw, G, Lg, SL, (int)S,
                     eps, silu);
  return 0;
}

// ws: >= 4*N*C floats scratch
KCA_API int kca_groupnorm_bwd(const void* dy, const void* x, const void* w, const void* b, const float* mean,
                              const float* rstd, void* dx, void* dw, void* db, float* ws, int N, int C,
                              int hw, int G, int silu, hipStream_t stream) {
  if (C % G) return 1;
  const int planes = N * C;
  if (hw % 8 == 0) {
    if (hw >= 2048) {
      hipLaunchKernelGGL((gn_plane_grads_v<256>), dim3(planes), dim3(256), 0, stream, (const bf16_t*)dy,
                         (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)b, mean, rstd, C, hw, G, silu,
                         (long long)planes, ws);
      hipLaunchKernelGGL((gn_dx_v<256>), dim3(planes), dim3(256), 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                         (const bf16_t*)w, (const bf16_t*)b, mean, rstd, ws, C, hw, G, silu, (long long)planes,
                         (bf16_t*)dx);
    } else {
      const int blocks = (planes + 3) / 4;
      hipLaunchKernelGGL((gn_plane_grads_v<64>), dim3(blocks), dim3(256), 0, stream, (const bf16_t*)dy,
                         (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)b, mean, rstd, C, hw, G, silu,
                         (long long)planes, ws);
      hipLaunchKernelGGL((gn_dx_v<64>), dim3(blocks), dim3(256), 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                         (const bf16_t*)w, (const bf16_t*)b, mean, rstd, ws, C, hw, G, silu, (long long)planes,
                         (bf16_t*)dx);
    }
  } else {
    const int th = hw >= 2048 ? 256 : (hw >= 512 ? 128 : 64);
    hipLaunchKernelGGL(gn_plane_grads, dim3(planes), dim3(th), 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, mean, rstd, C, hw, G, silu, ws);
    hipLaunchKernelGGL(gn_dx, dim3(planes), dim3(th), 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, mean, rstd, ws, C, hw, G, silu, (bf16_t*)dx);
  }
  hipLaunchKernelGGL(gn_param_grads, dim3((C + 255) / 256), dim3(256), 0, stream, ws, N, C, (bf16_t*)dw,
                     (bf16_t*)db);
  return 0;
}
