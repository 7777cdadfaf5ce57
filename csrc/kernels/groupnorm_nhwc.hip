// GroupNorm (+ fused SiLU) forward / backward on channels-last (NHWC)
// activations -- the layout the SD UNet / VAE run in end to end, so MIOpen's
// NHWC convolutions need no NCHW<->NHWC transposes around every call and the
// attention blocks' [B, HW, C] token view is free (K14).
//
// x is [N, P, C] (P = H*W pixels, C contiguous), G groups of cg = C/G
// consecutive channels; C % 8 == 0 (cg itself may be 10, 20, 40 ...: a 16-B
// vector of 8 channels can straddle two groups, so the group index is taken
// per channel).
//
//   fwd  1) chunk_stats : workgroup = (n, pixel chunk), thread tile =
//                         (8-channel vector, pixel row); per-channel Welford
//                         over the thread's pixels, merged over the rows in
//                         LDS -> (mean, M2) per (n, chunk, c)
//        2) group_stats : workgroup per (n, g): Chan-merges chunks x cg
//                         partials -> mean, rstd (exact parallel Welford, no
//                         E[x^2] - E[x]^2 cancellation)
//        3) apply       : 16-B vectors, per-channel scale/shift, SiLU
//   bwd  1) chunk_grads : per (n, chunk, c) sums of dz and dz*xhat
//                         (dz = dy * silu'(z) when SiLU is fused)
//        2) group_grads : per (n, g) the gamma-weighted means m1, m2
//        3) chan_grads  : dgamma / dbeta per channel over (n, chunk)
//        4) dx          : rstd * (dz*gamma - m1 - xhat*m2)
// No atomics anywhere (deterministic).
#include "common.h"

namespace {

// pixels per stats workgroup: >= 64 and at most 64 chunks per image, so the
// partial buffers and the per-channel reductions over them stay small
__host__ __device__ inline int chunk_of(int P) { return max(64, (P + 63) / 64); }

__device__ __forceinline__ float silu_of(float z) { return z / (1.f + __expf(-z)); }
__device__ __forceinline__ float silu_d(float z) {
  const float s = 1.f / (1.f + __expf(-z));
  return s * (1.f + z * (1.f - s));
}

__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float n2, float mu2, float q2) {
  const float nt = n + n2;
  if (nt > 0.f) {
    const float d = mu2 - mean;
    mean += d * n2 / nt;
    m2 += q2 + d * d * n * n2 / nt;
    n = nt;
  }
}

// grid (chunks, N, channel slabs), block (slab vectors, R); a slab is <= 256
// 8-channel vectors (C up to 2048 in one slab, the 2560-channel UNet up-block
// concat takes two)
__global__ void __launch_bounds__(256) nhwc_chunk_stats(const bf16_t* __restrict__ x, int P, int C,
                                                        float* __restrict__ part) {
  extern __shared__ float sm[];  // [R][W] mean, [R][W] m2, [R] count; W = slab width in channels
  const int lv = threadIdx.x, r = threadIdx.y, R = blockDim.y, W = blockDim.x * 8;
  const int cv = blockIdx.z * blockDim.x + lv;
  const bool live = cv * 8 < C;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunks = gridDim.x, CH = chunk_of(P);
  const int p0 = chunk * CH, p1 = min(P, p0 + CH);
  float mean[8], m2[8], cnt = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) mean[j] = m2[j] = 0.f;
  const bf16_t* base = x + ((long long)n * P) * C + cv * 8;
#pragma unroll 4
  for (int p = p0 + r; live && p < p1; p += R) {
    float v[8];
    load8(base + (long long)p * C, v);
    cnt += 1.f;
    const float inv = 1.f / cnt;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[j] - mean[j];
      mean[j] += d * inv;
      m2[j] += d * (v[j] - mean[j]);
    }
  }
  float* smean = sm;
  float* sm2 = sm + R * W;
  float* scnt = sm + 2 * R * W;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    smean[r * W + lv * 8 + j] = mean[j];
    sm2[r * W + lv * 8 + j] = m2[j];
  }
  if (lv == 0) scnt[r] = (float)((p1 - p0 - r + R - 1) / R);
  __syncthreads();
  if (r == 0 && live) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float nn = scnt[0], mu = smean[lv * 8 + j], q = sm2[lv * 8 + j];
      for (int rr = 1; rr < R; ++rr) chan_merge(nn, mu, q, scnt[rr], smean[rr * W + lv * 8 + j], sm2[rr * W + lv * 8 + j]);
      float* dst = part + (((long long)n * nchunks + chunk) * C + cv * 8 + j) * 2;
      dst[0] = mu;
      dst[1] = q;
    }
  }
}

// grid N*G, block 256: merge (chunk, channel) partials of one group
__global__ void __launch_bounds__(256) nhwc_group_stats(const float* __restrict__ part, int P, int C, int G,
                                                        int nchunks, float eps, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, const bf16_t* __restrict__ w,
                                                        const bf16_t* __restrict__ b, float* __restrict__ ss,
                                                        const float* __restrict__ add) {
  __shared__ float red[3 * 256];
  const int ng = blockIdx.x, n = ng / G, g = ng % G, cg = C / G;
  const int items = nchunks * cg, CH = chunk_of(P);
  float cnt = 0.f, mu = 0.f, q = 0.f;
  for (int i = threadIdx.x; i < items; i += blockDim.x) {
    const int ch = i / cg, c = g * cg + i % cg;
    const float cn = (float)(min(P, (ch + 1) * CH) - ch * CH);
    const float* s = part + (((long long)n * nchunks + ch) * C + c) * 2;
    // a per-(n, c) pre-add shifts that channel's mean and leaves its M2 unchanged
    chan_merge(cnt, mu, q, cn, s[0] + (add ? add[(long long)n * C + c] : 0.f), s[1]);
  }
  red[threadIdx.x] = cnt;
  red[256 + threadIdx.x] = mu;
  red[512 + threadIdx.x] = q;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      float a = red[threadIdx.x], b = red[256 + threadIdx.x], c2 = red[512 + threadIdx.x];
      chan_merge(a, b, c2, red[threadIdx.x + s], red[256 + threadIdx.x + s], red[512 + threadIdx.x + s]);
      red[threadIdx.x] = a;
      red[256 + threadIdx.x] = b;
      red[512 + threadIdx.x] = c2;
    }
    __syncthreads();
  }
  const float mu_g = red[256], rs_g = rsqrtf(red[512] / red[0] + eps);
  if (threadIdx.x == 0) {
    mean_out[ng] = mu_g;
    rstd_out[ng] = rs_g;
  }
  // per-(n, c) affine of the apply pass: y = x * scale + shift
  for (int j = threadIdx.x; j < cg; j += blockDim.x) {
    const int c = g * cg + j;
    const float sc = rs_g * bf2f(w[c]);
    const float t = add ? add[(long long)n * C + c] : 0.f;  // y = (x + t - mu) * sc + b
    ss[((long long)n * 2) * C + c] = sc;
    ss[((long long)n * 2 + 1) * C + c] = (b ? bf2f(b[c]) : 0.f) + (t - mu_g) * sc;
  }
}

// y = x * scale[n, c] + shift[n, c] (+ SiLU); ss = [N][2][C] fp32
__global__ void __launch_bounds__(256) nhwc_apply(const bf16_t* __restrict__ x, const float* __restrict__ ss,
                                                  bf16_t* __restrict__ y, int P, int C, int silu, int nvec) {
  const int cv8 = C / 8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += gridDim.x * blockDim.x) {
    const int pix = i / cv8;
    const int c0 = (i - pix * cv8) * 8;
    const int n = pix / P;
    float v[8], sc[8], sh[8];
    load8(x + (long long)i * 8, v);
    load8f(ss + (long long)n * 2 * C + c0, sc);
    load8f(ss + ((long long)n * 2 + 1) * C + c0, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = v[j] * sc[j] + sh[j];
      v[j] = silu ? silu_of(z) : z;
    }
    store8(y + (long long)i * 8, v);
  }
}

// backward partials: s1 = sum dz, s2 = sum dz*xhat per (n, chunk, c); grid (chunks, N), block (C/8, R)
__global__ void __launch_bounds__(256) nhwc_chunk_grads(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                        const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, int P, int C, int G, int silu,
                                                        float* __restrict__ part) {
  extern __shared__ float sm[];  // [R][W] s1, [R][W] s2
  const int lv = threadIdx.x, r = threadIdx.y, R = blockDim.y, W = blockDim.x * 8;
  const int cv = blockIdx.z * blockDim.x + lv;
  const bool live = cv * 8 < C;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunks = gridDim.x, CH = chunk_of(P);
  const int p0 = chunk * CH, p1 = min(P, p0 + CH);
  const int cg = C / G;
  float mu[8], rs[8], gw[8], gb[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = live ? cv * 8 + j : 0, ng = n * G + c / cg;
    mu[j] = mean[ng];
    rs[j] = rstd[ng];
    gw[j] = bf2f(w[c]);
    gb[j] = b ? bf2f(b[c]) : 0.f;
    s1[j] = s2[j] = 0.f;
  }
  const long long off = ((long long)n * P) * C + cv * 8;
  for (int p = p0 + r; live && p < p1; p += R) {
    float v[8], g[8];
    load8(x + off + (long long)p * C, v);
    load8(dy + off + (long long)p * C, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (v[j] - mu[j]) * rs[j];
      const float dz = silu ? g[j] * silu_d(xh * gw[j] + gb[j]) : g[j];
      s1[j] += dz;
      s2[j] += dz * xh;
    }
  }
  float* a1 = sm;
  float* a2 = sm + R * W;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a1[r * W + lv * 8 + j] = s1[j];
    a2[r * W + lv * 8 + j] = s2[j];
  }
  __syncthreads();
  if (r == 0 && live) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t1 = 0.f, t2 = 0.f;
      for (int rr = 0; rr < R; ++rr) {
        t1 += a1[rr * W + lv * 8 + j];
        t2 += a2[rr * W + lv * 8 + j];
      }
      float* dst = part + (((long long)n * nchunks + chunk) * C + cv * 8 + j) * 2;
      dst[0] = t1;
      dst[1] = t2;
    }
  }
}

// per (n, g): m1 = sum_c gamma_c s1 / cnt, m2 = sum_c gamma_c s2 / cnt
__global__ void __launch_bounds__(256) nhwc_group_grads(const float* __restrict__ part, const bf16_t* __restrict__ w,
                                                        int P, int C, int G, int nchunks, float* __restrict__ m1,
                                                        float* __restrict__ m2) {
  __shared__ float red[2 * 256];
  const int ng = blockIdx.x, n = ng / G, g = ng % G, cg = C / G;
  float a = 0.f, b2 = 0.f;
  for (int i = threadIdx.x; i < nchunks * cg; i += blockDim.x) {
    const int ch = i / cg, c = g * cg + i % cg;
    const float* s = part + (((long long)n * nchunks + ch) * C + c) * 2;
    const float gw = bf2f(w[c]);
    a += gw * s[0];
    b2 += gw * s[1];
  }
  red[threadIdx.x] = a;
  red[256 + threadIdx.x] = b2;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[threadIdx.x] += red[threadIdx.x + s];
      red[256 + threadIdx.x] += red[256 + threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float inv = 1.f / ((float)P * cg);
    m1[ng] = red[0] * inv;
    m2[ng] = red[256] * inv;
  }
}

// dgamma[c] = sum s2, dbeta[c] = sum s1 over the (n, chunk) rows; workgroup =
// 64 channels x 4 row groups, LDS combine
__global__ void __launch_bounds__(256) nhwc_chan_grads(const float* __restrict__ part, int rows, int C,
                                                       bf16_t* __restrict__ dw, bf16_t* __restrict__ db) {
  __shared__ float red[2][4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a = 0.f, b2 = 0.f;
  if (c < C) {
    for (int r = rg; r < rows; r += 4) {
      const float* s = part + ((long long)r * C + c) * 2;
      a += s[0];
      b2 += s[1];
    }
  }
  red[0][rg][cl] = a;
  red[1][rg][cl] = b2;
  __syncthreads();
  if (rg == 0 && c < C) {
    for (int k = 1; k < 4; ++k) {
      a += red[0][k][cl];
      b2 += red[1][k][cl];
    }
    dw[c] = f2bf(b2);
    if (db) db[c] = f2bf(a);
  }
}

__global__ void __launch_bounds__(256) nhwc_dx(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                               const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                               const float* __restrict__ mean, const float* __restrict__ rstd,
                                               const float* __restrict__ m1, const float* __restrict__ m2,
                                               bf16_t* __restrict__ dx, int P, int C, int G, int silu, int nvec) {
  const int cg = C / G, cv8 = C / 8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += gridDim.x * blockDim.x) {
    const int pix = i / cv8;
    const int c0 = (i - pix * cv8) * 8;
    const int n = pix / P;
    float v[8], g[8];
    load8(x + (long long)i * 8, v);
    load8(dy + (long long)i * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j, ng = n * G + c / cg;
      const float gw = bf2f(w[c]);
      const float xh = (v[j] - mean[ng]) * rstd[ng];
      const float dz = silu ? g[j] * silu_d(xh * gw + (b ? bf2f(b[c]) : 0.f)) : g[j];
      v[j] = rstd[ng] * (dz * gw - m1[ng] - xh * m2[ng]);
    }
    store8(dx + (long long)i * 8, v);
  }
}

bool geometry(int C, int G, dim3& block, int& slabs) {
  if (C % 8 || G <= 0 || C % G) return false;
  const int cv = C / 8;
  slabs = (cv + 255) / 256;
  const int w = (cv + slabs - 1) / slabs;
  int R = 256 / w;
  if (R > 64) R = 64;
  block = dim3(w, R);
  return true;
}

}  // namespace

KCA_API int kca_groupnorm_nhwc_ws(int N, int P, int C) {  // fp32 workspace floats needed
  const int nchunks = (P + chunk_of(P) - 1) / chunk_of(P);
  return 2 * N * nchunks * C + 2 * N * C;
}

// x, y: [N, P, C] bf16; mean/rstd: [N*G] fp32 out; ws: kca_groupnorm_nhwc_ws floats;
// add: optional fp32 [N, C] added to x before the norm (the ResNet block's time
// embedding, folded into the statistics and the apply pass's shift: no extra
// pass over x and no materialised x + temb)
KCA_API int kca_groupnorm_nhwc_fwd_add(const void* x, const void* w, const void* b, const float* add, void* y,
                                       float* mean, float* rstd, float* ws, int N, int P, int C, int G, float eps,
                                       int silu, hipStream_t stream) {
  dim3 block;
  int slabs;
  if (!geometry(C, G, block, slabs) || N <= 0 || P <= 0) return 1;
  if ((long long)N * P * C / 8 >= (1LL << 31)) return 2;
  const int nchunks = (P + chunk_of(P) - 1) / chunk_of(P);
  const size_t smem = (2 * block.y * block.x * 8 + block.y) * sizeof(float);
  hipLaunchKernelGGL(nhwc_chunk_stats, dim3(nchunks, N, slabs), block, smem, stream, (const bf16_t*)x, P, C, ws);
  float* ss = ws + 2LL * N * nchunks * C;
  hipLaunchKernelGGL(nhwc_group_stats, dim3(N * G), dim3(256), 0, stream, ws, P, C, G, nchunks, eps, mean, rstd,
                     (const bf16_t*)w, (const bf16_t*)b, ss, add);
  const int nvec = (int)((long long)N * P * C / 8);
  hipLaunchKernelGGL(nhwc_apply, dim3(kca_grid(nvec, 256, 8192)), dim3(256), 0, stream, (const bf16_t*)x, ss,
                     (bf16_t*)y, P, C, silu, nvec);
  return 0;
}

KCA_API int kca_groupnorm_nhwc_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                                   float* ws, int N, int P, int C, int G, float eps, int silu, hipStream_t stream) {
  return kca_groupnorm_nhwc_fwd_add(x, w, b, nullptr, y, mean, rstd, ws, N, P, C, G, eps, silu, stream);
}

// ws: kca_groupnorm_nhwc_ws floats + 2*N*G floats
KCA_API int kca_groupnorm_nhwc_bwd(const void* dy, const void* x, const void* w, const void* b, const float* mean,
                                   const float* rstd, void* dx, void* dw, void* db, float* ws, int N, int P, int C,
                                   int G, int silu, hipStream_t stream) {
  dim3 block;
  int slabs;
  if (!geometry(C, G, block, slabs) || N <= 0 || P <= 0) return 1;
  if ((long long)N * P * C / 8 >= (1LL << 31)) return 2;
  const int nchunks = (P + chunk_of(P) - 1) / chunk_of(P);
  float* part = ws;
  float* m1 = ws + 2LL * N * nchunks * C;
  float* m2 = m1 + N * G;
  const size_t smem = 2 * block.y * block.x * 8 * sizeof(float);
  hipLaunchKernelGGL(nhwc_chunk_grads, dim3(nchunks, N, slabs), block, smem, stream, (const bf16_t*)dy, (const bf16_t*)x,
                     (const bf16_t*)w, (const bf16_t*)b, mean, rstd, P, C, G, silu, part);
  hipLaunchKernelGGL(nhwc_group_grads, dim3(N * G), dim3(256), 0, stream, part, (const bf16_t*)w, P, C, G, nchunks,
                     m1, m2);
  hipLaunchKernelGGL(nhwc_chan_grads, dim3((C + 63) / 64), dim3(256), 0, stream, part, N * nchunks, C,
                     (bf16_t*)dw, (bf16_t*)db);
  const int nvec = (int)((long long)N * P * C / 8);
  hipLaunchKernelGGL(nhwc_dx, dim3(kca_grid(nvec, 256, 8192)), dim3(256), 0, stream, (const bf16_t*)dy,
                     (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)b, mean, rstd, m1, m2, (bf16_t*)dx,
                     P, C, G, silu, nvec);
  return 0;
}
