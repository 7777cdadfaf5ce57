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
//                         (8-channel vector, pixel row); per-channel sums
//                         shifted by the chunk's first pixel, added over the
//                         rows in LDS -> (mean, M2) per (n, chunk, c)
//        2) group_stats : workgroup per (n, g): Chan-merges chunks x cg
//                         partials -> mean, rstd (exact parallel Welford, no
//                         E[x^2] - E[x]^2 cancellation)
//        3) apply       : 16-B vectors, per-channel scale/shift, SiLU
//   bwd  1) chunk_grads : per (n, chunk, c) sums of dz and dz*xhat
//                         (dz = dy * silu'(z) when SiLU is fused)
//        2) group_grads : per (n, g) the gamma-weighted means m1, m2
//        3) chan_grads  : dgamma / dbeta per channel over (n, chunk)
//        4) dx          : rstd * (dz*gamma - m1 - xhat*m2), from per-(n, c)
//                         coefficients written by group_grads
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

// Where the normalised tensor's (n, pixel, channel) lives. SrcPlain: one [N, P, C] tensor.
// SrcCat: the UNet up-block's channel concat [x1 | x2] read in place (no concatenated copy is
// made for the norm), x1 optionally still in the sub-pixel phase layout of the upsampler's 2x2
// conv ([N, H/2+1, W/2+1, 4*C1]: high-res pixel (y, x) is phase (y&1, x&1) of low-res position
// (y>>1 + (y&1), x>>1 + (x&1)) -- models/unet.py phase_weights). C1 % 8 == 0: no 8-channel
// vector straddles the two inputs.
struct SrcPlain {
  const bf16_t* x;
  int C, P;
  __device__ __forceinline__ const bf16_t* ptr(int n, int p, int c) const {
    return x + ((long long)n * P + p) * C + c;
  }
};

struct SrcCat {
  const bf16_t* x1;
  const bf16_t* x2;
  int C1, C2, P, W, phase;
  __device__ __forceinline__ const bf16_t* ptr(int n, int p, int c) const {
    if (c >= C1) return x2 + ((long long)n * P + p) * C2 + (c - C1);
    if (!phase) return x1 + ((long long)n * P + p) * C1 + c;
    const int y = p / W, xx = p - y * W, a = y & 1, b = xx & 1;
    const int hs1 = (P / W) / 2 + 1, ws1 = W / 2 + 1;
    return x1 + (((long long)n * hs1 + (y >> 1) + a) * ws1 + (xx >> 1) + b) * 4 * C1 + (2 * a + b) * C1 + c;
  }
};

// grid (chunks, N, channel slabs), block (slab vectors, R); a slab is <= 256
// 8-channel vectors (C up to 2048 in one slab, the 2560-channel UNet up-block
// concat takes two)
template <typename Src>
__global__ void __launch_bounds__(256) nhwc_chunk_stats(const Src src, int P, int C, float* __restrict__ part) {
  // Shifted sums: every thread accumulates sum(v - K) and sum((v - K)^2) with
  // K = the chunk's first pixel of that channel (one data point, so |mean - K|
  // is O(std) and the final M2 = S2 - S1^2/N does not cancel), as independent
  // FMAs per pixel -- no per-pixel division and no serial Welford chain, so
  // the unrolled loads stay in flight. Rows of the workgroup share K, so
  // their partials merge by plain addition.
  extern __shared__ float sm[];  // [8][R][bw] s1, then [8][R][bw] s2 (lane-contiguous: conflict free)
  const int lv = threadIdx.x, r = threadIdx.y, R = blockDim.y, bw = blockDim.x;
  const int tid = r * bw + lv, nthr = R * bw;
  const int cv = blockIdx.z * bw + lv;
  const bool live = cv * 8 < C;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunks = gridDim.x, CH = chunk_of(P);
  const int p0 = chunk * CH, p1 = min(P, p0 + CH);
  float k[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
  if (live) {
    load8(src.ptr(n, p0, cv * 8), k);
#pragma unroll 4
    for (int p = p0 + r; p < p1; p += R) {
      float v[8];
      load8(src.ptr(n, p, cv * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[j] - k[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    }
  }
  float* a1 = sm;
  float* a2 = sm + 8 * R * bw;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a1[(j * R + r) * bw + lv] = s1[j];
    a2[(j * R + r) * bw + lv] = s2[j];
  }
  __syncthreads();
  const float nn = (float)(p1 - p0), inv = 1.f / nn;
  for (int i = tid; i < 8 * bw; i += nthr) {  // i = j * bw + lane
    const int j = i / bw, l = i % bw, c = (blockIdx.z * bw + l) * 8 + j;
    if (c >= C) continue;
    float t1 = 0.f, t2 = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      t1 += a1[(j * R + rr) * bw + l];
      t2 += a2[(j * R + rr) * bw + l];
    }
    const float kk = bf2f(*src.ptr(n, p0, c));
    float* dst = part + (((long long)n * nchunks + chunk) * C + c) * 2;
    dst[0] = kk + t1 * inv;
    dst[1] = fmaxf(t2 - t1 * t1 * inv, 0.f);
  }
}

// grid N*G, block 256: merge (chunk, channel) partials of one group
__global__ void __launch_bounds__(256) nhwc_group_stats(const float* __restrict__ part, int P, int C, int G,
                                                        int nchunks, float eps, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, const bf16_t* __restrict__ w,
                                                        const bf16_t* __restrict__ b, float* __restrict__ ss,
                                                        const float* __restrict__ add, long long add_ld) {
  __shared__ float red[3 * 256];
  const int ng = blockIdx.x, n = ng / G, g = ng % G, cg = C / G;
  const int items = nchunks * cg, CH = chunk_of(P);
  float cnt = 0.f, mu = 0.f, q = 0.f;
  for (int i = threadIdx.x; i < items; i += blockDim.x) {
    const int ch = i / cg, c = g * cg + i % cg;
    const float cn = (float)(min(P, (ch + 1) * CH) - ch * CH);
    const float* s = part + (((long long)n * nchunks + ch) * C + c) * 2;
    // a per-(n, c) pre-add shifts that channel's mean and leaves its M2 unchanged
    chan_merge(cnt, mu, q, cn, s[0] + (add ? add[(long long)n * add_ld + c] : 0.f), s[1]);
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
    const float t = add ? add[(long long)n * add_ld + c] : 0.f;  // y = (x + t - mu) * sc + b
    ss[((long long)n * 2) * C + c] = sc;
    ss[((long long)n * 2 + 1) * C + c] = (b ? bf2f(b[c]) : 0.f) + (t - mu_g) * sc;
  }
}

// y = x * scale[n, c] + shift[n, c] (+ SiLU); ss = [N][2][C] fp32; raw (optional): the input
// itself, contiguous [N, P, C] (the concat the up-block's 1x1 shortcut conv consumes)
template <typename Src>
__global__ void __launch_bounds__(256) nhwc_apply(const Src src, const float* __restrict__ ss,
                                                  bf16_t* __restrict__ y, bf16_t* __restrict__ raw,
                                                  const float* __restrict__ radd, int P, int C, int silu, int nvec) {
  const int cv8 = C / 8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += gridDim.x * blockDim.x) {
    const int pix = i / cv8;
    const int c0 = (i - pix * cv8) * 8;
    const int n = pix / P;
    float v[8], sc[8], sh[8];
    const bf16_t* xp = src.ptr(n, pix - n * P, c0);
    load8(xp, v);
    if (raw) {
      if (radd) {  // the per-(n, c) pre-add (the upsampler conv's bias) applies to the copy too
        float t[8], a[8];
        load8f(radd + (long long)n * C + c0, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = v[j] + a[j];
        store8(raw + (long long)i * 8, t);
      } else {
        *reinterpret_cast<uint4*>(raw + (long long)i * 8) = *reinterpret_cast<const uint4*>(xp);
      }
    }
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
  const int lv = threadIdx.x, r = threadIdx.y, R = blockDim.y;
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
#pragma unroll 2
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
  // [8][R][bw] layout (lane-contiguous, conflict free); every thread of the
  // workgroup then reduces one channel column over the R rows
  const int bw = blockDim.x, tid = r * bw + lv, nthr = R * bw;
  float* a1 = sm;
  float* a2 = sm + 8 * R * bw;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a1[(j * R + r) * bw + lv] = s1[j];
    a2[(j * R + r) * bw + lv] = s2[j];
  }
  __syncthreads();
  for (int i = tid; i < 8 * bw; i += nthr) {  // i = j * bw + lane
    const int j = i / bw, l = i % bw, c = (blockIdx.z * bw + l) * 8 + j;
    if (c >= C) continue;
    float t1 = 0.f, t2 = 0.f;
    for (int rr = 0; rr < R; ++rr) {
      t1 += a1[(j * R + rr) * bw + l];
      t2 += a2[(j * R + rr) * bw + l];
    }
    float* dst = part + (((long long)n * nchunks + chunk) * C + c) * 2;
    dst[0] = t1;
    dst[1] = t2;
  }
}

// per (n, g): m1 = sum_c gamma_c s1 / cnt, m2 = sum_c gamma_c s2 / cnt
__global__ void __launch_bounds__(256) nhwc_group_grads(const float* __restrict__ part, const bf16_t* __restrict__ w,
                                                        const bf16_t* __restrict__ b, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, int P, int C, int G,
                                                        int nchunks, float* __restrict__ m1, float* __restrict__ m2,
                                                        float* __restrict__ coef) {
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
  const float inv = 1.f / ((float)P * cg);
  const float gm1 = red[0] * inv, gm2 = red[256] * inv;
  if (threadIdx.x == 0) {
    m1[ng] = gm1;
    m2[ng] = gm2;
  }
  // dx = sc * dz + B * x + Cc with z = x * sc + sh (the forward's pre-SiLU value):
  // sc = rstd*gamma, sh = beta - mean*sc, B = -rstd^2*m2, Cc = rstd*(rstd*m2*mean - m1)
  const float mu = mean[ng], rs = rstd[ng];
  for (int j = threadIdx.x; j < cg; j += blockDim.x) {
    const int c = g * cg + j;
    const float sc = rs * bf2f(w[c]);
    float* cf = coef + (long long)n * 4 * C + c;
    cf[0] = sc;
    cf[C] = (b ? bf2f(b[c]) : 0.f) - mu * sc;
    cf[2 * C] = -rs * rs * gm2;
    cf[3 * C] = rs * (rs * gm2 * mu - gm1);
  }
}

// grid ceil(C/16), block 256 = 16 channels x 16 row groups: dgamma / dbeta
// per channel over the (n, chunk) rows. 16 row groups with 4 independent
// accumulators each keep ~64 loads in flight per channel column (the earlier
// 64-channel x 4-group shape left 5 workgroups on the chip for C = 320, each
// thread walking 128+ rows serially: 33 us for 1.3 MB of partials).
__global__ void __launch_bounds__(256) nhwc_chan_grads(const float* __restrict__ part, int rows, int C,
                                                       bf16_t* __restrict__ dw, bf16_t* __restrict__ db) {
  __shared__ float red[2][16][17];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int r = rg;
    for (; r + 48 < rows; r += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float2 s2 = *reinterpret_cast<const float2*>(part + ((long long)(r + 16 * u) * C + c) * 2);
        a[u] += s2.x;
        q[u] += s2.y;
      }
    }
    for (; r < rows; r += 16) {
      const float2 s2 = *reinterpret_cast<const float2*>(part + ((long long)r * C + c) * 2);
      a[0] += s2.x;
      q[0] += s2.y;
    }
  }
  red[0][rg][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  red[1][rg][cl] = (q[0] + q[1]) + (q[2] + q[3]);
  __syncthreads();
  if (rg == 0 && c < C) {
    float ta = 0.f, tq = 0.f;
    for (int k = 0; k < 16; ++k) {
      ta += red[0][k][cl];
      tq += red[1][k][cl];
    }
    dw[c] = f2bf(tq);
    if (db) db[c] = f2bf(ta);
  }
}

// grid (chunks, N, channel slabs), block (slab vectors, R) as chunk_grads:
// each thread keeps its 8 channels' coefficients in registers and streams
// dy / x of its pixels (16-B vectors) -> dx
__global__ void __launch_bounds__(256) nhwc_dx(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                               const float* __restrict__ coef, bf16_t* __restrict__ dx, int P,
                                               int C, int silu) {
  const int lv = threadIdx.x, r = threadIdx.y, R = blockDim.y;
  const int cv = blockIdx.z * blockDim.x + lv;
  if (cv * 8 >= C) return;
  const int n = blockIdx.y, CH = chunk_of(P);
  const int p0 = blockIdx.x * CH, p1 = min(P, p0 + CH);
  float sc[8], sh[8], cb[8], cc[8];
  const float* cf = coef + (long long)n * 4 * C + cv * 8;
  load8f(cf, sc);
  load8f(cf + C, sh);
  load8f(cf + 2 * C, cb);
  load8f(cf + 3 * C, cc);
  const long long off = ((long long)n * P) * C + cv * 8;
#pragma unroll 2
  for (int p = p0 + r; p < p1; p += R) {
    float v[8], g[8];
    load8(x + off + (long long)p * C, v);
    load8(dy + off + (long long)p * C, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dz = silu ? g[j] * silu_d(fmaf(v[j], sc[j], sh[j])) : g[j];
      v[j] = fmaf(sc[j], dz, fmaf(cb[j], v[j], cc[j]));
    }
    store8(dx + off + (long long)p * C, v);
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
  // fwd: partials + [N][2][C] scale/shift; bwd: + [N][4][C] dx coefs (+4: 16-B alignment slack)
  return 2 * N * nchunks * C + 4 * N * C + 4;
}

// x, y: [N, P, C] bf16; mean/rstd: [N*G] fp32 out; ws: kca_groupnorm_nhwc_ws floats;
// add: optional fp32 [N, C] (row stride add_ld >= C) added to x before the norm (the ResNet
// block's time embedding, folded into the statistics and the apply pass's shift: no extra pass
// over x and no materialised x + temb; add_ld lets every block read its slice of the UNet's one
// batched time-projection GEMM in place)
KCA_API int kca_groupnorm_nhwc_fwd_add(const void* x, const void* w, const void* b, const float* add,
                                       long long add_ld, void* y, float* mean, float* rstd, float* ws, int N, int P,
                                       int C, int G, float eps, int silu, hipStream_t stream) {
  dim3 block;
  int slabs;
  if (!geometry(C, G, block, slabs) || N <= 0 || P <= 0 || (add && add_ld < C)) return 1;
  if ((long long)N * P * C / 8 >= (1LL << 31)) return 2;
  const int nchunks = (P + chunk_of(P) - 1) / chunk_of(P);
  const size_t smem = 2 * block.y * block.x * 8 * sizeof(float);
  const SrcPlain src{(const bf16_t*)x, C, P};
  hipLaunchKernelGGL(nhwc_chunk_stats<SrcPlain>, dim3(nchunks, N, slabs), block, smem, stream, src, P, C, ws);
  float* ss = ws + 2LL * N * nchunks * C;
  hipLaunchKernelGGL(nhwc_group_stats, dim3(N * G), dim3(256), 0, stream, ws, P, C, G, nchunks, eps, mean, rstd,
                     (const bf16_t*)w, (const bf16_t*)b, ss, add, add_ld);
  const int nvec = (int)((long long)N * P * C / 8);
  hipLaunchKernelGGL(nhwc_apply<SrcPlain>, dim3(kca_grid(nvec, 256, 8192)), dim3(256), 0, stream, src, ss,
                     (bf16_t*)y, (bf16_t*)nullptr, (const float*)nullptr, P, C, silu, nvec);
  return 0;
}

// Inference GroupNorm(+SiLU) of the channel concat [x1 | x2] ([N, P, C1] and [N, P, C2], or x1 in
// the upsampler's phase layout when phase_w > 0 = the high-res width W, P = H * W) without
// materialising the concat for the norm: y = GN([x1 | x2]) ([N, P, C1 + C2]) and, when raw is
// given, the concat itself (the 1x1 shortcut's input) written by the same apply pass. add
// (optional, fp32 [N, C1 + C2]): added to the input before both (the upsampler conv's bias).
KCA_API int kca_groupnorm_nhwc_cat_fwd(const void* x1, const void* x2, const void* w, const void* b,
                                       const float* add, void* y, void* raw, float* mean, float* rstd, float* ws,
                                       int N, int P, int C1, int C2, int phase_w, int G, float eps, int silu,
                                       hipStream_t stream) {
  const int C = C1 + C2;
  dim3 block;
  int slabs;
  if (!x1 || !x2 || C1 % 8 || C2 % 8 || !geometry(C, G, block, slabs) || N <= 0 || P <= 0) return 1;
  if (phase_w > 0 && (phase_w % 2 || P % phase_w || (P / phase_w) % 2)) return 1;
  if ((long long)N * P * C / 8 >= (1LL << 31)) return 2;
  const int nchunks = (P + chunk_of(P) - 1) / chunk_of(P);
  const size_t smem = 2 * block.y * block.x * 8 * sizeof(float);
  const SrcCat src{(const bf16_t*)x1, (const bf16_t*)x2, C1, C2, P, phase_w > 0 ? phase_w : 1, phase_w > 0};
  hipLaunchKernelGGL(nhwc_chunk_stats<SrcCat>, dim3(nchunks, N, slabs), block, smem, stream, src, P, C, ws);
  float* ss = ws + 2LL * N * nchunks * C;
  hipLaunchKernelGGL(nhwc_group_stats, dim3(N * G), dim3(256), 0, stream, ws, P, C, G, nchunks, eps, mean, rstd,
                     (const bf16_t*)w, (const bf16_t*)b, ss, add, (long long)C);
  const int nvec = (int)((long long)N * P * C / 8);
  hipLaunchKernelGGL(nhwc_apply<SrcCat>, dim3(kca_grid(nvec, 256, 8192)), dim3(256), 0, stream, src, ss,
                     (bf16_t*)y, (bf16_t*)raw, add, P, C, silu, nvec);
  return 0;
}

KCA_API int kca_groupnorm_nhwc_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                                   float* ws, int N, int P, int C, int G, float eps, int silu, hipStream_t stream) {
  return kca_groupnorm_nhwc_fwd_add(x, w, b, nullptr, 0, y, mean, rstd, ws, N, P, C, G, eps, silu, stream);
}

// ws: kca_groupnorm_nhwc_ws floats + 2*N*G floats (partials, m1, m2, dx coefficients)
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
  float* coef = m1 + ((2 * N * G + 3) & ~3);  // [N][4][C], 16-B aligned for the float4 loads
  const size_t smem = 2 * block.y * block.x * 8 * sizeof(float);
  hipLaunchKernelGGL(nhwc_chunk_grads, dim3(nchunks, N, slabs), block, smem, stream, (const bf16_t*)dy, (const bf16_t*)x,
                     (const bf16_t*)w, (const bf16_t*)b, mean, rstd, P, C, G, silu, part);
  hipLaunchKernelGGL(nhwc_group_grads, dim3(N * G), dim3(256), 0, stream, part, (const bf16_t*)w, (const bf16_t*)b,
                     mean, rstd, P, C, G, nchunks, m1, m2, coef);
  hipLaunchKernelGGL(nhwc_chan_grads, dim3((C + 15) / 16), dim3(256), 0, stream, part, N * nchunks, C,
                     (bf16_t*)dw, (bf16_t*)db);
  hipLaunchKernelGGL(nhwc_dx, dim3(nchunks, N, slabs), block, 0, stream, (const bf16_t*)dy, (const bf16_t*)x,
                     coef, (bf16_t*)dx, P, C, silu);
  return 0;
}
