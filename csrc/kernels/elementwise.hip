// Memory-bound elementwise kernels (K3 RoPE, K5 GELU, grad accumulation,
// casts). All bf16 traffic is 16 B per lane; grids are grid-stride, capped at
// ~2048 workgroups of 256 threads (cdna_hip_programming.md Guideline 11/13).
#include "common.h"

// ---------------------------------------------------------------- GELU
// y = gelu(u), tanh approximation ("gelu_new"/"gelu_fast": GPT-J, GPT-2,
// NeoX-20B, BLOOM) or exact erf ("gelu": Pythia). The bias add is fused into
// the producing hipBLASLt GEMM epilogue (addmm), so the activation kernel only
// needs the pre-activation.
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

template <bool TANH, int DT = 0>  // DT: 0 bf16, 1 fp16 (common.h)
__global__ void gelu_fwd_kernel(const bf16_t* __restrict__ u,
                                bf16_t* __restrict__ y, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    load8_t<DT>(u + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = TANH ? gelu_tanh(v[j]) : gelu_erf(v[j]);
    store8_t<DT>(y + i * 8, v);
  }
}

template <bool TANH>
__global__ void gelu_bwd_kernel(const bf16_t* __restrict__ dy,
                                const bf16_t* __restrict__ u,
                                bf16_t* __restrict__ du, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float g[8], v[8];
    load8(dy + i * 8, g);
    load8(u + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = g[j] * (TANH ? gelu_tanh_grad(v[j]) : gelu_erf_grad(v[j]));
    store8(du + i * 8, v);
  }
}

KCA_API int kca_gelu_fwd(const void* u, void* y, long long n, int approx_tanh,
                         hipStream_t stream) {
  if (n % 8) return 1;
  const long long n8 = n / 8;
  if (approx_tanh)
    hipLaunchKernelGGL(gelu_fwd_kernel<true>, dim3(kca_grid(n8, 256)), dim3(256), 0,
                       stream, (const bf16_t*)u, (bf16_t*)y, n8);
  else
    hipLaunchKernelGGL(gelu_fwd_kernel<false>, dim3(kca_grid(n8, 256)), dim3(256), 0,
                       stream, (const bf16_t*)u, (bf16_t*)y, n8);
  return 0;
}

// fp16 (the FT / DS-Inference serving precision: decode fc_in after hipBLASLt at batch > the fused layer's)
KCA_API int kca_gelu_fwd_f16(const void* u, void* y, long long n, int approx_tanh, hipStream_t stream) {
  if (n % 8) return 1;
  const long long n8 = n / 8;
  if (approx_tanh)
    hipLaunchKernelGGL((gelu_fwd_kernel<true, 1>), dim3(kca_grid(n8, 256)), dim3(256), 0, stream, (const bf16_t*)u,
                       (bf16_t*)y, n8);
  else
    hipLaunchKernelGGL((gelu_fwd_kernel<false, 1>), dim3(kca_grid(n8, 256)), dim3(256), 0, stream, (const bf16_t*)u,
                       (bf16_t*)y, n8);
  return 0;
}

KCA_API int kca_gelu_bwd(const void* dy, const void* u, void* du, long long n,
                         int approx_tanh, hipStream_t stream) {
  if (n % 8) return 1;
  const long long n8 = n / 8;
  if (approx_tanh)
    hipLaunchKernelGGL(gelu_bwd_kernel<true>, dim3(kca_grid(n8, 256)), dim3(256), 0,
                       stream, (const bf16_t*)dy, (const bf16_t*)u, (bf16_t*)du, n8);
  else
    hipLaunchKernelGGL(gelu_bwd_kernel<false>, dim3(kca_grid(n8, 256)), dim3(256), 0,
                       stream, (const bf16_t*)dy, (const bf16_t*)u, (bf16_t*)du, n8);
  return 0;
}

// CLIP's quick GELU, x * sigmoid(1.702 x) (one pass instead of torch's mul + sigmoid + mul)
__global__ void quick_gelu_fwd_kernel(const bf16_t* __restrict__ u, bf16_t* __restrict__ y, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    load8(u + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] / (1.f + __expf(-1.702f * v[j]));
    store8(y + i * 8, v);
  }
}

__global__ void quick_gelu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ u,
                                      bf16_t* __restrict__ du, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float g[8], v[8];
    load8(dy + i * 8, g);
    load8(u + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-1.702f * v[j]));
      v[j] = g[j] * (sg + 1.702f * v[j] * sg * (1.f - sg));
    }
    store8(du + i * 8, v);
  }
}

KCA_API int kca_quick_gelu_fwd(const void* u, void* y, long long n, hipStream_t stream) {
  if (n % 8) return 1;
  hipLaunchKernelGGL(quick_gelu_fwd_kernel, dim3(kca_grid(n / 8, 256)), dim3(256), 0, stream, (const bf16_t*)u,
                     (bf16_t*)y, n / 8);
  return 0;
}

KCA_API int kca_quick_gelu_bwd(const void* dy, const void* u, void* du, long long n, hipStream_t stream) {
  if (n % 8) return 1;
  hipLaunchKernelGGL(quick_gelu_bwd_kernel, dim3(kca_grid(n / 8, 256)), dim3(256), 0, stream, (const bf16_t*)dy,
                     (const bf16_t*)u, (bf16_t*)du, n / 8);
  return 0;
}

// ---------------------------------------------------------------- RoPE
// In-place rotary embedding on the first `rot` dims of every head of a
// [tokens, heads, head_dim] view with arbitrary token/head strides (so it runs
// directly on the fused QKV GEMM output). cos/sin tables are precomputed on the
// host, [max_pos, rot/2] fp32 (Appendix B "trig-heavy ops": no device trig).
//   interleaved=1 : GPT-J "rotate_every_two", pairs (2i, 2i+1)
//   interleaved=0 : GPT-NeoX/Pythia "rotate_half", pairs (i, i + rot/2)
// sign=+1 forward rotation, sign=-1 the transpose (used by the backward).
// Each thread rotates 4 pairs (8 elements).
__global__ void rope_kernel(bf16_t* __restrict__ q, bf16_t* __restrict__ k,
                            int nh_q, int nh_k, long long tokens, int seq,
                            long long tok_stride_q, long long head_stride_q,
                            long long tok_stride_k, long long head_stride_k,
                            int rot, int interleaved,
                            const float* __restrict__ cos_t,
                            const float* __restrict__ sin_t,
                            const int* __restrict__ pos_ids, float sign) {
  const int half = rot >> 1;
  const int groups = half >> 2;  // 4 pairs per thread
  const int nh = nh_q + nh_k;
  const long long total = tokens * nh * groups;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
       idx < total; idx += (long long)gridDim.x * blockDim.x) {
    const int g = idx % groups;
    const long long th = idx / groups;
    const int hh = th % nh;
    const long long t = th / nh;
    const int pos = pos_ids ? pos_ids[t] : (int)(t % seq);
    bf16_t* base = hh < nh_q ? q + t * tok_stride_q + hh * head_stride_q
                             : k + t * tok_stride_k + (hh - nh_q) * head_stride_k;
    const float* ct = cos_t + (size_t)pos * half + g * 4;
    const float* st = sin_t + (size_t)pos * half + g * 4;
    float c[4], s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { c[j] = ct[j]; s[j] = sign * st[j]; }
    if (interleaved) {
      float x[8];
      load8(base + g * 8, x);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = x[2 * j], b = x[2 * j + 1];
        x[2 * j] = a * c[j] - b * s[j];
        x[2 * j + 1] = b * c[j] + a * s[j];
      }
      store8(base + g * 8, x);
    } else {
      U16x4 ua = *reinterpret_cast<const U16x4*>(base + g * 4);
      U16x4 ub = *reinterpret_cast<const U16x4*>(base + half + g * 4);
      U16x4 oa, ob;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = bf2f(ua.v[j]), b = bf2f(ub.v[j]);
        oa.v[j] = f2bf(a * c[j] - b * s[j]);
        ob.v[j] = f2bf(b * c[j] + a * s[j]);
      }
      *reinterpret_cast<U16x4*>(base + g * 4) = oa;
      *reinterpret_cast<U16x4*>(base + half + g * 4) = ob;
    }
  }
}

// One pair per thread: rot/2 not a multiple of 4 (Pythia-2.8B: rot = 20).
__global__ void rope_scalar_kernel(bf16_t* __restrict__ q,
                                   bf16_t* __restrict__ k, int nh_q, int nh_k,
                                   long long tokens, int seq,
                                   long long tok_stride_q,
                                   long long head_stride_q,
                                   long long tok_stride_k,
                                   long long head_stride_k, int rot,
                                   int interleaved,
                                   const float* __restrict__ cos_t,
                                   const float* __restrict__ sin_t,
                                   const int* __restrict__ pos_ids,
                                   float sign) {
  const int half = rot >> 1;
  const int nh = nh_q + nh_k;
  const long long total = tokens * nh * half;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x;
       idx < total; idx += (long long)gridDim.x * blockDim.x) {
    const int i = idx % half;
    const long long th = idx / half;
    const int hh = th % nh;
    const long long t = th / nh;
    const int pos = pos_ids ? pos_ids[t] : (int)(t % seq);
    bf16_t* base = hh < nh_q ? q + t * tok_stride_q + hh * head_stride_q
                             : k + t * tok_stride_k + (hh - nh_q) * head_stride_k;
    const float c = cos_t[(size_t)pos * half + i];
    const float s = sign * sin_t[(size_t)pos * half + i];
    const int ia = interleaved ? 2 * i : i;
    const int ib = interleaved ? 2 * i + 1 : i + half;
    const float a = bf2f(base[ia]), b = bf2f(base[ib]);
    base[ia] = f2bf(a * c - b * s);
    base[ib] = f2bf(b * c + a * s);
  }
}

KCA_API int kca_rope(void* q, void* k, int nh_q, int nh_k, long long tokens,
                     int seq, long long tok_stride_q, long long head_stride_q,
                     long long tok_stride_k, long long head_stride_k, int rot,
                     int interleaved, const float* cos_t, const float* sin_t,
                     const int* pos_ids, float sign, hipStream_t stream) {
  if (rot % 2) return 1;
  if (rot % 8) {
    const long long total = tokens * (nh_q + nh_k) * (rot / 2);
    hipLaunchKernelGGL(rope_scalar_kernel, dim3(kca_grid(total, 256)),
                       dim3(256), 0, stream, (bf16_t*)q, (bf16_t*)k, nh_q,
                       nh_k, tokens, seq, tok_stride_q, head_stride_q,
                       tok_stride_k, head_stride_k, rot, interleaved, cos_t,
                       sin_t, pos_ids, sign);
    return 0;
  }
  const long long total = tokens * (nh_q + nh_k) * (rot / 8);
  hipLaunchKernelGGL(rope_kernel, dim3(kca_grid(total, 256)), dim3(256), 0,
                     stream, (bf16_t*)q, (bf16_t*)k, nh_q, nh_k, tokens, seq,
                     tok_stride_q, head_stride_q, tok_stride_k, head_stride_k,
                     rot, interleaved, cos_t, sin_t, pos_ids, sign);
  return 0;
}

// ---------------------------------------------------------------- grads
// main_grad (fp32) += grad (bf16) * scale   -- fp32 gradient accumulation across
// micro-batches (DeepSpeed/Megatron keep grads in fp32 for bf16 training).
__global__ void accum_grad_kernel(float* __restrict__ acc,
                                  const bf16_t* __restrict__ g, float scale,
                                  int overwrite, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float v[8], a[8];
    load8(g + i * 8, v);
    if (overwrite) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = v[j] * scale;
    } else {
      load8f(acc + i * 8, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += v[j] * scale;
    }
    store8f(acc + i * 8, a);
  }
}

__global__ void accum_grad_tail_kernel(float* acc, const bf16_t* g, float scale,
                                       int overwrite, long long start,
                                       long long n) {
  long long i = start + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i < n) acc[i] = (overwrite ? 0.f : acc[i]) + bf2f(g[i]) * scale;
}

KCA_API int kca_accum_grad(float* acc, const void* g, float scale,
                           int overwrite, long long n, hipStream_t stream) {
  const long long n8 = n / 8;
  if (n8)
    hipLaunchKernelGGL(accum_grad_kernel, dim3(kca_grid(n8, 256)), dim3(256),
                       0, stream, acc, (const bf16_t*)g, scale, overwrite, n8);
  if (n % 8)
    hipLaunchKernelGGL(accum_grad_tail_kernel, dim3(1), dim3(64), 0, stream,
                       acc, (const bf16_t*)g, scale, overwrite, n8 * 8, n);
  return 0;
}

// The first two micro-batches' gradients of one parameter in one pass: acc = g1 * scale + g2 * scale
// (the same rounding as kca_accum_grad overwrite-then-accumulate, the fp32 accumulator written once
// instead of written, re-read and re-written: 8 instead of 14 bytes per element over the pair)
__global__ void accum_grad_pair_kernel(float* __restrict__ acc, const bf16_t* __restrict__ g1,
                                       const bf16_t* __restrict__ g2, float scale, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float v1[8], v2[8], a[8];
    load8(g1 + i * 8, v1);
    load8(g2 + i * 8, v2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = v1[j] * scale;
      a[j] += v2[j] * scale;
    }
    store8f(acc + i * 8, a);
  }
}

__global__ void accum_grad_pair_tail_kernel(float* acc, const bf16_t* g1, const bf16_t* g2, float scale,
                                            long long start, long long n) {
  long long i = start + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i < n) {
    float a = bf2f(g1[i]) * scale;
    a += bf2f(g2[i]) * scale;
    acc[i] = a;
  }
}

KCA_API int kca_accum_grad_pair(float* acc, const void* g1, const void* g2, float scale, long long n,
                                hipStream_t stream) {
  const long long n8 = n / 8;
  if (n8)
    hipLaunchKernelGGL(accum_grad_pair_kernel, dim3(kca_grid(n8, 256)), dim3(256), 0, stream, acc,
                       (const bf16_t*)g1, (const bf16_t*)g2, scale, n8);
  if (n % 8)
    hipLaunchKernelGGL(accum_grad_pair_tail_kernel, dim3(1), dim3(64), 0, stream, acc, (const bf16_t*)g1,
                       (const bf16_t*)g2, scale, n8 * 8, n);
  return 0;
}

// Many small gradients in one launch: the SD UNet has ~690 parameters, most of them norms,
// biases and small projections, and one kca_accum_grad launch each cost ~5 us of GPU time per
// micro-batch (profiled DreamBooth step) for a few KB of work. The entries {dst fp32*, src bf16*,
// n, first} travel BY VALUE in the kernel arguments (up to 96 per launch, 3 KB of the 4 KB
// kernarg segment): no device-side table, so nothing to allocate, copy or keep alive between
// launches. Block (x, y) handles elements [2048x, 2048x + 2048) of entry y; 16-B vectors when
// both pointers are aligned, scalars otherwise and in the tail.
struct AccumEntry {
  float* dst;
  const bf16_t* src;
  long long n;
  long long first;
};
constexpr int kAccumBatch = 96;
struct AccumBatch {
  AccumEntry e[kAccumBatch];
};

__global__ void __launch_bounds__(256) accum_grad_multi_kernel(const AccumBatch b, float scale) {
  const AccumEntry e = b.e[blockIdx.y];
  const long long i0 = (long long)blockIdx.x * 2048 + threadIdx.x * 8;
  if (i0 >= e.n) return;
  const bool ow = e.first != 0;
  if (i0 + 8 <= e.n && ((reinterpret_cast<uintptr_t>(e.dst) | reinterpret_cast<uintptr_t>(e.src)) & 15) == 0) {
    float v[8], a[8];
    load8(e.src + i0, v);
    if (ow) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = v[j] * scale;
    } else {
      load8f(e.dst + i0, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += v[j] * scale;
    }
    store8f(e.dst + i0, a);
    return;
  }
  for (long long i = i0; i < i0 + 8 && i < e.n; ++i) e.dst[i] = (ow ? 0.f : e.dst[i]) + bf2f(e.src[i]) * scale;
}

// ents: HOST array of `count` entries {dst, src, n, first} (int64 each), any count (launched in
// batches of kAccumBatch); the host memory may be reused as soon as this returns
KCA_API int kca_accum_grad_multi(const long long* ents, int count, float scale, hipStream_t stream) {
  if (count < 0 || (count && !ents)) return 1;
  for (int base = 0; base < count; base += kAccumBatch) {
    const int c = count - base < kAccumBatch ? count - base : kAccumBatch;
    AccumBatch b;
    long long max_n = 0;
    for (int i = 0; i < c; ++i) {
      const long long* r = ents + 4LL * (base + i);
      b.e[i] = AccumEntry{reinterpret_cast<float*>(r[0]), reinterpret_cast<const bf16_t*>(r[1]), r[2], r[3]};
      if (r[2] > max_n) max_n = r[2];
    }
    if (max_n <= 0) continue;
    const long long bx = (max_n + 2047) / 2048;
    if (bx > (1ll << 30)) return 1;
    hipLaunchKernelGGL(accum_grad_multi_kernel, dim3((unsigned)bx, (unsigned)c), dim3(256), 0, stream, b, scale);
    if (hipGetLastError() != hipSuccess) return 2;
  }
  return 0;
}

// EMA (K21): shadow <- shadow + (1 - decay) * (param - shadow), flat fp32.
__global__ void ema_kernel(float* __restrict__ shadow, const float* __restrict__ p, float w, long long n4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 s = reinterpret_cast<float4*>(shadow)[i];
    const float4 v = reinterpret_cast<const float4*>(p)[i];
    s.x += w * (v.x - s.x);
    s.y += w * (v.y - s.y);
    s.z += w * (v.z - s.z);
    s.w += w * (v.w - s.w);
    reinterpret_cast<float4*>(shadow)[i] = s;
  }
}

KCA_API int kca_ema(float* shadow, const float* p, float decay, long long n, hipStream_t stream) {
  if (n % 4) return 1;
  hipLaunchKernelGGL(ema_kernel, dim3(kca_grid(n / 4, 256)), dim3(256), 0, stream, shadow, p,
                     1.f - decay, n / 4);
  return 0;
}

// fp32 -> bf16 cast (master -> model copy, ZeRO all-gather staging).
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x,
                                     bf16_t* __restrict__ y, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    float v[8];
    load8f(x + i * 8, v);
    store8(y + i * 8, v);
  }
}

KCA_API int kca_cast_f32_bf16(const float* x, void* y, long long n,
                              hipStream_t stream) {
  if (n % 8) return 1;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(kca_grid(n / 8, 256)),
                     dim3(256), 0, stream, x, (bf16_t*)y, n / 8);
  return 0;
}

// GEGLU (K17, diffusers FeedForward in every UNet transformer block):
// x = [a | g] per row (2*I wide, the GEMM output), y = a * gelu_erf(g).
// One pass over x instead of chunk + fp32 cast + GELU + cast + multiply.
// Backward writes dx = [dy * gelu(g) | dy * a * gelu'(g)].
__global__ void geglu_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int i8, long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8;
       t += (long long)gridDim.x * blockDim.x) {
    const long long row = t / i8;
    const int c = (int)(t - row * i8) * 8;
    const bf16_t* xr = x + row * (16LL * i8);
    float a[8], g[8];
    load8(xr + c, a);
    load8(xr + 8LL * i8 + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] *= gelu_erf(g[j]);
    store8(y + t * 8, a);
  }
}

__global__ void geglu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                 bf16_t* __restrict__ dx, int i8, long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8;
       t += (long long)gridDim.x * blockDim.x) {
    const long long row = t / i8;
    const int c = (int)(t - row * i8) * 8;
    const long long ro = row * (16LL * i8);
    float a[8], g[8], d[8];
    load8(x + ro + c, a);
    load8(x + ro + 8LL * i8 + c, g);
    load8(dy + t * 8, d);
    float da[8], dg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      da[j] = d[j] * gelu_erf(g[j]);
      dg[j] = d[j] * a[j] * gelu_erf_grad(g[j]);
    }
    store8(dx + ro + c, da);
    store8(dx + ro + 8LL * i8 + c, dg);
  }
}

// x: [rows, 2*inner], y/dy: [rows, inner]; inner % 8 == 0
KCA_API int kca_geglu_fwd(const void* x, void* y, long long rows, int inner, hipStream_t stream) {
  if (inner % 8) return 1;
  const long long n8 = rows * (inner / 8);
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(geglu_fwd_kernel, dim3(kca_grid(n8, 256, 8192)), dim3(256), 0, stream, (const bf16_t*)x,
                     (bf16_t*)y, inner / 8, n8);
  return 0;
}

KCA_API int kca_geglu_bwd(const void* dy, const void* x, void* dx, long long rows, int inner, hipStream_t stream) {
  if (inner % 8) return 1;
  const long long n8 = rows * (inner / 8);
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(kca_grid(n8, 256, 8192)), dim3(256), 0, stream, (const bf16_t*)dy,
                     (const bf16_t*)x, (bf16_t*)dx, inner / 8, n8);
  return 0;
}

// ---------------------------------------------------------------- residual + conv bias (NHWC)
// out = a + b + bias[c] over channels-last rows of C channels (c = innermost index): the SD ResNet
// block's `shortcut(x) + conv2(h)` with conv2's (and the 1x1 shortcut conv's) bias folded in, so
// the convolutions run without their separate broadcast bias-add pass. b may be null.
__global__ void add_bias_nhwc_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                     const float* __restrict__ bias, bf16_t* __restrict__ out, int c8,
                                     long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % c8) * 8;
    float x[8], y[8];
    load8(a + t * 8, x);
    if (b) {
      load8(b + t * 8, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += y[j];
    }
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
    x[0] += b0.x; x[1] += b0.y; x[2] += b0.z; x[3] += b0.w;
    x[4] += b1.x; x[5] += b1.y; x[6] += b1.z; x[7] += b1.w;
    store8(out + t * 8, x);
  }
}

KCA_API int kca_add_bias_nhwc(const void* a, const void* b, const float* bias, void* out, long long n, int C,
                              hipStream_t stream) {
  if (C % 8 || n % C || !a || !bias || !out) return 1;
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out | (uintptr_t)bias) & 15) return 2;
  const long long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(add_bias_nhwc_kernel, dim3(kca_grid(n8, 256, 8192)), dim3(256), 0, stream, (const bf16_t*)a,
                     (const bf16_t*)b, bias, (bf16_t*)out, C / 8, n8);
  return 0;
}

// Training form: the two convolution biases (conv2's, the 1x1 shortcut's or null) are read as the
// bf16 parameters themselves -- no per-step fp32 casts and adds of them on the host side.
__global__ void add_bias2_nhwc_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                      const bf16_t* __restrict__ b1, const bf16_t* __restrict__ b2,
                                      bf16_t* __restrict__ out, int c8, long long n8) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n8;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % c8) * 8;
    float x[8], y[8];
    load8(a + t * 8, x);
    if (b) {
      load8(b + t * 8, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += y[j];
    }
    load8(b1 + c, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += y[j];
    if (b2) {
      load8(b2 + c, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] += y[j];
    }
    store8(out + t * 8, x);
  }
}

KCA_API int kca_add_bias2_nhwc(const void* a, const void* b, const void* bias1, const void* bias2, void* out,
                               long long n, int C, hipStream_t stream) {
  if (C % 8 || n % C || !a || !bias1 || !out) return 1;
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out | (uintptr_t)bias1 | (uintptr_t)bias2) & 15) return 2;
  const long long n8 = n / 8;
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(add_bias2_nhwc_kernel, dim3(kca_grid(n8, 256, 8192)), dim3(256), 0, stream, (const bf16_t*)a,
                     (const bf16_t*)b, (const bf16_t*)bias1, (const bf16_t*)bias2, (bf16_t*)out, C / 8, n8);
  return 0;
}

// ---------------------------------------------------------------- column sums (bias gradients)
// part[by][c] = sum over rows [by*RB, by*RB + RB) of x[r][c], x [M][N] bf16 row-major (N % 8 == 0):
// 32 column groups of 8 (16-B loads, coalesced along the row) x 8 row lanes per workgroup, the row
// lanes folded through LDS; the caller sums the few partial rows (deterministic: no atomics).
// PyTorch's reduction ran these tall-skinny sums at 0.4-1 TB/s (profiles/sd_train_gemm_attribution_r2.txt).
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                          int M, int N, int RB) {
  __shared__ float red[8][32 * 8 + 4];
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  const int r0 = blockIdx.y * RB, r1 = min(M, r0 + RB);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    for (int r = r0 + rl; r < r1; r += 8) {
      float v[8];
      load8(x + (long long)r * N + c0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cg * 8 + j] = acc[j];
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += red[i][threadIdx.x];
    part[(long long)blockIdx.y * N + c] = s;
  }
}

KCA_API int kca_colsum_bf16(const void* x, float* part, int M, int N, int RB, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 8 || RB <= 0 || ((uintptr_t)x & 15)) return 1;
  const dim3 grid((N + 255) / 256, (M + RB - 1) / RB);
  hipLaunchKernelGGL(colsum_bf16_kernel, grid, dim3(256), 0, stream, (const bf16_t*)x, part, M, N, RB);
  return 0;
}
