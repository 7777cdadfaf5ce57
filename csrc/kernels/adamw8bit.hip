// Block-wise 8-bit AdamW (N10 in SURVEY §2.2: the bitsandbytes AdamW8bit the SD
// trainer asks for with --use_8bit_adam, sd-finetuner-workflow/sd-finetuner/
// finetuner.py:669-678).
//
// State per 2048-element block: exp_avg as int8 codes + one fp32 absmax,
// exp_avg_sq as uint8 codes + one fp32 absmax (2.0 B/param of state instead of
// 8). Codes are companded so small magnitudes keep precision:
//   m = absmax_m * sign(c) * (|c| / 127)^2          c in [-127, 127]
//   v = absmax_v * (c / 255)^4                      c in [0, 255]
// One workgroup (256 threads x 8 elements) owns one block: dequantise, AdamW
// update in fp32 (master params stay fp32), block absmax of the new moments
// (LDS reduction), requantise, write master + bf16 copy. One launch for the
// whole flat buffer; clip coefficient / skip flag read from device memory as
// in adamw.hip (no host sync, graph-capturable).
#include "common.h"

namespace {

constexpr int kBlock = 2048;

struct Adam8Args {
  float lr, beta1, beta2, eps, wd, bc1, bc2;
};

__device__ __forceinline__ float deq_m(int8_t c, float amax) {
  const float t = fabsf((float)c) * (1.f / 127.f);
  return copysignf(amax * t * t, (float)c);
}
__device__ __forceinline__ float deq_v(uint8_t c, float amax) {
  const float t = (float)c * (1.f / 255.f);
  const float t2 = t * t;
  return amax * t2 * t2;
}
__device__ __forceinline__ int8_t q_m(float x, float inv_amax) {
  const float t = sqrtf(fminf(fabsf(x) * inv_amax, 1.f));
  const int c = (int)rintf(127.f * t);
  return (int8_t)(x < 0.f ? -c : c);
}
__device__ __forceinline__ uint8_t q_v(float x, float inv_amax) {
  const float t = sqrtf(sqrtf(fminf(fmaxf(x, 0.f) * inv_amax, 1.f)));
  return (uint8_t)(int)rintf(255.f * t);
}

__global__ void __launch_bounds__(256) adamw8_kernel(
    float* __restrict__ p, const float* __restrict__ g, int8_t* __restrict__ mq,
    float* __restrict__ mmax, uint8_t* __restrict__ vq, float* __restrict__ vmax,
    bf16_t* __restrict__ p_bf, long long n, const uint8_t* __restrict__ wd_mask, Adam8Args a,
    const float* __restrict__ gscale, const int* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ float red[2][8];
  const float gs = gscale ? *gscale : 1.f;
  const long long blk = blockIdx.x;
  const long long i0 = blk * kBlock + threadIdx.x * 8;
  const int nv = (int)max(0LL, min(8LL, n - i0));  // n % 4 == 0 -> 0, 4 or 8
  const float am = mmax[blk], av = vmax[blk];
  float pa[8], ma[8], va[8];
  int8_t mc[8];
  uint8_t vc[8];
  if (nv == 8) {
    *reinterpret_cast<uint2*>(mc) = *reinterpret_cast<const uint2*>(mq + i0);
    *reinterpret_cast<uint2*>(vc) = *reinterpret_cast<const uint2*>(vq + i0);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mc[j] = j < nv ? mq[i0 + j] : 0;
      vc[j] = j < nv ? vq[i0 + j] : 0;
    }
  }
  float ga[8];
  if (nv == 8) {
    load8f(p + i0, pa);
    load8f(g + i0, ga);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pa[j] = j < nv ? p[i0 + j] : 0.f;
      ga[j] = j < nv ? g[i0 + j] : 0.f;
    }
  }
  const bool dec = a.wd != 0.f && nv > 0 && (wd_mask == nullptr || wd_mask[i0 >> 6]);
  const float step_size = a.lr / a.bc1, inv_sqrt_bc2 = rsqrtf(a.bc2);
  float mx_m = 0.f, mx_v = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float gr = ga[j] * gs;
    ma[j] = a.beta1 * deq_m(mc[j], am) + (1.f - a.beta1) * gr;
    va[j] = a.beta2 * deq_v(vc[j], av) + (1.f - a.beta2) * gr * gr;
    const float denom = sqrtf(va[j]) * inv_sqrt_bc2 + a.eps;
    if (dec) pa[j] *= (1.f - a.lr * a.wd);
    pa[j] -= step_size * ma[j] / denom;
    if (j < nv) {
      mx_m = fmaxf(mx_m, fabsf(ma[j]));
      mx_v = fmaxf(mx_v, va[j]);
    }
  }
  // block absmax of the new moments
  mx_m = wave_max(mx_m);
  mx_v = wave_max(mx_v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = mx_m; red[1][wid] = mx_v; }
  __syncthreads();
  float nm = 0.f, nvx = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) { nm = fmaxf(nm, red[0][w]); nvx = fmaxf(nvx, red[1][w]); }
  const float inv_m = nm > 0.f ? 1.f / nm : 0.f, inv_v = nvx > 0.f ? 1.f / nvx : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mc[j] = q_m(ma[j], inv_m);
    vc[j] = q_v(va[j], inv_v);
  }
  if (threadIdx.x == 0) { mmax[blk] = nm; vmax[blk] = nvx; }
  if (nv == 8) {
    *reinterpret_cast<uint2*>(mq + i0) = *reinterpret_cast<const uint2*>(mc);
    *reinterpret_cast<uint2*>(vq + i0) = *reinterpret_cast<const uint2*>(vc);
    store8f(p + i0, pa);
    if (p_bf) store8(p_bf + i0, pa);
  } else {
    for (int j = 0; j < nv; ++j) {
      mq[i0 + j] = mc[j];
      vq[i0 + j] = vc[j];
      p[i0 + j] = pa[j];
      if (p_bf) p_bf[i0 + j] = f2bf(pa[j]);
    }
  }
}

}  // namespace

// n % 4 == 0; mmax / vmax hold ceil(n / 2048) floats (zero-initialised).
KCA_API int kca_adamw8bit(float* p, const float* g, int8_t* mq, float* mmax, uint8_t* vq,
                          float* vmax, void* p_bf, long long n, const uint8_t* wd_mask, float lr,
                          float beta1, float beta2, float eps, float wd, float bc1, float bc2,
                          const float* gscale, const int* skip, hipStream_t stream) {
  if (n % 4) return 1;
  const long long nb = (n + kBlock - 1) / kBlock;
  Adam8Args a{lr, beta1, beta2, eps, wd, bc1, bc2};
  hipLaunchKernelGGL(adamw8_kernel, dim3((unsigned)nb), dim3(256), 0, stream, p, g, mq, mmax, vq,
                     vmax, (bf16_t*)p_bf, n, wd_mask, a, gscale, skip);
  return 0;
}
