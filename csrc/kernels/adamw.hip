// Flat-buffer fused AdamW + global grad-norm (K7 in SURVEY §2.4).
//
// The optimizer state lives in contiguous fp32 buffers (master params, grads,
// exp_avg, exp_avg_sq) laid out in the same order as the model's flat bf16
// parameter buffer, so one launch updates every parameter (no multi-tensor
// pointer lists) and the ZeRO-1/2 shard of a rank is just a [lo, hi) slice.
// Weight decay is selected per 64-element block by a byte mask (every parameter
// starts on a 64-element boundary of the flat buffer), so biases / norms are
// excluded exactly as in the HF Trainer grouping the reference relies on
// (finetuner-workflow/finetuner/finetuner.py:987-1027 -> TrainingArguments).
//
// The clip coefficient / loss-scale is read from device memory, so the
// optimizer step needs no host synchronisation and can be graph-captured.
#include "common.h"

struct AdamWArgs {
  float lr, beta1, beta2, eps, wd, bc1, bc2;  // bc = 1 - beta^t
};

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v,
                             bf16_t* __restrict__ p_bf, long long n4,
                             const uint8_t* __restrict__ wd_mask, AdamWArgs a,
                             const float* __restrict__ gscale,
                             const int* __restrict__ skip) {
  if (skip && *skip) return;
  const float gs = gscale ? *gscale : 1.f;
  const float step_size = a.lr / a.bc1;
  const float inv_sqrt_bc2 = rsqrtf(a.bc2);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float pa[4] = {pp.x, pp.y, pp.z, pp.w};
    float ga[4] = {gg.x, gg.y, gg.z, gg.w};
    float ma[4] = {mm.x, mm.y, mm.z, mm.w};
    float va[4] = {vv.x, vv.y, vv.z, vv.w};
    const bool dec = a.wd != 0.f && (wd_mask == nullptr || wd_mask[i >> 4]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gr = ga[j] * gs;
      ma[j] = a.beta1 * ma[j] + (1.f - a.beta1) * gr;
      va[j] = a.beta2 * va[j] + (1.f - a.beta2) * gr * gr;
      const float denom = sqrtf(va[j]) * inv_sqrt_bc2 + a.eps;
      if (dec) pa[j] *= (1.f - a.lr * a.wd);
      pa[j] -= step_size * ma[j] / denom;
    }
    reinterpret_cast<float4*>(p)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
    reinterpret_cast<float4*>(m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
    reinterpret_cast<float4*>(v)[i] = make_float4(va[0], va[1], va[2], va[3]);
    if (p_bf) {
      uint2 o;
      o.x = pack_bf16x2(pa[0], pa[1]);
      o.y = pack_bf16x2(pa[2], pa[3]);
      reinterpret_cast<uint2*>(p_bf)[i] = o;
    }
  }
}

KCA_API int kca_adamw(float* p, const float* g, float* m, float* v, void* p_bf,
                      long long n, const uint8_t* wd_mask, float lr, float beta1,
                      float beta2, float eps, float wd, float bc1, float bc2,
                      const float* gscale, const int* skip,
                      hipStream_t stream) {
  if (n % 4) return 1;
  AdamWArgs a{lr, beta1, beta2, eps, wd, bc1, bc2};
  hipLaunchKernelGGL(adamw_kernel, dim3(kca_grid(n / 4, 256)), dim3(256), 0,
                     stream, p, g, m, v, (bf16_t*)p_bf, n / 4, wd_mask, a,
                     gscale, skip);
  return 0;
}

// ------------------------------------------------------------ grad norm
// partial[block] = sum(g^2) over a grid-stride slice; nonfinite counted too.
__global__ void sumsq_partial_kernel(const float* __restrict__ g, long long n4,
                                     float* __restrict__ partial) {
  __shared__ float red[8];
  float s = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    float4 x = reinterpret_cast<const float4*>(g)[i];
    s += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void sum_partials_kernel(const float* __restrict__ partial, int np,
                                    float* __restrict__ out) {
  __shared__ float red[8];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) *out = s;
}

// workspace: >= 1024 floats. out_sumsq: one device float.
KCA_API int kca_sumsq(const float* g, long long n, float* workspace,
                      float* out_sumsq, hipStream_t stream) {
  if (n % 4) return 1;
  const int grid = kca_grid(n / 4, 256, 1024);
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(grid), dim3(256), 0, stream, g,
                     n / 4, workspace);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, stream,
                     workspace, grid, out_sumsq);
  return 0;
}

// coef = min(1, max_norm / (sqrt(sumsq) + 1e-6)) * extra_scale;
// skip = !isfinite(sumsq) (fp16 overflow / NaN guard).
__global__ void clip_coef_kernel(const float* __restrict__ sumsq,
                                 float max_norm, float extra_scale,
                                 float* __restrict__ coef,
                                 float* __restrict__ norm_out,
                                 int* __restrict__ skip) {
  const float s = *sumsq;
  const float nrm = sqrtf(s) * extra_scale;
  float c = extra_scale;
  if (max_norm > 0.f && nrm > max_norm) c *= max_norm / (nrm + 1e-6f);
  *coef = c;
  if (norm_out) *norm_out = nrm;
  if (skip) *skip = isfinite(s) ? 0 : 1;
}

KCA_API int kca_clip_coef(const float* sumsq, float max_norm,
                          float extra_scale, float* coef, float* norm_out,
                          int* skip, hipStream_t stream) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, stream, sumsq,
                     max_norm, extra_scale, coef, norm_out, skip);
  return 0;
}
