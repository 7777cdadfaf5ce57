// Stable Diffusion sampler step, fused: classifier-free
// guidance combine + k-diffusion LMS / Euler update + the next step's scaled
// bf16 UNet input, in one pass over the latents.
//
// Replaces, per denoising step, the ~15 standalone elementwise launches of the
// torch formulation (eps.float(), chunk, eu + g*(ec - eu), x0 = x - s*eps,
// d = (x - x0)/s, the 4-term multistep sum, cat([x, x]), / sqrt(s^2+1), cast)
// that run between the UNet graph replays of the reference's diffusers
// pipeline (online-inference/stable-diffusion/service/service.py:245-252,
// LMSDiscreteScheduler). The derivative history is a ring of `order` fp32
// buffers; coefficient j multiplies the j-th newest derivative.
#include "common.h"

struct LmsArgs {
  float c[4];      // multistep coefficients, newest first
  int o;           // terms in use (<= order)
  int order;       // ring size
  int newest;      // ring slot receiving this step's derivative
  int pred;        // 0 epsilon, 1 v-prediction, 2 sample
  int cfg;         // eps holds [uncond; cond] halves
  float g;         // guidance scale
  float s;         // sigma_i
  float in_scale;  // 1/sqrt(sigma_{i+1}^2+1) for the next UNet input (xin == nullptr: last step)
};

__global__ __launch_bounds__(256) void sd_lms_step_kernel(const bf16_t* __restrict__ eps, float* __restrict__ x,
                                                          float* __restrict__ ring, bf16_t* __restrict__ xin,
                                                          long long n, LmsArgs a) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float e = bf2f(eps[i]);
    if (a.cfg) {
      const float ec = bf2f(eps[n + i]);
      e = e + a.g * (ec - e);
    }
    const float xv = x[i];
    float x0;
    if (a.pred == 0) x0 = xv - a.s * e;
    else if (a.pred == 1) x0 = e * (-a.s / sqrtf(a.s * a.s + 1.f)) + xv / (a.s * a.s + 1.f);
    else x0 = e;
    const float d = (xv - x0) / a.s;
    ring[(long long)a.newest * n + i] = d;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= a.o) break;
      const int slot = (a.newest - j + a.order) % a.order;
      acc += a.c[j] * (j == 0 ? d : ring[(long long)slot * n + i]);
    }
    const float out = xv + acc;
    x[i] = out;
    if (xin) {
      const bf16_t v = f2bf(out * a.in_scale);
      xin[i] = v;
      if (a.cfg) xin[n + i] = v;
    }
  }
}

KCA_API int kca_sd_lms_step(const void* eps, float* x, float* ring, void* xin, long long n, const float* coef,
                            int o, int order, int newest, int pred, int cfg, float g, float s, float in_scale,
                            hipStream_t stream) {
  if (n <= 0 || o < 1 || o > 4 || order < o || order > 4 || newest < 0 || newest >= order || s == 0.f) return 1;
  LmsArgs a{{0.f, 0.f, 0.f, 0.f}, o, order, newest, pred, cfg, g, s, in_scale};
  for (int j = 0; j < o; ++j) a.c[j] = coef[j];
  hipLaunchKernelGGL(sd_lms_step_kernel, dim3(kca_grid(n, 256)), dim3(256), 0, stream, (const bf16_t*)eps, x, ring,
                     (bf16_t*)xin, n, a);
  return 0;
}
