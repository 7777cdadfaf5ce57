// Fused softmax cross-entropy with ignore_index (K6 in SURVEY §2.4).
//
// The reference masks padded labels to -100 before HF's CrossEntropyLoss
// (finetuner-workflow/finetuner/finetuner.py:476-477). Here one workgroup owns
// one row of bf16 logits [N, V] (row stride ld): a single online pass computes
// max and sum(exp) (running-max rescale per thread, one block combine), so the
// vocab row is read once in the forward and once in the backward, and fp32
// logits are never materialised. The backward writes bf16 dlogits, optionally
// in place over the logits buffer.
#include "common.h"

template <bool VEC>
__global__ void __launch_bounds__(256) ce_fwd_kernel(
    const bf16_t* __restrict__ logits, long long ld,
    const long long* __restrict__ labels, int V, int ignore_index,
    float* __restrict__ loss, float* __restrict__ lse_out) {
  __shared__ float red[16];
  const long long row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  if (VEC) {
    const int nv = V >> 3;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
      float v[8];
      load8(x + i * 8, v);
      float lm = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
      if (lm > m) { s *= __expf(m - lm); m = lm; }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
    }
    for (int i = nv * 8 + threadIdx.x; i < V; i += blockDim.x) {
      float v = bf2f(x[i]);
      if (v > m) { s *= __expf(m - v); m = v; }
      s += __expf(v - m);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      float v = bf2f(x[i]);
      if (v > m) { s *= __expf(m - v); m = v; }
      s += __expf(v - m);
    }
  }
  const float gm = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  const float gs = block_sum(s, red + 8);
  if (threadIdx.x == 0) {
    const float lse = gm + __logf(gs);
    const long long lab = labels[row];
    KCA_DASSERT(lab == ignore_index || (lab >= 0 && lab < V));  // a label outside the vocab is a data bug
    lse_out[row] = lse;
    loss[row] = (lab == ignore_index || lab < 0 || lab >= V)
                    ? 0.f
                    : lse - bf2f(x[lab]);
  }
}

// dlogits = (softmax - onehot) * dloss[row]   (0 for ignored rows)
template <bool VEC>
__global__ void __launch_bounds__(256) ce_bwd_kernel(
    const bf16_t* __restrict__ logits, long long ld,
    const long long* __restrict__ labels, const float* __restrict__ lse_in,
    const float* __restrict__ dloss, float dloss_scale, int V,
    int ignore_index, bf16_t* __restrict__ dlogits, long long ldd) {
  const long long row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  bf16_t* dx = dlogits + row * ldd;
  const long long lab = labels[row];
  const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
  const float g = ign ? 0.f : (dloss ? dloss[row] : 1.f) * dloss_scale;
  const float lse = lse_in[row];
  if (VEC) {
    const int nv = V >> 3;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
      float v[8];
      load8(x + i * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(v[j] - lse);
        v[j] = g * (p - ((i * 8 + j) == lab ? 1.f : 0.f));
      }
      store8(dx + i * 8, v);
    }
    for (int i = nv * 8 + threadIdx.x; i < V; i += blockDim.x) {
      float p = __expf(bf2f(x[i]) - lse);
      dx[i] = f2bf(g * (p - (i == lab ? 1.f : 0.f)));
    }
  } else {
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      float p = __expf(bf2f(x[i]) - lse);
      dx[i] = f2bf(g * (p - (i == lab ? 1.f : 0.f)));
    }
  }
}

KCA_API int kca_cross_entropy_fwd(const void* logits, long long ld,
                                  const long long* labels, int n, int V,
                                  int ignore_index, float* loss, float* lse,
                                  hipStream_t stream) {
  if (n <= 0) return 0;
  const bool vec = (ld % 8 == 0) && ((uintptr_t)logits % 16 == 0);
  if (vec)
    hipLaunchKernelGGL(ce_fwd_kernel<true>, dim3(n), dim3(256), 0, stream,
                       (const bf16_t*)logits, ld, labels, V, ignore_index,
                       loss, lse);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<false>, dim3(n), dim3(256), 0, stream,
                       (const bf16_t*)logits, ld, labels, V, ignore_index,
                       loss, lse);
  return 0;
}

KCA_API int kca_cross_entropy_bwd(const void* logits, long long ld,
                                  const long long* labels, const float* lse,
                                  const float* dloss, float dloss_scale, int n,
                                  int V, int ignore_index, void* dlogits,
                                  long long ldd, hipStream_t stream) {
  if (n <= 0) return 0;
  const bool vec = (ld % 8 == 0) && (ldd % 8 == 0) &&
                   ((uintptr_t)logits % 16 == 0) &&
                   ((uintptr_t)dlogits % 16 == 0);
  if (vec)
    hipLaunchKernelGGL(ce_bwd_kernel<true>, dim3(n), dim3(256), 0, stream,
                       (const bf16_t*)logits, ld, labels, lse, dloss,
                       dloss_scale, V, ignore_index, (bf16_t*)dlogits, ldd);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<false>, dim3(n), dim3(256), 0, stream,
                       (const bf16_t*)logits, ld, labels, lse, dloss,
                       dloss_scale, V, ignore_index, (bf16_t*)dlogits, ldd);
  return 0;
}
