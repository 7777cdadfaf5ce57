// Nearest-x2 upsampling + 3x3 convolution of the SD-1.5 UNet / VAE upsamplers as ONE GEMM.
//
// nearest-x2 followed by a 3x3 conv (padding 1) equals, per output phase (a, b), a 2x2 conv of the
// low-resolution input (models/unet.py phase_weights): 16 instead of 36 multiply-adds per (input
// pixel, Cin, Cout), and the 4x upsampled activation is never written. MIOpen runs that 2x2 conv
// with 4*C outputs at ~190 TFLOP/s (bench/upsample_conv_bench.py), so it goes to hipBLASLt instead:
//
//   kca_im2col2x2_nhwc : x [N, h, w, C] -> A [N*(h+1)*(w+1), 4C], A[(n,i,j), (2s+t)*C + c] =
//                        x[n, i-1+s, j-1+t, c] (zero outside), 16-B vectors, one pass;
//   (hipBLASLt)        : T = A . Wp^T, Wp [4C, 4C] the phase kernels in (s, t, c) order: T is the
//                        "phase layout" [N, h+1, w+1, 4C], output phase (a, b) in channel block 2a+b
//                        at grid offset (a, b);
//   kca_phase_to_dense_nhwc : T (+ the conv bias) -> the dense [N, 2h, 2w, C] output, for consumers
//                        that do not read the phase layout in place (the VAE decoder; the UNet's
//                        concat GroupNorm reads it directly, groupnorm_nhwc.hip).
//   kca_upsample2x_nhwc : plain nearest-x2 (the A/B baseline and the non-GEMM fallback).
// Training (ops/upsample.py UpsampleConvPhase): the backward of the dense scatter is
// kca_dense_to_phase_nhwc (the gather, zero where a phase's grid position is unused) and the
// backward of the im2col is kca_col2im2x2_nhwc (each input pixel sums its 4 patch copies).
#include "common.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// one thread per 16-B chunk of A: chunk q of row r = ((n*(h+1) + i)*(w+1) + j); C8 = C / 8
__global__ void __launch_bounds__(256) im2col2x2_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ a,
                                                        int h, int w, int C8, long long total) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int q = (int)(idx % (4 * C8));
  const long long r = idx / (4 * C8);
  const int tap = q / C8, c8 = q % C8;
  const int s = tap >> 1, t = tap & 1;
  const int j = (int)(r % (w + 1));
  const long long ni = r / (w + 1);
  const int i = (int)(ni % (h + 1));
  const long long n = ni / (h + 1);
  const int si = i - 1 + s, sj = j - 1 + t;
  u32x4 v = {0u, 0u, 0u, 0u};
  if (si >= 0 && si < h && sj >= 0 && sj < w)
    v = *reinterpret_cast<const u32x4*>(x + (((n * h + si) * w + sj) * (long long)C8 + c8) * 8);
  *reinterpret_cast<u32x4*>(a + idx * 8) = v;
}

// one thread per 16-B chunk of the dense output [N, 2h, 2w, C]
__global__ void __launch_bounds__(256) phase_to_dense_kernel(const bf16_t* __restrict__ t, const bf16_t* __restrict__ bias,
                                                             bf16_t* __restrict__ out, int h, int w, int C8,
                                                             long long total) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  const long long pix = idx / C8;
  const int X = (int)(pix % (2 * w));
  const long long nY = pix / (2 * w);
  const int Y = (int)(nY % (2 * h));
  const long long n = nY / (2 * h);
  const int a = Y & 1, b = X & 1, i = Y >> 1, j = X >> 1;
  const long long src = (((n * (h + 1) + i + a) * (w + 1) + j + b) * 4 + (2 * a + b)) * (long long)C8 + c8;
  if (bias == nullptr) {
    *reinterpret_cast<u32x4*>(out + idx * 8) = *reinterpret_cast<const u32x4*>(t + src * 8);
    return;
  }
  float v[8], bb[8];
  load8(t + src * 8, v);
  load8(bias + c8 * 8, bb);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] += bb[k];
  store8(out + idx * 8, v);
}

// one thread per 16-B chunk of the output [N, 2h, 2w, C]
__global__ void __launch_bounds__(256) upsample2x_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                         int h, int w, int C8, long long total) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  const long long pix = idx / C8;
  const int X = (int)(pix % (2 * w));
  const long long nY = pix / (2 * w);
  const int Y = (int)(nY % (2 * h));
  const long long n = nY / (2 * h);
  const long long src = ((n * h + (Y >> 1)) * w + (X >> 1)) * (long long)C8 + c8;
  *reinterpret_cast<u32x4*>(out + idx * 8) = *reinterpret_cast<const u32x4*>(x + src * 8);
}

// one thread per 16-B chunk of the output [N, h+1, w+1, C]: x with one zero row below and one zero
// column to the right (the VAE encoder's Downsample2D pad (0, 1, 0, 1), channels-last in and out)
__global__ void __launch_bounds__(256) pad_br_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out, int h,
                                                     int w, int C8, long long total) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  const long long pix = idx / C8;
  const int X = (int)(pix % (w + 1));
  const long long nY = pix / (w + 1);
  const int Y = (int)(nY % (h + 1));
  const long long n = nY / (h + 1);
  u32x4 v{0u, 0u, 0u, 0u};
  if (Y < h && X < w) v = *reinterpret_cast<const u32x4*>(x + (((n * h + Y) * w + X) * (long long)C8 + c8) * 8);
  *reinterpret_cast<u32x4*>(out + idx * 8) = v;
}

// one thread per 16-B chunk of the phase layout [N, h+1, w+1, 4C]: the dense gradient [N, 2h, 2w, C]
// gathered back (phase (a, b) of grid position (i, j) is dense pixel (2(i-a)+a, 2(j-b)+b) when
// a <= i < h + a and b <= j < w + b, else unused: 0)
__global__ void __launch_bounds__(256) dense_to_phase_kernel(const bf16_t* __restrict__ d, bf16_t* __restrict__ t,
                                                             int h, int w, int C8, long long total) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int q = (int)(idx % (4 * C8));
  const long long r = idx / (4 * C8);
  const int k = q / C8, c8 = q % C8, a = k >> 1, b = k & 1;
  const int j = (int)(r % (w + 1));
  const long long ni = r / (w + 1);
  const int i = (int)(ni % (h + 1));
  const long long n = ni / (h + 1);
  u32x4 v = {0u, 0u, 0u, 0u};
  if (i >= a && i < h + a && j >= b && j < w + b) {
    const int Y = 2 * (i - a) + a, X = 2 * (j - b) + b;
    v = *reinterpret_cast<const u32x4*>(d + (((n * 2 * h + Y) * 2 * w + X) * (long long)C8 + c8) * 8);
  }
  *reinterpret_cast<u32x4*>(t + idx * 8) = v;
}

// one thread per 16-B chunk of dx [N, h, w, C]: dx[n, y, x] = sum over the 4 patches holding it,
// dA[(n, y+1-s, x+1-t), (2s+t)C + c] (fp32 sum, one rounding)
__global__ void __launch_bounds__(256) col2im2x2_kernel(const bf16_t* __restrict__ da, bf16_t* __restrict__ dx,
                                                        int h, int w, int C8, long long total) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int c8 = (int)(idx % C8);
  const long long pix = idx / C8;
  const int x = (int)(pix % w);
  const long long ny = pix / w;
  const int y = (int)(ny % h);
  const long long n = ny / h;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const long long row = (n * (h + 1) + (y + 1 - s)) * (w + 1) + (x + 1 - t);
      float v[8];
      load8(da + (row * 4 + (2 * s + t)) * (long long)C8 * 8 + c8 * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  store8(dx + idx * 8, acc);
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline unsigned blocks_for(long long total) { return (unsigned)((total + 255) / 256); }

}  // namespace

// x [N, h, w, C] bf16 (NHWC, C % 8 == 0) -> a [N*(h+1)*(w+1), 4*C]
KCA_API int kca_im2col2x2_nhwc(const void* x, void* a, int N, int h, int w, int C, hipStream_t stream) {
  if (C % 8 || N <= 0 || h <= 0 || w <= 0 || !aligned16(x) || !aligned16(a)) return 1;
  const long long total = (long long)N * (h + 1) * (w + 1) * 4 * (C / 8);
  hipLaunchKernelGGL(im2col2x2_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, (const bf16_t*)x, (bf16_t*)a,
                     h, w, C / 8, total);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// t [N, h+1, w+1, 4C] phase layout (+ bias [C] or null) -> out [N, 2h, 2w, C]
KCA_API int kca_phase_to_dense_nhwc(const void* t, const void* bias, void* out, int N, int h, int w, int C,
                                    hipStream_t stream) {
  if (C % 8 || N <= 0 || h <= 0 || w <= 0 || !aligned16(t) || !aligned16(out) || (bias && !aligned16(bias)))
    return 1;
  const long long total = (long long)N * (2 * h) * (2 * w) * (C / 8);
  hipLaunchKernelGGL(phase_to_dense_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, (const bf16_t*)t,
                     (const bf16_t*)bias, (bf16_t*)out, h, w, C / 8, total);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// x [N, h, w, C] -> out [N, 2h, 2w, C], nearest
KCA_API int kca_upsample2x_nhwc(const void* x, void* out, int N, int h, int w, int C, hipStream_t stream) {
  if (C % 8 || N <= 0 || h <= 0 || w <= 0 || !aligned16(x) || !aligned16(out)) return 1;
  const long long total = (long long)N * (2 * h) * (2 * w) * (C / 8);
  hipLaunchKernelGGL(upsample2x_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, (const bf16_t*)x,
                     (bf16_t*)out, h, w, C / 8, total);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// d [N, 2h, 2w, C] (dense gradient) -> t [N, h+1, w+1, 4C] phase layout
KCA_API int kca_dense_to_phase_nhwc(const void* d, void* t, int N, int h, int w, int C, hipStream_t stream) {
  if (C % 8 || N <= 0 || h <= 0 || w <= 0 || !aligned16(d) || !aligned16(t)) return 1;
  const long long total = (long long)N * (h + 1) * (w + 1) * 4 * (C / 8);
  hipLaunchKernelGGL(dense_to_phase_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, (const bf16_t*)d,
                     (bf16_t*)t, h, w, C / 8, total);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// da [N*(h+1)*(w+1), 4C] (im2col gradient) -> dx [N, h, w, C]
KCA_API int kca_col2im2x2_nhwc(const void* da, void* dx, int N, int h, int w, int C, hipStream_t stream) {
  if (C % 8 || N <= 0 || h <= 0 || w <= 0 || !aligned16(da) || !aligned16(dx)) return 1;
  const long long total = (long long)N * h * w * (C / 8);
  hipLaunchKernelGGL(col2im2x2_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, (const bf16_t*)da,
                     (bf16_t*)dx, h, w, C / 8, total);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// x [N, h, w, C] -> out [N, h+1, w+1, C], zero bottom row and right column
KCA_API int kca_pad_br_nhwc(const void* x, void* out, int N, int h, int w, int C, hipStream_t stream) {
  if (C % 8 || N <= 0 || h <= 0 || w <= 0 || !aligned16(x) || !aligned16(out)) return 1;
  const long long total = (long long)N * (h + 1) * (w + 1) * (C / 8);
  hipLaunchKernelGGL(pad_br_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, (const bf16_t*)x, (bf16_t*)out, h,
                     w, C / 8, total);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
