// Tile kernels that fuse the elementwise work around the GPT-J block GEMMs
// into the transposes the TN-layout weight-gradient GEMMs need anyway
// (ops/fused_block.py, K5 + K1 backward):
//
//   kca_gelu_fwd_t       g = gelu(h) written row-major (the A operand of the
//                        output GEMM) AND transposed (g^T, saved for dW), so
//                        the backward never re-reads g to transpose it;
//   kca_gelu_bwd_t       dh = dg * gelu'(h) written row-major (A operand of
//                        the dX GEMM) and transposed (dh^T, A operand of the
//                        dW GEMM), plus per-64-row partial column sums of dh
//                        (the fc_in bias gradient);
//   kca_transpose_colsum out = in^T plus partial column sums of in (the
//                        fc_out bias gradient rides on the dY transpose);
//   kca_col_reduce_f32   [nparts, C] fp32 partials -> C sums (bf16 / fp32);
//   kca_accum_grad_2d    fp32 grad accumulation from a row-strided bf16 grad
//                        (column slices of a concatenated-weight dW).
//
// Each wave owns one 64x64 tile like transpose.hip: lane (rb = lane & 7,
// cb = lane >> 3) holds an 8x8 block (8 rows x 16 B, 8 lanes per 128-B line),
// does the math in fp32, stores 8 row segments, transposes the 8x8 block in
// registers (byte permutes) and stores 8 column segments. Column sums are
// reduced over the 8 lanes sharing cb with 3 xor-shuffles; lane rb == 0 writes
// the tile's 8 partials. Every input and output is touched exactly once, so
// the kernels run at HBM speed; there are no atomics (deterministic).
#include "common.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned lo16(unsigned a, unsigned b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ unsigned hi16(unsigned a, unsigned b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

enum { MODE_TRANSPOSE = 0, MODE_GELU_FWD = 1, MODE_GELU_BWD = 2 };

struct TileArgs {
  const bf16_t* a;  // in / h / dg
  long long lda;
  const bf16_t* b;  // h (GELU backward)
  long long ldb;
  bf16_t* y;  // row-major output (g / dh), may be null
  long long ldy;
  bf16_t* yt;  // transposed output
  long long ldyt;
  float* part;  // [R/64, C] partial column sums, may be null
  int R, C;
};

__device__ __forceinline__ void unpack8(const u32x4 w, float (&f)[8]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(w[k] << 16);
    f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  u32x4 w;
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = pack_bf16x2(f[2 * k], f[2 * k + 1]);
  return w;
}

template <int MODE, bool TANH>
__global__ void __launch_bounds__(256) tile_fused_kernel(TileArgs p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_c = p.C >> 6;
  const long long tile = (long long)blockIdx.x * 4 + wave;
  if (tile >= (long long)(p.R >> 6) * tiles_c) return;
  const int tr = (int)(tile / tiles_c), tc = (int)(tile % tiles_c);
  const int rb = lane & 7, cb = lane >> 3;
  const long long r0 = (long long)tr * 64 + rb * 8;
  const long long c0 = (long long)tc * 64 + cb * 8;

  u32x4 w[8];
  float cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;

  if (MODE == MODE_TRANSPOSE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = *reinterpret_cast<const u32x4*>(p.a + (r0 + i) * p.lda + c0);
    if (p.part) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float f[8];
        unpack8(w[i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) cs[j] += f[j];
      }
    }
  } else {
    u32x4 src[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) src[i] = *reinterpret_cast<const u32x4*>(p.a + (r0 + i) * p.lda + c0);
    u32x4 hsrc[8];
    if (MODE == MODE_GELU_BWD) {
#pragma unroll
      for (int i = 0; i < 8; ++i) hsrc[i] = *reinterpret_cast<const u32x4*>(p.b + (r0 + i) * p.ldb + c0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float f[8];
      unpack8(src[i], f);
      if (MODE == MODE_GELU_FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = TANH ? gelu_tanh(f[j]) : 0.5f * f[j] * (1.f + erff(f[j] * 0.7071067811865476f));
      } else {
        float h[8];
        unpack8(hsrc[i], h);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float gr;
          if (TANH) {
            gr = gelu_tanh_grad(h[j]);
          } else {
            const float cdf = 0.5f * (1.f + erff(h[j] * 0.7071067811865476f));
            gr = cdf + h[j] * 0.3989422804014327f * __expf(-0.5f * h[j] * h[j]);
          }
          f[j] *= gr;
        }
      }
      w[i] = pack8(f);
      if (MODE == MODE_GELU_BWD && p.part) {
#pragma unroll
        for (int j = 0; j < 8; ++j) cs[j] += f[j];
      }
    }
    if (p.y) {
#pragma unroll
      for (int i = 0; i < 8; ++i) *reinterpret_cast<u32x4*>(p.y + (r0 + i) * p.ldy + c0) = w[i];
    }
  }

  // transposed store: column c0+j of the 8 rows, word k = rows (2k, 2k+1)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    u32x4 bj;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned x = w[2 * k][j >> 1], y = w[2 * k + 1][j >> 1];
      bj[k] = (j & 1) ? hi16(x, y) : lo16(x, y);
    }
    *reinterpret_cast<u32x4*>(p.yt + (c0 + j) * p.ldyt + r0) = bj;
  }

  if (MODE != MODE_GELU_FWD && p.part) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = cs[j];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      cs[j] = s;
    }
    if (rb == 0) {
      float* dst = p.part + (size_t)tr * p.C + c0;
      *reinterpret_cast<float4*>(dst) = make_float4(cs[0], cs[1], cs[2], cs[3]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
    }
  }
}

// [nparts, C] -> C: a workgroup owns 64 columns; 16 row groups x 16 float4
// lanes each sum a strided subset of the parts, one LDS pass combines them.
__global__ void __launch_bounds__(256) part_reduce_kernel(const float* __restrict__ part, int nparts, int C,
                                                          bf16_t* __restrict__ out_bf, float* __restrict__ out_f) {
  __shared__ float4 red[16][16];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cl * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int q = rg; q < nparts; q += 16) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)q * C + c);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0) {
#pragma unroll
    for (int g = 1; g < 16; ++g) {
      const float4 v = red[g][cl];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (out_bf) {
      uint2 u;
      u.x = pack_bf16x2(s.x, s.y);
      u.y = pack_bf16x2(s.z, s.w);
      *reinterpret_cast<uint2*>(out_bf + c) = u;
    }
    if (out_f) *reinterpret_cast<float4*>(out_f + c) = s;
  }
}

__global__ void accum_grad2d_kernel(float* __restrict__ acc, const bf16_t* __restrict__ g, long long ldg,
                                    int cols8, long long n8, float scale, int overwrite) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols8;
    const int c = (int)(i % cols8) * 8;
    float v[8], a[8];
    load8(g + r * ldg + c, v);
    float* dst = acc + i * 8;
    if (overwrite) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = v[j] * scale;
    } else {
      load8f(dst, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += v[j] * scale;
    }
    store8f(dst, a);
  }
}

bool tile_ok(const TileArgs& p) {
  if (p.R % 64 || p.C % 64 || p.R <= 0 || p.C <= 0) return false;
  if (p.lda % 8 || p.ldyt % 8 || p.lda < p.C || p.ldyt < p.R) return false;
  uintptr_t al = reinterpret_cast<uintptr_t>(p.a) | reinterpret_cast<uintptr_t>(p.yt);
  if (p.b) {
    if (p.ldb % 8 || p.ldb < p.C) return false;
    al |= reinterpret_cast<uintptr_t>(p.b);
  }
  if (p.y) {
    if (p.ldy % 8 || p.ldy < p.C) return false;
    al |= reinterpret_cast<uintptr_t>(p.y);
  }
  if (p.part) al |= reinterpret_cast<uintptr_t>(p.part);
  return (al & 15) == 0;
}

template <int MODE>
int launch_tile(const TileArgs& p, int tanh_approx, hipStream_t stream) {
  if (!tile_ok(p)) return 1;
  const long long tiles = (long long)(p.R / 64) * (p.C / 64);
  const dim3 grid((unsigned)((tiles + 3) / 4));
  if (tanh_approx)
    hipLaunchKernelGGL((tile_fused_kernel<MODE, true>), grid, dim3(256), 0, stream, p);
  else
    hipLaunchKernelGGL((tile_fused_kernel<MODE, false>), grid, dim3(256), 0, stream, p);
  return 0;
}

}  // namespace

// g[R, C] (ld_g) = gelu(h) and gt[C, R] (ld_gt) = g^T; h has row stride ld_h.
KCA_API int kca_gelu_fwd_t(const void* h, long long ld_h, void* g, long long ld_g, void* gt, long long ld_gt,
                           int R, int C, int tanh_approx, hipStream_t stream) {
  TileArgs p{(const bf16_t*)h, ld_h, nullptr, 0, (bf16_t*)g, ld_g, (bf16_t*)gt, ld_gt, nullptr, R, C};
  return launch_tile<MODE_GELU_FWD>(p, tanh_approx, stream);
}

// dh = dg * gelu'(h) -> dh[R, C] (ld_dh, may be null), dht[C, R] (ld_dht),
// part[R/64, C] partial column sums of dh (may be null).
KCA_API int kca_gelu_bwd_t(const void* dg, long long ld_dg, const void* h, long long ld_h, void* dh, long long ld_dh,
                           void* dht, long long ld_dht, float* part, int R, int C, int tanh_approx,
                           hipStream_t stream) {
  TileArgs p{(const bf16_t*)dg, ld_dg, (const bf16_t*)h, ld_h, (bf16_t*)dh, ld_dh, (bf16_t*)dht, ld_dht, part, R, C};
  return launch_tile<MODE_GELU_BWD>(p, tanh_approx, stream);
}

// out[C, R] = in[R, C]^T and part[R/64, C] partial column sums of in (nullable).
KCA_API int kca_transpose_colsum(const void* in, long long ld_in, void* out, long long ld_out, float* part, int R,
                                 int C, hipStream_t stream) {
  TileArgs p{(const bf16_t*)in, ld_in, nullptr, 0, nullptr, 0, (bf16_t*)out, ld_out, part, R, C};
  return launch_tile<MODE_TRANSPOSE>(p, 1, stream);
}

// out = sum over the nparts rows of part[nparts, C]; C % 64 == 0.
KCA_API int kca_col_reduce_f32(const float* part, int nparts, int C, void* out_bf, float* out_f, hipStream_t stream) {
  if (C % 64 || nparts <= 0) return 1;
  hipLaunchKernelGGL(part_reduce_kernel, dim3(C / 64), dim3(256), 0, stream, part, nparts, C, (bf16_t*)out_bf,
                     out_f);
  return 0;
}

// acc[rows, cols] (contiguous fp32) (+)= scale * g (bf16, row stride ldg); cols % 8 == 0.
KCA_API int kca_accum_grad_2d(float* acc, const void* g, long long ldg, int rows, int cols, float scale,
                              int overwrite, hipStream_t stream) {
  if (cols % 8 || ldg % 8 || ldg < cols || (reinterpret_cast<uintptr_t>(g) & 15)) return 1;
  const long long n8 = (long long)rows * (cols / 8);
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(accum_grad2d_kernel, dim3(kca_grid(n8, 256)), dim3(256), 0, stream, acc, (const bf16_t*)g,
                     ldg, cols / 8, n8, scale, overwrite);
  return 0;
}
