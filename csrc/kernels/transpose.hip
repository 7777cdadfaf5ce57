// bf16 matrix transpose for the weight-gradient GEMMs (K1 backward).
//
// dW = dY^T X reduces over the token dimension, which is the slow (row)
// dimension of both row-major activations, so PyTorch issues it as an "NT"
// GEMM with neither operand K-contiguous: 1.10-1.15 PFLOP/s on MI355X for the
// GPT-J shapes, against 1.43-1.54 PFLOP/s for the same math as a "TN" GEMM on
// transposed operands (profiles/gemm_layout_gptj_r1.jsonl). This kernel makes
// the transposed copies at HBM speed so the TN form wins net.
//
// One wave per 64x64 tile, no LDS: lane (rb = lane & 7, cb = lane >> 3) loads
// an 8x8 block -- 8 rows x 16 B, each row segment of the tile read by 8 lanes
// as one full 128-B line -- transposes it in registers (byte permutes of the
// 16-bit halves) and stores 8 x 16 B, again 8 lanes per full output line.
#include "common.h"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned lo16(unsigned a, unsigned b) {  // (a.lo, b.lo)
  return __builtin_amdgcn_perm(b, a, 0x05040100u);
}
__device__ __forceinline__ unsigned hi16(unsigned a, unsigned b) {  // (a.hi, b.hi)
  return __builtin_amdgcn_perm(b, a, 0x07060302u);
}

__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ in, long long ld_in,
                                                             bf16_t* __restrict__ out, long long ld_out,
                                                             int R, int C) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tiles_c = (C + 63) >> 6;
  const long long tile = (long long)blockIdx.x * 4 + wave;
  const long long ntiles = (long long)((R + 63) >> 6) * tiles_c;
  if (tile >= ntiles) return;
  const int tr = (int)(tile / tiles_c), tc = (int)(tile % tiles_c);
  const int rb = lane & 7, cb = lane >> 3;
  const long long r0 = (long long)tr * 64 + rb * 8;
  const long long c0 = (long long)tc * 64 + cb * 8;
  // edge tiles (R or C not a multiple of 64, both multiples of 8): a lane's 8 x 8 block is wholly
  // inside or wholly outside
  if (r0 >= R || c0 >= C) return;
  u32x4 a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    a[i] = *reinterpret_cast<const u32x4*>(in + (r0 + i) * ld_in + c0);
  // b[j] = column c0+j of the 8 rows: word k holds rows (2k, 2k+1)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    u32x4 bj;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned x = a[2 * k][j >> 1], y = a[2 * k + 1][j >> 1];
      bj[k] = (j & 1) ? hi16(x, y) : lo16(x, y);
    }
    *reinterpret_cast<u32x4*>(out + (c0 + j) * ld_out + r0) = bj;
  }
}

}  // namespace

// out[C, R] (row stride ld_out) = in[R, C]^T (row stride ld_in); R, C multiples
// of 8 (GPT-J's 50400-row LM head: its weight-gradient GEMM runs TN too), strides
// multiples of 8 elements, 16-B aligned pointers.
KCA_API int kca_transpose_bf16(const void* in, long long ld_in, void* out, long long ld_out, int R, int C,
                               hipStream_t stream) {
  if (R % 8 || C % 8 || ld_in % 8 || ld_out % 8 || ld_in < C || ld_out < R) return 1;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return 1;
  const long long tiles = (long long)((R + 63) / 64) * ((C + 63) / 64);
  if (tiles == 0) return 0;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, stream,
                     (const bf16_t*)in, ld_in, (bf16_t*)out, ld_out, R, C);
  return 0;
}
