// LayerNorm forward/backward with optional fused residual adds (K4 in SURVEY §2.4).
//
// Forward:  h = x (+ r1) (+ r2)          (stored when adds are present)
//           y = (h - mean) * rstd * gamma + beta
// One workgroup per row; every thread keeps NV x 8 elements of the row in
// registers, so the row is read from HBM exactly once and the two-pass
// (exact) variance costs no extra traffic. fp32 statistics, bf16 I/O.
//
// Backward: dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)) (+ dres)
// dgamma/dbeta are accumulated per workgroup in registers over a grid-stride
// row loop, written as fp32 partial rows, and summed by a column-reduce kernel
// (deterministic; no float atomics).
//
// Replaces what HF/Apex FusedLayerNorm supplied to the reference's GPT-J /
// NeoX / BLOOM / CLIP stacks (online-inference/custom-pytorch-aitextgen/
// custom-predictor/Dockerfile:9-11 builds Apex --cuda_ext for exactly this).
#include "common.h"

template <int NV>
__global__ void __launch_bounds__(256) ln_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ r1,
    const bf16_t* __restrict__ r2, bf16_t* __restrict__ h_out,
    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
    bf16_t* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int rows, int d, float eps) {
  __shared__ float red[16];
  const int nvec = d >> 3;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * d;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (vi < nvec) {
        load8(x + base + vi * 8, v[i]);
        if (r1) {
          float t[8];
          load8(r1 + base + vi * 8, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] += t[j];
        }
        if (r2) {
          float t[8];
          load8(r2 + base + vi * 8, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] += t[j];
        }
        if (h_out) {
          store8(h_out + base + vi * 8, v[i]);
          // statistics of the rounded residual that the backward will re-read
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j]));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      }
    }
    const float mean = block_sum(s, red) / d;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (vi < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float c = v[i][j] - mean;
          q += c * c;
        }
      }
    }
    const float var = block_sum(q, red + 8) / d;
    const float rstd = rsqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (vi < nvec) {
        float g[8], b[8], o[8];
        load8(gamma + vi * 8, g);
        if (beta) load8(beta + vi * 8, b);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) b[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + b[j];
        store8(y + base + vi * 8, o);
      }
    }
    if (threadIdx.x == 0) {
      if (mean_out) mean_out[row] = mean;
      if (rstd_out) rstd_out[row] = rstd;
    }
  }
}

template <int NV>
__global__ void __launch_bounds__(256) ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ dres,
    bf16_t* __restrict__ dx, float* __restrict__ dg_part,
    float* __restrict__ db_part, int rows, int d) {
  __shared__ float red[16];
  const int nvec = d >> 3;
  float acc_g[NV][8], acc_b[NV][8], g[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc_g[i][j] = 0.f; acc_b[i][j] = 0.f; g[i][j] = 0.f; }
    if (vi < nvec) load8(gamma + vi * 8, g[i]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * d;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NV][8], gy[NV][8], rr[NV][8];
    float s1 = 0.f, s2 = 0.f;
    // the residual gradient is loaded with h and dy, ahead of the two row reductions: loaded after
    // them (as before) its HBM round trip sat serially in every row (0.29 ms per GPT-J-shaped call,
    // ~2x its byte roofline)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (dres && vi < nvec) load8(dres + base + vi * 8, rr[i]);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (vi < nvec) {
        float hv[8], dv[8];
        load8(h + base + vi * 8, hv);
        load8(dy + base + vi * 8, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = (hv[j] - mean) * rstd;
          gy[i][j] = dv[j] * g[i][j];
          s1 += gy[i][j];
          s2 += gy[i][j] * xh[i][j];
          acc_g[i][j] += dv[j] * xh[i][j];
          acc_b[i][j] += dv[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { xh[i][j] = 0.f; gy[i][j] = 0.f; }
      }
    }
    const float m1 = block_sum(s1, red) / d;
    const float m2 = block_sum(s2, red + 8) / d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = threadIdx.x + i * blockDim.x;
      if (vi < nvec) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (gy[i][j] - m1 - xh[i][j] * m2);
        if (dres) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rr[i][j];
        }
        store8(dx + base + vi * 8, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = threadIdx.x + i * blockDim.x;
    if (vi < nvec) {
      store8f(dg_part + (size_t)blockIdx.x * d + vi * 8, acc_g[i]);
      store8f(db_part + (size_t)blockIdx.x * d + vi * 8, acc_b[i]);
    }
  }
}

// Sum fp32 partial rows [nparts, d] -> out[d] (bf16 or fp32). Each thread owns
// one column; consecutive threads read consecutive columns (coalesced).
// Narrow rows (d <= 1024: SD's 320/640-wide transformer LayerNorms, GPT-2 small): the block kernel
// above runs one 64-thread workgroup per partial -- 512 waves for the whole chip, each through
// ~128 dependent rows (1.9 TB/s on [65536, 320]). Here every wave of a 256-thread workgroup takes
// its own rows (wave-level sums, no barrier per row) and the 4 waves fold their dgamma / dbeta
// partials through LDS once: the same 512 partial rows, 4x the waves.
template <int NV>
__global__ void __launch_bounds__(256) ln_bwd_narrow_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ h,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ dres,
    bf16_t* __restrict__ dx, float* __restrict__ dg_part,
    float* __restrict__ db_part, int rows, int d) {
  __shared__ float sg[4][512 * NV], sb[4][512 * NV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float g[NV][8], acc_g[NV][8], acc_b[NV][8];
  bool act[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    act[i] = lane + 64 * i < (d >> 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) { g[i][j] = 0.f; acc_g[i][j] = 0.f; acc_b[i][j] = 0.f; }
    if (act[i]) load8(gamma + (lane + 64 * i) * 8, g[i]);
  }
  for (int row = blockIdx.x * 4 + wave; row < rows; row += gridDim.x * 4) {
    const size_t base = (size_t)row * d + lane * 8;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NV][8], gy[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (act[i]) {
        float hv[8], dv[8];
        load8(h + base + 512 * i, hv);
        load8(dy + base + 512 * i, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = (hv[j] - mean) * rstd;
          gy[i][j] = dv[j] * g[i][j];
          s1 += gy[i][j];
          s2 += gy[i][j] * xh[i][j];
          acc_g[i][j] += dv[j] * xh[i][j];
          acc_b[i][j] += dv[j];
        }
      }
    }
    const float m1 = wave_sum(s1) / d;
    const float m2 = wave_sum(s2) / d;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (act[i]) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (gy[i][j] - m1 - xh[i][j] * m2);
        if (dres) {
          float r[8];
          load8(dres + base + 512 * i, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        store8(dx + base + 512 * i, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (act[i]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sg[wave][(lane + 64 * i) * 8 + j] = acc_g[i][j];
        sb[wave][(lane + 64 * i) * 8 + j] = acc_b[i][j];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < d; c += 256) {
    dg_part[(size_t)blockIdx.x * d + c] = sg[0][c] + sg[1][c] + sg[2][c] + sg[3][c];
    db_part[(size_t)blockIdx.x * d + c] = sb[0][c] + sb[1][c] + sb[2][c] + sb[3][c];
  }
}

__global__ void col_reduce_kernel(const float* __restrict__ part, int nparts,
                                  int d, bf16_t* __restrict__ out_bf,
                                  float* __restrict__ out_f) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d) return;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(size_t)p * d + c];
  if (out_bf) out_bf[c] = f2bf(s);
  if (out_f) out_f[c] = s;
}

// Same reduction for d % 64 == 0, parallel over parts: a workgroup owns 64
// columns; 16 row groups x 16 float4 column lanes each sum a strided subset of
// the parts, then one LDS pass combines the 16 groups. (The one-thread-per-
// column form above runs d/256 workgroups that each walk all parts serially:
// 16 workgroups and ~160 us at d = 4096; this form is bandwidth-bound.)
__global__ void __launch_bounds__(256) col_reduce64_kernel(const float* __restrict__ part, int nparts, int d,
                                                           bf16_t* __restrict__ out_bf,
                                                           float* __restrict__ out_f) {
  __shared__ float4 red[16][16];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + cl * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
  for (int p = rg; p < nparts; p += 16) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)p * d + c);
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
      uint2 w;
      w.x = pack_bf16x2(s.x, s.y);
      w.y = pack_bf16x2(s.z, s.w);
      *reinterpret_cast<uint2*>(out_bf + c) = w;
    }
    if (out_f) *reinterpret_cast<float4*>(out_f + c) = s;
  }
}

static void col_reduce(const float* part, int nparts, int d, bf16_t* out_bf, float* out_f,
                       hipStream_t stream) {
  if (d % 64 == 0)
    hipLaunchKernelGGL(col_reduce64_kernel, dim3(d / 64), dim3(256), 0, stream, part, nparts, d, out_bf,
                       out_f);
  else
    hipLaunchKernelGGL(col_reduce_kernel, dim3((d + 255) / 256), dim3(256), 0, stream, part, nparts, d,
                       out_bf, out_f);
}

// A/B knob: KCA_LN_BWD_NARROW=0 keeps the block kernel for narrow rows (read once)
static bool narrow_bwd_enabled() {
  static const bool on = [] {
    const char* e = getenv("KCA_LN_BWD_NARROW");
    return !(e && e[0] == '0');
  }();
  return on;
}

static void ln_geometry(int d, int& nv, int& threads) {
  const int nvec = d / 8;
  nv = (nvec + 255) / 256;
  if (nv < 1) nv = 1;
  threads = ((nvec + nv - 1) / nv + 63) / 64 * 64;
  if (threads > 256) threads = 256;
}

#define LN_DISPATCH(NVV, ...)                      \
  switch (NVV) {                                   \
    case 1: { constexpr int NV = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int NV = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int NV = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int NV = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int NV = 5; __VA_ARGS__; } break; \
    case 6: { constexpr int NV = 6; __VA_ARGS__; } break; \
    case 7: { constexpr int NV = 7; __VA_ARGS__; } break; \
    case 8: { constexpr int NV = 8; __VA_ARGS__; } break; \
    default: return 2;                             \
  }

// Returns 0 on success, 1 if d is not a multiple of 8, 2 if d > 16384.
KCA_API int kca_layernorm_fwd(const void* x, const void* r1, const void* r2,
                              void* h_out, const void* gamma, const void* beta,
                              void* y, float* mean, float* rstd, int rows,
                              int d, float eps, hipStream_t stream) {
  if (d % 8) return 1;
  int nv, threads;
  ln_geometry(d, nv, threads);
  const int grid = rows < 65535 * 4 ? rows : 65535 * 4;
  LN_DISPATCH(nv, hipLaunchKernelGGL((ln_fwd_kernel<NV>), dim3(grid),
                                     dim3(threads), 0, stream,
                                     (const bf16_t*)x, (const bf16_t*)r1,
                                     (const bf16_t*)r2, (bf16_t*)h_out,
                                     (const bf16_t*)gamma, (const bf16_t*)beta,
                                     (bf16_t*)y, mean, rstd, rows, d, eps));
  return 0;
}

// workspace: 2 * nparts * d floats, nparts = kca_layernorm_bwd_parts(rows).
KCA_API int kca_layernorm_bwd_parts(int rows) {
  // 1024 workgroups (4 per CU) keep more rows' loads in flight than 512 did; the partials grow to
  // 2 x 1024 x d floats (32 MB at d = 4096), reduced by col_reduce
  return rows < 1024 ? (rows > 0 ? rows : 1) : 1024;
}

KCA_API int kca_layernorm_bwd(const void* dy, const void* h, const float* mean,
                              const float* rstd, const void* gamma,
                              const void* dres, void* dx, void* dgamma,
                              void* dbeta, int params_fp32, float* workspace,
                              int rows, int d, hipStream_t stream) {
  if (d % 8) return 1;
  int nv, threads;
  ln_geometry(d, nv, threads);
  const int parts = kca_layernorm_bwd_parts(rows);
  float* dgp = workspace;
  float* dbp = workspace + (size_t)parts * d;
  if (d <= 1024 && narrow_bwd_enabled()) {
    if (d <= 512)
      hipLaunchKernelGGL((ln_bwd_narrow_kernel<1>), dim3(parts), dim3(256), 0, stream, (const bf16_t*)dy,
                         (const bf16_t*)h, mean, rstd, (const bf16_t*)gamma, (const bf16_t*)dres, (bf16_t*)dx,
                         dgp, dbp, rows, d);
    else
      hipLaunchKernelGGL((ln_bwd_narrow_kernel<2>), dim3(parts), dim3(256), 0, stream, (const bf16_t*)dy,
                         (const bf16_t*)h, mean, rstd, (const bf16_t*)gamma, (const bf16_t*)dres, (bf16_t*)dx,
                         dgp, dbp, rows, d);
  } else {
  LN_DISPATCH(nv, hipLaunchKernelGGL((ln_bwd_kernel<NV>), dim3(parts),
                                     dim3(threads), 0, stream,
                                     (const bf16_t*)dy, (const bf16_t*)h, mean,
                                     rstd, (const bf16_t*)gamma,
                                     (const bf16_t*)dres, (bf16_t*)dx, dgp, dbp,
                                     rows, d));
  }
  col_reduce(dgp, parts, d, params_fp32 ? nullptr : (bf16_t*)dgamma,
             params_fp32 ? (float*)dgamma : nullptr, stream);
  if (dbeta)
    col_reduce(dbp, parts, d, params_fp32 ? nullptr : (bf16_t*)dbeta,
               params_fp32 ? (float*)dbeta : nullptr, stream);
  return 0;
}
