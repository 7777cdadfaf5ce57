// Skinny GEMM for decode: y[M, N] = act(x[M, K] . W[N, K]^T + b), M <= 16.
//
// Decode GEMMs are weight-streaming bound (BLOOM-176B TP=8: ~44 GB of weights
// per token per GPU; GPT-J: 12 GB), so the kernel is built to read W exactly
// once at HBM speed: every lane streams 16-byte chunks of R weight rows with
// 4 K-steps unrolled (R*4 independent 16 B loads in flight per lane), the M
// activation rows are staged once per workgroup in LDS (K-chunked so M*Kc
// fits in 64 KB) and read with conflict-free ds_read_b128, fp32 accumulation,
// one wave-reduction per (row, m) at the end. Bias and GELU (tanh or erf) are
// fused into the store, replacing the separate bias/GELU kernels of the
// FT / DS-Inference decoders (SURVEY K1/K5 decode shapes).
#include "gemv_m1.h"  // LnArgs, ld_w16 (shared with decode.hip's fused decode-layer kernels)

// LayerNorm prologue: every workgroup normalises the M activation rows itself
// (K*M*2 B of L2-resident reads, ~1 us) straight into the LDS tile the GEMM
// consumes, so the decode step needs no separate LN launch nor the HBM round
// trip of the normalised row. Statistics match ln_fwd_kernel (two-pass, fp32,
// over the bf16-rounded residual sum).
template <int M>
__device__ __forceinline__ void ln_prologue(const bf16_t* __restrict__ x, long long ldx, const LnArgs& a,
                                            bf16_t* xs, int K, int mv, float* red) {
  const int tid = threadIdx.x;
  for (int m = 0; m < M; ++m) {
    bf16_t* row = xs + m * K;
    if (m >= mv) {
      for (int k = tid * 8; k < K; k += 256 * 8) *reinterpret_cast<uint4*>(row + k) = make_uint4(0u, 0u, 0u, 0u);
      continue;
    }
    float s = 0.f;
    for (int k = tid * 8; k < K; k += 256 * 8) {
      float v[8], t[8];
      load8(x + m * ldx + k, v);
      if (a.r1) {
        load8(a.r1 + m * a.ldh + k, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += t[j];
      }
      if (a.r2) {
        load8(a.r2 + m * a.ldh + k, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += t[j];
      }
      store8(row + k, v);  // bf16-rounded residual sum
      if (a.h_out && blockIdx.x == 0) store8(a.h_out + m * a.ldh + k, v);
      load8(row + k, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    const float mean = block_sum(s, red) / K;
    float q = 0.f;
    for (int k = tid * 8; k < K; k += 256 * 8) {
      float v[8];
      load8(row + k, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) q += (v[j] - mean) * (v[j] - mean);
    }
    const float rstd = rsqrtf(block_sum(q, red + 8) / K + a.eps);
    for (int k = tid * 8; k < K; k += 256 * 8) {
      float v[8], g[8], b[8];
      load8(row + k, v);
      load8(a.gamma + k, g);
      if (a.beta) load8(a.beta + k, b);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (v[j] - mean) * rstd * g[j] + b[j];
      store8(row + k, v);
      if (a.xn_out && blockIdx.x == 0) store8(a.xn_out + m * K + k, v);
    }
  }
}

template <int M, int R, bool LN>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(
    const bf16_t* __restrict__ x, long long ldx, const bf16_t* __restrict__ w,
    const bf16_t* __restrict__ bias, bf16_t* __restrict__ y, long long ldy, int N, int K,
    int kc, int act, int mv, LnArgs ln) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];  // [M][kc]
  __shared__ float red[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;
  float acc[R][M];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
  const bf16_t* wr[R];
  bool rv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    rv[r] = n0 + r < N;
    wr[r] = w + (long long)(rv[r] ? n0 + r : 0) * K;
  }
  for (int k0 = 0; k0 < K; k0 += kc) {
    const int kn = min(kc, K - k0);
    __syncthreads();
    if constexpr (LN) {
      ln_prologue<M>(x, ldx, ln, xs, K, mv, red);  // kc == K: one chunk
    } else {
      for (int i = tid * 8; i < M * kn; i += 256 * 8) {
        const int m = i / kn, kk = i % kn;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);  // rows >= mv (padding of M) stay zero
        if (m < mv) v = *reinterpret_cast<const uint4*>(x + m * ldx + k0 + kk);
        *reinterpret_cast<uint4*>(xs + m * kc + kk) = v;
      }
    }
    __syncthreads();
    // 4 K-steps of 512 elements per iteration: R*4 independent 16 B loads per lane
    for (int kb = lane * 8; kb < kn; kb += 4 * 512) {
      uint4 wv[4][R];  // raw bf16 (4 VGPRs per 8 weights), widened at use
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + u * 512;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          wv[u][r] = make_uint4(0u, 0u, 0u, 0u);
          if (k < kn && rv[r]) wv[u][r] = ld_w16(wr[r] + k0 + k);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = kb + u * 512;
        if (k < kn) {
#pragma unroll
          for (int m = 0; m < M; ++m) {
            float xv[8];
            load8(xs + m * kc + k, xv);
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const uint32_t q[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                acc[r][m] = fmaf(__uint_as_float(q[j] << 16), xv[2 * j], acc[r][m]);
                acc[r][m] = fmaf(__uint_as_float(q[j] & 0xffff0000u), xv[2 * j + 1], acc[r][m]);
              }
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = wave_sum(acc[r][m]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!rv[r]) continue;
      const float b = bias ? bf2f(bias[n0 + r]) : 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        if (m >= mv) break;
        float v = acc[r][m] + b;
        if (act == 1) v = gelu_tanh(v);
        else if (act == 2) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        y[m * ldy + n0 + r] = f2bf(v);
      }
    }
  }
}

// Split-K form for M == 1 (single-sequence decode, the latency case): a
// workgroup owns R weight rows; lane (wave w, lane l) owns K positions
// i*2048 + w*512 + l*8 (i = 0, 1, ...) of every row, so its slice of the
// activation row is a handful of 16-B loads straight into registers -- no
// LDS stage and no barrier in front of the weight stream. Weights for the
// first U slabs are requested first; with a LayerNorm prologue (K <= 8192,
// the lane's whole slice in registers) the residual sum, the two block
// reductions and the normalisation all run while those loads are in flight.
// Per-lane loads: R*U weights + U activations, 16 B each. The 4 waves' partial
// dots meet in LDS. (Was: every workgroup staged / normalised the full row
// into LDS before its first weight load -- the LN form streamed 3.3 TB/s
// against 5.2 TB/s for the plain one at GPT-J shapes.)
// MR > 1 (decode batch 2..4, no LN prologue): the same K-split structure over MR activation rows
// held in registers -- W still streamed once, MR FMAs per weight element
template <int R, bool LN, int MR = 1, int DT = 0>
__global__ __launch_bounds__(256) void gemv1_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                    const bf16_t* __restrict__ bias, bf16_t* __restrict__ y,
                                                    int N, int K, int act, LnArgs ln, long long ldx = 0,
                                                    long long ldy = 0, int mv = 1) {
  static_assert(MR == 1 || !LN, "the LN prologue is single-row");
  constexpr int U = 4;
  __shared__ float red[16];
  __shared__ float part[4][R * MR];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = blockIdx.x * R;
  const int kl = wid * 512 + lane * 8;
  const bf16_t* wr[R];
  bool rv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    rv[r] = n0 + r < N;
    wr[r] = w + (long long)(rv[r] ? n0 + r : 0) * K;
  }
  float acc[MR][R];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;
  uint4 wv[U][R];
  auto load_w = [&](int i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (i0 + u) * 2048 + kl;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        wv[u][r] = make_uint4(0u, 0u, 0u, 0u);
        if (k < K && rv[r]) wv[u][r] = ld_w16(wr[r] + k);
      }
    }
  };
  auto fma_w = [&](int i0, const float (&xv)[U][8]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if ((i0 + u) * 2048 + kl >= K) continue;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t q[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[0][r] = fmaf(lo2f<DT>(q[j]), xv[u][2 * j], acc[0][r]);
          acc[0][r] = fmaf(hi2f<DT>(q[j]), xv[u][2 * j + 1], acc[0][r]);
        }
      }
    }
  };
  load_w(0);
  if constexpr (LN) {
    float xv[U][8];  // K <= 8192 = U * 2048: the lane's whole slice
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = u * 2048 + kl;
      if (k < K) {
        float t[8];
        load8_t<DT>(x + k, xv[u]);
        if (ln.r1) {
          load8_t<DT>(ln.r1 + k, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[u][j] += t[j];
        }
        if (ln.r2) {
          load8_t<DT>(ln.r2 + k, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[u][j] += t[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[u][j] = e2f<DT>(f2e<DT>(xv[u][j]));  // statistics over the rounded residual sum
          s += xv[u][j];
        }
        if (ln.h_out && blockIdx.x == 0) store8_t<DT>(ln.h_out + k, xv[u]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[u][j] = 0.f;
      }
    }
    const float mean = block_sum(s, red) / K;
    float q = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u * 2048 + kl >= K) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) q += (xv[u][j] - mean) * (xv[u][j] - mean);
    }
    const float rstd = rsqrtf(block_sum(q, red + 8) / K + ln.eps);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = u * 2048 + kl;
      if (k >= K) continue;
      float g[8], bb[8];
      load8_t<DT>(ln.gamma + k, g);
      if (ln.beta) load8_t<DT>(ln.beta + k, bb);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[u][j] = e2f<DT>(f2e<DT>((xv[u][j] - mean) * rstd * g[j] + bb[j]));
      if (ln.xn_out && blockIdx.x == 0) store8_t<DT>(ln.xn_out + k, xv[u]);
    }
    fma_w(0, xv);
  } else {
    const int NI = (K + 2047) / 2048;
    for (int i0 = 0; i0 < NI; i0 += U) {
      if (i0) load_w(i0);
      uint4 xr[MR][U];  // raw bf16, widened at use (keeps the MR = 1 kernel at 4 waves/SIMD)
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = (i0 + u) * 2048 + kl;
          xr[m][u] = make_uint4(0u, 0u, 0u, 0u);
          if (k < K && m < mv) xr[m][u] = *reinterpret_cast<const uint4*>(x + m * ldx + k);
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if ((i0 + u) * 2048 + kl >= K) continue;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t q[4] = {wv[u][r].x, wv[u][r].y, wv[u][r].z, wv[u][r].w};
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            const uint32_t xq[4] = {xr[m][u].x, xr[m][u].y, xr[m][u].z, xr[m][u].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[m][r] = dot2_acc<DT>(q[j], xq[j], acc[m][r]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = wave_sum(acc[m][r]);
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r) part[wid][m * R + r] = acc[m][r];
  }
  __syncthreads();
  const int m = tid / R, r = tid % R;
  if (tid < R * MR && m < mv && n0 + r < N) {
    const int i = m * R + r;
    float v = part[0][i] + part[1][i] + part[2][i] + part[3][i];
    v += bias ? e2f<DT>(bias[n0 + r]) : 0.f;
    if (act == 1) v = gelu_tanh(v);
    else if (act == 2) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    y[m * ldy + n0 + r] = (bf16_t)f2e<DT>(v);
  }
}

// Decode LayerNorm of a few rows (one workgroup per row, the row in
// registers): h = x (+ r1) (+ r2) -> h_out (bf16), xn = LN(h) -> xn_out. All
// five operand streams are requested in one round, then two block
// reductions -- the M = 1 decode step normalises once here and streams the
// weights with the plain gemv1 kernel (ops/gemv.py:_LN_SPLIT_M1).
// EmbedSrc (kca_embed_ln_rows): row m of x is embedding row id = chain[m] >= 0 ? prev[chain[m]] :
// tokens[m] (clamped to [0, V)): the decode step's first kernel gathers the token embedding, takes a
// chained token straight from the previous step's sampled ids on the device, and normalises it.
struct EmbedSrc {
  const long long* tokens;
  const int* chain;       // nullable
  const long long* prev;  // the previous step's sampled ids (with chain)
  int V;
};

template <int PER, bool GATHER = false, int DT = 0>
__global__ __launch_bounds__(256) void ln_rows_kernel(const bf16_t* __restrict__ x, long long ldx, LnArgs a,
                                                      int K, EmbedSrc es = EmbedSrc{}) {
  __shared__ float red[16];
  const int tid = threadIdx.x, m = blockIdx.x;
  if constexpr (GATHER) {
    const int c = es.chain ? es.chain[m] : -1;
    long long id = c >= 0 ? es.prev[c] : es.tokens[m];
    id = id < 0 ? 0 : (id >= es.V ? es.V - 1 : id);
    x += (id - m) * ldx;  // the row reads below index x + m * ldx
  }
  // gamma / beta requested with the row: they are independent of the statistics, so the
  // kernel pays one memory round trip instead of two
  U16x8 gr[PER], br[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k < K) {
      gr[i] = *reinterpret_cast<const U16x8*>(a.gamma + k);
      if (a.beta) br[i] = *reinterpret_cast<const U16x8*>(a.beta + k);
    }
  }
  float v[PER][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k < K) {
      float t[8];
      load8_t<DT>(x + m * ldx + k, v[i]);
      if (a.r1) {
        load8_t<DT>(a.r1 + m * a.ldh + k, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += t[j];
      }
      if (a.r2) {
        load8_t<DT>(a.r2 + m * a.ldh + k, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += t[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = e2f<DT>(f2e<DT>(v[i][j]));
        s += v[i][j];
      }
      if (a.h_out) store8_t<DT>(a.h_out + m * a.ldh + k, v[i]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = block_sum(s, red) / K;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if ((i * 256 + tid) * 8 >= K) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) q += (v[i][j] - mean) * (v[i][j] - mean);
  }
  const float rstd = rsqrtf(block_sum(q, red + 8) / K + a.eps);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = (i * 256 + tid) * 8;
    if (k >= K) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[i][j] = (v[i][j] - mean) * rstd * e2f<DT>(gr[i].v[j]) + (a.beta ? e2f<DT>(br[i].v[j]) : 0.f);
    store8_t<DT>(a.xn_out + (long long)m * K + k, v[i]);
  }
}

KCA_API int kca_ln_rows(const void* x, long long ldx, const void* r1, const void* r2, void* h_out, long long ldh,
                        const void* gamma, const void* beta, float eps, void* xn_out, int M, int K,
                        hipStream_t stream) {
  if (M < 1 || K % 8 || K > 16384 || ldx % 8 || ldh % 8 || !xn_out) return 1;
  if (((uintptr_t)x | (uintptr_t)r1 | (uintptr_t)r2 | (uintptr_t)h_out | (uintptr_t)gamma | (uintptr_t)beta |
       (uintptr_t)xn_out) & 15) return 2;
  LnArgs a{(const bf16_t*)r1, (const bf16_t*)r2, (bf16_t*)h_out, ldh, (const bf16_t*)gamma, (const bf16_t*)beta,
           eps, (bf16_t*)xn_out};
  const int per = (K + 2047) / 2048;
  if (per <= 2) hipLaunchKernelGGL((ln_rows_kernel<2>), dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, a, K);
  else if (per <= 4) hipLaunchKernelGGL((ln_rows_kernel<4>), dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, a, K);
  else hipLaunchKernelGGL((ln_rows_kernel<8>), dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, a, K);
  return 0;
}

// h_out[m] = wte[id_m] (bf16), xn_out[m] = LN(h_out[m]); id_m from tokens / chain / prev (EmbedSrc).
KCA_API int kca_embed_ln_rows(const void* wte, long long ldw, const long long* tokens, const int* chain,
                              const long long* prev, int V, void* h_out, long long ldh, const void* gamma,
                              const void* beta, float eps, void* xn_out, int M, int K, hipStream_t stream) {
  if (M < 1 || K % 8 || K > 16384 || ldw % 8 || ldh % 8 || !xn_out || !h_out || !tokens || V < 1) return 1;
  if (chain && !prev) return 1;
  if (((uintptr_t)wte | (uintptr_t)h_out | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)xn_out) & 15) return 2;
  LnArgs a{nullptr, nullptr, (bf16_t*)h_out, ldh, (const bf16_t*)gamma, (const bf16_t*)beta, eps, (bf16_t*)xn_out};
  EmbedSrc es{tokens, chain, prev, V};
  const int per = (K + 2047) / 2048;
  if (per <= 2)
    hipLaunchKernelGGL((ln_rows_kernel<2, true>), dim3(M), dim3(256), 0, stream, (const bf16_t*)wte, ldw, a, K, es);
  else if (per <= 4)
    hipLaunchKernelGGL((ln_rows_kernel<4, true>), dim3(M), dim3(256), 0, stream, (const bf16_t*)wte, ldw, a, K, es);
  else
    hipLaunchKernelGGL((ln_rows_kernel<8, true>), dim3(M), dim3(256), 0, stream, (const bf16_t*)wte, ldw, a, K, es);
  return 0;
}

// fp16 rows (FT / DS-Inference serve fp16): kca_ln_rows / kca_embed_ln_rows with fp16 loads and stores
KCA_API int kca_ln_rows_f16(const void* x, long long ldx, const void* r1, const void* r2, void* h_out, long long ldh,
                            const void* gamma, const void* beta, float eps, void* xn_out, int M, int K,
                            hipStream_t stream) {
  if (M < 1 || K % 8 || K > 16384 || ldx % 8 || ldh % 8 || !xn_out) return 1;
  if (((uintptr_t)x | (uintptr_t)r1 | (uintptr_t)r2 | (uintptr_t)h_out | (uintptr_t)gamma | (uintptr_t)beta |
       (uintptr_t)xn_out) & 15) return 2;
  LnArgs a{(const bf16_t*)r1, (const bf16_t*)r2, (bf16_t*)h_out, ldh, (const bf16_t*)gamma, (const bf16_t*)beta,
           eps, (bf16_t*)xn_out};
  const int per = (K + 2047) / 2048;
  if (per <= 2)
    hipLaunchKernelGGL((ln_rows_kernel<2, false, 1>), dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, a, K,
                       EmbedSrc{});
  else if (per <= 4)
    hipLaunchKernelGGL((ln_rows_kernel<4, false, 1>), dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, a, K,
                       EmbedSrc{});
  else
    hipLaunchKernelGGL((ln_rows_kernel<8, false, 1>), dim3(M), dim3(256), 0, stream, (const bf16_t*)x, ldx, a, K,
                       EmbedSrc{});
  return 0;
}

KCA_API int kca_embed_ln_rows_f16(const void* wte, long long ldw, const long long* tokens, const int* chain,
                                  const long long* prev, int V, void* h_out, long long ldh, const void* gamma,
                                  const void* beta, float eps, void* xn_out, int M, int K, hipStream_t stream) {
  if (M < 1 || K % 8 || K > 16384 || ldw % 8 || ldh % 8 || !xn_out || !h_out || !tokens || V < 1) return 1;
  if (chain && !prev) return 1;
  if (((uintptr_t)wte | (uintptr_t)h_out | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)xn_out) & 15) return 2;
  LnArgs a{nullptr, nullptr, (bf16_t*)h_out, ldh, (const bf16_t*)gamma, (const bf16_t*)beta, eps, (bf16_t*)xn_out};
  EmbedSrc es{tokens, chain, prev, V};
  const int per = (K + 2047) / 2048;
  if (per <= 2)
    hipLaunchKernelGGL((ln_rows_kernel<2, true, 1>), dim3(M), dim3(256), 0, stream, (const bf16_t*)wte, ldw, a, K, es);
  else if (per <= 4)
    hipLaunchKernelGGL((ln_rows_kernel<4, true, 1>), dim3(M), dim3(256), 0, stream, (const bf16_t*)wte, ldw, a, K, es);
  else
    hipLaunchKernelGGL((ln_rows_kernel<8, true, 1>), dim3(M), dim3(256), 0, stream, (const bf16_t*)wte, ldw, a, K, es);
  return 0;
}

// 1 = split-K kernel for M == 1 (default), 0 = row-per-wave kernel (A/B)
static int g_skinny_sk = 1;
KCA_API int kca_skinny_set_splitk(int on) {
  g_skinny_sk = on ? 1 : 0;
  return 0;
}

// rows per workgroup of the M = 1 GEMV when K <= 2048 (a BLOOM TP=8 out-projection row is 3.5 KB: two
// rows give a workgroup 7 KB of weight and the launch 7168 workgroups) -- A/B knob, 2 / 4 / 8
static int g_gemv_smallk_rows = 2;
KCA_API int kca_skinny_set_smallk(int rows) {
  g_gemv_smallk_rows = (rows == 4 || rows == 8) ? rows : 2;
  return 0;
}

template <int M, bool LN = false>
static void launch_skinny(const bf16_t* x, long long ldx, const bf16_t* w, const bf16_t* bias,
                          bf16_t* y, long long ldy, int mv, int N, int K, int act, hipStream_t s,
                          const LnArgs& ln = LnArgs{}) {
  constexpr int R = (M <= 4) ? 4 : 2;
  int kc = (32768 / M) / 512 * 512;  // M*kc*2 B <= 64 KB of LDS
  if (kc < 512) kc = 512;
  if (kc > K || LN) kc = (K + 7) / 8 * 8;
  // the LN prologue is redone by every workgroup: at BLOOM's K = 14336 the 4x workgroup count of the
  // split-K form costs more than it saves (B=1 8.75 -> 9.47 ms/token), so wide LN rows stay row-per-wave
  if constexpr (M == 1) if (g_skinny_sk && !(LN && K > 8192)) {
    // 2 weight rows per workgroup: twice the workgroups of the 4-row form, a shorter ragged end to
    // each launch (same box: BLOOM TP=8 B=1 9.03 -> 8.97 ms, GPT-J B=1 2.21 -> 2.20 ms;
    // profiles/decode_launch_structure_ab_r5.txt)
    if (!LN && K <= 2048 && g_gemv_smallk_rows == 8) {
      hipLaunchKernelGGL((gemv1_kernel<8, LN>), dim3((N + 7) / 8), dim3(256), 0, s, x, w, bias, y, N, K, act, ln, 0LL,
                         0LL, 1);
      return;
    }
    if (!LN && K <= 2048 && g_gemv_smallk_rows == 4) {
      hipLaunchKernelGGL((gemv1_kernel<4, LN>), dim3((N + 3) / 4), dim3(256), 0, s, x, w, bias, y, N, K, act, ln, 0LL,
                         0LL, 1);
      return;
    }
    constexpr int R1 = 2;
    const dim3 grid((N + R1 - 1) / R1);
    hipLaunchKernelGGL((gemv1_kernel<R1, LN>), grid, dim3(256), 0, s, x, w, bias, y, N, K, act, ln, 0LL, 0LL, 1);
    return;
  }
  // 2 rows without an LN prologue (decode batch 2): the K-split register-resident form, K <= 8192
  // (the lanes' x slices stay in registers). GPT-J B=2 decode 3.41-3.50 -> 3.13-3.16 ms/step vs
  // hipBLASLt; at 4 rows it lost to hipBLASLt (4.1-4.2 vs 3.5-3.6 ms, also with several weight-row
  // groups per workgroup), so 3-4 rows keep the kernel below (profiles/decode_skinny_ab_r2.txt)
  if constexpr (M == 2) if (g_skinny_sk && !LN && K <= 8192) {
    const dim3 grid((N + 3) / 4);
    hipLaunchKernelGGL((gemv1_kernel<4, false, 2>), grid, dim3(256), 0, s, x, w, bias, y, N, K, act, ln, ldx, ldy,
                       mv);
    return;
  }
  const int rows_per_block = 4 * R;
  const dim3 grid((N + rows_per_block - 1) / rows_per_block);
  hipLaunchKernelGGL((skinny_gemm_kernel<M, R, LN>), grid, dim3(256), (size_t)M * kc * sizeof(bf16_t), s,
                     x, ldx, w, bias, y, ldy, N, K, kc, act, mv, ln);
}

KCA_API int kca_skinny_gemm(const void* x, long long ldx, const void* w, const void* bias, void* y,
                            long long ldy, int M, int N, int K, int act, hipStream_t stream) {
  if (M < 1 || M > 16 || K % 8 || ldx % 8 || N < 1) return 1;
  if (((uintptr_t)x | (uintptr_t)w) & 15) return 2;
  const bf16_t* xp = (const bf16_t*)x;
  const bf16_t* wp = (const bf16_t*)w;
  const bf16_t* bp = (const bf16_t*)bias;
  bf16_t* yp = (bf16_t*)y;
  // one launch, M padded up to the next instantiated row count (W is read once)
  if (M == 1) launch_skinny<1>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else if (M == 2) launch_skinny<2>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else if (M <= 4) launch_skinny<4>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else if (M <= 8) launch_skinny<8>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  else launch_skinny<16>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream);
  return 0;
}

// fp16 twin of kca_skinny_gemm for the decode step's single-row projections (the batch-1 fused layer's
// QKV / fc_in / LM head GEMVs): M == 1 only (batch > 1 fp16 decode runs the matrix-core layer,
// skinny_mfma.hip); returns 3 for other M so the caller falls back
KCA_API int kca_skinny_gemm_f16(const void* x, long long ldx, const void* w, const void* bias, void* y,
                                long long ldy, int M, int N, int K, int act, hipStream_t stream) {
  if (M != 1) return 3;
  if (K % 8 || N < 1) return 1;
  if (((uintptr_t)x | (uintptr_t)w) & 15) return 2;
  constexpr int R1 = 2;
  hipLaunchKernelGGL((gemv1_kernel<R1, false, 1, 1>), dim3((N + R1 - 1) / R1), dim3(256), 0, stream,
                     (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)bias, (bf16_t*)y, N, K, act, LnArgs{}, 0LL,
                     0LL, 1);
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

// y = act(LayerNorm(x (+ r1) (+ r2)) . W^T + b); h_out (nullable) receives the
// bf16 residual sum. Needs the whole normalised rows in LDS: M*K <= 32768.
KCA_API int kca_ln_skinny_gemm(const void* x, long long ldx, const void* r1, const void* r2, void* h_out,
                               long long ldh, const void* gamma, const void* beta, float eps, const void* w,
                               const void* bias, void* y, long long ldy, int M, int N, int K, int act,
                               void* xn_out, hipStream_t stream) {
  if (M < 1 || M > 8 || K % 8 || ldx % 8 || ldh % 8 || N < 1) return 1;
  const int Mp = M == 1 ? 1 : M == 2 ? 2 : M <= 4 ? 4 : 8;
  if ((long long)Mp * K > 32768) return 1;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)r1 | (uintptr_t)r2 | (uintptr_t)h_out | (uintptr_t)gamma |
       (uintptr_t)beta | (uintptr_t)xn_out) & 15) return 2;
  LnArgs a{(const bf16_t*)r1, (const bf16_t*)r2, (bf16_t*)h_out, ldh, (const bf16_t*)gamma,
           (const bf16_t*)beta, eps, (bf16_t*)xn_out};
  const bf16_t* xp = (const bf16_t*)x;
  const bf16_t* wp = (const bf16_t*)w;
  const bf16_t* bp = (const bf16_t*)bias;
  bf16_t* yp = (bf16_t*)y;
  if (Mp == 1) launch_skinny<1, true>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream, a);
  else if (Mp == 2) launch_skinny<2, true>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream, a);
  else if (Mp == 4) launch_skinny<4, true>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream, a);
  else launch_skinny<8, true>(xp, ldx, wp, bp, yp, ldy, M, N, K, act, stream, a);
  return 0;
}
