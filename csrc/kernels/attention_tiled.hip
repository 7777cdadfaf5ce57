// Flash attention forward, full-tile fast path for head_dim 128 / 256 (K2).
//
// The generic kernels in attention.hip handle every shape (ALiBi, per-batch
// key lengths, ragged tiles, padded head dims). This file holds the path the
// GPT-J / NeoX-class training step actually runs -- causal or not, Sq % 128 ==
// 0, Sk % 32 == 0, d == D -- written around one rule: no per-tile address
// arithmetic and no guards inside the key loop.
//
// LDS image (cdna_hip_programming.md §5.5 T10, image (a)): a tile of 32 rows x
// D bf16 is stored as 8-row x 32-column sub-tiles of 512 B,
//   byte(row, ch) = (row>>3)*16*D + 512*(ch>>2) + 64*(row&7)
//                   + 16*((ch&3) ^ ((row>>2)&3))          (ch = 16-B chunk),
// which is bank-conflict free for both the ds_read_b128 K-row reads of the
// S^T = K.Q^T product and the ds_read_b64_tr_b16 V^T reads of O^T += V^T.P^T,
// and -- because the XOR only touches the two low chunk bits -- every read of
// a tile is one of 2 (K) / 2 (V) per-lane bases plus a compile-time offset.
//
// Per wave: 32 query rows, Q fragments and the O^T accumulator (D/32 x 32x32
// f32 tiles) resident; 32-key tiles double buffered in LDS with the next
// tile's global loads in flight under the current tile's MFMAs (T14); online
// softmax lane-local (query on the lane), max/row-sum in exp2 units with the
// scale folded into one FMA, deferred rescale (T13, threshold 8).
#include "common.h"

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThr = 8.0f;

struct FastFwdParams {
  const bf16_t* q; const bf16_t* k; const bf16_t* v;
  bf16_t* o; float* lse;
  long long q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh;
  long long o_sb, o_st, o_sh;
  int B, Sq, Sk, H, Hkv;
  float scale;
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x4 lds_tr4(const char* base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4_t*)(reinterpret_cast<uintptr_t>(base + byte_off)));
}

__device__ __forceinline__ bf16x8 lds_b128(const char* base, int byte_off) {
  return *reinterpret_cast<const bf16x8*>(base + byte_off);
}

// byte offset of 16-B chunk `ch` of row `row` in a [32][D] image (see header)
template <int D>
__device__ __forceinline__ int img_off(int row, int ch) {
  return (row >> 3) * 16 * D + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return pack_bf16x2(lo, hi);
}

template <int CPT, int RPI>
__device__ __forceinline__ void stage_load(u32x4 (&sk)[CPT], u32x4 (&sv)[CPT], const bf16_t* kst,
                                           const bf16_t* vst, int k0, long long k_st, long long v_st) {
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    sk[i] = *reinterpret_cast<const u32x4*>(kst + (long long)(k0 + i * RPI) * k_st);
    sv[i] = *reinterpret_cast<const u32x4*>(vst + (long long)(k0 + i * RPI) * v_st);
  }
}

// K image at `buf`, V image at buf + tile bytes; chunk i of this thread is
// (row0 + i*RPI, ch) -- the XOR term depends on the row, so each i gets its
// own offset (folded by the compiler to a few adds).
template <int CPT, int RPI, int D>
__device__ __forceinline__ void stage_store(const u32x4 (&sk)[CPT], const u32x4 (&sv)[CPT], char* buf,
                                            int row0, int ch) {
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int o = img_off<D>(row0 + i * RPI, ch);
    *reinterpret_cast<u32x4*>(buf + o) = sk[i];
    *reinterpret_cast<u32x4*>(buf + 32 * D * 2 + o) = sv[i];
  }
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, (D <= 128 ? 2 : 1)) attn_fwd_tiled_kernel(FastFwdParams p) {
  constexpr int BM = 128, BN = 32;
  constexpr int TILE = BN * D * 2;           // bytes per K or V tile
  constexpr int NCH = D / 8;                 // 16-B chunks per row
  constexpr int CPT = BN * NCH / 256;        // chunks per thread per tile
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // [buf][K|V]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15;
  const int nqb = p.Sq / BM;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int bh = lid / nqb;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hkv);
  const int off = p.Sk - p.Sq;
  const int q0 = qb * BM + wave * 32;
  const int qrow = q0 + l32;
  int kv_hi = p.Sk;
  if (CAUSAL) kv_hi = min(kv_hi, qb * BM + BM + off);
  const int ntiles = kv_hi > 0 ? (kv_hi + BN - 1) / BN : 0;
  const float sl2 = p.scale * kLog2e;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;

  // Q^T fragments (B operand of S^T = K.Q^T): lane (q = l32, half hh) holds
  // Q[q][16s + 8hh .. +7].
  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(qp + (long long)qrow * p.q_st + 16 * s + 8 * hh);

  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m = -INFINITY, lsum = 0.f;

  // staging: thread handles chunks idx = tid + i*256 -> row = tid/NCH + i*RPI,
  // ch = tid % NCH (256 % NCH == 0)
  constexpr int RPI = 256 / NCH;
  const int st_row = tid / NCH, st_ch = tid % NCH;
  const bf16_t* kst = kp + (long long)st_row * p.k_st + st_ch * 8;
  const bf16_t* vst = vp + (long long)st_row * p.v_st + st_ch * 8;
  u32x4 sk[CPT], sv[CPT];

  // per-lane read bases (bytes)
  const int xr = (l32 >> 2) & 3;
  const int kb_e = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * (hh ^ xr);        // s even
  const int kb_o = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * ((2 + hh) ^ xr);  // s odd
  const int c3 = 2 * ((lane >> 4) & 1) + ((gi & 3) >> 1);
  const int vb_1 = 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh) + 8 * (gi & 1);
  const int vb_2 = 16 * D + 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh ^ 2) + 8 * (gi & 1);

  // ntiles >= 1 on this path (Sk >= 32; causal: Sk >= Sq)
  stage_load<CPT, RPI>(sk, sv, kst, vst, 0, p.k_st, p.v_st);
  stage_store<CPT, RPI, D>(sk, sv, smem, st_row, st_ch);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int k0 = t * BN;
    const char* Ks = smem + (t & 1) * 2 * TILE;
    const char* Vs = Ks + TILE;
    // the last iteration re-loads its own tile (in bounds, never stored)
    stage_load<CPT, RPI>(sk, sv, kst, vst, min(k0 + BN, (ntiles - 1) * BN), p.k_st, p.v_st);
    // Keep the staging loads above and the LDS stores below on their own sides
    // of the MFMAs: without the fences the compiler merges the two `t + 1 <
    // ntiles` blocks and stores each load to LDS right after it (vmcnt(0)).
    asm volatile("" ::: "memory");
    const bool active = !CAUSAL || (k0 <= q0 + 31 + off);
    if (active) {
      f32x16 sacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        const bf16x8 a = lds_b128(Ks, ((s & 1) ? kb_o : kb_e) + 512 * (s >> 1));
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], sacc, 0, 0, 0);
      }
      // sacc[r] = S[key = k0 + (r&3) + 8(r>>2) + 4hh][q = qrow] (raw dot products)
      if (CAUSAL && (k0 + 31 > q0 + off)) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (key > qrow + off) sacc[r] = -INFINITY;
        }
      }
      float mt = sacc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mt = fmaxf(mt, sacc[r]);
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * sl2;
      if (!__all(mt <= m + kRescaleThr)) {
        const float mnew = fmaxf(m, mt);
        const float alpha = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m - mnew);
        lsum *= alpha;
        // one 32x32 tile at a time: the accumulators live in AGPRs and a
        // whole-O rescale in flight would need D*4/64 extra VGPRs
#pragma unroll
        for (int i = 0; i < D / 32; ++i) {
          oacc[i] *= alpha;
          __builtin_amdgcn_sched_barrier(0);
        }
        m = mnew;
      }
      const float nm = (m == -INFINITY) ? 0.f : -m;
      float ps = 0.f;
      bf16x8 pf0, pf1;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float e0 = __builtin_amdgcn_exp2f(fmaf(sacc[r], sl2, nm));
        const float e1 = __builtin_amdgcn_exp2f(fmaf(sacc[r + 8], sl2, nm));
        ps += e0 + e1;
        pf0[r] = (__bf16)e0;
        pf1[r] = (__bf16)e1;
      }
      lsum += ps;
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int o1 = vb_1 + 2 * s * 16 * D + 512 * db;
          const int o2 = vb_2 + 2 * s * 16 * D + 512 * db;
          const bf16x8 a = cat8(lds_tr4(Vs, o1), lds_tr4(Vs, o2));
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, s ? pf1 : pf0, oacc[db], 0, 0, 0);
        }
      }
    }
    asm volatile("" ::: "memory");
    if (t + 1 < ntiles) stage_store<CPT, RPI, D>(sk, sv, smem + ((t + 1) & 1) * 2 * TILE, st_row, st_ch);
    __syncthreads();
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
  if (hh == 0 && p.lse)
    p.lse[((long long)b * p.H + h) * p.Sq + qrow] = ltot > 0.f ? (m + log2f(ltot)) * kLn2 : INFINITY;
  bf16_t* op = p.o + b * p.o_sb + h * p.o_sh + (long long)qrow * p.o_st;
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 w;
      w.x = pk_bf16(oacc[db][4 * g] * inv, oacc[db][4 * g + 1] * inv);
      w.y = pk_bf16(oacc[db][4 * g + 2] * inv, oacc[db][4 * g + 3] * inv);
      *reinterpret_cast<uint2*>(op + db * 32 + 8 * g + 4 * hh) = w;
    }
  }
}

}  // namespace

// Returns 0 when launched, 1 when the shape is outside the fast path (the
// caller then uses the generic kernel).
KCA_API int kca_attn_fwd_tiled(const void* q, const void* k, const void* v, void* o, float* lse,
                               long long q_sb, long long q_st, long long q_sh, long long k_sb,
                               long long k_st, long long k_sh, long long v_sb, long long v_st,
                               long long v_sh, long long o_sb, long long o_st, long long o_sh,
                               int B, int Sq, int Sk, int H, int Hkv, int d, int causal,
                               float scale, hipStream_t stream) {
  if ((d != 128 && d != 256) || Sq % 128 || Sk % 32 || Sq <= 0 || H % Hkv) return 1;
  if (causal && Sk < Sq) return 1;
  FastFwdParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse,
                  q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh,
                  B, Sq, Sk, H, Hkv, scale};
  dim3 grid((Sq / 128) * B * H);
  if (d == 256) {
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<256, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<256, false>), grid, dim3(256), 0, stream, p);
  } else {
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<128, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<128, false>), grid, dim3(256), 0, stream, p);
  }
  return 0;
}
