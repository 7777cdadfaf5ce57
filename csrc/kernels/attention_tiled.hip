// Flash attention forward + backward, full-tile fast path for head_dim 64 / 96 / 128 / 160 / 256 (K2).
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

#include <type_traits>

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kRescaleThr = 8.0f;

// Diagnostic build only (-DKCA_ATTN_STAMPS, bench/attn_stamps.py): per-wave s_memtime segment
// sums of the main loops, added into g_attn_stamps once per wave at the end (fwd slots 0..7,
// dQ 16..23, dK/dV 32..39). The fences around each stamp forbid overlaps the real kernel has: read
// the shares, not the lengths. In the normal build every ASTAMP is empty.
#ifdef KCA_ATTN_STAMPS
__device__ unsigned long long g_attn_stamps[64];
__device__ __forceinline__ unsigned long long ast_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define ASTAMP_DECL                                            \
  unsigned long long st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long st_prev_ = ast_now();
#define ASTAMP(k)                           \
  do {                                      \
    const unsigned long long n_ = ast_now(); \
    st_acc_[k] += n_ - st_prev_;            \
    st_prev_ = n_;                          \
  } while (0)
#define ASTAMP_FLUSH(base)                                                          \
  do {                                                                              \
    st_acc_[7] = 1;                                                                 \
    if ((threadIdx.x & 63) == 0)                                                    \
      for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_attn_stamps[(base) + i_], st_acc_[i_]); \
  } while (0)
#else
#define ASTAMP_DECL
#define ASTAMP(k) \
  do {            \
  } while (0)
#define ASTAMP_FLUSH(base) \
  do {                     \
  } while (0)
#endif


struct FastFwdParams {
  const bf16_t* q; const bf16_t* k; const bf16_t* v;
  bf16_t* o; float* lse;
  int* flags;  // [grid * 4]: 1 = this wave's rows overflowed -> fixup kernel
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

// buffer resource over one (batch, head) slice; the base is workgroup-uniform (readfirstlane'd so
// the descriptor is provably scalar: no waterfall loop, T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const bf16_t* b) {
  const unsigned long long a = (unsigned long long)b;
  const unsigned long long au = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(a >> 32)) << 32) |
                                (unsigned)__builtin_amdgcn_readfirstlane((unsigned)a);
  return __builtin_amdgcn_make_buffer_rsrc((void*)au, (short)0, 0x7fffffff, 0x00020000);
}

// Staging of a 32-row x D tile by the 256 threads of a workgroup: chunk idx = tid + 256*i is
// (row idx / NCH, 16-B chunk idx % NCH). D = 96 / 160 serve SD-1.5's 80-wide heads (padded to
// 96) and its 160-wide heads (native) instead of padding them to 128 / 256.
template <int D, bool POW2 = (256 % (D / 8)) == 0>
struct Stager;

// D = 64 / 128 / 256: thread tid owns chunk column tid % NCH of rows tid / NCH + i * RPI.
// Loads go through buffer resources (T8): the per-thread byte offsets are loop constants in
// VGPRs and the tile's row offset k0 * stride is ONE scalar -- no 64-bit address arithmetic on the
// VALU per load, which at D = 64 (SD-1.5's padded heads) is VALU-issue-bound.
template <int D>
struct Stager<D, true> {
  static constexpr int NCH = D / 8, CPT = 32 * NCH / 256, RPI = 256 / NCH;
  long long ok_, ov_;  // element offset of this thread's first chunk in a K / V tile
  int row0_, ch_;
  __amdgpu_buffer_rsrc_t rk_, rv_;
  int vok_[CPT], vov_[CPT];  // byte offsets of this thread's chunks (tile row 0)
  __device__ __forceinline__ Stager(int tid, long long k_st, long long v_st) {
    row0_ = tid / NCH;
    ch_ = tid % NCH;
    ok_ = (long long)row0_ * k_st + ch_ * 8;
    ov_ = (long long)row0_ * v_st + ch_ * 8;
  }
  // kb / vb: the (batch, kv head) base pointers -- workgroup-uniform (readfirstlane'd so the
  // descriptor is provably scalar: no waterfall loop, T20). Offsets stay < 2^31 bytes per head slice.
  __device__ __forceinline__ void bind(const bf16_t* kb, const bf16_t* vb, long long k_st, long long v_st) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      vok_[i] = (int)((ok_ + (long long)i * RPI * k_st) * 2);
      vov_[i] = (int)((ov_ + (long long)i * RPI * v_st) * 2);
    }
    set_base(kb, vb);
  }
  // scalar work only: a kernel whose base changes per tile (dK/dV over GQA query heads) rebinds it
  __device__ __forceinline__ void set_base(const bf16_t* kb, const bf16_t* vb) {
    rk_ = head_rsrc(kb);
    rv_ = head_rsrc(vb);
  }
  __device__ __forceinline__ void load(u32x4 (&sk)[CPT], u32x4 (&sv)[CPT], const bf16_t* kb, const bf16_t* vb,
                                       int k0, long long k_st, long long v_st) const {
    const int sok = __builtin_amdgcn_readfirstlane((int)(k0 * k_st * 2));
    const int sov = __builtin_amdgcn_readfirstlane((int)(k0 * v_st * 2));
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(rk_, vok_[i], sok, 0);
      const auto b = __builtin_amdgcn_raw_buffer_load_b128(rv_, vov_[i], sov, 0);
      sk[i] = *reinterpret_cast<const u32x4*>(&a);
      sv[i] = *reinterpret_cast<const u32x4*>(&b);
    }
  }
  __device__ __forceinline__ void store(const u32x4 (&sk)[CPT], const u32x4 (&sv)[CPT], char* buf) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int o = img_off<D>(row0_ + i * RPI, ch_);
      *reinterpret_cast<u32x4*>(buf + o) = sk[i];
      *reinterpret_cast<u32x4*>(buf + 32 * D * 2 + o) = sv[i];
    }
  }
};

// D = 96 / 160 (NCH 12 / 20): 32 * NCH chunks are not a multiple of 256, so the last i covers
// the first (32 * NCH) % 256 threads (whole waves) and each i has its own (row, chunk), with the
// element offsets precomputed once, outside the key loop
template <int D>
struct Stager<D, false> {
  static constexpr int NCH = D / 8, TOT = 32 * NCH, CPT = (TOT + 255) / 256;
  static_assert(D % 32 == 0 && TOT % 64 == 0, "tiled attention: D multiple of 32");
  long long ok_[CPT], ov_[CPT];
  int lds_[CPT];
  bool tail_;  // this thread owns a chunk in the last, partial round
  __device__ __forceinline__ Stager(int tid, long long k_st, long long v_st) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = min(tid + 256 * i, TOT - 1);
      const int row = idx / NCH, ch = idx % NCH;
      ok_[i] = (long long)row * k_st + ch * 8;
      ov_[i] = (long long)row * v_st + ch * 8;
      lds_[i] = img_off<D>(row, ch);
    }
    tail_ = tid + 256 * (CPT - 1) < TOT;
  }
  __device__ __forceinline__ void bind(const bf16_t*, const bf16_t*, long long, long long) {}
  __device__ __forceinline__ void set_base(const bf16_t*, const bf16_t*) {}
  __device__ __forceinline__ void load(u32x4 (&sk)[CPT], u32x4 (&sv)[CPT], const bf16_t* kb, const bf16_t* vb,
                                       int k0, long long k_st, long long v_st) const {
    const bf16_t* kr = kb + (long long)k0 * k_st;
    const bf16_t* vr = vb + (long long)k0 * v_st;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {  // a clamped tail chunk re-reads a valid chunk (never stored)
      sk[i] = *reinterpret_cast<const u32x4*>(kr + ok_[i]);
      sv[i] = *reinterpret_cast<const u32x4*>(vr + ov_[i]);
    }
  }
  __device__ __forceinline__ void store(const u32x4 (&sk)[CPT], const u32x4 (&sv)[CPT], char* buf) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      if (i < CPT - 1 || tail_) {
        *reinterpret_cast<u32x4*>(buf + lds_[i]) = sk[i];
        *reinterpret_cast<u32x4*>(buf + 32 * D * 2 + lds_[i]) = sv[i];
      }
    }
  }
};

// DS < D ("narrow storage"): heads stored DS wide in memory (SD-1.5's 40-wide heads padded to 48
// instead of 64: 25 % fewer Q/K/V bytes and QKV-GEMM columns, 3 instead of 4 S MFMAs) staged into
// the D-wide LDS image; image chunks DS/8 .. D/8-1 are never loaded (the kernel zeroes V's once).
// 32 * DS/8 chunks per tile: threads below that count own one K and one V chunk, whole waves.
template <int D, int DS>
struct StagerNarrow {
  static constexpr int NCH = DS / 8, TOT = 32 * NCH, CPT = 1;
  static_assert(TOT <= 256 && TOT % 64 == 0, "narrow stager: one chunk per thread, whole waves");
  int vok_[1], vov_[1], lds_;
  bool on_;
  __amdgpu_buffer_rsrc_t rk_, rv_;
  __device__ __forceinline__ StagerNarrow(int tid, long long k_st, long long v_st) {
    const int idx = min(tid, TOT - 1), row = idx / NCH, ch = idx % NCH;
    vok_[0] = (int)(((long long)row * k_st + ch * 8) * 2);
    vov_[0] = (int)(((long long)row * v_st + ch * 8) * 2);
    lds_ = img_off<D>(row, ch);
    on_ = tid < TOT;
  }
  __device__ __forceinline__ void bind(const bf16_t* kb, const bf16_t* vb, long long, long long) { set_base(kb, vb); }
  __device__ __forceinline__ void set_base(const bf16_t* kb, const bf16_t* vb) {
    rk_ = head_rsrc(kb);
    rv_ = head_rsrc(vb);
  }
  __device__ __forceinline__ void load(u32x4 (&sk)[1], u32x4 (&sv)[1], const bf16_t*, const bf16_t*, int k0,
                                       long long k_st, long long v_st) const {
    const int sok = __builtin_amdgcn_readfirstlane((int)(k0 * k_st * 2));
    const int sov = __builtin_amdgcn_readfirstlane((int)(k0 * v_st * 2));
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rk_, vok_[0], sok, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rv_, vov_[0], sov, 0);
    sk[0] = *reinterpret_cast<const u32x4*>(&a);
    sv[0] = *reinterpret_cast<const u32x4*>(&b);
  }
  __device__ __forceinline__ void store(const u32x4 (&sk)[1], const u32x4 (&sv)[1], char* buf) const {
    if (on_) {
      *reinterpret_cast<u32x4*>(buf + lds_) = sk[0];
      *reinterpret_cast<u32x4*>(buf + 32 * D * 2 + lds_) = sv[0];
    }
  }
};

template <int D, int DS>
using StagerFor = std::conditional_t<DS == D, Stager<D>, StagerNarrow<D, DS>>;

// Epilogue through LDS (cdna_hip_programming.md T21): the wave's 32 x D accumulator tile (row =
// lane & 31) goes into a wave-private [32][D] bf16 LDS image -- 16-B chunks rotated by the row,
// so the per-lane 8-B writes and the row-contiguous 16-B reads are both conflict-free -- and every
// store instruction then writes two whole rows with 16-B stores, instead of 8-B stores that each
// touch 64 rows. `mul` is the lane's row scale. The LDS must be free (after the loop's barrier).
template <int D, int DS = D>
__device__ __forceinline__ void store_tile_lds(bf16_t* row0, long long st, const f32x16 (&acc)[D / 32], int lane,
                                               float mul, char* lds) {
  constexpr int NCH = D / 8, RB = D * 2, NCS = DS / 8;  // NCS: stored chunks per row
  const int l32 = lane & 31, hh = lane >> 5;
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 w;
      w.x = pk_bf16(acc[db][4 * g] * mul, acc[db][4 * g + 1] * mul);
      w.y = pk_bf16(acc[db][4 * g + 2] * mul, acc[db][4 * g + 3] * mul);
      *reinterpret_cast<uint2*>(lds + l32 * RB + ((4 * db + g + l32) % NCH) * 16 + hh * 8) = w;
    }
  }
  asm volatile("" ::: "memory");  // the wave's LDS accesses execute in order: reads see its writes
  static_assert((32 * NCS) % 64 == 0, "whole-wave epilogue rounds");
#pragma unroll
  for (int j = 0; j < 32 * NCS / 64; ++j) {
    const int idx = j * 64 + lane, r = idx / NCS, c = idx % NCS;
    const uint4 v = *reinterpret_cast<const uint4*>(lds + r * RB + ((c + r) % NCH) * 16);
    *reinterpret_cast<uint4*>(row0 + (long long)r * st + c * 8) = v;
  }
  asm volatile("" ::: "memory");
}

// OC >= 0 ("ones column"): V's zero-padded column OC holds 1.0 for every key (the SD UNet's
// padded QKV GEMM writes it through its bias), so O^T row OC accumulates the softmax row sum
// sum_k bf16(P) on the matrix pipe: the per-element f32 adds of the row sum leave the VALU, which
// bounds this loop at D = 64 (SD-1.5's 40-wide heads, padded).
// DS < D: heads stored DS wide (StagerNarrow); the contraction over d runs DS / 16 MFMA steps.
// MC >= 0 ("max column", with OC; non-causal): K arrives pre-scaled by scale * log2(e) with its zero-padded
// column MC set to 1.0 (the SD UNet folds both into its padded QKV weights), and the kernel writes
// -m into Q's column MC in registers once m is known, so the S MFMAs return s * log2(e) - m and
// P = exp2(S) needs no per-element FMA: the D <= 64 loop is bound by that VALU work, not the MFMAs.
template <int D, bool CAUSAL, int OC = -1, int DS = D, int MC = -1>
__global__ void __launch_bounds__(256, (D <= 128 ? 2 : 1)) attn_fwd_tiled_kernel(FastFwdParams p) {
  constexpr int BM = 128, BN = 32;
  constexpr int TILE = BN * D * 2;           // bytes per K or V tile (LDS image)
  constexpr int KS = DS / 16;                // S MFMA steps
  using Stg = StagerFor<D, DS>;
  constexpr int CPT = Stg::CPT;             // 16-B chunks per thread per tile
  __shared__ __attribute__((aligned(16))) char smem[3 * 2 * TILE];  // [buf 0..2][K|V]

  ASTAMP_DECL
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
  static_assert(MC < 0 || (!CAUSAL && OC >= 0 && MC < DS), "max column: non-causal, with the row-sum column");
  const float sl2 = MC >= 0 ? 1.f : p.scale * kLog2e;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;

  // Q^T fragments (B operand of S^T = K.Q^T): lane (q = l32, half hh) holds
  // Q[q][16s + 8hh .. +7].
  bf16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(qp + (long long)qrow * p.q_st + 16 * s + 8 * hh);

  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m = 0.f, lsum = 0.f;  // m: reference max (log2 units), set by tile 0

  // staging: thread handles chunks idx = tid + i*256 (Stager)
  Stg stg(tid, p.k_st, p.v_st);
  stg.bind(kp, vp, p.k_st, p.v_st);
  u32x4 sk[CPT], sv[CPT];
  if constexpr (DS < D) {  // V image chunks DS/8.. (read by the PV d-blocks, never loaded): zero once
    constexpr int PC = D / 8 - DS / 8, NZ = 3 * 32 * PC;
    for (int i = tid; i < NZ; i += 256) {
      const int buf = i / (32 * PC), row = (i / PC) % 32, ch = DS / 8 + i % PC;
      *reinterpret_cast<u32x4*>(smem + buf * 2 * TILE + TILE + img_off<D>(row, ch)) = u32x4{0, 0, 0, 0};
    }
  }

  // per-lane read bases (bytes)
  const int xr = (l32 >> 2) & 3;
  const int kb_e = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * (hh ^ xr);        // s even
  const int kb_o = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * ((2 + hh) ^ xr);  // s odd
  const int c3 = 2 * ((lane >> 4) & 1) + ((gi & 3) >> 1);
  const int vb_1 = 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh) + 8 * (gi & 1);
  const int vb_2 = 16 * D + 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh ^ 2) + 8 * (gi & 1);

  // ntiles >= 1 on this path (Sk >= 32; causal: Sk >= Sq)
  // Software pipeline over 32-key tiles, three LDS buffers: while the softmax
  // of tile t runs on the VALU, the S^T MFMAs of tile t+1 run on the matrix
  // pipe (independent instructions the scheduler interleaves, T15), then
  // O^T += V_t^T P_t^T; the global loads of tile t+2 are in flight throughout
  // and land in the buffer tile t-1 vacated (T14).
  auto qk = [&](const char* Ks) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // K fragments two k-steps ahead of their MFMA (pinned: hipcc otherwise waits lgkmcnt(1))
    bf16x8 fa[3];
    fa[0] = lds_b128(Ks, kb_e);
    fa[1] = lds_b128(Ks, kb_o);
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 2 < KS) {
        fa[(s + 2) % 3] = lds_b128(Ks, (((s + 2) & 1) ? kb_o : kb_e) + 512 * ((s + 2) >> 1));
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s % 3], qf[s], acc, 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
    }
    return acc;
  };
  // causal: keys past this lane's query -> -inf. sacc[r] holds key
  // k0 + (r&3) + 8(r>>2) + 4hh of query qrow. Tiles wholly above a wave's rows
  // are masked, not skipped (a skip puts O in a conditional region: spills).
  auto mask = [&](f32x16& acc, int k0) {
    const int lim = qrow + off - k0 - 4 * hh;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if ((r & 3) + 8 * (r >> 2) > lim) acc[r] = -INFINITY;
  };

  stg.load(sk, sv, kp, vp, 0, p.k_st, p.v_st);
  stg.store(sk, sv, smem);
  stg.load(sk, sv, kp, vp, min(BN, (ntiles - 1) * BN), p.k_st, p.v_st);
  stg.store(sk, sv, smem + 2 * TILE);
  // D = 256 (one wave per SIMD, no other wave to cover a load): two tiles of K/V loads in flight
  // in registers; tile 2 goes into set 0 before the loop (stored at the end of iteration 0).
  // GPT-J fwd 0.563 -> 0.535 ms; at D = 160 it measured 3-4 % slower (profiles/attn_stamps_r2.md)
  constexpr bool PF2 = D >= 256;
  u32x4 sk2[CPT], sv2[CPT];
  if constexpr (PF2) stg.load(sk, sv, kp, vp, min(2 * BN, (ntiles - 1) * BN), p.k_st, p.v_st);
  __syncthreads();

  const int nfree = CAUSAL ? ntiles - 4 : ntiles;  // tiles no wave needs masked
  f32x16 sa = qk(smem);
  if (CAUSAL && nfree <= 0) mask(sa, 0);
  {
    // No running max and no O rescale: the reference max m is the row max of
    // the first tile and stays fixed. Floating point is scale invariant, so
    // P = 2^(s - m) only needs to stay finite -- it can exceed 1 when a later
    // key scores higher. Overflow (a later score ~2^100 times the first
    // tile's best) is detected once, from the final row sum, and those rows
    // are recomputed by the generic kernel (kca_attn_fwd_tiled's fixup
    // launch). Keeping every rescale out of the loop keeps the O^T
    // accumulators in AGPRs, touched only by MFMAs (a conditional rescale
    // made hipcc copy all of O to VGPRs and back every tile).
    float mt = sa[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mt = fmaxf(mt, sa[r]);
    m = fmaxf(mt, __shfl_xor(mt, 32, 64)) * sl2;
  }
  if constexpr (MC >= 0) {
    // Q[MC] = -m (bf16: m is rounded so the MFMA's offset and lse agree); tile 0's S, taken
    // before m existed, gets the offset here; tiles >= 1 come out of qk() with it
    m = (float)(__bf16)m;
    if (hh == (MC % 16) / 8) qf[MC / 16][MC % 8] = (__bf16)(-m);
#pragma unroll
    for (int r = 0; r < 16; ++r) sa[r] -= m;
  }
  const float nm = -m;
  ASTAMP(0);

  auto tile_step = [&](int t, auto masked, auto par) {
    constexpr bool MASKED = decltype(masked)::value;
    const char* Vs = smem + (t % 3) * 2 * TILE + TILE;
    const char* Kn = smem + ((t + 1) % 3) * 2 * TILE;
    // PF2: tile t+3 is requested into one register set while the other (tile t+2, requested an
    // iteration ago) is stored at the end of this iteration; set parity = t & 1 = par.
    // Otherwise the loads of tile t+2. (Clamped: the last iterations re-load a tile that is never
    // stored.)
    constexpr bool ODD = PF2 && decltype(par)::value;
    u32x4(&ldk)[CPT] = (PF2 && !ODD) ? sk2 : sk;
    u32x4(&ldv)[CPT] = (PF2 && !ODD) ? sv2 : sv;
    u32x4(&stk)[CPT] = ODD ? sk2 : sk;
    u32x4(&stv)[CPT] = ODD ? sv2 : sv;
    stg.load(ldk, ldv, kp, vp, min((t + (PF2 ? 3 : 2)) * BN, (ntiles - 1) * BN), p.k_st, p.v_st);
    ASTAMP(1);
    // keep the staging loads above and the LDS stores below on their own
    // sides of the MFMAs (without the fences hipcc stores each load right
    // after it, behind a vmcnt(0))
    asm volatile("" ::: "memory");
    f32x16 sb = qk(Kn);  // S of tile t+1 (stale buffer on the last tile: unused)
    if constexpr (MASKED) mask(sa, t * BN);
    float ps = 0.f;
    bf16x8 pf0, pf1;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float e0 = __builtin_amdgcn_exp2f(MC >= 0 ? sa[r] : fmaf(sa[r], sl2, nm));
      const float e1 = __builtin_amdgcn_exp2f(MC >= 0 ? sa[r + 8] : fmaf(sa[r + 8], sl2, nm));
      if constexpr (OC < 0) ps += e0 + e1;
      pf0[r] = (__bf16)e0;
      pf1[r] = (__bf16)e1;
    }
    if constexpr (OC < 0) lsum += ps;
    ASTAMP(2);
    {  // O^T += V^T P^T, V^T fragments one d-block ahead of their MFMAs
      auto vfrag = [&](int db, int s) {
        return cat8(lds_tr4(Vs, vb_1 + 2 * s * 16 * D + 512 * db), lds_tr4(Vs, vb_2 + 2 * s * 16 * D + 512 * db));
      };
      bf16x8 va[2], vb2[2];
      va[0] = vfrag(0, 0);
      vb2[0] = vfrag(0, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        if (db + 1 < D / 32) {
          va[(db + 1) & 1] = vfrag(db + 1, 0);
          vb2[(db + 1) & 1] = vfrag(db + 1, 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        }
        oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[db & 1], pf0, oacc[db], 0, 0, 0);
        oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vb2[db & 1], pf1, oacc[db], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
      }
    }
    ASTAMP(3);
    sa = sb;
    asm volatile("" ::: "memory");
    if (t + 2 < ntiles) stg.store(stk, stv, smem + ((t + 2) % 3) * 2 * TILE);
    __syncthreads();
    ASTAMP(4);
  };
  if constexpr (PF2) {  // register-set parity must follow t: the loops advance two tiles per trip
  int t = 0;
  for (; t + 1 < nfree; t += 2) {
    tile_step(t, std::false_type{}, std::false_type{});
    tile_step(t + 1, std::false_type{}, std::true_type{});
  }
  if (t < nfree) {
    tile_step(t, std::false_type{}, std::false_type{});
    ++t;
    if (t < ntiles) { tile_step(t, std::true_type{}, std::true_type{}); ++t; }
  }
  t = max(t, 0);
  for (; t + 1 < ntiles; t += 2) {
    tile_step(t, std::true_type{}, std::false_type{});
    tile_step(t + 1, std::true_type{}, std::true_type{});
  }
  if (t < ntiles) tile_step(t, std::true_type{}, std::false_type{});
  } else {
  for (int t = 0; t < nfree; ++t) tile_step(t, std::false_type{}, std::false_type{});
  for (int t = max(nfree, 0); t < ntiles; ++t) tile_step(t, std::true_type{}, std::false_type{});
  }

  float ltot;
  if constexpr (OC >= 0) {
    // O^T row OC (d index) of query l32: register r = (OC & 3) + 4 * (OC >> 3) of d-block OC / 32 in
    // the half hh = (OC >> 2) & 1; the other half reads it across
    constexpr int ROW = OC % 32, RR = (ROW & 3) + 4 * (ROW >> 3), HH = (ROW >> 2) & 1;
    const float mine = oacc[OC / 32][RR];
    const float other = __shfl_xor(mine, 32, 64);
    ltot = hh == HH ? mine : other;
  } else {
    ltot = lsum + __shfl_xor(lsum, 32, 64);
  }
  // row sums past 2^100 (or inf / NaN) mean P may have overflowed: flag the
  // wave for the generic-kernel fixup (which then rewrites O and lse)
  const bool bad = !(ltot < 1.2676506e30f);
  const int any_bad = __any(bad);
  if (lane == 0) p.flags[lid * 4 + wave] = any_bad;
  const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
  if (hh == 0 && p.lse)
    p.lse[((long long)b * p.H + h) * p.Sq + qrow] = ltot > 0.f ? (m + log2f(ltot)) * kLn2 : INFINITY;
  store_tile_lds<D, DS>(p.o + b * p.o_sb + h * p.o_sh + (long long)q0 * p.o_st, p.o_st, oacc, lane, inv,
                        smem + wave * 32 * D * 2);
  ASTAMP(5);
  ASTAMP_FLUSH(0);
}


// ================================================== forward, 8 waves (2 per SIMD), 256 query rows
// The 4-wave kernel above runs one wave per SIMD: every LDS round trip, softmax and K/V tile wait of
// that wave idles its SIMD's matrix pipe (~0.29 MFMA busy at D = 256), and each 32-key tile feeds
// only 128 query rows, so the per-CU K/V stream bounds the loop (profiles/attn_stamps_r2.md). Here a
// workgroup holds 8 waves x 32 query rows = 256 rows: the two waves of a SIMD cover each other's
// stalls, and every staged K/V byte serves twice the MFMA work.
//
// The price is the register file: at two waves per SIMD a wave has 256 registers, and O^T (128),
// the Q^T fragments (D/4 = 64) and one S tile (16) leave no room for register-staged K/V tiles. So
// the tiles arrive by LDS-DMA (buffer_load ... lds: no VGPR destination), four buffers deep, issued
// three tiles ahead, one barrier per tile after a COUNTED vmcnt. hipcc drains every LDS-DMA
// (vmcnt(0)) before any LDS read it can see, so the loop's LDS reads (K rows: ds_read_b128; V^T:
// ds_read_b64_tr_b16) are inline asm with hand-counted lgkmcnt waits, each wait tied to the
// fragment it retires ("+v") so no MFMA can be scheduled above it.
// An LDS-DMA wave-instruction writes 1 KiB at consecutive addresses (lane-linear); the image's
// sub-tile swizzle (img_off) is applied on the per-lane SOURCE address instead.
// Causal: a wave skips the tiles past its own diagonal (its SIMD partner gets the matrix pipe).
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// (the asm bodies exist only in the device pass: the host pass parses this kernel for its launch
// stub and rejects the VGPR constraints)
template <int OFF>
__device__ __forceinline__ u32x4 ads_b128(unsigned addr) {
  u32x4 r;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
#endif
  return r;
}
template <int OFF>
__device__ __forceinline__ u32x2 ads_tr(unsigned addr) {
  u32x2 r;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
#endif
  return r;
}
// s_waitcnt lgkmcnt(N) that the named fragments depend on
template <int N>
__device__ __forceinline__ void lgkm_wait(u32x4& x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(x) : "n"(N));
#endif
}
template <int N>
__device__ __forceinline__ void lgkm_wait(u32x2& x, u32x2& y, u32x2& z, u32x2& w) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "n"(N));
#endif
}
__device__ __forceinline__ bf16x8 as_bf8(u32x4 x) { return *reinterpret_cast<bf16x8*>(&x); }
__device__ __forceinline__ bf16x8 as_bf8(u32x2 lo, u32x2 hi) {
  u32x4 x{lo[0], lo[1], hi[0], hi[1]};
  return *reinterpret_cast<bf16x8*>(&x);
}

// NW = 4, NBUF = 2, D = 512 (non-causal): the VAE mid-block's single 512-wide head (one wave per
// SIMD, O^T = 256 registers, Q^T fragments 128; two 64-KiB stages, the next tile's DMA in flight
// under the current tile). Inference only: the overflow flags go back to the caller, which has no
// generic D = 512 kernel to fix rows up with and reruns flagged calls on the GEMM path.
template <int D, bool CAUSAL, int NW = 8, int NBUF = 4>
__global__ void __launch_bounds__(NW * 64, 1) attn_fwd_w8_kernel(FastFwdParams p) {
  constexpr int BM = NW * 32, BN = 32;
  constexpr int TILE = BN * D * 2;            // one K or V image
  constexpr int STAGE = 2 * TILE;
  constexpr int KS = D / 16;
  constexpr int PIECES = TILE / 1024;         // 1-KiB LDS-DMA pieces per image
  constexpr int PPW = PIECES / NW;            // per wave per image
  constexpr int LEAD = NBUF - 1;                  // tiles issued ahead of the one computed
  constexpr int INFLIGHT = (LEAD - 1) * 2 * PPW;  // DMA instructions issued after tile t when t is waited
  static_assert(((D == 256 || D == 128) && NW == 8) || (D == 512 && NW == 4 && NBUF == 2 && !CAUSAL),
                "multi-wave LDS-DMA forward: 8 waves at D = 128 / 256, 4 waves at D = 512");
  static_assert(PPW >= 1 && PIECES % NW == 0, "whole pieces per wave");
  constexpr int SMEM = (NBUF * STAGE > NW * 32 * D * 2) ? NBUF * STAGE : NW * 32 * D * 2;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];  // [buf][K|V]; epilogue: [wave][32][D]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hh = lane >> 5;
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
  const int ntiles = kv_hi / BN;
  const int mytiles = CAUSAL ? min(ntiles, (q0 + 32 + off) / BN) : ntiles;
  const float sl2 = p.scale * kLog2e;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh;
  bf16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    qf[s] = *reinterpret_cast<const bf16x8*>(qp + (long long)qrow * p.q_st + 16 * s + 8 * hh);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // Q landed before any DMA is counted

  // LDS-DMA sources: piece j of an image covers image bytes [1024 j, 1024 j + 1024); lane L writes
  // byte 1024 j + 16 L, i.e. (row, chunk) = img_off^-1 of it
  const __amdgpu_buffer_rsrc_t rk = head_rsrc(p.k + b * p.k_sb + hk * p.k_sh);
  const __amdgpu_buffer_rsrc_t rv = head_rsrc(p.v + b * p.v_sb + hk * p.v_sh);
  // A wave's PPW pieces lie in one 8-row group (D / 64 pieces per group), piece i of them 2 sub-tiles
  // = 8 chunks = 128 source bytes after piece 0: one per-lane offset, the rest a scalar add
  static_assert((D / 64) % PPW == 0, "a wave's pieces within one row group");
  int kvo, vvo;
  {
    const int byte = 1024 * (wave * PPW) + 16 * lane;
    const int rg = byte / (16 * D), rem = byte % (16 * D);
    const int chh = rem / 512, w5 = rem % 512;
    const int row = rg * 8 + w5 / 64;
    const int ch = chh * 4 + (((w5 % 64) / 16) ^ ((row >> 2) & 3));
    kvo = (int)(((long long)row * p.k_st + ch * 8) * 2);
    vvo = (int)(((long long)row * p.v_st + ch * 8) * 2);
  }
  typedef __attribute__((address_space(3))) char lds_char;
  lds_char* lsm = (lds_char*)smem;
  auto issue = [&](int tile, int buf) {
    const int kt = min(tile, ntiles - 1);  // clamped: the last tiles re-load a tile nobody reads
    const int sok = __builtin_amdgcn_readfirstlane(kt * BN * (int)p.k_st * 2);
    const int sov = __builtin_amdgcn_readfirstlane(kt * BN * (int)p.v_st * 2);
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass drops the launch stub over this builtin)
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (void __attribute__((address_space(3)))*)(
          lsm + buf * STAGE + 1024 * (wave * PPW + i)), 16, kvo, sok + 128 * i, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (void __attribute__((address_space(3)))*)(
          lsm + buf * STAGE + TILE + 1024 * (wave * PPW + i)), 16, vvo, sov + 128 * i, 0, 0);
    }
#endif
  };

  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m = 0.f, lsum = 0.f;

  // per-lane LDS read bases (bytes, relative to a stage)
  const unsigned sbase = (unsigned)(size_t)lsm;
  const int xr = (l32 >> 2) & 3;
  const unsigned kb_e = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * (hh ^ xr);
  const unsigned kb_o = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * ((2 + hh) ^ xr);
  const int gi = lane & 15;
  const int c3 = 2 * ((lane >> 4) & 1) + ((gi & 3) >> 1);
  const unsigned vb_1 = TILE + 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh) + 8 * (gi & 1);
  const unsigned vb_2 = TILE + 16 * D + 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh ^ 2) + 8 * (gi & 1);

  ASTAMP_DECL
#pragma unroll
  for (int t = 0; t < LEAD; ++t) issue(t, t);

  bf16x8 pf0, pf1;  // P^T of the tile in flight (softmax -> PV)
  // S^T = K.Q^T of tile t (K row fragments two k-steps ahead of their MFMA), softmax into pf0/pf1
  auto sm_part = [&](int buf, auto masked, int t) {
    constexpr bool MASKED = decltype(masked)::value;
    const unsigned st0 = sbase + buf * STAGE;
    const unsigned ke = st0 + kb_e, ko = st0 + kb_o;
    f32x16 sa;
#pragma unroll
    for (int r = 0; r < 16; ++r) sa[r] = 0.f;
    u32x4 fk[3];
    fk[0] = ads_b128<0>(ke);
    fk[1] = ads_b128<0>(ko);
    static_for<0, KS>([&](auto S_) {
      constexpr int s = decltype(S_)::value;
      if constexpr (s + 2 < KS) fk[(s + 2) % 3] = ads_b128<512 * ((s + 2) >> 1)>(((s + 2) & 1) ? ko : ke);
      constexpr int after = (s + 2 < KS) ? 2 : (KS - 1 - s);
      lgkm_wait<after>(fk[s % 3]);
      sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(fk[s % 3]), qf[s], sa, 0, 0, 0);
    });
    ASTAMP(3);
    if constexpr (MASKED) {
      const int lim = qrow + off - t * BN - 4 * hh;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if ((r & 3) + 8 * (r >> 2) > lim) sa[r] = -INFINITY;
    }
    if (t == 0) {  // reference max = the first tile's row max (see attn_fwd_tiled_kernel)
      float mt = sa[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mt = fmaxf(mt, sa[r]);
      m = fmaxf(mt, __shfl_xor(mt, 32, 64)) * sl2;
    }
    const float nm = -m;
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float e0 = __builtin_amdgcn_exp2f(fmaf(sa[r], sl2, nm));
      const float e1 = __builtin_amdgcn_exp2f(fmaf(sa[r + 8], sl2, nm));
      ps += e0 + e1;
      pf0[r] = (__bf16)e0;
      pf1[r] = (__bf16)e1;
    }
    lsum += ps;
    ASTAMP(4);
  };
  // O^T += V^T.P^T of the tile in `buf`: the V^T reads of d-block db+1 in flight under block db's MFMAs
  auto pv_part = [&](int buf) {
    const unsigned st0 = sbase + buf * STAGE;
    const unsigned v1 = st0 + vb_1, v2 = st0 + vb_2;
    u32x2 va0 = ads_tr<0>(v1), va1 = ads_tr<0>(v2);
    u32x2 vb0 = ads_tr<2 * 16 * D>(v1), vb1 = ads_tr<2 * 16 * D>(v2);
    static_for<0, D / 32>([&](auto DB_) {
      constexpr int db = decltype(DB_)::value;
      u32x2 na0, na1, nb0, nb1;
      if constexpr (db + 1 < D / 32) {
        na0 = ads_tr<512 * (db + 1)>(v1);
        na1 = ads_tr<512 * (db + 1)>(v2);
        nb0 = ads_tr<2 * 16 * D + 512 * (db + 1)>(v1);
        nb1 = ads_tr<2 * 16 * D + 512 * (db + 1)>(v2);
        lgkm_wait<4>(va0, va1, vb0, vb1);
      } else {
        lgkm_wait<0>(va0, va1, vb0, vb1);
      }
      oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(va0, va1), pf0, oacc[db], 0, 0, 0);
      oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf8(vb0, vb1), pf1, oacc[db], 0, 0, 0);
      if constexpr (db + 1 < D / 32) {
        va0 = na0; va1 = na1; vb0 = nb0; vb1 = nb1;
      }
    });
    ASTAMP(5);
  };

  // Tile t: wait for this wave's pieces of tile t (INFLIGHT younger DMA instructions may remain),
  // barrier (every piece landed; every wave done with tile t-1), refill tile t-1's buffer with tile
  // t+LEAD, compute. Measured and not kept (same-box A/B, GPT-J fwd): a ping-pong schedule (waves 4-7
  // one PV behind, so the two waves of a SIMD never sit in softmax together; two tiles ahead) 5 %
  // slower; two tiles per barrier (vmcnt(0), one superstep ahead) 3-5 % slower.
  auto sync_issue = [&](int t) {
    ASTAMP(0);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INFLIGHT) : "memory");
    __builtin_amdgcn_s_barrier();
    ASTAMP(1);
    issue(t + LEAD, (t + LEAD) % NBUF);
    ASTAMP(2);
  };
  // causal: the mask is applied on every tile (16 selects that change nothing before the diagonal):
  // separate masked / mask-free bodies made hipcc spill ~170 registers
  constexpr auto CM = std::integral_constant<bool, CAUSAL>{};
  for (int t = 0; t < ntiles; ++t) {
    sync_issue(t);
    if (t < mytiles) {
      sm_part(t % NBUF, CM, t);
      pv_part(t % NBUF);
    }
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const bool bad = !(ltot < 1.2676506e30f);
  const int any_bad = __any(bad);
  // overflow flags in the 4-wave kernel's layout (4 per 128-row block, lid order of the generic fixup)
  {
    const int nqb128 = p.Sq / 128, qb128 = q0 / 128, w128 = (q0 % 128) / 32;
    const int lid128 = bh * nqb128 + (CAUSAL ? nqb128 - 1 - qb128 : qb128);
    if (lane == 0) p.flags[lid128 * 4 + w128] = any_bad;
  }
  const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
  if (hh == 0 && p.lse)
    p.lse[((long long)b * p.H + h) * p.Sq + qrow] = ltot > 0.f ? (m + log2f(ltot)) * kLn2 : INFINITY;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the clamped tail DMAs
  __syncthreads();  // the tile buffers become the epilogue images
  store_tile_lds<D, D>(p.o + b * p.o_sb + h * p.o_sh + (long long)q0 * p.o_st, p.o_st, oacc, lane, inv,
                       smem + wave * 32 * D * 2);
  ASTAMP(6);
  ASTAMP_FLUSH(48);
}

// ====================================================================== backward
// Same image and fragment conventions as the forward. Two kernels, no float
// atomics, deterministic:
//   dQ kernel  : wave = 32 queries; Q, dO fragments resident, dQ^T in AGPRs;
//                sweeps 32-key K/V tiles (double-buffered images).
//                S^T = K.Q^T, dP^T = V.dO^T (keys on registers, query on the
//                lane), dS^T = P^T (dP^T - delta), dQ^T += K^T.dS^T with K^T
//                from the K image by transposed reads.
//   dK/dV kernel: wave = 32 keys; K fragments resident, the workgroup's V rows
//                in one LDS image, dK^T / dV^T in AGPRs; sweeps 32-row Q/dO
//                tiles (and the query heads of its KV head for GQA).
//                S = Q.K^T, dP = dO.V^T (key on the lane), dV^T += dO^T.P,
//                dK^T += Q^T.dS with dO^T, Q^T by transposed reads.
struct FastBwdParams {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* dout;
  bf16_t* dq; bf16_t* dk; bf16_t* dv;
  const float* lse; const float* delta;
  long long q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, do_sb, do_st, do_sh;
  long long dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh, dv_sb, dv_st, dv_sh;
  int B, Sq, Sk, H, Hkv;
  float scale;
};

// A operand (32 rows x 16 k) read by rows from an image: lane (row l32, half hh)
// takes chunk 2s+hh of its row. Returns the two per-lane bases (s even / odd).
template <int D>
__device__ __forceinline__ void row_bases(int l32, int hh, int& e, int& o) {
  const int xr = (l32 >> 2) & 3;
  e = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * (hh ^ xr);
  o = (l32 >> 3) * 16 * D + 64 * (l32 & 7) + 16 * ((2 + hh) ^ xr);
}
// transposed A operand (32 columns x 16 permuted rows) from an image
template <int D>
__device__ __forceinline__ void tr_bases(int lane, int& b1, int& b2) {
  const int hh = lane >> 5, gi = lane & 15;
  const int c3 = 2 * ((lane >> 4) & 1) + ((gi & 3) >> 1);
  b1 = 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh) + 8 * (gi & 1);
  b2 = 16 * D + 64 * (4 * hh + (gi >> 2)) + 16 * (c3 ^ hh ^ 2) + 8 * (gi & 1);
}
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int b1, int b2, int s, int db) {
  return cat8(lds_tr4(img, b1 + 2 * s * 16 * D + 512 * db), lds_tr4(img, b2 + 2 * s * 16 * D + 512 * db));
}
template <int D>
__device__ __forceinline__ bf16x8 row_frag(const char* img, int be, int bo, int s) {
  return lds_b128(img, ((s & 1) ? bo : be) + 512 * (s >> 1));
}

// store a D/32 x f32x16 transposed accumulator (row d, column = lane token) as
// bf16 row `tok` of a [.., D] tensor, times `mul`
template <int D>
__device__ __forceinline__ void store_acc_t(bf16_t* rowp, const f32x16 (&acc)[D / 32], int hh, float mul) {
#pragma unroll
  for (int db = 0; db < D / 32; ++db) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint2 w;
      w.x = pk_bf16(acc[db][4 * g] * mul, acc[db][4 * g + 1] * mul);
      w.y = pk_bf16(acc[db][4 * g + 2] * mul, acc[db][4 * g + 3] * mul);
      *reinterpret_cast<uint2*>(rowp + db * 32 + 8 * g + 4 * hh) = w;
    }
  }
}

// DS < D ("narrow storage", as the forward): heads stored DS wide (SD-1.5's 40-wide heads in 48 columns,
// D = 64 images, the pad chunks of every image zeroed once); the S / dP contractions run DS / 16 MFMA
// steps, the dQ (dK, dV) tiles are stored DS wide.
// 64-wide heads without a causal mask (SD): registers capped for 4 waves per SIMD instead of 3 (a 16-byte
// spill in the 48-wide form; DreamBooth +1.5-2.8 % same box, profiles/decode_launch_structure_ab_r5.txt)
template <int D, bool CAUSAL, int DS = D>
__global__ void __launch_bounds__(256, (D <= 64 && !CAUSAL) ? 4 : 1) attn_bwd_dq_tiled_kernel(FastBwdParams p) {
  constexpr int BM = 128, BN = 32;
  constexpr int TILE = BN * D * 2;
  using Stg = StagerFor<D, DS>;
  constexpr int CPT = Stg::CPT;
  constexpr int KSD = DS / 16;  // contraction steps over the stored columns
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];
  ASTAMP_DECL

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
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
  const int ntiles = (kv_hi + BN - 1) / BN;
  const float sl2 = p.scale * kLog2e;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh + (long long)qrow * p.q_st;
  const bf16_t* gp = p.dout + b * p.do_sb + h * p.do_sh + (long long)qrow * p.do_st;
  bf16x8 qf[KSD], gf[KSD];
#pragma unroll
  for (int s = 0; s < KSD; ++s) {
    qf[s] = *reinterpret_cast<const bf16x8*>(qp + 16 * s + 8 * hh);
    gf[s] = *reinterpret_cast<const bf16x8*>(gp + 16 * s + 8 * hh);
  }
  const long long li = ((long long)b * p.H + h) * p.Sq + qrow;
  const float nlse = -p.lse[li] * kLog2e;
  const float dl = p.delta[li];
  f32x16 dq[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[i][r] = 0.f;

  const bf16_t* kst = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vst = p.v + b * p.v_sb + hk * p.v_sh;
  Stg stg(tid, p.k_st, p.v_st);
  stg.bind(kst, vst, p.k_st, p.v_st);
  u32x4 sk[CPT], sv[CPT];
  int be, bo, b1, b2;
  row_bases<D>(l32, hh, be, bo);
  tr_bases<D>(lane, b1, b2);
  if constexpr (DS < D) {  // K / V image chunks DS/8.. are never loaded: zero them in both buffers once
    constexpr int PC = D / 8 - DS / 8, NZ = 2 * 2 * 32 * PC;
    for (int i = tid; i < NZ; i += 256) {
      const int img = i / (32 * PC), row = (i / PC) % 32, ch = DS / 8 + i % PC;
      *reinterpret_cast<u32x4*>(smem + img * TILE + img_off<D>(row, ch)) = u32x4{0, 0, 0, 0};
    }
  }

  stg.load(sk, sv, kst, vst, 0, p.k_st, p.v_st);
  stg.store(sk, sv, smem);
  __syncthreads();
  ASTAMP(0);
  // the last 4 tiles hold the four waves' diagonals; earlier tiles run the
  // mask-free body. Tiles wholly above a wave's rows are masked, not skipped.
  auto tile_step = [&](int t, auto masked) {
    constexpr bool MASKED = decltype(masked)::value;
    const int k0 = t * BN;
    const char* Ks = smem + (t & 1) * 2 * TILE;
    const char* Vs = Ks + TILE;
    // (a second register set of loads in flight -- as the forward's PF2 -- only moved this kernel's
    // wait from the LDS store to the load issue: the K/V stream is throughput-bound per CU,
    // profiles/attn_stamps_r2.md)
    stg.load(sk, sv, kst, vst, min(k0 + BN, (ntiles - 1) * BN), p.k_st, p.v_st);
    asm volatile("" ::: "memory");
    ASTAMP(1);
    f32x16 st, dpt;
#pragma unroll
    for (int r = 0; r < 16; ++r) { st[r] = 0.f; dpt[r] = 0.f; }
    // K / V row fragments of k-step s+2 requested before the MFMAs of step s (pinned), so no MFMA
    // waits out an LDS round trip (see the dK/dV kernel)
    {
      bf16x8 fk[3], fv[3];
      fk[0] = row_frag<D>(Ks, be, bo, 0);
      fv[0] = row_frag<D>(Vs, be, bo, 0);
      fk[1] = row_frag<D>(Ks, be, bo, 1);
      fv[1] = row_frag<D>(Vs, be, bo, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int s = 0; s < KSD; ++s) {
        if (s + 2 < KSD) {
          fk[(s + 2) % 3] = row_frag<D>(Ks, be, bo, s + 2);
          fv[(s + 2) % 3] = row_frag<D>(Vs, be, bo, s + 2);
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        }
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fk[s % 3], qf[s], st, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fv[s % 3], gf[s], dpt, 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
      }
    }
    ASTAMP(2);
    const int lim = qrow + off - k0 - 4 * hh;  // visible key offsets (r&3)+8(r>>2) <= lim
    bf16x8 d0, d1;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float p0 = __builtin_amdgcn_exp2f(fmaf(st[r], sl2, nlse));
      float p1 = __builtin_amdgcn_exp2f(fmaf(st[r + 8], sl2, nlse));
      if constexpr (MASKED) {
        if ((r & 3) + 8 * (r >> 2) > lim) p0 = 0.f;
        if ((r & 3) + 8 * (r >> 2) + 16 > lim) p1 = 0.f;
      }
      d0[r] = (__bf16)(p0 * (dpt[r] - dl));
      d1[r] = (__bf16)(p1 * (dpt[r + 8] - dl));
    }
    ASTAMP(3);
    {
      bf16x8 t0[2], t1[2];
      t0[0] = tr_frag<D>(Ks, b1, b2, 0, 0);
      t1[0] = tr_frag<D>(Ks, b1, b2, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        if (db + 1 < D / 32) {
          t0[(db + 1) & 1] = tr_frag<D>(Ks, b1, b2, 0, db + 1);
          t1[(db + 1) & 1] = tr_frag<D>(Ks, b1, b2, 1, db + 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        }
        dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t0[db & 1], d0, dq[db], 0, 0, 0);
        dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t1[db & 1], d1, dq[db], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
      }
    }
    ASTAMP(4);
    asm volatile("" ::: "memory");
    if (t + 1 < ntiles) stg.store(sk, sv, smem + ((t + 1) & 1) * 2 * TILE);
    __syncthreads();
    ASTAMP(5);
  };
  const int nfree = CAUSAL ? ntiles - 4 : ntiles;
  for (int t = 0; t < nfree; ++t) tile_step(t, std::false_type{});
  for (int t = max(nfree, 0); t < ntiles; ++t) tile_step(t, std::true_type{});
  store_tile_lds<D, DS>(p.dq + b * p.dq_sb + h * p.dq_sh + (long long)q0 * p.dq_st, p.dq_st, dq, lane, p.scale,
                        smem + wave * 32 * D * 2);
  ASTAMP(6);
  ASTAMP_FLUSH(16);
}

// 64-wide heads without a causal mask (SD-1.5's 40-wide heads in narrow storage): registers capped for
// 3 waves per SIMD (165 VGPRs, no spill) instead of 2 -- DreamBooth 61.1 -> 62.3 samples/s same box
// (the causal D = 64 form spills at that cap and keeps 2)
template <int D, bool CAUSAL, int DS = D>
__global__ void __launch_bounds__(256, (D <= 64 && !CAUSAL) ? 3 : 1) attn_bwd_dkdv_tiled_kernel(FastBwdParams p) {
  constexpr int BK = 128, BQ = 32;
  constexpr int TILE = BQ * D * 2;                  // one 32-row image
  using Stg = StagerFor<D, DS>;
  constexpr int NCH = D / 8, NCS = DS / 8, CPT = Stg::CPT;
  constexpr int KSD = DS / 16;                      // contraction steps over the stored columns
  constexpr int VOFF = 4 * TILE;                    // V images of the 4 waves
  constexpr int LOFF = VOFF + 4 * TILE;             // lse/delta: [buf][64] floats
  __shared__ __attribute__((aligned(16))) char smem[LOFF + 2 * 64 * 4];
  ASTAMP_DECL

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int nkb = p.Sk / BK;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = lid % nkb, bh = lid / nkb;
  const int b = bh / p.Hkv, hk = bh % p.Hkv;
  const int grp = p.H / p.Hkv;
  const int off = p.Sk - p.Sq;
  const int kw = kb * BK + wave * 32;
  const int key = kw + l32;
  const float sl2 = p.scale * kLog2e;

  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;
  bf16x8 kf[KSD];
#pragma unroll
  for (int s = 0; s < KSD; ++s)
    kf[s] = *reinterpret_cast<const bf16x8*>(kp + (long long)key * p.k_st + 16 * s + 8 * hh);
  // this wave's 32 V rows -> its own image (read back by rows for dP; pad chunks zero)
  char* vimg = smem + VOFF + wave * TILE;
#pragma unroll
  for (int i = 0; i < 32 * NCH / 64; ++i) {
    const int idx = lane + 64 * i, row = idx / NCH, ch = idx % NCH;
    *reinterpret_cast<u32x4*>(vimg + img_off<D>(row, ch)) =
        ch < NCS ? *reinterpret_cast<const u32x4*>(vp + (long long)(kw + row) * p.v_st + ch * 8) : u32x4{0, 0, 0, 0};
  }
  if constexpr (DS < D) {  // Q / dO image chunks DS/8.. are never loaded: zero them in both buffers once
    constexpr int PC = NCH - NCS, NZ = 2 * 2 * 32 * PC;
    for (int i = tid; i < NZ; i += 256) {
      const int img = i / (32 * PC), row = (i / PC) % 32, ch = NCS + i % PC;
      *reinterpret_cast<u32x4*>(smem + img * TILE + img_off<D>(row, ch)) = u32x4{0, 0, 0, 0};
    }
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[i][r] = 0.f; dv[i][r] = 0.f; }

  int q_lo = 0;
  if (CAUSAL) q_lo = max(0, kb * BK - off) & ~(BQ - 1);
  const int nqt = (p.Sq - q_lo) / BQ;
  const int total = nqt * grp;

  Stg stg(tid, p.q_st, p.do_st);
  stg.bind(p.q + b * p.q_sb + hk * grp * p.q_sh, p.dout + b * p.do_sb + hk * grp * p.do_sh, p.q_st, p.do_st);
  u32x4 sq[CPT], sg[CPT];
  float lreg = 0.f;
  int be, bo, b1, b2;
  row_bases<D>(l32, hh, be, bo);
  tr_bases<D>(lane, b1, b2);

#define KCA_DKDV_LOAD(it_)                                                                     \
  {                                                                                            \
    const int hq_ = hk * grp + (it_) / nqt, qt_ = q_lo + ((it_) % nqt) * BQ;                   \
    if (grp > 1) stg.set_base(p.q + b * p.q_sb + hq_ * p.q_sh, p.dout + b * p.do_sb + hq_ * p.do_sh); \
    stg.load(sq, sg, p.q + b * p.q_sb + hq_ * p.q_sh, p.dout + b * p.do_sb + hq_ * p.do_sh, qt_,   \
             p.q_st, p.do_st);                                                                 \
    if (tid < 64) {                                                                            \
      const long long li_ = ((long long)b * p.H + hq_) * p.Sq + qt_ + (tid & 31);              \
      lreg = tid < 32 ? p.lse[li_] * kLog2e : p.delta[li_];                                    \
    }                                                                                          \
  }
#define KCA_DKDV_STORE(buf_)                                                                   \
  {                                                                                            \
    stg.store(sq, sg, smem + (buf_) * 2 * TILE);                                               \
    if (tid < 64) reinterpret_cast<float*>(smem + LOFF)[(buf_) * 64 + tid] = lreg;             \
  }

  if (total > 0) {
    KCA_DKDV_LOAD(0);
    KCA_DKDV_STORE(0);
  }
  __syncthreads();
  ASTAMP(0);
  auto tile_step = [&](int it, auto masked) {
    constexpr bool MASKED = decltype(masked)::value;
    const int qt = q_lo + (it % nqt) * BQ;
    const char* Qs = smem + (it & 1) * 2 * TILE;
    const char* Gs = Qs + TILE;
    const float* ls = reinterpret_cast<const float*>(smem + LOFF) + (it & 1) * 64;
    const int nx = min(it + 1, total - 1);
    KCA_DKDV_LOAD(nx);
    asm volatile("" ::: "memory");
    ASTAMP(1);
    // No skip of the (at most 3 per head) q tiles that lie wholly above this
    // wave's keys: they are masked to P = 0 like the diagonal, which costs
    // ~4 % extra MFMAs under a causal mask but keeps the 256 dK/dV accumulator
    // registers out of a conditional region (the skip made hipcc spill).
    f32x16 sacc, dpacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) { sacc[r] = 0.f; dpacc[r] = 0.f; }
    // S = Q.K^T, dP = dO.V^T with the three LDS fragments of k-step s+1 requested before the two
    // MFMAs of step s (pinned by sched_group_barrier): at ~445 live registers hipcc otherwise
    // issues each read right before its MFMA behind an lgkmcnt(0) -- 63 of this kernel's 64 MFMAs
    // waited out a full LDS round trip (20 % MFMA busy, profiles/pmc_kernels_r1.md).
    {
      bf16x8 fq0 = row_frag<D>(Qs, be, bo, 0), fg0 = row_frag<D>(Gs, be, bo, 0), fv0 = row_frag<D>(vimg, be, bo, 0);
      bf16x8 fq1, fg1, fv1;
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
      for (int s = 0; s < KSD; ++s) {
        bf16x8& cq = (s & 1) ? fq1 : fq0;
        bf16x8& cg = (s & 1) ? fg1 : fg0;
        bf16x8& cv = (s & 1) ? fv1 : fv0;
        bf16x8& nq = (s & 1) ? fq0 : fq1;
        bf16x8& ng = (s & 1) ? fg0 : fg1;
        bf16x8& nv = (s & 1) ? fv0 : fv1;
        if (s + 1 < KSD) {
          nq = row_frag<D>(Qs, be, bo, s + 1);
          ng = row_frag<D>(Gs, be, bo, s + 1);
          nv = row_frag<D>(vimg, be, bo, s + 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        }
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cq, kf[s], sacc, 0, 0, 0);
        dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cg, cv, dpacc, 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
      }
    }
    ASTAMP(2);
    // rows q = qt + 8g + 4hh + j (g = r>>2, j = r&3): lse / delta as float4;
    // visible iff key <= q + off, i.e. 8g + j >= key - qt - off - 4hh
    const int lim = key - qt - off - 4 * hh;
    bf16x8 p0, p1, s0, s1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 lq = *reinterpret_cast<const f32x4*>(ls + 8 * g + 4 * hh);
      const f32x4 dq4 = *reinterpret_cast<const f32x4*>(ls + 32 + 8 * g + 4 * hh);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * g + j;
        float pr = __builtin_amdgcn_exp2f(fmaf(sacc[r], sl2, -lq[j]));
        if constexpr (MASKED) {
          if (8 * g + j < lim) pr = 0.f;
        }
        const float ds = pr * (dpacc[r] - dq4[j]);
        if (r < 8) { p0[r] = (__bf16)pr; s0[r] = (__bf16)ds; }
        else { p1[r - 8] = (__bf16)pr; s1[r - 8] = (__bf16)ds; }
      }
    }
    ASTAMP(3);
    // dV^T += dO^T.P, dK^T += Q^T.dS: the 8 transposed reads of block db+1 in flight under the 4
    // MFMAs of block db (same pinning)
    {
      bf16x8 a0 = tr_frag<D>(Gs, b1, b2, 0, 0), a1 = tr_frag<D>(Gs, b1, b2, 1, 0);
      bf16x8 a2 = tr_frag<D>(Qs, b1, b2, 0, 0), a3 = tr_frag<D>(Qs, b1, b2, 1, 0);
      bf16x8 n0, n1, n2, n3;
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
        bf16x8& c0 = (db & 1) ? n0 : a0;
        bf16x8& c1 = (db & 1) ? n1 : a1;
        bf16x8& c2 = (db & 1) ? n2 : a2;
        bf16x8& c3 = (db & 1) ? n3 : a3;
        bf16x8& x0 = (db & 1) ? a0 : n0;
        bf16x8& x1 = (db & 1) ? a1 : n1;
        bf16x8& x2 = (db & 1) ? a2 : n2;
        bf16x8& x3 = (db & 1) ? a3 : n3;
        if (db + 1 < D / 32) {
          x0 = tr_frag<D>(Gs, b1, b2, 0, db + 1);
          x1 = tr_frag<D>(Gs, b1, b2, 1, db + 1);
          x2 = tr_frag<D>(Qs, b1, b2, 0, db + 1);
          x3 = tr_frag<D>(Qs, b1, b2, 1, db + 1);
          __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
        }
        dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c0, p0, dv[db], 0, 0, 0);
        dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c1, p1, dv[db], 0, 0, 0);
        dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c2, s0, dk[db], 0, 0, 0);
        dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(c3, s1, dk[db], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
      }
    }
    ASTAMP(4);
    asm volatile("" ::: "memory");
    if (it + 1 < total) KCA_DKDV_STORE((it + 1) & 1);
    __syncthreads();
    ASTAMP(5);
  };
  // One flat loop with the (cheap, select-only) causal mask on every tile:
  // splitting into masked / mask-free bodies -- by a per-tile branch or by
  // two loops per head -- pushed the 256 dK/dV accumulators into spills.
  for (int it = 0; it < total; ++it) tile_step(it, std::integral_constant<bool, CAUSAL>{});
#undef KCA_DKDV_LOAD
#undef KCA_DKDV_STORE
  if constexpr (D == 96) {  // the LDS staging's registers push this one past 256 (2 -> 1 wave per SIMD)
    store_acc_t<D>(p.dk + b * p.dk_sb + hk * p.dk_sh + (long long)key * p.dk_st, dk, hh, p.scale);
    store_acc_t<D>(p.dv + b * p.dv_sb + hk * p.dv_sh + (long long)key * p.dv_st, dv, hh, 1.f);
  } else {
    store_tile_lds<D, DS>(p.dk + b * p.dk_sb + hk * p.dk_sh + (long long)kw * p.dk_st, p.dk_st, dk, lane, p.scale,
                      smem + wave * 32 * D * 2);
    store_tile_lds<D, DS>(p.dv + b * p.dv_sb + hk * p.dv_sh + (long long)kw * p.dv_st, p.dv_st, dv, lane, 1.f,
                      smem + wave * 32 * D * 2);
  }
  ASTAMP(6);
  ASTAMP_FLUSH(32);
}

// the staged K/V (dK/dV: Q/dO) rows are addressed as 32-bit byte offsets from a
// per-head buffer resource; longer rows fall back to the generic kernel
inline bool offsets_fit(long long rows, long long stride) { return (rows + 128) * stride * 2 < (1ll << 31); }

}  // namespace

// A/B knob for the full-tile kernels: bit 0 = 8-wave D = 256 forward (attn_fwd_w8_kernel).
// (An LDS-DMA dQ kernel -- four buffers, three K/V tiles in flight, asm LDS reads -- measured
// 1.5-2.5 % slower on GPT-J fwd+bwd than the register-staged one and was dropped.)
static int g_attn_variant = 1;
KCA_API int kca_attn_set_variant(int v) {
  g_attn_variant = v;
  return 0;
}

// Returns 0 when launched, 1 when the shape is outside the fast path (the
// caller then uses the generic kernel).
KCA_API int kca_attn_fwd_tiled(const void* q, const void* k, const void* v, void* o, float* lse,
                               long long q_sb, long long q_st, long long q_sh, long long k_sb,
                               long long k_st, long long k_sh, long long v_sb, long long v_st,
                               long long v_sh, long long o_sb, long long o_st, long long o_sh,
                               int B, int Sq, int Sk, int H, int Hkv, int d, int causal,
                               float scale, int rowsum_col, int max_col, int* flags, hipStream_t stream) {
  if ((d != 48 && d != 64 && d != 96 && d != 128 && d != 160 && d != 256) || Sq % 128 || Sk % 32 || Sq <= 0 ||
      H % Hkv || !flags)
    return 1;
  if (max_col >= 0 && (max_col != 40 || rowsum_col != 40 || d != 48)) return 1;  // instantiated variant
  if (d == 48 && causal) return 1;  // narrow storage: SD-1.5's (non-causal) 40-wide heads
  if (rowsum_col >= 0 && (rowsum_col != 40 || (d != 64 && d != 48) || causal)) return 1;  // instantiated variants
  if (causal && Sk < Sq) return 1;
  if (!offsets_fit(Sk, k_st) || !offsets_fit(Sk, v_st)) return 1;  // buffer-load byte offsets are 32-bit
  FastFwdParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, flags,
                  q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh,
                  B, Sq, Sk, H, Hkv, scale};
  dim3 grid((Sq / 128) * B * H);
  (void)hipGetLastError();
  if (d == 256 && (g_attn_variant & 1) && Sq % 256 == 0) {
    dim3 g8((Sq / 256) * B * H);
    if (causal) hipLaunchKernelGGL((attn_fwd_w8_kernel<256, true>), g8, dim3(512), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_w8_kernel<256, false>), g8, dim3(512), 0, stream, p);
  } else if (d == 256) {
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<256, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<256, false>), grid, dim3(256), 0, stream, p);
  } else if (d == 160) {  // SD-1.5 1280-channel heads
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<160, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<160, false>), grid, dim3(256), 0, stream, p);
  } else if (d == 128) {
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<128, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<128, false>), grid, dim3(256), 0, stream, p);
  } else if (d == 96) {  // SD-1.5 640-channel heads (80) zero-padded by the UNet
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<96, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<96, false>), grid, dim3(256), 0, stream, p);
  } else if (d == 48) {  // SD-1.5 heads (40) zero-padded to 48 by the UNet inference path, D = 64 image
    if (max_col == 40) hipLaunchKernelGGL((attn_fwd_tiled_kernel<64, false, 40, 48, 40>), grid, dim3(256), 0, stream, p);
    else if (rowsum_col == 40) hipLaunchKernelGGL((attn_fwd_tiled_kernel<64, false, 40, 48>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<64, false, -1, 48>), grid, dim3(256), 0, stream, p);
  } else {  // 64: GPT-2 / CLIP heads
    if (causal) hipLaunchKernelGGL((attn_fwd_tiled_kernel<64, true>), grid, dim3(256), 0, stream, p);
    else if (rowsum_col == 40) hipLaunchKernelGGL((attn_fwd_tiled_kernel<64, false, 40>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_tiled_kernel<64, false>), grid, dim3(256), 0, stream, p);
  }
  // a failed launch leaves the flags unwritten: report it so the caller runs
  // the generic kernel on every block instead of trusting stale flags
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// The VAE's single 512-wide head (non-causal, no masks): 0 = launched (flags[4 * (Sq/128) * B * H]
// hold per-32-row overflow marks the caller must check), 1 = shape outside this path.
KCA_API int kca_attn_fwd_wide(const void* q, const void* k, const void* v, void* o, float* lse, long long q_sb,
                              long long q_st, long long q_sh, long long k_sb, long long k_st, long long k_sh,
                              long long v_sb, long long v_st, long long v_sh, long long o_sb, long long o_st,
                              long long o_sh, int B, int Sq, int Sk, int H, int Hkv, int d, float scale, int* flags,
                              hipStream_t stream) {
  if (d != 512 || Sq % 128 || Sk % 32 || Sq <= 0 || Sk <= 0 || H % Hkv || !flags) return 1;
  if (!offsets_fit(Sk, k_st) || !offsets_fit(Sk, v_st)) return 1;
  if ((q_st | k_st | v_st | o_st) % 8) return 1;  // 16-B row chunks
  FastFwdParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, flags,
                  q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh,
                  B, Sq, Sk, H, Hkv, scale};
  (void)hipGetLastError();
  hipLaunchKernelGGL((attn_fwd_w8_kernel<512, false, 4, 2>), dim3((Sq / 128) * B * H), dim3(256), 0, stream, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

KCA_API int kca_attn_bwd_tiled(const void* q, const void* k, const void* v, const void* dout,
                               void* dq, void* dk, void* dv, const float* lse, const float* delta,
                               long long q_sb, long long q_st, long long q_sh, long long k_sb,
                               long long k_st, long long k_sh, long long v_sb, long long v_st,
                               long long v_sh, long long do_sb, long long do_st, long long do_sh,
                               long long dq_sb, long long dq_st, long long dq_sh, long long dk_sb,
                               long long dk_st, long long dk_sh, long long dv_sb, long long dv_st,
                               long long dv_sh, int B, int Sq, int Sk, int H, int Hkv, int d,
                               int causal, float scale, hipStream_t stream) {
  if ((d != 48 && d != 64 && d != 96 && d != 128 && d != 160 && d != 256) || Sq % 128 || Sk % 128 || Sq <= 0 ||
      H % Hkv)
    return 1;
  if (d == 48 && causal) return 1;  // narrow storage: SD-1.5's (non-causal) 40-wide heads
  if (causal && Sk < Sq) return 1;
  if (!offsets_fit(Sk, k_st) || !offsets_fit(Sk, v_st) || !offsets_fit(Sq, q_st) || !offsets_fit(Sq, do_st)) return 1;
  FastBwdParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout,
                  (bf16_t*)dq, (bf16_t*)dk, (bf16_t*)dv, lse, delta,
                  q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, do_sb, do_st, do_sh,
                  dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh, dv_sb, dv_st, dv_sh,
                  B, Sq, Sk, H, Hkv, scale};
  dim3 g1((Sk / 128) * B * Hkv), g2((Sq / 128) * B * H);
  if (d == 48) {  // heads stored 48 wide in D = 64 images (the UNet's 40-wide heads, training)
    hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<64, false, 48>), g1, dim3(256), 0, stream, p);
    hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<64, false, 48>), g2, dim3(256), 0, stream, p);
  } else if (d == 256) {
    if (causal) {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<256, true>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<256, true>), g2, dim3(256), 0, stream, p);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<256, false>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<256, false>), g2, dim3(256), 0, stream, p);
    }
  } else if (d == 160) {
    if (causal) {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<160, true>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<160, true>), g2, dim3(256), 0, stream, p);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<160, false>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<160, false>), g2, dim3(256), 0, stream, p);
    }
  } else if (d == 96) {
    if (causal) {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<96, true>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<96, true>), g2, dim3(256), 0, stream, p);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<96, false>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<96, false>), g2, dim3(256), 0, stream, p);
    }
  } else if (d == 128) {
    if (causal) {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<128, true>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<128, true>), g2, dim3(256), 0, stream, p);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<128, false>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<128, false>), g2, dim3(256), 0, stream, p);
    }
  } else {
    if (causal) {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<64, true>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<64, true>), g2, dim3(256), 0, stream, p);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<64, false>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<64, false>), g2, dim3(256), 0, stream, p);
    }
  }
  return 0;
}

#ifdef KCA_ATTN_STAMPS
// diagnostic build: copy out (and optionally clear) the 64 segment sums
KCA_API int kca_attn_stamps(unsigned long long* host, int reset) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), sizeof(unsigned long long) * 64) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_attn_stamps), z, sizeof(z)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
