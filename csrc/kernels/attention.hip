// Flash attention forward / backward for gfx950 (K2, K13, K16 in SURVEY §2.4).
//
// Replaces flash-attn 1.0.4 (finetuner-workflow/finetuner/requirements-
// precompilable.txt:2), the NeoX "scaled-upper-triang-masked-softmax" fusion
// (kubeflow/training-operator/gpt-neox/04-finetune-workflow.yaml:216) and the
// DS-Inference BLOOM ALiBi softmax (online-inference/bloom-176b-deepspeed/
// files/isvc-patch.txt:85-92) with one CDNA4-native design:
//
// Forward  (MFMA v_mfma_f32_32x32x16_bf16, "swapped" products):
//   S^T = K . Q^T  -> the accumulator has the query on the LANE and 16 keys in
//                     registers, so the online softmax is lane-local (one
//                     cross-half max exchange per tile, no LDS round trip);
//   O^T += V^T . P^T -> P^T's accumulator registers ARE the B operand (the k
//                     index permuted to match, cdna_hip_programming.md §3
//                     "accumulator tile as the next MFMA's operand"), V^T comes
//                     from LDS with ds_read_b64_tr_b16 (T10), O rescales stay
//                     per lane.
//   A workgroup = 4 waves x 32 query rows; K/V tiles of 32 keys are
//   register-staged (issued before the tile's MFMAs, written to LDS after the
//   barrier: T14) into padded LDS images that are bank-conflict free for the
//   ds_read_b128 K rows (pad 16 B) and the transposed V reads (row stride
//   = 64 B x odd mod 256).
//
// Backward (MFMA v_mfma_f32_16x16x32_bf16, two deterministic kernels, no
// float atomics):
//   dK/dV kernel: a wave owns 16 keys (K, V fragments in registers, dK^T and
//     dV^T accumulators resident), sweeps query tiles of 32 rows. S and dP are
//     computed with the key on the lane, so P / dS feed dV^T += dO^T.P and
//     dK^T += Q^T.dS directly; dO^T, Q^T come from LDS by transposed reads.
//   dQ kernel: a wave owns 16 queries, sweeps key tiles; S^T, dP^T with the
//     query on the lane feed dQ^T += K^T.dS^T.
//   Q/dO/K/V LDS images use a 32-B row pad (row stride = 32 B x odd mod 256)
//   which is conflict free for both the row reads and the transposed reads.
//
// Layouts: q/k/v/o/do/dq/dk/dv are [B, S, H, D] views with arbitrary batch,
// token and head strides (so the fused QKV GEMM output is consumed in place);
// lse / delta are [B, H, Sq] fp32. Supports causal (bottom-right aligned,
// offset = Sk - Sq), per-batch key lengths (right padding), ALiBi, GQA, a
// sliding window (GPT-Neo local layers: tiles left of the band are skipped,
// not masked) and a per-key bitmap for masks with holes (the interior EOS
// separators of a pad == eos context, finetuner.py:674-691).
// Head dims are padded to a compiled D in {64, 96, 128, 160, 256}; the real
// head dim (a multiple of 8) is masked on load/store.
#include "common.h"

#define LOG2E 1.4426950408889634f
#define LN2 0.6931471805599453f

struct AttnParams {
  const bf16_t* q; const bf16_t* k; const bf16_t* v;
  bf16_t* o; float* lse;
  long long q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh;
  long long o_sb, o_st, o_sh;
  int B, Sq, Sk, H, Hkv, d_real, causal;
  float scale;
  const float* alibi;  // [H] slopes or null
  const int* kv_len;   // [B] or null
  const int* fix_flags;  // fixup mode: run only blocks whose tiled-path wave flags are set
  int window;                 // > 0: key visible only if key > q + off - window (GPT-Neo local layers)
  const unsigned* key_mask;   // [B, km_words] bitmap of attended keys (masks with holes) or null
  int km_words;
};

struct AttnBwdParams {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* o;
  const bf16_t* dout; bf16_t* dq; bf16_t* dk; bf16_t* dv;
  const float* lse; const float* delta;
  long long q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh;
  long long do_sb, do_st, do_sh;
  long long dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh, dv_sb, dv_st, dv_sh;
  int B, Sq, Sk, H, Hkv, d_real, causal;
  float scale;
  const float* alibi;
  const int* kv_len;
  int window;
  const unsigned* key_mask;
  int km_words;
};

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ bf16x4 tr_read(const bf16_t* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4*)(reinterpret_cast<uintptr_t>(lds_ptr)));
}

__device__ __forceinline__ bf16x8 cat44(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ bf16x8 ld_bf16x8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.f;
  return z;
}

__device__ __forceinline__ bf16x8 to_bf16x8(const float* x) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (__bf16)x[i];
  return r;
}

// Bank-conflict-free row strides (in bf16 elements), see header.
template <int D> struct FwdLds {
  static constexpr int KSTR = D + 8;  // 2D+16 bytes: odd # of 16-B slots
  static constexpr int VPADB = ((64 - (2 * D) % 256 + 256) % 256) <
                                       ((192 - (2 * D) % 256 + 256) % 256)
                                   ? ((64 - (2 * D) % 256 + 256) % 256)
                                   : ((192 - (2 * D) % 256 + 256) % 256);
  static constexpr int VSTR = D + VPADB / 2;
};
template <int D> struct BwdLds {
  static constexpr int STR = D + 16;  // 2D+32 bytes = 32 B x odd
};
// Stage rows [r0, r0+ROWS) of a [S, D] head slice into registers (16 B chunks).
// `full` (workgroup-uniform): every row in range and d_real == D -> no guards,
// so interior tiles compile to straight global_load_dwordx4 streams.
template <int D, int ROWS, int NT>
struct Stager {
  static constexpr int NC = D / 8;
  static constexpr int TOTAL = ROWS * NC;
  static constexpr int CPT = (TOTAL + NT - 1) / NT;
  uint4 r[CPT];
  __device__ __forceinline__ void load(const bf16_t* base, long long st, int r0,
                                       int nrows, int d_real, bool full) {
    if (full) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int idx = threadIdx.x + i * NT;
        const int row = idx / NC, ch = idx % NC;
        if (TOTAL % NT == 0 || idx < TOTAL)
          r[i] = *reinterpret_cast<const uint4*>(base + (long long)(r0 + row) * st + ch * 8);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = threadIdx.x + i * NT;
      const int row = idx / NC, ch = idx % NC;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (idx < TOTAL && r0 + row < nrows && ch * 8 < d_real)
        val = *reinterpret_cast<const uint4*>(base + (long long)(r0 + row) * st + ch * 8);
      r[i] = val;
    }
  }
  __device__ __forceinline__ void store(bf16_t* lds, int stride) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int idx = threadIdx.x + i * NT;
      if (TOTAL % NT == 0 || idx < TOTAL) {
        const int row = idx / NC, ch = idx % NC;
        *reinterpret_cast<uint4*>(lds + row * stride + ch * 8) = r[i];
      }
    }
  }
};

// bit `key` of batch row b of the attended-key bitmap (caller guarantees key < Sk)
__device__ __forceinline__ bool km_bit(const unsigned* km, int words, int b, int key) {
  return (km[(long long)b * words + (key >> 5)] >> (key & 31)) & 1u;
}

// Deferred-rescale threshold (log2 units): O / l are rescaled only when a row's
// running max grows by more than this, so P <= 2^8 between rescales (T13).
#define RESCALE_THR 8.0f

// ============================================================== forward
template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, (D <= 128 ? 2 : 1)) attn_fwd_kernel(AttnParams p) {
  using L = FwdLds<D>;
  constexpr int BM = 128, BN = 32;
  constexpr int KSZ = BN * L::KSTR, VSZ = BN * L::VSTR;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (KSZ + VSZ)];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int nqb = (p.Sq + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  if (p.fix_flags) {  // same grid / lid mapping as attn_fwd_tiled_kernel
    const int4 f = reinterpret_cast<const int4*>(p.fix_flags)[lid];
    if (!(f.x | f.y | f.z | f.w)) return;
  }
  const int qi = lid % nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int bh = lid / nqb;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hkv);
  const int off = p.Sk - p.Sq;
  int kv_end = p.Sk;
  KCA_DASSERT(!p.kv_len || (p.kv_len[b] >= 0 && p.kv_len[b] <= p.Sk));
  if (p.kv_len) kv_end = min(kv_end, p.kv_len[b]);
  const int q0 = qb * BM + wave * BN;
  const int qrow = q0 + l32;
  int kv_hi = kv_end;
  if (CAUSAL) kv_hi = min(kv_hi, qb * BM + BM - 1 + off + 1);
  const int ntiles = kv_hi > 0 ? (kv_hi + BN - 1) / BN : 0;
  // sliding window: tiles wholly left of the workgroup's band are never loaded
  const int t0 = p.window > 0 ? min(ntiles, max(0, qb * BM + off - p.window + 1) / BN) : 0;
  const bool dfull = p.d_real == D;

  const float sl2 = p.scale * LOG2E;
  const float slope = p.alibi ? p.alibi[h] * LOG2E : 0.f;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;

  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int d0 = 16 * s + 8 * hh;
    qf[s] = (qrow < p.Sq && d0 < p.d_real) ? ld_bf16x8(qp + (long long)qrow * p.q_st + d0)
                                           : zero_bf16x8();
  }
  f32x16 oacc[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[i][r] = 0.f;
  float m = -INFINITY, lsum = 0.f;

  Stager<D, BN, 256> sk, sv;
  if (ntiles > t0) {
    const bool full = dfull && (t0 + 1) * BN <= p.Sk;
    sk.load(kp, p.k_st, t0 * BN, p.Sk, p.d_real, full);
    sv.load(vp, p.v_st, t0 * BN, p.Sk, p.d_real, full);
    sk.store(smem + (t0 & 1) * (KSZ + VSZ), L::KSTR);
    sv.store(smem + (t0 & 1) * (KSZ + VSZ) + KSZ, L::VSTR);
  }
  __syncthreads();

  const int gi = lane & 15;
  const int dcol = 16 * ((lane >> 4) & 1) + 4 * (gi & 3);
  const int wlo = q0 + off - p.window + 1;  // window: first key visible to the wave's first row
  for (int t = t0; t < ntiles; ++t) {
    const int k0 = t * BN;
    const bf16_t* Ks = smem + (t & 1) * (KSZ + VSZ);
    const bf16_t* Vs = Ks + KSZ;
    if (t + 1 < ntiles) {  // T14: next tile's loads in flight under this tile's MFMAs
      const bool full = dfull && (k0 + 2 * BN <= p.Sk);
      sk.load(kp, p.k_st, k0 + BN, p.Sk, p.d_real, full);
      sv.load(vp, p.v_st, k0 + BN, p.Sk, p.d_real, full);
    }
    const bool active = (!CAUSAL || (k0 <= q0 + BN - 1 + off)) && (p.window <= 0 || k0 + BN - 1 >= wlo);
    if (active) {
      f32x16 sacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        bf16x8 a = ld_bf16x8(Ks + l32 * L::KSTR + 16 * s + 8 * hh);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], sacc, 0, 0, 0);
      }
      const bool need_mask = (CAUSAL && (k0 + BN - 1 > q0 + off)) || (k0 + BN > kv_end) ||
                             (p.window > 0 && k0 < wlo + BN - 1) || p.key_mask;
      float x[16];
      float mt = -INFINITY;
      if (need_mask || p.alibi) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          bool valid = key < kv_end;
          if (CAUSAL) valid = valid && (key <= qrow + off);
          if (p.window > 0) valid = valid && (key > qrow + off - p.window);
          if (p.key_mask) valid = valid && km_bit(p.key_mask, p.km_words, b, key);
          float v = sacc[r] * sl2;
          if (p.alibi) v += slope * (float)(key - qrow - off);
          x[r] = valid ? v : -INFINITY;
          mt = fmaxf(mt, x[r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          x[r] = sacc[r] * sl2;
          mt = fmaxf(mt, x[r]);
        }
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      if (!__all(mt <= m + RESCALE_THR)) {
        const float mnew = fmaxf(m, mt);
        const float alpha = (mnew == -INFINITY) ? 1.f : exp2f(m - mnew);
        lsum *= alpha;
#pragma unroll
        for (int i = 0; i < D / 32; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) oacc[i][r] *= alpha;
        m = mnew;
      }
      const float msub = (m == -INFINITY) ? 0.f : m;
      float ps = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        x[r] = exp2f(x[r] - msub);
        ps += x[r];
      }
      lsum += ps;
      const bf16x8 pf0 = to_bf16x8(x), pf1 = to_bf16x8(x + 8);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int row = 16 * s + 4 * hh + (gi >> 2);
          const bf16_t* vb = Vs + row * L::VSTR + db * 32 + dcol;
          bf16x8 a = cat44(tr_read(vb), tr_read(vb + 8 * L::VSTR));
          oacc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, s ? pf1 : pf0, oacc[db], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntiles) {  // other buffer: last read in tile t-1, fenced by its barrier
      bf16_t* Kn = smem + ((t + 1) & 1) * (KSZ + VSZ);
      sk.store(Kn, L::KSTR);
      sv.store(Kn + KSZ, L::VSTR);
    }
    __syncthreads();
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
  if (qrow < p.Sq) {
    if (hh == 0 && p.lse)
      p.lse[((long long)b * p.H + h) * p.Sq + qrow] =
          ltot > 0.f ? (m + log2f(ltot)) * LN2 : INFINITY;
    bf16_t* op = p.o + b * p.o_sb + h * p.o_sh + (long long)qrow * p.o_st;
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = db * 32 + 8 * g + 4 * hh;
        if (d < p.d_real) {
          uint2 w;
          w.x = pack_bf16x2(oacc[db][4 * g] * inv, oacc[db][4 * g + 1] * inv);
          w.y = pack_bf16x2(oacc[db][4 * g + 2] * inv, oacc[db][4 * g + 3] * inv);
          *reinterpret_cast<uint2*>(op + d) = w;
        }
      }
    }
  }
}

// ============================================================== backward
// delta[b,h,q] = sum_d dO[q,d] * O[q,d]
__global__ void attn_bwd_preprocess_kernel(const bf16_t* __restrict__ o,
                                           const bf16_t* __restrict__ dout,
                                           float* __restrict__ delta,
                                           long long o_sb, long long o_st,
                                           long long o_sh, long long do_sb,
                                           long long do_st, long long do_sh,
                                           int B, int S, int H, int d_real,
                                           int tpr) {
  const long long rows = (long long)B * H * S;
  const int rpb = blockDim.x / tpr;
  const long long row = (long long)blockIdx.x * rpb + threadIdx.x / tpr;
  const int sub = threadIdx.x % tpr;
  float s = 0.f;
  if (row < rows) {
    const int q = row % S;
    const long long bh = row / S;
    const int h = bh % H, b = bh / H;
    const bf16_t* op = o + b * o_sb + h * o_sh + (long long)q * o_st;
    const bf16_t* gp = dout + b * do_sb + h * do_sh + (long long)q * do_st;
    for (int d = sub * 8; d < d_real; d += tpr * 8) {
      float a[8], g[8];
      load8(op + d, a);
      load8(gp + d, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += a[j] * g[j];
    }
  }
  for (int w = tpr / 2; w > 0; w >>= 1) s += __shfl_xor(s, w, 64);
  if (row < rows && sub == 0) delta[row] = s;
}


template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, (D <= 128 ? 2 : 1)) attn_bwd_dkdv_kernel(AttnBwdParams p) {
  using L = BwdLds<D>;
  constexpr int BK = 64, BQ = 32;
  constexpr int TSZ = BQ * L::STR;
  constexpr int BUF = 2 * TSZ + 2 * BQ * 2;  // Q, dO tiles + lse, delta (as floats)
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * BUF];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, gi = lane & 15;
  const int nkb = (p.Sk + BK - 1) / BK;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = lid % nkb, bh = lid / nkb;
  const int b = bh / p.Hkv, hk = bh % p.Hkv;
  const int grp = p.H / p.Hkv;
  const int off = p.Sk - p.Sq;
  int kv_end = p.Sk;
  KCA_DASSERT(!p.kv_len || (p.kv_len[b] >= 0 && p.kv_len[b] <= p.Sk));
  if (p.kv_len) kv_end = min(kv_end, p.kv_len[b]);
  const int kw = kb * BK + wave * 16;
  const int key = kw + gi;
  const float sl2 = p.scale * LOG2E;
  const bool dfull = p.d_real == D;

  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;
  bf16x8 kf[D / 32], vf[D / 32];
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const int d0 = 32 * s + 8 * G;
    const bool ok = key < p.Sk && d0 < p.d_real;
    kf[s] = ok ? ld_bf16x8(kp + (long long)key * p.k_st + d0) : zero_bf16x8();
    vf[s] = ok ? ld_bf16x8(vp + (long long)key * p.v_st + d0) : zero_bf16x8();
  }
  f32x4 dk[D / 16], dv[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { dk[i][r] = 0.f; dv[i][r] = 0.f; }

  int q_lo = 0;
  if (CAUSAL) q_lo = max(0, kb * BK - off) & ~(BQ - 1);
  // window: queries past the last key's band see none of this block's keys
  const int q_end = p.window > 0 ? min(p.Sq, kb * BK + BK - 1 - off + p.window) : p.Sq;
  const int nqt = q_end > q_lo ? (q_end - q_lo + BQ - 1) / BQ : 0;
  const int total = (kb * BK < kv_end) ? nqt * grp : 0;
  const bool key_ok = key < kv_end && (!p.key_mask || km_bit(p.key_mask, p.km_words, b, key));

  Stager<D, BQ, 256> sq, sd;
  float lse_r = INFINITY, dl_r = 0.f;
  auto load_tile = [&](int it) {
    const int hq = hk * grp + it / nqt;
    const int qt = q_lo + (it % nqt) * BQ;
    const bool full = dfull && (qt + BQ <= p.Sq);
    sq.load(p.q + b * p.q_sb + hq * p.q_sh, p.q_st, qt, p.Sq, p.d_real, full);
    sd.load(p.dout + b * p.do_sb + hq * p.do_sh, p.do_st, qt, p.Sq, p.d_real, full);
    if (threadIdx.x < BQ) {
      const int q = qt + threadIdx.x;
      const long long li = ((long long)b * p.H + hq) * p.Sq + q;
      lse_r = q < p.Sq ? p.lse[li] : INFINITY;
      dl_r = q < p.Sq ? p.delta[li] : 0.f;
    }
  };
  auto store_tile = [&](int buf) {
    bf16_t* base = smem + buf * BUF;
    sq.store(base, L::STR);
    sd.store(base + TSZ, L::STR);
    float* f = reinterpret_cast<float*>(base + 2 * TSZ);
    if (threadIdx.x < BQ) {
      f[threadIdx.x] = lse_r;
      f[BQ + threadIdx.x] = dl_r;
    }
  };
  if (total > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  const int trow = 4 * G + (gi >> 2);
  const int tcol = 4 * (gi & 3);
  for (int it = 0; it < total; ++it) {
    const int hq = hk * grp + it / nqt;
    const int qt = q_lo + (it % nqt) * BQ;
    const bf16_t* Qs = smem + (it & 1) * BUF;
    const bf16_t* Ds = Qs + TSZ;
    const float* lse_s = reinterpret_cast<const float*>(Qs + 2 * TSZ);
    const float* dl_s = lse_s + BQ;
    if (it + 1 < total) load_tile(it + 1);
    const bool active = !CAUSAL || (kw <= qt + BQ - 1 + off);
    if (active) {
      f32x4 sacc[2], dpacc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) { sacc[j][r] = 0.f; dpacc[j][r] = 0.f; }
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int off_l = (j * 16 + gi) * L::STR + 32 * s + 8 * G;
          sacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_bf16x8(Qs + off_l), kf[s], sacc[j], 0, 0, 0);
          dpacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_bf16x8(Ds + off_l), vf[s], dpacc[j], 0, 0, 0);
        }
      }
      const bool need_mask = (CAUSAL && (kw + 15 > qt + off)) || (kw + 16 > kv_end) ||
                             (qt + BQ > p.Sq) || p.window > 0 || p.key_mask;
      const float slope = p.alibi ? p.alibi[hq] * LOG2E : 0.f;
      float pv[8], dsv[8];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = j * 16 + 4 * G + r;
          const int q = qt + ql;
          float x = sacc[j][r] * sl2 - lse_s[ql] * LOG2E;
          if (p.alibi) x += slope * (float)(key - q - off);
          float pr = exp2f(x);
          if (need_mask) {
            bool valid = q < p.Sq && key_ok;
            if (CAUSAL) valid = valid && (key <= q + off);
            if (p.window > 0) valid = valid && (key > q + off - p.window);
            pr = valid ? pr : 0.f;
          }
          pv[j * 4 + r] = pr;
          dsv[j * 4 + r] = pr * (dpacc[j][r] - dl_s[ql]);
        }
      }
      const bf16x8 pb = to_bf16x8(pv), dsb = to_bf16x8(dsv);
#pragma unroll
      for (int db = 0; db < D / 16; ++db) {
        const bf16_t* dob = Ds + trow * L::STR + db * 16 + tcol;
        const bf16x8 ado = cat44(tr_read(dob), tr_read(dob + 16 * L::STR));
        dv[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ado, pb, dv[db], 0, 0, 0);
        const bf16_t* qb_ = Qs + trow * L::STR + db * 16 + tcol;
        const bf16x8 aq = cat44(tr_read(qb_), tr_read(qb_ + 16 * L::STR));
        dk[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, dsb, dk[db], 0, 0, 0);
      }
    }
    if (it + 1 < total) store_tile((it + 1) & 1);
    __syncthreads();
  }
  if (key < p.Sk) {
    bf16_t* dkp = p.dk + b * p.dk_sb + hk * p.dk_sh + (long long)key * p.dk_st;
    bf16_t* dvp = p.dv + b * p.dv_sb + hk * p.dv_sh + (long long)key * p.dv_st;
#pragma unroll
    for (int db = 0; db < D / 16; ++db) {
      const int d = db * 16 + 4 * G;
      if (d < p.d_real) {
        uint2 w;
        w.x = pack_bf16x2(dk[db][0] * p.scale, dk[db][1] * p.scale);
        w.y = pack_bf16x2(dk[db][2] * p.scale, dk[db][3] * p.scale);
        *reinterpret_cast<uint2*>(dkp + d) = w;
        w.x = pack_bf16x2(dv[db][0], dv[db][1]);
        w.y = pack_bf16x2(dv[db][2], dv[db][3]);
        *reinterpret_cast<uint2*>(dvp + d) = w;
      }
    }
  }
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, (D <= 160 ? 2 : 1)) attn_bwd_dq_kernel(AttnBwdParams p) {
  using L = BwdLds<D>;
  constexpr int BQ = 64, BN = 32;
  constexpr int TSZ = BN * L::STR;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TSZ];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = lane >> 4, gi = lane & 15;
  const int nqb = (p.Sq + BQ - 1) / BQ;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int bh = lid / nqb;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hkv);
  const int off = p.Sk - p.Sq;
  int kv_end = p.Sk;
  KCA_DASSERT(!p.kv_len || (p.kv_len[b] >= 0 && p.kv_len[b] <= p.Sk));
  if (p.kv_len) kv_end = min(kv_end, p.kv_len[b]);
  const int qw = qb * BQ + wave * 16;
  const int q = qw + gi;
  const float sl2 = p.scale * LOG2E;
  const float slope = p.alibi ? p.alibi[h] * LOG2E : 0.f;
  const bool dfull = p.d_real == D;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* gp = p.dout + b * p.do_sb + h * p.do_sh;
  bf16x8 qf[D / 32], gf[D / 32];
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const int d0 = 32 * s + 8 * G;
    const bool ok = q < p.Sq && d0 < p.d_real;
    qf[s] = ok ? ld_bf16x8(qp + (long long)q * p.q_st + d0) : zero_bf16x8();
    gf[s] = ok ? ld_bf16x8(gp + (long long)q * p.do_st + d0) : zero_bf16x8();
  }
  const long long li = ((long long)b * p.H + h) * p.Sq + q;
  const float lse_q = q < p.Sq ? p.lse[li] * LOG2E : INFINITY;
  const float dl_q = q < p.Sq ? p.delta[li] : 0.f;
  f32x4 dq[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) dq[i][r] = 0.f;

  int kv_hi = kv_end;
  if (CAUSAL) kv_hi = min(kv_hi, qb * BQ + BQ - 1 + off + 1);
  const int ntiles = kv_hi > 0 ? (kv_hi + BN - 1) / BN : 0;
  const int t0 = p.window > 0 ? min(ntiles, max(0, qb * BQ + off - p.window + 1) / BN) : 0;
  const int wlo = qw + off - p.window + 1;
  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;
  Stager<D, BN, 256> sk, sv;
  if (ntiles > t0) {
    const bool full = dfull && (t0 + 1) * BN <= p.Sk;
    sk.load(kp, p.k_st, t0 * BN, p.Sk, p.d_real, full);
    sv.load(vp, p.v_st, t0 * BN, p.Sk, p.d_real, full);
    sk.store(smem + (t0 & 1) * 2 * TSZ, L::STR);
    sv.store(smem + (t0 & 1) * 2 * TSZ + TSZ, L::STR);
  }
  __syncthreads();
  const int trow = 4 * G + (gi >> 2);
  const int tcol = 4 * (gi & 3);
  for (int t = t0; t < ntiles; ++t) {
    const int k0 = t * BN;
    const bf16_t* Ks = smem + (t & 1) * 2 * TSZ;
    const bf16_t* Vs = Ks + TSZ;
    if (t + 1 < ntiles) {
      const bool full = dfull && (k0 + 2 * BN <= p.Sk);
      sk.load(kp, p.k_st, k0 + BN, p.Sk, p.d_real, full);
      sv.load(vp, p.v_st, k0 + BN, p.Sk, p.d_real, full);
    }
    const bool active = (!CAUSAL || (k0 <= qw + 15 + off)) && (p.window <= 0 || k0 + BN - 1 >= wlo);
    if (active) {
      f32x4 st[2], dpt[2];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) { st[j][r] = 0.f; dpt[j][r] = 0.f; }
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int off_l = (j * 16 + gi) * L::STR + 32 * s + 8 * G;
          st[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_bf16x8(Ks + off_l), qf[s], st[j], 0, 0, 0);
          dpt[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld_bf16x8(Vs + off_l), gf[s], dpt[j], 0, 0, 0);
        }
      }
      const bool need_mask = (CAUSAL && (k0 + BN - 1 > qw + off)) || (k0 + BN > kv_end) ||
                             (qw + 16 > p.Sq) || (p.window > 0 && k0 < wlo + 15) || p.key_mask;
      float dsv[8];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + j * 16 + 4 * G + r;
          float x = st[j][r] * sl2 - lse_q;
          if (p.alibi) x += slope * (float)(key - q - off);
          float pr = exp2f(x);
          if (need_mask) {
            bool valid = q < p.Sq && key < kv_end;
            if (CAUSAL) valid = valid && (key <= q + off);
            if (p.window > 0) valid = valid && (key > q + off - p.window);
            if (p.key_mask) valid = valid && km_bit(p.key_mask, p.km_words, b, key);
            pr = valid ? pr : 0.f;
          }
          dsv[j * 4 + r] = pr * (dpt[j][r] - dl_q);
        }
      }
      const bf16x8 dsb = to_bf16x8(dsv);
#pragma unroll
      for (int db = 0; db < D / 16; ++db) {
        const bf16_t* kb_ = Ks + trow * L::STR + db * 16 + tcol;
        const bf16x8 ak = cat44(tr_read(kb_), tr_read(kb_ + 16 * L::STR));
        dq[db] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ak, dsb, dq[db], 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) {
      bf16_t* Kn = smem + ((t + 1) & 1) * 2 * TSZ;
      sk.store(Kn, L::STR);
      sv.store(Kn + TSZ, L::STR);
    }
    __syncthreads();
  }
  if (q < p.Sq) {
    bf16_t* dqp = p.dq + b * p.dq_sb + h * p.dq_sh + (long long)q * p.dq_st;
#pragma unroll
    for (int db = 0; db < D / 16; ++db) {
      const int d = db * 16 + 4 * G;
      if (d < p.d_real) {
        uint2 w;
        w.x = pack_bf16x2(dq[db][0] * p.scale, dq[db][1] * p.scale);
        w.y = pack_bf16x2(dq[db][2] * p.scale, dq[db][3] * p.scale);
        *reinterpret_cast<uint2*>(dqp + d) = w;
      }
    }
  }
}

// ====================================================== backward, D >= 128
// 32x32x16 variants for head_dim 128 / 256 (GPT-J, BLOOM shards): a wave owns
// 32 keys (dK/dV kernel) or 32 queries (dQ kernel), halving LDS bytes per
// MFMA versus the 16-wide kernels above (each operand fragment feeds a 32-wide
// MFMA). Q/dO/K tiles are read both by rows (ds_read_b128) and transposed
// (ds_read_b64_tr_b16), so they use an XOR-swizzled image with unpadded rows:
// 16-B chunk c of row r lives at chunk c ^ (((r&3)<<2) | ((r>>2)&3)), which is
// conflict free for both access kinds (rows are 16-chunk multiples).
template <int D>
__device__ __forceinline__ int swz_off(int row, int ch) {
  return row * D + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 3);
}

template <int D, int ROWS, int NT>
__device__ __forceinline__ void store_swz(const Stager<D, ROWS, NT>& s, bf16_t* lds) {
#pragma unroll
  for (int i = 0; i < Stager<D, ROWS, NT>::CPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (Stager<D, ROWS, NT>::TOTAL % NT == 0 || idx < Stager<D, ROWS, NT>::TOTAL) {
      const int row = idx / (D / 8), ch = idx % (D / 8);
      *reinterpret_cast<uint4*>(lds + swz_off<D>(row, ch)) = s.r[i];
    }
  }
}

// transposed read of the 32x32x16 A operand (rows r0.., 32 columns at c0)
template <int D>
__device__ __forceinline__ bf16x8 tr_a32(const bf16_t* base, int s, int hh, int lane, int db) {
  const int gi = lane & 15;
  const int row = 16 * s + 4 * hh + (gi >> 2);
  const int col = db * 32 + 16 * ((lane >> 4) & 1) + 4 * (gi & 3);
  const int ch = col >> 3, in = col & 7;
  return cat44(tr_read(base + swz_off<D>(row, ch) + in), tr_read(base + swz_off<D>(row + 8, ch) + in));
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) attn_bwd_dkdv32_kernel(AttnBwdParams p) {
  constexpr int BK = 128, BQ = 32;
  constexpr int TSZ = BQ * D;
  constexpr int BUF = 2 * TSZ + 2 * BQ * 2;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * BUF];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int nkb = (p.Sk + BK - 1) / BK;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = lid % nkb, bh = lid / nkb;
  const int b = bh / p.Hkv, hk = bh % p.Hkv;
  const int grp = p.H / p.Hkv;
  const int off = p.Sk - p.Sq;
  int kv_end = p.Sk;
  KCA_DASSERT(!p.kv_len || (p.kv_len[b] >= 0 && p.kv_len[b] <= p.Sk));
  if (p.kv_len) kv_end = min(kv_end, p.kv_len[b]);
  const int kw = kb * BK + wave * 32;
  const int key = kw + l32;
  const float sl2 = p.scale * LOG2E;
  const bool dfull = p.d_real == D;

  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;
  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int d0 = 16 * s + 8 * hh;
    const bool ok = key < p.Sk && d0 < p.d_real;
    kf[s] = ok ? ld_bf16x8(kp + (long long)key * p.k_st + d0) : zero_bf16x8();
    vf[s] = ok ? ld_bf16x8(vp + (long long)key * p.v_st + d0) : zero_bf16x8();
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[i][r] = 0.f; dv[i][r] = 0.f; }

  int q_lo = 0;
  if (CAUSAL) q_lo = max(0, kb * BK - off) & ~(BQ - 1);
  const int q_end = p.window > 0 ? min(p.Sq, kb * BK + BK - 1 - off + p.window) : p.Sq;
  const int nqt = q_end > q_lo ? (q_end - q_lo + BQ - 1) / BQ : 0;
  const int total = (kb * BK < kv_end) ? nqt * grp : 0;
  const bool key_ok = key < kv_end && (!p.key_mask || km_bit(p.key_mask, p.km_words, b, key));

  Stager<D, BQ, 256> sq, sd;
  float lse_r = INFINITY, dl_r = 0.f;
  auto load_tile = [&](int it) {
    const int hq = hk * grp + it / nqt;
    const int qt = q_lo + (it % nqt) * BQ;
    const bool full = dfull && (qt + BQ <= p.Sq);
    sq.load(p.q + b * p.q_sb + hq * p.q_sh, p.q_st, qt, p.Sq, p.d_real, full);
    sd.load(p.dout + b * p.do_sb + hq * p.do_sh, p.do_st, qt, p.Sq, p.d_real, full);
    if (threadIdx.x < BQ) {
      const int q = qt + threadIdx.x;
      const long long li = ((long long)b * p.H + hq) * p.Sq + q;
      lse_r = q < p.Sq ? p.lse[li] : INFINITY;
      dl_r = q < p.Sq ? p.delta[li] : 0.f;
    }
  };
  auto store_tile = [&](int buf) {
    bf16_t* base = smem + buf * BUF;
    store_swz(sq, base);
    store_swz(sd, base + TSZ);
    float* f = reinterpret_cast<float*>(base + 2 * TSZ);
    if (threadIdx.x < BQ) {
      f[threadIdx.x] = lse_r;
      f[BQ + threadIdx.x] = dl_r;
    }
  };
  if (total > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const int hq = hk * grp + it / nqt;
    const int qt = q_lo + (it % nqt) * BQ;
    const bf16_t* Qs = smem + (it & 1) * BUF;
    const bf16_t* Ds = Qs + TSZ;
    const float* lse_s = reinterpret_cast<const float*>(Qs + 2 * TSZ);
    const float* dl_s = lse_s + BQ;
    if (it + 1 < total) load_tile(it + 1);
    const bool active = !CAUSAL || (kw <= qt + BQ - 1 + off);
    if (active) {
      f32x16 sacc, dpacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) { sacc[r] = 0.f; dpacc[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        const int o = swz_off<D>(l32, 2 * s + hh);
        sacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld_bf16x8(Qs + o), kf[s], sacc, 0, 0, 0);
        dpacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld_bf16x8(Ds + o), vf[s], dpacc, 0, 0, 0);
      }
      const bool need_mask = (CAUSAL && (kw + 31 > qt + off)) || (kw + 32 > kv_end) || (qt + BQ > p.Sq) ||
                             p.window > 0 || p.key_mask;
      const float slope = p.alibi ? p.alibi[hq] * LOG2E : 0.f;
      float pv[16], dsv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int q = qt + ql;
        float x = sacc[r] * sl2 - lse_s[ql] * LOG2E;
        if (p.alibi) x += slope * (float)(key - q - off);
        float pr = exp2f(x);
        if (need_mask) {
          bool valid = q < p.Sq && key_ok;
          if (CAUSAL) valid = valid && (key <= q + off);
          if (p.window > 0) valid = valid && (key > q + off - p.window);
          pr = valid ? pr : 0.f;
        }
        pv[r] = pr;
        dsv[r] = pr * (dpacc[r] - dl_s[ql]);
      }
      const bf16x8 pb0 = to_bf16x8(pv), pb1 = to_bf16x8(pv + 8);
      const bf16x8 db0 = to_bf16x8(dsv), db1 = to_bf16x8(dsv + 8);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          dv[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_a32<D>(Ds, s, hh, lane, db), s ? pb1 : pb0,
                                                           dv[db], 0, 0, 0);
          dk[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_a32<D>(Qs, s, hh, lane, db), s ? db1 : db0,
                                                           dk[db], 0, 0, 0);
        }
      }
    }
    if (it + 1 < total) store_tile((it + 1) & 1);
    __syncthreads();
  }
  if (key < p.Sk) {
    bf16_t* dkp = p.dk + b * p.dk_sb + hk * p.dk_sh + (long long)key * p.dk_st;
    bf16_t* dvp = p.dv + b * p.dv_sb + hk * p.dv_sh + (long long)key * p.dv_st;
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = db * 32 + 8 * g + 4 * hh;
        if (d < p.d_real) {
          uint2 w;
          w.x = pack_bf16x2(dk[db][4 * g] * p.scale, dk[db][4 * g + 1] * p.scale);
          w.y = pack_bf16x2(dk[db][4 * g + 2] * p.scale, dk[db][4 * g + 3] * p.scale);
          *reinterpret_cast<uint2*>(dkp + d) = w;
          w.x = pack_bf16x2(dv[db][4 * g], dv[db][4 * g + 1]);
          w.y = pack_bf16x2(dv[db][4 * g + 2], dv[db][4 * g + 3]);
          *reinterpret_cast<uint2*>(dvp + d) = w;
        }
      }
    }
  }
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) attn_bwd_dq32_kernel(AttnBwdParams p) {
  constexpr int BQ = 128, BN = 32;
  constexpr int TSZ = BN * D;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TSZ];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int nqb = (p.Sq + BQ - 1) / BQ;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int qi = lid % nqb;
  const int qb = CAUSAL ? (nqb - 1 - qi) : qi;
  const int bh = lid / nqb;
  const int b = bh / p.H, h = bh % p.H;
  const int hk = h / (p.H / p.Hkv);
  const int off = p.Sk - p.Sq;
  int kv_end = p.Sk;
  KCA_DASSERT(!p.kv_len || (p.kv_len[b] >= 0 && p.kv_len[b] <= p.Sk));
  if (p.kv_len) kv_end = min(kv_end, p.kv_len[b]);
  const int qw = qb * BQ + wave * 32;
  const int q = qw + l32;
  const float sl2 = p.scale * LOG2E;
  const float slope = p.alibi ? p.alibi[h] * LOG2E : 0.f;
  const bool dfull = p.d_real == D;

  const bf16_t* qp = p.q + b * p.q_sb + h * p.q_sh;
  const bf16_t* gp = p.dout + b * p.do_sb + h * p.do_sh;
  bf16x8 qf[D / 16], gf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    const int d0 = 16 * s + 8 * hh;
    const bool ok = q < p.Sq && d0 < p.d_real;
    qf[s] = ok ? ld_bf16x8(qp + (long long)q * p.q_st + d0) : zero_bf16x8();
    gf[s] = ok ? ld_bf16x8(gp + (long long)q * p.do_st + d0) : zero_bf16x8();
  }
  const long long li = ((long long)b * p.H + h) * p.Sq + q;
  const float lse_q = q < p.Sq ? p.lse[li] * LOG2E : INFINITY;
  const float dl_q = q < p.Sq ? p.delta[li] : 0.f;
  f32x16 dq[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[i][r] = 0.f;

  int kv_hi = kv_end;
  if (CAUSAL) kv_hi = min(kv_hi, qb * BQ + BQ - 1 + off + 1);
  const int ntiles = kv_hi > 0 ? (kv_hi + BN - 1) / BN : 0;
  const int t0 = p.window > 0 ? min(ntiles, max(0, qb * BQ + off - p.window + 1) / BN) : 0;
  const int wlo = qw + off - p.window + 1;
  const bf16_t* kp = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* vp = p.v + b * p.v_sb + hk * p.v_sh;
  Stager<D, BN, 256> sk, sv;
  if (ntiles > t0) {
    const bool full = dfull && (t0 + 1) * BN <= p.Sk;
    sk.load(kp, p.k_st, t0 * BN, p.Sk, p.d_real, full);
    sv.load(vp, p.v_st, t0 * BN, p.Sk, p.d_real, full);
    store_swz(sk, smem + (t0 & 1) * 2 * TSZ);
    store_swz(sv, smem + (t0 & 1) * 2 * TSZ + TSZ);
  }
  __syncthreads();
  for (int t = t0; t < ntiles; ++t) {
    const int k0 = t * BN;
    const bf16_t* Ks = smem + (t & 1) * 2 * TSZ;
    const bf16_t* Vs = Ks + TSZ;
    if (t + 1 < ntiles) {
      const bool full = dfull && (k0 + 2 * BN <= p.Sk);
      sk.load(kp, p.k_st, k0 + BN, p.Sk, p.d_real, full);
      sv.load(vp, p.v_st, k0 + BN, p.Sk, p.d_real, full);
    }
    const bool active = (!CAUSAL || (k0 <= qw + 31 + off)) && (p.window <= 0 || k0 + BN - 1 >= wlo);
    if (active) {
      f32x16 st, dpt;
#pragma unroll
      for (int r = 0; r < 16; ++r) { st[r] = 0.f; dpt[r] = 0.f; }
#pragma unroll
      for (int s = 0; s < D / 16; ++s) {
        const int o = swz_off<D>(l32, 2 * s + hh);
        st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld_bf16x8(Ks + o), qf[s], st, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ld_bf16x8(Vs + o), gf[s], dpt, 0, 0, 0);
      }
      const bool need_mask = (CAUSAL && (k0 + BN - 1 > qw + off)) || (k0 + BN > kv_end) || (qw + 32 > p.Sq) ||
                             (p.window > 0 && k0 < wlo + 31) || p.key_mask;
      float dsv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        float x = st[r] * sl2 - lse_q;
        if (p.alibi) x += slope * (float)(key - q - off);
        float pr = exp2f(x);
        if (need_mask) {
          bool valid = q < p.Sq && key < kv_end;
          if (CAUSAL) valid = valid && (key <= q + off);
          if (p.window > 0) valid = valid && (key > q + off - p.window);
          if (p.key_mask) valid = valid && km_bit(p.key_mask, p.km_words, b, key);
          pr = valid ? pr : 0.f;
        }
        dsv[r] = pr * (dpt[r] - dl_q);
      }
      const bf16x8 d0 = to_bf16x8(dsv), d1 = to_bf16x8(dsv + 8);
#pragma unroll
      for (int db = 0; db < D / 32; ++db) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
          dq[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr_a32<D>(Ks, s, hh, lane, db), s ? d1 : d0,
                                                           dq[db], 0, 0, 0);
      }
    }
    if (t + 1 < ntiles) {
      bf16_t* Kn = smem + ((t + 1) & 1) * 2 * TSZ;
      store_swz(sk, Kn);
      store_swz(sv, Kn + TSZ);
    }
    __syncthreads();
  }
  if (q < p.Sq) {
    bf16_t* dqp = p.dq + b * p.dq_sb + h * p.dq_sh + (long long)q * p.dq_st;
#pragma unroll
    for (int db = 0; db < D / 32; ++db) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = db * 32 + 8 * g + 4 * hh;
        if (d < p.d_real) {
          uint2 w;
          w.x = pack_bf16x2(dq[db][4 * g] * p.scale, dq[db][4 * g + 1] * p.scale);
          w.y = pack_bf16x2(dq[db][4 * g + 2] * p.scale, dq[db][4 * g + 3] * p.scale);
          *reinterpret_cast<uint2*>(dqp + d) = w;
        }
      }
    }
  }
}

// ============================================================== host API
static int pick_d(int d) {
  if (d <= 64) return 64;
  if (d <= 96) return 96;
  if (d <= 128) return 128;
  if (d <= 160) return 160;
  if (d <= 256) return 256;
  return 0;
}

#define ATTN_D_DISPATCH(DV, ...)                                   \
  switch (DV) {                                                    \
    case 64: { constexpr int DD = 64; __VA_ARGS__; } break;         \
    case 96: { constexpr int DD = 96; __VA_ARGS__; } break;         \
    case 128: { constexpr int DD = 128; __VA_ARGS__; } break;       \
    case 160: { constexpr int DD = 160; __VA_ARGS__; } break;       \
    case 256: { constexpr int DD = 256; __VA_ARGS__; } break;       \
    default: return 2;                                             \
  }

// Process-wide switch for the full-tile fast paths (A/B measurement and
// tests): 1 = use them where the shape allows (default), 0 = generic only.
static int g_attn_tiled = 1;
KCA_API int kca_attn_set_tiled(int enable) {
  g_attn_tiled = enable;
  return 0;
}

KCA_API int kca_attn_fwd_tiled(const void* q, const void* k, const void* v, void* o, float* lse,
                               long long q_sb, long long q_st, long long q_sh, long long k_sb,
                               long long k_st, long long k_sh, long long v_sb, long long v_st,
                               long long v_sh, long long o_sb, long long o_st, long long o_sh,
                               int B, int Sq, int Sk, int H, int Hkv, int d, int causal,
                               float scale, int rowsum_col, int max_col, int* flags, hipStream_t stream);

// workspace: >= 4 * ceil(Sq/128) * B * H ints for the full-tile fast path of
// attention_tiled.hip (its overflow flags), or null for the generic kernel.
// rowsum_col: >= 0 when V's padded column rowsum_col is all ones (the fast path then takes the
// row sums from O; the generic kernel ignores it), -1 otherwise. max_col: >= 0 when K is pre-scaled
// by scale' * log2(e) with column max_col = 1 (attention_tiled.hip MC; the caller passes scale = ln 2
// so the generic fixup kernel, which reads Q's zero column max_col, computes the same softmax).
KCA_API int kca_attn_fwd(const void* q, const void* k, const void* v, void* o,
                         float* lse, long long q_sb, long long q_st,
                         long long q_sh, long long k_sb, long long k_st,
                         long long k_sh, long long v_sb, long long v_st,
                         long long v_sh, long long o_sb, long long o_st,
                         long long o_sh, int B, int Sq, int Sk, int H, int Hkv,
                         int d_real, int causal, float scale,
                         const float* alibi, const int* kv_len, int window, const unsigned* key_mask,
                         int rowsum_col, int max_col, int* workspace, hipStream_t stream) {
  if (d_real % 8 || H % Hkv || window < 0) return 1;
  const int D = pick_d(d_real);
  AttnParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse,
               q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh, o_sb, o_st, o_sh,
               B, Sq, Sk, H, Hkv, d_real, causal, scale, alibi, kv_len, nullptr,
               window, key_mask, (Sk + 31) / 32};
  if (g_attn_tiled && workspace && !alibi && !kv_len && !window && !key_mask &&
      kca_attn_fwd_tiled(q, k, v, o, lse, q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh,
                         o_sb, o_st, o_sh, B, Sq, Sk, H, Hkv, d_real, causal, scale, rowsum_col, max_col,
                         workspace, stream) == 0)
    p.fix_flags = workspace;  // fixup launch below: only flagged blocks do work
  dim3 grid(((Sq + 127) / 128) * B * H);
  ATTN_D_DISPATCH(D, {
    if (causal)
      hipLaunchKernelGGL((attn_fwd_kernel<DD, true>), grid, dim3(256), 0, stream, p);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<DD, false>), grid, dim3(256), 0, stream, p);
  });
  return 0;
}

KCA_API int kca_attn_bwd_preprocess(const void* o, const void* dout,
                                    float* delta, long long o_sb,
                                    long long o_st, long long o_sh,
                                    long long do_sb, long long do_st,
                                    long long do_sh, int B, int S, int H,
                                    int d_real, hipStream_t stream) {
  int nc = (d_real + 7) / 8;
  int tpr = 1;
  while (tpr < nc && tpr < 64) tpr <<= 1;
  const int rpb = 256 / tpr;
  const long long rows = (long long)B * H * S;
  const long long grid = (rows + rpb - 1) / rpb;
  hipLaunchKernelGGL(attn_bwd_preprocess_kernel, dim3((unsigned)grid), dim3(256), 0, stream,
                     (const bf16_t*)o, (const bf16_t*)dout, delta, o_sb, o_st, o_sh,
                     do_sb, do_st, do_sh, B, S, H, d_real, tpr);
  return 0;
}

KCA_API int kca_attn_bwd_tiled(const void* q, const void* k, const void* v, const void* dout,
                               void* dq, void* dk, void* dv, const float* lse, const float* delta,
                               long long q_sb, long long q_st, long long q_sh, long long k_sb,
                               long long k_st, long long k_sh, long long v_sb, long long v_st,
                               long long v_sh, long long do_sb, long long do_st, long long do_sh,
                               long long dq_sb, long long dq_st, long long dq_sh, long long dk_sb,
                               long long dk_st, long long dk_sh, long long dv_sb, long long dv_st,
                               long long dv_sh, int B, int Sq, int Sk, int H, int Hkv, int d,
                               int causal, float scale, hipStream_t stream);

KCA_API int kca_attn_bwd(const void* q, const void* k, const void* v,
                         const void* o, const void* dout, void* dq, void* dk,
                         void* dv, const float* lse, const float* delta,
                         long long q_sb, long long q_st, long long q_sh,
                         long long k_sb, long long k_st, long long k_sh,
                         long long v_sb, long long v_st, long long v_sh,
                         long long do_sb, long long do_st, long long do_sh,
                         long long dq_sb, long long dq_st, long long dq_sh,
                         long long dk_sb, long long dk_st, long long dk_sh,
                         long long dv_sb, long long dv_st, long long dv_sh,
                         int B, int Sq, int Sk, int H, int Hkv, int d_real,
                         int causal, float scale, const float* alibi,
                         const int* kv_len, int window, const unsigned* key_mask, hipStream_t stream) {
  if (d_real % 8 || H % Hkv || window < 0) return 1;
  if (g_attn_tiled && !alibi && !kv_len && !window && !key_mask &&
      kca_attn_bwd_tiled(q, k, v, dout, dq, dk, dv, lse, delta, q_sb, q_st, q_sh, k_sb, k_st, k_sh,
                         v_sb, v_st, v_sh, do_sb, do_st, do_sh, dq_sb, dq_st, dq_sh, dk_sb, dk_st,
                         dk_sh, dv_sb, dv_st, dv_sh, B, Sq, Sk, H, Hkv, d_real, causal, scale,
                         stream) == 0)
    return 0;
  const int D = pick_d(d_real);
  AttnBwdParams p{(const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)o,
                  (const bf16_t*)dout, (bf16_t*)dq, (bf16_t*)dk, (bf16_t*)dv, lse, delta,
                  q_sb, q_st, q_sh, k_sb, k_st, k_sh, v_sb, v_st, v_sh,
                  do_sb, do_st, do_sh, dq_sb, dq_st, dq_sh, dk_sb, dk_st, dk_sh,
                  dv_sb, dv_st, dv_sh,
                  B, Sq, Sk, H, Hkv, d_real, causal, scale, alibi, kv_len, window, key_mask, (Sk + 31) / 32};
  if (D == 256) {  // dQ on the 32-wide kernel (D=128 measured faster on the 16-wide pair: occupancy)
    dim3 h1(((Sk + 127) / 128) * B * Hkv);
    dim3 h2(((Sq + 127) / 128) * B * H);
    dim3 g1w(((Sk + 63) / 64) * B * Hkv);
    if (D == 128) {
      if (causal) {
        hipLaunchKernelGGL((attn_bwd_dkdv32_kernel<128, true>), h1, dim3(256), 0, stream, p);
        hipLaunchKernelGGL((attn_bwd_dq32_kernel<128, true>), h2, dim3(256), 0, stream, p);
      } else {
        hipLaunchKernelGGL((attn_bwd_dkdv32_kernel<128, false>), h1, dim3(256), 0, stream, p);
        hipLaunchKernelGGL((attn_bwd_dq32_kernel<128, false>), h2, dim3(256), 0, stream, p);
      }
    } else {
      // D = 256: K, V, dK^T, dV^T of 32 keys exceed the 512-register file, so
      // the dK/dV pass keeps 16 keys per wave; dQ uses the 32-wide kernel.
      if (causal) {
        hipLaunchKernelGGL((attn_bwd_dkdv_kernel<256, true>), g1w, dim3(256), 0, stream, p);
        hipLaunchKernelGGL((attn_bwd_dq32_kernel<256, true>), h2, dim3(256), 0, stream, p);
      } else {
        hipLaunchKernelGGL((attn_bwd_dkdv_kernel<256, false>), g1w, dim3(256), 0, stream, p);
        hipLaunchKernelGGL((attn_bwd_dq32_kernel<256, false>), h2, dim3(256), 0, stream, p);
      }
    }
    return 0;
  }
  dim3 g1(((Sk + 63) / 64) * B * Hkv);
  dim3 g2(((Sq + 63) / 64) * B * H);
  ATTN_D_DISPATCH(D, {
    if (causal) {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<DD, true>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, true>), g2, dim3(256), 0, stream, p);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<DD, false>), g1, dim3(256), 0, stream, p);
      hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, false>), g2, dim3(256), 0, stream, p);
    }
  });
  return 0;
}
