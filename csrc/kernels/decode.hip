// Decode-path kernels for the serving engine:
//
//   kca_decode_prep     RoPE on the new token's Q/K (GPT-J interleaved or NeoX
//                       rotate-half, any rot) + append K/V into the slot cache
//   kca_decode_attn     split-K ("flash-decoding") attention of one query token
//                       per sequence over its cached K/V, ALiBi optional,
//                       GQA groups share one K/V read, + combine kernel
//   kca_sample_logits   fused repetition penalty + bans + temperature + top-k
//                       (radix select) + top-p (mass radix select) + Philox
//                       multinomial + log-prob, one workgroup per row
//
// Reference behaviour these replace: FasterTransformer's masked MHA / sampling
// layers behind online-inference/fastertransformer (runtime_top_k, runtime_top_p,
// temperature, repetition_penalty, bad_words_list, is_return_log_probs:
// download-weights-job-gptj.yml:101-204) and HF generate() sampling used by
// finetuner.py:861-875 / evaluator.py:201-213 / bloom.py:68-77.
//
// KV cache layout is head-major per slot: [slot][kv_head][pos][D] (strides
// passed in), so a (sequence, head) chunk of the cache is one contiguous
// stream of chunk*D*2 bytes -- decode is HBM-bound and reads exactly K+V once.
// Paged mode (tbl != nullptr): the cache is a pool of pages
// [page][kv_head][ps][D] (ps = 1 << ps_shift tokens) and token t of sequence
// `seq` lives in page tbl[seq * tbl_stride + (t >> ps_shift)] -- requests hold
// only the pages they use, and beams share their prefix pages.
#include <algorithm>
#include <cstdio>
#include <type_traits>

#include "decode_tail.h"  // DualLn + the last-arriver residual / LayerNorm tail
#include "gemv_m1.h"  // gemv_m1_accum / _finish for the fused decode-layer kernels

// element offset of token t of sequence `seq` (paged or contiguous)
__device__ __forceinline__ long long kv_row(const int* __restrict__ tbl, int tbl_stride, int ps_shift, int seq,
                                            int t, long long cs_slot, long long cs_pos) {
  if (!tbl) return (long long)seq * cs_slot + (long long)t * cs_pos;
  const int page = tbl[(long long)seq * tbl_stride + (t >> ps_shift)];
  KCA_DASSERT(page >= 0);
  return (long long)page * cs_slot + (long long)(t & ((1 << ps_shift) - 1)) * cs_pos;
}

// ------------------------------------------------------------------ prep
// One wave per (b, head-row) of the fused QKV GEMM output [B, (H+2Hkv)*D];
// lane owns dims lane, lane+64, ... Partner elements of the rotation live in the
// same wave, and every lane loads before any lane stores.
__global__ __launch_bounds__(256) void decode_prep_kernel(
    bf16_t* __restrict__ qkv, long long ld, int B, int H, int Hkv, int D, int rot,
    int interleaved, const float* __restrict__ cos_t, const float* __restrict__ sin_t,
    const int* __restrict__ pos, const int* __restrict__ slots, bf16_t* __restrict__ kc,
    bf16_t* __restrict__ vc, long long cs_slot, long long cs_head, long long cs_pos, const int* __restrict__ tbl,
    int tbl_stride, int ps_shift) {
  const int rows_per_b = H + 2 * Hkv;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long long)B * rows_per_b) return;
  const int lane = threadIdx.x & 63;
  const int b = (int)(row / rows_per_b), j = (int)(row % rows_per_b);
  bf16_t* src = qkv + b * ld + (long long)j * D;
  const int p = pos[b];
  KCA_DASSERT(p >= 0 && (tbl || (long long)p * cs_pos < cs_head));  // position inside the slot's KV capacity
  float x[4], y[4];
  const int half = rot >> 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = lane + 64 * i;
    x[i] = 0.f;
    y[i] = 0.f;
    if (d < D) {
      x[i] = bf2f(src[d]);
      y[i] = x[i];
      if (j < H + Hkv && d < rot) {
        int partner, fi;
        float sgn;
        if (interleaved) {
          partner = d ^ 1;
          fi = d >> 1;
          sgn = (d & 1) ? 1.f : -1.f;
        } else {
          partner = d < half ? d + half : d - half;
          fi = d < half ? d : d - half;
          sgn = d < half ? -1.f : 1.f;
        }
        const float xp = bf2f(src[partner]);
        const float c = cos_t[(long long)p * half + fi], s = sin_t[(long long)p * half + fi];
        y[i] = x[i] * c + sgn * xp * s;
      }
    }
  }
  if (j < H) {  // query: rotate in place (only if rotary)
    if (rot > 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = lane + 64 * i;
        if (d < D && d < rot) src[d] = f2bf(y[i]);
      }
    }
    return;
  }
  const bool is_k = j < H + Hkv;
  const int hk = is_k ? j - H : j - H - Hkv;
  bf16_t* dst = (is_k ? kc : vc) + kv_row(tbl, tbl_stride, ps_shift, slots[b], p, cs_slot, cs_pos) + hk * cs_head;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = lane + 64 * i;
    if (d < D) dst[d] = f2bf(y[i]);
  }
}

KCA_API int kca_decode_prep(void* qkv, long long ld, int B, int H, int Hkv, int D, int rot,
                            int interleaved, const float* cos_t, const float* sin_t,
                            const int* pos, const int* slots, void* kc, void* vc,
                            long long cs_slot, long long cs_head, long long cs_pos, const int* tbl,
                            int tbl_stride, int ps_shift, hipStream_t stream) {
  if (D > 256 || rot > D || (rot & 1) || B <= 0) return 1;
  if (tbl && (ps_shift < 0 || ps_shift > 20 || tbl_stride <= 0)) return 2;
  const long long rows = (long long)B * (H + 2 * Hkv);
  hipLaunchKernelGGL(decode_prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                     (bf16_t*)qkv, ld, B, H, Hkv, D, rot, interleaved, cos_t, sin_t, pos, slots,
                     (bf16_t*)kc, (bf16_t*)vc, cs_slot, cs_head, cs_pos, tbl, tbl_stride, ps_shift);
  return 0;
}

// ------------------------------------------------------------- attention
struct DecodeParams {
  const bf16_t* q;
  long long q_bs;  // q[b*q_bs + h*D + d]
  const bf16_t* kc;
  const bf16_t* vc;
  long long cs_slot, cs_head, cs_pos;
  const int* slots;
  const int* kv_lens;
  bf16_t* out;
  long long o_bs;
  float* ws_o;   // [B*H, nsplit, D]
  float* ws_ml;  // [B*H, nsplit, 2]
  const float* alibi;
  const int* tbl;  // paged cache: [seq][tbl_stride] page ids (nullptr: contiguous slots)
  int tbl_stride, ps_shift;
  int H, Hkv, D, chunk;
  float scale;
  // fused prep (kca_decode_prep_attn): q is the fused QKV row; the kernel applies RoPE to Q itself
  // and the split holding the new token (position kv_len-1) rotates its K, appends K/V to the cache
  // and uses them from LDS -- one launch instead of prep + attention
  int fused, rot, interleaved;
  const float* cos_t;
  const float* sin_t;
  unsigned long long* stamps;  // diagnostic: per-workgroup s_memrealtime stamps (nullptr in normal runs)
  // split-K fan-in (nsplit > 1): one arrival counter per (sequence, kv-head); the last split to
  // arrive combines the partials in place of the separate decode_combine_kernel (nullptr: that kernel)
  unsigned int* cnt;
  int window;  // > 0: attend only the last `window` positions (GPT-Neo local layers)
  // per-step descriptors uploaded with the step's inputs (fused batch-1 decode): bit 0 -- cos_t /
  // sin_t hold row b's RoPE angles at index b (not the position table); bit 1 -- tbl holds row b's
  // page ids at row b (not the slot's). Neither then waits for the length or the slot to arrive.
  int by_row;
};

template <int DT = 0>
__device__ __forceinline__ void store_out(const DecodeParams& p, long long i, float v) { p.out[i] = (bf16_t)f2e<DT>(v); }


// diagnostic stamps (bench/decode_attn_bench.py --stamps): 8 per workgroup, 100 MHz clock
static unsigned long long* g_decode_stamps = nullptr;
KCA_API int kca_decode_set_stamps(void* buf) {
  g_decode_stamps = (unsigned long long*)buf;
  return 0;
}
#define DSTAMP(k)                                                                                     \
  do {                                                                                                \
    if (p.stamps && threadIdx.x == 0)                                                                 \
      p.stamps[(((long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + (k)] = \
          __builtin_amdgcn_s_memrealtime();                                                           \
  } while (0)

// RoPE of the 8 dims [d0, d0+8) of a head row at position `pos`, matching
// decode_prep_kernel (partner values read from the unrotated row; the result is
// rounded to bf16 as the stored rotation would be).
template <int DT = 0>
__device__ __forceinline__ void rope8(const bf16_t* __restrict__ row, int d0, float (&x)[8], int pos, int rot,
                                      int interleaved, const float* __restrict__ cos_t,
                                      const float* __restrict__ sin_t) {
  const int half = rot >> 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int d = d0 + j;
    if (d >= rot) continue;
    int partner, fi;
    float sgn;
    if (interleaved) {
      partner = d ^ 1;
      fi = d >> 1;
      sgn = (d & 1) ? 1.f : -1.f;
    } else {
      partner = d < half ? d + half : d - half;
      fi = d < half ? d : d - half;
      sgn = d < half ? -1.f : 1.f;
    }
    const float c = cos_t[(long long)pos * half + fi], sn = sin_t[(long long)pos * half + fi];
    x[j] = e2f<DT>(f2e<DT>(x[j] * c + sgn * e2f<DT>(row[partner]) * sn));
  }
}

// The cos / sin of dims [d0, d0+8) at table row `pos` (rope8's entries), loaded ahead of use.
__device__ __forceinline__ void rope_tab8(const float* __restrict__ cos_t, const float* __restrict__ sin_t, int pos,
                                          int d0, int rot, int interleaved, float (&c)[8], float (&sn)[8]) {
  const int half = rot >> 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int d = d0 + j;
    c[j] = 1.f;
    sn[j] = 0.f;
    if (d >= rot) continue;
    const int fi = interleaved ? d >> 1 : (d < half ? d : d - half);
    c[j] = cos_t[(long long)pos * half + fi];
    sn[j] = sin_t[(long long)pos * half + fi];
  }
}

// rope8 with the angles in registers (rope_tab8); interleaved pairs take the partner from the
// lane's own raw values, rotate-half partners are read from the unrotated row as rope8 does.
template <int DT = 0>
__device__ __forceinline__ void rope8_reg(const bf16_t* __restrict__ row, int d0, float (&x)[8],
                                          const float (&raw)[8], const float (&c)[8], const float (&sn)[8],
                                          int rot, int interleaved) {
  const int half = rot >> 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int d = d0 + j;
    if (d >= rot) continue;
    float pv, sgn;
    if (interleaved) {
      pv = raw[j ^ 1];
      sgn = (d & 1) ? 1.f : -1.f;
    } else {
      pv = e2f<DT>(row[d < half ? d + half : d - half]);
      sgn = d < half ? -1.f : 1.f;
    }
    x[j] = e2f<DT>(f2e<DT>(x[j] * c[j] + sgn * pv * sn[j]));
  }
}

// Sum over the LPT lanes of a lane group (LPT = 8/16/32 consecutive lanes), the result in every lane
// of the group: DPP quad swaps, then half-row / row mirrors, then a 32-lane swizzle -- VALU-latency
// steps instead of a chain of ds_bpermute round trips through the LDS crossbar. Each step adds the
// same two partial sums in every lane of a pair, so all lanes agree bit for bit.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int LPT>
__device__ __forceinline__ float group_sum(float v) {
  v += dpp_mov<0xB1>(v);                 // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_mov<0x4E>(v);                 // quad_perm [2,3,0,1]: lane ^ 2
  if constexpr (LPT > 4) v += dpp_mov<0x141>(v);  // row_half_mirror: quad <-> quad in 8 lanes
  if constexpr (LPT > 8) v += dpp_mov<0x140>(v);  // row_mirror: 8 <-> 8 in 16 lanes
  if constexpr (LPT > 16)                          // ds_swizzle xor 16 within 32 lanes
    v += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
  return v;
}

// Split-K fan-in at the end of every split's workgroup (nsplit > 1): its partials (st_pub) are
// drained by every storing wave, then one lane adds to the (sequence, kv-head) counter; the
// workgroup that brings it to nsplit re-arms it, acquires (agent scope: drops this CU's stale
// lines) and combines the G heads' splits -- what decode_combine_kernel does, minus a launch and
// its dependency gap on the decode critical path (one per layer).
template <int G, int DT = 0>
__device__ void fanin_combine(const DecodeParams& p, int b, int hk, int nsplit) {
  __shared__ float wsp[1024];
  __shared__ float red[8];
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid == 0) {
    unsigned int* c = p.cnt + ((long long)b * p.Hkv + hk);
    const unsigned prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)(nsplit - 1);
    if (last) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm for the next call
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int D = p.D;
  for (int g = 0; g < G; ++g) {
    const long long bh = (long long)b * p.H + hk * G + g;
    const float* ml = p.ws_ml + bh * nsplit * 2;
    const float* o = p.ws_o + bh * nsplit * D;
    float m = -INFINITY;
    for (int s = tid; s < nsplit; s += 256) m = fmaxf(m, ml[2 * s]);
    const float M = block_max(m, red);
    float l = 0.f;
    for (int s = tid; s < nsplit; s += 256) {
      const float ms = ml[2 * s];
      const float w = ms == -INFINITY ? 0.f : __expf(ms - M);
      wsp[s] = w;
      l += w * ml[2 * s + 1];
    }
    const float Lsum = block_sum(l, red + 4);  // block_sum's barriers also publish wsp
    const float inv = Lsum > 0.f ? 1.f / Lsum : 0.f;
    if (tid < D) {  // D <= 256: one output dim per lane
      float acc = 0.f;
#pragma unroll 8
      for (int s = 0; s < nsplit; ++s) {  // an empty split's partial was never written: may hold NaN
        const float ov = o[(long long)s * D + tid];
        acc = wsp[s] > 0.f ? fmaf(wsp[s], ov, acc) : acc;
      }
      store_out<DT>(p, b * p.o_bs + (hk * G + g) * (long long)D + tid, acc * inv);
    }
    __syncthreads();  // wsp / red reused by the next head
  }
}

// LPT lanes cooperate on one token row (8 dims per lane); TPW = 64/LPT tokens per
// wave step; G query heads share each K/V row (GQA group).
// (the workgroup's (split, kv-head, sequence) coordinates are arguments: decode_attn_kernel passes
// its block index, the fused decode-layer kernel below a slice of its grid)
template <int LPT, int G, bool PAGED, bool ONLINE, bool PF = false, int DT = 0>
__device__ __forceinline__ void decode_attn_body(const DecodeParams& p, const int split, const int hk, const int b,
                                                 const int nsplit) {
  constexpr int TPW = 64 / LPT;
  constexpr int TPB = 4 * TPW;
  constexpr int U = 4;  // tokens per lane per iteration: 2U independent 16-B row loads in flight
  extern __shared__ float smem[];
  DSTAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int D = p.D, ND = D >> 3;
  const int dslot = lane % LPT, tsub = lane / LPT;
  const bool dact = dslot < ND;
  const long long bh0 = (long long)b * p.H + hk * G;
  const int c0 = split * p.chunk;
  // every load that does not depend on the sequence length is issued before the length arrives:
  // the length, the slot, the raw Q rows, the new token's raw K/V rows (fused) and, once the slot
  // is known, this split's page ids -- so the K/V stream starts after two memory round trips, not four
  const int L = p.kv_lens[b];
  const int seq = p.slots[b];
  U16x8 qraw[G];  // inactive lanes read dims [0, 8) (unused) instead of branching around the load
  const bf16_t* krow = p.q + b * p.q_bs + (long long)(p.H + hk) * D;
  const bf16_t* vrow = p.q + b * p.q_bs + (long long)(p.H + p.Hkv + hk) * D;
  U16x8 knraw, vnraw;  // the new token's K / V slice of lane tid (< ND), from the fused QKV row
  auto load_qkv_rows = [&]() {
#pragma unroll
    for (int g = 0; g < G; ++g)
      qraw[g] = *reinterpret_cast<const U16x8*>(p.q + b * p.q_bs + (long long)(hk * G + g) * D + (dact ? dslot : 0) * 8);
    if (p.fused && tid < ND) {
      knraw = *reinterpret_cast<const U16x8*>(krow + tid * 8);
      vnraw = *reinterpret_cast<const U16x8*>(vrow + tid * 8);
    }
  };
  load_qkv_rows();
  // per-step RoPE row (by_row bit 0): the angles do not wait for the length
  const bool pre_rope = (p.by_row & 1) && p.fused && p.rot > 0;
  float rc[8], rs[8];
  if (pre_rope && dact) rope_tab8(p.cos_t, p.sin_t, b, dslot * 8, p.rot, p.interleaved, rc, rs);
  // paged: this split's page ids staged in LDS (chunk <= 1024 tokens, pages >= 16 tokens), so a
  // token's address costs an LDS read instead of a dependent global load in front of every K/V
  // load; the whole chunk's range is staged (clipped to the table row), independent of the length
  __shared__ int pg[1024 / 16 + 2];
  const int pg0 = c0 >> p.ps_shift;
  if constexpr (PAGED) {
    const int npg = min(((c0 + p.chunk - 1) >> p.ps_shift) - pg0 + 1, p.tbl_stride - pg0);
    KCA_DASSERT(npg <= 1024 / 16 + 2);
    const int trow = (p.by_row & 2) ? b : seq;  // per-step page rows: no wait for the slot
    for (int i = tid; i < npg; i += 256) pg[i] = p.tbl[(long long)trow * p.tbl_stride + pg0 + i];
  }
  const int c1 = min(c0 + p.chunk, L);
  // sliding window: positions below L - window are never read (splits left of it are empty)
  const int ca = p.window > 0 ? max(c0, L - p.window) : c0;
  if (ca >= c1) {
    if (nsplit > 1 && tid < G) {
      st_pub(&p.ws_ml[((bh0 + tid) * nsplit + split) * 2], -INFINITY);
      st_pub(&p.ws_ml[((bh0 + tid) * nsplit + split) * 2 + 1], 0.f);
    }
    if (nsplit > 1 && p.cnt) fanin_combine<G, DT>(p, b, hk, nsplit);
    return;
  }
  DSTAMP(1);
  KCA_DASSERT(seq >= 0);
  const long long kvoff = (PAGED ? 0 : (long long)seq * p.cs_slot) + hk * p.cs_head + dslot * 8;
  const bf16_t* kb = p.kc + kvoff;
  const bf16_t* vb = p.vc + kvoff;
  const int pnew = L - 1;  // the new token's position (fused prep)
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (dact) {
#pragma unroll
      for (int j = 0; j < 8; ++j) q[g][j] = e2f<DT>(qraw[g].v[j]);
      if (pre_rope) {
        float raw[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) raw[j] = q[g][j];
        rope8_reg<DT>(p.q + b * p.q_bs + (long long)(hk * G + g) * D, dslot * 8, q[g], raw, rc, rs, p.rot, p.interleaved);
      } else if (p.fused && p.rot > 0) {
        rope8<DT>(p.q + b * p.q_bs + (long long)(hk * G + g) * D, dslot * 8, q[g], pnew, p.rot, p.interleaved, p.cos_t,
              p.sin_t);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) q[g][j] *= p.scale;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) q[g][j] = 0.f;
    }
  }
  float slope[G];
#pragma unroll
  for (int g = 0; g < G; ++g) slope[g] = p.alibi ? p.alibi[hk * G + g] : 0.f;
  if (p.stamps && tid == 0) {  // diagnostic: wait for Q (and its RoPE) before stamping
    float z = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) z += q[g][0];
    if (z == 12345.f) p.stamps[0] = 0;
  }
  DSTAMP(2);
  if constexpr (PAGED) __syncthreads();  // pg[] published
  DSTAMP(3);
  // offset of token t inside this sequence's storage
  auto toff = [&](int t) -> long long {
    if constexpr (PAGED)
      return (long long)pg[(t >> p.ps_shift) - pg0] * p.cs_slot + (long long)(t & ((1 << p.ps_shift) - 1)) * p.cs_pos;
    return (long long)t * p.cs_pos;
  };

  // fused prep: the split holding the new token (position L-1) rotates its K and appends K and V to
  // the cache; no other split reads position L-1. The one-pass path folds the token in after its
  // loop (registers); the two-phase path serves it from LDS.
  const bool own_new = p.fused && c1 == L;
  // one-pass path: the split holding the last token (position L-1) folds it in after its loop, in
  // both modes (fused: the new row from registers; plain: the cached row), so the fused launch
  // stays bit-identical to prep + attention
  const bool own_last = ONLINE && c1 == L;
  float kx[8], vx[8];  // two-phase path: the new row, staged to LDS below
  if (own_new && tid < ND) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      kx[j] = e2f<DT>(knraw.v[j]);
      vx[j] = e2f<DT>(vnraw.v[j]);
    }
    if (pre_rope) {  // tid < ND <= LPT: this lane's dslot is tid, its angles are rc / rs
      float raw[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) raw[j] = kx[j];
      rope8_reg<DT>(krow, tid * 8, kx, raw, rc, rs, p.rot, p.interleaved);
    } else if (p.rot > 0) {
      rope8<DT>(krow, tid * 8, kx, pnew, p.rot, p.interleaved, p.cos_t, p.sin_t);
    }
    const long long o = toff(pnew) + hk * p.cs_head + tid * 8;  // toff: offset inside the sequence
    store8_t<DT>(const_cast<bf16_t*>(p.kc) + (PAGED ? 0 : (long long)seq * p.cs_slot) + o, kx);
    store8_t<DT>(const_cast<bf16_t*>(p.vc) + (PAGED ? 0 : (long long)seq * p.cs_slot) + o, vx);
#pragma unroll
    for (int j = 0; j < 8; ++j) knraw.v[j] = (uint16_t)f2e<DT>(kx[j]);  // exact: the rotation is bf16-rounded
  } else if (own_last && tid < ND) {
    const long long o = (PAGED ? 0 : (long long)seq * p.cs_slot) + toff(pnew) + hk * p.cs_head + tid * 8;
    knraw = *reinterpret_cast<const U16x8*>(p.kc + o);
    vnraw = *reinterpret_cast<const U16x8*>(p.vc + o);
  }
  __shared__ float knew[ONLINE ? 1 : 256], vnew[ONLINE ? 1 : 256];
  if constexpr (!ONLINE) {
    if (own_new) {
      if (tid < ND) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          knew[tid * 8 + j] = kx[j];
          vnew[tid * 8 + j] = vx[j];
        }
      }
      __syncthreads();
    }
  }

  if constexpr (ONLINE) {
  // ---- one pass over the split: a token's K and V rows are requested together (2U 16-B loads in flight
  // per lane) and folded into an online softmax per lane group (the LPT lanes sharing a token row keep
  // their own running max / sum / P.V), so a long split is one latency chain, not a K pass, a block-wide
  // softmax and a V pass
  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }
  // the tokens [c0, ce); the last one (own_last) is folded in below from registers
  const int ce = own_last ? c1 - 1 : c1;
  // inactive lanes (dslot >= ND) and tokens past the split read an in-range row instead of branching
  // around their loads: no branch in the loop, so all 2U loads of an iteration are in flight together
  const long long dfix = dact ? 0 : -(long long)dslot * 8;
  auto load_kv = [&](int tb, U16x8 (&kk)[U], U16x8 (&vv)[U]) {
    long long o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) o[u] = toff(min(tb + u * TPB, ce - 1)) + dfix;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      kk[u] = *reinterpret_cast<const U16x8*>(kb + o[u]);
      vv[u] = *reinterpret_cast<const U16x8*>(vb + o[u]);
    }
  };
  // PF (long splits, the standalone launch): the next iteration's K / V rows are requested before this
  // iteration's scores, so a split of many iterations streams instead of paying one round trip each
  U16x8 kr[U], vr[U];
  if (PF && ca + wid * TPW + tsub < ce) load_kv(ca + wid * TPW + tsub, kr, vr);
  for (int t0 = ca + wid * TPW + tsub; t0 < ce; t0 += TPB * U) {
    U16x8 kn[U], vn[U];
    if constexpr (PF) {
      if (t0 + TPB * U < ce) load_kv(t0 + TPB * U, kn, vn);
    } else {
      load_kv(t0, kr, vr);
    }
    // the U scores of this iteration are independent (their lane-group sums overlap), then ONE
    // online-softmax update folds them in: the dependent chain per iteration is one reduction and
    // one rescale, not U of each. Token t0 (u = 0) is always valid, so the running max is finite.
    float sv[G][U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * TPB;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d = fmaf(q[g][j], e2f<DT>(kr[u].v[j]), d);  // q == 0 on inactive lanes
        d = group_sum<LPT>(d);
        sv[g][u] = t < ce ? d + slope[g] * (float)(t - (L - 1)) : -INFINITY;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = sv[g][0];
#pragma unroll
      for (int u = 1; u < U; ++u) mx = fmaxf(mx, sv[g][u]);
      const float mn = fmaxf(m[g], mx);
      const float cs = __expf(m[g] - mn);
      float pu[U], ps = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pu[u] = __expf(sv[g][u] - mn);  // 0 for tokens past the split
        ps += pu[u];
      }
      l[g] = l[g] * cs + ps;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = acc[g][j] * cs;
#pragma unroll
        for (int u = 0; u < U; ++u) a = fmaf(pu[u], e2f<DT>(vr[u].v[j]), a);
        acc[g][j] = a;
      }
      m[g] = mn;
    }
    if constexpr (PF) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        kr[u] = kn[u];
        vr[u] = vn[u];
      }
    }
  }
  DSTAMP(4);
  // the last token, into lane group (wave 0, tsub 0): its lanes 0..ND-1 are the threads tid < ND
  // that hold its K / V slices (every LPT >= ND)
  if (own_last && wid == 0 && tsub == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float sv = 0.f;
      if (dact) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sv = fmaf(q[g][j], e2f<DT>(knraw.v[j]), sv);
      }
      sv = group_sum<LPT>(sv);
      const float mn = fmaxf(m[g], sv);
      const float cs = __expf(m[g] - mn), pv = __expf(sv - mn);
      l[g] = l[g] * cs + pv;
      if (dact) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] = fmaf(acc[g][j], cs, pv * e2f<DT>(vnraw.v[j]));
      }
      m[g] = mn;
    }
  }

  // ---- merge the lane groups: the TPW groups of a wave by shuffles, the 4 waves through LDS; then
  // write the split's (O, max, sum) or the final row
#pragma unroll
  for (int o = LPT; o < 64; o <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mo = __shfl_xor(m[g], o, 64), lo = __shfl_xor(l[g], o, 64);
      const float M = fmaxf(m[g], mo);
      const float wa = m[g] == -INFINITY ? 0.f : __expf(m[g] - M);
      const float wb = mo == -INFINITY ? 0.f : __expf(mo - M);
      l[g] = l[g] * wa + lo * wb;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] = acc[g][j] * wa + __shfl_xor(acc[g][j], o, 64) * wb;
      m[g] = M;
    }
  }
  float* gm = smem;            // [4][G]
  float* gl = gm + 4 * G;      // [4][G]
  float* gacc = gl + 4 * G;    // [4][G][D]
  if (lane == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      gm[wid * G + g] = m[g];
      gl[wid * G + g] = l[g];
    }
  }
  if (tsub == 0 && dact) {
#pragma unroll
    for (int g = 0; g < G; ++g) store8f(gacc + (long long)(wid * G + g) * D + dslot * 8, acc[g]);
  }
  __syncthreads();
  DSTAMP(5);
  for (int idx = tid; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) M = fmaxf(M, gm[r * G + g]);
    float Ls = 0.f, O = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mr = gm[r * G + g];
      const float w = mr == -INFINITY ? 0.f : __expf(mr - M);
      Ls = fmaf(w, gl[r * G + g], Ls);
      O = fmaf(w, gacc[(r * G + g) * D + d], O);
    }
    if (nsplit == 1) {
      store_out<DT>(p, b * p.o_bs + (long long)(hk * G + g) * D + d, Ls > 0.f ? O / Ls : 0.f);
    } else {
      st_pub(&p.ws_o[((bh0 + g) * nsplit + split) * D + d], O);
      if (d == 0) {
        st_pub(&p.ws_ml[((bh0 + g) * nsplit + split) * 2], M);
        st_pub(&p.ws_ml[((bh0 + g) * nsplit + split) * 2 + 1], Ls);
      }
    }
  }
  DSTAMP(6);
  } else {
    // short splits (one iteration of U tokens per lane group: every B=1 split): scores of the split
    // into LDS, a block-wide softmax, then P.V -- measured faster there than the online form's
    // dependent per-token updates (GPT-J B=1 decode 2.71 vs 2.80 ms/token, same box)
  // V rows of the first P.V iteration, issued together with the K loads: they do not depend on the
  // scores, so a chunk of <= TPB*U tokens (every B=1 split) costs one HBM round trip, not two
  const int tv0 = ca + wid * TPW + tsub;
  U16x8 vpre[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = tv0 + u * TPB;
    if (t < c1 && dact && !(own_new && t == pnew)) vpre[u] = *reinterpret_cast<const U16x8*>(vb + toff(t));
  }

  float* sc = smem;                 // [G][chunk]
  float* red = smem + G * p.chunk;  // [4][G][D]
  __shared__ float red_s[8];

  // ---- scores
  for (int t0 = ca + wid * TPW + tsub; t0 < c1; t0 += TPB * U) {
    float kr[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * TPB;
      if (t < c1 && dact) {
        if (own_new && t == pnew) {
#pragma unroll
          for (int j = 0; j < 8; ++j) kr[u][j] = knew[dslot * 8 + j];
        } else {
          load8_t<DT>(kb + toff(t), kr[u]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) kr[u][j] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * TPB;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = fmaf(q[g][j], kr[u][j], s);
#pragma unroll
        for (int o = 1; o < LPT; o <<= 1) s += __shfl_xor(s, o, 64);
        if (dslot == 0 && t < c1) sc[g * p.chunk + (t - ca)] = s + slope[g] * (float)(t - (L - 1));
      }
    }
  }
  __syncthreads();

  // ---- softmax over this chunk
  const int n = c1 - ca;
  float mg[G], lg[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float m = -INFINITY;
    for (int i = tid; i < n; i += 256) m = fmaxf(m, sc[g * p.chunk + i]);
    m = block_max(m, red_s);
    float l = 0.f;
    for (int i = tid; i < n; i += 256) {
      const float e = __expf(sc[g * p.chunk + i] - m);
      sc[g * p.chunk + i] = e;
      l += e;
    }
    l = block_sum(l, red_s);
    mg[g] = m;
    lg[g] = l;
  }
  __syncthreads();

  // ---- P.V
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  for (int t0 = tv0; t0 < c1; t0 += TPB * U) {
    float vr[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * TPB;
      if (t < c1 && dact) {
        if (own_new && t == pnew) {
#pragma unroll
          for (int j = 0; j < 8; ++j) vr[u][j] = vnew[dslot * 8 + j];
        } else if (t0 == tv0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) vr[u][j] = e2f<DT>(vpre[u].v[j]);
        } else {
          load8_t<DT>(vb + toff(t), vr[u]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) vr[u][j] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int t = t0 + u * TPB;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float pg = t < c1 ? sc[g * p.chunk + (t - ca)] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] = fmaf(pg, vr[u][j], acc[g][j]);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int o = LPT; o < 64; o <<= 1) acc[g][j] += __shfl_xor(acc[g][j], o, 64);
  if (tsub == 0 && dact) {
#pragma unroll
    for (int g = 0; g < G; ++g) store8f(red + (wid * G + g) * D + dslot * 8, acc[g]);
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    for (int d = tid; d < D; d += 256) {
      const float s = red[(0 * G + g) * D + d] + red[(1 * G + g) * D + d] +
                      red[(2 * G + g) * D + d] + red[(3 * G + g) * D + d];
      if (nsplit == 1) {
        store_out<DT>(p, b * p.o_bs + (long long)(hk * G + g) * D + d, lg[g] > 0.f ? s / lg[g] : 0.f);
      } else {
        st_pub(&p.ws_o[((bh0 + g) * nsplit + split) * D + d], s);
      }
    }
    if (nsplit > 1 && tid == 0) {
      st_pub(&p.ws_ml[((bh0 + g) * nsplit + split) * 2], mg[g]);
      st_pub(&p.ws_ml[((bh0 + g) * nsplit + split) * 2 + 1], lg[g]);
    }
  }
  }
  if (nsplit > 1 && p.cnt) fanin_combine<G, DT>(p, b, hk, nsplit);
}

template <int LPT, int G, bool PAGED, bool ONLINE, int DT = 0>
__global__ __launch_bounds__(256) void decode_attn_kernel(DecodeParams p) {
  // G == 1 only: the prefetched rows cost GQA groups a residency step (G = 2: 119 -> 135 VGPRs)
  decode_attn_body<LPT, G, PAGED, ONLINE, ONLINE && G == 1, DT>(p, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x);
}

// ---------------------------------------------------------------- fused decode layer (batch 1)
// A parallel-residual layer (GPT-J: h' = h + attn(LN h) + mlp(LN h)) at batch 1 is weight
// streaming plus a latency-bound attention chain. Two streams (attention on one, the MLP GEMVs on
// the other) overlap them but pay a cross-queue fork and join per layer (~10 us each in the graph
// timeline, profiles/decode_gptj_b1_timeline_r3.txt). One queue, three launches instead:
//   QKV GEMV  ->  decode_attn_gemv_kernel: workgroups [0, n_attn) run the RoPE + KV append +
//                 split-K attention, the rest the fc_in GEMV (+ GELU) -- the attention hides in the
//                 weight stream, dispatched first so it starts at once
//             ->  gemv_dual_ln_kernel: y = o Wout^T + g Wfc_out^T + b in one K-concatenated GEMV
//                 (two weight streams, one output), and the last workgroup to finish (arrival
//                 counter) adds y to the residual stream and normalises it for the next layer --
//                 no separate LayerNorm launch.
struct GemvM1 {
  const bf16_t* x;
  const bf16_t* w;
  const bf16_t* bias;
  bf16_t* y;
  int N, K, act;
};

template <int LPT, int G, bool PAGED, bool ONLINE, int DT = 0>
__global__ __launch_bounds__(256) void decode_attn_gemv_kernel(DecodeParams p, int nsplit, int n_attn, GemvM1 g) {
  constexpr int R = 4;
  __shared__ float part[4][R];
  const int bid = blockIdx.x;
  if (bid < n_attn) {
    const int split = bid % nsplit, rest = bid / nsplit;
    decode_attn_body<LPT, G, PAGED, ONLINE, false, DT>(p, split, rest % p.Hkv, rest / p.Hkv, nsplit);
    DSTAMP(7);
    return;
  }
  DSTAMP(0);
  const int n0 = (bid - n_attn) * R;
  float acc[R] = {0.f, 0.f, 0.f, 0.f};
  gemv_m1_accum<R, 0, DT>(g.x, g.w, g.N, g.K, n0, acc);
  const float v = gemv_m1_finish<R, DT>(acc, part, g.bias, n0, g.N, g.act);
  if (threadIdx.x < R && n0 + threadIdx.x < g.N) g.y[n0 + threadIdx.x] = (bf16_t)f2e<DT>(v);
  DSTAMP(7);
}

// Workgroup g: R rows over W1 . x1 (+ W2 . x2) -- one weight stream per row group, the shape the QKV
// GEMV reaches ~6 TB/s with; its R results go to ypart. The last workgroup to arrive (two-level
// counter) adds bias + residual, rounds h' to bf16 and normalises it for the next projection(s):
// the out-projection / fc_out, the residual add and the next LayerNorm in one launch, no LayerNorm
// launch of its own.
template <int R, int PER, int DT = 0>
__global__ __launch_bounds__(256) void gemv_dual_ln_kernel(DualLn a) {
  __shared__ float part[4][R];
  const int tid = threadIdx.x;
  // row groups g = blockIdx.x, + gridDim.x, ... (no workgroup waits on another: dispatch order does
  // not matter)
  const int ngrp = (a.N + R - 1) / R;
  for (int grp = blockIdx.x; grp < ngrp; grp += gridDim.x) {
    const int n0 = grp * R;
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.f;
    // (the two streams as two loops: one loop across the seam measured 1.5 us slower at GPT-J / NeoX
    // shapes, profiles/decode_launch_structure_ab_r5.txt)
    // 2 weight slabs in flight per lane (8 loads at 4 rows), not 16: 84 instead of 124 VGPRs, 5 instead
    // of 4 waves per SIMD -- BLOOM TP=8 B=1 9.36 -> 9.06 ms/token, GPT-J neutral
    // (profiles/decode_launch_structure_ab_r5.txt)
    gemv_m1_accum<R, 2, DT>(a.x1, a.w1, a.N, a.K1, n0, acc);
    if (a.x2) gemv_m1_accum<R, 2, DT>(a.x2, a.w2, a.N, a.K2, n0, acc);
    const float v = gemv_m1_finish<R, DT>(acc, part, nullptr, n0, a.N, 0);
    if (tid < R && n0 + tid < a.N) {  // this row's h' = bf16(h + y + bias), handed to the tail
      const int n = n0 + tid;
      st_pub_e<DT>(a.h_out + n, e2f<DT>(a.h[n]) + (v + (a.bias ? e2f<DT>(a.bias[n]) : 0.f)));
    }
    __syncthreads();  // part[] is rewritten by the next group
  }
  dual_ln_arrive_tail<PER, DT>(a);
}

// One workgroup per (sequence, head): split maxima and weights in one
// parallel pass into LDS, then every lane owns one output dim and sums the
// splits with 8 independent loads in flight (the old per-split serial chain
// of dependent L2 loads cost ~9 us per layer at B=1).
template <int DT = 0>
__global__ __launch_bounds__(256) void decode_combine_kernel(const float* __restrict__ ws_o,
                                                             const float* __restrict__ ws_ml,
                                                             bf16_t* __restrict__ out, long long o_bs,
                                                             int H, int D, int nsplit) {
  __shared__ float wsp[1024];
  __shared__ float red[8];
  const long long bh = blockIdx.x;
  const int b = (int)(bh / H), h = (int)(bh % H);
  const int tid = threadIdx.x;
  const float* ml = ws_ml + bh * nsplit * 2;
  const float* o = ws_o + bh * nsplit * D;
  // the first 16 splits' partial outputs of this lane's dim are requested together with the split
  // maxima (one memory round trip, not two: at B=1 every split count is <= 16..32)
  constexpr int PRE = 16;
  float opre[PRE];
  if (tid < D) {
#pragma unroll
    for (int s = 0; s < PRE; ++s) opre[s] = s < nsplit ? o[(long long)s * D + tid] : 0.f;
  }
  float m = -INFINITY;
  for (int s = tid; s < nsplit; s += 256) m = fmaxf(m, ml[2 * s]);
  const float M = block_max(m, red);
  float l = 0.f;
  for (int s = tid; s < nsplit; s += 256) {
    const float ms = ml[2 * s];
    const float w = ms == -INFINITY ? 0.f : __expf(ms - M);
    wsp[s] = w;
    l += w * ml[2 * s + 1];
  }
  const float Lsum = block_sum(l, red + 4);  // block_sum's barriers also publish wsp
  const float inv = Lsum > 0.f ? 1.f / Lsum : 0.f;
  if (tid < D) {  // D <= 256: one output dim per lane
    float acc = 0.f;
#pragma unroll
    for (int s = 0; s < PRE; ++s)  // an empty split's partial was never written: may hold NaN
      acc = (s < nsplit && wsp[s] > 0.f) ? fmaf(wsp[s], opre[s], acc) : acc;
#pragma unroll 8
    for (int s = PRE; s < nsplit; ++s) {
      const float ov = o[(long long)s * D + tid];
      acc = wsp[s] > 0.f ? fmaf(wsp[s], ov, acc) : acc;
    }
    out[b * o_bs + (long long)h * D + tid] = (bf16_t)f2e<DT>(acc * inv);
  }
}

// Split size (ops/decode.py:decode_chunk documents the cold-cache sweep behind it):
// ~256 (sequence, kv-head, split) workgroups of >= 64 tokens, one split for a cache
// of <= 256 tokens, splits of at most 256 tokens once the cache reaches 2048.
KCA_API int kca_decode_chunk(int B, int Hkv, int max_kv) {
  if (max_kv <= 256) return max(64, (max_kv + 31) / 32 * 32);
  const long long work = (long long)B * Hkv;
  const long long want = (256 + work - 1) / work;
  long long c = (max_kv + want - 1) / want;
  c = (c + 31) / 32 * 32;
  const long long cap = max_kv >= 2048 ? 256 : 1024;
  if (c > cap) c = cap;
  if (c < 64) c = 64;
  return (int)c;
}

// Fan-in counters live at the start of the workspace: B*H words (indexed by (sequence, kv-head)),
// padded to 16 B, that must be zero when the workspace is first used (the callers allocate it
// zeroed, ops/decode.py) and that every fan-in re-arms -- so concurrent launches on separate
// workspaces never share a counter. KCA_DECODE_FANIN=0 selects the separate combine kernel.
static bool fanin_enabled() {
  static int enabled = -1;
  if (enabled < 0) {
    const char* e = getenv("KCA_DECODE_FANIN");
    enabled = !(e && e[0] == '0');
  }
  return enabled;
}
static long long fanin_words(int B, int H) { return ((long long)B * H + 3) / 4 * 4; }

KCA_API long long kca_decode_ws_floats(int B, int H, int D, int max_kv, int chunk) {
  const long long ns = (max_kv + chunk - 1) / chunk;
  return ns > 1 ? fanin_words(B, H) + (long long)B * H * ns * (D + 2) : 0;
}

template <int LPT, int G, int DT = 0>
static void launch_decode(const DecodeParams& p, int B, int nsplit, hipStream_t stream) {
  constexpr int TPB = 4 * (64 / LPT), U = 4;
  const dim3 grid(nsplit, p.Hkv, B);
  if (p.chunk > TPB * U) {  // long splits: one pass with online softmax
    const size_t lds = (size_t)4 * G * (2 + p.D) * sizeof(float);
    if (p.tbl) hipLaunchKernelGGL((decode_attn_kernel<LPT, G, true, true, DT>), grid, dim3(256), lds, stream, p);
    else hipLaunchKernelGGL((decode_attn_kernel<LPT, G, false, true, DT>), grid, dim3(256), lds, stream, p);
  } else {
    const size_t lds = (size_t)(G * p.chunk + 4 * G * p.D) * sizeof(float);
    if (p.tbl) hipLaunchKernelGGL((decode_attn_kernel<LPT, G, true, false, DT>), grid, dim3(256), lds, stream, p);
    else hipLaunchKernelGGL((decode_attn_kernel<LPT, G, false, false, DT>), grid, dim3(256), lds, stream, p);
  }
}

template <int LPT, int DT = 0>
static int launch_decode_g(const DecodeParams& p, int G, int B, int nsplit, hipStream_t s) {
  switch (G) {
    case 1: launch_decode<LPT, 1, DT>(p, B, nsplit, s); return 0;
    case 2: launch_decode<LPT, 2, DT>(p, B, nsplit, s); return 0;
    case 4: launch_decode<LPT, 4, DT>(p, B, nsplit, s); return 0;
    case 8: launch_decode<LPT, 8, DT>(p, B, nsplit, s); return 0;
  }
  return 3;
}

static int decode_attn_launch(DecodeParams p, float* ws, long long ws_floats, int B, int max_kv, int chunk,
                              hipStream_t stream, int dt = 0);

KCA_API int kca_decode_attn(const void* q, long long q_bs, const void* kc, const void* vc,
                            long long cs_slot, long long cs_head, long long cs_pos,
                            const int* slots, const int* kv_lens, void* out, long long o_bs,
                            float* ws, long long ws_floats, int B, int H, int Hkv, int D,
                            int max_kv, int chunk, float scale, const float* alibi, const int* tbl,
                            int tbl_stride, int ps_shift, int window, hipStream_t stream) {
  if (window < 0) return 9;
  DecodeParams p{(const bf16_t*)q, q_bs, (const bf16_t*)kc, (const bf16_t*)vc, cs_slot, cs_head,
                 cs_pos, slots, kv_lens, (bf16_t*)out, o_bs, nullptr, nullptr, alibi, tbl, tbl_stride, ps_shift,
                 H, Hkv, D, chunk, scale, 0, 0, 0, nullptr, nullptr, g_decode_stamps, nullptr, window};
  return decode_attn_launch(p, ws, ws_floats, B, max_kv, chunk, stream);
}

// Fused decode prep + attention: qkv is the fused QKV GEMM output [B, (H+2Hkv)*D]
// (row stride ld); RoPE (rot dims, GPT-J interleaved or NeoX rotate-half) of the
// new token at position kv_lens[b]-1, its K/V appended to the cache, then the
// split-K attention -- replaces kca_decode_prep + kca_decode_attn.
KCA_API int kca_decode_prep_attn(const void* qkv, long long ld, const void* kc, const void* vc,
                                 long long cs_slot, long long cs_head, long long cs_pos,
                                 const int* slots, const int* kv_lens, void* out, long long o_bs,
                                 float* ws, long long ws_floats, int B, int H, int Hkv, int D,
                                 int max_kv, int chunk, float scale, const float* alibi, const int* tbl,
                                 int tbl_stride, int ps_shift, int rot, int interleaved, const float* cos_t,
                                 const float* sin_t, int window, int by_row, hipStream_t stream) {
  if (rot > D || (rot & 1) || (rot > 0 && (!cos_t || !sin_t))) return 8;
  if (window < 0) return 9;
  DecodeParams p{(const bf16_t*)qkv, ld, (const bf16_t*)kc, (const bf16_t*)vc, cs_slot, cs_head,
                 cs_pos, slots, kv_lens, (bf16_t*)out, o_bs, nullptr, nullptr, alibi, tbl, tbl_stride, ps_shift,
                 H, Hkv, D, chunk, scale, 1, rot, interleaved, cos_t, sin_t, g_decode_stamps, nullptr, window};
  p.by_row = by_row;  // per-step RoPE / page rows (see DecodeParams::by_row)
  return decode_attn_launch(p, ws, ws_floats, B, max_kv, chunk, stream);
}

// kca_decode_prep_attn on fp16 rows / caches (the precision FT and DS-Inference serve, BASELINE
// config 4): the same kernels instantiated with fp16 loads, RoPE rounding and stores.
KCA_API int kca_decode_prep_attn_f16(const void* qkv, long long ld, const void* kc, const void* vc,
                                     long long cs_slot, long long cs_head, long long cs_pos,
                                     const int* slots, const int* kv_lens, void* out, long long o_bs,
                                     float* ws, long long ws_floats, int B, int H, int Hkv, int D,
                                     int max_kv, int chunk, float scale, const float* alibi, const int* tbl,
                                     int tbl_stride, int ps_shift, int rot, int interleaved, const float* cos_t,
                                     const float* sin_t, int window, int by_row, hipStream_t stream) {
  if (rot > D || (rot & 1) || (rot > 0 && (!cos_t || !sin_t))) return 8;
  if (window < 0) return 9;
  DecodeParams p{(const bf16_t*)qkv, ld, (const bf16_t*)kc, (const bf16_t*)vc, cs_slot, cs_head,
                 cs_pos, slots, kv_lens, (bf16_t*)out, o_bs, nullptr, nullptr, alibi, tbl, tbl_stride, ps_shift,
                 H, Hkv, D, chunk, scale, 1, rot, interleaved, cos_t, sin_t, g_decode_stamps, nullptr, window};
  p.by_row = by_row;
  return decode_attn_launch(p, ws, ws_floats, B, max_kv, chunk, stream, 1);
}

static int decode_attn_launch(DecodeParams p, float* ws, long long ws_floats, int B, int max_kv, int chunk,
                              hipStream_t stream, int dt) {
  const int H = p.H, Hkv = p.Hkv, D = p.D;
  const int* tbl = p.tbl;
  const int ps_shift = p.ps_shift, tbl_stride = p.tbl_stride;
  if (D % 8 || D > 256 || H % Hkv || B <= 0 || max_kv <= 0) return 1;
  if (tbl && (ps_shift < 4 || ps_shift > 20 || tbl_stride <= 0)) return 5;  // pages of >= 16 tokens
  if (chunk <= 0) chunk = kca_decode_chunk(B, Hkv, max_kv);
  const int G = H / Hkv;
  if (tbl && chunk > 1024) return 6;  // the LDS page-id stage holds 1024 tokens of pages
  const int nsplit = (max_kv + chunk - 1) / chunk;
  if (nsplit > 1024) return 7;  // combine keeps the split weights in LDS
  p.chunk = chunk;
  if (nsplit > 1) {
    const long long cw = fanin_words(B, H);
    const long long need = cw + (long long)B * H * nsplit * (D + 2);
    if (!ws || ws_floats < need) return 4;
    if (fanin_enabled()) p.cnt = reinterpret_cast<unsigned int*>(ws);
    p.ws_o = ws + cw;
    p.ws_ml = p.ws_o + (long long)B * H * nsplit * D;
  }
  const int nd = D / 8;
  int rc;
  if (dt == 1) {
    if (nd <= 8) rc = launch_decode_g<8, 1>(p, G, B, nsplit, stream);
    else if (nd <= 16) rc = launch_decode_g<16, 1>(p, G, B, nsplit, stream);
    else rc = launch_decode_g<32, 1>(p, G, B, nsplit, stream);
  } else {
    if (nd <= 8) rc = launch_decode_g<8>(p, G, B, nsplit, stream);
    else if (nd <= 16) rc = launch_decode_g<16>(p, G, B, nsplit, stream);
    else rc = launch_decode_g<32>(p, G, B, nsplit, stream);
  }
  if (rc) return rc;
  if (nsplit > 1 && !p.cnt) {
    if (dt == 1)
      hipLaunchKernelGGL((decode_combine_kernel<1>), dim3(B * H), dim3(256), 0, stream, p.ws_o, p.ws_ml, p.out,
                         p.o_bs, H, D, nsplit);
    else
      hipLaunchKernelGGL((decode_combine_kernel<0>), dim3(B * H), dim3(256), 0, stream, p.ws_o, p.ws_ml, p.out,
                         p.o_bs, H, D, nsplit);
  }
  return 0;
}

// Fused decode layer, part 1 (batch 1, see decode_attn_gemv_kernel): kca_decode_prep_attn's
// arguments plus the fc_in GEMV (gx [gK] -> gy [gN], bias, act). Returns 10 when the shape is
// outside the instantiated fused variants (G == 1, head_dim 128 / 256, split-K fan-in or one
// split): the caller then runs the two-stream path.
template <int DT>
static int prep_attn_gemv(const void* qkv, long long ld, const void* kc, const void* vc, long long cs_slot,
                          long long cs_head, long long cs_pos, const int* slots, const int* kv_lens, void* out,
                          long long o_bs, float* ws, long long ws_floats, int B, int H, int Hkv, int D, int max_kv,
                          int chunk, float scale, const float* alibi, const int* tbl, int tbl_stride, int ps_shift,
                          int rot, int interleaved, const float* cos_t, const float* sin_t, int window,
                          const void* gx, const void* gw, const void* gbias, void* gy, int gN, int gK, int gact,
                          int by_row, hipStream_t stream) {
  if (rot > D || (rot & 1) || (rot > 0 && (!cos_t || !sin_t))) return 8;
  if (window < 0) return 9;
  if (B != 1 || H != Hkv || D % 8 || D > 256 || max_kv <= 0 || gK % 8 || gN <= 0) return 10;
  const int nd = D / 8;
  if (nd <= 8) return 10;
  if (((uintptr_t)gx | (uintptr_t)gw) & 15) return 10;
  DecodeParams p{(const bf16_t*)qkv, ld, (const bf16_t*)kc, (const bf16_t*)vc, cs_slot, cs_head,
                 cs_pos, slots, kv_lens, (bf16_t*)out, o_bs, nullptr, nullptr, alibi, tbl, tbl_stride, ps_shift,
                 H, Hkv, D, chunk, scale, 1, rot, interleaved, cos_t, sin_t, g_decode_stamps, nullptr, window};
  p.by_row = by_row;
  if (tbl && (ps_shift < 4 || ps_shift > 20 || tbl_stride <= 0)) return 5;
  if (chunk <= 0) chunk = kca_decode_chunk(B, Hkv, max_kv);
  if (tbl && chunk > 1024) return 6;
  const int nsplit = (max_kv + chunk - 1) / chunk;
  if (nsplit > 1024) return 7;
  p.chunk = chunk;
  if (nsplit > 1) {
    if (!fanin_enabled()) return 10;  // the fused launch has no room for the separate combine kernel
    const long long cw = fanin_words(B, H);
    const long long need = cw + (long long)B * H * nsplit * (D + 2);
    if (!ws || ws_floats < need) return 4;
    p.cnt = reinterpret_cast<unsigned int*>(ws);
    p.ws_o = ws + cw;
    p.ws_ml = p.ws_o + (long long)B * H * nsplit * D;
  }
  const GemvM1 g{(const bf16_t*)gx, (const bf16_t*)gw, (const bf16_t*)gbias, (bf16_t*)gy, gN, gK, gact};
  const int n_attn = nsplit * Hkv * B;
  const dim3 grid(n_attn + (gN + 3) / 4);
  auto go = [&](auto lpt) {
    constexpr int LPT = decltype(lpt)::value;
    constexpr int TPB = 4 * (64 / LPT), U = 4;
    if (p.chunk > TPB * U) {
      const size_t lds = (size_t)4 * (2 + p.D) * sizeof(float);
      if (p.tbl) hipLaunchKernelGGL((decode_attn_gemv_kernel<LPT, 1, true, true, DT>), grid, dim3(256), lds, stream, p, nsplit, n_attn, g);
      else hipLaunchKernelGGL((decode_attn_gemv_kernel<LPT, 1, false, true, DT>), grid, dim3(256), lds, stream, p, nsplit, n_attn, g);
    } else {
      const size_t lds = (size_t)(p.chunk + 4 * p.D) * sizeof(float);
      if (p.tbl) hipLaunchKernelGGL((decode_attn_gemv_kernel<LPT, 1, true, false, DT>), grid, dim3(256), lds, stream, p, nsplit, n_attn, g);
      else hipLaunchKernelGGL((decode_attn_gemv_kernel<LPT, 1, false, false, DT>), grid, dim3(256), lds, stream, p, nsplit, n_attn, g);
    }
  };
  if (nd <= 16) go(std::integral_constant<int, 16>{});
  else go(std::integral_constant<int, 32>{});
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

KCA_API int kca_decode_prep_attn_gemv(const void* qkv, long long ld, const void* kc, const void* vc,
                                      long long cs_slot, long long cs_head, long long cs_pos,
                                      const int* slots, const int* kv_lens, void* out, long long o_bs,
                                      float* ws, long long ws_floats, int B, int H, int Hkv, int D,
                                      int max_kv, int chunk, float scale, const float* alibi, const int* tbl,
                                      int tbl_stride, int ps_shift, int rot, int interleaved, const float* cos_t,
                                      const float* sin_t, int window, const void* gx, const void* gw,
                                      const void* gbias, void* gy, int gN, int gK, int gact, int by_row,
                                      hipStream_t stream) {
  return prep_attn_gemv<0>(qkv, ld, kc, vc, cs_slot, cs_head, cs_pos, slots, kv_lens, out, o_bs, ws, ws_floats, B,
                           H, Hkv, D, max_kv, chunk, scale, alibi, tbl, tbl_stride, ps_shift, rot, interleaved,
                           cos_t, sin_t, window, gx, gw, gbias, gy, gN, gK, gact, by_row, stream);
}

// fp16 twin (same arguments; qkv / caches / out / gx / gw / gbias / gy fp16)
KCA_API int kca_decode_prep_attn_gemv_f16(const void* qkv, long long ld, const void* kc, const void* vc,
                                          long long cs_slot, long long cs_head, long long cs_pos,
                                          const int* slots, const int* kv_lens, void* out, long long o_bs,
                                          float* ws, long long ws_floats, int B, int H, int Hkv, int D,
                                          int max_kv, int chunk, float scale, const float* alibi, const int* tbl,
                                          int tbl_stride, int ps_shift, int rot, int interleaved,
                                          const float* cos_t, const float* sin_t, int window, const void* gx,
                                          const void* gw, const void* gbias, void* gy, int gN, int gK, int gact,
                                          int by_row, hipStream_t stream) {
  return prep_attn_gemv<1>(qkv, ld, kc, vc, cs_slot, cs_head, cs_pos, slots, kv_lens, out, o_bs, ws, ws_floats, B,
                           H, Hkv, D, max_kv, chunk, scale, alibi, tbl, tbl_stride, ps_shift, rot, interleaved,
                           cos_t, sin_t, window, gx, gw, gbias, gy, gN, gK, gact, by_row, stream);
}

// Fused decode layer, tail: y = x1 W1^T (+ x2 W2^T) + bias ([N]), h_out = bf16(h + y), xn_out =
// LN(h_out) (gamma, beta, eps) and, with gamma2, xn2_out = the second LayerNorm of h_out (same
// statistics). x2 / w2 nullable (K2 = 0: one GEMV -- a sequential-residual layer's out-projection or
// fc_out). ypart: >= N fp32 words; cnt: 32 * (1 + kDualSub) zero-initialised unsigned counters
// (re-armed by every launch).
// Geometry: 4 weight rows per workgroup, one workgroup per row group (8 or 16 rows measured equal or
// slower inside the decode steps; a grid capped at one residency round slower:
// profiles/decode_launch_structure_ab_r5.txt).
template <int DT>
static int gemv_dual_ln(const void* x1, const void* w1, int K1, const void* x2, const void* w2, int K2,
                        const void* bias, float* ypart, unsigned int* cnt, const void* h, void* h_out,
                        const void* gamma, const void* beta, float eps, void* xn_out, const void* gamma2,
                        const void* beta2, void* xn2_out, int N, hipStream_t stream) {
  if (N <= 0 || N % 8 || N > 16384 || K1 % 8 || K1 <= 0 || !ypart || !cnt || !gamma || !xn_out || !h || !h_out)
    return 1;
  if (x2 && (K2 <= 0 || K2 % 8 || !w2)) return 1;
  if (xn2_out && !gamma2) return 1;
  if (((uintptr_t)x1 | (uintptr_t)w1 | (uintptr_t)x2 | (uintptr_t)w2 | (uintptr_t)h | (uintptr_t)h_out |
       (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)xn_out | (uintptr_t)ypart | (uintptr_t)gamma2 |
       (uintptr_t)beta2 | (uintptr_t)xn2_out) & 15)
    return 2;
  const DualLn a{(const bf16_t*)x1, (const bf16_t*)w1, (const bf16_t*)x2, (const bf16_t*)w2, (const bf16_t*)bias,
                 ypart, cnt, (const bf16_t*)h, (bf16_t*)h_out, (const bf16_t*)gamma, (const bf16_t*)beta, eps,
                 (bf16_t*)xn_out, (const bf16_t*)gamma2, (const bf16_t*)beta2, (bf16_t*)xn2_out,
                 N, K1, x2 ? K2 : 0};
  const dim3 grid((unsigned)((N + 3) / 4));
  if (N <= 8192) hipLaunchKernelGGL((gemv_dual_ln_kernel<4, 4, DT>), grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((gemv_dual_ln_kernel<4, 8, DT>), grid, dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

KCA_API int kca_gemv_dual_ln(const void* x1, const void* w1, int K1, const void* x2, const void* w2, int K2,
                             const void* bias, float* ypart, unsigned int* cnt, const void* h, void* h_out,
                             const void* gamma, const void* beta, float eps, void* xn_out, const void* gamma2,
                             const void* beta2, void* xn2_out, int N, hipStream_t stream) {
  return gemv_dual_ln<0>(x1, w1, K1, x2, w2, K2, bias, ypart, cnt, h, h_out, gamma, beta, eps, xn_out, gamma2,
                         beta2, xn2_out, N, stream);
}

// fp16 twin (same arguments)
KCA_API int kca_gemv_dual_ln_f16(const void* x1, const void* w1, int K1, const void* x2, const void* w2, int K2,
                                 const void* bias, float* ypart, unsigned int* cnt, const void* h, void* h_out,
                                 const void* gamma, const void* beta, float eps, void* xn_out, const void* gamma2,
                                 const void* beta2, void* xn2_out, int N, hipStream_t stream) {
  return gemv_dual_ln<1>(x1, w1, K1, x2, w2, K2, bias, ypart, cnt, h, h_out, gamma, beta, eps, xn_out, gamma2,
                         beta2, xn2_out, N, stream);
}

// --------------------------------------------------------------- sampling
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ uint32_t fkey(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int SAMPLE_THREADS = 1024;
constexpr int SAMPLE_CMAX = 2048;  // top-k survivors held in LDS (compact mode)
constexpr int SAMPLE_UN = 8;       // loads in flight per thread in the vocabulary passes

// f(i, x[i]) for i = tid, tid + T, ... < n (increasing i per thread), SAMPLE_UN loads issued before
// any is used: ONE workgroup walks the whole vocabulary, so a load-use-load loop is latency bound
// (~50 dependent L2 round trips per pass at V = 50400)
template <typename F>
__device__ __forceinline__ void vocab_pass(const float* __restrict__ x, int n, F&& f) {
  for (int base = threadIdx.x; base < n; base += SAMPLE_THREADS * SAMPLE_UN) {
    float v[SAMPLE_UN];
#pragma unroll
    for (int u = 0; u < SAMPLE_UN; ++u) {
      const int i = base + u * SAMPLE_THREADS;
      v[u] = i < n ? x[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < SAMPLE_UN; ++u) {
      const int i = base + u * SAMPLE_THREADS;
      if (i < n) f(i, v[u]);
    }
  }
}

// Wave 0 scans the 256-bin histogram from the top bin down and finds the bin in
// which the running total first reaches `target` (excl < target <= incl).
// Writes bin/excl to sh[0..1]; bin = -1 if not reached.
__device__ void find_bin_desc(const float* hist, float target, float* sh_excl, int* sh_bin) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    float v[4], loc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = hist[255 - 4 * lane - i];
      loc += v[i];
    }
    float incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    float excl = incl - loc;
    if (lane == 0) *sh_bin = -1;
    // the (unique) lane whose range contains the crossing
    const bool mine = excl < target && target <= incl;
    const unsigned long long bal = __ballot(mine);
    const int first = bal ? __ffsll((long long)bal) - 1 : -1;
    if (lane == first) {
      float run = excl;
      int bin = 255 - 4 * lane - 3;
      for (int i = 0; i < 4; ++i) {
        if (run + v[i] >= target && v[i] > 0.f) {
          bin = 255 - 4 * lane - i;
          break;
        }
        run += v[i];
      }
      *sh_bin = bin;
      *sh_excl = run;
    }
  }
  __syncthreads();
}

// One workgroup per row. ws: fp32 scratch [B, V] (processed logits).
// rows of the multi-workgroup sampler (sample_mwg_kernel): greedy, top-k in [1, 64], or top-p only
// (top-k off, top_p < 1). A top-p-only row's merge falls back -- out_ids[b] = -1 -- when its candidates
// do not hold the nucleus; the one-workgroup kernel launched after it then takes the row (mwg_took).
constexpr int MWG_KMAX_ = 64;  // (= MWG_KMAX below)
__device__ __forceinline__ bool mwg_row(float T, int k, float p) {
  return !(T > 0.f) || (k >= 1 && k <= MWG_KMAX_) || (k <= 0 && p < 1.f);
}
__device__ __forceinline__ bool mwg_took(float T, int k, float p, const long long* out_ids, int b) {
  if (!mwg_row(T, k, p)) return false;
  return !(T > 0.f && k <= 0) || out_ids[b] >= 0;
}

__global__ __launch_bounds__(SAMPLE_THREADS) void sample_kernel(
    const void* __restrict__ logits, long long ld, int is_bf16, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const float* __restrict__ rep_pen, uint8_t* __restrict__ seen,
    const int* __restrict__ slots, const int* __restrict__ ban_ids, int n_ban,
    const unsigned long long* __restrict__ seeds, long long step, float* __restrict__ ws,
    long long* __restrict__ out_ids, float* __restrict__ out_lp, int* __restrict__ out_kept, int compact,
    int skip_mwg) {
  __shared__ float hist[256];
  __shared__ float red[SAMPLE_THREADS / 64];
  __shared__ float sh_excl;
  __shared__ int sh_bin;
  __shared__ float scan[SAMPLE_THREADS / 64];
  __shared__ int sh_idx;
  __shared__ float c_v[SAMPLE_CMAX];  // top-k survivors, index order (compact mode)
  __shared__ int c_i[SAMPLE_CMAX];
  __shared__ int iscan[SAMPLE_THREADS / 64];
  const int b = blockIdx.x, tid = threadIdx.x;
  // rows the multi-workgroup sampler took (launched first): decided on the device, as sample_reg_kernel
  if (skip_mwg && mwg_took(temperature ? temperature[b] : 1.f, top_k ? top_k[b] : 0, top_p ? top_p[b] : 1.f,
                           out_ids, b))
    return;
  const float T = temperature ? temperature[b] : 1.f;
  const float rp = rep_pen ? rep_pen[b] : 1.f;
  const int slot = slots ? slots[b] : b;
  const uint8_t* sn = seen ? seen + (long long)slot * V : nullptr;
  float* x = ws + (long long)b * V;
  const bool greedy = !(T > 0.f);
  const float inv_t = (greedy || T == 1.f) ? 1.f : 1.f / T;

  // pass 1: penalties + temperature -> ws
  const bool pen = rp != 1.f && sn;
  for (int base = tid; base < V; base += SAMPLE_THREADS * SAMPLE_UN) {
    float v[SAMPLE_UN];
    uint8_t sv[SAMPLE_UN];
#pragma unroll
    for (int u = 0; u < SAMPLE_UN; ++u) {
      const int i = base + u * SAMPLE_THREADS;
      v[u] = 0.f;
      sv[u] = 0;
      if (i < V) {
        // is_bf16: the logits' dtype -- 0 fp32, 1 bf16, 2 fp16
        v[u] = is_bf16 == 1 ? bf2f(((const bf16_t*)logits)[b * ld + i])
               : (is_bf16 == 2 ? e2f<1>(((const bf16_t*)logits)[b * ld + i]) : ((const float*)logits)[b * ld + i]);
        if (pen) sv[u] = sn[i];
      }
    }
#pragma unroll
    for (int u = 0; u < SAMPLE_UN; ++u) {
      const int i = base + u * SAMPLE_THREADS;
      float w = v[u];
      if (sv[u]) w = w < 0.f ? w * rp : w / rp;
      if (i < V) x[i] = w * inv_t;
    }
  }
  __syncthreads();
  if (ban_ids)
    for (int j = tid; j < n_ban; j += SAMPLE_THREADS) {
      const int id = ban_ids[(long long)b * n_ban + j];
      if (id >= 0 && id < V) x[id] = -INFINITY;
    }
  __syncthreads();

  // pass 2: max (+ argmax) and softmax normaliser
  float m = -INFINITY, s = 0.f;
  int am = 0x7fffffff;
  vocab_pass(x, V, [&](int i, float v) {
    if (v > m) {
      s = s * __expf(m - v) + 1.f;
      m = v;
      am = i;
    } else if (v != -INFINITY) {
      s += __expf(v - m);
    }
  });
  const float M = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float Z = block_sum(s, red);
  const float lZ = M + __logf(Z);
  if (greedy) {
    int cand = (m == M) ? am : 0x7fffffff;
    // first occurrence: block min of candidate indices
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = __int_as_float(cand);
    __syncthreads();
    if (tid == 0) {
      int best = 0x7fffffff;
      for (int w = 0; w < SAMPLE_THREADS / 64; ++w) best = min(best, __float_as_int(red[w]));
      out_ids[b] = best;
      if (out_lp) out_lp[b] = x[best] - lZ;
      if (seen) seen[(long long)slot * V + best] = 1;
      if (out_kept) out_kept[b] = 1;
    }
    return;
  }

  // top-k: radix select of the k-th largest key (ties at the threshold kept, as
  // HF's `logits < topk(...)[-1]` mask does)
  uint32_t thr = 0;
  const int k = top_k ? top_k[b] : 0;
  if (k > 0 && k < V) {
    uint32_t prefix = 0, mask = 0;
    float remaining = (float)k;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += SAMPLE_THREADS) hist[i] = 0.f;
      __syncthreads();
      vocab_pass(x, V, [&](int, float v) {
        const uint32_t key = fkey(v);
        if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1.f);
      });
      __syncthreads();
      find_bin_desc(hist, remaining, &sh_excl, &sh_bin);
      const int bin = sh_bin;
      if (bin < 0) break;
      prefix |= (uint32_t)bin << shift;
      mask |= 255u << shift;
      remaining -= sh_excl;
      __syncthreads();
    }
    thr = prefix;
  }
  // compact mode: after a top-k select the survivors (k + ties) move to LDS in index order, so the
  // top-p select and the multinomial below scan them instead of V (5 of the kernel's ~11 passes
  // over the vocabulary); the index order keeps the multinomial's cumulative order unchanged
  int nc = V;
  bool cmp = false;
  if (compact && k > 0 && k < V) {
    const int sg = (V + SAMPLE_THREADS - 1) / SAMPLE_THREADS;
    const int l0 = min(V, tid * sg), l1 = min(V, l0 + sg);
    int cnt = 0;
#pragma unroll 8
    for (int i = l0; i < l1; ++i) {
      const float v = x[i];
      cnt += (v != -INFINITY && fkey(v) >= thr) ? 1 : 0;
    }
    const int lane_ = tid & 63, wid_ = tid >> 6;
    int inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane_ >= o) inc += t;
    }
    if (lane_ == 63) iscan[wid_] = inc;
    __syncthreads();
    int off = inc - cnt, tot = 0;
    for (int w = 0; w < SAMPLE_THREADS / 64; ++w) {
      if (w < wid_) off += iscan[w];
      tot += iscan[w];
    }
    if (tot <= SAMPLE_CMAX) {
      for (int i = l0; i < l1 && cnt > 0; ++i) {
        const float v = x[i];
        if (v != -INFINITY && fkey(v) >= thr) {
          c_v[off] = v;
          c_i[off] = i;
          ++off;
          --cnt;
        }
      }
      nc = tot;
      cmp = true;
    }
    __syncthreads();
  }
  // top-p: smallest key whose inclusive descending mass reaches p (HF keeps the
  // tokens whose ascending cumulative probability exceeds 1-p)
  const float pp = top_p ? top_p[b] : 1.f;
  if (pp < 1.f) {
    uint32_t prefix = 0, mask = 0;
    float above = 0.f, target = 0.f;
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int i = tid; i < 256; i += SAMPLE_THREADS) hist[i] = 0.f;
      __syncthreads();
      vocab_pass(cmp ? c_v : x, nc, [&](int, float v) {
        const uint32_t key = fkey(v);
        if (key >= thr && (key & mask) == prefix && v != -INFINITY)
          atomicAdd(&hist[(key >> shift) & 255], __expf(v - M));
      });
      __syncthreads();
      if (shift == 24) {  // total kept mass after top-k
        float t = 0.f;
        for (int i = tid; i < 256; i += SAMPLE_THREADS) t += hist[i];
        target = pp * block_sum(t, red);
      }
      find_bin_desc(hist, target - above, &sh_excl, &sh_bin);
      const int bin = sh_bin;
      if (bin < 0) {  // rounding: target not reached -> keep everything so far
        prefix = 0;
        mask = 0;
        break;
      }
      prefix |= (uint32_t)bin << shift;
      mask |= 255u << shift;
      above += sh_excl;
      __syncthreads();
    }
    if (mask == 0xffffffffu && prefix > thr) thr = prefix;
  }

  // multinomial over kept tokens in index order: segment sums + block scan
  const int seg = (nc + SAMPLE_THREADS - 1) / SAMPLE_THREADS;
  const int lo = min(nc, tid * seg), hi = min(nc, lo + seg);
  float ssum = 0.f;
  int kept = 0;
#pragma unroll 8
  for (int i = lo; i < hi; ++i) {
    const float v = cmp ? c_v[i] : x[i];
    if (v != -INFINITY && fkey(v) >= thr) {
      ssum += __expf(v - M);
      ++kept;
    }
  }
  // inclusive scan of ssum across the block
  const int lane = tid & 63, wid = tid >> 6;
  float incl = ssum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  __syncthreads();
  if (lane == 63) scan[wid] = incl;
  __syncthreads();
  float woff = 0.f, total = 0.f;
  for (int w = 0; w < SAMPLE_THREADS / 64; ++w) {
    if (w < wid) woff += scan[w];
    total += scan[w];
  }
  incl += woff;
  const float excl = incl - ssum;
  int kept_tot = kept;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kept_tot += __shfl_xor(kept_tot, o, 64);
  __syncthreads();
  if (lane == 0) red[wid] = __int_as_float(kept_tot);
  if (tid == 0) sh_idx = -1;
  __syncthreads();
  // counter = (row if no per-row seeds, step); per-row seeds make a request's
  // stream independent of the batch row it happens to occupy
  uint32_t c[4] = {seeds ? 0u : (uint32_t)b, (uint32_t)step,
                   (uint32_t)((unsigned long long)step >> 32), 0x5eedu};
  const unsigned long long sd = seeds ? seeds[b] : 0ull;
  philox4x32_10(c, (uint32_t)sd, (uint32_t)(sd >> 32));
  const float r = ((c[0] >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
  const float u = r * total;
  if (ssum > 0.f && excl < u && u <= incl) {
    float run = excl;
    int pick = -1;
    for (int i = lo; i < hi; ++i) {
      const float v = cmp ? c_v[i] : x[i];
      if (v != -INFINITY && fkey(v) >= thr) {
        pick = cmp ? c_i[i] : i;
        run += __expf(v - M);
        if (run >= u) break;
      }
    }
    atomicMax(&sh_idx, pick);
  }
  __syncthreads();
  if (tid == 0) {
    int id = sh_idx;
    if (id < 0) {  // float rounding at the very top of the range: last kept token
      for (int i = nc - 1; i >= 0; --i) {
        const float v = cmp ? c_v[i] : x[i];
        if (v != -INFINITY && fkey(v) >= thr) {
          id = cmp ? c_i[i] : i;
          break;
        }
      }
      if (id < 0) id = 0;
    }
    out_ids[b] = id;
    if (out_lp) out_lp[b] = x[id] - lZ;
    if (seen) seen[(long long)slot * V + id] = 1;
    if (out_kept) {
      int kt = 0;
      for (int w = 0; w < SAMPLE_THREADS / 64; ++w) kt += __float_as_int(red[w]);
      out_kept[b] = kt;
    }
  }
}


// Register-resident sampler (bf16 logits, V <= RPT * 1024, GPT-J's 50400 at 128 per thread x 512 threads): the row is read
// ONCE into registers (element i = u * 1024 + tid, value u of the thread) and every later pass -- max / normaliser, the top-k
// and top-p radix selects, the multinomial -- runs on registers and LDS histograms, not on a fp32
// copy re-read from memory: one workgroup walking the vocabulary from L2 was ~15-20 us per pass.
// Same selection semantics as sample_kernel (ties at the top-k / top-p thresholds kept, first index
// for greedy); the multinomial's cumulative order is thread-major (tid, then u), fixed per seed.
template <int RPT, int NT>
__global__ __launch_bounds__(NT) void sample_reg_kernel(
    const void* __restrict__ logits, long long ld, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const float* __restrict__ rep_pen, uint8_t* __restrict__ seen,
    const int* __restrict__ slots, const int* __restrict__ ban_ids, int n_ban,
    const unsigned long long* __restrict__ seeds, long long step,
    long long* __restrict__ out_ids, float* __restrict__ out_lp, int* __restrict__ out_kept, int skip_mwg) {
  __shared__ float hist[16];
  __shared__ float red[NT / 64];
  __shared__ float scan[NT / 64];
  __shared__ int sh_key;
  __shared__ uint32_t cnt16[NT / 64 * 8];
  __shared__ int tot16[16];
  __shared__ int sel[2];
  __shared__ float selp[2];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float T = temperature ? temperature[b] : 1.f;
  if (skip_mwg && mwg_took(T, top_k ? top_k[b] : 0, top_p ? top_p[b] : 1.f, out_ids, b)) return;  // mwg's row
  const float rp = rep_pen ? rep_pen[b] : 1.f;
  const int slot = slots ? slots[b] : b;
  const uint8_t* sn = seen ? seen + (long long)slot * V : nullptr;
  const bool greedy = !(T > 0.f);
  const float inv_t = (greedy || T == 1.f) ? 1.f : 1.f / T;
  const bool pen = rp != 1.f && sn;

  // bf16 logits kept as raw bits, two per register (128 values in 64 VGPRs at 512 threads), the
  // penalty as one bit per value; val(u) rebuilds the processed logit with the same fp32 ops every
  // pass (bans and padding: bf16 -inf)
  uint32_t raw[RPT / 2];
  unsigned long long pbits[(RPT + 63) / 64] = {};
  static_assert(RPT <= 128 && RPT % 2 == 0 && NT % 64 == 0, "register sampler: <= 128 values per thread");
#pragma unroll
  for (int u = 0; u < RPT; u += 2) {
    uint32_t lo = 0xff80u, hi = 0xff80u;
    const int i0 = u * NT + tid, i1 = i0 + NT;
    const bf16_t* row = (const bf16_t*)logits + b * ld;
    if (i0 < V) {
      lo = row[i0];
      if (pen && sn[i0]) pbits[u / 64] |= 1ull << (u % 64);
    }
    if (i1 < V) {
      hi = row[i1];
      if (pen && sn[i1]) pbits[(u + 1) / 64] |= 1ull << ((u + 1) % 64);
    }
    raw[u / 2] = lo | (hi << 16);
  }
  if (ban_ids)
    for (int j = 0; j < n_ban; ++j) {
      const int id = ban_ids[(long long)b * n_ban + j];
      if (id >= 0 && id < V && (id & (NT - 1)) == tid) {
        const int uu = id / NT;
#pragma unroll
        for (int u = 0; u < RPT; ++u)
          if (u == uu) raw[u / 2] = (u & 1) ? ((raw[u / 2] & 0xffffu) | 0xff800000u) : ((raw[u / 2] & 0xffff0000u) | 0xff80u);
      }
    }
  // each pass re-derives the values from the packed bits: the opaque touch stops the compiler from
  // hoisting 64 unpacked floats out of the radix loops (they would not fit beside the packed copy)
  auto touch = [&]() {
#pragma unroll
    for (int q = 0; q < RPT / 2; ++q) asm volatile("" : "+v"(raw[q]));
  };
  auto val = [&](int u) -> float {
    float w = __uint_as_float((u & 1) ? (raw[u / 2] & 0xffff0000u) : (raw[u / 2] << 16));
    if ((pbits[u / 64] >> (u % 64)) & 1ull) w = w < 0.f ? w * rp : w / rp;
    return w * inv_t;
  };
  // max (+ first argmax) and softmax normaliser
  float m = -INFINITY, s = 0.f;
  int am = 0x7fffffff;
  touch();
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const float w = val(u);
    if (w > m) {
      s = s * __expf(m - w) + 1.f;
      m = w;
      am = u * NT + tid;
    } else if (w != -INFINITY) {
      s += __expf(w - m);
    }
  }
  const float M = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float Z = block_sum(s, red);
  const float lZ = M + __logf(Z);
  if (greedy) {
    int cand = (m == M) ? am : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    __syncthreads();
    if ((tid & 63) == 0) red[tid >> 6] = __int_as_float(cand);
    __syncthreads();
    int best = 0x7fffffff;
    for (int w = 0; w < NT / 64; ++w) best = min(best, __float_as_int(red[w]));
    if (best < V && (best & (NT - 1)) == tid) {  // the owner of the winning element
      const int uu = best / NT;
      float xb = 0.f;
#pragma unroll
      for (int u = 0; u < RPT; ++u)
        if (u == uu) xb = val(u);
      out_ids[b] = best;
      if (out_lp) out_lp[b] = xb - lZ;
      if (seen) seen[(long long)slot * V + best] = 1;
      if (out_kept) out_kept[b] = 1;
    }
    return;
  }

  // Radix selects on 4-bit digits (MSB first) with per-thread counters in registers: a 256-bin LDS
  // histogram of the first digits takes most of the vocabulary into a few bins, and those LDS
  // atomics serialise (~20 us per digit). Counts: 16 x 8-bit counters packed in 4 words (<= RPT
  // per thread), reduced as 16-bit pairs (8 words) per wave then across waves in LDS.
  // top-k: the k-th largest key among the valid elements (ties at it kept)
  uint32_t thr = 0;
  const int k = top_k ? top_k[b] : 0;
  const int lane = tid & 63, wid = tid >> 6;
  if (k > 0 && k < V) {
    uint32_t prefix = 0, mask = 0;
    int remaining = k;
    for (int shift = 28; shift >= 0; shift -= 4) {
      uint32_t w4[4] = {0u, 0u, 0u, 0u};
      touch();
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        const uint32_t key = fkey(val(u));
        if (u * NT + tid < V && (key & mask) == prefix) {
          const uint32_t d = (key >> shift) & 15u, inc = 1u << ((d & 3u) << 3);
          w4[0] += d < 4 ? inc : 0u;
          w4[1] += (d >> 2) == 1 ? inc : 0u;
          w4[2] += (d >> 2) == 2 ? inc : 0u;
          w4[3] += d >= 12 ? inc : 0u;
        }
      }
      // 8-bit counters -> 16-bit pairs (digit 2j in the low half, 2j + 1 in the high half), wave sums
      uint32_t w8[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w8[2 * q] = (w4[q] & 0xffu) | ((w4[q] & 0xff00u) << 8);
        w8[2 * q + 1] = ((w4[q] >> 16) & 0xffu) | ((w4[q] >> 8) & 0xff0000u);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) w8[q] += __shfl_xor(w8[q], o, 64);
      __syncthreads();
      if (lane < 8) {
        uint32_t mine = w8[0];
#pragma unroll
        for (int q = 1; q < 8; ++q)
          if (lane == q) mine = w8[q];
        cnt16[wid * 8 + lane] = mine;
      }
      __syncthreads();
      if (tid < 16) {  // digit totals, then one thread picks the digit
        uint32_t t = 0;
        for (int w = 0; w < NT / 64; ++w) t += cnt16[w * 8 + (tid >> 1)];
        tot16[tid] = (int)((tid & 1) ? (t >> 16) : (t & 0xffffu));
      }
      __syncthreads();
      if (tid == 0) {
        int run = 0, dsel = -1;
        for (int j = 15; j >= 0; --j) {
          if (run + tot16[j] >= remaining) {
            dsel = j;
            break;
          }
          run += tot16[j];
        }
        sel[0] = dsel;
        sel[1] = run;
      }
      __syncthreads();
      const int dsel = sel[0], run = sel[1];
      if (dsel < 0) break;  // fewer valid elements than k (cannot happen: k < V)
      prefix |= (uint32_t)dsel << shift;
      mask |= 15u << shift;
      remaining -= run;
    }
    thr = prefix;
  }
  // top-p over the survivors: the smallest key whose descending inclusive mass reaches p * kept mass
  // (LDS float atomics: after a top-k only a few dozen elements take part)
  const float pp = top_p ? top_p[b] : 1.f;
  if (pp < 1.f) {
    uint32_t prefix = 0, mask = 0;
    float above = 0.f, target = -1.f;
    for (int shift = 28; shift >= 0; shift -= 4) {
      if (tid < 16) hist[tid] = 0.f;
      __syncthreads();
      touch();
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        const float w = val(u);
        const uint32_t key = fkey(w);
        if (key >= thr && (key & mask) == prefix && w != -INFINITY)
          atomicAdd(&hist[(key >> shift) & 15u], __expf(w - M));
      }
      __syncthreads();
      if (tid == 0) {
        if (target < 0.f) {  // first digit: total kept mass after top-k
          float t = 0.f;
          for (int j = 0; j < 16; ++j) t += hist[j];
          target = pp * t;
        }
        float run = 0.f;
        int dsel = -1;
        for (int j = 15; j >= 0; --j) {
          if (hist[j] > 0.f && run + hist[j] >= target - above) {
            dsel = j;
            break;
          }
          run += hist[j];
        }
        sel[0] = dsel;
        selp[0] = run;
        selp[1] = target;
      }
      __syncthreads();
      const int dsel = sel[0];
      const float run = selp[0];
      target = selp[1];
      if (dsel < 0) {  // rounding: target not reached -> keep everything so far
        prefix = 0;
        mask = 0;
        break;
      }
      prefix |= (uint32_t)dsel << shift;
      mask |= 15u << shift;
      above += run;
    }
    if (mask == 0xffffffffu && prefix > thr) thr = prefix;
  }

  // multinomial over the kept elements, thread-major order: per-thread mass, block scan
  float ssum = 0.f;
  int kept = 0, last_u = -1;
  touch();
#pragma unroll
  for (int u = 0; u < RPT; ++u) {
    const float w = val(u);
    if (w != -INFINITY && fkey(w) >= thr) {
      ssum += __expf(w - M);
      ++kept;
      last_u = u;
    }
  }
  float incl = ssum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  __syncthreads();
  if (lane == 63) scan[wid] = incl;
  int kept_tot = kept;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) kept_tot += __shfl_xor(kept_tot, o, 64);
  if (lane == 0) red[wid] = __int_as_float(kept_tot);
  if (tid == 0) sh_key = -1;
  __syncthreads();
  float woff = 0.f, total = 0.f;
  for (int w = 0; w < NT / 64; ++w) {
    if (w < wid) woff += scan[w];
    total += scan[w];
  }
  incl += woff;
  const float excl = incl - ssum;
  uint32_t c[4] = {seeds ? 0u : (uint32_t)b, (uint32_t)step, (uint32_t)((unsigned long long)step >> 32), 0x5eedu};
  const unsigned long long sd = seeds ? seeds[b] : 0ull;
  philox4x32_10(c, (uint32_t)sd, (uint32_t)(sd >> 32));
  const float r = ((c[0] >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
  const float uu = r * total;
  if (ssum > 0.f && excl < uu && uu <= incl) {
    float run = excl;
    int pick = -1;
    touch();
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const float w = val(u);
      if (pick < 0 && w != -INFINITY && fkey(w) >= thr) {
        run += __expf(w - M);
        if (run >= uu || u == last_u) pick = u;
      }
    }
    if (pick >= 0) atomicMax(&sh_key, tid * RPT + pick);
  }
  __syncthreads();
  if (sh_key < 0 && kept > 0) atomicMax(&sh_key, tid * RPT + last_u);  // rounding at the top of the range
  __syncthreads();
  const int key = sh_key;
  if (key >= 0 && key / RPT == tid) {
    const int pu = key % RPT, id = pu * NT + tid;
    float xb = 0.f;
#pragma unroll
    for (int u = 0; u < RPT; ++u)
      if (u == pu) xb = val(u);
    out_ids[b] = id;
    if (out_lp) out_lp[b] = xb - lZ;
    if (seen) seen[(long long)slot * V + id] = 1;
    if (out_kept) {
      int kt = 0;
      for (int w = 0; w < NT / 64; ++w) kt += __float_as_int(red[w]);
      out_kept[b] = kt;
    }
  } else if (key < 0 && tid == 0) {  // nothing kept (all -inf): token 0, as sample_kernel
    out_ids[b] = 0;
    if (out_lp) out_lp[b] = -INFINITY;
    if (out_kept) out_kept[b] = 0;
  }
}

// ------------------------------------------------------ multi-workgroup sampler (top-k <= 64 or greedy)
// The register sampler above runs one workgroup per row: at batch 1 the whole 50400-entry row and
// every radix pass sit on ONE of 256 CUs (top-k 50: 93 us, + top-p: 133 us, profiles/sampler_r3.txt).
// Here a row is split over MWG_G workgroups of 256 threads (a contiguous chunk each, ~13 values per
// thread): each computes its chunk's max / softmax sum / first argmax and -- for a sampled row -- its
// local k-th largest key t_g by a 4-bit radix select, and writes the chunk's elements >= t_g (in index
// order, at most MWG_CMAX) to the workspace. The global k-th largest key is >= every t_g (chunk g
// alone holds k elements >= t_g), so the union of the chunk lists, cut at T0 = max_g t_g, holds the
// global top-k with its ties. The last workgroup to arrive (agent-scope release / acquire around one
// counter per row) merges: global max and normaliser, the top-k select over the ~k..2k candidates,
// top-p over the survivors (4-bit radix on the mass, as the register sampler), and the Philox
// multinomial in index order. Top-p-only rows (top_k off) list each chunk's top 3/4 CMAX; the merge
// samples them when the union -- every element >= T0 -- holds p of the row's mass (the nucleus is
// then inside it), else it marks the row (out_ids = -1). Rows with top_k > 64, pure multinomial rows
// and marked rows are left to sample_reg_kernel, launched after this one with `skip_mwg` (each kernel
// takes exactly the rows the other leaves: the choice is made on the device, so captured decode
// graphs keep working whatever the requests' parameters are).
constexpr int MWG_G = 16, MWG_NT = 256, MWG_CMAX = 128, MWG_KMAX = MWG_KMAX_;
constexpr int MWG_PART = 8;  // floats per workgroup partial: max, sum, t_g (key bits), count, argmax

// Wave sum of a uint32 (every lane gets it): DPP quad swaps and row mirrors within 16 lanes, then
// two cross-row steps.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// (wave-uniform result: the four 16-lane row sums are read out with v_readlane -- no LDS crossbar
// round trips, which at one dependent ds_swizzle / ds_bpermute pair per word made every radix pass
// ~2 us, profiles/sampler_r4.txt)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp_mov_u<0xB1>(v);
  v += dpp_mov_u<0x4E>(v);
  v += dpp_mov_u<0x141>(v);
  v += dpp_mov_u<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
template <int CTRL>
__device__ __forceinline__ float dpp_mov_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov_f<0xB1>(v));
  v = fmaxf(v, dpp_mov_f<0x4E>(v));
  v = fmaxf(v, dpp_mov_f<0x141>(v));
  v = fmaxf(v, dpp_mov_f<0x140>(v));
  return fmaxf(fmaxf(rl(v, 0), rl(v, 16)), fmaxf(rl(v, 32), rl(v, 48)));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_mov_f<0xB1>(v);
  v += dpp_mov_f<0x4E>(v);
  v += dpp_mov_f<0x141>(v);
  v += dpp_mov_f<0x140>(v);
  return (rl(v, 0) + rl(v, 16)) + (rl(v, 32) + rl(v, 48));
}
// wave OR / AND of a uint32 (uniform result), the same butterfly as wave_sum_u32
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  v |= dpp_mov_u<0xB1>(v);
  v |= dpp_mov_u<0x4E>(v);
  v |= dpp_mov_u<0x141>(v);
  v |= dpp_mov_u<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) | (uint32_t)__builtin_amdgcn_readlane((int)v, 16) |
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
__device__ __forceinline__ uint32_t wave_and_u32(uint32_t v) {
  v &= dpp_mov_u<0xB1>(v);
  v &= dpp_mov_u<0x4E>(v);
  v &= dpp_mov_u<0x141>(v);
  v &= dpp_mov_u<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) & (uint32_t)__builtin_amdgcn_readlane((int)v, 16) &
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) & (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
__device__ __forceinline__ int wave_min_i(int v) {
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, false));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// 4-bit radix select of the k-th largest key over (key, valid) pairs spread across the block:
// per-thread packed 8-bit counters (<= 255 elements per thread), DPP wave sums of 16-bit pairs into
// a double-buffered LDS table (one barrier per pass), and the digit picked redundantly by every lane
// from that table (no broadcast round). Returns the key prefix (ties at it kept); 0 when fewer than
// k are valid. cnt16: 2 x (blockDim/64) x 8 words.
//
// Digits every valid key shares (the bits where the block's OR equals its AND) select themselves:
// such a pass would find all candidates in one bucket, so it is skipped -- bf16 logits leave the
// low 16 key bits constant, and bunched top values share the sign / exponent nibbles, so most
// selections run 2-4 of the 8 passes (same threshold, same kept set).
template <int EPT, int NW>
__device__ uint32_t block_kth_key(int k, const uint32_t (&key)[EPT], const bool (&ok)[EPT], uint32_t* cnt16) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t prefix = 0, mask = 0;
  int remaining = k;
  int pass = 0;  // executed passes (the count tables alternate between them)
  uint32_t common, vary;
  {
    uint32_t vo = 0u, va = ~0u;
#pragma unroll
    for (int e = 0; e < EPT; ++e)
      if (ok[e]) {
        vo |= key[e];
        va &= key[e];
      }
    vo = wave_or_u32(vo);
    va = wave_and_u32(va);
    // (table 1 is next written by the second executed pass, after every thread passed the first's barrier)
    if (lane == 0) {
      cnt16[NW * 8 + 2 * wid] = vo;
      cnt16[NW * 8 + 2 * wid + 1] = va;
    }
    __syncthreads();
    vo = 0u;
    va = ~0u;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      vo |= cnt16[NW * 8 + 2 * w];
      va &= cnt16[NW * 8 + 2 * w + 1];
    }
    common = va;
    vary = vo ^ va;
  }
#pragma unroll 1
  for (int shift = 28; shift >= 0; shift -= 4) {
    if (((vary >> shift) & 15u) == 0u) {  // forced digit
      prefix |= common & (15u << shift);
      mask |= 15u << shift;
      continue;
    }
    uint32_t w4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int e = 0; e < EPT; ++e) {  // branch-free: selects, no exec-mask regions per element
      const uint32_t d = (key[e] >> shift) & 15u;
      const uint32_t inc = (ok[e] && (key[e] & mask) == prefix) ? 1u << ((d & 3u) << 3) : 0u;
      const uint32_t g4 = d >> 2;
      w4[0] += g4 == 0 ? inc : 0u;
      w4[1] += g4 == 1 ? inc : 0u;
      w4[2] += g4 == 2 ? inc : 0u;
      w4[3] += g4 == 3 ? inc : 0u;
    }
    uint4* tab = reinterpret_cast<uint4*>(cnt16) + (pass & 1) * NW * 2;
    uint32_t sw[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sw[2 * q] = wave_sum_u32((w4[q] & 0xffu) | ((w4[q] & 0xff00u) << 8));
      sw[2 * q + 1] = wave_sum_u32(((w4[q] >> 16) & 0xffu) | ((w4[q] >> 8) & 0xff0000u));
    }
    if (lane == 0) {
      tab[wid * 2] = make_uint4(sw[0], sw[1], sw[2], sw[3]);
      tab[wid * 2 + 1] = make_uint4(sw[4], sw[5], sw[6], sw[7]);
    }
    __syncthreads();
    // digit j's count: 16-bit half (j & 1) of word j >> 1, summed over the waves (all 2 NW rows
    // requested before the first use)
    uint4 rows[2 * NW];
#pragma unroll
    for (int i = 0; i < 2 * NW; ++i) rows[i] = tab[i];
    uint32_t words[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      words[0] += rows[2 * w].x; words[1] += rows[2 * w].y; words[2] += rows[2 * w].z; words[3] += rows[2 * w].w;
      words[4] += rows[2 * w + 1].x; words[5] += rows[2 * w + 1].y; words[6] += rows[2 * w + 1].z;
      words[7] += rows[2 * w + 1].w;
    }
    int run = 0, dsel = -1, csel = 0;
#pragma unroll
    for (int j = 15; j >= 0; --j) {
      const int c = (int)((j & 1) ? (words[j >> 1] >> 16) : (words[j >> 1] & 0xffffu));
      if (dsel < 0) {
        if (run + c >= remaining) {
          dsel = j;
          csel = c;
        } else {
          run += c;
        }
      }
    }
    if (dsel < 0) return 0u;  // fewer than k valid: keep every valid element
    prefix |= (uint32_t)dsel << shift;
    mask |= 15u << shift;
    remaining -= run;
    ++pass;
    // the selected bucket holds exactly the elements still needed: every key >= prefix (lower
    // bits zero) is in the top k -- done, the remaining passes would only walk that bucket down
    if (csel == remaining) return prefix;
  }
  return prefix;
}

// block_kth_key for keys held by ONE wave: the counts are wave sums (uniform scalars), so no LDS
// table and no barrier per pass -- the small selections (256 thread maxima, <= 256 candidates) run
// here while the other waves wait at one barrier.
template <int EPT>
__device__ uint32_t wave_kth_key(int k, const uint32_t (&key)[EPT], const bool (&ok)[EPT]) {
  uint32_t prefix = 0, mask = 0;
  int remaining = k;
  uint32_t vo = 0u, va = ~0u;  // forced digits skipped as in block_kth_key
#pragma unroll
  for (int e = 0; e < EPT; ++e)
    if (ok[e]) {
      vo |= key[e];
      va &= key[e];
    }
  const uint32_t common = wave_and_u32(va), vary = wave_or_u32(vo) ^ common;
#pragma unroll 1
  for (int shift = 28; shift >= 0; shift -= 4) {
    if (((vary >> shift) & 15u) == 0u) {
      prefix |= common & (15u << shift);
      mask |= 15u << shift;
      continue;
    }
    uint32_t w4[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const uint32_t d = (key[e] >> shift) & 15u;
      const uint32_t inc = (ok[e] && (key[e] & mask) == prefix) ? 1u << ((d & 3u) << 3) : 0u;
      const uint32_t g4 = d >> 2;
      w4[0] += g4 == 0 ? inc : 0u;
      w4[1] += g4 == 1 ? inc : 0u;
      w4[2] += g4 == 2 ? inc : 0u;
      w4[3] += g4 == 3 ? inc : 0u;
    }
    uint32_t words[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      words[2 * q] = wave_sum_u32((w4[q] & 0xffu) | ((w4[q] & 0xff00u) << 8));
      words[2 * q + 1] = wave_sum_u32(((w4[q] >> 16) & 0xffu) | ((w4[q] >> 8) & 0xff0000u));
    }
    int run = 0, dsel = -1, csel = 0;
#pragma unroll
    for (int j = 15; j >= 0; --j) {
      const int c = (int)((j & 1) ? (words[j >> 1] >> 16) : (words[j >> 1] & 0xffffu));
      if (dsel < 0) {
        if (run + c >= remaining) {
          dsel = j;
          csel = c;
        } else {
          run += c;
        }
      }
    }
    if (dsel < 0) return 0u;
    prefix |= (uint32_t)dsel << shift;
    mask |= 15u << shift;
    remaining -= run;
    if (csel == remaining) return prefix;
  }
  return prefix;
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, dpp_mov_u<0xB1>(v));
  v = min(v, dpp_mov_u<0x4E>(v));
  v = min(v, dpp_mov_u<0x141>(v));
  v = min(v, dpp_mov_u<0x140>(v));
  return min(min((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
             min((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}

// The exact k-th largest valid key of the keys ONE wave holds (0 when fewer than k are valid), by
// 8-bit digits: per pass the candidates' digits go into a wave-private 256-bin LDS histogram (ds_add),
// each lane reads 4 bins from the top, one wave scan finds the bin where the count from the top reaches
// the rank. Digits all valid keys share are forced (no pass), so bf16 logits (low 16 key bits
// constant) take at most 2 passes; once the chosen bin holds exactly the remaining rank, the k-th key
// is the bin's smallest (a wave min). hist: 256 words of LDS this wave alone uses (16-byte aligned).
template <int EPT>
__device__ __forceinline__ uint32_t wave_kth_key8(int k, const uint32_t (&key)[EPT], const bool (&ok)[EPT],
                                                  uint32_t* hist) {
  const int lane = threadIdx.x & 63;
  uint32_t vo = 0u, va = ~0u;
#pragma unroll
  for (int e = 0; e < EPT; ++e)
    if (ok[e]) {
      vo |= key[e];
      va &= key[e];
    }
  const uint32_t common = wave_and_u32(va), vary = wave_or_u32(vo) ^ common;
  uint32_t prefix = 0, mask = 0;
  int remaining = k;
#pragma unroll 1
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (((vary >> shift) & 255u) == 0u) {
      prefix |= common & (255u << shift);
      mask |= 255u << shift;
      continue;
    }
    reinterpret_cast<uint4*>(hist)[lane] = make_uint4(0u, 0u, 0u, 0u);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int e = 0; e < EPT; ++e)
      if (ok[e] && (key[e] & mask) == prefix) __hip_atomic_fetch_add(&hist[(key[e] >> shift) & 255u], 1u,
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
    // lane l: bins 255-4l (c.w) .. 252-4l (c.x), highest first
    const uint4 c = reinterpret_cast<const uint4*>(hist)[63 - lane];
    const int ls = (int)(c.x + c.y + c.z + c.w);
    int incl = ls;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const unsigned long long reach = __ballot(incl >= remaining);
    if (!reach) return 0u;  // fewer than k valid
    const int L = __builtin_ctzll(reach);
    int run = incl - ls, dsel = 0, csel = 0;
    {
      const int cw = (int)c.w, cz = (int)c.z, cy = (int)c.y, cx = (int)c.x;
      const int base = 255 - 4 * lane;
      if (run + cw >= remaining) { dsel = base; csel = cw; }
      else if (run + cw + cz >= remaining) { dsel = base - 1; csel = cz; run += cw; }
      else if (run + cw + cz + cy >= remaining) { dsel = base - 2; csel = cy; run += cw + cz; }
      else { dsel = base - 3; csel = cx; run += cw + cz + cy; }
    }
    dsel = __builtin_amdgcn_readlane(dsel, L);
    csel = __builtin_amdgcn_readlane(csel, L);
    run = __builtin_amdgcn_readlane(run, L);
    prefix |= (uint32_t)dsel << shift;
    mask |= 255u << shift;
    remaining -= run;
    if (csel == remaining) break;
  }
  // the top k are the keys above the chosen bins plus the whole last bin: the k-th is its smallest
  uint32_t mn = ~0u;
#pragma unroll
  for (int e = 0; e < EPT; ++e)
    if (ok[e] && (key[e] & mask) == prefix) mn = min(mn, key[e]);
  return wave_min_u32(mn);
}

// Wave-wide inclusive prefix sum (Hillis-Steele over ds_bpermute shuffles)
__device__ __forceinline__ float wave_incl_scan(float v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Diagnostic build only (tools/build_ext.py --stamps, tools/sample_stamps.py): s_memtime segment
// sums of the multi-workgroup sampler -- chunk phase of workgroup 0 of row 0 (slots 0..5) and the
// merging workgroup of row 0 (slots 8..13); slot 15 counts launches. Empty in the normal build.
#ifdef KCA_ATTN_STAMPS
__device__ unsigned long long g_sample_stamps[16];
__device__ __forceinline__ unsigned long long sst_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define SSTAMP_DECL unsigned long long sst_prev_ = sst_now();
#define SSTAMP_COUNT(on) \
  if ((on) && threadIdx.x == 0) atomicAdd(&g_sample_stamps[15], 1ull)
#define SSTAMP(k, on)                                                   \
  do {                                                                  \
    const unsigned long long n_ = sst_now();                            \
    if ((on) && threadIdx.x == 0) atomicAdd(&g_sample_stamps[k], n_ - sst_prev_); \
    sst_prev_ = n_;                                                     \
  } while (0)
KCA_API int kca_sample_stamps(unsigned long long* out, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sample_stamps), sizeof(g_sample_stamps)) != hipSuccess) return 2;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sample_stamps), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#else
#define SSTAMP_DECL
#define SSTAMP_COUNT(on)
#define SSTAMP(k, on) \
  do {                \
  } while (0)
#endif

template <int VPT, int G = MWG_G, int CMAX = MWG_CMAX, int DT = 0>
__global__ __launch_bounds__(MWG_NT) void sample_mwg_kernel(
    const bf16_t* __restrict__ logits, long long ld, int V, int CS,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const float* __restrict__ rep_pen, uint8_t* __restrict__ seen,
    const int* __restrict__ slots, const int* __restrict__ ban_ids, int n_ban,
    const unsigned long long* __restrict__ seeds, long long step, float* __restrict__ ws,
    unsigned int* __restrict__ cnt, long long* __restrict__ out_ids, float* __restrict__ out_lp,
    int* __restrict__ out_kept) {
  __shared__ __attribute__((aligned(16))) float red[8 + MWG_NT];  // [0, 8): per-wave partials; [8, 8 + NT): thread maxima
  __shared__ __attribute__((aligned(16))) uint32_t cnt16[2 * MWG_NT / 64 * 8];
  __shared__ int sel[2];
  __shared__ int iscan[MWG_NT / 64];
  __shared__ int sh_last;
  __shared__ __attribute__((aligned(16))) float Lv[G * CMAX];
  __shared__ int Li[G * CMAX];
  __shared__ __attribute__((aligned(16))) float L2v[G * CMAX];  // the candidates after the per-wave narrowing
  __shared__ int L2i[G * CMAX];
  __shared__ __attribute__((aligned(16))) float hist[48];
  __shared__ float Kv[64];
  __shared__ int Kj[64];
  const int g = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float T = temperature ? temperature[b] : 1.f;
  const int k = top_k ? top_k[b] : 0;
  const float pp = top_p ? top_p[b] : 1.f;
  if (!mwg_row(T, k, pp)) return;  // sample_reg_kernel's row
  SSTAMP_DECL
  const bool st0 = g == 0 && b == 0;
  const bool greedy = !(T > 0.f);
  // top-p only: each chunk lists its top KC (3/4 of the list, room for bf16 ties at the cut); the merge
  // checks that the union -- every element >= T0 -- holds the nucleus's mass before it samples
  const bool tponly = !greedy && k <= 0;
  const int kc = tponly ? CMAX * 3 / 4 : k;
  const float rp = rep_pen ? rep_pen[b] : 1.f;
  const int slot = slots ? slots[b] : b;
  const uint8_t* sn = seen ? seen + (long long)slot * V : nullptr;
  const float inv_t = (greedy || T == 1.f) ? 1.f : 1.f / T;
  const bool pen = rp != 1.f && sn;
  float* part = ws + (long long)b * G * (MWG_PART + 2 * CMAX);  // [G][PART + 2*CMAX]
  float* mine = part + g * (MWG_PART + 2 * CMAX);

  // ---- this workgroup's chunk [c0, c1): thread t owns the contiguous run [c0 + t*VPT, +VPT)
  const int c0 = g * CS, c1 = min(V, c0 + CS);
  const int e0 = c0 + tid * VPT;
  float x[VPT];
  const bf16_t* row = logits + b * ld;
#pragma unroll
  for (int e = 0; e < VPT; ++e) {
    const int i = e0 + e;
    float w = -INFINITY;
    if (i < c1) {
      w = e2f<DT>(row[i]);
      if (pen && sn[i]) w = w < 0.f ? w * rp : w / rp;
      w *= inv_t;
    }
    x[e] = w;
  }
  if (ban_ids)
    for (int j = 0; j < n_ban; ++j) {
      const int id = ban_ids[(long long)b * n_ban + j];
      if (id >= e0 && id < e0 + VPT && id < c1) {
#pragma unroll
        for (int e = 0; e < VPT; ++e)
          if (e0 + e == id) x[e] = -INFINITY;
      }
    }
  float m = -INFINITY, s = 0.f;
  int am = 0x7fffffff;
  SSTAMP(0, st0);
#pragma unroll
  for (int e = 0; e < VPT; ++e) {
    const float w = x[e];
    if (w > m) {
      s = s * __expf(m - w) + 1.f;
      m = w;
      am = e0 + e;
    } else if (w != -INFINITY) {
      s += __expf(w - m);
    }
  }
  // chunk max / normaliser / first argmax: per wave by DPP + readlane, combined after ONE barrier
  float Mg, Sg;
  int amg;
  {
    const float wm = wave_max_dpp(m);
    const float ws_ = wave_sum_dpp(m == -INFINITY ? 0.f : s * __expf(m - wm));
    const int wi = wave_min_i((m == wm && wm != -INFINITY) ? am : 0x7fffffff);
    if (lane == 0) {
      red[wid] = wm;
      red[4 + wid] = ws_;
      iscan[wid] = wi;
    }
    __syncthreads();
    Mg = -INFINITY;
#pragma unroll
    for (int w = 0; w < MWG_NT / 64; ++w) Mg = fmaxf(Mg, red[w]);
    Sg = 0.f;
    amg = 0x7fffffff;
#pragma unroll
    for (int w = 0; w < MWG_NT / 64; ++w) {
      if (red[w] != -INFINITY) Sg += red[4 + w] * __expf(red[w] - Mg);
      if (red[w] == Mg && Mg != -INFINITY) amg = min(amg, iscan[w]);
    }
  }
  SSTAMP(1, st0);

  // ---- local top-k threshold and the chunk's candidates (index order, at most CMAX)
  // t_g only has to leave k <= count(x >= t_g) <= CMAX. First try the k-th largest of the 256
  // per-thread maxima (k threads each hold an element >= it; one key per thread makes the radix
  // passes ~13x cheaper); when that keeps more than CMAX (top values bunched in few threads, e.g.
  // sorted logits), the exact k-th largest element.
  int count = 0, over = 0;
  uint32_t tg = 0;
  if (!greedy) {
    uint32_t xk[VPT];
    bool xo[VPT];
    float tmx = -INFINITY;
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
      xk[e] = fkey(x[e]);
      xo[e] = x[e] != -INFINITY;
      tmx = fmaxf(tmx, x[e]);
    }
    {  // the 256 thread maxima to wave 0 (4 per lane), selected there; one barrier each way
      red[8 + tid] = tmx;
      __syncthreads();
      if (wid == 0) {
        uint32_t mk[4];
        bool mo[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = red[8 + 4 * lane + e];
          mk[e] = fkey(v);
          mo[e] = v != -INFINITY;
        }
        const uint32_t t = wave_kth_key8<4>(kc, mk, mo, reinterpret_cast<uint32_t*>(Lv));  // (Lv: merge only)
        if (lane == 0) sel[0] = (int)t;
      }
      __syncthreads();
      tg = (uint32_t)sel[0];
    }
    SSTAMP(2, st0);
    int c, off, tot;
    auto scan = [&]() {
      c = 0;
#pragma unroll
      for (int e = 0; e < VPT; ++e) c += (xo[e] && xk[e] >= tg) ? 1 : 0;
      int inc = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      __syncthreads();
      if (lane == 63) iscan[wid] = inc;
      __syncthreads();
      off = inc - c;
      tot = 0;
#pragma unroll
      for (int w = 0; w < MWG_NT / 64; ++w) {
        if (w < wid) off += iscan[w];
        tot += iscan[w];
      }
    };
    scan();
    if (tot > CMAX) {  // uniform: every thread read the same iscan
      tg = block_kth_key<VPT, MWG_NT / 64>(kc, xk, xo, cnt16);
      scan();
    }
    over = tot > CMAX;
    count = min(tot, CMAX);  // (> CMAX only with massive ties at t_g: the first CMAX by index stay)
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
      if (xo[e] && xk[e] >= tg) {
        if (off < CMAX) {
          mine[MWG_PART + off] = x[e];
          reinterpret_cast<int*>(mine)[MWG_PART + CMAX + off] = e0 + e;
        }
        ++off;
      }
    }
  }
  SSTAMP(3, st0);
  if (tid == 0) {  // (integer fields stored as integers: key / index bit patterns as floats could be NaNs)
    mine[0] = Mg;
    mine[1] = Sg;
    unsigned* mu = reinterpret_cast<unsigned*>(mine);
    mu[2] = tg;
    mu[3] = (unsigned)count;
    mu[4] = (unsigned)amg;
    mu[5] = (unsigned)over;  // the list dropped elements tied at t_g (a top-p-only row falls back)
  }
  // ---- arrival: every wave's stores drained, one agent-scope release, one counter per row
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(&cnt[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_last = prev == G - 1;
    if (sh_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  SSTAMP(4, st0);
  if (!sh_last) return;
  const bool sm0 = b == 0;
  SSTAMP_COUNT(sm0);

  // ================= merge (the last workgroup of the row)
  if (tid == 0) cnt[b] = 0;  // re-armed for the next launch
  // candidate slots: thread t takes slots [SPT t, SPT t + SPT) of one chunk's list, requested together
  // with the chunk headers (one round trip; the slots past the chunk's count are ignored below)
  constexpr int SPT = G * CMAX / MWG_NT;
  static_assert(CMAX % SPT == 0, "a thread's slots within one chunk");
  const int j0 = tid * SPT, qs = j0 / CMAX, p0 = j0 % CMAX;
  const float* pqs = part + qs * (MWG_PART + 2 * CMAX);
  float rv[SPT];
  int ri[SPT], cq = 0;
  if (!greedy) {
#pragma unroll
    for (int e = 0; e < SPT; ++e) {
      rv[e] = pqs[MWG_PART + p0 + e];
      ri[e] = reinterpret_cast<const int*>(pqs)[MWG_PART + CMAX + p0 + e];
    }
    cq = reinterpret_cast<const int*>(pqs)[3];
  }
  float M = -INFINITY;
  for (int q = 0; q < G; ++q) M = fmaxf(M, part[q * (MWG_PART + 2 * CMAX)]);
  float Z = 0.f;
  int best = 0x7fffffff;
  uint32_t T0 = 0, anyover = 0;
  for (int q = 0; q < G; ++q) {
    const float* pq = part + q * (MWG_PART + 2 * CMAX);
    if (pq[0] != -INFINITY) Z += pq[1] * __expf(pq[0] - M);
    const unsigned* pu = reinterpret_cast<const unsigned*>(pq);
    if (pq[0] == M && best == 0x7fffffff) best = (int)pu[4];  // first chunk holding the max
    T0 = max(T0, pu[2]);
    anyover |= pu[5];
  }
  const float lZ = M + __logf(Z);
  if (greedy || M == -INFINITY) {
    if (tid == 0) {
      const int id = (M == -INFINITY || best >= V) ? 0 : best;
      out_ids[b] = id;
      if (out_lp) out_lp[b] = M == -INFINITY ? -INFINITY : M - lZ;
      if (seen && M != -INFINITY) seen[(long long)slot * V + id] = 1;
      if (out_kept) out_kept[b] = M == -INFINITY ? 0 : 1;
    }
    return;
  }
  // candidates >= T0, compacted into LDS in (chunk, position) = index order: a block scan places
  // the slots loaded above
  int nv;
  {
    float sv[SPT];
    int si[SPT];
    int c = 0;
#pragma unroll
    for (int e = 0; e < SPT; ++e) {
      sv[e] = -INFINITY;
      si[e] = 0;
      if (p0 + e < cq && fkey(rv[e]) >= T0) {
        sv[e] = rv[e];
        si[e] = ri[e];
        ++c;
      }
    }
    int inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    __syncthreads();
    if (lane == 63) iscan[wid] = inc;
    __syncthreads();
    int off = inc - c;
    nv = 0;
#pragma unroll
    for (int w = 0; w < MWG_NT / 64; ++w) {
      if (w < wid) off += iscan[w];
      nv += iscan[w];
    }
#pragma unroll
    for (int e = 0; e < SPT; ++e)
      if (sv[e] != -INFINITY) {
        Lv[off] = sv[e];
        Li[off] = si[e];
        ++off;
      }
    __syncthreads();
  }
  SSTAMP(8, sm0);
  uint32_t c4[4] = {seeds ? 0u : (uint32_t)b, (uint32_t)step, (uint32_t)((unsigned long long)step >> 32), 0x5eedu};
  const unsigned long long sd = seeds ? seeds[b] : 0ull;
  philox4x32_10(c4, (uint32_t)sd, (uint32_t)(sd >> 32));
  const float r = ((c4[0] >> 8) + 1) * (1.0f / 16777216.0f);  // (0, 1]
  SSTAMP(9, sm0);
  // top-k, top-p and the multinomial over the nv compacted candidates, E per thread (contiguous,
  // index order): E = 1 in the common case (nv <= 256), so each radix pass costs one key per thread
  auto tail = [&](auto EC) {
    constexpr int E = decltype(EC)::value;
    float lv[E], lm[E];
    uint32_t lk[E];
    bool lo[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int j = tid * E + e;
      lo[e] = j < nv;
      lv[e] = lo[e] ? Lv[j] : -INFINITY;
      lk[e] = fkey(lv[e]);
      lm[e] = lo[e] ? __expf(lv[e] - M) : 0.f;
    }
    uint32_t thr = tponly ? 0u : block_kth_key<E, MWG_NT / 64>(k, lk, lo, cnt16);
    SSTAMP(10, sm0);
    // top-p over the survivors: the smallest key whose descending inclusive mass reaches p * kept mass
    if (pp < 1.f) {
      uint32_t prefix = 0, mask = 0;
      float above = 0.f, target = -1.f;
      // triple-buffered histogram: pass p accumulates into buffer p % 3 and, after its barrier,
      // clears buffer (p + 2) % 3 (read in pass p - 1, filled in pass p + 2); every lane picks the
      // digit from its own read of the table (no broadcast round). Digits all survivors share are
      // forced (no pass, as in block_kth_key; p counts executed passes); Kj is free scratch here.
      uint32_t vo = 0u, va = ~0u;
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (lo[e] && lk[e] >= thr) {
          vo |= lk[e];
          va &= lk[e];
        }
      vo = wave_or_u32(vo);
      va = wave_and_u32(va);
      if (lane == 0) {
        Kj[2 * wid] = (int)vo;
        Kj[2 * wid + 1] = (int)va;
      }
      if (tid < 48) hist[tid] = 0.f;
      __syncthreads();
      vo = 0u;
      va = ~0u;
#pragma unroll
      for (int w = 0; w < MWG_NT / 64; ++w) {
        vo |= (uint32_t)Kj[2 * w];
        va &= (uint32_t)Kj[2 * w + 1];
      }
      const uint32_t common = va, vary = vo ^ va;
      int pass = 0;
#pragma unroll 1
      for (int shift = 28; shift >= 0; shift -= 4) {
        if (((vary >> shift) & 15u) == 0u) {
          prefix |= common & (15u << shift);
          mask |= 15u << shift;
          continue;
        }
        float* hb = hist + 16 * (pass % 3);
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (lo[e] && lk[e] >= thr && (lk[e] & mask) == prefix) atomicAdd(&hb[(lk[e] >> shift) & 15u], lm[e]);
        __syncthreads();
        float hv[16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float4 t4 = reinterpret_cast<const float4*>(hb)[j];
          hv[4 * j] = t4.x; hv[4 * j + 1] = t4.y; hv[4 * j + 2] = t4.z; hv[4 * j + 3] = t4.w;
        }
        if (tid < 16) hist[16 * ((pass + 2) % 3) + tid] = 0.f;
        if (target < 0.f) {  // p x the kept mass; top-p only: p x the whole row's (the merge checked
          float t = 0.f;      // that the candidates hold it)
#pragma unroll
          for (int j = 0; j < 16; ++j) t += hv[j];
          target = pp * (tponly ? Z : t);
        }
        float run = 0.f;
        int dsel = -1;
#pragma unroll
        for (int j = 15; j >= 0; --j) {
          if (dsel < 0) {
            if (hv[j] > 0.f && run + hv[j] >= target - above) dsel = j;
            else run += hv[j];
          }
        }
        if (dsel < 0) {
          prefix = 0;
          mask = 0;
          break;
        }
        prefix |= (uint32_t)dsel << shift;
        mask |= 15u << shift;
        above += run;
        ++pass;
      }
      if (mask == 0xffffffffu && prefix > thr) thr = prefix;
    }
    SSTAMP(11, sm0);
    // multinomial over the kept candidates, index order: per-thread mass, block scan, Philox draw
    float ssum = 0.f;
    int kept = 0, last_j = -1;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (lo[e] && lk[e] >= thr) {
        ssum += lm[e];
        ++kept;
        last_j = tid * E + e;
      }
    }
    float incl = ssum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    int kept_tot = kept;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) kept_tot += __shfl_xor(kept_tot, o, 64);
    __syncthreads();
    if (lane == 63) red[wid] = incl;
    if (lane == 0) iscan[wid] = kept_tot;
    if (tid == 0) sel[0] = -1;
    __syncthreads();
    float woff = 0.f, total = 0.f;
    int ktot = 0;
    for (int w = 0; w < MWG_NT / 64; ++w) {
      if (w < wid) woff += red[w];
      total += red[w];
      ktot += iscan[w];
    }
    incl += woff;
    const float excl = incl - ssum;
    const float u = r * total;
    if (ssum > 0.f && excl < u && u <= incl) {
      float run = excl;
      int pick = -1;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = tid * E + e;
        if (pick < 0 && lo[e] && lk[e] >= thr) {
          run += lm[e];
          if (run >= u || j == last_j) pick = j;
        }
      }
      if (pick >= 0) atomicMax(&sel[0], pick);
    }
    __syncthreads();
    if (sel[0] < 0 && kept > 0) atomicMax(&sel[0], last_j);  // rounding at the top of the range
    __syncthreads();
    if (tid == 0) {
      const int j = sel[0];
      const int id = j >= 0 ? Li[j] : 0;
      out_ids[b] = id;
      if (out_lp) out_lp[b] = j >= 0 ? Lv[j] - lZ : -INFINITY;
      if (seen && j >= 0) seen[(long long)slot * V + id] = 1;
      if (out_kept) out_kept[b] = ktot;
    }
  };
  if (tponly) {
    // the candidates are every element >= T0 (no chunk list dropped a tie): the nucleus lies among
    // them iff their mass reaches p x Z -- else the one-workgroup kernel launched next takes the row
    float mc = 0.f;
    for (int j = tid; j < nv; j += MWG_NT) mc += __expf(Lv[j] - M);
    mc = wave_sum_dpp(mc);
    __syncthreads();
    if (lane == 0) red[wid] = mc;
    __syncthreads();
    float mt = 0.f;
#pragma unroll
    for (int w = 0; w < MWG_NT / 64; ++w) mt += red[w];
    __syncthreads();  // (red is reused by the tail's scan)
    if (anyover || !(mt > pp * Z)) {
      if (tid == 0) out_ids[b] = -1;
      return;
    }
    if (nv <= MWG_NT) tail(std::integral_constant<int, 1>{});
    else tail(std::integral_constant<int, SPT>{});
    return;
  }
  // Narrowing: each wave's exact top-k key over its 512 compacted slots (wave sums only, the four
  // waves in parallel); T1 = the largest of them is <= the global k-th key (that wave alone holds k
  // elements >= T1), so the candidates >= T1 -- about 4k -- still hold the top k with its ties.
  int n2;
  {
    uint32_t k8[SPT];
    bool o8[SPT];
    int c = 0;
#pragma unroll
    for (int e = 0; e < SPT; ++e) {
      const int j = tid * SPT + e;
      o8[e] = j < nv;
      k8[e] = o8[e] ? fkey(Lv[j]) : 0u;
    }
    // (L2v is written only after the barrier below: each wave's histogram lives there until then)
    const uint32_t tw = wave_kth_key8<SPT>(k, k8, o8, reinterpret_cast<uint32_t*>(L2v) + 256 * wid);
    if (lane == 0) Kj[wid] = (int)tw;
    __syncthreads();
    uint32_t T1 = 0;
#pragma unroll
    for (int w = 0; w < MWG_NT / 64; ++w) T1 = max(T1, (uint32_t)Kj[w]);
#pragma unroll
    for (int e = 0; e < SPT; ++e) c += (o8[e] && k8[e] >= T1) ? 1 : 0;
    int inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) iscan[wid] = inc;
    __syncthreads();
    int off = inc - c;
    n2 = 0;
#pragma unroll
    for (int w = 0; w < MWG_NT / 64; ++w) {
      if (w < wid) off += iscan[w];
      n2 += iscan[w];
    }
#pragma unroll
    for (int e = 0; e < SPT; ++e)
      if (o8[e] && k8[e] >= T1) {
        L2v[off] = Lv[tid * SPT + e];
        L2i[off] = Li[tid * SPT + e];
        ++off;
      }
    __syncthreads();
  }
  SSTAMP(10, sm0);
  // Fast path, one wave, no barriers: <= 256 candidates (4 per lane) -> top-k key; the kept ones
  // (<= 64: one per lane, index order) -> top-p by each element's mass of strictly larger keys
  // (kept iff that mass is below p x the kept mass: the tied cut key stays whole), multinomial in
  // index order -- the same selection and draw as the block path below, which takes the rest.
  if (wid == 0) {
    int done = 0;
    if (n2 <= 256) {
      float v4[4];
      uint32_t k4[4];
      bool o4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = lane * 4 + e;
        o4[e] = j < n2;
        v4[e] = o4[e] ? L2v[j] : -INFINITY;
        k4[e] = fkey(v4[e]);
      }
      // (red[8..]: the thread maxima of the chunk phase, free in the merge until the block tail's scan)
      const uint32_t thr = wave_kth_key8<4>(k, k4, o4, reinterpret_cast<uint32_t*>(red + 8));
      int kc = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) kc += (o4[e] && k4[e] >= thr) ? 1 : 0;
      int kin = kc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(kin, o, 64);
        if (lane >= o) kin += t;
      }
      const int nk = __builtin_amdgcn_readlane(kin, 63);
      if (nk <= 64) {
        int w = kin - kc;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (o4[e] && k4[e] >= thr) {
            Kv[w] = v4[e];
            Kj[w] = lane * 4 + e;
            ++w;
          }
        // (one wave: its LDS accesses execute in order, the reads below see these writes)
        const bool kv_ok = lane < nk;
        const float kv = kv_ok ? Kv[lane] : -INFINITY;
        const int kj = kv_ok ? Kj[lane] : 0;
        const uint32_t kk = fkey(kv);
        const float mass = kv_ok ? __expf(kv - M) : 0.f;
        bool keep = kv_ok;
        if (pp < 1.f) {
          const float tot = wave_sum_dpp(mass);
          float above = 0.f;
          for (int t = 0; t < nk; ++t) {
            const uint32_t kt = (uint32_t)__builtin_amdgcn_readlane((int)kk, t);
            const float mt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mass), t));
            above += kt > kk ? mt : 0.f;
          }
          keep = kv_ok && above < pp * tot;
        }
        const float km = keep ? mass : 0.f;
        const float incl = wave_incl_scan(km, lane);
        const float total = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 63));
        const float u = r * total;
        const unsigned long long hit = __ballot(keep && incl >= u && total > 0.f);
        const unsigned long long kb = __ballot(keep);
        int pl = -1;
        if (hit) pl = __builtin_ctzll(hit);
        else if (kb) pl = 63 - __builtin_clzll(kb);  // rounding at the top of the range
        if (lane == 0) {
          const int j = pl >= 0 ? __builtin_amdgcn_readlane(kj, pl) : -1;
          const float vj = pl >= 0 ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kv), pl)) : -INFINITY;
          const int id = j >= 0 ? L2i[j] : 0;
          out_ids[b] = id;
          if (out_lp) out_lp[b] = j >= 0 ? vj - lZ : -INFINITY;
          if (seen && j >= 0) seen[(long long)slot * V + id] = 1;
          if (out_kept) out_kept[b] = (int)__popcll(kb);
        }
        done = 1;
      }
    }
    if (lane == 0) sel[1] = done;
  }
  __syncthreads();
  if (!sel[1]) {
    if (nv <= MWG_NT) tail(std::integral_constant<int, 1>{});
    else tail(std::integral_constant<int, SPT>{});
  }
  SSTAMP(12, sm0);
}

// cnt: >= B zero-initialised counters (the multi-workgroup path re-arms them), or null to keep every
// row on the one-workgroup kernels.
KCA_API int kca_sample_logits(const void* logits, long long ld, int is_bf16, int B, int V,
                              const float* temperature, const int* top_k, const float* top_p,
                              const float* rep_pen, void* seen, const int* slots,
                              const int* ban_ids, int n_ban, const unsigned long long* seeds,
                              long long step, float* ws, long long* out_ids, float* out_lp,
                              int* out_kept, unsigned int* cnt, int mwg_complete, hipStream_t stream) {
  if (B <= 0 || V <= 0 || !ws || !out_ids) return 1;
  static int mwg = -1;  // KCA_SAMPLE_MWG=0: every row on the one-workgroup kernels (A/B)
  if (mwg < 0) {
    const char* e = getenv("KCA_SAMPLE_MWG");
    mwg = !(e && e[0] == '0');
  }
  // the large-vocabulary form (BLOOM's 250,880: 32 chunks of 7,840, 64 candidates each) runs its
  // greedy, top-k and top-p-only rows here too; the rest take the one-workgroup memory-pass kernel
  const bool big = V > 50 * 1024;
  const int G = big ? 32 : MWG_G;
  const int CS = (V + G - 1) / G, vpt = (CS + MWG_NT - 1) / MWG_NT;
  // (is_bf16: the logits' dtype -- 0 fp32, 1 bf16, 2 fp16; the multi-workgroup kernel reads 16-bit logits)
  const bool use_mwg = mwg && cnt && is_bf16 && (big ? vpt <= 32 : vpt <= 16) &&
                       (long long)G * (MWG_PART + 2 * (big ? 64 : MWG_CMAX)) <= V;  // (the rest: sample_reg_kernel)
  if (use_mwg && big) {
    if (is_bf16 == 2)
      hipLaunchKernelGGL((sample_mwg_kernel<32, 32, 64, 1>), dim3(32, B), dim3(MWG_NT), 0, stream,
                         (const bf16_t*)logits, ld, V, CS, temperature, top_k, top_p, rep_pen, (uint8_t*)seen, slots,
                         ban_ids, n_ban, seeds, step, ws, cnt, out_ids, out_lp, out_kept);
    else
      hipLaunchKernelGGL((sample_mwg_kernel<32, 32, 64>), dim3(32, B), dim3(MWG_NT), 0, stream,
                         (const bf16_t*)logits, ld, V, CS, temperature, top_k, top_p, rep_pen, (uint8_t*)seen, slots,
                         ban_ids, n_ban, seeds, step, ws, cnt, out_ids, out_lp, out_kept);
  } else if (use_mwg) {
#define KCA_SAMPLE_MWG_LAUNCH(P)                                                                               \
  if (is_bf16 == 2)                                                                                            \
    hipLaunchKernelGGL((sample_mwg_kernel<P, MWG_G, MWG_CMAX, 1>), dim3(MWG_G, B), dim3(MWG_NT), 0, stream,    \
                       (const bf16_t*)logits, ld, V, CS, temperature, top_k, top_p, rep_pen, (uint8_t*)seen, slots, \
                       ban_ids, n_ban, seeds, step, ws, cnt, out_ids, out_lp, out_kept);                      \
  else                                                                                                         \
    hipLaunchKernelGGL((sample_mwg_kernel<P>), dim3(MWG_G, B), dim3(MWG_NT), 0, stream, (const bf16_t*)logits,  \
                       ld, V, CS, temperature, top_k, top_p, rep_pen, (uint8_t*)seen, slots, ban_ids, n_ban, seeds, \
                       step, ws, cnt, out_ids, out_lp, out_kept)
    if (vpt <= 4) {
      KCA_SAMPLE_MWG_LAUNCH(4);
    } else if (vpt <= 8) {
      KCA_SAMPLE_MWG_LAUNCH(8);
    } else if (vpt <= 13) {
      KCA_SAMPLE_MWG_LAUNCH(13);  // GPT-2 / GPT-J / NeoX vocabularies
    } else {
      KCA_SAMPLE_MWG_LAUNCH(16);
    }
#undef KCA_SAMPLE_MWG_LAUNCH
  }
  // mwg_complete: the caller knows every row is greedy or has 1 <= top_k <= 64 -- rows the multi-workgroup
  // merge always finishes -- so the closing one-workgroup kernel (4-5 us even when every row skips it,
  // profiles/sampler_r5.txt) is not launched
  if (use_mwg && mwg_complete) return hipGetLastError() == hipSuccess ? 0 : 2;
  static int compact = -1;  // KCA_SAMPLE_COMPACT=0: top-p / multinomial over the full vocabulary (A/B)
  if (compact < 0) {
    const char* e = getenv("KCA_SAMPLE_COMPACT");
    compact = !(e && e[0] == '0');
  }
  static int reg = -1;  // KCA_SAMPLE_REG=0: the memory-pass kernel for every vocabulary (A/B)
  if (reg < 0) {
    const char* e = getenv("KCA_SAMPLE_REG");
    reg = !(e && e[0] == '0');
  }
  if (reg && is_bf16 == 1 && V <= 50 * 1024) {  // (bit-level bf16 candidate packing: bf16 logits only)
#define KCA_SAMPLE_REG_LAUNCH(R)                                                                          \
  hipLaunchKernelGGL((sample_reg_kernel<R, 1024>), dim3(B), dim3(1024), 0, stream, logits, ld, V,            \
                     temperature, top_k, top_p, rep_pen, (uint8_t*)seen, slots, ban_ids, n_ban, seeds, step,     \
                     out_ids, out_lp, out_kept, (int)use_mwg)
    if (V <= 16 * 1024) KCA_SAMPLE_REG_LAUNCH(16);
    else if (V <= 32 * 1024) KCA_SAMPLE_REG_LAUNCH(32);
    else KCA_SAMPLE_REG_LAUNCH(50);  // GPT-2 / GPT-J / NeoX vocabularies (50257 / 50400 / 50432)
#undef KCA_SAMPLE_REG_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(SAMPLE_THREADS), 0, stream, logits, ld, is_bf16,
                     V, temperature, top_k, top_p, rep_pen, (uint8_t*)seen, slots, ban_ids, n_ban,
                     seeds, step, ws, out_ids, out_lp, out_kept, compact, (int)use_mwg);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
