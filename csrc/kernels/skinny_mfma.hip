// Batched-decode GEMM on the matrix cores: y[M, N] = epilogue(x[M, K] . W[N, K]^T), M = 1..64.
//
// FasterTransformer's / DS-Inference's decoder at batch > 1 (max_batch_size 1024 in the FT GPT-J /
// NeoX services, the BLOOM predictors' batched instances): every decode linear streams its weight
// once per step and does 2*M FLOP per weight element -- 64 FLOP/B at M = 64, 4x what the VALU can
// issue next to an 8 TB/s stream once the bf16 -> fp32 unpacking is counted. So the dot products run
// on v_mfma_f32_16x16x32_{bf16,f16}, and the kernel is built around the weight stream
// (measurements: profiles/stream_probe_r6.jsonl, profiles/mm_bench_r6_*.jsonl):
//
//   * weight: each wave owns NRW 16-row tiles of the workgroup's N block and streams them as row
//     runs (RPI rows x KC*2 contiguous bytes per load instruction, non-temporal). The mfma A-operand
//     map itself (16 rows x 64 B per instruction) tops out near 5 TB/s; 256-B-1-KB row runs reach
//     6-6.8. The run is transposed through the wave's own LDS slot, 16-B pieces XOR-swizzled by row
//     (conflict-free writes and ds_read_b128 fragment reads), one chunk prefetched in registers.
//   * activation: the workgroup's 4 waves split N, not K, so they share each K chunk of x: staged
//     once per workgroup in LDS (double-buffered, same swizzle), read as B fragments. Per-wave K
//     splits re-read x from L2 once per wave -- as many bytes as the weight itself at M = 16, which
//     capped the first version at 3-4 TB/s and 1.2-1.8 TB/s at M = 64.
//   * LN-on-load: when the activation is the residual stream h, its per-row (mean, rstd) -- published
//     by the previous projection's tail (mm_tail.h) -- and gamma / beta normalise the chunk as it is
//     staged (once per workgroup), ln_rows' math rounded to the element type. No LayerNorm launch,
//     no normalised-row buffer.
//   * K split over workgroups (grid.y) so a launch fills the chip whatever N is: fp32 partial tiles
//     published write-through, the last arriving workgroup of an N block sums them (fan-in counter
//     per block, re-armed) and runs the epilogue.
//   * epilogues: bias + GELU (fc_in); bias + residual add -> new residual stream, plus the row-stats
//     tail (out-projection / fc_out), whose last arriver writes the next LayerNorm's (mean, rstd).
//   * two jobs per launch: N-concatenated (QKV and fc_in of a parallel-residual layer share their
//     input) or one job with two K-concatenated parts (GPT-J's out-projection + fc_out into one
//     residual: y = o.Wo^T + g.Wf^T).
//
// SURVEY N6 / K1 / K5 (decode shapes); the batch-1 GEMV path is gemv.hip / decode.hip.
#include "common.h"
#include "gemv_m1.h"
#include "mm_tail.h"

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// DT 0 = bf16, 1 = fp16 (e2f / f2e: common.h)
template <int DT>
__device__ __forceinline__ f32x4 mfma16(const u32x4v& a, const u32x4v& b, const f32x4& c) {
  if constexpr (DT == 0)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
}

__device__ __forceinline__ u32x4v ld_nt16(const uint16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p));
}
__device__ __forceinline__ u32x4v ld16(const uint16_t* p) { return *reinterpret_cast<const u32x4v*>(p); }

struct MmPart {
  const uint16_t* x;      // [M, K] activation rows (row stride ldx)
  long long ldx;
  const uint16_t* w;      // [N, K] weight (row stride ldw), or packed (below)
  long long ldw;
  int K;
  // 1: w is the packed stream layout [ceil(N/16)][ceil(K/128)][16][128] (zero-padded; ldw = elements
  // per 16-row block): a wave's 16 x 128 sub-tile is 4 KB contiguous and a KC = 128 load instruction
  // reads 1 KB contiguous (the row-run pattern that streams at 6-6.8 TB/s, profiles/stream_probe_r6)
  int packed;
  const float* stats;     // [M][2] (mean, rstd): x is the residual stream, normalised on load (or null)
  const uint16_t* gamma;  // [K] (with stats)
  const uint16_t* beta;   // [K] (nullable)
  // st_nt > 0: `stats` holds the producer's unmerged per-slice partials [M][st_nt][2] (mean, M2 of K /
  // st_nt columns each, mm_tail.h rs_publish) and every workgroup merges them in its prologue (st_eps:
  // the LayerNorm's eps) -- the producing tail then needs no arrival count and no last-arriver merge
  int st_nt;
  float st_eps;
};

struct MmJob {
  MmPart p[2];
  int nparts;             // 1, or 2: K-concatenated parts summed into one output
  int N;
  int tiles;              // workgroups of this job (set by the host entry point)
  const uint16_t* bias;   // [N] (nullable)
  int act;                // 0 none, 1 GELU tanh, 2 GELU erf (not with res)
  uint16_t* y;            // [M, N] (row stride ldy)
  long long ldy;
  const uint16_t* res;    // [M, N] residual added after the bias (nullable; may alias y)
  long long ldr;
  float* part;            // row-stats tail (nullable): RowStats.part
  float* stats_out;       // RowStats.stats
  unsigned* cnt;          // RowStats.cnt
  float eps;
};

struct MmArgs {
  MmJob j[2];
  int njobs;
  int M;
  int ks;         // K split over workgroups (0: host picks; the kernel sees the chosen value)
  int nr;         // 16-row weight tiles per wave (0: host picks)
  int kc;         // K per chunk, 128 / 256 (0: host picks)
  int wv;         // waves per workgroup, 4 / 8 (0: host picks)
  float* ws;      // split-K partial tiles (ks > 1): kca_mm_skinny_plan floats
  unsigned* bcnt; // per-N-block arrival counters (ks > 1), zero-initialised, re-armed every launch
  long long ws_floats;
  int bcnt_n;
  int pf;         // weight chunks in flight per wave (1; the kernel's PF ring, see mm_go)
};

// One finished 16x16 tile: rows n_base + 4*(lane>>4) + i (i < 4) of the output's N axis, column m =
// mt*16 + (lane & 15) of its M axis (the mfma_f32_16x16x32 C layout).
template <int DT>
__device__ __forceinline__ void mm_store(const MmJob& J, int M, int n_base, int mt, int lane, const f32x4& v,
                                         float& mean_t, float& m2_t) {
  const int r16 = lane & 15, g = lane >> 4;
  const int m = mt * 16 + r16;
  const int n = n_base + g * 4;
  const bool nok = n < J.N, ok = nok && m < M;
  float o[4] = {v[0], v[1], v[2], v[3]};
  if (J.bias && nok) {
    const uint2 b = *reinterpret_cast<const uint2*>(J.bias + n);
    o[0] += e2f<DT>(b.x & 0xffffu);
    o[1] += e2f<DT>(b.x >> 16);
    o[2] += e2f<DT>(b.y & 0xffffu);
    o[3] += e2f<DT>(b.y >> 16);
  }
  if (J.act == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = gelu_tanh(o[i]);
  } else if (J.act == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = 0.5f * o[i] * (1.f + erff(o[i] * 0.70710678118654752f));
  }
  if (J.res && ok) {
    const uint2 r = *reinterpret_cast<const uint2*>(J.res + (long long)m * J.ldr + n);
    o[0] += e2f<DT>(r.x & 0xffffu);
    o[1] += e2f<DT>(r.x >> 16);
    o[2] += e2f<DT>(r.y & 0xffffu);
    o[3] += e2f<DT>(r.y >> 16);
  }
  uint32_t q[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = f2e<DT>(o[i]);
  if (ok) *reinterpret_cast<uint2*>(J.y + (long long)m * J.ldy + n) = make_uint2(q[0] | (q[1] << 16), q[2] | (q[3] << 16));
  if (J.part) {
    // statistics over the rounded new residual stream (ln_rows' convention); every lane shuffles
    float f[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = e2f<DT>(q[i]);
    rs_tile16(f, mean_t, m2_t);
  }
}

// Wave-local ordering of the LDS transpose: the lanes that read a fragment are not the lanes that
// wrote it, so the compiler must not move a read above the writes; the LDS runs one wave's
// operations in issue order.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Chunk c of the job's concatenated K (part 0's chunks, then part 1's): part index and offset.
__device__ __forceinline__ int chunk_part(const MmJob& J, int c, int nc0, int kc, int& k0) {
  const int pi = (J.nparts > 1 && c >= nc0) ? 1 : 0;
  k0 = (c - (pi ? nc0 : 0)) * kc;
  return pi;
}

template <int MT, int NRW, int KC, int WV>
struct MmTile {
  static constexpr int PPR = KC / 8;    // 16-B pieces per row per chunk
  static constexpr int RPI = 64 / PPR;  // weight rows per load instruction
  static constexpr int NI = 16 / RPI;   // load instructions per 16-row tile
  static constexpr int S = KC / 32;     // MFMA steps per chunk
  static constexpr int XP = (MT * 16 * PPR + WV * 64 - 1) / (WV * 64);  // x pieces per thread per chunk
  static constexpr int XS = MT * 16 * KC;                 // one x stage (elements)
  static constexpr int SLOT = NRW * 16 * KC;              // one wave's transpose slot (elements)
  static constexpr int LDS = (2 * XS + WV * SLOT) * 2;
  static_assert(PPR >= 16 && PPR <= 64, "swizzle needs 16..64 pieces per row");
};

template <int DT, int MT, int NRW, int KC, int WV, bool LN, int PF>
__global__ __launch_bounds__(WV * 64) void mm_skinny_kernel(MmArgs a) {
  using T = MmTile<MT, NRW, KC, WV>;
  extern __shared__ __attribute__((aligned(16))) uint16_t mm_lds[];  // xs[2][MT*16][KC], slots[WV][NRW*16][KC]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  int b = blockIdx.x;
  const int bglob = b;
  const bool second = b >= a.j[0].tiles;
  const MmJob& J = second ? a.j[1] : a.j[0];
  if (second) b -= a.j[0].tiles;
  const int M = a.M, N = J.N;
  const int kz = blockIdx.y, KS = gridDim.y;
  const int nw0 = b * (WV * NRW * 16) + wv * (NRW * 16);  // this wave's first row
  uint16_t* xs = mm_lds;
  uint16_t* slot = mm_lds + 2 * T::XS + wv * T::SLOT;

  // K chunks of the concatenated parts, this workgroup's share [c_lo, c_hi)
  const int nc0 = (J.p[0].K + KC - 1) / KC;
  const int nct = nc0 + (J.nparts > 1 ? (J.p[1].K + KC - 1) / KC : 0);
  const int per = (nct + KS - 1) / KS;
  const int c_lo = kz * per, c_hi = min(nct, c_lo + per);

  // weight load map: lane takes row lr of each instruction, piece lp
  const int lr = lane / T::PPR, lp = lane % T::PPR;
  auto load_w = [&](int c, u32x4v (&wr)[NRW][T::NI]) {
    int k0;
    const MmPart& P = J.p[chunk_part(J, c, nc0, KC, k0)];
    const bool kv = k0 + lp * 8 < P.K;
#pragma unroll
    for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
      for (int i = 0; i < T::NI; ++i) {
        int n = nw0 + nr * 16 + i * T::RPI + lr;
        n = n < N ? n : N - 1;  // rows past N: any valid row (their outputs are never stored)
        const int kk = k0 + lp * 8;
        const long long off = P.packed ? (long long)(n >> 4) * P.ldw + ((long long)(kk >> 7) * 16 + (n & 15)) * 128 +
                                             (kk & 127)
                                       : (long long)n * P.ldw + kk;
        wr[nr][i] = kv ? ld_nt16(P.w + off) : u32x4v{0u, 0u, 0u, 0u};
      }
  };
  // activation chunk: piece q = tid + WV*64 j of the [MT*16][PPR] stage
  // activation chunk: piece q = tid + WV*64 j of the [MT*16][PPR] stage -- row m_j = q / PPR (fixed per
  // thread and j), column piece tid % PPR (the same for every j). LN-on-load: the rows' (mean, rstd)
  // are read once per part, gamma / beta once per chunk, the normalisation runs at staging time (the
  // first version re-read all four per piece: 5 loads per 16 B of activation)
  static_assert((WV * 64) % T::PPR == 0, "a thread's pieces share one column");
  const int xp = tid % T::PPR;
  float mu[2][T::XP], rsd[2][T::XP];
  // the rows' (mean, rstd) per part: read (merged stats) or merged here from the producer's partials
  // (st_nt > 0: one wave per row, lanes over slices, Chan's equal-count merge as mm_tail.h rs_merge)
  __shared__ float s_ms[2][64][2];  // merged (mean, rstd) per part and row (st_nt > 0)
  auto ln_stats = [&]() {
    if constexpr (LN) {
      bool merged = false;
#pragma unroll
      for (int pi = 0; pi < 2; ++pi) {
        if (pi >= J.nparts || J.p[pi].st_nt <= 0) continue;
        merged = true;
        const MmPart& P = J.p[pi];
        const int NT = P.st_nt;
        const float c = (float)P.K / (float)NT;
        for (int m = wv; m < M; m += WV) {
          const float* pp = P.stats + (long long)m * NT * 2;
          float2 v[16];  // NT <= 1024 slices per row
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int t = lane + 64 * i;
            v[i] = t < NT ? *reinterpret_cast<const float2*>(pp + 2 * t) : make_float2(0.f, 0.f);
          }
          float sm = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i) sm += v[i].x;
          const float mean = wave_sum(sm) / (float)NT;
          float q = 0.f;
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (lane + 64 * i < NT) q += v[i].y + c * (v[i].x - mean) * (v[i].x - mean);
          const float var = wave_sum(q) / (float)P.K;
          if (lane == 0) {
            s_ms[pi][m][0] = mean;
            s_ms[pi][m][1] = rsqrtf(var + P.st_eps);
          }
        }
      }
      if (merged) __syncthreads();
#pragma unroll
      for (int pi = 0; pi < 2; ++pi)
#pragma unroll
        for (int j = 0; j < T::XP; ++j) {
          const int m = (tid + WV * 64 * j) / T::PPR;
          mu[pi][j] = 0.f;
          rsd[pi][j] = 0.f;
          if (pi < J.nparts && m < M) {
            if (J.p[pi].st_nt > 0) {
              mu[pi][j] = s_ms[pi][m][0];
              rsd[pi][j] = s_ms[pi][m][1];
            } else {
              const float2 v = *reinterpret_cast<const float2*>(J.p[pi].stats + 2 * m);
              mu[pi][j] = v.x;
              rsd[pi][j] = v.y;
            }
          }
        }
    }
  };
  auto load_x = [&](int c, u32x4v (&xr)[T::XP], u32x4v& gv, u32x4v& bv) {
    int k0;
    const MmPart& P = J.p[chunk_part(J, c, nc0, KC, k0)];
    const int k = k0 + xp * 8;
#pragma unroll
    for (int j = 0; j < T::XP; ++j) {
      const int m = (tid + WV * 64 * j) / T::PPR;
      xr[j] = (m < M && k < P.K) ? ld16(P.x + (long long)m * P.ldx + k) : u32x4v{0u, 0u, 0u, 0u};
    }
    if constexpr (LN) {
      gv = k < P.K ? ld16(P.gamma + k) : u32x4v{0u, 0u, 0u, 0u};
      bv = (P.beta && k < P.K) ? ld16(P.beta + k) : u32x4v{0u, 0u, 0u, 0u};
    }
  };
  auto store_x = [&](u32x4v (&xr)[T::XP], const u32x4v& gv, const u32x4v& bv, int c, int buf) {
#pragma unroll
    for (int j = 0; j < T::XP; ++j) {
      const int m = (tid + WV * 64 * j) / T::PPR;
      if (m >= MT * 16) continue;
      if constexpr (LN) {
        int k0;
        const int pi = chunk_part(J, c, nc0, KC, k0);
        const float mj = pi ? mu[1][j] : mu[0][j], rj = pi ? rsd[1][j] : rsd[0][j];
        u32x4v o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t hx = xr[j][e], gg = gv[e], bb = bv[e];
          const float lo = (e2f<DT>(hx & 0xffffu) - mj) * rj * e2f<DT>(gg & 0xffffu) + e2f<DT>(bb & 0xffffu);
          const float hi = (e2f<DT>(hx >> 16) - mj) * rj * e2f<DT>(gg >> 16) + e2f<DT>(bb >> 16);
          o[e] = f2e<DT>(lo) | (f2e<DT>(hi) << 16);
        }
        xr[j] = m < M ? o : u32x4v{0u, 0u, 0u, 0u};
      }
      *reinterpret_cast<u32x4v*>(xs + buf * T::XS + m * KC + ((xp ^ (m & 15)) << 3)) = xr[j];
    }
  };

  f32x4 acc[NRW][MT];
#pragma unroll
  for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[nr][mt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one chunk: its weight registers -> the wave's LDS slot, then chunk c + PF is requested into the
  // freed registers (PF register sets in a ring: PF chunks of weight in flight per wave), the next
  // activation chunk is staged, the MFMAs run. PF > 1 pays where the LDS, not the registers, caps the
  // resident workgroups (M = 32: 64 KB per workgroup, 2 per CU)
  u32x4v xr[T::XP], gv = {0u, 0u, 0u, 0u}, bv = {0u, 0u, 0u, 0u};
  auto chunk = [&](int c, u32x4v (&w)[NRW][T::NI]) {
    const int buf = (c - c_lo) & 1;
    wave_lds_sync();
#pragma unroll
    for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
      for (int i = 0; i < T::NI; ++i) {
        const int row = i * T::RPI + lr;
        *reinterpret_cast<u32x4v*>(slot + (nr * 16 + row) * KC + ((lp ^ (row & 15)) << 3)) = w[nr][i];
      }
    if (c + PF < c_hi) load_w(c + PF, w);
    const bool nx = c + 1 < c_hi;
    if (nx) load_x(c + 1, xr, gv, bv);
    wave_lds_sync();
    const uint16_t* xb = xs + buf * T::XS;
#pragma unroll
    for (int st = 0; st < T::S; ++st) {
      u32x4v bf[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        bf[mt] = *reinterpret_cast<const u32x4v*>(xb + (mt * 16 + r16) * KC + (((4 * st + g) ^ r16) << 3));
#pragma unroll
      for (int nr = 0; nr < NRW; ++nr) {
        const u32x4v af = *reinterpret_cast<const u32x4v*>(slot + (nr * 16 + r16) * KC + (((4 * st + g) ^ r16) << 3));
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[nr][mt] = mfma16<DT>(af, bf[mt], acc[nr][mt]);
      }
    }
    if (nx) store_x(xr, gv, bv, c + 1, buf ^ 1);
    __syncthreads();
  };
  u32x4v wa[PF][NRW][T::NI];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (c_lo + q < c_hi) load_w(c_lo + q, wa[q]);
  ln_stats();  // (under the first weight chunk's loads)
  if (c_lo < c_hi) {
    load_x(c_lo, xr, gv, bv);
    store_x(xr, gv, bv, c_lo, 0);
  }
  __syncthreads();
  for (int c0 = c_lo; c0 < c_hi; c0 += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q)
      if (c0 + q < c_hi) chunk(c0 + q, wa[q]);
  }

  // split-K: publish this slice's tiles, the last arriving slice of the N block sums and stores
  bool fin = true;
  if (KS > 1) {
    constexpr int TPW = NRW * MT;  // tiles per wave
    const long long blk = (long long)bglob * (WV * TPW) + wv * TPW;
    const long long nblk = (long long)gridDim.x * (WV * TPW);
#pragma unroll
    for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float* d = a.ws + ((kz * nblk + blk + nr * MT + mt) * 64 + lane) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) st_pub(d + e, acc[nr][mt][e]);
      }
    __shared__ int s_fin;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned* bc = a.bcnt + bglob;
      const int last = __hip_atomic_fetch_add(bc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)KS - 1;
      if (last) {
        __hip_atomic_store(bc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_fin = last;
    }
    __syncthreads();
    fin = s_fin != 0;
    if (fin) {
      // every slice's tile summed in slice order 0..KS-1 (this slice's own from registers), whichever
      // slice arrives last -- the result is deterministic (seeded sampling reproduces under replay);
      // UZ slices' loads in flight at a time (a serial chain of KS - 1 L2 round trips sat on every
      // block's critical path: profiles/mm_bench_r6_v4_nsplit_splitk.jsonl)
      constexpr int UZ = TPW >= 4 ? 2 : (TPW >= 2 ? 4 : 8);
      f32x4 own[NRW][MT];
#pragma unroll
      for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          own[nr][mt] = acc[nr][mt];
          acc[nr][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      for (int z0 = 0; z0 < KS; z0 += UZ) {
        f32x4 part[UZ][NRW][MT];
#pragma unroll
        for (int u = 0; u < UZ; ++u) {
          const int z = z0 + u;
#pragma unroll
          for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
              part[u][nr][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
              if (z < KS && z != kz)
                part[u][nr][mt] =
                    *reinterpret_cast<const f32x4*>(a.ws + ((z * nblk + blk + nr * MT + mt) * 64 + lane) * 4);
            }
        }
#pragma unroll
        for (int u = 0; u < UZ; ++u)
#pragma unroll
          for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[nr][mt] += (z0 + u == kz) ? own[nr][mt] : part[u][nr][mt];
      }
    }
  }
  if (!fin) return;  // (workgroup-uniform)
  float tm[NRW][MT], tq[NRW][MT];
#pragma unroll
  for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) mm_store<DT>(J, M, nw0 + nr * 16, mt, lane, acc[nr][mt], tm[nr][mt], tq[nr][mt]);
  if (J.part && !J.stats_out) {
    // publish-only (the consumer merges, MmPart.st_nt): every 16-row tile's (mean, M2) per row, slice
    // index = tile row / 16 -- no LDS reduction, no arrival
    const RowStats s{J.part, nullptr, nullptr, M, J.N, J.eps, 16};
#pragma unroll
    for (int nr = 0; nr < NRW; ++nr)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = mt * 16 + r16;
        if (g == 0 && m < M && nw0 + nr * 16 < J.N) rs_publish(s, m, (nw0 + nr * 16) >> 4, tm[nr][mt], tq[nr][mt]);
      }
  } else if (J.part) {
    // the block's row statistics: the wave's NRW tiles merged in registers, the WV waves through LDS,
    // one (mean, M2) per row per block published (N % (WV * NRW * 16) == 0 for a stats job)
    float* red = reinterpret_cast<float*>(mm_lds);  // [WV][MT*16][2]
    __syncthreads();  // (the LDS held the last chunk's stages)
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float mean[NRW], m2[NRW], mo, qo;
#pragma unroll
        for (int nr = 0; nr < NRW; ++nr) {
          mean[nr] = tm[nr][mt];
          m2[nr] = tq[nr][mt];
        }
        chan_merge<NRW>(mean, m2, 16.f, mo, qo);
        red[(wv * MT * 16 + mt * 16 + r16) * 2] = mo;
        red[(wv * MT * 16 + mt * 16 + r16) * 2 + 1] = qo;
      }
    }
    __syncthreads();
    const RowStats s{J.part, J.stats_out, J.cnt, M, J.N, J.eps, WV * NRW * 16};
    for (int m = tid; m < M; m += WV * 64) {
      float mean[WV], m2[WV], mo, qo;
#pragma unroll
      for (int w = 0; w < WV; ++w) {
        mean[w] = red[(w * MT * 16 + m) * 2];
        m2[w] = red[(w * MT * 16 + m) * 2 + 1];
      }
      chan_merge<WV>(mean, m2, 16.f * NRW, mo, qo);
      rs_publish(s, m, b, mo, qo);
    }
    rs_arrive_of(s, b, J.tiles);
  }
}

// launch-shape knob (same-box A/B): workgroups a launch aims for when it splits K
// launch-shape knob (same-box A/B): workgroups a K-split launch aims for (0: built-in, mm_plan_ks)
static int g_mm_target_wg = 0;
KCA_API int kca_mm_skinny_set(int target_wg) {
  g_mm_target_wg = target_wg > 0 ? target_wg : 0;
  return 0;
}

// Variants: KC (K per chunk: 256 = 2 weight rows x 512 B per load instruction, 128 = 4 rows x
// 256 B) and WV (waves per workgroup, 4 or 8: an 8-wave block shares each activation chunk over
// twice the weight rows). Defaults per (MT, NRW) from the mm_bench sweeps (profiles/mm_sweep_r6/);
// a.kc / a.wv override (A/B).
constexpr int mm_kc_default(int MT, int NRW) { return MT * NRW >= 4 ? 128 : 256; }

struct MmPlan {
  int mt, nrw, kc, wv, pf, ks, nblk;
  long long ws_floats;
};

// K split: about T workgroups per launch, T = 512 (one 16-row activation tile) / 384 (more), i.e.
// ks = round(T / blocks). From a forced-split sweep over the fused-layer shapes
// (profiles/mm_ks_sweep_r6/): the best split landed every launch at 448-768 workgroups at M = 8 and
// 224-512 at M = 32 (2 resident per CU there); filling the resident slots exactly (ks = cap / blocks)
// under-filled the 448-block GPT-J [QKV | fc_in] launch's neighbours and a time model that charged
// a workgroup one chunk of overhead over-split every shape (profiles/mm_bench_r6_v6_ks_model_rejected.jsonl).
static void mm_plan_ks(MmArgs& a, MmPlan& p, int target) {
  int nct = 1;
  for (int i = 0; i < a.njobs; ++i) {
    int c = 0;
    for (int q = 0; q < a.j[i].nparts; ++q) c += (a.j[i].p[q].K + p.kc - 1) / p.kc;
    nct = c > nct ? c : nct;
  }
  int ks = a.ks > 0 ? a.ks : (2 * target + p.nblk) / (2 * p.nblk);
  if (ks > nct) ks = nct;
  if (ks > 32) ks = 32;
  if (ks < 1) ks = 1;
  const int per = (nct + ks - 1) / ks;
  ks = (nct + per - 1) / per;
  p.ks = ks;
  p.ws_floats = ks > 1 ? (long long)ks * p.nblk * p.wv * p.nrw * p.mt * 256 : 0;
}

template <int DT, int MT, int NRW, int KC, int WV, bool LN>
static void mm_go(MmArgs& a, MmPlan& p, hipStream_t s, bool launch) {
  using T = MmTile<MT, NRW, KC, WV>;
  mm_plan_ks(a, p, g_mm_target_wg > 0 ? g_mm_target_wg : (MT == 1 ? 512 : 384));
  if (!launch) return;
  a.ks = p.ks;
  // (PF = 2 / 3 chunks in flight measured slower at every M, KC and shape: profiles/mm_pf_sweep_r6/ --
  // the ring stays in the kernel, one instantiation is built)
  hipLaunchKernelGGL((mm_skinny_kernel<DT, MT, NRW, KC, WV, LN, 1>), dim3(p.nblk, p.ks), dim3(WV * 64), T::LDS, s, a);
}

template <int DT, int MT, int NRW, bool LN>
static void mm_dispatch_kc(MmArgs& a, MmPlan& p, hipStream_t s, bool launch) {
  if (p.kc == 256) {
    if (p.wv == 8) mm_go<DT, MT, NRW, 256, 8, LN>(a, p, s, launch);
    else mm_go<DT, MT, NRW, 256, 4, LN>(a, p, s, launch);
  } else {
    if (p.wv == 8) mm_go<DT, MT, NRW, 128, 8, LN>(a, p, s, launch);
    else mm_go<DT, MT, NRW, 128, 4, LN>(a, p, s, launch);
  }
}

template <int DT, int MT, bool LN>
static void mm_dispatch_nr(MmArgs& a, MmPlan& p, hipStream_t s, bool launch) {
  if constexpr (MT < 4) {
    if (p.nrw == 2) {
      mm_dispatch_kc<DT, MT, 2, LN>(a, p, s, launch);
      return;
    }
  }
  mm_dispatch_kc<DT, MT, 1, LN>(a, p, s, launch);
}

template <int DT, bool LN>
static void mm_dispatch_mt(MmArgs& a, MmPlan& p, hipStream_t s, bool launch) {
  if (p.mt == 1) mm_dispatch_nr<DT, 1, LN>(a, p, s, launch);
  else if (p.mt == 2) mm_dispatch_nr<DT, 2, LN>(a, p, s, launch);
  else mm_dispatch_nr<DT, 4, LN>(a, p, s, launch);
}

static MmPlan mm_plan(MmArgs& a) {
  MmPlan p;
  p.mt = a.M <= 16 ? 1 : (a.M <= 32 ? 2 : 4);
  p.nrw = (a.nr == 2 && p.mt < 4) ? 2 : 1;
  // 32-64 rows with a long K: 8-wave workgroups over 128-wide K chunks -- twice the weight rows share
  // each staged activation chunk, whose L2 re-reads grow with M (M = 32: 465 -> 448 us, M = 64:
  // 621 -> 541 us summed over the fused-layer shapes; short-K shapes lose: profiles/mm_shape_sweep_r6/)
  int kmax = 0;
  for (int i = 0; i < a.njobs; ++i) {
    int k = 0;
    for (int q = 0; q < a.j[i].nparts; ++q) k += a.j[i].p[q].K;
    kmax = k > kmax ? k : kmax;
  }
  const bool wide = p.mt >= 2 && kmax >= 6144;
  p.kc = a.kc == 128 || a.kc == 256 ? a.kc : (wide ? 128 : mm_kc_default(p.mt, p.nrw));
  if (p.kc == 256 && p.mt * p.nrw >= 4) p.kc = 128;  // (register budget)
  p.wv = a.wv == 4 || a.wv == 8 ? a.wv : (wide ? 8 : 4);
  p.pf = 1;
  const int rows = p.wv * p.nrw * 16;
  p.nblk = 0;
  for (int i = 0; i < a.njobs; ++i) {
    a.j[i].tiles = (a.j[i].N + rows - 1) / rows;
    p.nblk += a.j[i].tiles;
    if (a.j[i].part && (a.j[i].N % rows || a.j[i].N / rows > 256)) p.nblk = -1;  // whole blocks, <= 256 slices
  }
  if (a.njobs < 2) a.j[1].tiles = 0;
  p.ks = 1;
  p.ws_floats = 0;
  return p;
}

static void mm_dispatch(MmArgs& a, MmPlan& p, int dtype, int ln, hipStream_t s, bool launch) {
  if (dtype == 0) {
    if (ln) mm_dispatch_mt<0, true>(a, p, s, launch);
    else mm_dispatch_mt<0, false>(a, p, s, launch);
  } else {
    if (ln) mm_dispatch_mt<1, true>(a, p, s, launch);
    else mm_dispatch_mt<1, false>(a, p, s, launch);
  }
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static bool al8(const void* p) { return ((uintptr_t)p & 7) == 0; }

static int mm_check(const MmArgs& a, int dtype, int& ln) {
  if (a.njobs < 1 || a.njobs > 2 || a.M < 1 || a.M > 64 || dtype < 0 || dtype > 1) return 1;
  ln = -1;
  for (int i = 0; i < a.njobs; ++i) {
    const MmJob& J = a.j[i];
    if (J.N < 1 || J.N % 4 || J.nparts < 1 || J.nparts > 2 || !J.y || J.ldy % 4 || !al8(J.y) || !al8(J.bias)) return 1;
    if (J.res && (J.ldr % 4 || !al8(J.res) || J.act)) return 1;
    if (J.part && (J.N % 16 || (J.stats_out && !J.cnt))) return 1;
    for (int q = 0; q < J.nparts; ++q) {
      const MmPart& P = J.p[q];
      if (P.K < 8 || P.K % 8 || P.ldx % 8 || P.ldw % 8 || !P.x || !P.w || !al16(P.x) || !al16(P.w)) return 2;
      const int l = P.stats ? 1 : 0;
      if (ln >= 0 && l != ln) return 3;  // one LN mode per launch
      ln = l;
      if (l && (!P.gamma || !al16(P.gamma) || !al16(P.beta))) return 2;
      if (l && P.st_nt > 0 && (P.st_nt > 1024 || P.K % P.st_nt || !al8(P.stats))) return 2;
    }
  }
  return 0;
}

// Workspace a launch of these arguments needs: ws floats and per-block counters (0 if no K split).
KCA_API int kca_mm_skinny_plan(const MmArgs* in, int dtype, long long* ws_floats, int* bcnt_n, int* ks) {
  if (!in) return 1;
  MmArgs a = *in;
  int ln;
  const int rc = mm_check(a, dtype, ln);
  if (rc) return rc;
  MmPlan p = mm_plan(a);
  if (p.nblk < 0) return 6;
  mm_dispatch(a, p, dtype, ln, nullptr, false);
  *ws_floats = p.ws_floats;
  *bcnt_n = p.ks > 1 ? p.nblk : 0;
  *ks = p.ks;
  return 0;
}

// dtype: 0 bf16, 1 fp16. Returns nonzero (nothing launched) for shapes outside the kernel or a
// workspace smaller than kca_mm_skinny_plan's.
KCA_API int kca_mm_skinny(const MmArgs* in, int dtype, hipStream_t stream) {
  if (!in) return 1;
  MmArgs a = *in;
  int ln;
  const int rc = mm_check(a, dtype, ln);
  if (rc) return rc;
  MmPlan p = mm_plan(a);
  if (p.nblk < 0) return 6;
  mm_dispatch(a, p, dtype, ln, stream, false);
  if (p.ks > 1 && (!a.ws || !a.bcnt || a.ws_floats < p.ws_floats || a.bcnt_n < p.nblk || !al16(a.ws))) return 5;
  mm_dispatch(a, p, dtype, ln, stream, true);
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

// Sizes the Python mirror of the descriptor checks (ctypes.Structure layout == this ABI)
KCA_API int kca_mm_skinny_abi(int* sizes) {
  sizes[0] = (int)sizeof(MmPart);
  sizes[1] = (int)sizeof(MmJob);
  sizes[2] = (int)sizeof(MmArgs);
  return 0;
}
