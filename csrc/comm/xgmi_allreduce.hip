// Custom all-reduce over xGMI peer memory.
//
// BLOOM TP=8 decode runs ~140 all-reduces of B x 14336 bf16 per token and TP
// prefill / NeoX TP training run MB-sized ones; RCCL's ring pays 2(W-1) link
// latencies per call. On an 8-GPU xGMI mesh every GPU has a direct link to
// every peer, so a kernel can read all 7 peers' buffers concurrently:
//
//   * one-shot  (small, latency-bound): every rank reads the WHOLE message
//     from all W staging buffers and sums -> 1 sync round, (W-1)*n bytes over
//     the links per rank;
//   * two-shot  (medium/large, bandwidth-bound): reduce-scatter then
//     all-gather through peer memory -> 2 sync rounds, 2(W-1)/W*n bytes per
//     rank, all 7 links busy in both phases.
//
// Memory: per rank, two staging buffers (double-buffered by call parity) and a
// signal block (per-block arrival flags written by peers) in device-uncached
// memory shared through hipIpc handles, plus a local control block (call
// sequence number, finished-block counter, sticky error word).
//
// Ordering/race argument (this replaces round 1's per-block counters, whose
// parities drifted apart when the block count or slice map changed between
// calls): the call number is ONE per-rank sequence word, read by every block
// at kernel start and advanced once every block has read it (by the last block
// to finish, or -- in the fused LayerNorm / row-statistics closes -- by the
// block that sees the launch's own all-blocks exchange complete). Flags compare
// `>= call`, so blocks that sat out intermediate calls are still correct.
// Call k+2 reuses call k's parity; before ANY block of call k+1 on rank X
// finished, it observed every peer Y arriving at call k+1, and Y's call-(k+1)
// kernel can only start after Y's call-k kernel completed (same stream) --
// so no peer is still reading X's call-k staging when X's call k+2 writes it,
// whatever the slice->block mapping of the three calls.
//
// A bounded spin sets the sticky error word and poisons the output with NaN
// (never a plausible wrong sum); the host wrapper raises on it.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../kernels/common.h"
#include "../kernels/decode_tail.h"
#include "../kernels/mm_tail.h"

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 128;

struct ARSignal {  // uncached, IPC-shared: written by peers
  uint32_t flag[2][AR_MAX_BLOCKS][AR_MAX_RANKS];  // [phase][block][peer] = last call the peer reached
};

struct ARCtl {  // local (cached) control words, touched only by this rank's kernels
  uint32_t seq;    // calls completed
  uint32_t done;   // blocks finished in the running call
  uint32_t error;  // sticky: 1 = spin timeout
  uint32_t pad;
};

struct ARPeers {
  bf16_t* stage[2][AR_MAX_RANKS];  // staging buffers of every rank (own included)
  ARSignal* sig[AR_MAX_RANKS];     // signal blocks of every rank
};

__device__ __forceinline__ void st_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t ar_begin(ARCtl* ctl) {
  __shared__ uint32_t s_call;
  if (threadIdx.x == 0) s_call = __hip_atomic_load(&ctl->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  return s_call;
}

// Last block out advances the sequence word (all blocks have read it by then:
// the nb-th finisher runs after every block started).
__device__ __forceinline__ void ar_end(ARCtl* ctl, uint32_t call) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t old = __hip_atomic_fetch_add(&ctl->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(&ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ctl->seq, call, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Publish this block's arrival at (phase, call) to every peer, then wait until
// every peer's same-index block arrived. Returns false on timeout.
template <int W>
__device__ __forceinline__ bool ar_sync(const ARPeers& peers, ARCtl* ctl, int rank, int phase, uint32_t call,
                                        long long spin_limit) {
  __shared__ int s_ok;
  const int b = blockIdx.x, tid = threadIdx.x;
  // W = 1 (a TP rank emulated on one GPU, parallel/tp_emulation.py): no peer to order the staging
  // against, so the round is a drain + barrier + relaxed flag store / poll without the system-scope
  // L2 writeback / invalidate (res_stats 13.3 -> 10.3 us per call at B = 8, profiles/ar_tail_r6.jsonl).
  // W > 1 keeps the system-scope release / acquire: whether a drained store to a peer's uncached
  // memory over xGMI is visible before the flag is not something this tree can test on one GPU.
  constexpr bool light = W == 1;
  if constexpr (light) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    __threadfence_system();
  }
  __syncthreads();
  if (tid == 0) s_ok = 1;
  if (tid < W) {
    if constexpr (light)
      __hip_atomic_store(&peers.sig[tid]->flag[phase][b][rank], call, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      st_sys(&peers.sig[tid]->flag[phase][b][rank], call);
  }
  __syncthreads();
  if (tid < W) {
    const uint32_t* f = &peers.sig[rank]->flag[phase][b][tid];
    long long spins = 0;
    while ((light ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : ld_sys(f)) < call) {
      if (++spins > spin_limit) {
        __hip_atomic_fetch_or(&ctl->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  return s_ok != 0;
}

__device__ __forceinline__ void debug_delay(int delay) {
  for (int i = 0; i < delay; ++i) __builtin_amdgcn_s_sleep(127);
}

// fp32 sums of 8 elements (one 16-byte chunk `i`) over the W stagings. DT: 0 bf16, 1 fp16 (common.h)
template <int W, int DT>
__device__ __forceinline__ void sum_peers8(const ARPeers& peers, int par, long long i, float (&acc)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int r = 0; r < W; ++r) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(peers.stage[par][r]) + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[2 * j] += e2f<DT>(v[j] & 0xffffu);
      acc[2 * j + 1] += e2f<DT>(v[j] >> 16);
    }
  }
}

template <int W, int DT>
__device__ __forceinline__ uint4 sum_peers(const ARPeers& peers, int par, long long i) {
  float acc[8];
  sum_peers8<W, DT>(peers, par, i, acc);
  uint4 o;
  o.x = f2e<DT>(acc[0]) | (f2e<DT>(acc[1]) << 16);
  o.y = f2e<DT>(acc[2]) | (f2e<DT>(acc[3]) << 16);
  o.z = f2e<DT>(acc[4]) | (f2e<DT>(acc[5]) << 16);
  o.w = f2e<DT>(acc[6]) | (f2e<DT>(acc[7]) << 16);
  return o;
}

// 8 quiet NaNs of the element type: the poison a timed-out sync leaves in the output
template <int DT>
__device__ __forceinline__ uint4 nan8() {
  const uint32_t q = DT == 0 ? 0x7fc07fc0u : 0x7e007e00u;
  return make_uint4(q, q, q, q);
}

// ---------------------------------------------------------------- one-shot
template <int W, int DT>
__global__ __launch_bounds__(512) void ar_one_shot_kernel(ARPeers peers, ARCtl* ctl, int rank,
                                                          const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                          long long n8, long long spin_limit, int delay) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  const uint32_t call = ar_begin(ctl);
  const int par = call & 1;
  const long long per = (n8 + nb - 1) / nb;
  const long long lo = b * per, hi = min(n8, lo + per);
  uint4* mine = reinterpret_cast<uint4*>(peers.stage[par][rank]);
  for (long long i = lo + tid; i < hi; i += blockDim.x) mine[i] = reinterpret_cast<const uint4*>(in)[i];
  const bool ok = ar_sync<W>(peers, ctl, rank, 0, call, spin_limit);
  debug_delay(delay);
  for (long long i = lo + tid; i < hi; i += blockDim.x)
    reinterpret_cast<uint4*>(out)[i] = ok ? sum_peers<W, DT>(peers, par, i) : nan8<DT>();
  ar_end(ctl, call);
}

// ---------------------------------------------------------------- two-shot
// The message is cut into W partitions; block b owns sub-slice b of every
// partition on every rank, so phase flags are per block index.
//   phase A: copy own input into staging; sync
//   reduce : rank r sums sub-slice b of partition r over all W stagings and
//            writes the bf16 result in place into its OWN staging (no peer
//            reads partition r of rank r's staging before phase B); sync
//   gather : read sub-slice b of partition p from rank p's staging, all p.
template <int W, int DT>
__global__ __launch_bounds__(512) void ar_two_shot_kernel(ARPeers peers, ARCtl* ctl, int rank,
                                                          const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                          long long n8, long long spin_limit, int delay) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  const uint32_t call = ar_begin(ctl);
  const int par = call & 1;
  const long long part = (n8 + W - 1) / W;
  const long long sub = (part + nb - 1) / nb;
  uint4* mine = reinterpret_cast<uint4*>(peers.stage[par][rank]);
  const uint4* src = reinterpret_cast<const uint4*>(in);
#pragma unroll
  for (int p = 0; p < W; ++p) {
    const long long pend = min(n8, (p + 1) * part);
    const long long lo = p * part + b * sub, hi = min(pend, lo + sub);
    for (long long i = lo + tid; i < hi; i += blockDim.x) mine[i] = src[i];
  }
  bool ok = ar_sync<W>(peers, ctl, rank, 0, call, spin_limit);
  debug_delay(delay);
  {
    const long long pend = min(n8, (long long)(rank + 1) * part);
    const long long lo = rank * part + b * sub, hi = min(pend, lo + sub);
    for (long long i = lo + tid; i < hi; i += blockDim.x) {
      const uint4 v = sum_peers<W, DT>(peers, par, i);
      mine[i] = ok ? v : nan8<DT>();
    }
  }
  ok = ar_sync<W>(peers, ctl, rank, 1, call, spin_limit) && ok;
  uint4* dst = reinterpret_cast<uint4*>(out);
#pragma unroll
  for (int p = 0; p < W; ++p) {
    const long long pend = min(n8, (p + 1) * part);
    const long long lo = p * part + b * sub, hi = min(pend, lo + sub);
    const u32x4* s = reinterpret_cast<const u32x4*>(peers.stage[par][p]);
    for (long long i = lo + tid; i < hi; i += blockDim.x) {
      const u32x4 v = __builtin_nontemporal_load(s + i);
      dst[i] = ok ? make_uint4(v[0], v[1], v[2], v[3]) : nan8<DT>();
    }
  }
  ar_end(ctl, call);
}

// ---------------------------------------------------------------- all-gather
// Rank r's n8 chunks land at out[r*n8 ...] on every rank (the vocab-parallel
// LM head's logits): stage own input, one sync round, read every
// peer's staging. Shares the call sequence (and its race argument) with the
// all-reduce kernels above, so the two can be interleaved freely.
template <int W, int DT>
__global__ __launch_bounds__(512) void ag_kernel(ARPeers peers, ARCtl* ctl, int rank,
                                                 const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                 long long n8, long long spin_limit, int delay) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  const uint32_t call = ar_begin(ctl);
  const int par = call & 1;
  const long long per = (n8 + nb - 1) / nb;
  const long long lo = b * per, hi = min(n8, lo + per);
  uint4* mine = reinterpret_cast<uint4*>(peers.stage[par][rank]);
  const uint4* src = reinterpret_cast<const uint4*>(in);
  for (long long i = lo + tid; i < hi; i += blockDim.x) mine[i] = src[i];
  const bool ok = ar_sync<W>(peers, ctl, rank, 0, call, spin_limit);
  debug_delay(delay);
  uint4* dst = reinterpret_cast<uint4*>(out);
#pragma unroll
  for (int p = 0; p < W; ++p) {
    const u32x4* s = reinterpret_cast<const u32x4*>(peers.stage[par][p]);
    for (long long i = lo + tid; i < hi; i += blockDim.x) {
      const u32x4 v = __builtin_nontemporal_load(s + i);
      dst[p * n8 + i] = ok ? make_uint4(v[0], v[1], v[2], v[3]) : nan8<DT>();
    }
  }
  ar_end(ctl, call);
}

// ------------------------------------------------- one-shot + residual + LayerNorm (TP decode)
// Closes a row-parallel projection of the batch-1 decode layer (BLOOM TP=8: the out-projection and
// fc_out, N = 14336): every rank stages its partial y, one sync round, each workgroup sums its slice
// over the W stagings in fp32 and publishes it (st_pub) -- then the decode tail's last arriver adds
// bias + residual, rounds h' and writes LN(h') for the next projection (dual_ln_arrive_tail). The
// separate bias add and LayerNorm launches of a plain all-reduce disappear from every layer. 256
// threads (the tail's shape); the call sequence / parity protocol is the one-shot kernel's.
template <int W, int PER, int DT = 0>
__global__ __launch_bounds__(256) void ar_res_ln_kernel(ARPeers peers, ARCtl* ctl, int rank,
                                                        const bf16_t* __restrict__ in, long long n8,
                                                        long long spin_limit, DualLn a) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  const uint32_t call = ar_begin(ctl);
  const int par = call & 1;
  const long long per = (n8 + nb - 1) / nb;
  const long long lo = b * per, hi = min(n8, lo + per);
  uint4* mine = reinterpret_cast<uint4*>(peers.stage[par][rank]);
  for (long long i = lo + tid; i < hi; i += blockDim.x) mine[i] = reinterpret_cast<const uint4*>(in)[i];
  const bool ok = ar_sync<W>(peers, ctl, rank, 0, call, spin_limit);
  for (long long i = lo + tid; i < hi; i += blockDim.x) {
    float acc[8];
    sum_peers8<W, DT>(peers, par, i, acc);
    // h' = bf16(h + y + bias) for these 8 columns, handed to the LayerNorm tail (NaN on a timed-out sync)
    float h8[8], b8[8];
    load8_t<DT>(a.h + i * 8, h8);
    if (a.bias) load8_t<DT>(a.bias + i * 8, b8);
#pragma unroll
    for (int j = 0; j < 8; ++j) h8[j] = ok ? h8[j] + (acc[j] + (a.bias ? b8[j] : 0.f)) : __int_as_float(0x7fc00000);
    st_pub_x8<DT>(a.h_out + i * 8, h8);
  }
  ar_end(ctl, call);
  dual_ln_arrive_tail<PER, DT>(a);
}

// The same close with the LayerNorm distributed over the launch (the default; kca_ar_set_variant(1)
// selects the last-arriver form above): one 16-byte chunk per thread (blocks = ceil(N / 2048)), the
// thread's residual / bias / gamma / beta requested before the sync round, h' kept in registers; each
// block publishes its slice's (mean, M2), a launch-wide barrier (all blocks co-resident: <= 8 at N <=
// 16384), every block merges the partials (Chan) and normalises its own slice. No block re-reads h'
// and no single block walks the whole row (the last-arriver tail: ~10.4 us of a 10.8-us call at
// N = 14336, world 1).
template <int W, int DT>
__global__ __launch_bounds__(256) void ar_res_ln_dist_kernel(ARPeers peers, ARCtl* ctl, int rank,
                                                             const bf16_t* __restrict__ in, long long n8,
                                                             long long spin_limit, DualLn a) {
  __shared__ float red[16];
  __shared__ float s_stat[2];
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x, lane = tid & 63;
  const long long i = (long long)b * 256 + tid;
  const bool live = i < n8;
  // local operands first: independent of the peers
  u32x4 xin = {0u, 0u, 0u, 0u};
  float h8[8], b8[8], g8[8], e8[8];
  if (live) {
    xin = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint4*>(in) + i);
    load8_t<DT>(a.h + i * 8, h8);
    load8_t<DT>(a.gamma + i * 8, g8);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) b8[j] = e8[j] = 0.f;
  if (live && a.bias) load8_t<DT>(a.bias + i * 8, b8);
  if (live && a.beta) load8_t<DT>(a.beta + i * 8, e8);
  const uint32_t call = ar_begin(ctl);
  const int par = call & 1;
  if (live) reinterpret_cast<uint4*>(peers.stage[par][rank])[i] = make_uint4(xin[0], xin[1], xin[2], xin[3]);
  const bool ok = ar_sync<W>(peers, ctl, rank, 0, call, spin_limit);
  float v[8];
  float sm = 0.f;
  if (live) {
    float acc[8];
    sum_peers8<W, DT>(peers, par, i, acc);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = ok ? h8[j] + (acc[j] + b8[j]) : __int_as_float(0x7fc00000);
      v[j] = e2f<DT>(f2e<DT>(v[j]));  // h' rounded (the statistics are over the rounded stream)
      sm += v[j];
    }
    store8_t<DT>(a.h_out + i * 8, v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  // this block's slice: (mean, M2) over its cnt = 8 * live-chunks values
  const long long hi = min(n8, (long long)(b + 1) * 256);
  const float cnt = 8.f * (float)(hi - (long long)b * 256);
  const float mb = block_sum(sm, red) / cnt;
  float q = 0.f;
  if (live) {
#pragma unroll
    for (int j = 0; j < 8; ++j) q += (v[j] - mb) * (v[j] - mb);
  }
  const float m2b = block_sum(q, red + 8);
  // launch-wide exchange without a counter: each block publishes (mean, M2) as two 64-bit words
  // {call, value} (single-copy atomic: a word is this call's or a stale one), and wave 0 of every block
  // polls the nb slots until all carry this call -- one store + one poll round instead of publish,
  // drain, count, re-arm and a generation spin (ypart: >= 2 nb 64-bit words, zeroed once)
  unsigned long long* slot = reinterpret_cast<unsigned long long*>(a.ypart);
  if (tid == 0) {
    const unsigned long long tag = (unsigned long long)call << 32;
    __hip_atomic_store(slot + 2 * b, tag | __float_as_uint(mb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(slot + 2 * b + 1, tag | __float_as_uint(m2b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < 64) {  // wave 0 gathers and merges the nb (<= 64) partials
    float nt = 0.f, mt = 0.f, qt = 0.f, bad = 0.f;
    if (lane < nb) {
      unsigned long long w0 = 0ull, w1 = 0ull;
      long long spins = 0;
      while (true) {
        w0 = __hip_atomic_load(slot + 2 * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        w1 = __hip_atomic_load(slot + 2 * lane + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(w0 >> 32) == call && (uint32_t)(w1 >> 32) == call) break;
        if (++spins > spin_limit) {
          __hip_atomic_fetch_or(&ctl->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bad = 1.f;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const long long lo_t = (long long)lane * 256, hi_t = min(n8, lo_t + 256);
      nt = 8.f * (float)(hi_t - lo_t);
      mt = __uint_as_float((uint32_t)w0);
      qt = __uint_as_float((uint32_t)w1);
    }
    const float ntot = wave_sum(nt);
    const float mean = wave_sum(nt * mt) / ntot;
    const float m2 = wave_sum(qt + nt * (mt - mean) * (mt - mean));
    const bool good = wave_sum(bad) == 0.f;
    if (lane == 0) {
      s_stat[0] = mean;
      s_stat[1] = good ? rsqrtf(m2 / ntot + a.eps) : __int_as_float(0x7fc00000);
      // every block has published, so every block has read the sequence word: block 0 advances it
      // here instead of a finished-block count at exit (ar_end)
      if (b == 0) __hip_atomic_store(&ctl->seq, call, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  const float mean = s_stat[0], rstd = s_stat[1];
  if (live) {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = (v[j] - mean) * rstd;
      o[j] = v[j] * g8[j] + e8[j];
    }
    store8_t<DT>(a.xn_out + i * 8, o);
    if (a.xn2_out) {
      load8_t<DT>(a.gamma2 + i * 8, g8);
#pragma unroll
      for (int j = 0; j < 8; ++j) e8[j] = 0.f;
      if (a.beta2) load8_t<DT>(a.beta2 + i * 8, e8);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[j] * g8[j] + e8[j];
      store8_t<DT>(a.xn2_out + i * 8, o);
    }
  }
}

// ----------------------------------------- one-shot + residual + row statistics (TP decode, M rows)
// The batch 2..64 form of ar_res_ln_kernel for the matrix-core decode layer (skinny_mfma.hip): `in` is
// this rank's partial [M, N] (row-parallel out-projection / fc_out), every rank stages it, one sync
// round, each workgroup sums its slice over the W stagings in fp32 and writes h_out = bf16(h + sum +
// bias) -- then the row-statistics tail (mm_tail.h): each 8-thread group (64 columns of one row)
// publishes (mean, M2) of its rounded values, the last arriving workgroup merges them into the next
// LayerNorm's per-row (mean, rstd), which the next projection applies to h_out on load. Block slices
// are whole 64-column groups (N % 64 == 0).
template <int W, int DT>
__global__ __launch_bounds__(256) void ar_res_stats_kernel(ARPeers peers, ARCtl* ctl, int rank,
                                                           const bf16_t* __restrict__ in, long long n8,
                                                           long long spin_limit, const bf16_t* __restrict__ bias,
                                                           const bf16_t* h, bf16_t* h_out, RowStats rs) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  const uint32_t call = ar_begin(ctl);
  const int par = call & 1;
  const long long groups = n8 / 8;  // 8 x 16 B = 64 columns
  const long long gper = (groups + nb - 1) / nb;
  const long long lo = b * gper * 8, hi = min(n8, lo + gper * 8);
  uint4* mine = reinterpret_cast<uint4*>(peers.stage[par][rank]);
  for (long long i = lo + tid; i < hi; i += blockDim.x) mine[i] = reinterpret_cast<const uint4*>(in)[i];
  const long long n8row = rs.N / 8;
  // the first PRE chunks' residual / bias are requested before the sync round (local, peer-independent)
  constexpr int PRE = 2;
  u32x4 hpre[PRE], bpre[PRE];
#pragma unroll
  for (int u = 0; u < PRE; ++u) {
    const long long i = lo + tid + (long long)u * blockDim.x;
    hpre[u] = bpre[u] = u32x4{0u, 0u, 0u, 0u};
    if (i < hi) {
      hpre[u] = *reinterpret_cast<const u32x4*>(h + i * 8);
      if (bias) bpre[u] = *reinterpret_cast<const u32x4*>(bias + (i % n8row) * 8);
    }
  }
  const bool ok = ar_sync<W>(peers, ctl, rank, 0, call, spin_limit);
  int it = 0;
  for (long long i = lo + tid; i < hi; i += blockDim.x, ++it) {  // (8-thread groups stay whole: lo, hi, 256 % 8)
    float acc[8];
    sum_peers8<W, DT>(peers, par, i, acc);
    const long long row = i / n8row, col = (i % n8row) * 8;
    float h8[8], b8[8];
    if (it < PRE) {
      const u32x4 hq = it == 0 ? hpre[0] : hpre[1], bq = it == 0 ? bpre[0] : bpre[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        h8[2 * j] = e2f<DT>(hq[j] & 0xffffu);
        h8[2 * j + 1] = e2f<DT>(hq[j] >> 16);
        b8[2 * j] = e2f<DT>(bq[j] & 0xffffu);
        b8[2 * j + 1] = e2f<DT>(bq[j] >> 16);
      }
    } else {
      load8_t<DT>(h + i * 8, h8);
      if (bias) load8_t<DT>(bias + col, b8);
    }
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = ok ? h8[j] + (acc[j] + (bias ? b8[j] : 0.f)) : __int_as_float(0x7fc00000);
      v[j] = e2f<DT>(f2e<DT>(v[j]));  // statistics over the rounded stream (ln_rows' convention)
    }
    store8_t<DT>(h_out + i * 8, v);
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) sm += v[j];
    sm += __shfl_xor(sm, 1, 64);
    sm += __shfl_xor(sm, 2, 64);
    sm += __shfl_xor(sm, 4, 64);
    const float mean = sm * (1.f / 64.f);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) q += (v[j] - mean) * (v[j] - mean);
    q += __shfl_xor(q, 1, 64);
    q += __shfl_xor(q, 2, 64);
    q += __shfl_xor(q, 4, 64);
    if ((tid & 7) == 0) rs_publish(rs, (int)row, (int)(col / 64), mean, q);
  }
  if (rs.stats)
    rs_arrive_of(rs, b, nb, &ctl->seq, call);  // (its last arrival advances the sequence word)
  else
    ar_end(ctl, call);  // publish-only: the consuming projection merges the partials (MmPart.st_nt)
}

KCA_API int kca_ar_signal_bytes() { return (int)sizeof(ARSignal); }
KCA_API int kca_ar_max_blocks() { return AR_MAX_BLOCKS; }

// Uncached device allocation (coherent for peer access over xGMI).
KCA_API int kca_ar_alloc(long long bytes, void** ptr) {
  if (hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  return hipMemset(*ptr, 0, (size_t)bytes) == hipSuccess ? 0 : 2;
}

KCA_API int kca_ar_ctl_alloc(void** ptr) {
  if (hipMalloc(ptr, sizeof(ARCtl)) != hipSuccess) return 1;
  return hipMemset(*ptr, 0, sizeof(ARCtl)) == hipSuccess ? 0 : 2;
}

KCA_API int kca_ar_free(void* ptr) { return hipFree(ptr) == hipSuccess ? 0 : 1; }

KCA_API int kca_ipc_handle(void* ptr, void* handle_out /* 64 bytes */) {
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, ptr) != hipSuccess) return 1;
  memcpy(handle_out, &h, sizeof(h));
  return 0;
}

KCA_API int kca_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 1;
}

KCA_API int kca_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? 0 : 1; }

// stage0/stage1/sig: arrays of `world` device pointers (host memory).
// algo 0 = one-shot, 1 = two-shot all-reduce (in/out: n elements); algo 2 =
// all-gather (in: n elements, out: world*n). `n` bf16 elements, multiple of 8,
// and n*2 must fit the staging buffers (checked by the Python wrapper).
template <int DT>
static int ar_run(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank, int world,
                  int algo, const void* in, void* out, long long n, int blocks, long long spin_limit, int delay,
                  hipStream_t stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || n % 8 || n <= 0 || blocks < 1 ||
      blocks > AR_MAX_BLOCKS || algo < 0 || algo > 2)
    return 1;
  if (((uintptr_t)in | (uintptr_t)out) & 15) return 2;
  ARPeers p{};
  for (int r = 0; r < world; ++r) {
    p.stage[0][r] = (bf16_t*)stage0[r];
    p.stage[1][r] = (bf16_t*)stage1[r];
    p.sig[r] = (ARSignal*)sig[r];
  }
  const long long n8 = n / 8;
  ARCtl* c = (ARCtl*)ctl;
  switch (world) {
#define KCA_AR_CASE(WW)                                                                                        \
  case WW:                                                                                                     \
    if (algo == 0)                                                                                             \
      hipLaunchKernelGGL((ar_one_shot_kernel<WW, DT>), dim3(blocks), dim3(512), 0, stream, p, c, rank,               \
                         (const bf16_t*)in, (bf16_t*)out, n8, spin_limit, delay);                              \
    else if (algo == 2)                                                                                        \
      hipLaunchKernelGGL((ag_kernel<WW, DT>), dim3(blocks), dim3(512), 0, stream, p, c, rank, (const bf16_t*)in,     \
                         (bf16_t*)out, n8, spin_limit, delay);                                                 \
    else                                                                                                       \
      hipLaunchKernelGGL((ar_two_shot_kernel<WW, DT>), dim3(blocks), dim3(512), 0, stream, p, c, rank,               \
                         (const bf16_t*)in, (bf16_t*)out, n8, spin_limit, delay);                              \
    break;
    KCA_AR_CASE(1) KCA_AR_CASE(2) KCA_AR_CASE(3) KCA_AR_CASE(4) KCA_AR_CASE(5) KCA_AR_CASE(6)
    KCA_AR_CASE(7) KCA_AR_CASE(8)
#undef KCA_AR_CASE
    default:
      return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

KCA_API int kca_ar_run(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank, int world,
                       int algo, const void* in, void* out, long long n, int blocks, long long spin_limit, int delay,
                       hipStream_t stream) {
  return ar_run<0>(stage0, stage1, sig, ctl, rank, world, algo, in, out, n, blocks, spin_limit, delay, stream);
}

// fp16 elements (the sums; the all-gather copies bytes either way)
KCA_API int kca_ar_run_f16(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank,
                           int world, int algo, const void* in, void* out, long long n, int blocks,
                           long long spin_limit, int delay, hipStream_t stream) {
  return ar_run<1>(stage0, stage1, sig, ctl, rank, world, algo, in, out, n, blocks, spin_limit, delay, stream);
}

KCA_API int kca_ar_error(const void* ctl, int* err) {
  uint32_t e = 0;
  if (hipMemcpy(&e, (const char*)ctl + offsetof(ARCtl, error), 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  *err = (int)e;
  return 0;
}

// Row-parallel projection close for batch-1 decode: all-reduce `in` (bf16 [N], this rank's partial),
// then h_out = bf16(h + sum + bias), xn_out = LN(h_out) (gamma / beta / eps; gamma2 -> xn2_out: a
// second LayerNorm of the same h_out). ypart: >= N fp32 local words; cnt: 32 * 65 zero-initialised
// arrival counters (re-armed by every call). N % 8 == 0, N <= 16384, 2N bytes <= the staging size.
static int g_ar_ln_variant = 0;  // 0: distributed LayerNorm (ar_res_ln_dist_kernel), 1: last-arriver tail
KCA_API int kca_ar_set_variant(int v) {
  g_ar_ln_variant = v ? 1 : 0;
  return 0;
}

template <int DT>
static int ar_res_ln(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank, int world,
                     const void* in, int N, int blocks, long long spin_limit, const void* bias, const void* h,
                     void* h_out, const void* gamma, const void* beta, float eps, void* xn_out, const void* gamma2,
                     const void* beta2, void* xn2_out, float* ypart, unsigned int* cnt, hipStream_t stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || N % 8 || N <= 0 || N > 16384 || blocks < 1 ||
      blocks > AR_MAX_BLOCKS || !ypart || !cnt || !h || !h_out || !gamma || !xn_out || (xn2_out && !gamma2))
    return 1;
  if (((uintptr_t)in | (uintptr_t)h | (uintptr_t)h_out | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)xn_out |
       (uintptr_t)ypart | (uintptr_t)gamma2 | (uintptr_t)beta2 | (uintptr_t)xn2_out) & 15)
    return 2;
  ARPeers p{};
  for (int r = 0; r < world; ++r) {
    p.stage[0][r] = (bf16_t*)stage0[r];
    p.stage[1][r] = (bf16_t*)stage1[r];
    p.sig[r] = (ARSignal*)sig[r];
  }
  const DualLn a{nullptr, nullptr, nullptr, nullptr, (const bf16_t*)bias, ypart, cnt, (const bf16_t*)h,
                 (bf16_t*)h_out, (const bf16_t*)gamma, (const bf16_t*)beta, eps, (bf16_t*)xn_out,
                 (const bf16_t*)gamma2, (const bf16_t*)beta2, (bf16_t*)xn2_out, N, 0, 0};
  ARCtl* c = (ARCtl*)ctl;
  const long long n8 = N / 8;
  if (g_ar_ln_variant == 0) {
    const int nb = (int)((n8 + 255) / 256);
    switch (world) {
#define KCA_AR_LND_CASE(WW)                                                                                     \
  case WW:                                                                                                      \
    hipLaunchKernelGGL((ar_res_ln_dist_kernel<WW, DT>), dim3(nb), dim3(256), 0, stream, p, c, rank,             \
                       (const bf16_t*)in, n8, spin_limit, a);                                                   \
    break;
      KCA_AR_LND_CASE(1) KCA_AR_LND_CASE(2) KCA_AR_LND_CASE(3) KCA_AR_LND_CASE(4) KCA_AR_LND_CASE(5)
      KCA_AR_LND_CASE(6) KCA_AR_LND_CASE(7) KCA_AR_LND_CASE(8)
#undef KCA_AR_LND_CASE
      default:
        return 3;
    }
    return hipGetLastError() == hipSuccess ? 0 : 4;
  }
  switch (world) {
#define KCA_AR_LN_CASE(WW)                                                                                      \
  case WW:                                                                                                      \
    if (N <= 8192)                                                                                              \
      hipLaunchKernelGGL((ar_res_ln_kernel<WW, 4, DT>), dim3(blocks), dim3(256), 0, stream, p, c, rank,             \
                         (const bf16_t*)in, n8, spin_limit, a);                                                 \
    else                                                                                                        \
      hipLaunchKernelGGL((ar_res_ln_kernel<WW, 8, DT>), dim3(blocks), dim3(256), 0, stream, p, c, rank,             \
                         (const bf16_t*)in, n8, spin_limit, a);                                                 \
    break;
    KCA_AR_LN_CASE(1) KCA_AR_LN_CASE(2) KCA_AR_LN_CASE(3) KCA_AR_LN_CASE(4) KCA_AR_LN_CASE(5) KCA_AR_LN_CASE(6)
    KCA_AR_LN_CASE(7) KCA_AR_LN_CASE(8)
#undef KCA_AR_LN_CASE
    default:
      return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

KCA_API int kca_ar_res_ln(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank, int world,
                          const void* in, int N, int blocks, long long spin_limit, const void* bias, const void* h,
                          void* h_out, const void* gamma, const void* beta, float eps, void* xn_out,
                          const void* gamma2, const void* beta2, void* xn2_out, float* ypart, unsigned int* cnt,
                          hipStream_t stream) {
  return ar_res_ln<0>(stage0, stage1, sig, ctl, rank, world, in, N, blocks, spin_limit, bias, h, h_out, gamma, beta,
                      eps, xn_out, gamma2, beta2, xn2_out, ypart, cnt, stream);
}

// fp16 twin (same arguments)
KCA_API int kca_ar_res_ln_f16(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank,
                              int world, const void* in, int N, int blocks, long long spin_limit, const void* bias,
                              const void* h, void* h_out, const void* gamma, const void* beta, float eps,
                              void* xn_out, const void* gamma2, const void* beta2, void* xn2_out, float* ypart,
                              unsigned int* cnt, hipStream_t stream) {
  return ar_res_ln<1>(stage0, stage1, sig, ctl, rank, world, in, N, blocks, spin_limit, bias, h, h_out, gamma, beta,
                      eps, xn_out, gamma2, beta2, xn2_out, ypart, cnt, stream);
}

// Row-parallel projection close for batch 2..64 decode: all-reduce `in` (bf16 [M, N], this rank's
// partial), h_out = bf16(h + sum + bias) (h_out may alias h), and the row statistics of h_out for the
// next LayerNorm (stats [M][2] = (mean, rstd) with eps) through part ([M][N/64][2] fp32) and cnt
// (32 * 65 zero-initialised counters, re-armed by every call). N % 64 == 0, N <= 16384, M <= 64.
template <int DT>
static int ar_res_stats(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank,
                        int world, const void* in, int M, int N, int blocks, long long spin_limit,
                        const void* bias, const void* h, void* h_out, float eps, float* part, float* stats,
                        unsigned int* cnt, hipStream_t stream) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world || N % 64 || N <= 0 || N > 16384 || M < 1 ||
      M > 64 || blocks < 1 || blocks > AR_MAX_BLOCKS || !part || (stats && !cnt) || !h || !h_out)
    return 1;
  if (((uintptr_t)in | (uintptr_t)h | (uintptr_t)h_out | (uintptr_t)bias | (uintptr_t)part | (uintptr_t)stats) & 15)
    return 2;
  ARPeers p{};
  for (int r = 0; r < world; ++r) {
    p.stage[0][r] = (bf16_t*)stage0[r];
    p.stage[1][r] = (bf16_t*)stage1[r];
    p.sig[r] = (ARSignal*)sig[r];
  }
  const RowStats rs{part, stats, cnt, M, N, eps, 64};
  ARCtl* c = (ARCtl*)ctl;
  const long long n8 = (long long)M * N / 8;
  switch (world) {
#define KCA_AR_ST_CASE(WW)                                                                                      \
  case WW:                                                                                                      \
    hipLaunchKernelGGL((ar_res_stats_kernel<WW, DT>), dim3(blocks), dim3(256), 0, stream, p, c, rank,               \
                       (const bf16_t*)in, n8, spin_limit, (const bf16_t*)bias, (const bf16_t*)h, (bf16_t*)h_out, \
                       rs);                                                                                     \
    break;
    KCA_AR_ST_CASE(1) KCA_AR_ST_CASE(2) KCA_AR_ST_CASE(3) KCA_AR_ST_CASE(4) KCA_AR_ST_CASE(5) KCA_AR_ST_CASE(6)
    KCA_AR_ST_CASE(7) KCA_AR_ST_CASE(8)
#undef KCA_AR_ST_CASE
    default:
      return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

KCA_API int kca_ar_res_stats(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank,
                             int world, const void* in, int M, int N, int blocks, long long spin_limit,
                             const void* bias, const void* h, void* h_out, float eps, float* part, float* stats,
                             unsigned int* cnt, hipStream_t stream) {
  return ar_res_stats<0>(stage0, stage1, sig, ctl, rank, world, in, M, N, blocks, spin_limit, bias, h, h_out, eps,
                         part, stats, cnt, stream);
}

// fp16 twin: the fp16 serving layer's row-parallel close (same arguments, fp16 tensors)
KCA_API int kca_ar_res_stats_f16(void* const* stage0, void* const* stage1, void* const* sig, void* ctl, int rank,
                                 int world, const void* in, int M, int N, int blocks, long long spin_limit,
                                 const void* bias, const void* h, void* h_out, float eps, float* part,
                                 float* stats, unsigned int* cnt, hipStream_t stream) {
  return ar_res_stats<1>(stage0, stage1, sig, ctl, rank, world, in, M, N, blocks, spin_limit, bias, h, h_out, eps,
                         part, stats, cnt, stream);
}
