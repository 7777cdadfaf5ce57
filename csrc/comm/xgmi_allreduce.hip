// One-shot all-reduce over xGMI peer memory for small (latency-bound) messages
// (BLOOM TP=8 decode runs ~140 all-reduces of
// B x 14336 bf16 per token; RCCL's ring latency dominates at that size).
//
// Each rank owns, in device-uncached memory shared with its peers through
// hipIpc handles:
//   * two staging buffers (double-buffered by call parity), and
//   * a signal block: per workgroup a monotonically increasing call counter
//     and one arrival slot per peer.
// One kernel launch per all-reduce; workgroup b:
//   1. copies its slice of the input into its own staging[parity] buffer;
//   2. system-scope fence, then stores the new call count into slot[b][rank]
//      of EVERY peer's signal block (remote stores over xGMI);
//   3. spins (bounded) until all peers' counts arrived in its own slots;
//   4. reads its slice from all W peers' staging[parity] (uncached, straight
//      over the links -- 7 links in parallel on an 8-GPU mesh), sums in fp32
//      and writes the output.
// Double buffering removes the exit barrier: a peer can only overwrite
// staging[parity] two calls later, after it saw this rank arrive at the next
// call, i.e. after this rank finished reading. Counters live in device memory
// so the kernel is HIP-graph capturable (no host-side sequence numbers).
// A bounded spin sets an error word instead of hanging the GPU.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../kernels/common.h"

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_BLOCKS = 64;

struct ARSignal {
  uint32_t slot[AR_MAX_BLOCKS][AR_MAX_RANKS];  // written by peers
  uint32_t count[AR_MAX_BLOCKS];               // this rank's call counter per block
  uint32_t error;
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

template <int W>
__global__ __launch_bounds__(512) void ar_one_shot_kernel(ARPeers peers, int rank, const bf16_t* __restrict__ in,
                                                          bf16_t* __restrict__ out, long long n8,
                                                          long long spin_limit) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  ARSignal* me = peers.sig[rank];
  __shared__ uint32_t s_call;
  if (tid == 0) s_call = me->count[b] + 1;
  __syncthreads();
  const uint32_t call = s_call;
  const int par = call & 1;
  // slice of 16-byte chunks owned by this block
  const long long per = (n8 + nb - 1) / nb;
  const long long lo = b * per, hi = min(n8, lo + per);
  bf16_t* mine = peers.stage[par][rank];
  for (long long i = lo + tid; i < hi; i += blockDim.x)
    reinterpret_cast<uint4*>(mine)[i] = reinterpret_cast<const uint4*>(in)[i];
  __threadfence_system();
  __syncthreads();
  if (tid < W) st_sys(&peers.sig[tid]->slot[b][rank], call);
  if (tid < W) {
    long long spins = 0;
    while (ld_sys(&me->slot[b][tid]) < call) {
      if (++spins > spin_limit) {
        atomicOr(&me->error, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  for (long long i = lo + tid; i < hi; i += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < W; ++r) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(peers.stage[par][r]) + i);
      const uint32_t q[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[2 * j] += __uint_as_float(q[j] << 16);
        acc[2 * j + 1] += __uint_as_float(q[j] & 0xffff0000u);
      }
    }
    store8(out + i * 8, acc);
  }
  if (tid == 0) me->count[b] = call;
}

KCA_API int kca_ar_signal_bytes() { return (int)sizeof(ARSignal); }

// Uncached device allocation (coherent for peer access over xGMI).
KCA_API int kca_ar_alloc(long long bytes, void** ptr) {
  if (hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) return 1;
  return hipMemset(*ptr, 0, (size_t)bytes) == hipSuccess ? 0 : 2;
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
KCA_API int kca_ar_one_shot(void* const* stage0, void* const* stage1, void* const* sig, int rank, int world,
                            const void* in, void* out, long long n, int blocks, long long spin_limit,
                            hipStream_t stream) {
  if (world < 1 || world > AR_MAX_RANKS || n % 8 || blocks < 1 || blocks > AR_MAX_BLOCKS) return 1;
  if (((uintptr_t)in | (uintptr_t)out) & 15) return 2;
  ARPeers p{};
  for (int r = 0; r < world; ++r) {
    p.stage[0][r] = (bf16_t*)stage0[r];
    p.stage[1][r] = (bf16_t*)stage1[r];
    p.sig[r] = (ARSignal*)sig[r];
  }
  const long long n8 = n / 8;
  switch (world) {
#define KCA_AR_CASE(WW)                                                                                   \
  case WW:                                                                                                \
    hipLaunchKernelGGL(ar_one_shot_kernel<WW>, dim3(blocks), dim3(512), 0, stream, p, rank,                \
                       (const bf16_t*)in, (bf16_t*)out, n8, spin_limit);                                  \
    break;
    KCA_AR_CASE(1) KCA_AR_CASE(2) KCA_AR_CASE(3) KCA_AR_CASE(4) KCA_AR_CASE(5) KCA_AR_CASE(6)
    KCA_AR_CASE(7) KCA_AR_CASE(8)
#undef KCA_AR_CASE
    default:
      return 3;
  }
  return 0;
}

KCA_API int kca_ar_error(const void* sig, int* err) {
  uint32_t e = 0;
  if (hipMemcpy(&e, (const char*)sig + offsetof(ARSignal, error), 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  *err = (int)e;
  return 0;
}
