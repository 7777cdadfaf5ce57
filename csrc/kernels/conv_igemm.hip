// 3x3 / stride 1 / pad 1 convolution, NHWC bf16, as an implicit GEMM on the matrix cores (SURVEY K15:
// the SD-1.5 UNet's and VAE's convolutions, ~35 % of txt2img on the vendor kernels at 0.33-0.83
// PFLOP/s, profiles/conv_bench_sd_r2.jsonl).
//
//   y[p, co] = sum_{tap, c} x[n, h + r - 1, w + s - 1, c] * wt[co, r, s, c]      p = (n, h, w)
//
// GEMM view: M = N*H*W output pixels, N = Cout, K = 9*C ordered (tap, channel), so one K chunk of
// BK = 64 channels belongs to one tap: the A tile (BM pixels x 64 channels) is BM rows of 128 B read
// straight from the NHWC input at the tap's shifted pixel (rows that fall in the padding are zeros),
// the B tile (BN output channels x 64) is BN rows of 128 B of the KRSC weight (PyTorch channels-last
// [Cout, C, 3, 3]). No im2col buffer.
//
//   * workgroup: 256 threads, a BM = 128 x BN = 128 output tile, waves 2 x 2 over it (64 x 64 each,
//     2 x 2 v_mfma_f32_32x32x16_bf16 accumulators = 64 fp32 per lane);
//   * LDS: A and B tiles double-buffered (64 KB, 2 workgroups per CU), 16-B pieces XOR-swizzled by
//     row so the 32-row fragment reads are bank-conflict free (swz);
//   * global loads: PF chunks in flight per thread in registers (a ring), issued two LDS stages ahead
//     of their MFMAs;
//   * block order: the BN tiles of one pixel block are consecutive ids, remapped so they share an
//     XCD (its L2 serves the A tile to all of them; cdna_hip_programming.md XCD remap);
//   * epilogue: fp32 accumulators (+ bias) -> bf16 through LDS, stored as whole 16-B pieces.
//
// Shapes taken: C % 64 == 0, Cout % 64 == 0, N*H*W % 128 == 0 (every UNet / VAE conv but conv_in);
// kca_conv3x3_fwd returns 1 for others (the caller keeps the vendor path).
#include "common.h"

namespace {

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

constexpr int BK = 64;  // channels per K chunk (one tap)

struct ConvArgs {
  const uint16_t* x;     // [N, H, W, C]
  const uint16_t* w;     // [Co, 3, 3, C]
  const uint16_t* bias;  // [Co] (nullable)
  uint16_t* y;           // [N, H, W, Co]
  int N, H, W, C, Co;
};

// 16-B piece p of row r lives at piece p ^ ((r >> 1) & 7): a ds_read_b128 lane group (16 lanes, rows
// {0-3, 12-15, 20-27} or {4-11, 16-19, 28-31} of a 32-row fragment, MI355X_MICROARCH.md LDS table)
// then covers all 64 banks -- the r & 7 swizzle left 2-way conflicts (33-36 % of the LDS cycles,
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)
__device__ __forceinline__ int swz(int row, int piece) { return row * BK + ((piece ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ u32x4v ld16(const uint16_t* p) { return *reinterpret_cast<const u32x4v*>(p); }

// WM x WN waves of 64 x 64 output each: BM = 64 WM pixels x BN = 64 WN output channels per workgroup
template <int WM, int WN>
struct ConvTile {
  static constexpr int NT = WM * WN * 64, BM = 64 * WM, BN = 64 * WN;
  static constexpr int RS = NT / 8;          // rows per load round (8 pieces of 16 B per 64-channel row)
  static constexpr int LA = BM / RS, LB = BN / RS;
  static constexpr int STAGE = (BM + BN) * BK;  // elements
  static constexpr int LDS_BYTES = 2 * STAGE * 2;
};

template <int WM, int WN, int PF>
__global__ __launch_bounds__(WM * WN * 64, 1) void conv3x3_fwd_kernel(ConvArgs a) {
  using T = ConvTile<WM, WN>;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv / WN, wn = wv % WN;
  const int nbn = (a.Co + T::BN - 1) / T::BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = bid / nbn, bn = bid % nbn;
  const int p0 = bm * T::BM, n0 = bn * T::BN;
  const int HW = a.H * a.W;

  // load map: 16-B piece q of rows r0 + RS i (A: pixels, B: output channels)
  const int q = tid & 7, r0 = tid >> 3;
  int pn[T::LA], ph[T::LA], pw[T::LA];
#pragma unroll
  for (int i = 0; i < T::LA; ++i) {
    const int p = p0 + r0 + T::RS * i;
    pn[i] = p / HW;
    const int rem = p - pn[i] * HW;
    ph[i] = rem / a.W;
    pw[i] = rem - ph[i] * a.W;
  }
  const int KC = a.C / BK;
  const int nch = 9 * KC;

  u32x4v ra[PF][T::LA], rb[PF][T::LB];
  auto load = [&](int c, u32x4v (&xa)[T::LA], u32x4v (&xb)[T::LB]) {
    const int tap = c / KC, cc = (c - tap * KC) * BK + q * 8;
    const int dr = tap / 3 - 1, ds = tap % 3 - 1;
#pragma unroll
    for (int i = 0; i < T::LA; ++i) {
      const int hh = ph[i] + dr, ww = pw[i] + ds;
      const bool ok = (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      xa[i] = ok ? ld16(a.x + ((long long)(pn[i] * a.H + hh) * a.W + ww) * a.C + cc) : u32x4v{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < T::LB; ++i) {
      const int co = n0 + r0 + T::RS * i;
      xb[i] = co < a.Co ? ld16(a.w + ((long long)co * 9 + tap) * a.C + cc) : u32x4v{0u, 0u, 0u, 0u};
    }
  };
  auto store = [&](int buf, const u32x4v (&xa)[T::LA], const u32x4v (&xb)[T::LB]) {
    uint16_t* A = lds + buf * T::STAGE;
    uint16_t* B = A + T::BM * BK;
#pragma unroll
    for (int i = 0; i < T::LA; ++i) *reinterpret_cast<u32x4v*>(A + swz(r0 + T::RS * i, q)) = xa[i];
#pragma unroll
    for (int i = 0; i < T::LB; ++i) *reinterpret_cast<u32x4v*>(B + swz(r0 + T::RS * i, q)) = xb[i];
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // prologue: chunk 0 staged, chunks 1..PF in flight
  load(0, ra[0], rb[0]);
  store(0, ra[0], rb[0]);
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (1 + u < nch) load(1 + u, ra[u], rb[u]);
  __syncthreads();

  auto step = [&](int c, u32x4v (&xa)[T::LA], u32x4v (&xb)[T::LB]) {
    const int buf = c & 1;
    const uint16_t* A = lds + buf * T::STAGE;
    const uint16_t* B = A + T::BM * BK;
    // fragments of k-step ks + 1 requested before the MFMAs of ks (pinned)
    bf16x8 af[2][2], bf[2][2];
    auto rd = [&](int ks, int sl) {
      const int piece = 2 * ks + (lane >> 5);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[sl][i] = *reinterpret_cast<const bf16x8*>(A + swz(wm * 64 + i * 32 + (lane & 31), piece));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[sl][j] = *reinterpret_cast<const bf16x8*>(B + swz(wn * 64 + j * 32 + (lane & 31), piece));
    };
    rd(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      if (ks + 1 < BK / 16) {
        rd(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][i], bf[ks & 1][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
    }
    // chunk c + 1 (in xa / xb since PF chunks ago) -> the other stage, then chunk c + 1 + PF requested
    if (c + 1 < nch) {
      store(buf ^ 1, xa, xb);
      if (c + 1 + PF < nch) load(c + 1 + PF, xa, xb);
    }
    __syncthreads();
  };
  for (int c0 = 0; c0 < nch; c0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (c0 + u < nch) step(c0 + u, ra[u], rb[u]);
  }

  // epilogue: each wave's 64 x 64 tile -> bf16 in LDS ([64 pixels][64 channels], 8 KB per wave), then
  // 16-B pieces to y
  uint16_t* st = lds + wv * 64 * 64;
  const int col = lane & 31, hi = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int co = n0 + wn * 64 + j * 32 + col;
    const float b = (a.bias && co < a.Co) ? bf2f(a.bias[co]) : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int prow = i * 32 + 8 * (r >> 2) + 4 * hi + (r & 3);
        st[prow * 64 + j * 32 + col] = f2bf(acc[i][j][r] + b);
      }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int cbase = n0 + wn * 64;
  if (cbase < a.Co) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int row = (lane >> 3) + 8 * t, pc = lane & 7;
      const long long p = p0 + wm * 64 + row;
      *reinterpret_cast<u32x4v*>(a.y + p * a.Co + cbase + pc * 8) =
          *reinterpret_cast<const u32x4v*>(st + row * 64 + pc * 8);
    }
  }
}

int g_conv_pf = 2;

template <int WM, int WN>
int conv_launch(const ConvArgs& a, hipStream_t stream) {
  using T = ConvTile<WM, WN>;
  const long long npix = (long long)a.N * a.H * a.W;
  if (npix % T::BM) return 1;
  const long long nblk = npix / T::BM * ((a.Co + T::BN - 1) / T::BN);
  if (nblk > (1ll << 30)) return 1;
  if (g_conv_pf == 4)
    hipLaunchKernelGGL((conv3x3_fwd_kernel<WM, WN, 4>), dim3((unsigned)nblk), dim3(T::NT), T::LDS_BYTES, stream, a);
  else if (g_conv_pf == 3)
    hipLaunchKernelGGL((conv3x3_fwd_kernel<WM, WN, 3>), dim3((unsigned)nblk), dim3(T::NT), T::LDS_BYTES, stream, a);
  else
    hipLaunchKernelGGL((conv3x3_fwd_kernel<WM, WN, 2>), dim3((unsigned)nblk), dim3(T::NT), T::LDS_BYTES, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 4;
}

int g_conv_variant = 0;  // 0: by shape, 1: 128 x 128 tiles, 2: 256 x 128 tiles (A/B)

}  // namespace

KCA_API int kca_conv3x3_set_variant(int v) {
  g_conv_variant = v % 10;
  g_conv_pf = v / 10 ? v / 10 : 2;  // tens digit: chunks in flight (A/B)
  return 0;
}

// y = conv3x3(x, w) (+ bias), NHWC / KRSC bf16. Returns 1 (nothing launched) for unsupported shapes.
KCA_API int kca_conv3x3_fwd(const void* x, const void* w, const void* bias, void* y, int N, int H, int W, int C,
                            int Co, hipStream_t stream) {
  if (N < 1 || H < 1 || W < 1 || C % BK || Co % 64 || ((long long)N * H * W) % 128 || C < BK) return 1;
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) & 15) return 2;
  const ConvArgs a{(const uint16_t*)x, (const uint16_t*)w, (const uint16_t*)bias, (uint16_t*)y, N, H, W, C, Co};
  const long long npix = (long long)N * H * W;
  // 256 x 128 tiles (8 waves, one workgroup per CU) when they fill the chip at least twice over
  const bool big = g_conv_variant == 2 || (g_conv_variant == 0 && npix % 256 == 0 &&
                                           npix / 256 * ((Co + 127) / 128) >= 512);
  if (big && npix % 256 == 0) return conv_launch<4, 2>(a, stream);
  return conv_launch<2, 2>(a, stream);
}
