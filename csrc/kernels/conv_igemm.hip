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
// Two forms (kca_conv3x3_fwd picks; profiles/conv_bench_r6.jsonl):
//   * conv3x3_dma_kernel (default where 256-pixel blocks tile the batch): 8 waves over a 256 x 128
//     tile, the stages filled by LDS-DMA three deep -- 606-799 TFLOP/s on the SD UNet shapes, ahead
//     of MIOpen on the 64x64 and 16x16 ones;
//   * conv3x3_fwd_kernel: register-staged tiles (128 x 128 or 256 x 128) through ds_write_b128, whose
//     transfer cost (~79 B/clk/CU) bounded it at 510-715 TFLOP/s.
// Common to both: waves of 64 x 64 outputs (2 x 2 v_mfma_f32_32x32x16_bf16 accumulators), LDS pieces
// swizzled conflict-free (swz), the BN tiles of one pixel block on one XCD (its L2 serves the A tile to
// all of them), fp32 accumulators (+ bias) -> bf16 through LDS, stored as 16-B pieces.
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

// ---- LDS-DMA form: the A / B stages arrive by buffer_load ... lds (no VGPR staging, none of the
// ds_write_b128 transfer cost that bounds the register-staged kernel), NBUF stages deep, one counted
// vmcnt + one barrier per chunk; 8 waves over a 256 x 128 tile, one workgroup per CU. An LDS-DMA
// wave-instruction writes 1 KiB lane-linearly (8 tile rows of 128 B), so the swizzle (swz) is applied
// to each lane's SOURCE channel; rows in the padding (and output channels past Cout) read past the
// buffer's end and land as zeros. hipcc drains every LDS-DMA before an LDS read it can see, so the
// fragment reads are inline asm with counted lgkmcnt waits (attention_tiled.hip's pattern).
__device__ __forceinline__ u32x4v cds_b128(unsigned addr) {
  u32x4v r;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
#endif
  return r;
}
template <int N>
__device__ __forceinline__ void clgkm_wait(u32x4v& a, u32x4v& b, u32x4v& c, u32x4v& d) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
#endif
}
template <int N>
__device__ __forceinline__ void cvm_wait() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#endif
}
__device__ __forceinline__ bf16x8 cbf8(u32x4v x) { return *reinterpret_cast<bf16x8*>(&x); }

constexpr unsigned kOOB = 0x7ffffff0u;

// physical 16-B piece of logical piece p in tile row r: conflict-free ds_read_b128 lane groups for
// 128-B rows (BK 64: p ^ ((r >> 1) & 7)) and 64-B rows (BK 32: p ^ ((r >> 2) & 3))
template <int BKX>
__device__ __forceinline__ int dswz(int r, int p) {
  if constexpr (BKX == 64) return p ^ ((r >> 1) & 7);
  else return p ^ ((r >> 2) & 3);
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}  // a source offset past every buffer this kernel is given

template <int NBUF, int BKX>
__global__ __launch_bounds__(512, 1) void conv3x3_dma_kernel(ConvArgs a) {
  constexpr int BM = 256, BN = 128, WN = 2;
  constexpr int RB = BKX * 2;                       // bytes per tile row
  constexpr int RPI = 1024 / RB;                    // tile rows per DMA wave-instruction
  constexpr int PPR = BKX / 8;                      // 16-B pieces per row
  constexpr int ABYTES = BM * RB, STAGE = (BM + BN) * RB;
  constexpr int AI = ABYTES / 1024 / 8, BI = BN * RB / 1024 / 8;  // DMA instructions per wave per stage
  constexpr int KS = BKX / 16;                      // MFMA k-steps per chunk
  constexpr int PER = AI + BI;
  extern __shared__ __attribute__((aligned(1024))) char csm[];
  typedef __attribute__((address_space(3))) char lds_char;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nbn = (a.Co + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bm = bid / nbn, bn = bid % nbn;
  const int p0 = bm * BM, n0 = bn * BN;
  const int HW = a.H * a.W;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.x, (short)0, (int)min((long long)a.N * HW * a.C * 2, (long long)kOOB - 1), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w, (short)0, (int)min((long long)a.Co * 9 * a.C * 2, (long long)kOOB - 1), 0x00020000);

  // this lane's DMA rows: A rows 8 (wave AI + i) + lane / 8, B rows 8 (wave BI + i) + lane / 8; the
  // 16-B piece it writes is lane % 8, so it reads logical piece (lane % 8) ^ ((row >> 1) & 7)
  int apix[AI], ah[AI], aw[AI], alp[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = RPI * (wave * AI + i) + lane / PPR;
    const int p = p0 + row;
    const int n = p / HW, rem = p - n * HW;
    ah[i] = rem / a.W;
    aw[i] = rem - ah[i] * a.W;
    apix[i] = p;
    alp[i] = dswz<BKX>(row, lane % PPR) * 16;
  }
  unsigned vb[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = RPI * (wave * BI + i) + lane / PPR;
    const int co = n0 + row;
    vb[i] = co < a.Co ? (unsigned)(co * 9 * a.C * 2 + dswz<BKX>(row, lane % PPR) * 16) : kOOB;
  }
  const int KC = a.C / BKX;
  const int nch = 9 * KC;
  lds_char* lsm = (lds_char*)csm;
  auto issue = [&](int cu, int buf) {
    const int c = min(cu, nch - 1);  // past the end: re-load the last chunk (keeps the vmcnt count fixed)
#ifdef KCA_CONV_TAP_MAJOR
    const int tap = c / KC, cc = (c - tap * KC) * BKX;
#else
    // channel-major: the 9 taps of one 64-channel slice back to back, so the shifted re-reads of the
    // block's pixels (+ halo: ~50 KB per workgroup) hit the XCD's L2 instead of the Infinity Cache
    const int tap = c % 9, cc = (c / 9) * BKX;
#endif
    const int dr = tap / 3 - 1, ds = tap % 3 - 1;
    const int sb = __builtin_amdgcn_readfirstlane((tap * a.C + cc) * 2);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int hh = ah[i] + dr, ww = aw[i] + ds;
      const bool ok = (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const unsigned vo = ok ? (unsigned)(((apix[i] + dr * a.W + ds) * a.C + cc) * 2 + alp[i]) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (void __attribute__((address_space(3)))*)(
          lsm + buf * STAGE + 1024 * (wave * AI + i)), 16, vo, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (void __attribute__((address_space(3)))*)(
          lsm + buf * STAGE + ABYTES + 1024 * (wave * BI + i)), 16, vb[i], sb, 0, 0);  // (kOOB + sb stays past the end)
#endif
  };

  // fragment addresses (bytes from the stage base): k-step ks, A rows i, B rows j
  const unsigned lbase = (unsigned)(size_t)lsm;
  unsigned fa[KS][2], fb[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int piece = 2 * ks + (lane >> 5);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wm * 64 + i * 32 + (lane & 31);
      fa[ks][i] = lbase + row * RB + (dswz<BKX>(row, piece) << 4);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wn * 64 + j * 32 + (lane & 31);
      fb[ks][j] = lbase + ABYTES + row * RB + (dswz<BKX>(row, piece) << 4);
    }
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(s, s);
  for (int c = 0; c < nch; ++c) {
    const int buf = c % NBUF;
    cvm_wait<(NBUF - 2) * PER>();  // this wave's DMAs of chunk c have landed
    __syncthreads();                // ... and every wave's; chunk c - 1's stage is free
    issue(c + NBUF - 1, (c + NBUF - 1) % NBUF);
    const unsigned so = buf * STAGE;
    u32x4v fr[KS][4];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      fr[ks][0] = cds_b128(fa[ks][0] + so);
      fr[ks][1] = cds_b128(fa[ks][1] + so);
      fr[ks][2] = cds_b128(fb[ks][0] + so);
      fr[ks][3] = cds_b128(fb[ks][1] + so);
    }
    static_for<0, KS>([&](auto kk) {
      constexpr int ks = decltype(kk)::value;
      clgkm_wait<4 * (KS - 1 - ks)>(fr[ks][0], fr[ks][1], fr[ks][2], fr[ks][3]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] =
              __builtin_amdgcn_mfma_f32_32x32x16_bf16(cbf8(fr[ks][i]), cbf8(fr[ks][2 + j]), acc[i][j], 0, 0, 0);
    });
  }
  cvm_wait<0>();  // the clamped re-loads past the end land before the stages are reused
  __syncthreads();

  uint16_t* st = reinterpret_cast<uint16_t*>(csm) + wave * 64 * 64;
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

int g_conv_variant = 0;  // 0: LDS-DMA where it tiles, else 128 x 128; 1 / 2: register-staged 128 x 128 /
                         // 256 x 128 tiles; 3: LDS-DMA (A/B)

}  // namespace

KCA_API int kca_conv3x3_set_variant(int v) {
  g_conv_variant = v % 10;
  g_conv_pf = (v / 10) % 10 ? (v / 10) % 10 : 2;  // tens digit: chunks in flight (A/B)
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
  // default: the LDS-DMA kernel whenever its 256-pixel blocks tile the batch
  if ((g_conv_variant == 3 || g_conv_variant == 0) && npix % 256 == 0 && (long long)N * H * W * C * 2 < 0x70000000ll &&
      (long long)Co * 9 * C * 2 < 0x70000000ll) {
    const long long nblk = npix / 256 * ((Co + 127) / 128);
    // (32-channel chunks six stages deep measured 8-20 % slower: the per-chunk barrier + wait is the
    // fixed cost, profiles/conv_bench_r6.jsonl)
    hipLaunchKernelGGL((conv3x3_dma_kernel<3, 64>), dim3((unsigned)nblk), dim3(512), 3 * (256 + 128) * 128, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : 4;
  }
  if (big && npix % 256 == 0) return conv_launch<4, 2>(a, stream);
  return conv_launch<2, 2>(a, stream);
}
