// Host AdamW for ZeRO-Offload configurations (N2 in SURVEY §2.2).
//
// The reference builds DeepSpeed's CPU-Adam op with a Fortran compiler shim
// that forces AVX256/skylake codegen (finetuner-workflow/finetuner/
// compiler_wrapper.f95:24-27, Dockerfile:26-35) and activates it through
// `offload_optimizer: cpu` (ds_config.json:35-37). Here one source carries an
// AVX-512 and an AVX2 body selected at run time with __builtin_cpu_supports
// (EPYC hosts of MI355X nodes have AVX-512), parallelised with OpenMP over
// the flat fp32 buffers, with an optional bf16 copy-back of the updated
// parameters into a pinned staging buffer for the H2D upload.
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#define KCA_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

struct Hyper {
  float lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, gscale;
};

inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

inline void scalar_range(float* p, const float* g, float* m, float* v, uint16_t* pb, const uint8_t* mask,
                         int64_t lo, int64_t hi, const Hyper& h) {
  for (int64_t i = lo; i < hi; ++i) {
    const float gr = g[i] * h.gscale;
    m[i] = h.b1 * m[i] + (1.f - h.b1) * gr;
    v[i] = h.b2 * v[i] + (1.f - h.b2) * gr * gr;
    const float den = std::sqrt(v[i]) * h.inv_sqrt_bc2 + h.eps;
    if (h.wd != 0.f && (!mask || mask[i >> 6])) p[i] *= (1.f - h.lr * h.wd);
    p[i] -= h.step_size * m[i] / den;
    if (pb) pb[i] = f2bf(p[i]);
  }
}

__attribute__((target("avx512f,avx512bw")))
void avx512_range(float* p, const float* g, float* m, float* v, uint16_t* pb, const uint8_t* mask,
                  int64_t lo, int64_t hi, const Hyper& h) {
  const __m512 b1 = _mm512_set1_ps(h.b1), nb1 = _mm512_set1_ps(1.f - h.b1);
  const __m512 b2 = _mm512_set1_ps(h.b2), nb2 = _mm512_set1_ps(1.f - h.b2);
  const __m512 eps = _mm512_set1_ps(h.eps), ss = _mm512_set1_ps(h.step_size);
  const __m512 ib = _mm512_set1_ps(h.inv_sqrt_bc2), gs = _mm512_set1_ps(h.gscale);
  const __m512 dec = _mm512_set1_ps(1.f - h.lr * h.wd), one = _mm512_set1_ps(1.f);
  int64_t i = lo;
  for (; i + 16 <= hi; i += 16) {
    __m512 gr = _mm512_mul_ps(_mm512_loadu_ps(g + i), gs);
    __m512 mm = _mm512_fmadd_ps(b1, _mm512_loadu_ps(m + i), _mm512_mul_ps(nb1, gr));
    __m512 vv = _mm512_fmadd_ps(b2, _mm512_loadu_ps(v + i), _mm512_mul_ps(nb2, _mm512_mul_ps(gr, gr)));
    __m512 den = _mm512_fmadd_ps(_mm512_sqrt_ps(vv), ib, eps);
    __m512 pp = _mm512_loadu_ps(p + i);
    const bool d = h.wd != 0.f && (!mask || mask[i >> 6]);
    pp = _mm512_mul_ps(pp, d ? dec : one);
    pp = _mm512_fnmadd_ps(ss, _mm512_div_ps(mm, den), pp);
    _mm512_storeu_ps(m + i, mm);
    _mm512_storeu_ps(v + i, vv);
    _mm512_storeu_ps(p + i, pp);
    if (pb) {
      // round-to-nearest-even bf16 of 16 lanes
      __m512i u = _mm512_castps_si512(pp);
      __m512i lsb = _mm512_and_si512(_mm512_srli_epi32(u, 16), _mm512_set1_epi32(1));
      __m512i r = _mm512_add_epi32(u, _mm512_add_epi32(lsb, _mm512_set1_epi32(0x7fff)));
      __m256i hi16 = _mm512_cvtepi32_epi16(_mm512_srli_epi32(r, 16));
      _mm256_storeu_si256((__m256i*)(pb + i), hi16);
    }
  }
  scalar_range(p, g, m, v, pb, mask, i, hi, h);
}

__attribute__((target("avx2,fma")))
void avx2_range(float* p, const float* g, float* m, float* v, uint16_t* pb, const uint8_t* mask,
                int64_t lo, int64_t hi, const Hyper& h) {
  const __m256 b1 = _mm256_set1_ps(h.b1), nb1 = _mm256_set1_ps(1.f - h.b1);
  const __m256 b2 = _mm256_set1_ps(h.b2), nb2 = _mm256_set1_ps(1.f - h.b2);
  const __m256 eps = _mm256_set1_ps(h.eps), ss = _mm256_set1_ps(h.step_size);
  const __m256 ib = _mm256_set1_ps(h.inv_sqrt_bc2), gs = _mm256_set1_ps(h.gscale);
  const __m256 dec = _mm256_set1_ps(1.f - h.lr * h.wd), one = _mm256_set1_ps(1.f);
  int64_t i = lo;
  for (; i + 8 <= hi; i += 8) {
    __m256 gr = _mm256_mul_ps(_mm256_loadu_ps(g + i), gs);
    __m256 mm = _mm256_fmadd_ps(b1, _mm256_loadu_ps(m + i), _mm256_mul_ps(nb1, gr));
    __m256 vv = _mm256_fmadd_ps(b2, _mm256_loadu_ps(v + i), _mm256_mul_ps(nb2, _mm256_mul_ps(gr, gr)));
    __m256 den = _mm256_fmadd_ps(_mm256_sqrt_ps(vv), ib, eps);
    __m256 pp = _mm256_loadu_ps(p + i);
    const bool d = h.wd != 0.f && (!mask || mask[i >> 6]);
    pp = _mm256_mul_ps(pp, d ? dec : one);
    pp = _mm256_fnmadd_ps(ss, _mm256_div_ps(mm, den), pp);
    _mm256_storeu_ps(m + i, mm);
    _mm256_storeu_ps(v + i, vv);
    _mm256_storeu_ps(p + i, pp);
    if (pb)
      for (int j = 0; j < 8; ++j) pb[i + j] = f2bf(p[i + j]);
  }
  scalar_range(p, g, m, v, pb, mask, i, hi, h);
}

}  // namespace

KCA_HOST_API int kca_host_simd_level() {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) return 512;
  if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return 256;
  return 0;
}

// p/g/m/v: fp32 [n]; pb: optional bf16 out [n]; mask: optional uint8 [n/64]
// (1 = weight decay on that 64-element block); force_level: 0 auto, else 512/256/1.
KCA_HOST_API int kca_host_adamw(float* p, const float* g, float* m, float* v, uint16_t* pb,
                                const uint8_t* mask, int64_t n, float lr, float b1, float b2,
                                float eps, float wd, float bc1, float bc2, float gscale,
                                int force_level) {
  Hyper h{lr, b1, b2, eps, wd, lr / bc1, 1.f / std::sqrt(bc2), gscale};
  const int lvl = force_level ? force_level : kca_host_simd_level();
  const int64_t block = 1 << 16;  // multiple of 64 so masks align per block
  const int64_t nb = (n + block - 1) / block;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t lo = b * block, hi = std::min(n, lo + block);
    if (lvl >= 512)
      avx512_range(p, g, m, v, pb, mask, lo, hi, h);
    else if (lvl >= 256)
      avx2_range(p, g, m, v, pb, mask, lo, hi, h);
    else
      scalar_range(p, g, m, v, pb, mask, lo, hi, h);
  }
  return 0;
}
