// hipBLASLt GEMMs with fused epilogues: D = A . W^T + bias + beta * C (row-major bf16, f32 accumulate).
//
// PyTorch's F.linear / addmm carry either a bias vector OR a full C matrix into hipBLASLt, never
// both, so a residual block `x + linear(h)` costs a separate bf16 add pass over the activations
// (the SD UNet's transformer residuals: aten::add on [16, 4096, 320] ... [16, 1280, 16, 16] in
// profiles/sd_unet_add_attribution_r2.txt). hipBLASLt's epilogue takes both: bias broadcast along
// the output rows and C read by the same kernel that writes D.
//
// Row-major D[M, N] is column-major D^T[N, M]; F.linear's A[M, K] . W[N, K]^T becomes
// D^T = op_T(W as K x N) . (A as K x M) -- the "TN" form hipBLASLt tiles best on MI355X -- and the
// bias (length N) runs along D^T's rows, which is what HIPBLASLT_EPILOGUE_BIAS broadcasts.
//
// Algorithm choice: per shape, the first call outside a HIP-graph capture times up to kTune of the
// heuristic's candidates on the live operands (3 launches each, hipEvents) and keeps the fastest;
// a call during capture with no tuned plan takes the heuristic's first choice. Plans are cached
// for the process (one handle per device).
#include "common.h"

#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace {

constexpr int kTune = 8;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool tuned = false;
};

using Key = std::tuple<int, int, int, int, long long, long long, long long, long long, int, int, int>;

std::mutex g_mu;
std::map<Key, Plan> g_plans;
std::map<int, hipblasLtHandle_t> g_handles;

hipblasLtHandle_t handle_for(int dev) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  g_handles[dev] = h;
  return h;
}

bool ok(hipblasStatus_t s) { return s == HIPBLAS_STATUS_SUCCESS; }

bool build(Plan& p, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldd, bool bias,
           bool has_c, bool f32out = false, uint32_t epi_over = 0, long long ldaux = 0, int opts = 0) {
  if (!ok(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F))) return false;
  const int32_t opT = HIPBLAS_OP_T, opN = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opT, sizeof(opT));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opN, sizeof(opN));
  const uint32_t epi = epi_over ? epi_over : bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  if (bias) {
    // DGELU_BGRAD writes the bias gradient: fp32 sums; the other epilogues read a bf16 bias
    const int32_t bt = (epi == HIPBLASLT_EPILOGUE_DGELU_BGRAD || (opts & 4)) ? HIP_R_32F : HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  if (ldaux) {  // the GELU epilogues' pre-activation matrix, laid out like D
    const int64_t ld = ldaux;
    const int32_t at = HIP_R_16BF;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
    if (!(opts & 8)) hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at));
  }
  // A operand of the column-major problem = W (K x N, ld ldw, transposed); B = A (K x M, ld lda)
  if (!ok(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, ldw))) return false;
  if (!ok(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, lda))) return false;
  const hipDataType cd = f32out ? HIP_R_32F : HIP_R_16BF;
  if (!ok(hipblasLtMatrixLayoutCreate(&p.lc, cd, N, M, has_c ? ldc : ldd))) return false;
  if (!ok(hipblasLtMatrixLayoutCreate(&p.ld, cd, N, M, ldd))) return false;
  return true;
}

}  // namespace

namespace {

int run(const void* A, long long lda, const void* W, long long ldw, const void* bias, const void* C, long long ldc,
        void* D, long long ldd, int M, int N, int K, float beta, uint32_t epi, void* aux, long long ldaux, void* ws,
        long long ws_bytes, hipStream_t stream, int opts = 0) {
  int dev = 0;
  hipGetDevice(&dev);
  const bool has_c = C != nullptr && beta != 0.f;
  const Key key{dev, M, N, K, lda, ldw, has_c ? ldc : 0, ldd, bias != nullptr, has_c, (int)epi | (opts << 20)};
  std::lock_guard<std::mutex> lock(g_mu);
  hipblasLtHandle_t h = handle_for(dev);
  if (!h) return 2;
  auto it = g_plans.find(key);
  if (it == g_plans.end()) {
    Plan p;
    if (!build(p, M, N, K, lda, ldw, ldc, ldd, bias != nullptr, has_c, false, epi, aux ? ldaux : 0, opts)) return 2;
    it = g_plans.emplace(key, p).first;
  }
  Plan& p = it->second;
  if (bias) hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
  if (aux) hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux));
  const float alpha = 1.f, b = has_c ? beta : 0.f;
  const void* cptr = has_c ? C : D;

  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  hipStreamIsCapturing(stream, &cap);
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (!p.tuned) {
    hipblasLtMatmulPreference_t pref = nullptr;
    hipblasLtMatmulPreferenceCreate(&pref);
    const uint64_t wsb = (uint64_t)ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[kTune];
    int n = 0;
    hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.ld, pref, kTune, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (n <= 0) return 4;
    int best = 0;
    while (best < n && (res[best].state != HIPBLAS_STATUS_SUCCESS || res[best].workspaceSize > (size_t)ws_bytes)) ++best;
    if (best == n) return 2;
    if (!capturing && n > 1 && (!has_c || C != D)) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float best_ms = 1e30f;
      for (int i = 0; i < n; ++i) {
        if (res[i].state != HIPBLAS_STATUS_SUCCESS || res[i].workspaceSize > (size_t)ws_bytes) continue;
        if (!ok(hipblasLtMatmul(h, p.desc, &alpha, W, p.la, A, p.lb, &b, cptr, p.lc, D, p.ld, &res[i].algo, ws,
                                res[i].workspaceSize, stream)))
          continue;
        hipEventRecord(e0, stream);
        for (int r = 0; r < 3; ++r)
          hipblasLtMatmul(h, p.desc, &alpha, W, p.la, A, p.lb, &b, cptr, p.lc, D, p.ld, &res[i].algo, ws,
                          res[i].workspaceSize, stream);
        hipEventRecord(e1, stream);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best_ms) best_ms = ms, best = i;
      }
      hipEventDestroy(e0);
      hipEventDestroy(e1);
    }
    p.algo = res[best].algo;
    p.ws = res[best].workspaceSize;
    p.tuned = !capturing;  // a pick made during a capture is timed at the next eager call
  }
  (void)hipGetLastError();
  if (!ok(hipblasLtMatmul(h, p.desc, &alpha, W, p.la, A, p.lb, &b, cptr, p.lc, D, p.ld, &p.algo, ws, p.ws, stream)))
    return 3;
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

// Returns 0 on success; 1 bad arguments; 2 no hipBLASLt algorithm; 3 launch failure.
// C may be null (beta ignored); C must not alias D when the shape still has to be tuned.
KCA_API int kca_gemm_lt(const void* A, long long lda, const void* W, long long ldw, const void* bias,
                        const void* C, long long ldc, void* D, long long ldd, int M, int N, int K, float beta,
                        void* ws, long long ws_bytes, hipStream_t stream) {
  if (!A || !W || !D || M <= 0 || N <= 0 || K <= 0 || lda < K || ldw < K || ldd < N || (C && ldc < N) ||
      ws_bytes < 0)
    return 1;
  return run(A, lda, W, ldw, bias, C, ldc, D, ldd, M, N, K, beta, 0, nullptr, 0, ws, ws_bytes, stream);
}

// D = act(A . W^T + bias) with hipBLASLt's GELU epilogues (tanh form), row-major bf16:
//   kind 1  GELU_AUX_BIAS  D = gelu(A W^T + bias), aux = A W^T + bias (the pre-activation, ld ldaux)
//   kind 2  DGELU_BGRAD    D = (A W^T) * gelu'(aux); bias <- fp32 column sums of D (the bias gradient)
// (kind | 4: the GELU_AUX_BIAS bias in fp32; kind | 8: aux type left at hipBLASLt's default)
// Measured against the separate GELU passes in bench/gelu_epilogue_bench.py.
KCA_API int kca_gemm_lt_gelu(const void* A, long long lda, const void* W, long long ldw, int kind, void* bias,
                             void* aux, long long ldaux, void* D, long long ldd, int M, int N, int K, void* ws,
                             long long ws_bytes, hipStream_t stream) {
  if (!A || !W || !D || !aux || M <= 0 || N <= 0 || K <= 0 || lda < K || ldw < K || ldd < N || ldaux < N ||
      ws_bytes < 0 || (kind & 3) == 0)
    return 1;
  const int opts = kind & ~3;
  kind &= 3;
  const uint32_t epi = kind == 1   ? (bias ? HIPBLASLT_EPILOGUE_GELU_AUX_BIAS : HIPBLASLT_EPILOGUE_GELU_AUX)
                       : kind == 2 ? (bias ? HIPBLASLT_EPILOGUE_DGELU_BGRAD : HIPBLASLT_EPILOGUE_DGELU)
                                   : (bias ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_GELU);
  return run(A, lda, W, ldw, bias, nullptr, 0, D, ldd, M, N, K, 0.f, epi, kind == 3 ? nullptr : aux, ldaux, ws,
             ws_bytes, stream, opts);
}

