// Plain (epilogue-free) bf16 GEMMs through hipBLASLt: the MAR backward's dX = dY . W and
// dW += dY^T . X products (model/autoregressive/functional.py BlockFn.backward; reference
// timm Block / nn.Linear autograd, models/mar.py Block stack).  Every GEMM with a fused epilogue
// (bias, GELU + pre-activation copy, dropout, residual, adaLN gate, GroupNorm-prologue convs)
// stays on the hand-written kernels of gemm.hip / conv.hip; this file only routes the products
// the library does at its peak (bf16 in, fp32 accumulate, bf16 or fp32 out, beta in {0, 1}, an
// optional fp32 bias: the forward's bias-only products -- qkv, and fc1 / fc2 whose GELU + dropout
// and dropout + residual then run as one elementwise pass, uva_act_drop_fwd).
//
// Row-major C[M][N] = op(A)[M][K] . op(B)[K][N] (gemm.hip operand convention: ta = 0 -> A stored
// [M][K], ta = 1 -> [K][M]; tb = 0 -> B stored [N][K], tb = 1 -> [K][N]) is the column-major
// product C^T (N x M) = op(B)^T-view (N x K) . op(A)^T-view (K x M), so the library's "A" is our B
// and its "B" is our A.  Descriptors + the heuristic's first 8 algorithms are cached per shape key;
// gemm.hip times them against its own kernel once per shape and keeps the fastest.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <stdlib.h>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>
#include "blaslt.h"
#include "common.h"

namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  std::vector<hipblasLtMatmulAlgo_t> algos;
  std::vector<size_t> ws;
};

using LtKey = std::tuple<int, int, int, int, int, int, long long, long long, long long, int, int>;

struct LtState {
  hipblasLtHandle_t handle = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 0;
  std::map<LtKey, LtPlan> plans;
  std::mutex mu;
};

LtState& lt_state(int dev) {
  static LtState st[16];
  return st[dev & 15];
}

constexpr size_t kLtWorkspace = 64ull << 20;

int g_lt_mode = -1;  // -1: from UVA_GEMM_LIB (default 0: the hand-written kernels only)

LtKey key_of(const LtShape& s) {
  return LtKey{s.out_dtype, s.ta, s.tb, s.M, s.N, s.K, s.lda, s.ldb, s.ldc, s.beta_nonzero, s.bias};
}

// plan (descriptors + up to max_algos heuristic algorithms) for the shape, created on first use
LtPlan* plan_for(LtState& st, const LtShape& s, int max_algos) {
  if (!st.handle) {
    if (hipblasLtCreate(&st.handle) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    if (hipMalloc(&st.ws, kLtWorkspace) != hipSuccess) return nullptr;
    st.ws_bytes = kLtWorkspace;
  }
  auto it = st.plans.find(key_of(s));
  if (it != st.plans.end()) return &it->second;
  LtPlan p;
  const hipDataType tc = s.out_dtype == UVA_DT_BF16 ? HIP_R_16BF : HIP_R_32F;
  hipblasOperation_t opA = s.tb == 0 ? HIPBLAS_OP_T : HIPBLAS_OP_N;  // library A = our B
  hipblasOperation_t opB = s.ta == 0 ? HIPBLAS_OP_N : HIPBLAS_OP_T;  // library B = our A
  bool good = hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opA, sizeof(opA)) ==
                     HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opB, sizeof(opB)) ==
                     HIPBLAS_STATUS_SUCCESS;
  if (s.bias) {  // bias[N] = per row of the column-major D (N x M); fp32 vector
    const hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_BIAS;
    const hipDataType bt = HIP_R_32F;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)) ==
                       HIPBLAS_STATUS_SUCCESS;
    good = good && hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)) ==
                       HIPBLAS_STATUS_SUCCESS;
  }
  // stored shapes (column-major rows x cols, ld)
  good = good && hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, s.tb == 0 ? s.K : s.N, s.tb == 0 ? s.N : s.K,
                                             s.ldb) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, s.ta == 0 ? s.K : s.M, s.ta == 0 ? s.M : s.K,
                                             s.lda) == HIPBLAS_STATUS_SUCCESS;
  good = good && hipblasLtMatrixLayoutCreate(&p.lc, tc, s.N, s.M, s.ldc) == HIPBLAS_STATUS_SUCCESS;
  if (good) {
    hipblasLtMatmulPreference_t pref;
    if (hipblasLtMatmulPreferenceCreate(&pref) == HIPBLAS_STATUS_SUCCESS) {
      uint64_t wsb = st.ws_bytes;
      hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
      std::vector<hipblasLtMatmulHeuristicResult_t> res(max_algos > 0 ? max_algos : 1);
      int n = 0;
      if (hipblasLtMatmulAlgoGetHeuristic(st.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, (int)res.size(),
                                          res.data(), &n) == HIPBLAS_STATUS_SUCCESS) {
        for (int i = 0; i < n; ++i)
          if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= st.ws_bytes) {
            p.algos.push_back(res[i].algo);
            p.ws.push_back(res[i].workspaceSize);
          }
      }
      hipblasLtMatmulPreferenceDestroy(pref);
    }
  }
  return &st.plans.emplace(key_of(s), p).first->second;
}

}  // namespace

int lt_prepare(const LtShape& s, int max_algos) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  LtState& st = lt_state(dev);
  std::lock_guard<std::mutex> lock(st.mu);
  LtPlan* p = plan_for(st, s, max_algos);
  return p ? (int)p->algos.size() : 0;
}

int lt_run(const LtShape& s, int idx, const void* A, const void* B, const void* C, void* D, float alpha, float beta,
           const float* bias, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (int)hipErrorInvalidDevice;
  LtState& st = lt_state(dev);
  std::lock_guard<std::mutex> lock(st.mu);
  LtPlan* p = plan_for(st, s, 8);
  if (!p || idx < 0 || idx >= (int)p->algos.size()) return -1;
  if (s.bias) {
    const void* bp = bias;
    if (hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)) !=
        HIPBLAS_STATUS_SUCCESS)
      return -1;
  }
  const hipblasStatus_t r = hipblasLtMatmul(st.handle, p->desc, &alpha, B, p->la, A, p->lb, &beta, C, p->lc, D,
                                            p->lc, &p->algos[idx], st.ws, p->ws[idx], stream);
  return r == HIPBLAS_STATUS_SUCCESS ? 0 : 1000 + (int)r;
}

extern "C" int uva_lt_mode(int mode) {
  const int prev = g_lt_mode;
  g_lt_mode = mode < 0 ? 0 : mode;
  return prev;
}

extern "C" int uva_lt_enabled() {
  if (g_lt_mode < 0) {
    const char* e = getenv("UVA_GEMM_LIB");
    g_lt_mode = e ? atoi(e) : 0;
  }
  return g_lt_mode;
}

// the library's first heuristic algorithm (no tuning): 0 on success, -1 when the library has no
// algorithm for the shape, an error code otherwise
extern "C" int uva_lt_gemm(int out_dtype, int ta, int tb, const void* A, const void* B, void* C, int M, int N,
                           int K, long long lda, long long ldb, long long ldc, float alpha, float beta,
                           hipStream_t stream) {
  const LtShape s{out_dtype, ta, tb, M, N, K, lda, ldb, ldc, beta != 0.f, 0};
  if (lt_prepare(s, 8) <= 0) return -1;
  return lt_run(s, 0, A, B, C, C, alpha, beta, nullptr, stream);
}
