// Internal interface between gemm.hip's plain-GEMM autotuner and the hipBLASLt wrapper (blaslt.hip).
#pragma once
#include <hip/hip_runtime.h>

struct LtShape {
  int out_dtype, ta, tb, M, N, K;
  long long lda, ldb, ldc;
  int beta_nonzero;
  int bias;  // fp32 bias[N] epilogue (HIPBLASLT_EPILOGUE_BIAS), beta must be 0
};

// number of library algorithms (<= max_algos, heuristic order) prepared for the shape; 0 = none
int lt_prepare(const LtShape& s, int max_algos);
// run prepared algorithm idx: D = alpha op(A) op(B) + beta C  (C may equal D)
int lt_run(const LtShape& s, int idx, const void* A, const void* B, const void* C, void* D, float alpha, float beta,
           const float* bias, hipStream_t stream);
