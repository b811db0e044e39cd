// In-kernel phase stamps (s_memtime cycles per block and wave) for the diagnostic builds that DESIGN.md §3c / §3d
// cite (scripts/exp/x6_trace.py, scripts/exp/bf_trace.py).  A kernel file defines its stamp macro with these helpers
// only under its trace flag (-DICA_X6_TRACE / -DICA_BF_TRACE); the product build compiles every stamp to nothing and
// exports no trace symbols.
#pragma once
#include <hip/hip_runtime.h>

// the stamp buffer of a translation unit ([block < 32768][wave][8 stamps]) and its host read / clear entry points
#define ICA_TRACE_DEFINE(buf, readfn, clearfn)                                                          \
  __device__ unsigned long long buf[32768 * 4 * 8];                                                      \
  extern "C" int readfn(void* dst, size_t bytes) {                                                       \
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(buf), bytes, 0, hipMemcpyDeviceToHost);              \
  }                                                                                                      \
  extern "C" int clearfn(const void* zeros, size_t bytes) {                                              \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(buf), zeros, bytes, 0, hipMemcpyHostToDevice);              \
  }

// stamp k of this (block, wave), written by lane 0 with a vector store
#define ICA_TRACE_STAMP(buf, k)                                                                          \
  do {                                                                                                   \
    if ((threadIdx.x & 63) == 0) {                                                                       \
      const unsigned b_ = blockIdx.x + gridDim.x * blockIdx.y;                                           \
      if (b_ < 32768) buf[((size_t)b_ * 4 + (threadIdx.x >> 6)) * 8 + (k)] = __builtin_readcyclecounter(); \
    }                                                                                                    \
  } while (0)
