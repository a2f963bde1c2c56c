// cnslmat/hip-util.h -- small device helpers shared by the gfx950 kernels.
#ifndef KCNN_CNSLMAT_HIP_UTIL_H_
#define KCNN_CNSLMAT_HIP_UTIL_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cnsl-hip-kernels.h"
#include "kaldi-lite/kcnn-knobs.h"

namespace kcnn {

// Division by a runtime-invariant divisor with one mul-hi + add + shift
// (Granlund-Montgomery).  Valid for numerators < 2^31, divisor >= 1.
struct FastDiv {
  uint32_t d, m, s;
  FastDiv() : d(1), m(1), s(0) {}
  explicit FastDiv(uint32_t div) : d(div) {
    s = 0;
    while (s < 31 && (1u << s) < div) ++s;
    const uint64_t one = 1;
    m = (uint32_t)(((one << 32) * ((one << s) - div)) / div + 1);
  }
  __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
#ifdef __HIP_DEVICE_COMPILE__
    const uint32_t t = __umulhi(n, m);
#else
    const uint32_t t = (uint32_t)(((uint64_t)n * m) >> 32);
#endif
    return (t + n) >> s;
  }
  __host__ __device__ __forceinline__ void divmod(uint32_t n, uint32_t &q,
                                                  uint32_t &r) const {
    q = div(n);
    r = n - q * d;
  }
};

inline hipStream_t as_stream(kcnn_stream_t s) {
  return reinterpret_cast<hipStream_t>(s);
}

inline int launch_status() { return (int)hipGetLastError(); }

// Blocks for a grid-stride elementwise kernel over `n` items: capped so a
// launch is ~8 waves per SIMD on 256 CUs and the rest is grid-strided.
inline unsigned grid_for(int64_t n, int block = 256) {
  int64_t b = (n + block - 1) / block;
  if (b < 1) b = 1;
  if (b > 256 * 32) b = 256 * 32;
  return (unsigned)b;
}

}  // namespace kcnn

#endif  // KCNN_CNSLMAT_HIP_UTIL_H_
