// cnslmat/lds-dma.h -- publishing LDS written by LDS-DMA.
//
// An LDS-DMA load (buffer_load_dword* ... lds, __builtin_amdgcn_raw_ptr_
// buffer_load_lds) writes LDS, not VGPRs: the compiler tracks no dependency
// from it to any LDS read, least of all to another wave's.  So the barrier
// that hands DMA-landed data to the workgroup must first wait for this
// wave's outstanding vector-memory loads (s_waitcnt vmcnt(0)).  Every such
// barrier in the library is publish_dma(); a bare __syncthreads() after an
// LDS-DMA lets another wave read LDS before the data lands (r02: an
// intermittent gradient mismatch in the gradient-only backward, whose
// split-only waves reached the barrier early).
#ifndef KCNN_CNSLMAT_LDS_DMA_H_
#define KCNN_CNSLMAT_LDS_DMA_H_

#include <hip/hip_runtime.h>

namespace kcnn {
namespace x6 {

// vmcnt(0) (gfx9 encoding: expcnt and lgkmcnt fields at their no-wait maxima)
__device__ __forceinline__ void wait_dma() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// this wave's LDS-DMA has landed, then the barrier: the data is the workgroup's
__device__ __forceinline__ void publish_dma() {
  wait_dma();
  __syncthreads();
}

}  // namespace x6
}  // namespace kcnn

#endif  // KCNN_CNSLMAT_LDS_DMA_H_
