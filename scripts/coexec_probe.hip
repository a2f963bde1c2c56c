// scripts/coexec_probe.hip -- do VALU instructions of one wave execute while
// another wave's v_mfma_f32_32x32x2_f32 chain occupies the SIMD's matrix
// pipe?  (standalone probe, not part of the library)
//   hipcc --offload-arch=gfx950 -O3 scripts/coexec_probe.hip -o /tmp/coexec
// Block = 8 waves (2 per SIMD).  Mode 0: all waves MFMA; 1: all waves VALU;
// 2: waves 0-3 MFMA, 4-7 VALU (partners on one SIMD); 3: both kinds in
// every wave, interleaved.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(512) void probe(float *out, int iters) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  floatx16 a = {0};
  float x = 1e-3f * threadIdx.x, y = 2e-3f, v0 = x, v1 = y, v2 = x + y, v3 = x - y;
  const bool do_mfma = MODE == 0 || MODE == 3 || (MODE == 2 && wave < 4);
  const bool do_valu = MODE == 1 || MODE == 3 || (MODE == 2 && wave >= 4);
  for (int it = 0; it < iters; it++) {
    if (do_mfma) {
#pragma unroll
      for (int s = 0; s < 16; s++) a = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a, 0, 0, 0);
    }
    if (do_valu) {
#pragma unroll
      for (int s = 0; s < 64; s++) {  // 256 independent-ish FMAs ~ 16 MFMA slots
        v0 = __builtin_fmaf(v0, 1.0001f, 1e-7f);
        v1 = __builtin_fmaf(v1, 1.0001f, 1e-7f);
        v2 = __builtin_fmaf(v2, 1.0001f, 1e-7f);
        v3 = __builtin_fmaf(v3, 1.0001f, 1e-7f);
      }
    }
  }
  float s = v0 + v1 + v2 + v3;
  for (int r = 0; r < 16; r++) s += a[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(const char *name) {
  const int nb = 256, iters = 2000;
  float *out;
  hipMalloc(&out, sizeof(float) * nb * 512);
  hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(512), 0, 0, out, 10);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(512), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("%-40s %8.3f ms\n", name, ms);
  hipFree(out);
}

int main() {
  run<0>("all waves MFMA (16/iter)");
  run<1>("all waves VALU (256 fma/iter)");
  run<2>("waves 0-3 MFMA, 4-7 VALU");
  run<3>("every wave MFMA + VALU");
  run<0>("all waves MFMA (16/iter)");
  run<2>("waves 0-3 MFMA, 4-7 VALU");
  return 0;
}
