// scripts/mfma_probe.hip -- measures the issue rate of v_mfma_f32_32x32x2_f32
// chains on gfx950 in the shapes the conv kernels use (standalone probe, not
// part of the library).
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_probe.hip -o /tmp/mfma_probe
// Prints cycles per MFMA per SIMD for: one dependent chain from registers;
// two interleaved chains; a chain whose A operand is an LDS read issued just
// before (the compiler's default schedule); the same with reads 8 ahead.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(float *out, long long *cyc, int iters) {
  __shared__ float lds[64 * 64];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) lds[i] = 1e-3f * (i & 7);
  __syncthreads();
  floatx16 a0 = {0}, a1 = {0};
  float x = 1e-3f * lane, y = 2e-3f;
  const long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
    if (MODE == 0) {
#pragma unroll
      for (int s = 0; s < 16; s++) a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
    } else if (MODE == 1) {
#pragma unroll
      for (int s = 0; s < 8; s++) {
        a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, a1, 0, 0, 0);
      }
    } else if (MODE == 2) {
#pragma unroll
      for (int s = 0; s < 16; s++) {
        const float v = lds[(s * 64 + lane + it) & 4095];
        a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v, y, a0, 0, 0, 0);
      }
    } else if (MODE == 3) {
      float v[16];
#pragma unroll
      for (int s = 0; s < 16; s++) v[s] = lds[(s * 64 + lane + it) & 4095];
#pragma unroll
      for (int s = 0; s < 16; s++) a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[s], y, a0, 0, 0, 0);
    } else if (MODE == 4) {  // A and B from LDS, read just before
#pragma unroll
      for (int s = 0; s < 16; s++) {
        const float v = lds[(s * 64 + lane + it) & 4095];
        const float w = lds[(s * 64 + 2048 + lane + it) & 4095];
        a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v, w, a0, 0, 0, 0);
      }
    } else {  // A and B from LDS, 8 steps staged
#pragma unroll
      for (int s0 = 0; s0 < 16; s0 += 8) {
        float v[8], w[8];
#pragma unroll
        for (int s = 0; s < 8; s++) {
          v[s] = lds[((s0 + s) * 64 + lane + it) & 4095];
          w[s] = lds[((s0 + s) * 64 + 2048 + lane + it) & 4095];
        }
#pragma unroll
        for (int s = 0; s < 8; s++) a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[s], w[s], a0, 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const long long t1 = clock64();
  float s = 0;
  for (int r = 0; r < 16; r++) s += a0[r] + a1[r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int threads, int blocks_per_cu) {
  const int cus = 256, nb = cus * blocks_per_cu, iters = 2000;
  float *out;
  long long *cyc;
  hipMalloc(&out, sizeof(float) * nb * threads);
  hipMalloc(&cyc, sizeof(long long) * nb * threads / 64);
  hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(threads), 0, 0, out, cyc, 10);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(nb), dim3(threads), 0, 0, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const int nw = nb * threads / 64;
  long long *h = new long long[nw];
  hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < nw; i++) avg += h[i];
  avg /= nw;
  const double mfma_per_wave = 16.0 * iters * (MODE == 1 ? 1.0 : 1.0);
  const double waves_per_simd = threads / 64.0 * blocks_per_cu / 4.0;
  const double flops = 2.0 * 32 * 32 * 2 * mfma_per_wave * nw;
  printf("%-34s waves/SIMD %.0f: %6.1f clk/MFMA/wave, %6.1f clk/MFMA/SIMD, %6.1f TFLOP/s\n",
         name, waves_per_simd, avg / mfma_per_wave, avg / mfma_per_wave / waves_per_simd,
         flops / (ms * 1e-3) / 1e12);
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int wps : {1, 2}) {
    const int bpc = wps;  // 256 threads = 1 wave per SIMD per block
    run<0>("1 chain, registers", 256, bpc);
    run<1>("2 interleaved chains, registers", 256, bpc);
    run<2>("A from LDS, read just before", 256, bpc);
    run<3>("A from LDS, 16 reads ahead", 256, bpc);
    run<4>("A,B from LDS, read just before", 256, bpc);
    run<5>("A,B from LDS, 8 steps staged", 256, bpc);
  }
  return 0;
}
