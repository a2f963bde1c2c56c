// kaldi-lite/cu-kernels-lite.hip -- the generic CuMatrix/CuVector kernels
// the plugin needs from upstream cudamatrix (Set, Scale, AddMat, CopyFromMat,
// CopyRowsFromVec, AddRowSumMat, TraceMatMat/VecVec).  Reductions are
// two-pass with a fixed order, so results are bitwise reproducible.
#include <hip/hip_runtime.h>
#include <algorithm>

#include "../cnslmat/hip-util.h"
#include "cu-kernels-lite.h"

using kcnn::FastDiv;

namespace {

template <typename F>
__global__ __launch_bounds__(256) void kl_elem_kernel(int64_t r0, uint32_t n,
                                                      FastDiv divc, F f) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += gridDim.x * blockDim.x) {
    uint32_t i, j;
    divc.divmod(e, i, j);
    f(r0 + (int64_t)i, (int)j);
  }
}

template <typename F>
int kl_launch(int64_t rows, int cols, F f, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t max_rows = ((int64_t)1 << 30) / cols;
  FastDiv divc((uint32_t)cols);
  for (int64_t r0 = 0; r0 < rows; r0 += max_rows) {
    const int64_t nr = rows - r0 < max_rows ? rows - r0 : max_rows;
    const uint32_t n = (uint32_t)(nr * cols);
    hipLaunchKernelGGL(kl_elem_kernel<F>, dim3(kcnn::grid_for(n)), dim3(256), 0,
                       st, r0, n, divc, f);
  }
  return kcnn::launch_status();
}

struct SetF {
  float *d; int s; float v;
  __device__ void operator()(int64_t i, int j) const { d[i * s + j] = v; }
};
struct ScaleF {
  float *d; int s; float a;
  __device__ void operator()(int64_t i, int j) const { d[i * s + j] *= a; }
};
struct AddF {
  float *d; int s; float a;
  __device__ void operator()(int64_t i, int j) const { d[i * s + j] += a; }
};
// dst = alpha * op(A) + beta * dst   (Kaldi's _add_mat computes alpha*src + dst)
struct AddMatF {
  const float *a; int as; int trans; float *d; int ds; float alpha, beta;
  __device__ void operator()(int64_t i, int j) const {
    const float x = trans ? a[(int64_t)j * as + i] : a[i * as + j];
    float *y = d + i * ds + j;
    *y = beta == 0.0f ? alpha * x : alpha * x + beta * *y;
  }
};
struct CopyRowsFromVecF {
  const float *v; float *d; int ds;
  __device__ void operator()(int64_t i, int j) const { d[i * ds + j] = v[j]; }
};

// Column sums: pass 1 -- block (x: 256 columns, y: row slab) sums its slab.
__global__ __launch_bounds__(256) void kl_colsum_partial(
    const float *__restrict__ M, MatrixDim md, int rows_per_slab,
    float *__restrict__ part) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= md.cols) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slab;
  int64_t r1 = r0 + rows_per_slab;
  if (r1 > md.rows) r1 = md.rows;
  // 8 rows' loads in flight per step (a plain loop waits on each load);
  // rows past the slab add +0, the order of the sum is unchanged
  float s = 0.0f;
  for (int64_t r = r0; r < r1; r += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = r + u < r1 ? M[(r + u) * md.stride + j] : 0.0f;
#pragma unroll
    for (int u = 0; u < 8; u++) s += v[u];
  }
  part[(int64_t)blockIdx.y * md.cols + j] = s;
}
// pass 2 -- v = beta*v + alpha*sum_slabs: block = 64 columns x 4 slab
// groups (group g sums slabs g, g + 4, ... in increasing order, lanes along
// the columns: 256-B coalesced reads), then (g0 + g1) + (g2 + g3) -- a fixed
// order, so the bits are deterministic.
__global__ __launch_bounds__(256) void kl_colsum_final(
    const float *__restrict__ part, int slabs, int cols, float alpha,
    float beta, float *__restrict__ v) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  float s = 0.0f;
  if (j < cols) {
    int b = grp;
    for (; b + 28 < slabs; b += 32) {  // 8 partials' loads in flight
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; u++) t[u] = part[(int64_t)(b + 4 * u) * cols + j];
#pragma unroll
      for (int u = 0; u < 8; u++) s += t[u];
    }
    for (; b < slabs; b += 4) s += part[(int64_t)b * cols + j];
  }
  red[grp][lane] = s;
  __syncthreads();
  if (grp != 0 || j >= cols) return;
  s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  // beta 1: one rounding, the bits of BiasUpdate's fma(a_g, gb, b)
  // (cnsl-hip-kernels.hip), so a bias row updated here equals one updated
  // from a stored column sum
  v[j] = beta == 0.0f   ? alpha * s
         : beta == 1.0f ? __builtin_fmaf(alpha, s, v[j])
                        : beta * v[j] + alpha * s;
}

// C = sum_s P_s + beta C  (split-K partials [S][m][n], fixed order).
struct SumPartialsF {
  const float *p; int64_t pstride; int n; float *c; int cs; float beta; int S;
  __device__ void operator()(int64_t i, int j) const {
    const float *q = p + i * n + j;
    float acc = q[0];
    for (int s0 = 1; s0 < S; s0 += 4) {  // 4 partials' loads in flight
      float t[4];
#pragma unroll
      for (int u = 0; u < 4; u++) t[u] = s0 + u < S ? q[(int64_t)(s0 + u) * pstride] : 0.0f;
#pragma unroll
      for (int u = 0; u < 4; u++) acc += t[u];
    }
    float *y = c + i * cs + j;
    *y = beta == 0.0f ? acc : acc + beta * *y;
  }
};

// sum_{i,j} A[i][j] * op(B)[i][j] in double, one block, fixed order.
__global__ __launch_bounds__(256) void kl_dot_kernel(
    const float *__restrict__ A, MatrixDim ad, const float *__restrict__ B,
    MatrixDim bd, int transB, double *__restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  const int64_t n = (int64_t)ad.rows * ad.cols;
  for (int64_t e = threadIdx.x; e < n; e += 256) {
    const int64_t i = e / ad.cols, j = e - i * ad.cols;
    const float b = transB ? B[j * bd.stride + i] : B[i * bd.stride + j];
    s += (double)A[i * ad.stride + j] * (double)b;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

}  // namespace

extern "C" {

int kl_set(float *d, MatrixDim dim, float v, kcnn_stream_t st) {
  return kl_launch(dim.rows, dim.cols, SetF{d, dim.stride, v}, kcnn::as_stream(st));
}
int kl_scale(float *d, MatrixDim dim, float a, kcnn_stream_t st) {
  return kl_launch(dim.rows, dim.cols, ScaleF{d, dim.stride, a}, kcnn::as_stream(st));
}
int kl_add(float *d, MatrixDim dim, float a, kcnn_stream_t st) {
  return kl_launch(dim.rows, dim.cols, AddF{d, dim.stride, a}, kcnn::as_stream(st));
}
int kl_add_mat(float alpha, const float *A, MatrixDim ad, int transA,
               float beta, float *D, MatrixDim dd, kcnn_stream_t st) {
  (void)ad;
  return kl_launch(dd.rows, dd.cols,
                   AddMatF{A, ad.stride, transA, D, dd.stride, alpha, beta},
                   kcnn::as_stream(st));
}
int kl_copy_rows_from_vec(const float *v, float *D, MatrixDim dd,
                          kcnn_stream_t st) {
  return kl_launch(dd.rows, dd.cols, CopyRowsFromVecF{v, D, dd.stride},
                   kcnn::as_stream(st));
}
int kl_sum_partials(const float *parts, int S, int m, int n, float beta,
                    float *C, MatrixDim cd, kcnn_stream_t st) {
  return kl_launch(m, n,
                   SumPartialsF{parts, (int64_t)m * n, n, C, cd.stride, beta, S},
                   kcnn::as_stream(st));
}
// rows per slab of kl_colsum_partial: a multiple of 8, at least 16, and at
// most 256 slabs (c2's 4096-row FC derivative: 16 rows, 256 slabs, 1024
// blocks of the 1024 columns -- 64-row slabs gave 256 blocks, one wave per
// SIMD, 2.2 TB/s)
static int colsum_rows_per_slab(int rows) {
  const int r = (rows + 255) / 256;
  return std::max(16, (r + 7) / 8 * 8);
}
size_t kl_col_sum_workspace_bytes(MatrixDim md) {
  const int rps = colsum_rows_per_slab(md.rows);
  const int slabs = (md.rows + rps - 1) / rps;
  return (size_t)(slabs > 0 ? slabs : 1) * (size_t)md.cols * sizeof(float);
}
int kl_col_sum(const float *M, MatrixDim md, float alpha, float beta, float *v,
               void *ws, kcnn_stream_t st) {
  hipStream_t s = kcnn::as_stream(st);
  if (md.cols <= 0) return 0;
  const int rps = colsum_rows_per_slab(md.rows);
  int slabs = (md.rows + rps - 1) / rps;
  float *part = static_cast<float *>(ws);
  if (slabs == 0) {
    slabs = 1;
    if (hipMemsetAsync(part, 0, sizeof(float) * md.cols, s) != hipSuccess)
      return (int)hipErrorInvalidValue;
  } else {
    hipLaunchKernelGGL(kl_colsum_partial, dim3((md.cols + 255) / 256, slabs),
                       dim3(256), 0, s, M, md, rps, part);
  }
  hipLaunchKernelGGL(kl_colsum_final, dim3((md.cols + 63) / 64), dim3(256), 0,
                     s, part, slabs, md.cols, alpha, beta, v);
  return kcnn::launch_status();
}
int kl_dot(const float *A, MatrixDim ad, const float *B, MatrixDim bd,
           int transB, double *out_dev, kcnn_stream_t st) {
  hipLaunchKernelGGL(kl_dot_kernel, dim3(1), dim3(256), 0, kcnn::as_stream(st),
                     A, ad, B, bd, transB, out_dev);
  return kcnn::launch_status();
}

}  // extern "C"
