// nnet2/nnet-kernels.hip -- RectifiedLinearComponent and SpliceComponent on
// gfx950.  Both are HBM-bound copies/element-wise maps: one pass over the
// data, lanes along columns (coalesced rows), 64-bit row offsets, and the
// ReLU statistics reduced in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include "nnet-kernels.h"
#include "../cnslmat/hip-util.h"

using kcnn::FastDiv;

namespace {

// ---- ReLU ------------------------------------------------------------------
// Block: 256 consecutive columns; rows grid-strided over blockIdx.y.
__global__ __launch_bounds__(256) void relu_prop_kernel(const float *__restrict__ in,
                                                        int64_t is, float *__restrict__ out,
                                                        int64_t os, int rows, int cols) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  for (int r = blockIdx.y; r < rows; r += gridDim.y) {
    float v = in[(int64_t)r * is + c];
    if (v < 0.0f) v = 0.0f;  // ApplyFloor(0): `if (x < floor) x = floor`
    out[(int64_t)r * os + c] = v;
  }
}

// The same four columns to a lane (16-B accesses; see kn_relu_prop)
__global__ __launch_bounds__(256) void relu_prop4_kernel(const float *__restrict__ in,
                                                         int64_t is, float *__restrict__ out,
                                                         int64_t os, int rows, int cols) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (c >= cols) return;
  for (int r = blockIdx.y; r < rows; r += gridDim.y) {
    float4 v = *reinterpret_cast<const float4 *>(in + (int64_t)r * is + c);
    if (v.x < 0.0f) v.x = 0.0f;
    if (v.y < 0.0f) v.y = 0.0f;
    if (v.z < 0.0f) v.z = 0.0f;
    if (v.w < 0.0f) v.w = 0.0f;
    *reinterpret_cast<float4 *>(out + (int64_t)r * os + c) = v;
  }
}

constexpr int kReluRowsPerPart = 64;

// Block: 256 consecutive columns x one chunk of kReluRowsPerPart rows.
__global__ __launch_bounds__(256) void relu_backprop_kernel(
    const float *__restrict__ ov, int64_t ovs, const float *__restrict__ od, int64_t ods,
    float *__restrict__ id, int64_t ids, int rows, int cols, float *__restrict__ part_v,
    float *__restrict__ part_h) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int r0 = blockIdx.y * kReluRowsPerPart;
  if (c >= cols) return;
  const int r1 = min(rows, r0 + kReluRowsPerPart);
  float sv = 0.0f, sh = 0.0f;
  for (int r = r0; r < r1; r++) {
    const float o = ov[(int64_t)r * ovs + c];
    const float h = o > 0.0f ? 1.0f : 0.0f;  // ApplyHeaviside
    id[(int64_t)r * ids + c] = h * od[(int64_t)r * ods + c];  // MulElements
    sv += o;
    sh += h;
  }
  if (part_v) {
    part_v[(int64_t)blockIdx.y * cols + c] = sv;
    part_h[(int64_t)blockIdx.y * cols + c] = sh;
  }
}

// The same map four columns to a lane (16-B accesses; cols, strides and
// pointers multiples of 4 floats): a block is 256 columns x one 64-row part,
// wave w taking rows w, w + 4, ...; the part's column sums are the four
// waves' sums added in wave order.
__global__ __launch_bounds__(256) void relu_backprop4_kernel(
    const float *__restrict__ ov, int64_t ovs, const float *__restrict__ od, int64_t ods,
    float *__restrict__ id, int64_t ids, int rows, int cols, float *__restrict__ part_v,
    float *__restrict__ part_h) {
  __shared__ float4 red[2][3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + lane) * 4;
  const int r0 = blockIdx.y * kReluRowsPerPart;
  const int r1 = min(rows, r0 + kReluRowsPerPart);
  float4 sv = make_float4(0.0f, 0.0f, 0.0f, 0.0f), sh = sv;
  if (c < cols) {
#pragma unroll 4
    for (int r = r0 + w; r < r1; r += 4) {
      const float4 o = *reinterpret_cast<const float4 *>(ov + (int64_t)r * ovs + c);
      const float4 d = *reinterpret_cast<const float4 *>(od + (int64_t)r * ods + c);
      const float4 h = make_float4(o.x > 0.0f ? 1.0f : 0.0f, o.y > 0.0f ? 1.0f : 0.0f,
                                   o.z > 0.0f ? 1.0f : 0.0f, o.w > 0.0f ? 1.0f : 0.0f);
      *reinterpret_cast<float4 *>(id + (int64_t)r * ids + c) =
          make_float4(h.x * d.x, h.y * d.y, h.z * d.z, h.w * d.w);
      sv.x += o.x; sv.y += o.y; sv.z += o.z; sv.w += o.w;
      sh.x += h.x; sh.y += h.y; sh.z += h.z; sh.w += h.w;
    }
  }
  if (part_v == nullptr) return;
  if (w > 0) {
    red[0][w - 1][lane] = sv;
    red[1][w - 1][lane] = sh;
  }
  __syncthreads();
  if (w > 0 || c >= cols) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float4 a = red[0][k][lane], b = red[1][k][lane];
    sv.x += a.x; sv.y += a.y; sv.z += a.z; sv.w += a.w;
    sh.x += b.x; sh.y += b.y; sh.z += b.z; sh.w += b.w;
  }
  *reinterpret_cast<float4 *>(part_v + (int64_t)blockIdx.y * cols + c) = sv;
  *reinterpret_cast<float4 *>(part_h + (int64_t)blockIdx.y * cols + c) = sh;
}

__global__ __launch_bounds__(256) void relu_stats_final_kernel(
    const float *__restrict__ part_v, const float *__restrict__ part_h, int nparts,
    int cols, double *__restrict__ value_sum, double *__restrict__ deriv_sum) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  float sv = 0.0f, sh = 0.0f;  // CuVector<BaseFloat> temp (:355-361)
#pragma unroll 16
  for (int p = 0; p < nparts; p++) {
    sv += part_v[(int64_t)p * cols + c];
    sh += part_h[(int64_t)p * cols + c];
  }
  value_sum[c] += (double)sv;
  deriv_sum[c] += (double)sh;
}

// ---- Splice ----------------------------------------------------------------
struct SpliceArgs {
  kn_splice_geom g;
  FastDiv div_cols, div_dim, div_ocs, div_ics;
};

__global__ __launch_bounds__(256) void splice_prop_kernel(const float *__restrict__ in,
                                                          int64_t is, float *__restrict__ out,
                                                          int64_t os, SpliceArgs a,
                                                          int64_t total) {
  const kn_splice_geom &g = a.g;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    uint32_t orow, col, chunk, oi;
    a.div_cols.divmod((uint32_t)e, orow, col);
    a.div_ocs.divmod(orow, chunk, oi);
    int irow, icol;
    if ((int)col < g.num_splice * g.dim) {
      uint32_t c, d;
      a.div_dim.divmod(col, c, d);
      irow = (int)chunk * g.in_cs + (g.table ? (int)g.in_index[c * g.out_cs + oi]
                                             : g.out_first + (int)oi + g.context[c] - g.in_first);
      icol = (int)d;
    } else {
      irow = (int)chunk * g.in_cs + (int)oi;
      icol = g.dim + ((int)col - g.num_splice * g.dim);
    }
    out[(int64_t)orow * os + col] = in[(int64_t)irow * is + icol];
  }
}

__global__ __launch_bounds__(256) void splice_backprop_kernel(
    const float *__restrict__ od, int64_t ods, float *__restrict__ id, int64_t ids,
    SpliceArgs a, int64_t total) {
  const kn_splice_geom &g = a.g;
  const int in_cols = g.dim + g.const_dim;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    const int irow = (int)(e / in_cols), icol = (int)(e - (int64_t)irow * in_cols);
    uint32_t chunk, ii;
    a.div_ics.divmod((uint32_t)irow, chunk, ii);
    float v = 0.0f;
    if (icol < g.dim) {
      for (int c = 0; c < g.num_splice; c++) {
        int oi = -1;
        if (g.table) {  // the output row of block c that read row ii (at most one)
          for (int o = 0; o < g.out_cs; o++)
            if (g.in_index[c * g.out_cs + o] == (int)ii) { oi = o; break; }
        } else {
          oi = g.in_first + (int)ii - g.context[c] - g.out_first;
        }
        if (oi >= 0 && oi < g.out_cs)
          v += od[((int64_t)chunk * g.out_cs + oi) * ods + c * g.dim + icol];
      }
    } else if ((int)ii < g.out_cs) {  // const part: copied from row (chunk, ii)
      v = od[((int64_t)chunk * g.out_cs + ii) * ods + g.num_splice * g.dim + (icol - g.dim)];
    }
    id[(int64_t)irow * ids + icol] = v;
  }
}

__global__ __launch_bounds__(256) void dvec_update_kernel(double *__restrict__ y,
                                                          const double *__restrict__ x,
                                                          double alpha, double beta, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  y[i] = beta * y[i] + (x ? alpha * x[i] : 0.0);
}

SpliceArgs splice_args(const kn_splice_geom &g, int out_cols) {
  SpliceArgs a;
  a.g = g;
  a.div_cols = FastDiv((uint32_t)(out_cols > 0 ? out_cols : 1));
  a.div_dim = FastDiv((uint32_t)(g.dim > 0 ? g.dim : 1));
  a.div_ocs = FastDiv((uint32_t)(g.out_cs > 0 ? g.out_cs : 1));
  a.div_ics = FastDiv((uint32_t)(g.in_cs > 0 ? g.in_cs : 1));
  return a;
}

}  // namespace

extern "C" {

int kn_relu_prop(const float *in, MatrixDim in_dim, float *out, MatrixDim out_dim,
                 kcnn_stream_t st) {
  if (in_dim.rows != out_dim.rows || in_dim.cols != out_dim.cols)
    return (int)hipErrorInvalidValue;
  if (in_dim.rows == 0 || in_dim.cols == 0) return 0;
  const bool vec4 = in_dim.cols % 4 == 0 && in_dim.stride % 4 == 0 && out_dim.stride % 4 == 0 &&
                    (uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0;
  const int cpb = vec4 ? 1024 : 256;  // columns per block
  const unsigned cb = (unsigned)((in_dim.cols + cpb - 1) / cpb);
  unsigned rb = (unsigned)in_dim.rows;
  const unsigned cap = 8192u / cb + 1u;  // ~8k blocks, rows grid-strided
  if (rb > cap) rb = cap;
  if (rb > 65535u) rb = 65535u;
  if (vec4)
    hipLaunchKernelGGL(relu_prop4_kernel, dim3(cb, rb), dim3(256), 0, kcnn::as_stream(st), in,
                       (int64_t)in_dim.stride, out, (int64_t)out_dim.stride, in_dim.rows,
                       in_dim.cols);
  else
    hipLaunchKernelGGL(relu_prop_kernel, dim3(cb, rb), dim3(256), 0, kcnn::as_stream(st), in,
                       (int64_t)in_dim.stride, out, (int64_t)out_dim.stride, in_dim.rows,
                       in_dim.cols);
  return kcnn::launch_status();
}

size_t kn_relu_stats_ws(MatrixDim dim) {
  const int nparts = (dim.rows + kReluRowsPerPart - 1) / kReluRowsPerPart;
  return (size_t)2 * nparts * (dim.cols > 0 ? dim.cols : 1) * sizeof(float);
}

int kn_relu_backprop(const float *out_value, MatrixDim ov_dim, const float *out_deriv,
                     MatrixDim od_dim, float *in_deriv, MatrixDim id_dim,
                     double *value_sum, double *deriv_sum, void *ws, kcnn_stream_t st) {
  if (ov_dim.rows != od_dim.rows || ov_dim.cols != od_dim.cols ||
      id_dim.rows != od_dim.rows || id_dim.cols != od_dim.cols)
    return (int)hipErrorInvalidValue;
  if (od_dim.rows == 0 || od_dim.cols == 0) return 0;
  const bool stats = value_sum != nullptr;
  if (stats && ws == nullptr) return (int)hipErrorInvalidValue;
  const int nparts = (od_dim.rows + kReluRowsPerPart - 1) / kReluRowsPerPart;
  float *pv = stats ? static_cast<float *>(ws) : nullptr;
  float *ph = stats ? pv + (size_t)nparts * od_dim.cols : nullptr;
  hipStream_t s = kcnn::as_stream(st);
  const bool vec4 = od_dim.cols % 4 == 0 && ov_dim.stride % 4 == 0 &&
                    od_dim.stride % 4 == 0 && id_dim.stride % 4 == 0 &&
                    (uintptr_t)out_value % 16 == 0 && (uintptr_t)out_deriv % 16 == 0 &&
                    (uintptr_t)in_deriv % 16 == 0 && (uintptr_t)pv % 16 == 0;
  if (vec4)
    hipLaunchKernelGGL(relu_backprop4_kernel, dim3((od_dim.cols + 255) / 256, nparts),
                       dim3(256), 0, s, out_value, (int64_t)ov_dim.stride, out_deriv,
                       (int64_t)od_dim.stride, in_deriv, (int64_t)id_dim.stride, od_dim.rows,
                       od_dim.cols, pv, ph);
  else
    hipLaunchKernelGGL(relu_backprop_kernel, dim3((od_dim.cols + 255) / 256, nparts),
                       dim3(256), 0, s, out_value, (int64_t)ov_dim.stride, out_deriv,
                       (int64_t)od_dim.stride, in_deriv, (int64_t)id_dim.stride, od_dim.rows,
                       od_dim.cols, pv, ph);
  int rc = kcnn::launch_status();
  if (rc || !stats) return rc;
  hipLaunchKernelGGL(relu_stats_final_kernel, dim3((od_dim.cols + 255) / 256), dim3(256),
                     0, s, pv, ph, nparts, od_dim.cols, value_sum, deriv_sum);
  return kcnn::launch_status();
}

}  // extern "C"

namespace {
// The geometry checks both splice directions share: shapes against the
// chunk layout, and every input row a table (or a contiguous range) names
// inside the input chunk, the table within its kernel-argument array.
bool splice_geom_ok(MatrixDim in_dim, MatrixDim out_dim, const kn_splice_geom &g) {
  if (g.num_splice <= 0 || g.num_splice > KN_SPLICE_MAX_CONTEXT ||
      in_dim.rows != g.num_chunks * g.in_cs || out_dim.rows != g.num_chunks * g.out_cs ||
      in_dim.cols != g.dim + g.const_dim ||
      out_dim.cols != g.num_splice * g.dim + g.const_dim)
    return false;
  if (g.table) {
    if ((int64_t)g.num_splice * g.out_cs > KN_SPLICE_MAX_TAB) return false;
    for (int e = 0; e < g.num_splice * g.out_cs; e++)
      if (g.in_index[e] < 0 || g.in_index[e] >= g.in_cs) return false;
  } else {
    for (int c = 0; c < g.num_splice; c++) {
      const int lo = g.out_first + g.context[c] - g.in_first;
      if (lo < 0 || lo + g.out_cs > g.in_cs) return false;
    }
  }
  return true;
}
}  // namespace

extern "C" {

int kn_splice_prop(const float *in, MatrixDim in_dim, float *out, MatrixDim out_dim,
                   kn_splice_geom g, kcnn_stream_t st) {
  if (!splice_geom_ok(in_dim, out_dim, g)) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)out_dim.rows * out_dim.cols;
  if (total == 0) return 0;
  if (total >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(splice_prop_kernel, dim3(kcnn::grid_for(total)), dim3(256), 0,
                     kcnn::as_stream(st), in, (int64_t)in_dim.stride, out,
                     (int64_t)out_dim.stride, splice_args(g, out_dim.cols), total);
  return kcnn::launch_status();
}

int kn_splice_backprop(const float *out_deriv, MatrixDim od_dim, float *in_deriv,
                       MatrixDim id_dim, kn_splice_geom g, kcnn_stream_t st) {
  if (!splice_geom_ok(id_dim, od_dim, g)) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)id_dim.rows * id_dim.cols;
  if (total == 0) return 0;
  if (total >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(splice_backprop_kernel, dim3(kcnn::grid_for(total)), dim3(256), 0,
                     kcnn::as_stream(st), out_deriv, (int64_t)od_dim.stride, in_deriv,
                     (int64_t)id_dim.stride, splice_args(g, od_dim.cols), total);
  return kcnn::launch_status();
}

int kn_dvec_update(double *y, const double *x, double alpha, double beta, int n,
                   kcnn_stream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(dvec_update_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     kcnn::as_stream(st), y, x, alpha, beta, n);
  return kcnn::launch_status();
}

}  // extern "C"
