// cnslmat/cnsl-hip-kernels.hip -- gfx950 bandwidth kernels of the CNN hot
// path: the reshape helpers behind CuMatrixBase::{FlipMat, PaddingZero,
// TpBlock, TpInsideBlock, ModPermuteRow, AddMatRepVec} (conv2D.cc:213-463),
// 3-D max pooling forward/backward (conv2D.cc:465-684) and the momentum
// update (nnet-component-nnet0.cc:769-775, :1137-1142).
//
// The reference launches every op as one thread per output element on 16x16
// blocks with int32 offsets (cnsl-cu-kernels.cu:10-529).  Here an op is a
// grid-stride loop over a flattened index with one FastDiv per element, 256
// threads (4 wave64s) per block, 64-bit element offsets, and -- for pooling,
// the only one of these on the training step -- wave-contiguous output
// columns so every wave reads and writes whole 256-B row segments.
#include <hip/hip_runtime.h>
#include <cstdlib>

#include "hip-util.h"
#include "momentum-step.h"

using kcnn::FastDiv;

namespace {

// ---------------------------------------------------------------------------
// Elementwise over a [rows x cols] output.  Rows are processed in slabs so
// the flattened index stays below 2^31 (FastDiv domain).
template <typename F>
__global__ __launch_bounds__(256) void elem2d_kernel(int64_t r0, uint32_t n,
                                                     FastDiv divc, F f) {
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += gridDim.x * blockDim.x) {
    uint32_t i, j;
    divc.divmod(e, i, j);
    f(r0 + (int64_t)i, (int)j);
  }
}

template <typename F>
int launch_elem2d(int64_t rows, int cols, F f, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t max_rows = ((int64_t)1 << 31) / 2 / cols;  // keep e < 2^30
  FastDiv divc((uint32_t)cols);
  for (int64_t r0 = 0; r0 < rows; r0 += max_rows) {
    const int64_t nr = rows - r0 < max_rows ? rows - r0 : max_rows;
    const uint32_t n = (uint32_t)(nr * cols);
    hipLaunchKernelGGL(elem2d_kernel<F>, dim3(kcnn::grid_for(n)), dim3(256), 0,
                       st, r0, n, divc, f);
  }
  return kcnn::launch_status();
}

// ---- functors (one per reference kernel) -----------------------------------

// conv2D.cc:120-133 / cnsl-cu-kernels.cu:10-38 (im2col).
struct SpanRowToConvmat {
  const float *in; MatrixDim in_dim; float *span; MatrixDim span_dim;
  int in_height, in_width, kernel_height; int64_t row_offset;
  FastDiv div_ks, div_kh, div_rows, div_q;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t J, Jr, I, Ir, a, b, kx, ky;
    div_ks.divmod((uint32_t)j, J, Jr);
    div_rows.divmod((uint32_t)(i + row_offset), I, Ir);
    div_q.divmod(I, b, a);                    // Q = I % q + I / q * H
    div_kh.divmod(Jr, kx, ky);                // P = Jr % kh + Jr / kh * H
    const int64_t col = (int64_t)a + (int64_t)b * in_height + ky +
                        (int64_t)kx * in_height +
                        (int64_t)J * in_height * in_width;
    span[i * span_dim.stride + j] = in[(int64_t)Ir * in_dim.stride + col];
  }
};

// conv2D.cc:190-196 / cnsl-cu-kernels.cu:42-59 (col2im).
struct ConvmatToOut {
  const float *conv; MatrixDim conv_dim; float *out; MatrixDim out_dim;
  int64_t plane; FastDiv div_ns;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t I, Ir;
    div_ns.divmod((uint32_t)i, I, Ir);
    out[(int64_t)Ir * out_dim.stride + I + j * plane] =
        conv[i * conv_dim.stride + j];
  }
};

// conv2D.cc:232-239 / cnsl-cu-kernels.cu:61-75.
struct AddMatRepVec {
  const float *vec; float *out; MatrixDim out_dim; FastDiv div_rep;
  __device__ void operator()(int64_t i, int j) const {
    out[i * out_dim.stride + j] += vec[div_rep.div((uint32_t)j)];
  }
};

// conv2D.cc:270-281 / cnsl-cu-kernels.cu:78-97.
struct FlipMat {
  const float *orig; MatrixDim orig_dim; float *flip; MatrixDim flip_dim;
  int ksize; FastDiv div_ks;
  __device__ void operator()(int64_t i, int j) const {
    const int gi = (int)div_ks.div((uint32_t)i);
    const int p = (gi + 1) * ksize - 1 - (int)i;
    const int64_t m = p + (int64_t)j * ksize;
    flip[i * flip_dim.stride + j] = orig[m * orig_dim.stride + gi];
  }
};

// conv2D.cc:318-339 / cnsl-cu-kernels.cu:100-134.
struct PadZero {
  const float *orig; MatrixDim orig_dim; float *pad; MatrixDim pad_dim;
  int oh, ow, kh, kw; FastDiv div_psize, div_ph;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t chan, p, J, I;
    div_psize.divmod((uint32_t)j, chan, p);
    div_ph.divmod(p, J, I);
    float v = 0.0f;
    if ((int)I >= kh - 1 && (int)I < kh + oh - 1 && (int)J >= kw - 1 &&
        (int)J < kw + ow - 1) {
      const int m = (int)I - kh + 1, n = (int)J - kw + 1;
      v = orig[i * orig_dim.stride + (int64_t)n * oh + m +
               (int64_t)chan * oh * ow];
    }
    pad[i * pad_dim.stride + j] = v;
  }
};

// conv2D.cc:376-383 / cnsl-cu-kernels.cu:138-161.
struct TpBlock {
  const float *in; MatrixDim in_dim; float *out; MatrixDim out_dim;
  int bs; FastDiv div_bs;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t row, r;
    div_bs.divmod((uint32_t)j, row, r);
    out[i * out_dim.stride + j] =
        in[(int64_t)row * in_dim.stride + i * bs + r];
  }
};

// conv2D.cc:416-423 / cnsl-cu-kernels.cu:165-185.
struct TpInsideBlock {
  const float *in; MatrixDim in_dim; float *out; MatrixDim out_dim;
  int bs; FastDiv div_bs;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t row, r;
    div_bs.divmod((uint32_t)i, row, r);
    out[i * out_dim.stride + j] =
        in[(int64_t)row * in_dim.stride + (int64_t)j * bs + r];
  }
};

// conv2D.cc:453-460 / cnsl-cu-kernels.cu:189-210.
struct ModPermuteRow {
  const float *in; MatrixDim in_dim; float *out; MatrixDim out_dim;
  int bs; FastDiv div_c;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t pos, chan;
    div_c.divmod((uint32_t)i, pos, chan);
    out[((int64_t)chan * bs + pos) * out_dim.stride + j] =
        in[i * in_dim.stride + j];
  }
};

// cnsl-cu-kernels.cu:214-228.
struct CopyRowsAt {
  const float *src; MatrixDim src_dim; float *dst; MatrixDim dst_dim;
  int64_t off;
  __device__ void operator()(int64_t i, int j) const {
    dst[(i + off) * dst_dim.stride + j] = src[i * src_dim.stride + j];
  }
};

// conv2D.cc:706-725 / cnsl-cu-kernels.cu:505-528.
struct ModPermuteChannels {
  float *comp; MatrixDim comp_dim; float *cont; MatrixDim cont_dim;
  int comp_idx, num_component, plane, to_container; FastDiv div_plane;
  __device__ void operator()(int64_t i, int j) const {
    uint32_t chan, pos;
    div_plane.divmod((uint32_t)j, chan, pos);
    const int64_t o = i * cont_dim.stride +
                      ((int64_t)chan * num_component + comp_idx) * plane + pos;
    if (to_container) cont[o] = comp[i * comp_dim.stride + j];
    else comp[i * comp_dim.stride + j] = cont[o];
  }
};

// ---------------------------------------------------------------------------
// Max pooling.  Window of output column j (same enumeration order as the
// reference: channel, width, height; cnsl-cu-kernels.cu:253-263).
struct PoolGeom {
  int in_h, in_w, ph, pw, pc, mode;
  int64_t plane;           // in_h * in_w
  FastDiv div_outplane;    // oh' * ow'   (mode 0/1) | in_h*in_w (mode 2)
  FastDiv div_outh;        // oh'
  int out_2d, in_2d;       // mode 2
  FastDiv div_out2d;
};

__device__ __forceinline__ int64_t pool_start(const PoolGeom &g, int j) {
  uint32_t oc, pos;
  g.div_outplane.divmod((uint32_t)j, oc, pos);
  if (g.mode == 2) return (int64_t)pos;  // channel part added per element
  uint32_t wi, hi;
  g.div_outh.divmod(pos, wi, hi);
  const int64_t cbase =
      g.mode == 1 ? (int64_t)oc * g.plane : (int64_t)oc * g.pc * g.plane;
  return cbase + (int64_t)wi * g.pw * g.in_h + (int64_t)hi * g.ph;
}

struct MaxpoolProp {
  const float *src; MatrixDim src_dim; float *pool; MatrixDim pool_dim;
  PoolGeom g;
  __device__ void operator()(int64_t i, int j) const {
    const float *row = src + i * src_dim.stride;
    float val = -1e20f;
    if (g.mode == 2) {  // cnsl-cu-kernels.cu:434-446
      const int64_t pos = pool_start(g, j);
      uint32_t oc = g.div_outplane.div((uint32_t)j), x, y;
      g.div_out2d.divmod(oc, x, y);
      for (int cx = 0; cx < g.pc; cx++)
        for (int cy = 0; cy < g.pc; cy++) {
          const int64_t ic = (int64_t)(x + cx) * g.in_2d + (y + cy);
          const float v = row[ic * g.plane + pos];
          if (val < v) val = v;
        }
    } else {            // cnsl-cu-kernels.cu:253-263 / :340-350
      const int64_t start = pool_start(g, j);
      for (int c = 0; c < g.pc; c++)
        for (int w = 0; w < g.pw; w++)
          for (int h = 0; h < g.ph; h++) {
            const float v = row[start + h + (int64_t)w * g.in_h + c * g.plane];
            if (val < v) val = v;
          }
    }
    pool[i * pool_dim.stride + j] = val;
  }
};

// Non-overlap backprop, scatter form: each output element owns its window
// (disjoint windows), one writer per in_deriv element.
struct MaxpoolBackpropDisjoint {
  const float *in_val; MatrixDim in_dim; const float *out_val; MatrixDim ov_dim;
  const float *out_der; MatrixDim od_dim; float *dest; MatrixDim dest_dim;
  PoolGeom g; int write_all;
  __device__ void operator()(int64_t i, int j) const {
    const float o = out_val[i * ov_dim.stride + j];
    const float e = out_der[i * od_dim.stride + j];  // own stride
    const float *x = in_val + i * in_dim.stride;
    float *d = dest + i * dest_dim.stride;
    const int64_t start = pool_start(g, j);
    for (int c = 0; c < g.pc; c++)
      for (int w = 0; w < g.pw; w++)
        for (int h = 0; h < g.ph; h++) {
          const int64_t idx = start + h + (int64_t)w * g.in_h + c * g.plane;
          const bool hit = x[idx] == o;
          if (write_all) d[idx] = hit ? e : 0.0f;
          else if (hit) d[idx] = e;
        }
  }
};

// Overlapping modes, gather form: thread per in_deriv element; sums the
// derivatives of every output whose window contains it, in increasing output
// column order (the order of the CPU loop conv2D.cc:645-681), from 0.
struct MaxpoolBackpropGather {
  const float *in_val; MatrixDim in_dim; const float *out_val; MatrixDim ov_dim;
  const float *out_der; MatrixDim od_dim; float *dest; MatrixDim dest_dim;
  PoolGeom g; int out_channels; int write_all; FastDiv div_plane, div_in2d;
  __device__ void operator()(int64_t i, int col) const {
    uint32_t ic, pos;
    div_plane.divmod((uint32_t)col, ic, pos);
    const float x = in_val[i * in_dim.stride + col];
    const float *ov = out_val + i * ov_dim.stride;
    const float *od = out_der + i * od_dim.stride;
    float acc = 0.0f;
    bool any = false;
    if (g.mode == 1) {  // out channel oc covers input channels oc..oc+pc-1
      int lo = (int)ic - g.pc + 1;
      if (lo < 0) lo = 0;
      int hi = (int)ic < out_channels - 1 ? (int)ic : out_channels - 1;
      for (int oc = lo; oc <= hi; oc++) {
        const int64_t j = (int64_t)oc * g.plane + pos;
        if (x == ov[j]) { acc += od[j]; any = true; }
      }
    } else {            // overlap2D: (X,Y) in in_2d map, outputs (x,y) on out_2d
      uint32_t X, Y;
      div_in2d.divmod(ic, X, Y);
      for (int xo = (int)X - g.pc + 1; xo <= (int)X; xo++) {
        if (xo < 0 || xo >= g.out_2d) continue;
        for (int yo = (int)Y - g.pc + 1; yo <= (int)Y; yo++) {
          if (yo < 0 || yo >= g.out_2d) continue;
          const int64_t j = ((int64_t)xo * g.out_2d + yo) * g.plane + pos;
          if (x == ov[j]) { acc += od[j]; any = true; }
        }
      }
    }
    float *d = dest + i * dest_dim.stride + col;
    if (write_all) *d = acc;
    else if (any) *d += acc;
  }
};

struct MomentumUpdate {
  float *W; MatrixDim wd; float *prev; MatrixDim pd; const float *grad;
  MatrixDim gd; float momentum, a_wd, a_g;
  __device__ void operator()(int64_t i, int j) const {
    // momentum-step.h: the same code as the gradient GEMM's fused store
    float p = prev[i * pd.stride + j], w = W[i * wd.stride + j];
    kcnn::momentum_step(grad[i * gd.stride + j], p, w, momentum, a_wd, a_g);
    prev[i * pd.stride + j] = p;
    W[i * wd.stride + j] = w;
  }
};

struct BiasUpdate {
  float *b; const float *gb; float a_g;
  __device__ void operator()(int64_t, int j) const { b[j] = __builtin_fmaf(a_g, gb[j], b[j]); }
};

// Both in one launch: rows [0, rows) of W as MomentumUpdate, the extra row
// `rows` as BiasUpdate over its first b_dim columns (b_dim <= W's columns),
// one kernel instead of two for the step's few-KB bias.
struct MomentumBiasUpdate {
  MomentumUpdate w;
  BiasUpdate b;
  int rows, b_dim;
  __device__ void operator()(int64_t i, int j) const {
    if (i < rows) w(i, j);
    else if (j < b_dim) b(0, j);
  }
};

// ---------------------------------------------------------------------------
// Channel-group pooling (non-overlap, ph = pw = 1: the c2 1x1x4 intermap pool).
// The pc maps of one pool group are a contiguous run of a row (pc*plane
// floats) and so is the group's output (plane floats), so a workgroup moves
// whole groups with 16-B loads/stores; the cross-map max / routing goes
// through LDS.  Same window order and comparison as MaxpoolProp (A.8/A.9).
constexpr int kPoolGroups = 4;  // groups per workgroup iteration

struct PoolGroups {
  int64_t total;     // rows * groups per row
  FastDiv div_gpr;   // groups per row
  FastDiv div_gs4;   // pc*plane/4 (float4 per group)
  FastDiv div_plane;
  int plane, pc;
};

__device__ __forceinline__ int64_t group_off(const PoolGroups &pg, int64_t G,
                                             int64_t stride, int64_t size) {
  uint32_t row, gi;
  pg.div_gpr.divmod((uint32_t)G, row, gi);
  return (int64_t)row * stride + (int64_t)gi * size;
}

__global__ __launch_bounds__(256) void maxpool_group_prop_kernel(
    const float *__restrict__ src, int64_t ss, float *__restrict__ dst,
    int64_t ds, PoolGroups pg) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [kPoolGroups][pc*plane]
  const int gs = pg.pc * pg.plane, gs4 = gs >> 2;
  for (int64_t gb = (int64_t)blockIdx.x * kPoolGroups; gb < pg.total;
       gb += (int64_t)gridDim.x * kPoolGroups) {
    const int ng = pg.total - gb < kPoolGroups ? (int)(pg.total - gb) : kPoolGroups;
    for (int e = threadIdx.x; e < ng * gs4; e += 256) {
      uint32_t k, f;
      pg.div_gs4.divmod((uint32_t)e, k, f);
      const float4 *g4 = reinterpret_cast<const float4 *>(
          src + group_off(pg, gb + k, ss, gs));
      reinterpret_cast<float4 *>(sm)[e] = g4[f];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < ng * pg.plane; e += 256) {
      uint32_t k, q;
      pg.div_plane.divmod((uint32_t)e, k, q);
      const float *m = sm + k * gs + q;
      float val = -1e20f;
      for (int c = 0; c < pg.pc; c++) {
        const float v = m[c * pg.plane];
        if (val < v) val = v;
      }
      dst[group_off(pg, gb + k, ds, pg.plane) + q] = val;
    }
    __syncthreads();
  }
}

// Direct channel-group forward: no LDS and no barriers.  Output e of the
// flattened [rows x cols_out] index space reads its PC inputs straight from
// HBM; consecutive lanes read consecutive floats of each map, so every load
// instruction is a 256-B coalesced run and each input byte is read once.  All
// kPoolDirectOut * PC loads of a thread are issued before the first max.
constexpr int kPoolDirectOut = 8;

template <int PC, bool NT = false>
__global__ __launch_bounds__(256) void maxpool_direct_prop_kernel(
    const float *__restrict__ src, int64_t ss, float *__restrict__ dst,
    int64_t ds, uint32_t total, FastDiv div_cols, FastDiv div_plane, int plane) {
  const uint32_t base = blockIdx.x * (256u * kPoolDirectOut) + threadIdx.x;
  float v[kPoolDirectOut][PC];
  int64_t out[kPoolDirectOut];
#pragma unroll
  for (int t = 0; t < kPoolDirectOut; t++) {
    const uint32_t e = base + 256u * t;
    const uint32_t ec = e < total ? e : total - 1;
    uint32_t row, j, k, q;
    div_cols.divmod(ec, row, j);
    div_plane.divmod(j, k, q);
    const float *m = src + (int64_t)row * ss + (int64_t)k * PC * plane + q;
#pragma unroll
    for (int c = 0; c < PC; c++)
      v[t][c] = NT ? __builtin_nontemporal_load(m + c * plane) : m[c * plane];
    out[t] = e < total ? (int64_t)row * ds + j : -1;
  }
#pragma unroll
  for (int t = 0; t < kPoolDirectOut; t++) {
    float val = -1e20f;
#pragma unroll
    for (int c = 0; c < PC; c++)
      if (val < v[t][c]) val = v[t][c];
    if (out[t] >= 0) {
      if (NT) __builtin_nontemporal_store(val, dst + out[t]);
      else dst[out[t]] = val;
    }
  }
}

// Direct channel-group backprop (write_all semantics, like the group kernel
// below): output e routes dP[e] to every input of its window equal to P[e].
template <int PC, bool NT = false>
__global__ __launch_bounds__(256) void maxpool_direct_backprop_kernel(
    const float *__restrict__ x, int64_t xs, const float *__restrict__ y,
    int64_t ys, const float *__restrict__ dy, int64_t dys,
    float *__restrict__ dx, int64_t dxs, uint32_t total, FastDiv div_cols,
    FastDiv div_plane, int plane) {
  const uint32_t base = blockIdx.x * (256u * kPoolDirectOut) + threadIdx.x;
  float v[kPoolDirectOut][PC], pv[kPoolDirectOut], dv[kPoolDirectOut];
  int64_t in_off[kPoolDirectOut];
  bool ok[kPoolDirectOut];
#pragma unroll
  for (int t = 0; t < kPoolDirectOut; t++) {
    const uint32_t e = base + 256u * t;
    ok[t] = e < total;
    const uint32_t ec = ok[t] ? e : total - 1;
    uint32_t row, j, k, q;
    div_cols.divmod(ec, row, j);
    div_plane.divmod(j, k, q);
    const int64_t w = (int64_t)k * PC * plane + q;
    const float *m = x + (int64_t)row * xs + w;
#pragma unroll
    for (int c = 0; c < PC; c++)
      v[t][c] = NT ? __builtin_nontemporal_load(m + c * plane) : m[c * plane];
    pv[t] = NT ? __builtin_nontemporal_load(y + (int64_t)row * ys + j)
               : y[(int64_t)row * ys + j];
    dv[t] = NT ? __builtin_nontemporal_load(dy + (int64_t)row * dys + j)
               : dy[(int64_t)row * dys + j];  // own stride (B14)
    in_off[t] = (int64_t)row * dxs + w;
  }
#pragma unroll
  for (int t = 0; t < kPoolDirectOut; t++) {
    if (!ok[t]) continue;
#pragma unroll
    for (int c = 0; c < PC; c++) {
      const float r = v[t][c] == pv[t] ? dv[t] : 0.0f;
      if (NT) __builtin_nontemporal_store(r, dx + in_off[t] + c * plane);
      else dx[in_off[t] + c * plane] = r;
    }
  }
}

// Non-overlap backprop for general (ph x pw x pc) windows (c5's 3-D pools),
// gather form with write_all semantics: a thread takes 4 consecutive inputs
// (16-B load and store), finds each one's window j and writes
// dP[j] if in == P[j], else 0 (A.9; the window's P/dP reads hit L1/L2).
constexpr int kPoolWinVec = 2;  // float4 groups per thread in flight
__global__ __launch_bounds__(256) void maxpool_window_backprop_kernel(
    const float *__restrict__ x, int64_t xs, const float *__restrict__ y, int64_t ys,
    const float *__restrict__ dy, int64_t dys, float *__restrict__ dx, int64_t dxs,
    uint32_t total4, FastDiv div_cols4, FastDiv div_plane, FastDiv div_h, FastDiv div_ph,
    FastDiv div_pw, FastDiv div_pc, int H, int W, int outplane, int outh) {
  const uint32_t base = blockIdx.x * (256u * kPoolWinVec) + threadIdx.x;
  float4 xv[kPoolWinVec];
  float pv[kPoolWinVec][4], dv[kPoolWinVec][4];
  int64_t off[kPoolWinVec];
#pragma unroll
  for (int t = 0; t < kPoolWinVec; t++) {
    const uint32_t e0 = base + 256u * t;
    const uint32_t e = e0 < total4 ? e0 : total4 - 1;
    uint32_t row, q4, c, rem, w, h;
    div_cols4.divmod(e, row, q4);
    const uint32_t col = 4 * q4;
    div_plane.divmod(col, c, rem);
    div_h.divmod(rem, w, h);
    xv[t] = *reinterpret_cast<const float4 *>(x + (int64_t)row * xs + col);
    const float *yr = y + (int64_t)row * ys;
    const float *dr = dy + (int64_t)row * dys;  // own stride (B14)
    // window coordinates once, then stepped with the element (h fastest)
    uint32_t jc, bc, jw, bw, jh, bh;
    div_pc.divmod(c, jc, bc);
    div_pw.divmod(w, jw, bw);
    div_ph.divmod(h, jh, bh);
    const uint32_t ph = div_ph.d, pw = div_pw.d, pc = div_pc.d;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t j = jc * (uint32_t)outplane + jw * (uint32_t)outh + jh;
      pv[t][k] = yr[j];
      dv[t][k] = dr[j];
      if (++bh == ph) { bh = 0; ++jh; }
      if (++h == (uint32_t)H) {
        h = 0; bh = 0; jh = 0;
        if (++bw == pw) { bw = 0; ++jw; }
        if (++w == (uint32_t)W) {
          w = 0; bw = 0; jw = 0;
          if (++bc == pc) { bc = 0; ++jc; }
        }
      }
    }
    off[t] = (int64_t)row * dxs + col;
  }
#pragma unroll
  for (int t = 0; t < kPoolWinVec; t++) {
    if (base + 256u * t >= total4) continue;
    float4 o;
    o.x = xv[t].x == pv[t][0] ? dv[t][0] : 0.0f;
    o.y = xv[t].y == pv[t][1] ? dv[t][1] : 0.0f;
    o.z = xv[t].z == pv[t][2] ? dv[t][2] : 0.0f;
    o.w = xv[t].w == pv[t][3] ? dv[t][3] : 0.0f;
    *reinterpret_cast<float4 *>(dx + off[t]) = o;
  }
}

// 3-D windows (ph x pw x pc, c5's P1/P2), one wave per (row, output
// channel group): the group's pc input maps are one contiguous run of the
// row (pc*H*W floats) and its outputs another (OP = H/ph * W/pw), so every
// HBM access is a coalesced 16-B-per-lane run; the window gathers happen in
// LDS.  Forward: A.8 (val = -1e20, `val < x`).  (A plane backprop measured
// slower than maxpool_window_backprop_kernel's 16-B gather: 0.99 vs 0.85 ms
// at c5.)
struct PoolPlane {
  int H, W, ph, pw, pc, HW, blk, OP, oh2, units, vec;
  FastDiv div_groups, div_oh2;
};

__device__ __forceinline__ void plane_copy_in(float *dst, const float *src, int n, int vec,
                                              int lane) {
  if (vec) {
    for (int i = lane; i < n / 4; i += 64)
      reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(src)[i];
  } else {
    for (int i = lane; i < n; i += 64) dst[i] = src[i];
  }
}

__global__ __launch_bounds__(64) void maxpool_plane_prop_kernel(
    const float *__restrict__ src, int64_t ss, float *__restrict__ pool, int64_t ps,
    PoolPlane q) {
  extern __shared__ __attribute__((aligned(16))) float blk[];
  const int lane = threadIdx.x;
  for (int u = blockIdx.x; u < q.units; u += gridDim.x) {
    uint32_t n, oc;
    q.div_groups.divmod((uint32_t)u, n, oc);
    plane_copy_in(blk, src + (int64_t)n * ss + (int64_t)oc * q.blk, q.blk, q.vec, lane);
    __syncthreads();
    float *out = pool + (int64_t)n * ps + (int64_t)oc * q.OP;
    for (int o = lane; o < q.OP; o += 64) {
      uint32_t wi, hi;
      q.div_oh2.divmod((uint32_t)o, wi, hi);
      const float *b = blk + wi * q.pw * q.H + hi * q.ph;
      float val = -1e20f;
      for (int c = 0; c < q.pc; c++)
        for (int w = 0; w < q.pw; w++)
          for (int h = 0; h < q.ph; h++) {
            const float x = b[c * q.HW + w * q.H + h];
            if (val < x) val = x;
          }
      out[o] = val;
    }
    __syncthreads();
  }
}

PoolPlane make_pool_plane(int64_t rows, int in_cols, int H, int W, int ph, int pw, int pc,
                          bool vec) {
  PoolPlane q;
  q.H = H; q.W = W; q.ph = ph; q.pw = pw; q.pc = pc;
  q.HW = H * W;
  q.blk = pc * q.HW;
  q.oh2 = H / ph;
  q.OP = q.oh2 * (W / pw);
  const int groups = in_cols / q.blk;
  q.units = (int)(rows * groups);
  q.vec = vec ? 1 : 0;
  q.div_groups = FastDiv((uint32_t)groups);
  q.div_oh2 = FastDiv((uint32_t)q.oh2);
  return q;
}

bool env_pool_direct();

// Plane kernels apply to non-overlap windows with ph*pw > 1 whose group of
// pc maps fits the LDS budget; 16-B copies when the runs are aligned.
bool pool_plane_ok(int in_cols, int H, int W, int ph, int pw, int pc, int mode,
                   int64_t rows) {
  // a wave per run pays off for runs of >= 256 floats (c5 P1: 1452, P2: 288;
  // nnet.config's 1x2x1 pool has 12-float runs and goes element-wise)
  return mode == 0 && (ph > 1 || pw > 1) && H % ph == 0 && W % pw == 0 && pc * H * W >= 256 &&
         in_cols % (pc * H * W) == 0 && (size_t)(pc * H * W + 2 * (H / ph) * (W / pw)) * 4 <= 32768 &&
         rows * (in_cols / (pc * H * W)) < ((int64_t)1 << 31) && env_pool_direct();
}

unsigned plane_grid(int units) { return (unsigned)(units < 256 * 24 ? units : 256 * 24); }

// Intermap pooling (reference cnsl-cu-kernels.cu:310-503)
// as channel streams: a thread owns one (row, map position) -- lanes along
// the position, so every access is a coalesced row segment -- and walks the
// channels in order with the last PC values in registers.  Each input, pool
// value and derivative is read once (overlap2D: once per output-grid row
// that uses it, from L2).  Same comparisons, start value and summation
// order as the element-wise forms (A.10; backprop in the gather form of B2,
// increasing output channel, from 0).
template <int PC>
__global__ __launch_bounds__(256) void maxpool_overlap_prop_kernel(
    const float *__restrict__ x, int64_t xs, float *__restrict__ y, int64_t ys, int rows,
    int plane, int C) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)rows * plane) return;
  const int r = (int)(t / plane), pos = (int)(t - (int64_t)r * plane);
  const float *xr = x + (int64_t)r * xs + pos;
  float *yr = y + (int64_t)r * ys + pos;
  float ring[PC];
#pragma unroll
  for (int k = 0; k < PC - 1; k++) ring[k + 1] = xr[(int64_t)k * plane];
#pragma unroll 16
  for (int oc = 0; oc + PC - 1 < C; oc++) {
#pragma unroll
    for (int k = 0; k < PC - 1; k++) ring[k] = ring[k + 1];
    ring[PC - 1] = xr[(int64_t)(oc + PC - 1) * plane];
    float val = -1e20f;
#pragma unroll
    for (int k = 0; k < PC; k++)
      if (val < ring[k]) val = ring[k];
    yr[(int64_t)oc * plane] = val;
  }
}

template <int PC>
__global__ __launch_bounds__(256) void maxpool_overlap_backprop_kernel(
    const float *__restrict__ x, int64_t xs, const float *__restrict__ y, int64_t ys,
    const float *__restrict__ dy, int64_t dys, float *__restrict__ dx, int64_t dxs,
    int rows, int plane, int C, int write_all) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)rows * plane) return;
  const int r = (int)(t / plane), pos = (int)(t - (int64_t)r * plane);
  const int OC = C - PC + 1;
  const float *xr = x + (int64_t)r * xs + pos;
  const float *yr = y + (int64_t)r * ys + pos;
  const float *er = dy + (int64_t)r * dys + pos;  // own stride (B14)
  float *dr = dx + (int64_t)r * dxs + pos;
  // ring slot k holds output channel c - (PC-1) + k (invalid: NaN never matches)
  float ov[PC], ev[PC];
#pragma unroll
  for (int k = 0; k < PC; k++) { ov[k] = __builtin_nanf(""); ev[k] = 0.0f; }
#pragma unroll 16
  for (int c = 0; c < C; c++) {
#pragma unroll
    for (int k = 0; k < PC - 1; k++) { ov[k] = ov[k + 1]; ev[k] = ev[k + 1]; }
    if (c < OC) {
      ov[PC - 1] = yr[(int64_t)c * plane];
      ev[PC - 1] = er[(int64_t)c * plane];
    } else {
      ov[PC - 1] = __builtin_nanf("");
      ev[PC - 1] = 0.0f;
    }
    const float xv = xr[(int64_t)c * plane];
    float acc = 0.0f;
    bool any = false;
#pragma unroll
    for (int k = 0; k < PC; k++)
      if (xv == ov[k]) { acc += ev[k]; any = true; }
    if (write_all) dr[(int64_t)c * plane] = acc;
    else if (any) dr[(int64_t)c * plane] += acc;
  }
}

// overlap2D: channels form an in2 x in2 grid, outputs an o2 x o2 grid
// (o2 = in2 - PC + 1); output (ox, oy) = max over input (ox+cx, oy+cy).
// A thread owns (row, position, output-grid row ox).
template <int PC>
__global__ __launch_bounds__(256) void maxpool_overlap2d_prop_kernel(
    const float *__restrict__ x, int64_t xs, float *__restrict__ y, int64_t ys, int rows,
    int plane, int o2) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)plane * o2;
  if (t >= (int64_t)rows * per) return;
  const int r = (int)(t / per);
  const int rem = (int)(t - (int64_t)r * per);
  const int ox = rem / plane, pos = rem - ox * plane;
  const int in2 = o2 + PC - 1;
  const float *xr = x + (int64_t)r * xs + pos;
  float *yr = y + (int64_t)r * ys + pos;
  // col[cy][cx] = input (ox + cx, oy + cy): a ring of PC grid columns, one
  // new column per output (each input read once by this thread)
  float col[PC][PC];
#pragma unroll
  for (int cy = 1; cy < PC; cy++)
#pragma unroll
    for (int cx = 0; cx < PC; cx++)
      col[cy][cx] = xr[(int64_t)((ox + cx) * in2 + cy - 1) * plane];
#pragma unroll 4
  for (int oy = 0; oy < o2; oy++) {
#pragma unroll
    for (int cy = 0; cy < PC - 1; cy++)
#pragma unroll
      for (int cx = 0; cx < PC; cx++) col[cy][cx] = col[cy + 1][cx];
#pragma unroll
    for (int cx = 0; cx < PC; cx++)
      col[PC - 1][cx] = xr[(int64_t)((ox + cx) * in2 + oy + PC - 1) * plane];
    float val = -1e20f;
#pragma unroll
    for (int cx = 0; cx < PC; cx++)
#pragma unroll
      for (int cy = 0; cy < PC; cy++)
        if (val < col[cy][cx]) val = col[cy][cx];
    yr[(int64_t)(ox * o2 + oy) * plane] = val;
  }
}

// A thread owns (row, position, input-grid row X) and sums, for each input
// (X, Y), the outputs (xo, yo) whose window holds it, xo then yo increasing.
template <int PC>
__global__ __launch_bounds__(256) void maxpool_overlap2d_backprop_kernel(
    const float *__restrict__ x, int64_t xs, const float *__restrict__ y, int64_t ys,
    const float *__restrict__ dy, int64_t dys, float *__restrict__ dx, int64_t dxs,
    int rows, int plane, int o2, int write_all) {
  const int in2 = o2 + PC - 1;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t per = (int64_t)plane * in2;
  if (t >= (int64_t)rows * per) return;
  const int r = (int)(t / per);
  const int rem = (int)(t - (int64_t)r * per);
  const int X = rem / plane, pos = rem - X * plane;
  const float *xr = x + (int64_t)r * xs + pos;
  const float *yr = y + (int64_t)r * ys + pos;
  const float *er = dy + (int64_t)r * dys + pos;
  float *dr = dx + (int64_t)r * dxs + pos;
  // ring [a][b]: output (X - a, Y - b); a new column yo = Y enters per step
  // (NaN: no such output, never equal)
  float ov[PC][PC], ev[PC][PC];
#pragma unroll
  for (int a = 0; a < PC; a++)
#pragma unroll
    for (int b = 0; b < PC; b++) { ov[a][b] = __builtin_nanf(""); ev[a][b] = 0.0f; }
#pragma unroll 4
  for (int Y = 0; Y < in2; Y++) {
#pragma unroll
    for (int a = 0; a < PC; a++) {
#pragma unroll
      for (int b = PC - 1; b > 0; b--) { ov[a][b] = ov[a][b - 1]; ev[a][b] = ev[a][b - 1]; }
      const int xo = X - a;
      if (xo >= 0 && xo < o2 && Y < o2) {
        const int64_t j = (int64_t)(xo * o2 + Y) * plane;
        ov[a][0] = yr[j];
        ev[a][0] = er[j];
      } else {
        ov[a][0] = __builtin_nanf("");
        ev[a][0] = 0.0f;
      }
    }
    const float xv = xr[(int64_t)(X * in2 + Y) * plane];
    float acc = 0.0f;
    bool any = false;
#pragma unroll
    for (int a = PC - 1; a >= 0; a--)      // xo = X - a, increasing
#pragma unroll
      for (int b = PC - 1; b >= 0; b--)    // yo = Y - b, increasing
        if (xv == ov[a][b]) { acc += ev[a][b]; any = true; }
    if (write_all) dr[(int64_t)(X * in2 + Y) * plane] = acc;
    else if (any) dr[(int64_t)(X * in2 + Y) * plane] += acc;
  }
}

// Backprop of a 3-D window pool from the fused forward's 16-bit mask: a
// thread takes 4 consecutive inputs (16-B store), each one's window j and bit
// b = (c % pc)*pw*ph + (w % pw)*ph + (h % ph); dX = bit ? dP[j] : 0.
__global__ __launch_bounds__(256) void maxpool_mask3d_backprop_kernel(
    const unsigned short *__restrict__ mask, int64_t ms, const float *__restrict__ dy,
    int64_t dys, float *__restrict__ dx, int64_t dxs, uint32_t total4, FastDiv div_cols4,
    FastDiv div_plane, FastDiv div_h, FastDiv div_ph, FastDiv div_pw, FastDiv div_pc,
    int H, int W, int outplane, int outh) {
  const uint32_t base = blockIdx.x * (256u * kPoolWinVec) + threadIdx.x;
  float res[kPoolWinVec][4];
  int64_t off[kPoolWinVec];
#pragma unroll
  for (int t = 0; t < kPoolWinVec; t++) {
    const uint32_t e0 = base + 256u * t;
    const uint32_t e = e0 < total4 ? e0 : total4 - 1;
    uint32_t row, q4, c, rem, w, h;
    div_cols4.divmod(e, row, q4);
    const uint32_t col = 4 * q4;
    div_plane.divmod(col, c, rem);
    div_h.divmod(rem, w, h);
    const unsigned short *mr = mask + (int64_t)row * ms;
    const float *dr = dy + (int64_t)row * dys;
    // window coordinates once, then stepped with the element (h fastest)
    uint32_t jc, bc, jw, bw, jh, bh;
    div_pc.divmod(c, jc, bc);
    div_pw.divmod(w, jw, bw);
    div_ph.divmod(h, jh, bh);
    const uint32_t ph = div_ph.d, pw = div_pw.d, pc = div_pc.d;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t j = jc * (uint32_t)outplane + jw * (uint32_t)outh + jh;
      const uint32_t bit = (bc * pw + bw) * ph + bh;
      res[t][k] = (mr[j] >> bit) & 1u ? dr[j] : 0.0f;
      if (++bh == ph) { bh = 0; ++jh; }
      if (++h == (uint32_t)H) {
        h = 0; bh = 0; jh = 0;
        if (++bw == pw) { bw = 0; ++jw; }
        if (++w == (uint32_t)W) {
          w = 0; bw = 0; jw = 0;
          if (++bc == pc) { bc = 0; ++jc; }
        }
      }
    }
    off[t] = (int64_t)row * dxs + col;
  }
#pragma unroll
  for (int t = 0; t < kPoolWinVec; t++) {
    if (base + 256u * t >= total4) continue;
    *reinterpret_cast<float4 *>(dx + off[t]) =
        make_float4(res[t][0], res[t][1], res[t][2], res[t][3]);
  }
}

// Scatter form of the same: a thread owns one pooled value (window) and
// writes its ph*pw*pc inputs (pc runs of pw runs of ph consecutive floats;
// the runs of neighbouring lanes tile each map column).  The window index is
// computed once per window instead of once per input.
// PH/PW/PC > 0: the window fixed at compile time (c5's 3x1x4, 2x1x4), so the
// loops unroll into straight stores; 0 = runtime dims.
template <int PH, int PW, int PC>
__global__ __launch_bounds__(256) void maxpool_mask3d_scatter_kernel(
    const unsigned short *__restrict__ mask, int64_t ms, const float *__restrict__ dy,
    int64_t dys, float *__restrict__ dx, int64_t dxs, uint32_t total, FastDiv div_cols,
    FastDiv div_OP, FastDiv div_oh2, int H, int plane, int ph_, int pw_, int pc_) {
  const int ph = PH > 0 ? PH : ph_, pw = PW > 0 ? PW : pw_, pc = PC > 0 ? PC : pc_;
  const uint32_t e = blockIdx.x * 256u + threadIdx.x;
  if (e >= total) return;
  uint32_t row, j, jc, q, wi, hi;
  div_cols.divmod(e, row, j);
  div_OP.divmod(j, jc, q);
  div_oh2.divmod(q, wi, hi);
  const unsigned m = mask[(int64_t)row * ms + j];
  const float d = dy[(int64_t)row * dys + j];
  float *base = dx + (int64_t)row * dxs + (int64_t)jc * pc * plane + (int64_t)wi * pw * H +
                (int64_t)hi * ph;
  if constexpr (PH > 0) {  // compile-time window: straight-line stores
#pragma unroll
    for (int c = 0; c < PC; c++)
#pragma unroll
      for (int w = 0; w < PW; w++)
#pragma unroll
        for (int h = 0; h < PH; h++)
          base[(int64_t)c * plane + (int64_t)w * H + h] =
              (m >> ((c * PW + w) * PH + h)) & 1u ? d : 0.0f;
  } else {
    int bit = 0;
    for (int c = 0; c < pc; c++)
      for (int w = 0; w < pw; w++) {
        float *col = base + (int64_t)c * plane + (int64_t)w * H;
        for (int h = 0; h < ph; h++, bit++) col[h] = (m >> bit) & 1u ? d : 0.0f;
      }
  }
}

// Backprop of the channel-only pool from the routing mask saved by the fused
// forward (hipF_conv2d_maxpool): dX[(PC j + c) plane + q] = bit c of
// mask[j plane + q] ? dP[j plane + q] : 0 -- the same values A.9 produces
// from in_value == out_value, read from 1 byte instead of PC + 1 floats.
template <int PC>
__global__ __launch_bounds__(256) void maxpool_mask_backprop_kernel(
    const unsigned char *__restrict__ mask, int64_t ms,
    const float *__restrict__ dy, int64_t dys, float *__restrict__ dx,
    int64_t dxs, uint32_t total, FastDiv div_cols, FastDiv div_plane, int plane) {
  const uint32_t base = blockIdx.x * (256u * kPoolDirectOut) + threadIdx.x;
  unsigned mv[kPoolDirectOut];
  float dv[kPoolDirectOut];
  int64_t off[kPoolDirectOut];
#pragma unroll
  for (int t = 0; t < kPoolDirectOut; t++) {
    const uint32_t e = base + 256u * t;
    const uint32_t ec = e < total ? e : total - 1;
    uint32_t row, j, k, q;
    div_cols.divmod(ec, row, j);
    div_plane.divmod(j, k, q);
    mv[t] = mask[(int64_t)row * ms + j];
    dv[t] = dy[(int64_t)row * dys + j];
    off[t] = e < total ? (int64_t)row * dxs + (int64_t)k * PC * plane + q : -1;
  }
#pragma unroll
  for (int t = 0; t < kPoolDirectOut; t++) {
    if (off[t] < 0) continue;
#pragma unroll
    for (int c = 0; c < PC; c++)
      dx[off[t] + c * plane] = (mv[t] >> c) & 1u ? dv[t] : 0.0f;
  }
}

// Writes every element of the group (routed derivative or 0): the fused
// in_deriv->Resize(kSetZero) of MaxpoolComponent::Backprop (:889).
__global__ __launch_bounds__(256) void maxpool_group_backprop_kernel(
    const float *__restrict__ x, int64_t xs, const float *__restrict__ y,
    int64_t ys, const float *__restrict__ dy, int64_t dys,
    float *__restrict__ dx, int64_t dxs, PoolGroups pg) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [2][kPoolGroups][plane]
  float *sy = sm, *sd = sm + kPoolGroups * pg.plane;
  const int gs = pg.pc * pg.plane, gs4 = gs >> 2;
  for (int64_t gb = (int64_t)blockIdx.x * kPoolGroups; gb < pg.total;
       gb += (int64_t)gridDim.x * kPoolGroups) {
    const int ng = pg.total - gb < kPoolGroups ? (int)(pg.total - gb) : kPoolGroups;
    for (int e = threadIdx.x; e < ng * pg.plane; e += 256) {
      uint32_t k, q;
      pg.div_plane.divmod((uint32_t)e, k, q);
      sy[e] = y[group_off(pg, gb + k, ys, pg.plane) + q];
      sd[e] = dy[group_off(pg, gb + k, dys, pg.plane) + q];  // own stride (B14)
    }
    __syncthreads();
    for (int e = threadIdx.x; e < ng * gs4; e += 256) {
      uint32_t k, f;
      pg.div_gs4.divmod((uint32_t)e, k, f);
      const int64_t gx = group_off(pg, gb + k, xs, gs);
      const int64_t gd = group_off(pg, gb + k, dxs, gs);
      const float4 v = reinterpret_cast<const float4 *>(x + gx)[f];
      uint32_t c, q;
      pg.div_plane.divmod(4 * f, c, q);
      const float *yk = sy + k * pg.plane, *dk = sd + k * pg.plane;
      float o[4];
      const float in[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int t = 0; t < 4; t++) {
        o[t] = in[t] == yk[q] ? dk[q] : 0.0f;
        if (++q == (uint32_t)pg.plane) q = 0;
      }
      reinterpret_cast<float4 *>(dx + gd)[f] = make_float4(o[0], o[1], o[2], o[3]);
    }
    __syncthreads();
  }
}

// KCNN_POOL_DIRECT=0 selects the LDS-staged group forward (A/B measurements).
bool env_pool_direct() {
  static const int v = KCNN_KNOB("KCNN_POOL_DIRECT", 1);
  return v != 0;
}

// The group kernels apply when the pool is channel-only and every group of
// every row starts 16-B aligned.
bool pool_groups_ok(const void *a, int64_t stride, int plane, int pc, int ph,
                    int pw, int mode) {
  return mode == 0 && ph == 1 && pw == 1 && ((plane * pc) & 3) == 0 &&
         (stride & 3) == 0 && ((uintptr_t)a & 15) == 0 &&
         (size_t)kPoolGroups * plane * pc * 4 <= 64 * 1024;
}

PoolGroups make_pool_groups(int64_t rows, int cols_out, int plane, int pc) {
  PoolGroups pg;
  const int gpr = cols_out / plane;
  pg.total = rows * gpr;
  pg.div_gpr = FastDiv((uint32_t)gpr);
  pg.div_gs4 = FastDiv((uint32_t)(plane * pc / 4));
  pg.div_plane = FastDiv((uint32_t)plane);
  pg.plane = plane;
  pg.pc = pc;
  return pg;
}

// Grid-stride pool kernels launch exactly one resident wave of workgroups:
// with more blocks than fit (the forward's 23 KB of LDS allows 6 per CU at
// c2), the surplus runs as a second, mostly idle round.
template <typename K>
unsigned pool_grid(int64_t total, K kernel, size_t lds_bytes) {
  static thread_local int dev = -1, cus = 0;
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) d = 0;
  if (d != dev) {
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) !=
        hipSuccess || cus <= 0)
      cus = 256;
    dev = d;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds_bytes) !=
          hipSuccess || per_cu <= 0)
    per_cu = 1;
  const int64_t b = (total + kPoolGroups - 1) / kPoolGroups;
  const int64_t cap = (int64_t)cus * per_cu;
  return (unsigned)(b < cap ? (b > 0 ? b : 1) : cap);
}

PoolGeom make_pool_geom(int in_h, int in_w, int ph, int pw, int pc, int mode,
                        int out_cols) {
  PoolGeom g;
  g.in_h = in_h; g.in_w = in_w; g.ph = ph; g.pw = pw; g.pc = pc; g.mode = mode;
  g.plane = (int64_t)in_h * in_w;
  const int oh = in_h / ph, ow = in_w / pw;
  g.div_outplane = FastDiv((uint32_t)(mode == 2 ? in_h * in_w : oh * ow));
  g.div_outh = FastDiv((uint32_t)oh);
  g.out_2d = g.in_2d = 1;
  g.div_out2d = FastDiv(1);
  if (mode == 2) {
    const int out_channel = out_cols / (in_h * in_w);
    int o2 = 0;
    while ((o2 + 1) * (o2 + 1) <= out_channel) o2++;  // (int)sqrt
    g.out_2d = o2 > 0 ? o2 : 1;
    g.in_2d = g.out_2d + pc - 1;
    g.div_out2d = FastDiv((uint32_t)g.out_2d);
  }
  return g;
}

}  // namespace

// ===========================================================================
// extern "C" shim (include/cnsl-hip-kernels.h)
// ===========================================================================
extern "C" {

int hipF_span_row_to_convmat(const float *in, MatrixDim in_dim, float *span,
                             MatrixDim span_dim, int in_height, int in_width,
                             int in_channel, int kernel_height,
                             int kernel_width, int64_t row_offset,
                             kcnn_stream_t stream) {
  (void)in_channel;
  SpanRowToConvmat f{in, in_dim, span, span_dim, in_height, in_width,
                     kernel_height, row_offset,
                     FastDiv((uint32_t)(kernel_height * kernel_width)),
                     FastDiv((uint32_t)kernel_height),
                     FastDiv((uint32_t)in_dim.rows),
                     FastDiv((uint32_t)(in_height - kernel_height + 1))};
  return launch_elem2d(span_dim.rows, span_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_convmat_to_out(const float *conv_mat, MatrixDim conv_dim, float *out,
                        MatrixDim out_dim, int out_height, int out_width,
                        int num_sample, kcnn_stream_t stream) {
  ConvmatToOut f{conv_mat, conv_dim, out, out_dim,
                 (int64_t)out_height * out_width,
                 FastDiv((uint32_t)num_sample)};
  return launch_elem2d(conv_dim.rows, conv_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_add_mat_rep_vec(const float *vec, int rep, float *out,
                         MatrixDim out_dim, kcnn_stream_t stream) {
  AddMatRepVec f{vec, out, out_dim, FastDiv((uint32_t)rep)};
  return launch_elem2d(out_dim.rows, out_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_flip_mat(const float *orig, MatrixDim orig_dim, int kernel_height,
                  int kernel_width, int group, float *flip, MatrixDim flip_dim,
                  kcnn_stream_t stream) {
  (void)group;
  const int ks = kernel_height * kernel_width;
  FlipMat f{orig, orig_dim, flip, flip_dim, ks, FastDiv((uint32_t)ks)};
  return launch_elem2d(flip_dim.rows, flip_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_pad_zero(const float *orig, MatrixDim orig_dim, int orig_height,
                  int orig_width, int kernel_height, int kernel_width,
                  float *padmat, MatrixDim padmat_dim, kcnn_stream_t stream) {
  const int ph = orig_height + 2 * (kernel_height - 1);
  const int pw = orig_width + 2 * (kernel_width - 1);
  PadZero f{orig, orig_dim, padmat, padmat_dim, orig_height, orig_width,
            kernel_height, kernel_width, FastDiv((uint32_t)(ph * pw)),
            FastDiv((uint32_t)ph)};
  return launch_elem2d(padmat_dim.rows, padmat_dim.cols, f,
                       kcnn::as_stream(stream));
}

int hipF_tp_block(const float *in, MatrixDim in_dim, float *out,
                  MatrixDim out_dim, int block_size, kcnn_stream_t stream) {
  TpBlock f{in, in_dim, out, out_dim, block_size,
            FastDiv((uint32_t)block_size)};
  return launch_elem2d(out_dim.rows, out_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_tp_inside_block(const float *in, MatrixDim in_dim, float *out,
                         MatrixDim out_dim, int block_size,
                         kcnn_stream_t stream) {
  TpInsideBlock f{in, in_dim, out, out_dim, block_size,
                  FastDiv((uint32_t)block_size)};
  return launch_elem2d(out_dim.rows, out_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_mod_permute_row(const float *in, MatrixDim in_dim, float *out,
                         MatrixDim out_dim, int block_size, int in_channel,
                         kcnn_stream_t stream) {
  ModPermuteRow f{in, in_dim, out, out_dim, block_size,
                  FastDiv((uint32_t)in_channel)};
  return launch_elem2d(in_dim.rows, in_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_maxpool_backprop_mask3d(const unsigned short *mask, int mask_stride,
                                 const float *out_deriv, MatrixDim out_deriv_dim,
                                 float *in_deriv, MatrixDim in_deriv_dim,
                                 int in_height, int in_width, int pool_height_dim,
                                 int pool_width_dim, int pool_channel_dim,
                                 kcnn_stream_t stream) {
  const int ph = pool_height_dim, pw = pool_width_dim, pc = pool_channel_dim;
  const int plane = in_height * in_width;
  if (plane <= 0 || ph <= 0 || pw <= 0 || pc <= 0 || in_height % ph != 0 ||
      in_width % pw != 0 || ph * pw * pc > 16 || mask_stride < out_deriv_dim.cols ||
      in_deriv_dim.rows != out_deriv_dim.rows ||
      (int64_t)out_deriv_dim.cols * ph * pw * pc != in_deriv_dim.cols ||
      in_deriv_dim.cols % (plane * pc) != 0 || in_deriv_dim.cols % 4 != 0 ||
      in_deriv_dim.stride % 4 != 0 || (uintptr_t)in_deriv % 16 != 0)
    return (int)hipErrorInvalidValue;
  const int outh = in_height / ph;
  const int outplane = outh * (in_width / pw);
  static const int scatter = KCNN_KNOB("KCNN_MASK3D_SCATTER", 1);
  if (scatter) {
    const int64_t nout = (int64_t)out_deriv_dim.rows * out_deriv_dim.cols;
    if (nout == 0) return 0;
    if (nout >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
    auto kern = maxpool_mask3d_scatter_kernel<0, 0, 0>;
    if (ph == 3 && pw == 1 && pc == 4) kern = maxpool_mask3d_scatter_kernel<3, 1, 4>;
    else if (ph == 2 && pw == 1 && pc == 4) kern = maxpool_mask3d_scatter_kernel<2, 1, 4>;
    else if (ph == 2 && pw == 2 && pc == 2) kern = maxpool_mask3d_scatter_kernel<2, 2, 2>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((nout + 255) / 256)), dim3(256), 0,
                       kcnn::as_stream(stream), mask, (int64_t)mask_stride, out_deriv,
                       (int64_t)out_deriv_dim.stride, in_deriv, (int64_t)in_deriv_dim.stride,
                       (uint32_t)nout, FastDiv((uint32_t)out_deriv_dim.cols),
                       FastDiv((uint32_t)outplane), FastDiv((uint32_t)outh), in_height, plane,
                       ph, pw, pc);
    return kcnn::launch_status();
  }
  const int64_t n4 = (int64_t)in_deriv_dim.rows * in_deriv_dim.cols / 4;
  if (n4 == 0) return 0;
  if (n4 >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  const uint32_t total4 = (uint32_t)n4;
  const unsigned blocks = (total4 + 256 * kPoolWinVec - 1) / (256 * kPoolWinVec);
  hipLaunchKernelGGL(maxpool_mask3d_backprop_kernel, dim3(blocks), dim3(256), 0,
                     kcnn::as_stream(stream), mask, (int64_t)mask_stride, out_deriv,
                     (int64_t)out_deriv_dim.stride, in_deriv, (int64_t)in_deriv_dim.stride,
                     total4, FastDiv((uint32_t)(in_deriv_dim.cols / 4)),
                     FastDiv((uint32_t)plane), FastDiv((uint32_t)in_height),
                     FastDiv((uint32_t)ph), FastDiv((uint32_t)pw), FastDiv((uint32_t)pc),
                     in_height, in_width, outplane, outh);
  return kcnn::launch_status();
}

int hipF_maxpool_backprop_mask(const unsigned char *mask, int mask_stride,
                               const float *out_deriv, MatrixDim out_deriv_dim,
                               float *in_deriv, MatrixDim in_deriv_dim,
                               int in_height, int in_width,
                               int pool_channel_dim, kcnn_stream_t stream) {
  const int plane = in_height * in_width;
  const int pc = pool_channel_dim;
  if (plane <= 0 || !(pc == 2 || pc == 4 || pc == 8) ||
      out_deriv_dim.cols % plane != 0 || mask_stride < out_deriv_dim.cols ||
      in_deriv_dim.rows != out_deriv_dim.rows ||
      in_deriv_dim.cols != out_deriv_dim.cols * pc)
    return (int)hipErrorInvalidValue;
  const int64_t nout = (int64_t)out_deriv_dim.rows * out_deriv_dim.cols;
  if (nout == 0) return 0;
  if (nout >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  const unsigned blocks =
      (unsigned)((nout + 256 * kPoolDirectOut - 1) / (256 * kPoolDirectOut));
  auto kern = pc == 2 ? maxpool_mask_backprop_kernel<2>
              : pc == 4 ? maxpool_mask_backprop_kernel<4>
                        : maxpool_mask_backprop_kernel<8>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, kcnn::as_stream(stream), mask,
                     (int64_t)mask_stride, out_deriv, (int64_t)out_deriv_dim.stride,
                     in_deriv, (int64_t)in_deriv_dim.stride, (uint32_t)nout,
                     FastDiv((uint32_t)out_deriv_dim.cols), FastDiv((uint32_t)plane),
                     plane);
  return kcnn::launch_status();
}

int hipF_mod_permute_channels(float *comp, MatrixDim comp_dim, float *container,
                              MatrixDim container_dim, int comp_idx,
                              int num_component, int in_height, int in_width,
                              int from_comp_to_container, kcnn_stream_t stream) {
  const int plane = in_height * in_width;
  if (plane <= 0 || comp_idx < 0 || comp_idx >= num_component ||
      container_dim.rows < comp_dim.rows ||
      (comp_dim.cols > 0 &&
       ((int64_t)((comp_dim.cols - 1) / plane) * num_component + comp_idx) * plane +
               (comp_dim.cols - 1) % plane >= container_dim.cols))
    return (int)hipErrorInvalidValue;
  ModPermuteChannels f{comp, comp_dim, container, container_dim, comp_idx,
                       num_component, plane, from_comp_to_container,
                       FastDiv((uint32_t)plane)};
  return launch_elem2d(comp_dim.rows, comp_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_copy_rows_at(const float *src, MatrixDim src_dim, float *dest,
                      MatrixDim dest_dim, int64_t row_offset,
                      kcnn_stream_t stream) {
  CopyRowsAt f{src, src_dim, dest, dest_dim, row_offset};
  return launch_elem2d(src_dim.rows, src_dim.cols, f, kcnn::as_stream(stream));
}

// Streaming (nontemporal) loads and stores in the direct pool kernels.
// KCNN_POOL_NT: bit 1 forward (default on: Y read once, P written once; c2
// in the unfused step 225 -> 177-197 us, 52.8 % -> 60-67 % of HBM), bit 0
// backprop (default off: 355 -> 461 us measured).
static int pool_nt() {
  static const int v = KCNN_KNOB("KCNN_POOL_NT", 2);
  return v;
}

int hipF_maxpool_prop(const float *src, MatrixDim src_dim, float *pool,
                      MatrixDim pool_dim, int in_height, int in_width,
                      int pool_height_dim, int pool_width_dim,
                      int pool_channel_dim, int mode, kcnn_stream_t stream) {
  if (mode != 0) pool_height_dim = pool_width_dim = 1;  // cnsl-cu-kernels.cu:316
  const int plane = in_height * in_width;
  const int64_t nout = (int64_t)pool_dim.rows * pool_dim.cols;
  if (mode == 0 && pool_height_dim == 1 && pool_width_dim == 1 &&
      pool_channel_dim >= 2 && pool_channel_dim <= 4 && pool_dim.cols % plane == 0 &&
      src_dim.cols == pool_dim.cols * pool_channel_dim && nout < ((int64_t)1 << 31) &&
      env_pool_direct()) {
    if (nout == 0) return 0;
    const unsigned blocks =
        (unsigned)((nout + 256 * kPoolDirectOut - 1) / (256 * kPoolDirectOut));
    static const int nt = pool_nt();
    auto kern = pool_channel_dim == 4   ? (nt >= 2 ? maxpool_direct_prop_kernel<4, true>
                                              : maxpool_direct_prop_kernel<4>)
                : pool_channel_dim == 3 ? maxpool_direct_prop_kernel<3>
                                        : maxpool_direct_prop_kernel<2>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, kcnn::as_stream(stream),
                       src, (int64_t)src_dim.stride, pool, (int64_t)pool_dim.stride,
                       (uint32_t)nout, FastDiv((uint32_t)pool_dim.cols),
                       FastDiv((uint32_t)plane), plane);
    return kcnn::launch_status();
  }
  if (pool_plane_ok(src_dim.cols, in_height, in_width, pool_height_dim, pool_width_dim,
                    pool_channel_dim, mode, src_dim.rows) &&
      pool_dim.cols * pool_height_dim * pool_width_dim * pool_channel_dim == src_dim.cols) {
    const bool vec = ((pool_channel_dim * plane) & 3) == 0 && (src_dim.stride & 3) == 0 &&
                     ((uintptr_t)src & 15) == 0;
    PoolPlane q = make_pool_plane(src_dim.rows, src_dim.cols, in_height, in_width,
                                  pool_height_dim, pool_width_dim, pool_channel_dim, vec);
    if (q.units == 0) return 0;
    hipLaunchKernelGGL(maxpool_plane_prop_kernel, dim3(plane_grid(q.units)), dim3(64),
                       (size_t)q.blk * 4, kcnn::as_stream(stream), src,
                       (int64_t)src_dim.stride, pool, (int64_t)pool_dim.stride, q);
    return kcnn::launch_status();
  }
  if (pool_groups_ok(src, src_dim.stride, plane, pool_channel_dim,
                     pool_height_dim, pool_width_dim, mode) &&
      (int64_t)pool_dim.rows * (pool_dim.cols / plane) < ((int64_t)1 << 31) &&
      pool_dim.cols % plane == 0 && src_dim.cols == pool_dim.cols * pool_channel_dim) {
    PoolGroups pg = make_pool_groups(pool_dim.rows, pool_dim.cols, plane,
                                     pool_channel_dim);
    if (pg.total == 0) return 0;
    const size_t lds = (size_t)kPoolGroups * plane * pool_channel_dim * 4;
    hipLaunchKernelGGL(maxpool_group_prop_kernel,
                       dim3(pool_grid(pg.total, maxpool_group_prop_kernel, lds)),
                       dim3(256), lds, kcnn::as_stream(stream), src, (int64_t)src_dim.stride, pool,
                       (int64_t)pool_dim.stride, pg);
    return kcnn::launch_status();
  }
  if (mode != 0 && pool_channel_dim >= 2 && pool_channel_dim <= 4 && env_pool_direct()) {
    if (pool_dim.rows == 0 || plane == 0) return 0;
    const int C = src_dim.cols / plane;
    hipStream_t st = kcnn::as_stream(stream);
    if (mode == 1 && pool_dim.cols == (C - pool_channel_dim + 1) * plane) {
      const int64_t n = (int64_t)pool_dim.rows * plane;
      const unsigned blocks = (unsigned)((n + 255) / 256);
#define KCNN_OVP(PC_)                                                                       \
  hipLaunchKernelGGL(maxpool_overlap_prop_kernel<PC_>, dim3(blocks), dim3(256), 0, st, src, \
                     (int64_t)src_dim.stride, pool, (int64_t)pool_dim.stride, pool_dim.rows, \
                     plane, C)
      if (pool_channel_dim == 2) KCNN_OVP(2); else if (pool_channel_dim == 3) KCNN_OVP(3); else KCNN_OVP(4);
#undef KCNN_OVP
      return kcnn::launch_status();
    }
    PoolGeom g2 = make_pool_geom(in_height, in_width, 1, 1, pool_channel_dim, mode,
                                 pool_dim.cols);
    if (mode == 2 && g2.in_2d * g2.in_2d * plane <= src_dim.cols &&
        pool_dim.cols == g2.out_2d * g2.out_2d * plane) {
      const int64_t n = (int64_t)pool_dim.rows * plane * g2.out_2d;
      const unsigned blocks = (unsigned)((n + 255) / 256);
#define KCNN_OV2P(PC_)                                                                        \
  hipLaunchKernelGGL(maxpool_overlap2d_prop_kernel<PC_>, dim3(blocks), dim3(256), 0, st, src, \
                     (int64_t)src_dim.stride, pool, (int64_t)pool_dim.stride, pool_dim.rows,   \
                     plane, g2.out_2d)
      if (pool_channel_dim == 2) KCNN_OV2P(2); else if (pool_channel_dim == 3) KCNN_OV2P(3); else KCNN_OV2P(4);
#undef KCNN_OV2P
      return kcnn::launch_status();
    }
  }
  PoolGeom g = make_pool_geom(in_height, in_width, pool_height_dim,
                              pool_width_dim, pool_channel_dim, mode,
                              pool_dim.cols);
  MaxpoolProp f{src, src_dim, pool, pool_dim, g};
  return launch_elem2d(pool_dim.rows, pool_dim.cols, f, kcnn::as_stream(stream));
}

int hipF_maxpool_backprop(const float *in_val, MatrixDim in_val_dim,
                          const float *out_val, MatrixDim out_val_dim,
                          const float *out_deriv, MatrixDim out_deriv_dim,
                          float *dest, MatrixDim dest_dim, int in_height,
                          int in_width, int pool_height_dim,
                          int pool_width_dim, int pool_channel_dim, int mode,
                          int write_all, kcnn_stream_t stream) {
  hipStream_t st = kcnn::as_stream(stream);
  const int plane0 = in_height * in_width;
  const int64_t nout = (int64_t)out_val_dim.rows * out_val_dim.cols;
  if (write_all && mode == 0 && pool_height_dim == 1 && pool_width_dim == 1 &&
      pool_channel_dim >= 2 && pool_channel_dim <= 4 && out_val_dim.cols % plane0 == 0 &&
      in_val_dim.cols == out_val_dim.cols * pool_channel_dim &&
      nout < ((int64_t)1 << 31) && env_pool_direct()) {
    if (nout == 0) return 0;
    const unsigned blocks =
        (unsigned)((nout + 256 * kPoolDirectOut - 1) / (256 * kPoolDirectOut));
    static const int nt = pool_nt();
    auto kern = pool_channel_dim == 4   ? (nt == 1 || nt == 3 ? maxpool_direct_backprop_kernel<4, true>
                                                              : maxpool_direct_backprop_kernel<4>)
                : pool_channel_dim == 3 ? maxpool_direct_backprop_kernel<3>
                                        : maxpool_direct_backprop_kernel<2>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, in_val, (int64_t)in_val_dim.stride, out_val,
                       (int64_t)out_val_dim.stride, out_deriv,
                       (int64_t)out_deriv_dim.stride, dest, (int64_t)dest_dim.stride,
                       (uint32_t)nout, FastDiv((uint32_t)out_val_dim.cols),
                       FastDiv((uint32_t)plane0), plane0);
    return kcnn::launch_status();
  }
  if (write_all && mode == 0 && (pool_height_dim > 1 || pool_width_dim > 1) &&
      in_val_dim.cols % 4 == 0 && in_val_dim.stride % 4 == 0 && dest_dim.stride % 4 == 0 &&
      dest_dim.cols == in_val_dim.cols && (uintptr_t)in_val % 16 == 0 &&
      (uintptr_t)dest % 16 == 0 && in_height % pool_height_dim == 0 &&
      in_width % pool_width_dim == 0 &&
      in_val_dim.cols == out_val_dim.cols * pool_height_dim * pool_width_dim * pool_channel_dim &&
      (int64_t)in_val_dim.rows * in_val_dim.cols < ((int64_t)1 << 33) && env_pool_direct()) {
    const uint32_t total4 = (uint32_t)((int64_t)in_val_dim.rows * in_val_dim.cols / 4);
    if (total4 == 0) return 0;
    const int outh = in_height / pool_height_dim;
    const int outplane = outh * (in_width / pool_width_dim);
    const unsigned blocks = (total4 + 256 * kPoolWinVec - 1) / (256 * kPoolWinVec);
    hipLaunchKernelGGL(maxpool_window_backprop_kernel, dim3(blocks), dim3(256), 0, st,
                       in_val, (int64_t)in_val_dim.stride, out_val,
                       (int64_t)out_val_dim.stride, out_deriv, (int64_t)out_deriv_dim.stride,
                       dest, (int64_t)dest_dim.stride, total4,
                       FastDiv((uint32_t)(in_val_dim.cols / 4)), FastDiv((uint32_t)plane0),
                       FastDiv((uint32_t)in_height), FastDiv((uint32_t)pool_height_dim),
                       FastDiv((uint32_t)pool_width_dim), FastDiv((uint32_t)pool_channel_dim),
                       in_height, in_width, outplane, outh);
    return kcnn::launch_status();
  }
  if (write_all &&
      pool_groups_ok(in_val, in_val_dim.stride, plane0, pool_channel_dim,
                     pool_height_dim, pool_width_dim, mode) &&
      pool_groups_ok(dest, dest_dim.stride, plane0, pool_channel_dim,
                     pool_height_dim, pool_width_dim, mode) &&
      out_val_dim.cols % plane0 == 0 &&
      in_val_dim.cols == out_val_dim.cols * pool_channel_dim &&
      (int64_t)out_val_dim.rows * (out_val_dim.cols / plane0) < ((int64_t)1 << 31)) {
    PoolGroups pg = make_pool_groups(out_val_dim.rows, out_val_dim.cols, plane0,
                                     pool_channel_dim);
    if (pg.total == 0) return 0;
    const size_t lds = (size_t)2 * kPoolGroups * plane0 * 4;
    hipLaunchKernelGGL(maxpool_group_backprop_kernel,
                       dim3(pool_grid(pg.total, maxpool_group_backprop_kernel, lds)),
                       dim3(256), lds, st, in_val,
                       (int64_t)in_val_dim.stride, out_val, (int64_t)out_val_dim.stride,
                       out_deriv, (int64_t)out_deriv_dim.stride, dest,
                       (int64_t)dest_dim.stride, pg);
    return kcnn::launch_status();
  }
  if (mode == 0) {
    PoolGeom g = make_pool_geom(in_height, in_width, pool_height_dim,
                                pool_width_dim, pool_channel_dim, 0,
                                out_val_dim.cols);
    MaxpoolBackpropDisjoint f{in_val, in_val_dim, out_val, out_val_dim,
                              out_deriv, out_deriv_dim, dest, dest_dim, g,
                              write_all};
    return launch_elem2d(out_val_dim.rows, out_val_dim.cols, f, st);
  }
  PoolGeom g = make_pool_geom(in_height, in_width, 1, 1, pool_channel_dim,
                              mode, out_val_dim.cols);
  const int plane = in_height * in_width;
  if (pool_channel_dim >= 2 && pool_channel_dim <= 4 && plane > 0 && env_pool_direct()) {
    const int C = in_val_dim.cols / plane;
    if (in_val_dim.rows == 0) return 0;
    if (mode == 1 && out_val_dim.cols == (C - pool_channel_dim + 1) * plane &&
        in_val_dim.cols == C * plane) {
      const int64_t n = (int64_t)in_val_dim.rows * plane;
      const unsigned blocks = (unsigned)((n + 255) / 256);
#define KCNN_OVB(PC_)                                                                         \
  hipLaunchKernelGGL(maxpool_overlap_backprop_kernel<PC_>, dim3(blocks), dim3(256), 0, st,    \
                     in_val, (int64_t)in_val_dim.stride, out_val, (int64_t)out_val_dim.stride, \
                     out_deriv, (int64_t)out_deriv_dim.stride, dest, (int64_t)dest_dim.stride, \
                     in_val_dim.rows, plane, C, write_all)
      if (pool_channel_dim == 2) KCNN_OVB(2); else if (pool_channel_dim == 3) KCNN_OVB(3); else KCNN_OVB(4);
#undef KCNN_OVB
      return kcnn::launch_status();
    }
    if (mode == 2 && in_val_dim.cols == g.in_2d * g.in_2d * plane &&
        out_val_dim.cols == g.out_2d * g.out_2d * plane) {
      const int64_t n = (int64_t)in_val_dim.rows * plane * g.in_2d;
      const unsigned blocks = (unsigned)((n + 255) / 256);
#define KCNN_OV2B(PC_)                                                                        \
  hipLaunchKernelGGL(maxpool_overlap2d_backprop_kernel<PC_>, dim3(blocks), dim3(256), 0, st,  \
                     in_val, (int64_t)in_val_dim.stride, out_val, (int64_t)out_val_dim.stride, \
                     out_deriv, (int64_t)out_deriv_dim.stride, dest, (int64_t)dest_dim.stride, \
                     in_val_dim.rows, plane, g.out_2d, write_all)
      if (pool_channel_dim == 2) KCNN_OV2B(2); else if (pool_channel_dim == 3) KCNN_OV2B(3); else KCNN_OV2B(4);
#undef KCNN_OV2B
      return kcnn::launch_status();
    }
  }
  MaxpoolBackpropGather f{in_val, in_val_dim, out_val, out_val_dim, out_deriv,
                          out_deriv_dim, dest, dest_dim, g,
                          out_val_dim.cols / plane, write_all,
                          FastDiv((uint32_t)plane),
                          FastDiv((uint32_t)g.in_2d)};
  return launch_elem2d(in_val_dim.rows, in_val_dim.cols, f, st);
}

int hipF_momentum_update(float *W, MatrixDim W_dim, float *prev,
                         MatrixDim prev_dim, const float *grad,
                         MatrixDim grad_dim, float momentum, float a_wd,
                         float a_g, float *b, const float *grad_b, int b_dim,
                         kcnn_stream_t stream) {
  hipStream_t st = kcnn::as_stream(stream);
  MomentumUpdate f{W, W_dim, prev, prev_dim, grad, grad_dim, momentum, a_wd, a_g};
  const bool bias = b != nullptr && grad_b != nullptr && b_dim > 0;
  if (bias && b_dim <= W_dim.cols) {
    MomentumBiasUpdate fw{f, BiasUpdate{b, grad_b, a_g}, W_dim.rows, b_dim};
    return launch_elem2d(W_dim.rows + 1, W_dim.cols, fw, st);
  }
  int rc = launch_elem2d(W_dim.rows, W_dim.cols, f, st);
  if (rc == 0 && bias) {
    BiasUpdate fb{b, grad_b, a_g};
    rc = launch_elem2d(1, b_dim, fb, st);
  }
  return rc;
}

}  // extern "C"
