/*
 * oracle/kcnn_oracle.c -- see kcnn_oracle.h.  TEST INFRASTRUCTURE ONLY;
 * PARITY UNPINNED (the reference has no golden vectors and cannot be built
 * here; see DESIGN.md "Oracle").
 *
 * Each routine restates the CPU branch of the reference method named in its
 * comment.  Index arithmetic is written out with the reference's variable
 * meaning (row = sample, column = h + w*H + c*H*W) but element offsets are
 * computed in 64-bit (the reference's int32 overflows past 2^31).
 */
#include "kcnn_oracle.h"

#include <dlfcn.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int g_accum_mode = 0;
static int g_threads = 1;
static char g_err[512];

#define AT(m, r, c) ((m)->data[(int64_t)(r) * (m)->stride + (c)])

static int fail(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return -1;
}
#define CHECK(cond)                                             \
  do {                                                          \
    if (!(cond)) return fail("assertion failed: %s (%s:%d)", #cond, \
                             __func__, __LINE__);               \
  } while (0)

/* Optional CBLAS for the mode-0 GEMMs (the CPU-baseline timing only; the
 * parity tests keep the sequential-k loops below).  Upstream Kaldi's CPU
 * AddMatMat is cblas_sgemm (ATLAS / OpenBLAS / MKL); orc_use_blas binds the
 * OpenBLAS that numpy ships (64-bit-int interface, symbols scipy_*64_).     */
typedef void (*sgemm64_fn)(int order, int ta, int tb, int64_t m, int64_t n, int64_t k,
                           float alpha, const float *a, int64_t lda, const float *b,
                           int64_t ldb, float beta, float *c, int64_t ldc);
typedef void (*blas_threads_fn)(int64_t n);
static sgemm64_fn g_sgemm = NULL;
static blas_threads_fn g_blas_threads = NULL;

int orc_use_blas(const char *path) {
  if (!path) {
    g_sgemm = NULL;
    return 0;
  }
  void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail("dlopen %s: %s", path, dlerror());
  g_sgemm = (sgemm64_fn)dlsym(h, "scipy_cblas_sgemm64_");
  g_blas_threads = (blas_threads_fn)dlsym(h, "scipy_openblas_set_num_threads64_");
  if (!g_sgemm) return fail("%s has no scipy_cblas_sgemm64_", path);
  if (g_blas_threads) g_blas_threads(g_threads);
  return 0;
}
int orc_blas_active(void) { return g_sgemm != NULL; }

void orc_set_accum_mode(int mode) { g_accum_mode = mode; }
int orc_get_accum_mode(void) { return g_accum_mode; }
void orc_set_num_threads(int n) {
  g_threads = n < 1 ? 1 : n;
  if (g_blas_threads) g_blas_threads(g_threads);
}
int orc_num_threads(void) { return g_threads; }
const char *orc_last_error(void) { return g_err; }

static orc_mat mat_alloc(int rows, int cols) {
  orc_mat m;
  m.rows = rows;
  m.cols = cols;
  m.stride = cols;
  m.data = (float *)calloc((size_t)rows * (size_t)(cols > 0 ? cols : 1),
                           sizeof(float));
  return m;
}
static void mat_free(orc_mat *m) {
  free(m->data);
  m->data = NULL;
}

/* ------------------------------------------------------------------------ */
/* BLAS stand-in.  Kaldi's AddMatMat calls cuBLAS/CBLAS sgemm (upstream); the
 * summation order there is unspecified, so the oracle fixes the simplest one:
 * sequential in k.  Mode 1/2 accumulate in double (truth / error scale).    */
int orc_gemm(float alpha, const orc_mat *A, int transA, const orc_mat *B,
             int transB, float beta, orc_mat *C) {
  const int M = transA ? A->cols : A->rows;
  const int K = transA ? A->rows : A->cols;
  const int KB = transB ? B->cols : B->rows;
  const int N = transB ? B->rows : B->cols;
  CHECK(K == KB && C->rows == M && C->cols == N);
  const int mode = g_accum_mode;
  if (mode == 0 && g_sgemm) {
    if (M == 0 || N == 0) return 0;
    /* CblasRowMajor = 101, CblasNoTrans = 111, CblasTrans = 112 */
    g_sgemm(101, transA ? 112 : 111, transB ? 112 : 111, M, N, K, alpha, A->data,
            A->rows > 0 ? A->stride : 1, B->data, B->rows > 0 ? B->stride : 1, beta, C->data,
            C->stride);
    return 0;
  }
  if (mode == 0 && !transB) {
    /* i-k-j loop: per (i,j) still sequential in k, vectorises over j. */
    float *acc_all = NULL;
#pragma omp parallel num_threads(g_threads)
    {
      float *acc = (float *)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1));
#pragma omp for schedule(static)
      for (int i = 0; i < M; i++) {
        for (int j = 0; j < N; j++) acc[j] = 0.0f;
        for (int k = 0; k < K; k++) {
          const float a = transA ? AT(A, k, i) : AT(A, i, k);
          const float *brow = &B->data[(int64_t)k * B->stride];
          for (int j = 0; j < N; j++) acc[j] += a * brow[j];
        }
        float *crow = &C->data[(int64_t)i * C->stride];
        for (int j = 0; j < N; j++)
          crow[j] = alpha * acc[j] + (beta == 0.0f ? 0.0f : beta * crow[j]);
      }
      free(acc);
    }
    (void)acc_all;
    return 0;
  }
  if (!transB) {
    /* modes 1/2, i-k-j order with double accumulators (cache friendly). */
#pragma omp parallel num_threads(g_threads)
    {
      double *acc = (double *)malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
#pragma omp for schedule(static)
      for (int i = 0; i < M; i++) {
        for (int j = 0; j < N; j++) acc[j] = 0.0;
        for (int k = 0; k < K; k++) {
          const double a = transA ? AT(A, k, i) : AT(A, i, k);
          const float *brow = &B->data[(int64_t)k * B->stride];
          if (mode == 1) {
            for (int j = 0; j < N; j++) acc[j] += a * (double)brow[j];
          } else {
            const double aa = fabs(a);
            for (int j = 0; j < N; j++) acc[j] += aa * fabs((double)brow[j]);
          }
        }
        float *crow = &C->data[(int64_t)i * C->stride];
        for (int j = 0; j < N; j++) {
          if (mode == 1)
            crow[j] = (float)((double)alpha * acc[j] +
                              (beta == 0.0f ? 0.0 : (double)beta * crow[j]));
          else
            crow[j] = (float)(fabs((double)alpha) * acc[j] +
                              (beta == 0.0f ? 0.0 : fabs((double)beta * crow[j])));
        }
      }
      free(acc);
    }
    return 0;
  }
#pragma omp parallel for schedule(static) num_threads(g_threads)
  for (int i = 0; i < M; i++) {
    for (int j = 0; j < N; j++) {
      double dsum = 0.0;
      float fsum = 0.0f;
      for (int k = 0; k < K; k++) {
        const float a = transA ? AT(A, k, i) : AT(A, i, k);
        const float b = transB ? AT(B, j, k) : AT(B, k, j);
        if (mode == 0)
          fsum += a * b;
        else if (mode == 1)
          dsum += (double)a * (double)b;
        else
          dsum += fabs((double)a) * fabs((double)b);
      }
      float *c = &AT(C, i, j);
      if (mode == 0)
        *c = alpha * fsum + (beta == 0.0f ? 0.0f : beta * *c);
      else if (mode == 1)
        *c = (float)((double)alpha * dsum +
                     (beta == 0.0f ? 0.0 : (double)beta * (double)*c));
      else
        *c = (float)(fabs((double)alpha) * dsum +
                     (beta == 0.0f ? 0.0 : fabs((double)beta * (double)*c)));
    }
  }
  return 0;
}

/* Kaldi CuVectorBase::AddRowSumMat(alpha, M, beta): v = beta v + alpha * sum
 * over rows (upstream).  Sequential over rows in mode 0.                     */
static void add_row_sum_mat(float *v, float alpha, const orc_mat *M,
                            float beta) {
  const int mode = g_accum_mode;
  const int n = M->cols;
  /* Row-streaming; every column is still summed sequentially over rows. */
  float *f = (float *)calloc((size_t)(n > 0 ? n : 1), sizeof(float));
  double *d = (double *)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  for (int r = 0; r < M->rows; r++) {
    const float *row = &M->data[(int64_t)r * M->stride];
    if (mode == 0)
      for (int j = 0; j < n; j++) f[j] += row[j];
    else if (mode == 1)
      for (int j = 0; j < n; j++) d[j] += row[j];
    else
      for (int j = 0; j < n; j++) d[j] += fabs((double)row[j]);
  }
  for (int j = 0; j < n; j++) {
    if (mode == 0)
      v[j] = beta * v[j] + alpha * f[j];
    else if (mode == 1)
      v[j] = (float)((double)beta * v[j] + (double)alpha * d[j]);
    else
      v[j] = (float)(fabs((double)beta * v[j]) + fabs((double)alpha) * d[j]);
  }
  free(f);
  free(d);
}

/* ------------------------------------------------------------------------ */
/* CuMatrixBase::Conv2D, conv2D.cc:43-201.
 * 1) im2col of a row block ("spanThis", :120-133), 2) convMat_tmp = span *
 * kernel (:138-139, beta = 1 on a zeroed matrix), 3) copy into convMat
 * (:162-166), 4) concat ? col2im into out (:190-196) : out = convMat (:199).
 * The memory split loop (:65-93) is kept with the CPU budget of :69.        */
int orc_conv2d(const orc_mat *in, const orc_mat *kernel, int in_height,
               int in_width, int in_channel, int kernel_height,
               int kernel_width, int group, orc_mat *out, int concat) {
  CHECK(in->cols == in_height * in_width * in_channel);      /* :55 */
  CHECK(kernel->cols == group);                               /* :56 */
  CHECK(kernel->rows == kernel_height * kernel_width * in_channel); /* :57 */
  const int out_height = in_height - kernel_height + 1;       /* :59 */
  const int out_width = in_width - kernel_width + 1;          /* :60 */
  CHECK(out_height > 0 && out_width > 0);
  const int64_t span_height_org = (int64_t)out_height * out_width * in->rows;
  const int span_width = kernel_height * kernel_width * in_channel;
  if (concat) {
    CHECK(out->rows == in->rows && out->cols == out_height * out_width * group);
  } else {
    CHECK(out->rows == span_height_org && out->cols == group);
  }
  int64_t max_row = (int64_t)((0.5 * 1024 * 1024 * 1024) /
                              ((double)span_width * sizeof(float))); /* :69 */
  if (span_height_org <= max_row) max_row = span_height_org;        /* :77 */
  if (max_row < 1) max_row = 1;
  const int64_t split = span_height_org / max_row;                   /* :79 */

  orc_mat convMat = mat_alloc((int)span_height_org, group);          /* :81 */
  if (!convMat.data) return fail("oracle out of memory");
  const int kernelsize = kernel_height * kernel_width;
  const int q = in_height - kernel_height + 1;
  const int64_t in_rows = in->rows;

  for (int64_t split_idx = 0; split_idx < split + 1; split_idx++) {  /* :84 */
    const int64_t span_height = split_idx < split
                                    ? max_row
                                    : span_height_org - max_row * split;
    if (span_height == 0) break;                                     /* :93 */
    orc_mat span = mat_alloc((int)span_height, span_width);          /* :96 */
    if (!span.data) return fail("oracle out of memory");
    const int64_t row_offset = split_idx * max_row;                  /* :97 */
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int64_t i = 0; i < span_height; i++) {                      /* :120 */
      for (int j = 0; j < span_width; j++) {
        const int64_t i_offset = i + row_offset;
        const int64_t Ir = i_offset % in_rows;     /* sample             */
        const int64_t I = i_offset / in_rows;      /* output position    */
        const int Jr = j % kernelsize, J = j / kernelsize;
        const int64_t Q = I % q + I / q * in_height;
        const int P = (Jr % kernel_height) + (Jr / kernel_height) * in_height;
        AT(&span, i, j) =
            AT(in, Ir, Q + P + (int64_t)J * in_height * in_width);   /* :131 */
      }
    }
    orc_mat tmp = mat_alloc((int)span_height, group);                /* :138 */
    int rc = orc_gemm(1.0f, &span, 0, kernel, 0, 1.0f, &tmp);        /* :139 */
    mat_free(&span);
    if (rc) { mat_free(&tmp); mat_free(&convMat); return rc; }
    for (int64_t i = 0; i < span_height; i++)                        /* :162 */
      memcpy(&convMat.data[(i + row_offset) * convMat.stride],
             &tmp.data[i * tmp.stride], sizeof(float) * group);
    mat_free(&tmp);
  }
  if (concat) {                                                      /* :172 */
    const int64_t plane = (int64_t)out_height * out_width;
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (int64_t i = 0; i < span_height_org; i++) {                  /* :190 */
      for (int j = 0; j < group; j++) {
        const int64_t Ir = i % in_rows, I = i / in_rows;
        AT(out, Ir, I + j * plane) = AT(&convMat, i, j);             /* :194 */
      }
    }
  } else {
    for (int64_t i = 0; i < span_height_org; i++)                    /* :199 */
      memcpy(&out->data[i * out->stride], &convMat.data[i * convMat.stride],
             sizeof(float) * group);
  }
  mat_free(&convMat);
  return 0;
}

/* CuMatrixBase::AddMatRepVec, conv2D.cc:213-242 (CPU :231-240). */
int orc_add_mat_rep_vec(orc_mat *m, const float *vec, int vec_dim, int rep) {
  CHECK((int64_t)vec_dim * rep == m->cols);                          /* :216 */
  const int mode = g_accum_mode;
  for (int i = 0; i < m->rows; i++)
    for (int j = 0; j < m->cols; j++) {
      const int group = j / rep;
      if (mode == 2) AT(m, i, j) = fabsf(AT(m, i, j)) + fabsf(vec[group]);
      else AT(m, i, j) += vec[group];                                /* :237 */
    }
  return 0;
}

/* CuMatrixBase::FlipMat, conv2D.cc:244-287 (CPU :269-284): this is
 * [kh*kw*C x G], flip is [kh*kw*G x C]; flip(i, j) = this(p + j*ks, i/ks)
 * with p = (i/ks + 1)*ks - 1 - i.                                           */
int orc_flip_mat(const orc_mat *m, int kernel_height, int kernel_width,
                 int in_channel, int group, orc_mat *flip) {
  CHECK(m->rows == kernel_height * kernel_width * in_channel);       /* :247 */
  CHECK(flip->rows == kernel_height * kernel_width * group &&
        flip->cols == in_channel);                                   /* :251 */
  const int ksize = kernel_height * kernel_width;                    /* :270 */
  for (int i = 0; i < flip->rows; i++)
    for (int j = 0; j < flip->cols; j++) {
      const int group_idx = i / ksize;
      const int p = (group_idx + 1) * ksize - 1 - i;
      const int mm = p + j * ksize;
      AT(flip, i, j) = AT(m, mm, group_idx);                         /* :279 */
    }
  return 0;
}

/* CuMatrixBase::PaddingZero, conv2D.cc:289-344 (CPU :316-342): pads every
 * H x W map by (kernel-1) on each side.                                     */
int orc_padding_zero(const orc_mat *m, int orig_height, int orig_width,
                     int orig_channel, int kernel_height, int kernel_width,
                     orc_mat *padmat) {
  CHECK(m->cols == orig_height * orig_width * orig_channel);         /* :292 */
  const int ph = orig_height + 2 * (kernel_height - 1);              /* :295 */
  const int pw = orig_width + 2 * (kernel_width - 1);
  CHECK(padmat->rows == m->rows && padmat->cols == ph * pw * orig_channel);
  const int padmat_size = ph * pw;                                   /* :318 */
#pragma omp parallel for schedule(static) num_threads(g_threads)
  for (int i = 0; i < padmat->rows; i++)
    for (int j = 0; j < padmat->cols; j++) {
      const int chan_idx = j / padmat_size, p = j % padmat_size;
      const int I = p % ph, J = p / ph;
      if ((kernel_height - 1) <= I && I < (kernel_height + orig_height - 1) &&
          (kernel_width - 1) <= J && J < (kernel_width + orig_width - 1)) {
        const int mm = I - kernel_height + 1, n = J - kernel_width + 1;
        const int idx = (n * orig_height + mm) + chan_idx * (orig_height * orig_width);
        AT(padmat, i, j) = AT(m, i, idx);                            /* :334 */
      } else {
        AT(padmat, i, j) = 0.0f;                                     /* :337 */
      }
    }
  return 0;
}

/* CuMatrixBase::TpBlock, conv2D.cc:348-386 (CPU :375-385):
 * out[C x R*bs](i, j) = this(j / bs, i*bs + j % bs).                        */
int orc_tp_block(const orc_mat *m, int in_channel, int block_size,
                 orc_mat *out) {
  CHECK(m->cols == block_size * in_channel);                         /* :353 */
  CHECK(out->rows == in_channel &&
        out->cols == (int64_t)m->rows * block_size);                 /* :357 */
#pragma omp parallel for schedule(static) num_threads(g_threads)
  for (int i = 0; i < out->rows; i++)
    for (int j = 0; j < out->cols; j++) {
      const int row = j / block_size, col = i * block_size + j % block_size;
      AT(out, i, j) = AT(m, row, col);                               /* :382 */
    }
  return 0;
}

/* CuMatrixBase::TpInsideBlock, conv2D.cc:388-426 (CPU :415-425):
 * out[bs*R x G](i, j) = this(i / bs, j*bs + i % bs).                        */
int orc_tp_inside_block(const orc_mat *m, int group, int block_size,
                        orc_mat *out) {
  CHECK(m->cols == block_size * group);                              /* :393 */
  CHECK(out->rows == (int64_t)block_size * m->rows && out->cols == group);
#pragma omp parallel for schedule(static) num_threads(g_threads)
  for (int64_t i = 0; i < out->rows; i++)
    for (int j = 0; j < out->cols; j++) {
      const int64_t row = i / block_size;
      const int col = j * block_size + (int)(i % block_size);
      AT(out, i, j) = AT(m, row, col);                               /* :422 */
    }
  return 0;
}

/* CuMatrixBase::ModPermuteRow, conv2D.cc:429-463 (CPU :452-462):
 * out((i % C)*bs + i / C, j) = this(i, j).                                  */
int orc_mod_permute_row(const orc_mat *m, int in_channel, int block_size,
                        orc_mat *out) {
  CHECK(out->rows == m->rows && out->cols == m->cols);               /* :434 */
  for (int i = 0; i < out->rows; i++) {
    const int chan_idx = i % in_channel, pos_idx = i / in_channel;
    const int dst = chan_idx * block_size + pos_idx;
    CHECK(dst < out->rows);
    for (int j = 0; j < out->cols; j++) AT(out, dst, j) = AT(m, i, j); /* :459 */
  }
  return 0;
}

/* conv2D.cc:706-725 (CPU branch of ModPermuteChannel). */
int orc_mod_permute_channel(orc_mat *comp, int comp_idx, int num_component,
                            int in_height, int in_width, orc_mat *container,
                            int from_comp_to_container) {
  const int plane = in_height * in_width;
  for (int i = 0; i < comp->rows; i++) {
    for (int j = 0; j < comp->cols; j++) {
      const int chan_idx = j / plane, pos_idx = j % plane;
      const int out_chan_idx = chan_idx * num_component + comp_idx;
      const int oc = out_chan_idx * plane + pos_idx;
      CHECK(i < container->rows && oc < container->cols);
      if (from_comp_to_container) AT(container, i, oc) = AT(comp, i, j);
      else AT(comp, i, j) = AT(container, i, oc);
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Window enumeration shared by Maxpool_prop/backprop.  For output column j it
 * lists the input columns of its pooling window in the reference's loop
 * order (c, w, h).  Returns the count.                                       */
static int pool_window(int j, int out_cols, int in_height, int in_width,
                       int ph, int pw, int pc, int overlap, int overlap2D,
                       int64_t *idx) {
  const int out_height = in_height / ph, out_width = in_width / pw;
  int n = 0;
  if (overlap2D) {
    /* cnsl-cu-kernels.cu:418-446 (pool sizes are 1: out map == in map). */
    const int plane = in_height * in_width;
    const int out_channel = out_cols / plane;
    const int out_2d_map = (int)sqrt((double)out_channel);
    const int in_2d_map = out_2d_map + pc - 1;
    const int oc = j / plane, pos = j % plane;
    const int x = oc / out_2d_map, y = oc % out_2d_map;
    for (int cx = 0; cx < pc; cx++)
      for (int cy = 0; cy < pc; cy++) {
        const int ic = (x + cx) * in_2d_map + (y + cy);
        idx[n++] = (int64_t)ic * plane + pos;
      }
    return n;
  }
  const int oc = j / (out_height * out_width);                  /* :535 */
  const int pos = j % (out_height * out_width);
  const int wi = pos / out_height, hi = pos % out_height;
  int64_t start;
  if (overlap)                                                  /* :541 */
    start = (int64_t)oc * in_height * in_width + (int64_t)wi * pw * in_height +
            (int64_t)hi * ph;
  else                                                          /* :544 */
    start = (int64_t)oc * pc * in_height * in_width +
            (int64_t)wi * pw * in_height + (int64_t)hi * ph;
  for (int c = 0; c < pc; c++)                                  /* :547 */
    for (int w = 0; w < pw; w++)
      for (int h = 0; h < ph; h++)
        idx[n++] = start + h + (int64_t)w * in_height +
                   (int64_t)c * in_height * in_width;           /* :551 */
  return n;
}

/* CuMatrixBase::Maxpool_prop, conv2D.cc:465-559: pool(:, j) = -1e20, then
 * pool.Max(in(:, window)) one column at a time (:532-556); Kaldi's Max keeps
 * the running value unless it is < the candidate (NaN never wins).          */
int orc_maxpool_prop(const orc_mat *in, int in_height, int in_width,
                     int pool_height_dim, int pool_width_dim,
                     int pool_channel_dim, int overlap, int overlap2D,
                     orc_mat *out) {
  CHECK(out->rows == in->rows);
  CHECK(pool_height_dim > 0 && pool_width_dim > 0 && pool_channel_dim > 0);
  const int wmax = pool_height_dim * pool_width_dim * pool_channel_dim *
                   (overlap2D ? pool_channel_dim : 1);
  int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)wmax + 8);
  for (int j = 0; j < out->cols; j++) {                          /* :532 */
    const int n = pool_window(j, out->cols, in_height, in_width,
                              pool_height_dim, pool_width_dim,
                              pool_channel_dim, overlap, overlap2D, idx);
    for (int k = 0; k < n; k++) CHECK(idx[k] < in->cols);
    for (int r = 0; r < in->rows; r++) {
      float v = -1e20f;                                          /* :534 */
      for (int k = 0; k < n; k++) {
        const float x = AT(in, r, idx[k]);
        if (v < x) v = x;                                        /* :552 */
      }
      AT(out, r, j) = v;
    }
  }
  free(idx);
  return 0;
}

/* CuMatrixBase::Maxpool_backprop, conv2D.cc:565-684 (CPU :645-681). */
int orc_maxpool_backprop(const orc_mat *in_value, const orc_mat *out_value,
                         const orc_mat *out_deriv, orc_mat *in_deriv,
                         int in_height, int in_width, int pool_height_dim,
                         int pool_width_dim, int pool_channel_dim, int overlap,
                         int overlap2D) {
  CHECK(in_deriv->rows == in_value->rows && in_deriv->cols == in_value->cols);
  CHECK(out_deriv->rows == out_value->rows &&
        out_deriv->cols == out_value->cols);
  for (int r = 0; r < in_deriv->rows; r++)                       /* :889 */
    for (int c = 0; c < in_deriv->cols; c++) AT(in_deriv, r, c) = 0.0f;
  const int wmax = pool_height_dim * pool_width_dim * pool_channel_dim *
                   (overlap2D ? pool_channel_dim : 1);
  int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)wmax + 8);
  for (int j = 0; j < out_value->cols; j++) {                    /* :645 */
    const int n = pool_window(j, out_value->cols, in_height, in_width,
                              pool_height_dim, pool_width_dim,
                              pool_channel_dim, overlap, overlap2D, idx);
    for (int k = 0; k < n; k++) CHECK(idx[k] < in_value->cols);
    for (int r = 0; r < in_value->rows; r++) {
      const float o = AT(out_value, r, j);
      const float e = AT(out_deriv, r, j);
      for (int k = 0; k < n; k++)
        if (AT(in_value, r, idx[k]) == o)                        /* :673 */
          AT(in_deriv, r, idx[k]) += e;                          /* :675 */
    }
  }
  free(idx);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* ConvolutionComponent (nnet0/nnet-component-nnet0.cc).                      */

/* Propagate :423-446. */
int orc_conv_propagate(const orc_conv *c, const orc_mat *in, orc_mat *out) {
  int rc;
  if (c->in_pad_height > 0 || c->in_pad_width > 0) {             /* :430 */
    const int hh = c->in_height + 2 * c->in_pad_height;
    const int ww = c->in_width + 2 * c->in_pad_width;
    orc_mat padded = mat_alloc(in->rows, hh * ww * c->in_channel); /* :431 */
    rc = orc_padding_zero(in, c->in_height, c->in_width, c->in_channel,
                          c->in_pad_height + 1, c->in_pad_width + 1, &padded);
    if (!rc)
      rc = orc_conv2d(&padded, &c->W, hh, ww, c->in_channel, c->kernel_height,
                      c->kernel_width, c->group, out, 1);        /* :435 */
    mat_free(&padded);
  } else {
    rc = orc_conv2d(in, &c->W, c->in_height, c->in_width, c->in_channel,
                    c->kernel_height, c->kernel_width, c->group, out, 1);
  }
  if (rc) return rc;
  return orc_add_mat_rep_vec(out, c->b, c->group,
                             c->out_height * c->out_width);      /* :443 */
}

int orc_conv_flip_branch(const orc_conv *c) {
  /* :489-497 */
  const int pkh = c->kernel_height + 2 * (c->out_height - c->in_pad_height - 1);
  const int pkw = c->kernel_width + 2 * (c->out_width - c->in_pad_width - 1);
  const int poh = c->out_height + 2 * (c->kernel_height - c->in_pad_height - 1);
  const int pow_ = c->out_width + 2 * (c->kernel_width - c->in_pad_width - 1);
  return !((pkh * pkw) < (poh * pow_));
}

/* Backprop :461-544. */
int orc_conv_backprop(orc_conv *c, const orc_mat *in_value,
                      const orc_mat *out_deriv, orc_mat *in_deriv,
                      int do_update) {
  const int num_chunks = out_deriv->rows;                        /* :469 */
  const int kh = c->kernel_height, kw = c->kernel_width;
  const int oh = c->out_height, ow = c->out_width;
  const int C = c->in_channel, G = c->group;
  const int pkh = kh + 2 * (oh - c->in_pad_height - 1);          /* :489 */
  const int pkw = kw + 2 * (ow - c->in_pad_width - 1);
  const int poh = oh + 2 * (kh - c->in_pad_height - 1);          /* :492 */
  const int pow_ = ow + 2 * (kw - c->in_pad_width - 1);
  int rc = 0;
  CHECK(in_deriv->rows == num_chunks &&
        in_deriv->cols == c->in_height * c->in_width * C);
  if (!orc_conv_flip_branch(c)) {                                /* :499 */
    /* 1) TpInsideBlock(dY) 2) FlipMat -> flip_out_deriv [oh*ow*G x N]. */
    orc_mat flip_od = mat_alloc(oh * ow * G, num_chunks);        /* :501 */
    {
      orc_mat od_tp = mat_alloc(oh * ow * num_chunks, G);        /* :503 */
      rc = orc_tp_inside_block(out_deriv, G, oh * ow, &od_tp);   /* :505 */
      if (!rc) rc = orc_flip_mat(&od_tp, oh, ow, num_chunks, G, &flip_od); /* :507 */
      mat_free(&od_tp);
    }
    orc_mat pad_kernel = mat_alloc(C, pkh * pkw * G);            /* :510 */
    if (!rc) {
      orc_mat wt = mat_alloc(G, kh * kw * C);                    /* :513 */
      orc_mat wt2 = mat_alloc(C, kh * kw * G);                   /* :514 */
      for (int i = 0; i < G; i++)                                /* :516 AddMat kTrans */
        for (int j = 0; j < kh * kw * C; j++) AT(&wt, i, j) += 1.0f * AT(&c->W, j, i);
      rc = orc_tp_block(&wt, C, kh * kw, &wt2);                  /* :517 */
      if (!rc)
        rc = orc_padding_zero(&wt2, kh, kw, G, oh - c->in_pad_height,
                              ow - c->in_pad_width, &pad_kernel); /* :519 */
      mat_free(&wt);
      mat_free(&wt2);
    }
    if (!rc) {
      orc_mat tmp = mat_alloc(C, c->in_height * c->in_width * num_chunks); /* :522 */
      rc = orc_conv2d(&pad_kernel, &flip_od, pkh, pkw, G, oh, ow, num_chunks,
                      &tmp, 1);                                  /* :524 */
      if (!rc) rc = orc_tp_block(&tmp, num_chunks,
                                 c->in_height * c->in_width, in_deriv); /* :525 */
      mat_free(&tmp);
    }
    mat_free(&pad_kernel);
    mat_free(&flip_od);
  } else {
    orc_mat pad_od = mat_alloc(num_chunks, poh * pow_ * G);      /* :530 */
    orc_mat flipk = mat_alloc(kh * kw * G, C);                   /* :531 */
    rc = orc_padding_zero(out_deriv, oh, ow, G, kh - c->in_pad_height,
                          kw - c->in_pad_width, &pad_od);        /* :534 */
    if (!rc) rc = orc_flip_mat(&c->W, kh, kw, C, G, &flipk);     /* :536 */
    if (!rc)
      rc = orc_conv2d(&pad_od, &flipk, poh, pow_, G, kh, kw, C, in_deriv, 1); /* :538 */
    mat_free(&pad_od);
    mat_free(&flipk);
  }
  if (rc) return rc;
  if (do_update) {                                               /* :541 */
    orc_mat gW = mat_alloc(kh * kw * C, G);
    float *gb = (float *)calloc((size_t)G, sizeof(float));
    rc = orc_conv_gradient(c, in_value, out_deriv, &gW, gb);
    if (!rc) rc = orc_conv_apply(c, &gW, gb, in_value->rows);
    mat_free(&gW);
    free(gb);
  }
  return rc;
}

/* Update :738-765 (gradient part): TpBlock(X) (:754/:757), TpInsideBlock(dY)
 * (:760), Conv2D(concat=false) (:763), ModPermuteRow (:765); bias gradient
 * is the row sum of out_deriv_tmp (:775).                                   */
int orc_conv_gradient(const orc_conv *c, const orc_mat *in_value,
                      const orc_mat *out_deriv, orc_mat *grad_W,
                      float *grad_b) {
  const int num_sample = in_value->rows;                         /* :741 */
  const int H = c->in_height + 2 * c->in_pad_height;             /* :742 */
  const int W = c->in_width + 2 * c->in_pad_width;
  const int C = c->in_channel, G = c->group;
  const int kk = c->kernel_height * c->kernel_width;
  const int P = c->out_height * c->out_width;
  int rc;
  CHECK(grad_W->rows == kk * C && grad_W->cols == G);
  orc_mat xt = mat_alloc(C, num_sample * H * W);                 /* :745 */
  orc_mat odt = mat_alloc(P * num_sample, G);                    /* :746 */
  orc_mat lpt = mat_alloc(kk * C, G);                            /* :748 */
  if (c->in_pad_height > 0 || c->in_pad_width > 0) {             /* :751 */
    orc_mat padded = mat_alloc(num_sample, H * W * C);
    rc = orc_padding_zero(in_value, c->in_height, c->in_width, C,
                          c->in_pad_height + 1, c->in_pad_width + 1, &padded);
    if (!rc) rc = orc_tp_block(&padded, C, H * W, &xt);          /* :754 */
    mat_free(&padded);
  } else {
    rc = orc_tp_block(in_value, C, H * W, &xt);                  /* :757 */
  }
  if (!rc) rc = orc_tp_inside_block(out_deriv, G, P, &odt);      /* :760 */
  if (!rc)
    rc = orc_conv2d(&xt, &odt, H, W, num_sample, c->out_height, c->out_width,
                    G, &lpt, 0);                                 /* :763 */
  if (!rc) rc = orc_mod_permute_row(&lpt, C, kk, grad_W);        /* :765 */
  if (!rc) {
    for (int j = 0; j < G; j++) grad_b[j] = 0.0f;
    add_row_sum_mat(grad_b, 1.0f, &odt, 0.0f);                   /* :775 */
  }
  mat_free(&xt);
  mat_free(&odt);
  mat_free(&lpt);
  return rc;
}

/* Update :767-775 (apply part). learning_rate is a double (:767) that
 * reaches Kaldi's float AddMat/AddRowSumMat alphas as floats.               */
int orc_conv_apply(orc_conv *c, const orc_mat *grad_W, const float *grad_b,
                   int num_sample) {
  const double lr = (double)c->learning_rate / num_sample;       /* :767 */
  const float a_wd = (float)(-1 * lr * c->weight_decay);
  const float a_g = (float)lr;
  for (int i = 0; i < c->W.rows; i++)
    for (int j = 0; j < c->W.cols; j++) {
      float p = AT(&c->prev, i, j) * c->momentum;                /* :769 */
      p += a_wd * AT(&c->W, i, j);                               /* :770 */
      p += a_g * AT(grad_W, i, j);                               /* :771 */
      AT(&c->prev, i, j) = p;
      AT(&c->W, i, j) += 1.0f * p;                               /* :772 */
    }
  for (int j = 0; j < c->group; j++)                             /* :775 */
    c->b[j] = 1.0f * c->b[j] + a_g * grad_b[j];
  return 0;
}

/* MaxpoolComponent::InitFromString output_dim, :835-847. */
int orc_pool_output_dim(const orc_pool *p) {
  const int input_dim = p->in_height * p->in_width * p->in_channel;
  if (p->overlap2D) {
    const int oc = (int)pow(sqrt((double)p->in_channel) - p->pool_channel_dim + 1, 2);
    return input_dim / p->in_channel * oc;
  }
  if (p->overlap)
    return input_dim / p->in_channel * (p->in_channel - p->pool_channel_dim + 1);
  return input_dim / (p->pool_height_dim * p->pool_width_dim * p->pool_channel_dim);
}

/* ------------------------------------------------------------------------ */
/* FullyConnectedComponent: AffineComponent::Propagate
 * (nnet2/nnet-component.cc:1216-1228): out = bias rows, out += in W^T.      */
int orc_fc_propagate(const orc_fc *f, const orc_mat *in, orc_mat *out) {
  CHECK(in->cols == f->input_dim && out->cols == f->output_dim &&
        out->rows == in->rows);
  const int mode = g_accum_mode;
  for (int r = 0; r < out->rows; r++)                           /* :1225 */
    for (int j = 0; j < out->cols; j++)
      AT(out, r, j) = mode == 2 ? fabsf(f->b[j]) : f->b[j];
  return orc_gemm(1.0f, in, 0, &f->W, 1, 1.0f, out);            /* :1227 */
}

/* AffineComponent::Backprop (nnet-component.cc:1237-1258). */
int orc_fc_backprop(orc_fc *f, const orc_mat *in_value,
                    const orc_mat *out_deriv, orc_mat *in_deriv,
                    int do_update) {
  CHECK(in_deriv->rows == out_deriv->rows && in_deriv->cols == f->input_dim);
  int rc = orc_gemm(1.0f, out_deriv, 0, &f->W, 0, 0.0f, in_deriv); /* :1247 */
  if (rc || !do_update) return rc;
  orc_mat gW = mat_alloc(f->output_dim, f->input_dim);
  float *gb = (float *)calloc((size_t)f->output_dim, sizeof(float));
  rc = orc_fc_gradient(f, in_value, out_deriv, &gW, gb);
  if (!rc) rc = orc_fc_apply(f, &gW, gb, in_value->rows);
  mat_free(&gW);
  free(gb);
  return rc;
}

/* UpdateSimple (nnet-component-nnet0.cc:1133-1150), gradient part:
 * dY^T X (:1141) and the bias row sum (:1137).                              */
int orc_fc_gradient(const orc_fc *f, const orc_mat *in_value,
                    const orc_mat *out_deriv, orc_mat *grad_W, float *grad_b) {
  CHECK(grad_W->rows == f->output_dim && grad_W->cols == f->input_dim);
  for (int j = 0; j < f->output_dim; j++) grad_b[j] = 0.0f;
  add_row_sum_mat(grad_b, 1.0f, out_deriv, 0.0f);
  return orc_gemm(1.0f, out_deriv, 1, in_value, 0, 0.0f, grad_W);
}

/* UpdateSimple apply part.  Order of the reference: bias first (:1137),
 * then prev = m prev - lr wd W + lr gW (:1139-1141), W += prev (:1142).     */
int orc_fc_apply(orc_fc *f, const orc_mat *grad_W, const float *grad_b,
                 int num_sample) {
  const double lr = (double)f->learning_rate / num_sample;       /* :1136 */
  const float a_wd = (float)(-1 * lr * f->weight_decay);
  const float a_g = (float)lr;
  for (int j = 0; j < f->output_dim; j++)
    f->b[j] = 1.0f * f->b[j] + a_g * grad_b[j];                  /* :1137 */
  for (int i = 0; i < f->W.rows; i++)
    for (int j = 0; j < f->W.cols; j++) {
      float p = AT(&f->prev, i, j) * f->momentum;                /* :1139 */
      p += a_wd * AT(&f->W, i, j);                               /* :1140 */
      p += a_g * AT(grad_W, i, j);                               /* :1141 */
      AT(&f->prev, i, j) = p;
      AT(&f->W, i, j) += 1.0f * p;                               /* :1142 */
    }
  return 0;
}

/* ===========================================================================
 * RectifiedLinearComponent (nnet2/nnet-component.cc:799-827)
 * ======================================================================== */
int orc_relu_propagate(const orc_mat *in, orc_mat *out) {
  CHECK(in->rows == out->rows && in->cols == out->cols);
  for (int i = 0; i < in->rows; i++)
    for (int j = 0; j < in->cols; j++) {
      float v = AT(in, i, j);          /* CopyFromMat :804 */
      if (v < 0.0f) v = 0.0f;          /* ApplyFloor(0.0) :805 */
      AT(out, i, j) = v;
    }
  return 0;
}

int orc_relu_backprop(const orc_mat *out_value, const orc_mat *out_deriv,
                      orc_mat *in_deriv, double *value_sum, double *deriv_sum,
                      double *count) {
  CHECK(out_value->rows == out_deriv->rows && out_value->cols == out_deriv->cols);
  CHECK(in_deriv->rows == out_deriv->rows && in_deriv->cols == out_deriv->cols);
  const int R = out_value->rows, C = out_value->cols;
  for (int i = 0; i < R; i++)          /* CopyFromMat + ApplyHeaviside :817-818 */
    for (int j = 0; j < C; j++)
      AT(in_deriv, i, j) = AT(out_value, i, j) > 0.0f ? 1.0f : 0.0f;
  if (value_sum) {                     /* UpdateStats :822 -> :337-363 */
    *count += R;
    for (int j = 0; j < C; j++) {
      float tv = 0.0f, td = 0.0f;      /* CuVector<BaseFloat> temp; AddRowSumMat */
      for (int i = 0; i < R; i++) {
        tv += AT(out_value, i, j);
        td += AT(in_deriv, i, j);
      }
      value_sum[j] += (double)tv;      /* value_sum_.AddVec(1.0, temp) */
      deriv_sum[j] += (double)td;
    }
  }
  for (int i = 0; i < R; i++)          /* MulElements(out_deriv) :826 */
    for (int j = 0; j < C; j++) AT(in_deriv, i, j) *= AT(out_deriv, i, j);
  return 0;
}

/* ===========================================================================
 * SpliceComponent (nnet2/nnet-component.cc:2638-2819), contiguous chunks:
 * GetOffset(i) = first + i, GetIndex(o) = o - first (asserted in range).
 * ======================================================================== */
/* ChunkInfo::GetIndex over an explicit offset list (nnet-component.h
 * ChunkInfo; upstream nnet2's offsets_ vector): -1 when absent */
static int chunk_index(const int *offsets, int n, int offset) {
  for (int i = 0; i < n; i++)
    if (offsets[i] == offset) return i;
  return -1;
}

/* SpliceComponent::Propagate (nnet-component.cc:2638-2720) with the chunk
 * offsets as lists (in_offsets[in_cs], out_offsets[out_cs], ascending; the
 * rows of a chunk in that order): out row (chunk, oi), splice block c copies
 * in row (chunk, GetIndex(out_offsets[oi] + context[c])) (:2674-2681); the
 * const part copies in row (chunk, oi) (:2692-2698) */
int orc_splice_propagate_offsets(const orc_mat *in, orc_mat *out, int num_chunks,
                                 const int *in_offsets, int in_cs, const int *out_offsets,
                                 int out_cs, const int *context, int num_splice,
                                 int const_dim) {
  const int input_dim = in->cols, dim = input_dim - const_dim;
  CHECK(in->rows == num_chunks * in_cs && out->rows == num_chunks * out_cs);
  CHECK(out->cols == dim * num_splice + const_dim);
  for (int c = 0; c < num_splice; c++)                     /* :2697-2705 */
    for (int oi = 0; oi < out_cs; oi++) {
      const int ii = chunk_index(in_offsets, in_cs, out_offsets[oi] + context[c]);
      CHECK(ii >= 0);                                      /* GetIndex: KALDI_ERR */
      for (int chunk = 0; chunk < num_chunks; chunk++)
        for (int d = 0; d < dim; d++)
          AT(out, chunk * out_cs + oi, c * dim + d) = AT(in, chunk * in_cs + ii, d);
    }
  if (const_dim != 0)                                      /* :2706-2713 */
    for (int chunk = 0; chunk < num_chunks; chunk++)
      for (int oi = 0; oi < out_cs; oi++)
        for (int d = 0; d < const_dim; d++)
          AT(out, chunk * out_cs + oi, num_splice * dim + d) =
              AT(in, chunk * in_cs + oi, dim + d);
  return 0;
}

/* SpliceComponent::Backprop (nnet-component.cc:2723-2819), offsets as lists:
 * per splice block c the in_deriv rows are CopyRows of the out_deriv row
 * that read them (-1: zero), c = 0 copied, later blocks added (AddMat) */
int orc_splice_backprop_offsets(const orc_mat *out_deriv, orc_mat *in_deriv, int num_chunks,
                                const int *in_offsets, int in_cs, const int *out_offsets,
                                int out_cs, const int *context, int num_splice,
                                int const_dim) {
  const int input_dim = in_deriv->cols, dim = input_dim - const_dim;
  CHECK(in_deriv->rows == num_chunks * in_cs && out_deriv->rows == num_chunks * out_cs);
  CHECK(out_deriv->cols == dim * num_splice + const_dim);
  const int R = in_deriv->rows;
  int *idx = (int *)malloc(sizeof(int) * (size_t)R);
  float *temp = (float *)malloc(sizeof(float) * (size_t)R * (dim > 0 ? dim : 1));
  if (!idx || !temp) { free(idx); free(temp); return -1; }
  for (int c = 0; c < num_splice; c++) {
    for (int r = 0; r < R; r++) idx[r] = -1;               /* :2757-2759 */
    for (int oi = 0; oi < out_cs; oi++) {
      const int ii = chunk_index(in_offsets, in_cs, out_offsets[oi] + context[c]);
      if (ii < 0) { free(idx); free(temp); return -1; }
      for (int chunk = 0; chunk < num_chunks; chunk++)
        idx[chunk * in_cs + ii] = chunk * out_cs + oi;     /* :2766-2781 */
    }
    for (int r = 0; r < R; r++)                            /* CopyRows :2804/2806 */
      for (int d = 0; d < dim; d++)
        temp[(size_t)r * dim + d] = idx[r] < 0 ? 0.0f : AT(out_deriv, idx[r], c * dim + d);
    for (int r = 0; r < R; r++)
      for (int d = 0; d < dim; d++) {
        if (c == 0) AT(in_deriv, r, d) = temp[(size_t)r * dim + d];
        else AT(in_deriv, r, d) += 1.0f * temp[(size_t)r * dim + d];  /* AddMat :2807 */
      }
  }
  if (const_dim != 0) {                                    /* :2810-2818 */
    for (int r = 0; r < R; r++) idx[r] = -1;
    for (int chunk = 0; chunk < num_chunks; chunk++)
      for (int oi = 0; oi < out_cs; oi++) idx[chunk * in_cs + oi] = chunk * out_cs + oi;
    for (int r = 0; r < R; r++)
      for (int d = 0; d < const_dim; d++)
        AT(in_deriv, r, dim + d) =
            idx[r] < 0 ? 0.0f : AT(out_deriv, idx[r], num_splice * dim + d);
  }
  free(idx);
  free(temp);
  return 0;
}

/* contiguous chunks: offsets in_first + [0, in_cs), out_first + [0, out_cs) */
static int *range_offsets(int first, int n) {
  int *o = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  if (o)
    for (int i = 0; i < n; i++) o[i] = first + i;
  return o;
}

int orc_splice_propagate(const orc_mat *in, orc_mat *out, int num_chunks, int in_first,
                         int in_cs, int out_first, int out_cs, const int *context,
                         int num_splice, int const_dim) {
  int *io = range_offsets(in_first, in_cs), *oo = range_offsets(out_first, out_cs);
  const int rc = io && oo ? orc_splice_propagate_offsets(in, out, num_chunks, io, in_cs, oo,
                                                         out_cs, context, num_splice, const_dim)
                          : -1;
  free(io);
  free(oo);
  return rc;
}

int orc_splice_backprop(const orc_mat *out_deriv, orc_mat *in_deriv, int num_chunks,
                        int in_first, int in_cs, int out_first, int out_cs,
                        const int *context, int num_splice, int const_dim) {
  int *io = range_offsets(in_first, in_cs), *oo = range_offsets(out_first, out_cs);
  const int rc = io && oo ? orc_splice_backprop_offsets(out_deriv, in_deriv, num_chunks, io,
                                                        in_cs, oo, out_cs, context,
                                                        num_splice, const_dim)
                          : -1;
  free(io);
  free(oo);
  return rc;
}
