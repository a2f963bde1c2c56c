// cnslmat/conv-geom.h -- geometry shared by the convolution kernels.
#ifndef KCNN_CNSLMAT_CONV_GEOM_H_
#define KCNN_CNSLMAT_CONV_GEOM_H_

#include "hip-util.h"
#include "pool-stats.h"

namespace kcnn {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// One convolution instance: R rows (frames) of H x W x C maps (column
// h + w*H + c*H*W), virtual zero padding (pad_h, pad_w), kernel kh x kw,
// G output maps of oh x ow (p = px*oh + py).
struct ConvGeom {
  int R, H, W, C, pad_h, pad_w, kh, kw, G, oh, ow, P, Kdim, HW;
  int Gtot;   // the layer's filter count (G is one chunk's when a launch splits G)
  int64_t M;  // R * P
  FastDiv div_P, div_oh, div_khkw, div_kh, div_H, div_HW;
};

inline ConvGeom make_geom(int R, int H, int W, int C, int pad_h, int pad_w,
                          int kh, int kw, int G) {
  ConvGeom g;
  g.R = R; g.H = H; g.W = W; g.C = C; g.pad_h = pad_h; g.pad_w = pad_w;
  g.kh = kh; g.kw = kw; g.G = G; g.Gtot = G;
  g.oh = H + 2 * pad_h - kh + 1;
  g.ow = W + 2 * pad_w - kw + 1;
  g.P = g.oh * g.ow;
  g.Kdim = kh * kw * C;
  g.HW = H * W;
  g.M = (int64_t)R * g.P;
  g.div_P = FastDiv((uint32_t)(g.P > 0 ? g.P : 1));
  g.div_oh = FastDiv((uint32_t)(g.oh > 0 ? g.oh : 1));
  g.div_khkw = FastDiv((uint32_t)(kh * kw > 0 ? kh * kw : 1));
  g.div_kh = FastDiv((uint32_t)(kh > 0 ? kh : 1));
  g.div_H = FastDiv((uint32_t)(H > 0 ? H : 1));
  g.div_HW = FastDiv((uint32_t)(g.HW > 0 ? g.HW : 1));
  return g;
}

// MFMA 32x32 accumulator register r of lane l holds row
// (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31.
__device__ __forceinline__ int mfma32_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

}  // namespace kcnn

// Frame-resident kernels (cnsl-conv-frame.hip).  Each returns -1 when the
// shape is not eligible (caller falls back to the implicit-GEMM path).
int kcnn_conv_fwd_frame(const kcnn::ConvGeom &g, const float *X, int xs,
                        const float *K, int ks, const float *bias, float *out,
                        int os, hipStream_t st);
// the pooled output's statistics: pool-stats.h
size_t kcnn_pool_stats_partial_words(const kcnn::ConvGeom &g, int pc);
int kcnn_conv_fwd_frame_pool(const kcnn::ConvGeom &g, const float *X, int xs,
                             const float *K, int ks, const float *bias,
                             float *out, int os, float *pool, int ps,
                             unsigned char *mask, int ms, int pc,
                             hipStream_t st, int ph = 1, int pw = 1,
                             PoolStatsOut *stats = nullptr);
int kcnn_conv_dgrad_frame(const kcnn::ConvGeom &g, const float *dY, int dys,
                          const float *K, int ks, float *dX, int dxs,
                          hipStream_t st);
// Fused backward (one pass over dY): dX (nullable) and gW/gb.  ws must hold
// kcnn_conv_bwd_frame_ws(g) bytes (0 = shape not eligible).
size_t kcnn_conv_bwd_frame_ws(const kcnn::ConvGeom &g);
// pc > 0: dY / dys are instead the derivative of a ph x 1 x pc Maxpool over
// Y and pmask / pms its routing mask (hipF_conv2d_maxpool[3d]: 1 byte per
// pooled value when ph == 1, else 2; pms in bytes); dY is built per slab in
// LDS and never stored.  ph > 1 runs on the bf16x6 kernel only.
int kcnn_conv_bwd_frame(const kcnn::ConvGeom &g, const float *X, int xs,
                        const float *dY, int dys, const float *K, int ks,
                        float *dX, int dxs, float *gW, int gws, float *gb,
                        void *ws, size_t ws_bytes, hipStream_t st,
                        const unsigned char *pmask = nullptr, int pms = 0,
                        int pc = 0, int ph = 1);
// The same fused backward on the bf16 MFMAs with exact three-way operand
// splits (cnsl-conv-x6.hip); ws_part == NULL runs the data gradient only.
bool kcnn_conv_bwd_x6_eligible(const kcnn::ConvGeom &g, bool dx, int pc, int ph = 1);
int kcnn_conv_bwd_x6(const kcnn::ConvGeom &g, const float *X, int xs, const float *dY,
                     int dys, const float *K, int ks, float *dX, int dxs, float *ws_part,
                     int S, int dx_acc, hipStream_t st, const unsigned char *pmask,
                     int pms, int pc, int ph, int dbg = 0);
// Conv2D(concat) + bias (+ ReLU when relu) as an implicit GEMM on the f16
// (f16x3, igemm_x6 family 2 / 3) or bf16 (bf16x6) MFMAs
// (cnsl-conv-igemm-x6.hip); -1 when the shape is outside its limits.
int kcnn_conv_igemm_x6(const kcnn::ConvGeom &g, const float *X, int xs, const float *K,
                       int ks, const float *bias, float *out, int os, int relu,
                       hipStream_t st);
// kcnn_conv_igemm_x6 with a ph x pw x pc Maxpool of two-position windows in
// its epilogue (pooled output and 16-bit routing mask); -1 when not covered.
int kcnn_conv_igemm_x6_pool(const kcnn::ConvGeom &g, const float *X, int xs, const float *K,
                            int ks, const float *bias, float *out, int os, float *pool,
                            int ps, unsigned short *mask, int ms, int ph, int pw, int pc,
                            hipStream_t st);
// Weight gradient on the bf16 MFMAs (cnsl-conv-igemm-x6.hip): the split
// plan (false = not eligible), then partials [S][G*Kdim + G] into ws for
// kcnn_reduce_splits_wgrad.
bool kcnn_conv_wgrad_x6_plan(const kcnn::ConvGeom &g, int xs, int dys, int &S, int &fps,
                             size_t &ws_bytes);
int kcnn_conv_wgrad_x6(const kcnn::ConvGeom &g, const float *X, int xs, const float *dY,
                       int dys, float *ws, int S, int fps, hipStream_t st);
size_t kcnn_conv_wgrad_frame_ws(const kcnn::ConvGeom &g);
int kcnn_conv_wgrad_frame(const kcnn::ConvGeom &g, const float *X, int xs,
                          const float *dY, int dys, float *gW, int gws,
                          float *gb, void *ws, size_t ws_bytes, hipStream_t st);
// Deterministic column sums of a [S x E] fp32 slab, out[e] = sum_s in[s][e]
// in a fixed order: pass 1 sums groups of 32 rows into tmp [ceil(S/32) x E],
// pass 2 sums the groups (cnsl-conv-frame.hip).
size_t kcnn_reduce_splits_ws(int S, int E);
int kcnn_reduce_splits(const float *in, int S, int E, float *tmp, float *out,
                       hipStream_t st);
int kcnn_reduce_splits_pass1(const float *in, int S, int E, float *tmp,
                             hipStream_t st);
// pass 2 into the implicit-GEMM wgrad layout: e = g*inner + k (e < nw) ->
// gW[k][g]; e >= nw -> gb[e - nw].
int kcnn_reduce_splits_wgrad(const float *in, int S, int E, float *tmp, int nw,
                             int inner, float *gW, int gws, float *gb,
                             hipStream_t st);

#endif  // KCNN_CNSLMAT_CONV_GEOM_H_
