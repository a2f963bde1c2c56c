// cnslmat/cnsl-conv-frame.hip -- frame-resident convolution kernels for
// layers with a small kernel volume (K = kh*kw*C <= 32, e.g. the fbank input
// layer of BASELINE c2: 8x1x3 = 24), where the contraction is too thin to
// feed MFMA from an im2col tile and the layer is HBM-bound.
//
// One workgroup walks frames (grid-stride over rows); per frame:
//   forward  Y[g][p] = sum_k W[k][g] X[c][p + off_k]
//            the frame's X map (5.3 KB) is staged in LDS, W in LDS; MFMA
//            32x32x2 with g on the accumulator rows and p on the lanes, so
//            each store writes two 128-B runs of Y; bias fused.
//   dgrad    Z[p][k] = sum_g dY[g][p] W[k][g]   (a plain GEMM: K = G, N = K)
//            with dY read straight from HBM as the MFMA A operand (lanes along
//            p: coalesced, no LDS), Z kept in LDS, then the col2im
//            dX[c][q] = sum_taps Z[q - tap][tap, c] from LDS.  No padded dY,
//            no flipped kernel, no im2col matrix (the reference's flip branch
//            moves ~30x the bytes).
//   wgrad    gW[k][g] = sum_{n,p} X[c][p + off_k] dY[g][p]; each wave owns a
//            32-wide g block, stages its dY tile through LDS (transpose), and
//            gathers the im2col operand from the LDS-resident X map.  Row
//            K of the A operand is all ones, so the bias gradient sum_p dY
//            falls out of the same MFMAs.  Per-workgroup partials are reduced
//            in a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include "conv-geom.h"

using namespace kcnn;

namespace {

constexpr int kFrameLdsMax = 96 * 1024;
constexpr int ZS = 33;  // padded row stride (floats) of the LDS Z / dY tiles

__host__ __device__ inline int align16(int bytes) { return (bytes + 15) & ~15; }

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

// ---------------------------------------------------------------------------
template <int NGB>
__global__ __launch_bounds__(256) void conv_fwd_frame_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ K, int ks, const float *__restrict__ bias,
    float *__restrict__ out, int os, int Kpad, int Gp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int2 *koff = reinterpret_cast<int2 *>(smem);
  float *Ws = reinterpret_cast<float *>(smem + align16(Kpad * 8));
  float *Xs = Ws + Kpad * Gp;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  for (int e = tid; e < Kpad * Gp; e += 256) {
    const int k = e / Gp, gg = e - k * Gp;
    Ws[e] = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
  }
  for (int k = tid; k < Kpad; k += 256) {
    int2 v = make_int2(0, 0x7fff << 16);  // padded tap: never in bounds
    if (k < g.Kdim) {
      uint32_t c, r, kx, ky;
      g.div_khkw.divmod((uint32_t)k, c, r);
      g.div_kh.divmod(r, kx, ky);
      v = make_int2((int)c * g.HW, (int)((kx << 16) | ky));
    }
    koff[k] = v;
  }
  const int CHW = g.C * g.HW;
  const int ntile = (g.P + 31) >> 5;
  const int ksteps = Kpad >> 1;

  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();
    const float *xr = X + (int64_t)n * xs;
    for (int e = tid; e < CHW; e += 256) Xs[e] = xr[e];
    __syncthreads();
    for (int pt = wave; pt < ntile; pt += 4) {
      const int p = pt * 32 + (lane & 31);
      const bool pv = p < g.P;
      uint32_t px = 0, py = 0;
      if (pv) g.div_oh.divmod((uint32_t)p, px, py);
      for (int gs = 0; gs < Gp; gs += 32 * NGB) {  // Gp: multiple of 32*NGB
        floatx16 acc[NGB];
#pragma unroll
        for (int b = 0; b < NGB; b++) acc[b] = zero16();
        for (int s = 0; s < ksteps; s++) {
          const int k = 2 * s + (lane >> 5);
          // branch-free gather: padded taps (k >= Kdim) carry zero weights,
          // invalid positions / padding read a clamped address and are
          // zeroed by a select (no exec-masked regions around the MFMAs).
          const int2 ko = koff[k];
          const int xx = (int)px + (ko.y >> 16) - g.pad_w;
          const int yy = (int)py + (ko.y & 0xffff) - g.pad_h;
          const bool ok = pv && (unsigned)xx < (unsigned)g.W &&
                          (unsigned)yy < (unsigned)g.H;
          const float xv = Xs[ok ? ko.x + xx * g.H + yy : 0];
          const float bv = ok ? xv : 0.0f;
          const float *wrow = Ws + k * Gp + gs + (lane & 31);
#pragma unroll
          for (int b = 0; b < NGB; b++)
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(wrow[b * 32], bv, acc[b], 0, 0, 0);
        }
        if (pv) {
          float *orow = out + (int64_t)n * os + p;
#pragma unroll
          for (int b = 0; b < NGB; b++) {
#pragma unroll
            for (int r = 0; r < 16; r++) {
              const int gg = gs + b * 32 + mfma32_row(r, lane);
              if (gg < g.G) {
                float v = acc[b][r];
                if (bias) v = v + bias[gg];
                orow[(int64_t)gg * g.P] = v;
              }
            }
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// NK = G/2 k-steps, fully unrolled: every A load of a 32-position tile is
// issued before the MFMA chain consumes it (64 x 256 B in flight per wave at
// G = 128), which is what hides HBM latency here.  Lanes past the last
// position read a clamped address; their Z rows are never stored.
template <int NK>
__global__ __launch_bounds__(256) void conv_dgrad_frame_kernel(
    ConvGeom g, const float *__restrict__ dY, int dys,
    const float *__restrict__ K, int ks, float *__restrict__ dX, int dxs,
    int ZZ) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float *Wt = reinterpret_cast<float *>(smem);   // [2*NK][32]: Wt[g][k] = W[k][g]
  float *Zs = Wt + 2 * NK * 32;                  // [P][ZZ]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < 2 * NK * 32; e += 256) {
    const int gg = e >> 5, k = e & 31;
    Wt[e] = (gg < g.G && k < g.Kdim) ? K[(int64_t)k * ks + gg] : 0.0f;
  }
  const int ntile = (g.P + 31) >> 5;
  const int CHW = g.C * g.HW;
  const int khkw = g.kh * g.kw;
  const float *wcol = Wt + (lane >> 5) * 32 + (lane & 31);

  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();  // Wt ready / previous col2im done with Zs
    const float *dyr = dY + (int64_t)n * dys;
    for (int pt = wave; pt < ntile; pt += 4) {
      const int p = pt * 32 + (lane & 31);
      const int pc = p < g.P ? p : g.P - 1;
      const float *col = dyr + pc + (int64_t)(lane >> 5) * g.P;
      float a[NK];
#pragma unroll
      for (int s = 0; s < NK; s++) a[s] = col[(int64_t)(2 * s) * g.P];
      floatx16 acc = zero16();
#pragma unroll
      for (int s = 0; s < NK; s++)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], wcol[s * 64], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int pl = pt * 32 + mfma32_row(r, lane);
        if (pl < g.P && (lane & 31) < g.Kdim) Zs[pl * ZZ + (lane & 31)] = acc[r];
      }
    }
    __syncthreads();
    float *dxr = dX + (int64_t)n * dxs;
    for (int e = tid; e < CHW; e += 256) {
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)e, c, q);
      g.div_H.divmod(q, wi, hi);
      float sum = 0.0f;
      for (int kx = 0; kx < g.kw; kx++) {
        const int px = (int)wi + g.pad_w - kx;
        if ((unsigned)px >= (unsigned)g.ow) continue;
        const float *zr = Zs + (int64_t)(px * g.oh) * ZZ + (int)c * khkw + kx * g.kh;
        for (int ky = 0; ky < g.kh; ky++) {
          const int py = (int)hi + g.pad_h - ky;
          if ((unsigned)py < (unsigned)g.oh) sum += zr[py * ZZ + ky];
        }
      }
      dxr[e] = sum;
    }
  }
}

// ---------------------------------------------------------------------------
template <int NSUP>
__global__ __launch_bounds__(256) void conv_wgrad_frame_kernel(
    ConvGeom g, const float *__restrict__ X, int xs,
    const float *__restrict__ dY, int dys, float *__restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float *Ds = reinterpret_cast<float *>(smem);   // [4 waves][32][ZS]
  float *Xs = Ds + 4 * 32 * ZS;                   // [C*HW]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float *myD = Ds + wave * 32 * ZS;

  // A-row of this lane: conv row j (< Kdim), the ones row (== Kdim), or pad.
  const int j = lane & 31;
  int koff = 0, kx = 0, ky = 0;
  if (j < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)j, c, r);
    g.div_kh.divmod(r, qx, qy);
    koff = (int)c * g.HW;
    kx = (int)qx;
    ky = (int)qy;
  }
  const bool is_ones = (j == g.Kdim);
  const int CHW = g.C * g.HW;

  floatx16 acc[NSUP];
#pragma unroll
  for (int su = 0; su < NSUP; su++) acc[su] = zero16();

  for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
    __syncthreads();
    const float *xr = X + (int64_t)n * xs;
    for (int e = tid; e < CHW; e += 256) Xs[e] = xr[e];
    __syncthreads();
    const float *dyr = dY + (int64_t)n * dys;
#pragma unroll
    for (int su = 0; su < NSUP; su++) {
      const int g0 = (su * 4 + wave) * 32;
      if (g0 >= g.G) continue;  // wave-uniform
      // dY tile rows g0 + 2i + (lane >> 5), column pc + (lane & 31); rows past
      // G or columns past P read a clamped address and are zeroed.
      const int gl0 = lane >> 5, pl0 = lane & 31;
      float nxt[16];
      auto load_tile = [&](int pc) {
        const bool pv = pc + pl0 < g.P;
        const int pcl = pv ? pc + pl0 : g.P - 1;
#pragma unroll
        for (int i = 0; i < 16; i++) {
          const int gg = g0 + 2 * i + gl0;
          const bool v = pv && gg < g.G;
          const float x = dyr[(int64_t)(v ? gg : 0) * g.P + pcl];
          nxt[i] = v ? x : 0.0f;
        }
      };
      load_tile(0);
      for (int pc = 0; pc < g.P; pc += 32) {
#pragma unroll
        for (int i = 0; i < 16; i++) myD[(2 * i + gl0) * ZS + pl0] = nxt[i];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (pc + 32 < g.P) load_tile(pc + 32);  // in flight during the MFMAs
        // im2col operand for p = pc + 2s + (lane >> 5), walked incrementally
        uint32_t px, py;
        g.div_oh.divmod((uint32_t)(pc + gl0), px, py);
        int ipx = (int)px, ipy = (int)py;
#pragma unroll 4
        for (int s = 0; s < 16; s++) {
          const int p = pc + 2 * s + gl0;
          const int xx = ipx + kx - g.pad_w, yy = ipy + ky - g.pad_h;
          const bool ok = j < g.Kdim && p < g.P && (unsigned)xx < (unsigned)g.W &&
                          (unsigned)yy < (unsigned)g.H;
          const float xv = Xs[ok ? koff + xx * g.H + yy : 0];
          const float av = ok ? xv : ((is_ones && p < g.P) ? 1.0f : 0.0f);
          const float bv = myD[(lane & 31) * ZS + 2 * s + gl0];
          acc[su] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[su], 0, 0, 0);
          ipy += 2;
          while (ipy >= g.oh) { ipy -= g.oh; ipx++; }
        }
      }
    }
  }
  // partial [Kdim + 1][G] of this workgroup
  const int E = (g.Kdim + 1) * g.G;
  float *dst = ws + (int64_t)blockIdx.x * E;
#pragma unroll
  for (int su = 0; su < NSUP; su++) {
    const int gl = (su * 4 + wave) * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int i = mfma32_row(r, lane);
      if (i <= g.Kdim && gl < g.G) dst[i * g.G + gl] = acc[su][r];
    }
  }
}

// ---------------------------------------------------------------------------
// Deterministic reduction of S partial rows: pass 1 sums groups of 32 rows,
// pass 2 sums the groups in order.
__global__ __launch_bounds__(256) void reduce_pass1(const float *__restrict__ in,
                                                    int S, int E,
                                                    float *__restrict__ tmp) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  const int s0 = blockIdx.y * 32, s1 = min(S, s0 + 32);
  float acc = 0.0f;
  for (int s = s0; s < s1; s++) acc += in[(int64_t)s * E + e];
  tmp[(int64_t)blockIdx.y * E + e] = acc;
}

// out mapping: e < nw -> gW[row][col] with (row, col) = gk_layout ?
// (e % inner, e / inner) : (e / inner, e % inner); e >= nw -> gb[e - nw].
__global__ __launch_bounds__(256) void reduce_pass2(const float *__restrict__ tmp,
                                                    int Q, int E, int nw,
                                                    int inner, int gk_layout,
                                                    float *__restrict__ gW,
                                                    int gws,
                                                    float *__restrict__ gb) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= E) return;
  float acc = 0.0f;
  for (int q = 0; q < Q; q++) acc += tmp[(int64_t)q * E + e];
  if (e < nw) {
    const int a = e / inner, b = e - a * inner;
    const int row = gk_layout ? b : a, col = gk_layout ? a : b;
    gW[(int64_t)row * gws + col] = acc;
  } else if (gb) {
    gb[e - nw] = acc;
  }
}

size_t fwd_lds(const ConvGeom &g, int Kpad, int Gp) {
  return (size_t)align16(Kpad * 8) + (size_t)Kpad * Gp * 4 + (size_t)g.C * g.HW * 4;
}

unsigned frame_grid(const ConvGeom &g, int blocks_per_cu) {
  int64_t b = 256LL * blocks_per_cu;
  if (b > g.R) b = g.R;
  return (unsigned)(b > 0 ? b : 1);
}

}  // namespace

int kcnn_conv_fwd_frame(const ConvGeom &g, const float *X, int xs,
                        const float *K, int ks, const float *bias, float *out,
                        int os, hipStream_t st) {
  if (g.Kdim > 64 || g.P < 16) return -1;
  const int Kpad = (g.Kdim + 1) & ~1;
  const int ngb = g.G > 64 ? 4 : (g.G > 32 ? 2 : 1);
  const int Gp = (g.G + 32 * ngb - 1) / (32 * ngb) * (32 * ngb);
  const size_t lds = fwd_lds(g, Kpad, Gp);
  if (lds > (size_t)kFrameLdsMax) return -1;
  const unsigned grid = frame_grid(g, 4);
  if (ngb == 4) {
    hipLaunchKernelGGL(conv_fwd_frame_kernel<4>, dim3(grid), dim3(256), lds, st,
                       g, X, xs, K, ks, bias, out, os, Kpad, Gp);
  } else if (ngb == 2) {
    hipLaunchKernelGGL(conv_fwd_frame_kernel<2>, dim3(grid), dim3(256), lds, st,
                       g, X, xs, K, ks, bias, out, os, Kpad, Gp);
  } else {
    hipLaunchKernelGGL(conv_fwd_frame_kernel<1>, dim3(grid), dim3(256), lds, st,
                       g, X, xs, K, ks, bias, out, os, Kpad, Gp);
  }
  return (int)hipGetLastError();
}

int kcnn_conv_dgrad_frame(const ConvGeom &g, const float *dY, int dys,
                          const float *K, int ks, float *dX, int dxs,
                          hipStream_t st) {
  if (g.Kdim > 32) return -1;
  if (g.G != 64 && g.G != 128) return -1;  // NK = G/2, fully unrolled
  const int ZZ = g.Kdim | 1;               // odd row stride: conflict-free col2im
  const size_t lds = ((size_t)g.G * 32 + (size_t)g.P * ZZ) * 4;
  if (lds > (size_t)kFrameLdsMax) return -1;
  if (g.G == 128)
    hipLaunchKernelGGL(conv_dgrad_frame_kernel<64>, dim3(frame_grid(g, 3)),
                       dim3(256), lds, st, g, dY, dys, K, ks, dX, dxs, ZZ);
  else
    hipLaunchKernelGGL(conv_dgrad_frame_kernel<32>, dim3(frame_grid(g, 3)),
                       dim3(256), lds, st, g, dY, dys, K, ks, dX, dxs, ZZ);
  return (int)hipGetLastError();
}

static int wgrad_frame_blocks(const ConvGeom &g) { return (int)frame_grid(g, 2); }

size_t kcnn_conv_wgrad_frame_ws(const ConvGeom &g) {
  if (g.Kdim > 31 || g.G > 256) return 0;
  const size_t lds = (size_t)(4 * 32 * ZS + g.C * g.HW) * 4;
  if (lds > (size_t)kFrameLdsMax) return 0;
  const int S = wgrad_frame_blocks(g);
  const int E = (g.Kdim + 1) * g.G;
  return (size_t)S * E * 4 + kcnn_reduce_splits_ws(S, E);
}

int kcnn_conv_wgrad_frame(const ConvGeom &g, const float *X, int xs,
                          const float *dY, int dys, float *gW, int gws,
                          float *gb, void *ws, size_t ws_bytes, hipStream_t st) {
  const size_t need = kcnn_conv_wgrad_frame_ws(g);
  if (need == 0 || ws == nullptr || ws_bytes < need) return -1;
  const int S = wgrad_frame_blocks(g);
  const int E = (g.Kdim + 1) * g.G;
  float *part = static_cast<float *>(ws);
  float *tmp = part + (size_t)S * E;
  const size_t lds = (size_t)(4 * 32 * ZS + g.C * g.HW) * 4;
  if (g.G <= 128)
    hipLaunchKernelGGL(conv_wgrad_frame_kernel<1>, dim3(S), dim3(256), lds, st,
                       g, X, xs, dY, dys, part);
  else
    hipLaunchKernelGGL(conv_wgrad_frame_kernel<2>, dim3(S), dim3(256), lds, st,
                       g, X, xs, dY, dys, part);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  const int Q = (S + 31) / 32;
  hipLaunchKernelGGL(reduce_pass1, dim3((E + 255) / 256, Q), dim3(256), 0, st,
                     part, S, E, tmp);
  hipLaunchKernelGGL(reduce_pass2, dim3((E + 255) / 256), dim3(256), 0, st, tmp,
                     Q, E, g.Kdim * g.G, g.G, 0, gW, gws, gb);
  return (int)hipGetLastError();
}

size_t kcnn_reduce_splits_ws(int S, int E) {
  return (size_t)((S + 31) / 32) * (size_t)E * 4;
}

// Generic: in [S][E] -> tmp [Q][E] -> out (with the gW/gb mapping of the
// implicit-GEMM wgrad: e = g*Kdim + k for e < G*Kdim).
int kcnn_reduce_splits_wgrad(const float *in, int S, int E, float *tmp, int nw,
                             int inner, float *gW, int gws, float *gb,
                             hipStream_t st) {
  const int Q = (S + 31) / 32;
  hipLaunchKernelGGL(reduce_pass1, dim3((E + 255) / 256, Q), dim3(256), 0, st,
                     in, S, E, tmp);
  hipLaunchKernelGGL(reduce_pass2, dim3((E + 255) / 256), dim3(256), 0, st, tmp,
                     Q, E, nw, inner, 1, gW, gws, gb);
  return (int)hipGetLastError();
}

int kcnn_reduce_splits_pass1(const float *in, int S, int E, float *tmp,
                             hipStream_t st) {
  const int Q = (S + 31) / 32;
  hipLaunchKernelGGL(reduce_pass1, dim3((E + 255) / 256, Q), dim3(256), 0, st,
                     in, S, E, tmp);
  return (int)hipGetLastError();
}

int kcnn_reduce_splits(const float *in, int S, int E, float *tmp, float *out,
                       hipStream_t st) {
  const int Q = (S + 31) / 32;
  hipLaunchKernelGGL(reduce_pass1, dim3((E + 255) / 256, Q), dim3(256), 0, st,
                     in, S, E, tmp);
  hipLaunchKernelGGL(reduce_pass2, dim3((E + 255) / 256), dim3(256), 0, st, tmp,
                     Q, E, E, E, 0, out, 0, nullptr);
  return (int)hipGetLastError();
}
