// cnslmat/cnsl-conv-x6.hip -- the fused convolution backward of the thin
// frame layers (Kdim = kh*kw*C <= 31, P <= 384: BASELINE c2's 8x1x3 input
// layer) on the bf16 matrix cores, with every fp32 operand split exactly
// into three bf16 parts (x = h + m + l) and the six leading cross products
// of each product kept (the bf16x6 scheme of kaldi-lite/cu-gemm-x6.hip; the
// three dropped terms are below fp32's own rounding of a product).
//
// Reference: ConvolutionComponent::Backprop (nnet-component-nnet0.cc:461-544)
// = dX by Conv2D of the padded dY with the flipped kernel (:489-540) and the
// update gradient of Update (:738-777: TpBlock(X) conv TpInsideBlock(dY),
// ModPermuteRow, bias = row sum of dY).  Here both come out of one pass over
// dY, as in conv_bwd_dma_kernel (cnsl-conv-frame.hip), whose fp32 MFMA
// (v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD) holds the SIMD's vector issue
// for all of its 64 cycles.  v_mfma_f32_32x32x16_bf16 does 8x the work in
// half the cycles; six of them replace eight fp32 MFMAs of the same tile at
// 3/8 of the matrix-pipe time.
//
// One workgroup (512 threads) per CU walks frames; per frame and 32-filter
// slab of dY:
//   split   the slab's dY (PCM > 0: built from the pooled derivative dP and
//           the routing mask of a fused PH x 1 x PCM Maxpool, i.e.
//           MaxpoolComponent::Backprop folded in) is gated, split and written
//           as three bf16 planes of a [g][p] LDS image (768-B rows, 16-B
//           chunks XOR-swizzled per 256-B segment, so that 32-lane row reads
//           and ds_read_b64_tr_b16 column reads are both conflict-free);
//   dgrad   Z[p][k] += sum_g dY[g][p] W[k][g]: A = dY^T by transposed reads of
//           the image, B = W from its own plane image; each wave owns position
//           tiles, Z stays in its accumulators for the frame;
//   wgrad   gW[k][g] += sum_p im2col(X)[k][p] dY[g][p]: A = the frame's im2col
//           values (gathered once per frame from the LDS-resident map and split
//           in registers; row Kdim is the constant 1, so the bias gradient falls
//           out of the same MFMAs), B = row reads of the image; the k16 steps
//           over p are dealt to the waves so every wave runs the same number
//           of MFMAs.
// At the end of a frame Z goes to LDS and is col2im'ed into dX during the
// next frame's first split phase.  Per-wave gradient partials are summed in a
// fixed order through LDS, workgroup partials by reduce_splits_kernel:
// deterministic, and bitwise the same with or without dX.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <type_traits>

#include "conv-geom.h"
#include "x6-util.h"

using namespace kcnn;

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void_t;
using x6::bf16x8;
using x6::split2;
using x6::split8;
using x6::mfma6;
using x6::zero16;

constexpr int NT = 512, NW = NT / 64;
constexpr int PP = 384;             // positions per image row (768 B)
constexpr int ROWB = PP * 2;
constexpr int YPL = 32 * ROWB;      // one plane of a 32-filter slab: 24 KB
constexpr int WROWB = 256;          // W image row: 128 filters
constexpr int WPL = 32 * WROWB;     // 8 KB
constexpr int MAXS = 6;             // wgrad k16 steps per wave (24 over waves 4-7)
constexpr int MAXT = 3;             // dgrad position tiles per wave (12 over waves 0-3)
constexpr int MAXU = 2;             // split units per thread (8 * 96 <= 2 * 512)
constexpr int MAXX = 4;             // X values per thread (C*H*W <= 2048)
constexpr int PZ = PP + 4;          // Z row (k-major) of conv_bwd_x6p_kernel: 16-B aligned,
                                    // rows 4 banks apart

struct X6Steps {
  uint8_t s[NW][MAXS];  // wgrad k16 steps of each wave, 0xff = none
};

__device__ __forceinline__ int swz4(int row) {
  return ((row & 3) << 2) | ((row >> 2) & 3);
}
// byte offset of (row, p) in a [row][384] bf16 image
__device__ __forceinline__ int yoff(int row, int p) {
  return row * ROWB + ((p >> 7) << 8) + ((((p >> 3) & 15) ^ swz4(row)) << 4) +
         ((p & 7) << 1);
}
// byte offset of (k, g) in the [32][128] bf16 W image
__device__ __forceinline__ int woff(int k, int g) {
  return k * WROWB + ((((g >> 3) & 15) ^ swz4(k)) << 4) + ((g & 7) << 1);
}

__host__ __device__ inline int round4(int n) { return (n + 3) & ~3; }
// staging floats for one slab's dP rows and bytes for its mask: whole DMA
// chunks (1 KiB, 256 B) and room for the split's reads past the last row (up
// to 16 values, masked off); ph > 1: P / ph pooled positions per row, 2-byte
// mask
__host__ __device__ inline int x6_stage_floats(int P, int pcm, int ph) {
  return (((pcm > 0 ? 32 / pcm : 32) * (P / ph) * 4 + 64 + 1023) & ~1023) / 4;
}
__host__ __device__ inline int x6_stage_mask_bytes(int P, int pcm, int ph) {
  return pcm > 0 ? (((32 / pcm) * (P / ph) * (ph > 1 ? 2 : 1) + 32 + 255) & ~255) : 0;
}

// PCM > 0: dY / dys are the pooled derivative dP of a PH x 1 x PCM Maxpool
// (PH = 1: channel-only; PH > 1 divides oh, so map position p = x*oh + y
// pools into p / PH), pmask / pms (bytes) its routing mask, 1 byte (PH = 1)
// or 2 (PH > 1) per pooled value:
//   dY[g][p] = bit (g % PCM)*PH + p % PH of mask[g / PCM][p / PH] ?
//              dP[g / PCM][p / PH] : +0
// (hipF_maxpool_backprop_mask, hipF_maxpool_backprop_mask3d with pw = 1).
template <int NCH, bool DX, bool WG, int PCM, int PH>
__global__ __launch_bounds__(NT, 1) void conv_bwd_x6_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dY, int dys,
    const float *__restrict__ K, int ks, float *__restrict__ dX, int dxs,
    float *__restrict__ ws_part, int ZZ, X6Steps steps, int dx_acc,
    const unsigned char *__restrict__ pmask, int pms, int dbg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef KCNN_PHASE_TIMING  // per-phase clock totals of block 0's waves (dbg & 16)
  long long tm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tprev = clock64();
#define KCNN_TMARK(i)                                   \
  if (dbg & 16) {                                       \
    const long long tn = clock64();                     \
    tm[i] += tn - tprev;                                \
    tprev = tn;                                         \
  }
#else
#define KCNN_TMARK(i)
  (void)dbg;
#endif
  const int P = g.P;
  const int Hp = g.H + 2 * g.pad_h, Wp = g.W + 2 * g.pad_w;
  const int CHWp = g.C * Hp * Wp;
  // DEFER (PCM > 0): Z has its own buffer and the col2im of frame n runs in
  // frame n+1's first split phase.  PCM == 0 needs that space to stage the
  // raw dY slab (46 KB at c2), so Z goes to the image at the frame's end and
  // is col2im'ed there, between two more barriers.
  constexpr bool DEFER = PCM > 0;
  using MaskT = typename std::conditional<(PH > 1), unsigned short, unsigned char>::type;
  const int Q = P / PH;  // pooled positions per dP row
  char *Yp = smem;                                   // [3][32][384] bf16
  char *Wimg = Yp + 3 * YPL;                         // [3][32][128] bf16
  float *Zs = DEFER ? reinterpret_cast<float *>(Wimg + (DX ? 3 * WPL : 0))  // [P][ZZ]
                    : reinterpret_cast<float *>(Yp);
  float *Xs = reinterpret_cast<float *>(Wimg + (DX ? 3 * WPL : 0)) +
              (DX && DEFER ? round4(P * ZZ) : 0);    // padded map + {1}
  int *qtab = reinterpret_cast<int *>(Xs + round4(CHWp + 1));  // [384]
  // the next slab's raw values, landed by LDS-DMA: PCM > 0 its dP rows and
  // mask bytes, PCM == 0 its 32 rows of dY
  constexpr int NJ = PCM > 0 ? 32 / PCM : 32;
  float *Sdp = reinterpret_cast<float *>(qtab + PP);          // [NJ][P] (+ DMA tail)
  MaskT *Smk = reinterpret_cast<MaskT *>(Sdp + x6_stage_floats(P, PCM, PH));
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = lane & 31, hf = lane >> 5;
  const int CHW = g.C * g.HW;
  const bool unpadded = g.pad_h == 0 && g.pad_w == 0;
  const int ntile = (P + 31) >> 5;
  const int PW = (P + 15) & ~15;     // wgrad contraction range (k16 steps)
  const int NPQ = PW >> 2;           // position quads per image row
  const int NU = (PCM > 0 ? NJ : 8) * NPQ;  // split units per slab
  (void)Smk;

  // W planes (dgrad B operand): rows k < Kdim, filters g < G; zero elsewhere
  if (DX) {
    for (int e = tid; e < 32 * 64; e += NT) {
      const int k = e >> 6, gg = (e & 63) * 2;
      const float v0 = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
      const float v1 = (k < g.Kdim && gg + 1 < g.G) ? K[(int64_t)k * ks + gg + 1] : 0.0f;
      uint32_t h, m, lo;
      split2(v0, v1, h, m, lo);
      const int o = woff(k, gg);
      *reinterpret_cast<uint32_t *>(Wimg + o) = h;
      *reinterpret_cast<uint32_t *>(Wimg + WPL + o) = m;
      *reinterpret_cast<uint32_t *>(Wimg + 2 * WPL + o) = lo;
    }
  }
  // im2col addressing: lane l's A row is k = l (row Kdim and above: the
  // constant-1 slot); position p of the frame at qtab[p] (past P: clamped to
  // the constant slot too, where the dY image is 0)
  int abase = CHWp * 4, qmul = 0;
  if (l < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)l, c, r);
    g.div_kh.divmod(r, qx, qy);
    abase = ((int)c * Hp * Wp + (int)qx * Hp + (int)qy) * 4;
    qmul = 1;
  }
  if (WG) {
    for (int e = tid; e < CHWp; e += NT) Xs[e] = 0.0f;
    if (tid == 0) Xs[CHWp] = 1.0f;
    for (int p = tid; p < PP; p += NT) {
      uint32_t px, py;
      g.div_oh.divmod((uint32_t)p, px, py);
      qtab[p] = p < P ? ((int)px * Hp + (int)py) * 4 : 0x3fffffff;
    }
  }
  const uint32_t amax = (uint32_t)CHWp * 4;
  const char *Xb = reinterpret_cast<const char *>(Xs);

  // ---- staging of one slab ----
  // LDS-DMA into Sdp (16 B per lane) / Smk (4 B per lane); a DMA lands by
  // the next barrier (s_waitcnt vmcnt(0)).  PCM > 0: the slab's NJ rows of
  // dP and of the mask, unit u = (pooled row j, position quad pq); PCM == 0:
  // its 32 rows of dY, unit u = (filter quad gq, position quad pq).
  auto load_slab = [&](int n, int ch) {
    const int rowf = (PCM > 0 ? g.G / PCM : g.G) * Q;  // values per frame row
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(dY + (int64_t)n * dys), (short)0, rowf * 4, 0x00020000);
    const int nq = (NJ * Q * 4 + 1023) >> 10;
    for (int q = wave; q < nq; q += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (lds_void_t *)(Sdp + q * 256), 16,
                                               (uint32_t)lane * 16u,
                                               (uint32_t)(ch * NJ * Q * 4 + q * 1024), 0, 0);
    if constexpr (PCM > 0) {
      constexpr int MB = (int)sizeof(MaskT);
      const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(pmask + (int64_t)n * pms), (short)0, rowf * MB, 0x00020000);
      const int nm = (NJ * Q * MB + 255) >> 8;
      for (int q = wave; q < nm; q += NW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rm, (lds_void_t *)(reinterpret_cast<char *>(Smk) + q * 256), 4,
            (uint32_t)lane * 4u, (uint32_t)(ch * NJ * Q * MB + q * 256), 0, 0);
    }
  };
  // PCM > 0: this thread's split units (pooled row j, position quad p0) are
  // the same in every slab: their image offsets are computed once.  yoff(row,
  // p0) for row = PCM*j + c is ubase + c*ROWB + ((ux[c >> 2] ^ ((c & 3) << 2)) << 4)
  int uj[MAXU], up0[MAXU], ubase[MAXU], ux[MAXU][2];
#pragma unroll
  for (int i = 0; i < MAXU; ++i) {
    const int u = min(tid + NT * i, NU - 1);
    uj[i] = u / NPQ;
    up0[i] = (u - uj[i] * NPQ) * 4;
    const int r0 = (PCM > 0 ? PCM : 4) * uj[i];
    ubase[i] = r0 * ROWB + ((up0[i] >> 7) << 8) + ((up0[i] & 7) << 1);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh)
      ux[i][hh] = ((up0[i] >> 3) & 15) ^ ((((r0 >> 2) + hh)) & 3);
  }
  auto split_slab = [&](int ch) {
#pragma unroll
    for (int i = 0; i < MAXU; ++i) {
      const int u = tid + NT * i;
      if (u >= NU) break;
      if constexpr (PCM > 0) {
        // split the pooled values once, then gate the planes per map: map c
        // of the pool group gets the value where its mask bit is set (the
        // in_value == out_value test of Maxpool_backprop), +0 else.
        // Positions past P get mask 0, so their values (the next row's, or
        // the staging tail) never reach the image: the AND writes +0.
        const int j = uj[i], p0 = up0[i];
        float x[4];
        unsigned mk[4];
        short rq[4];  // p % PH: the window row, the low part of the mask bit
        if constexpr (PH > 1) {
          // the quad's 4 positions fall in 2 windows (p0 % 4 == 0, PH <= 3)
          const int pq0 = p0 / PH, r0 = p0 - pq0 * PH, s0 = j * Q + pq0;
          const float x0 = Sdp[s0], x1 = Sdp[s0 + 1];
          const unsigned m0 = Smk[s0], m1 = Smk[s0 + 1];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool sel = r0 + q >= PH;
            rq[q] = (short)(r0 + q - (sel ? PH : 0));
            x[q] = sel ? x1 : x0;
            mk[q] = p0 + q < P ? (sel ? m1 : m0) : 0u;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            rq[q] = 0;
            x[q] = Sdp[j * Q + p0 + q];
            mk[q] = p0 + q < P ? (unsigned)Smk[j * Q + p0 + q] : 0u;
          }
        }
        uint32_t h01, m01, l01, h23, m23, l23;
        split2(x[0], x[1], h01, m01, l01);
        split2(x[2], x[3], h23, m23, l23);
        const s16x2 w01 = __builtin_bit_cast(s16x2, mk[0] | (mk[1] << 16));
        const s16x2 w23 = __builtin_bit_cast(s16x2, mk[2] | (mk[3] << 16));
        const s16x2 b01 = {(short)(15 - rq[0]), (short)(15 - rq[1])};
        const s16x2 b23 = {(short)(15 - rq[2]), (short)(15 - rq[3])};
#pragma unroll
        for (int c = 0; c < PCM; ++c) {
          // bit c*PH + p % PH of each 16-bit half, sign-extended to 0 / 0xffff
          const s16x2 cc = {(short)(c * PH), (short)(c * PH)}, k15 = {15, 15};
          const s16x2 sh01 = b01 - cc, sh23 = b23 - cc;
          const uint32_t s01 = __builtin_bit_cast(uint32_t, (s16x2)((w01 << sh01) >> k15));
          const uint32_t s23 = __builtin_bit_cast(uint32_t, (s16x2)((w23 << sh23) >> k15));
          // yoff(j * PCM + c, p0) from the unit's precomputed parts
          const int o = ubase[i] + c * ROWB + ((ux[i][c >> 2] ^ ((c & 3) << 2)) << 4);
          *reinterpret_cast<uint2 *>(Yp + o) = make_uint2(h01 & s01, h23 & s23);
          *reinterpret_cast<uint2 *>(Yp + YPL + o) = make_uint2(m01 & s01, m23 & s23);
          *reinterpret_cast<uint2 *>(Yp + 2 * YPL + o) = make_uint2(l01 & s01, l23 & s23);
        }
      } else {
        const int gq = u / NPQ, p0 = (u - gq * NPQ) * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float *srow = Sdp + (4 * gq + r) * P + p0;
          float x[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) x[q] = p0 + q < P ? srow[q] : 0.0f;
          uint32_t h0, m0, l0, h1, m1, l1;
          split2(x[0], x[1], h0, m0, l0);
          split2(x[2], x[3], h1, m1, l1);
          const int o = yoff(4 * gq + r, p0);
          *reinterpret_cast<uint2 *>(Yp + o) = make_uint2(h0, h1);
          *reinterpret_cast<uint2 *>(Yp + YPL + o) = make_uint2(m0, m1);
          *reinterpret_cast<uint2 *>(Yp + 2 * YPL + o) = make_uint2(l0, l1);
        }
      }
    }
    (void)ch;
  };

  // ---- X map (wgrad) ----
  float xv[MAXX];
  auto load_x = [&](int n) {
#pragma unroll
    for (int i = 0; i < MAXX; i++)
      if (tid + NT * i < CHW) xv[i] = X[(int64_t)n * xs + tid + NT * i];
  };
  auto commit_x = [&]() {
#pragma unroll
    for (int i = 0; i < MAXX; i++) {
      const int e = tid + NT * i;
      if (e < CHW) {
        int slot = e;
        if (!unpadded) {
          uint32_t c, q, wi, hi;
          g.div_HW.divmod((uint32_t)e, c, q);
          g.div_H.divmod(q, wi, hi);
          slot = (int)c * Hp * Wp + ((int)wi + g.pad_w) * Hp + (int)hi + g.pad_h;
        }
        Xs[slot] = xv[i];
      }
    }
  };

  // ---- col2im (dX) from Zs, as conv_bwd_dma_kernel (tap ranges per call:
  // a few VALU per output and frame instead of two registers held all along)
  const int khkw = g.kh * g.kw;
  const int zax = g.oh * ZZ - g.kh, zby = ZZ - 1;
  auto col2im = [&](int nn) {
#pragma unroll
    for (int i = 0; i < MAXX; i++) {
      const int e = tid + NT * i;
      if (e >= CHW) continue;
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)e, c, q);
      g.div_H.divmod(q, wi, hi);
      const int ty = (int)hi + g.pad_h, tx = (int)wi + g.pad_w;
      const int zb = (tx * g.oh + ty) * ZZ + (int)c * khkw;
      const int ylo = max(0, ty - g.oh + 1), ny = min(g.kh - 1, ty) - ylo;
      const int xlo = max(0, tx - g.ow + 1), xhi = min(g.kw - 1, tx);
      float sum = 0.0f;
      for (int kx = xlo; kx <= xhi; kx++) {
        const int zk = zb - kx * zax;
        for (int k0 = 0; k0 < g.kh; k0 += 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; u++) v[u] = Zs[zk - (k0 + u) * zby];
#pragma unroll
          for (int u = 0; u < 8; u++)
            sum += (unsigned)(k0 + u - ylo) <= (unsigned)ny ? v[u] : 0.0f;
        }
      }
      float *d = dX + (int64_t)nn * dxs + e;
      *d = dx_acc ? *d + sum : sum;
    }
  };

  // Roles.  With both outputs, waves 0-3 run the data gradient (position
  // tiles w, w + 4, w + 8) and waves 4-7 the weight gradient (the host's
  // step table), so each SIMD pairs one of each (waves w and w + 4 share a
  // SIMD) and each wave keeps only its own accumulators: the dgrad waves Z
  // (3 tiles), the wgrad waves the frame's im2col fragments and the four
  // slabs' gradient partials.  dX only: all 8 waves, tiles w and w + 8.
  // Gradient only: the same wgrad waves and table as with dX (bitwise the
  // same gradient), waves 0-3 only split.  Both roles run the same barrier
  // sequence: every thread splits, commits the map and runs the col2im.
  const bool dgrad_wave = DX && (!WG || wave < 4);
  const int tslot = WG ? wave : wave, tstride = WG ? 4 : NW;
  auto frames = [&](auto role) {
    constexpr bool RD = decltype(role)::value == 1;  // dgrad role
    constexpr bool RW = decltype(role)::value == 2;  // wgrad role
    int my_steps = 0;
    int stp[MAXS];
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      stp[s] = steps.s[wave][s];
      if (RW && stp[s] != 0xff) my_steps = s + 1;
    }
    floatx16 wacc[RW ? NCH : 1];
#pragma unroll
    for (int c = 0; c < (RW ? NCH : 1); c++) wacc[c] = zero16();
    bf16x8 ain[RW ? MAXS : 1][3];
    int nprev = -1;
    for (int n = blockIdx.x; n < g.R; n += gridDim.x) {
      floatx16 zacc[RD ? MAXT : 1];
#pragma unroll
      for (int t = 0; t < (RD ? MAXT : 1); ++t) zacc[t] = zero16();
#pragma unroll
      for (int ch = 0; ch < NCH; ch++) {
        // B1: the slab (and map) DMA has landed for every wave; the image's
        // readers are done; last frame's Z is in LDS
        KCNN_TMARK(7)
        x6::publish_dma();
        KCNN_TMARK(0)
        if (ch == 0) {
          if (WG) commit_x();
          if (DX && DEFER && nprev >= 0) col2im(nprev);
        }
        KCNN_TMARK(1)
        split_slab(ch);
        KCNN_TMARK(2)
        __syncthreads();  // B2: the slab (and the frame's map) are in LDS
        KCNN_TMARK(3)
        if (RW && ch == 0) {
          // the frame's im2col values of this wave's steps, split once
#pragma unroll
          for (int s = 0; s < MAXS; ++s) {
            if (s >= my_steps) break;
            const int pbase = 16 * stp[s] + 8 * hf;
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t off = min((uint32_t)(abase + qmul * qtab[pbase + e]), amax);
              v[e] = *reinterpret_cast<const float *>(Xb + off);
            }
            split8(v, ain[s][0], ain[s][1], ain[s][2]);
          }
        }
        KCNN_TMARK(4)
        // the next slab (or the next frame's first slab and map) into registers
        {
          const int nn = ch + 1 < NCH ? n : n + (int)gridDim.x;
          const int cc = ch + 1 < NCH ? ch + 1 : 0;
          if (nn < g.R) {
            load_slab(nn, cc);
            if (WG && ch + 1 == NCH) load_x(nn);
          }
        }
        KCNN_TMARK(5)
        if constexpr (RD) {
          // Z[p][k] += dY^T W on this wave's position tiles
          bf16x8 wf[2][3];
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
              wf[s][pl] = *reinterpret_cast<const bf16x8 *>(
                  Wimg + pl * WPL + woff(l, ch * 32 + 16 * s + 8 * hf));
          const int G4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
          for (int t = 0; t < MAXT; ++t) {
            const int pt = tslot + tstride * t;
            if (pt >= ntile) break;  // uniform
            const int col = pt * 32 + 16 * (G4 & 1) + 4 * pp;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              bf16x8 af[3];
              const int row = 16 * s + 8 * (G4 >> 1) + q;
#pragma unroll
              for (int pl = 0; pl < 3; ++pl) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4 *)(Yp + pl * YPL + yoff(row, col)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s16x4 *)(Yp + pl * YPL + yoff(row + 4, col)));
                af[pl] = __builtin_bit_cast(
                    bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
              }
              zacc[t] = mfma6(af, wf[s], zacc[t]);
            }
          }
        }
        if constexpr (RW) {
          // gW[k][g] += im2col(X) dY^T over this wave's k16 steps of p
#pragma unroll
          for (int s = 0; s < MAXS; ++s) {
            if (s >= my_steps) break;
            bf16x8 bf[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
              bf[pl] = *reinterpret_cast<const bf16x8 *>(Yp + pl * YPL +
                                                         yoff(l, 16 * stp[s] + 8 * hf));
            wacc[ch] = mfma6(ain[s], bf, wacc[ch]);
          }
        }
        KCNN_TMARK(6)
      }
      if (DX && !DEFER) __syncthreads();  // the image is read no more: Z goes there
      if constexpr (RD) {
        // Z of this frame -> LDS (DEFER: its last reader, the col2im in this
        // frame's first split phase, finished before that phase's barrier)
#pragma unroll
        for (int t = 0; t < MAXT; ++t) {
          const int pt = tslot + tstride * t;
          if (pt >= ntile) break;
#pragma unroll
          for (int r = 0; r < 16; r++) {
            const int pl = pt * 32 + mfma32_row(r, lane);
            if (pl < P && l < g.Kdim) Zs[pl * ZZ + l] = zacc[t][r];
          }
        }
      }
      if (DX && !DEFER) {
        __syncthreads();
        col2im(n);
      }
      nprev = n;
    }
    if (DX && DEFER && nprev >= 0) {
      __syncthreads();
      col2im(nprev);
    }
#ifdef KCNN_PHASE_TIMING
    if ((dbg & 16) && blockIdx.x == 0 && lane == 0)
      printf("bwdx6 wave %d: B1 %lld ch0 %lld split %lld B2 %lld im2col %lld dma %lld mfma %lld "
             "tail %lld\n", wave, tm[0], tm[1], tm[2], tm[3], tm[4], tm[5], tm[6], tm[7]);
#endif
    if (!WG) return;
    // the wgrad waves' partials (waves 4-7) summed in a fixed order
    const int E = (g.Kdim + 1) * g.G;
    float *dst = ws_part + (int64_t)blockIdx.x * E;
    float *red = reinterpret_cast<float *>(Yp);  // [4][32 x 32], 16 KB
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      __syncthreads();
      if constexpr (RW) {
        if (wave >= 4) {
#pragma unroll
          for (int r = 0; r < 16; r++)
            red[(wave - 4) * 1024 + mfma32_row(r, lane) * 32 + l] = wacc[ch][r];
        }
      }
      __syncthreads();
      for (int e = tid; e < 1024; e += NT) {
        const int i = e >> 5, j = e & 31;
        if (i > g.Kdim) continue;
        float sum = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; w++) sum += red[w * 1024 + e];
        // (dbg bit 30: add to the partial an earlier frame range left there)
        dst[i * g.G + ch * 32 + j] = (dbg & (1 << 30)) ? dst[i * g.G + ch * 32 + j] + sum : sum;
      }
    }
  };
  if (blockIdx.x < (unsigned)g.R) {
    load_slab(blockIdx.x, 0);
    if (WG) load_x(blockIdx.x);
  }
  if (dgrad_wave) frames(std::integral_constant<int, 1>{});
  else frames(std::integral_constant<int, 2>{});
#undef KCNN_TMARK
}

// ---------------------------------------------------------------------------
#ifdef KCNN_EXPERIMENTS  // the round-2/3 pipelined kernel, x6q's predecessor:
                         // only the experiment build (KCNN_BWD_X6P=1) has it
// conv_bwd_x6p_kernel: conv_bwd_x6_kernel's math bit for bit -- the same
// image contents, operand fragments, and order of the MFMAs into every
// accumulator -- software-pipelined, for the pooled backward with both
// outputs (DX and WG, a folded PH x 1 x PCM Maxpool, NCH >= 2 slabs per
// frame: c2, c5 C1).
//
// conv_bwd_x6_kernel alternates an all-VALU phase (every wave splits the
// next slab into the image) with an all-MFMA phase, two barriers apart, so
// each SIMD's matrix pipe idles while its waves split (c2, block 0: split
// 134 k, MFMA phase 167 k of 495 k cycles per wave, MFMA pipe 28 % busy).
// Here the split of slab t+1 runs beside the MFMAs of slab t.  A thread
// keeps its split units' gated bf16 planes in registers until the image is
// free, and its raw dP / mask values come from HBM into registers one slab
// ahead (no staging buffer, no LDS-DMA).  Per SIMD, the dgrad wave w and the
// wgrad wave w + 4:
//
//   MFMA phase t   dgrad wave: split its 2 units of slab t+1, prefetch their
//                  raw values of slab t+2, then its dgrad MFMAs of slab t
//                  (position tiles w, w + 4, w + 8);  wgrad wave: its wgrad
//                  MFMAs of slab t, then the frame work (col2im of the
//                  previous frame on the first slab, the next frame's im2col
//                  gather on the last), then its 1 unit of slab t+1 -- so
//                  each wave's VALU runs beside its partner's MFMAs.  The
//                  dgrad waves store the frame's Z on its last slab.
//   barrier Ba     the image of slab t is read no more
//   write phase    the held planes of slab t+1 -> the image; the map of the
//                  frame after next -> LDS (last slab)
//   barrier Bb     the image of slab t+1 is published
//
// Z is kept k-major here ([Kdim][PZ], a lane's accumulator rows are 16-B
// runs); the col2im adds the same values in the same order.
template <int NCH, int PCM, int PH>
__global__ __launch_bounds__(NT, 1) void conv_bwd_x6p_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dP, int dps,
    const float *__restrict__ K, int ks, float *__restrict__ dX, int dxs,
    float *__restrict__ ws_part, int ZZ, X6Steps steps, int dx_acc,
    const unsigned char *__restrict__ pmask, int pms, int dbg) {
  static_assert(NCH >= 2 && PCM > 0, "pooled backward with >= 2 slabs per frame");
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef KCNN_PHASE_TIMING  // per-phase clock totals of block 0's waves (dbg & 16)
  long long tm[6] = {0, 0, 0, 0, 0, 0};
  long long tprev = clock64();
#define KCNN_TMARK(i)               \
  if (dbg & 16) {                   \
    const long long tn = clock64(); \
    tm[i] += tn - tprev;            \
    tprev = tn;                     \
  }
#else
#define KCNN_TMARK(i)
  (void)dbg;
#endif
  using MaskT = typename std::conditional<(PH > 1), unsigned short, unsigned char>::type;
  constexpr int MB = (int)sizeof(MaskT);
  constexpr int NJ = 32 / PCM;                         // pooled rows per slab
  constexpr int SPL = NT;                                 // splitting threads
  constexpr int MAXUP = (NJ * (PP / 4) + SPL - 1) / SPL;  // split units per thread
  const int P = g.P;
  const int Q = P / PH;  // pooled positions per dP row
  const int Hp = g.H + 2 * g.pad_h, Wp = g.W + 2 * g.pad_w;
  const int CHWp = g.C * Hp * Wp;
  char *Yp = smem;                                            // [3][32][384] bf16
  char *Wimg = Yp + 3 * YPL;                                  // [3][32][128] bf16
  // Z k-major, [Kdim][PZ]: a lane's accumulator rows are runs of 4
  // consecutive positions of one k, stored as 16-B writes
  float *Zt = reinterpret_cast<float *>(Wimg + 3 * WPL);
  float *Xs = Zt + g.Kdim * PZ;                               // padded map + {1}
  int *qtab = reinterpret_cast<int *>(Xs + round4(CHWp + 1));  // [384]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = lane & 31, hf = lane >> 5;
  const int CHW = g.C * g.HW;
  const bool unpadded = g.pad_h == 0 && g.pad_w == 0;
  const int ntile = (P + 31) >> 5;
  const int PW = (P + 15) & ~15;
  const int NPQ = PW >> 2;
  const int NU = NJ * NPQ;
  const int G = (int)gridDim.x;
  const int rowf = (g.G / PCM) * Q;  // pooled values per frame row

  // W planes (dgrad B operand), as conv_bwd_x6_kernel
  for (int e = tid; e < 32 * 64; e += NT) {
    const int k = e >> 6, gg = (e & 63) * 2;
    const float v0 = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
    const float v1 = (k < g.Kdim && gg + 1 < g.G) ? K[(int64_t)k * ks + gg + 1] : 0.0f;
    uint32_t h, m, lo;
    split2(v0, v1, h, m, lo);
    const int o = woff(k, gg);
    *reinterpret_cast<uint32_t *>(Wimg + o) = h;
    *reinterpret_cast<uint32_t *>(Wimg + WPL + o) = m;
    *reinterpret_cast<uint32_t *>(Wimg + 2 * WPL + o) = lo;
  }
  int abase = CHWp * 4, qmul = 0;
  if (l < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)l, c, r);
    g.div_kh.divmod(r, qx, qy);
    abase = ((int)c * Hp * Wp + (int)qx * Hp + (int)qy) * 4;
    qmul = 1;
  }
  for (int e = tid; e < CHWp; e += NT) Xs[e] = 0.0f;
  if (tid == 0) Xs[CHWp] = 1.0f;
  for (int p = tid; p < PP; p += NT) {
    uint32_t px, py;
    g.div_oh.divmod((uint32_t)p, px, py);
    qtab[p] = p < P ? ((int)px * Hp + (int)py) * 4 : 0x3fffffff;
  }
  const uint32_t amax = (uint32_t)CHWp * 4;
  const char *Xb = reinterpret_cast<const char *>(Xs);

  // ---- split units: (pooled row j, position quad p0), the same in every
  // slab; the dgrad waves' threads own units tid + 256 i
  int uj[MAXUP], up0[MAXUP], ubase[MAXUP], ux[MAXUP][2];
#pragma unroll
  for (int i = 0; i < MAXUP; ++i) {
    const int u = min(tid + SPL * i, NU - 1);
    uj[i] = u / NPQ;
    up0[i] = (u - uj[i] * NPQ) * 4;
    const int r0 = PCM * uj[i];
    ubase[i] = r0 * ROWB + ((up0[i] >> 7) << 8) + ((up0[i] & 7) << 1);
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) ux[i][hh] = ((up0[i] >> 3) & 15) ^ (((r0 >> 2) + hh) & 3);
  }
  // raw values of a unit: PH == 1 the quad's 4 dP values, PH > 1 the 2
  // windows' values; the mask bytes of the same positions as two dwords
  // (aligned down) and the byte shift.  U: units per thread of the role
  // (MAXUP for the dgrad waves; the wgrad waves split nothing)
  constexpr int NX = PH > 1 ? 2 : 4;
  auto load_raw = [&](auto Uc, float (&rx)[decltype(Uc)::value][NX],
                      uint32_t (&rm)[decltype(Uc)::value][2], int (&rsh)[decltype(Uc)::value],
                      int nn, int cc) {
    constexpr int U = decltype(Uc)::value;
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(dP + (int64_t)nn * dps), (short)0, rowf * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(pmask + (int64_t)nn * pms), (short)0, rowf * MB, 0x00020000);
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (tid + SPL * i >= NU) break;
      const int s = (cc * NJ + uj[i]) * Q + (PH > 1 ? up0[i] / PH : up0[i]);
      if constexpr (NX == 4) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rd, (unsigned)s * 4u, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) rx[i][q] = __uint_as_float(v[q]);
      } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rd, (unsigned)s * 4u, 0, 0);
        rx[i][0] = __uint_as_float(v[0]);
        rx[i][1] = __uint_as_float(v[1]);
      }
      const unsigned mo = (unsigned)s * MB;
      const auto w = __builtin_amdgcn_raw_buffer_load_b64(rk, mo & ~3u, 0, 0);
      rm[i][0] = w[0];
      rm[i][1] = w[1];
      rsh[i] = (int)(mo & 3u);
    }
  };
  // gated planes of a unit: [map c][plane][2 dwords]
  auto split_raw = [&](auto Uc, const float (&rx)[decltype(Uc)::value][NX],
                       const uint32_t (&rm)[decltype(Uc)::value][2],
                       const int (&rsh)[decltype(Uc)::value],
                       uint32_t (&sres)[decltype(Uc)::value][PCM][6]) {
    constexpr int U = decltype(Uc)::value;
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (tid + SPL * i >= NU) break;
      const int p0 = up0[i];
      const uint32_t mw = __builtin_amdgcn_alignbyte(rm[i][1], rm[i][0], (uint32_t)rsh[i]);
      float x[4];
      unsigned mk[4];
      short rq[4];
      if constexpr (PH > 1) {
        const int pq0 = p0 / PH, r0 = p0 - pq0 * PH;
        const unsigned m0 = mw & 0xffffu, m1 = mw >> 16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bool sel = r0 + q >= PH;
          rq[q] = (short)(r0 + q - (sel ? PH : 0));
          x[q] = sel ? rx[i][1] : rx[i][0];
          mk[q] = p0 + q < P ? (sel ? m1 : m0) : 0u;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rq[q] = 0;
          x[q] = rx[i][q];
          mk[q] = p0 + q < P ? (mw >> (8 * q)) & 0xffu : 0u;
        }
      }
      uint32_t h01, m01, l01, h23, m23, l23;
      split2(x[0], x[1], h01, m01, l01);
      split2(x[2], x[3], h23, m23, l23);
      const s16x2 w01 = __builtin_bit_cast(s16x2, mk[0] | (mk[1] << 16));
      const s16x2 w23 = __builtin_bit_cast(s16x2, mk[2] | (mk[3] << 16));
      const s16x2 b01 = {(short)(15 - rq[0]), (short)(15 - rq[1])};
      const s16x2 b23 = {(short)(15 - rq[2]), (short)(15 - rq[3])};
#pragma unroll
      for (int c = 0; c < PCM; ++c) {
        const s16x2 cc = {(short)(c * PH), (short)(c * PH)}, k15 = {15, 15};
        const s16x2 sh01 = b01 - cc, sh23 = b23 - cc;
        const uint32_t s01 = __builtin_bit_cast(uint32_t, (s16x2)((w01 << sh01) >> k15));
        const uint32_t s23 = __builtin_bit_cast(uint32_t, (s16x2)((w23 << sh23) >> k15));
        sres[i][c][0] = h01 & s01;
        sres[i][c][1] = h23 & s23;
        sres[i][c][2] = m01 & s01;
        sres[i][c][3] = m23 & s23;
        sres[i][c][4] = l01 & s01;
        sres[i][c][5] = l23 & s23;
      }
    }
  };
  auto write_sres = [&](auto Uc, const uint32_t (&sres)[decltype(Uc)::value][PCM][6]) {
    constexpr int U = decltype(Uc)::value;
#pragma unroll
    for (int i = 0; i < U; ++i) {
      if (tid + SPL * i >= NU) break;
#pragma unroll
      for (int c = 0; c < PCM; ++c) {
        const int o = ubase[i] + c * ROWB + ((ux[i][c >> 2] ^ ((c & 3) << 2)) << 4);
        *reinterpret_cast<uint2 *>(Yp + o) = make_uint2(sres[i][c][0], sres[i][c][1]);
        *reinterpret_cast<uint2 *>(Yp + YPL + o) = make_uint2(sres[i][c][2], sres[i][c][3]);
        *reinterpret_cast<uint2 *>(Yp + 2 * YPL + o) = make_uint2(sres[i][c][4], sres[i][c][5]);
      }
    }
  };

  // ---- X map (wgrad A operand) ----
  float xv[MAXX];
  auto load_x = [&](int n) {
#pragma unroll
    for (int i = 0; i < MAXX; i++)
      if (tid + NT * i < CHW) xv[i] = X[(int64_t)n * xs + tid + NT * i];
  };
  auto commit_x = [&]() {
#pragma unroll
    for (int i = 0; i < MAXX; i++) {
      const int e = tid + NT * i;
      if (e < CHW) {
        int slot = e;
        if (!unpadded) {
          uint32_t c, q, wi, hi;
          g.div_HW.divmod((uint32_t)e, c, q);
          g.div_H.divmod(q, wi, hi);
          slot = (int)c * Hp * Wp + ((int)wi + g.pad_w) * Hp + (int)hi + g.pad_h;
        }
        Xs[slot] = xv[i];
      }
    }
  };
  // ---- col2im (dX) from Zs: conv_bwd_x6_kernel's, the same sums in the same order
  const int khkw = g.kh * g.kw;
  // element (p, k) at k * PZ + p: tap (kx, ky) of output (c, tx, ty) at
  // c khkw PZ + tx oh + ty + kx (kh PZ - oh) + ky (PZ - 1)
  const int zax = g.kh * PZ - g.oh, zby = PZ - 1;
  auto col2im = [&](int nn) {
#pragma unroll 1
    for (int i = 0; i < MAXX; i++) {
      const int e = tid + NT * i;
      if (e >= CHW) continue;
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)e, c, q);
      g.div_H.divmod(q, wi, hi);
      const int ty = (int)hi + g.pad_h, tx = (int)wi + g.pad_w;
      const int zb = (int)c * khkw * PZ + tx * g.oh + ty;
      const int ylo = max(0, ty - g.oh + 1), ny = min(g.kh - 1, ty) - ylo;
      const int xlo = max(0, tx - g.ow + 1), xhi = min(g.kw - 1, tx);
      float sum = 0.0f;
      for (int kx = xlo; kx <= xhi; kx++) {
        const int zk = zb + kx * zax;
        for (int k0 = 0; k0 < g.kh; k0 += 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; u++) v[u] = Zt[zk + (k0 + u) * zby];
#pragma unroll
          for (int u = 0; u < 8; u++)
            sum += (unsigned)(k0 + u - ylo) <= (unsigned)ny ? v[u] : 0.0f;
        }
      }
      float *d = dX + (int64_t)nn * dxs + e;
      *d = dx_acc ? *d + sum : sum;
    }
  };

  const bool dgrad_wave = wave < 4;
  int my_steps = 0;
  int stp[MAXS];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    stp[s] = steps.s[wave][s];
    if (!dgrad_wave && stp[s] != 0xff) my_steps = s + 1;
  }
  // the frame's im2col values of this wave's steps, split once per frame
  auto gather = [&](auto &a) {
#pragma unroll
    for (int s = 0; s < MAXS; ++s) {
      if (s >= my_steps) break;
      const int pbase = 16 * stp[s] + 8 * hf;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t off = min((uint32_t)(abase + qmul * qtab[pbase + e]), amax);
        v[e] = *reinterpret_cast<const float *>(Xb + off);
      }
      split8(v, a[s][0], a[s][1], a[s][2]);
      __builtin_amdgcn_sched_barrier(0);  // one step's temporaries at a time
    }
  };

  const int n0 = blockIdx.x;
  auto frames = [&](auto role) {
    constexpr bool RD = decltype(role)::value == 1;  // dgrad waves
    constexpr int U = RD ? MAXUP : 1;
    using UC = std::integral_constant<int, U>;
    float rx[U][NX];
    uint32_t rm[U][2];
    int rsh[U];
    uint32_t sres[U][PCM][6];
    // (defined on every path: steps past my_steps are never used, but an
    // undefined register set costs the allocator spills)
    bf16x8 ain[RD ? 1 : MAXS][3];
#pragma unroll
    for (int s = 0; s < (RD ? 1 : MAXS); ++s)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) ain[s][pl] = bf16x8{};
    // ---- prologue: the maps of the first two frames, the first frame's
    // im2col values, its first slab in the image, its second slab's raw values
    load_x(n0);
    load_raw(UC{}, rx, rm, rsh, n0, 0);
    __syncthreads();  // Xs zeroed, qtab and the W image written
    commit_x();
    if (n0 + G < g.R) load_x(n0 + G);
    __syncthreads();
    if constexpr (!RD) gather(ain);
    split_raw(UC{}, rx, rm, rsh, sres);
    load_raw(UC{}, rx, rm, rsh, n0, 1);
    __syncthreads();  // the gather's reads of Xs are done
    if (n0 + G < g.R) commit_x();
    write_sres(UC{}, sres);
    __syncthreads();  // Bb: slab (n0, 0) in the image, frame n0 + G's map in Xs

    floatx16 wacc[RD ? 1 : NCH];
#pragma unroll
    for (int c = 0; c < (RD ? 1 : NCH); c++) wacc[c] = zero16();
    int nprev = -1;

    for (int n = n0; n < g.R; n += G) {
      // dgrad position tiles: the dgrad waves w, w + 4; the wgrad waves take
      // one each (w + 4 = tiles 8-11), beside their weight-gradient steps
      constexpr int TT = RD ? MAXT : 1;
      floatx16 zacc[TT];
#pragma unroll
      for (int t = 0; t < TT; ++t) zacc[t] = zero16();
      auto tile_of = [&](int t) { return wave + 4 * t; };
      // Z[p][k] += dY^T W on this wave's position tiles: MFMA group gi =
      // (tile t = gi / 2, k16 slice s = gi % 2), the next group's transposed
      // reads issued before the current group's MFMAs (two fragment sets live,
      // not every group's: the wgrad role's registers are tight)
      auto dgrad = [&](int ch) {
        bf16x8 wf[2][3];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            wf[s][pl] = *reinterpret_cast<const bf16x8 *>(
                Wimg + pl * WPL + woff(l, ch * 32 + 16 * s + 8 * hf));
        const int G4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
        auto load_af = [&](int gi, bf16x8 (&af)[3]) {
          const int col = tile_of(gi >> 1) * 32 + 16 * (G4 & 1) + 4 * pp;
          const int row = 16 * (gi & 1) + 8 * (G4 >> 1) + q;
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4 *)(Yp + pl * YPL + yoff(row, col)));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4 *)(Yp + pl * YPL + yoff(row + 4, col)));
            af[pl] = __builtin_bit_cast(
                bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
        };
        constexpr int NG = 2 * TT;
        bf16x8 afb[2][3];
        if (tile_of(0) < ntile) load_af(0, afb[0]);
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) {
          if (tile_of(gi >> 1) >= ntile) break;  // uniform
          if (gi + 1 < NG && tile_of((gi + 1) >> 1) < ntile) load_af(gi + 1, afb[(gi + 1) & 1]);
          zacc[gi >> 1] = mfma6(afb[gi & 1], wf[gi & 1], zacc[gi >> 1]);
        }
      };
      // Z of this frame -> LDS: its last reader, the col2im of the previous
      // frame in this frame's first slab, is two barriers back
      auto store_z = [&]() {
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          const int pt = tile_of(t);
          if (pt >= ntile) break;
          // rows (r & 3) + 8 (r >> 2) + 4 hf: four runs of 4 positions
          // (positions past P land in the row's tail, never read)
          if (l < g.Kdim) {
            float *zr = Zt + l * PZ + pt * 32 + 4 * hf;
#pragma unroll
            for (int i = 0; i < 4; i++)
              *reinterpret_cast<float4 *>(zr + 8 * i) =
                  make_float4(zacc[t][4 * i], zacc[t][4 * i + 1], zacc[t][4 * i + 2],
                              zacc[t][4 * i + 3]);
          }
        }
      };
#pragma unroll
      for (int ch = 0; ch < NCH; ch++) {
        // slab t = (n, ch); t+1 and t+2 in frame order
        const int n1 = ch + 1 < NCH ? n : n + G;
        const int n2 = ch + 2 < NCH ? n : n + G, c2 = ch + 2 < NCH ? ch + 2 : ch + 2 - NCH;
        const bool next = n1 < g.R;
        KCNN_TMARK(5)
        if (ch == 0 && n + 2 * G < g.R) load_x(n + 2 * G);
        if constexpr (RD) {
          // the split of slab t+1 beside the wgrad waves' MFMAs, then ours
          if (next) {
            split_raw(UC{}, rx, rm, rsh, sres);
            if (n2 < g.R) load_raw(UC{}, rx, rm, rsh, n2, c2);
          }
          KCNN_TMARK(0)
          dgrad(ch);
          KCNN_TMARK(1)
          if (ch == 0 && nprev >= 0) col2im(nprev);
        } else {
          // gW[k][g] += im2col(X) dY^T over this wave's k16 steps of p (the
          // next step's row reads issued before the current step's MFMAs)
          // yoff(l, 16 stp + 8 hf) = l ROWB + (stp >> 3) 256 + (((stp & 7) << 5) ^
          // ((hf ^ swz4(l)) << 4)): the lane part passes through an opaque
          // move each slab, so the compiler does not hoist (and spill) six
          // per-step addresses out of the frame loop
          int lx, lrow;
          asm volatile("v_mov_b32 %0, %1" : "=v"(lx) : "v"((hf ^ swz4(l)) << 4));
          asm volatile("v_mov_b32 %0, %1" : "=v"(lrow) : "v"(l * ROWB));
          auto load_bf = [&](int s, bf16x8 (&bf)[3]) {
            const int off = lrow + ((stp[s] >> 3) << 8) + (((stp[s] & 7) << 5) ^ lx);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
              bf[pl] = *reinterpret_cast<const bf16x8 *>(Yp + pl * YPL + off);
          };
          bf16x8 bfb[2][3];
          if (my_steps > 0) load_bf(0, bfb[0]);
#pragma unroll
          for (int s = 0; s < MAXS; ++s) {
            if (s >= my_steps) break;
            if (s + 1 < MAXS && s + 1 < my_steps) load_bf(s + 1, bfb[(s + 1) & 1]);
            wacc[ch] = mfma6(ain[s], bfb[s & 1], wacc[ch]);
          }
          KCNN_TMARK(1)
          if (ch == 0 && nprev >= 0) col2im(nprev);
          // the next frame's im2col values (its map went to Xs two barriers
          // ago; this slab's MFMAs were the last readers of ain)
          if (ch == NCH - 1 && n + G < g.R) gather(ain);
        }
        if (RD && ch == NCH - 1) store_z();
        KCNN_TMARK(2)
        __syncthreads();  // Ba: the image of slab t is read no more
        KCNN_TMARK(3)
        if (next) {
          // the wgrad waves split their unit here, beside the dgrad waves'
          // LDS writes (its planes are not held through the MFMA phase)
          if constexpr (!RD) {
            split_raw(UC{}, rx, rm, rsh, sres);
            if (n2 < g.R) load_raw(UC{}, rx, rm, rsh, n2, c2);
          }
          write_sres(UC{}, sres);
        }
        // the map of the frame after next (Xs was last read by this slab's gather)
        if (ch == NCH - 1 && n + 2 * G < g.R) commit_x();
        __syncthreads();  // Bb: slab t+1 published
        KCNN_TMARK(4)
      }
      nprev = n;
    }
    __syncthreads();  // the last frame's Z
    if (nprev >= 0) col2im(nprev);
#ifdef KCNN_PHASE_TIMING
    if ((dbg & 16) && blockIdx.x == 0 && lane == 0)
      printf("bwdx6p wave %d: split %lld mfma %lld frame %lld Ba %lld write+Bb %lld top %lld\n",
             wave, tm[0], tm[1], tm[2], tm[3], tm[4], tm[5]);
#endif
    // the wgrad waves' partials summed in a fixed order, as conv_bwd_x6_kernel
    const int E = (g.Kdim + 1) * g.G;
    float *dst = ws_part + (int64_t)blockIdx.x * E;
    float *red = reinterpret_cast<float *>(Yp);
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      __syncthreads();
      if constexpr (!RD) {
#pragma unroll
        for (int r = 0; r < 16; r++)
          red[(wave - 4) * 1024 + mfma32_row(r, lane) * 32 + l] = wacc[ch][r];
      }
      __syncthreads();
      for (int e = tid; e < 1024; e += NT) {
        const int i = e >> 5, j = e & 31;
        if (i > g.Kdim) continue;
        float sum = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; w++) sum += red[w * 1024 + e];
        // (dbg bit 30: add to the partial an earlier frame range left there)
        dst[i * g.G + ch * 32 + j] = (dbg & (1 << 30)) ? dst[i * g.G + ch * 32 + j] + sum : sum;
      }
    }
  };
  if (dgrad_wave) frames(std::integral_constant<int, 1>{});
  else frames(std::integral_constant<int, 2>{});
#undef KCNN_TMARK
}
#endif  // KCNN_EXPERIMENTS

// ---------------------------------------------------------------------------
// conv_bwd_x6q_kernel: conv_bwd_x6p_kernel's math bit for bit (the same image
// contents, fragments and MFMA order into every accumulator), with the slab
// image consumed in two position halves so that its LDS writes run beside
// the MFMAs instead of between them.
//
// Half A = positions 0-255 (dgrad tiles 0-7: tiles w and w + 4 of dgrad wave
// w; wgrad steps 0-15: steps 0-3 of every wgrad wave), half B = 256-383
// (tile w + 8; steps 4-5).  Every accumulator still sees its MFMAs in the
// same order: a dgrad tile lives in one half, and a wgrad wave's A steps come
// before its B steps.  Per slab t, two phases a barrier apart:
//
//   P_A(t)  MFMAs on half A of slab t; the B-half planes of slab t -> image
//           (split during P_B(t-1)); the A units of slab t+1 split
//   P_B(t)  MFMAs on half B of slab t; the A-half planes of slab t+1 -> image;
//           the B units of slab t+1 split
//
// so one LDS image serves both halves and each phase pairs one half's MFMAs
// with the other half's stores.  Split units: A unit u (quad u % 64 of
// pooled row u / 64) belongs to thread u, B unit u (positions 256 + ...) to
// dgrad-wave thread u.  Frame work sits where an accumulator's last reader
// is behind a barrier: the wgrad waves gather the next frame's A-step
// im2col values in P_A of the last slab, behind that phase's MFMAs on them
// (KCNN_X6Q_GA of them; the rest in its P_B), and its B-step values in P_A
// of the first; the next frame's map goes to Xs in P_B of the first slab; the
// dgrad waves col2im the previous frame over P_A of every slab (from a
// per-element tap table, ahead of the last slab's store of Z; on the wgrad
// waves instead it measured 205 against 174 us).
//
// The steady-state loop issues its global loads and stores on every path
// (buffer loads and stores past the buffer's range stand in for the lanes
// and frames that have none): a load or store under a branch, or in a loop
// of unknown trip count, leaves the compiler unsure how many vector-memory
// operations are younger than the one a split waits for, and it then waits
// for all of them (vmcnt(0)), the prefetch just issued included.  For the
// same reason a phase issues its dX stores before its raw-value loads.
template <int NCH, int PCM, int PH>
__global__ __launch_bounds__(NT, 1) void conv_bwd_x6q_kernel(
    ConvGeom g, const float *__restrict__ X, int xs, const float *__restrict__ dP, int dps,
    const float *__restrict__ K, int ks, float *__restrict__ dX, int dxs,
    float *__restrict__ ws_part, int ZZ, X6Steps steps, int dx_acc,
    const unsigned char *__restrict__ pmask, int pms, int dbg) {
  static_assert(NCH >= 2 && PCM > 0, "pooled backward with >= 2 slabs per frame");
  extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef KCNN_PHASE_TIMING  // per-phase clock totals of block 0's waves (dbg & 16)
  long long tm[5 * NCH] = {};
  long long tprev = clock64();
#define KCNN_TMARK(i)               \
  if (dbg & 16) {                   \
    const long long tn = clock64(); \
    tm[i] += tn - tprev;            \
    tprev = tn;                     \
  }
// timing experiments that skip work (wrong results): 32 no image stores, 64
// no MFMAs, 128 no splits, 256 no frame work (gather, col2im, map, Z), 512
// no gather, 1024 no col2im
#define KCNN_SKIP(b) (dbg & (b))
#else
#define KCNN_TMARK(i)
#define KCNN_SKIP(b) false
  (void)dbg;
#endif
  (void)ZZ;
  using MaskT = typename std::conditional<(PH > 1), unsigned short, unsigned char>::type;
  constexpr int MB = (int)sizeof(MaskT);
  constexpr int NJ = 32 / PCM;  // pooled rows per slab
  constexpr int HALF = 256;     // positions of half A
  constexpr int SA = HALF / 16 / 4;  // wgrad steps per wave in half A
  constexpr int MAXC = 2 * MAXX;     // col2im elements per dgrad-wave thread
  const int P = g.P;
  const int Q = P / PH;
  const int Hp = g.H + 2 * g.pad_h, Wp = g.W + 2 * g.pad_w;
  const int CHWp = g.C * Hp * Wp;
  char *Yp = smem;                                            // [3][32][384] bf16
  char *Wimg = Yp + 3 * YPL;                                  // [3][32][128] bf16
  float *Zt = reinterpret_cast<float *>(Wimg + 3 * WPL);      // [Kdim][PZ]
  // the padded map + {1}, split once per frame: element e is (m << 16 | h, l)
  // of its three bf16 parts (bf16-split.h), so the wgrad waves' im2col
  // gather packs fragments from them (3 v_perm per pair) instead of splitting
  // every gathered copy of a value (11 VALU per pair; each value is gathered
  // kh * kw times)
  uint2 *Xs = reinterpret_cast<uint2 *>(Zt + g.Kdim * PZ);
  int *qtab = reinterpret_cast<int *>(Xs + round4(CHWp + 1));  // [384]
  // col2im taps of each dX element (kw == 1, kh <= 8): Z offset | ylo << 16 |
  // ny << 20, the same every frame
  int *ctab = qtab + PP;  // [CHW]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = lane & 31, hf = lane >> 5;
  const int CHW = g.C * g.HW;
  const bool unpadded = g.pad_h == 0 && g.pad_w == 0;
  const int ntile = (P + 31) >> 5;
  const int PW = (P + 15) & ~15;
  const int NPQ = PW >> 2;
  const int NPQA = min(NPQ, HALF / 4), NPQB = NPQ - NPQA;
  const int G = (int)gridDim.x;
  const int rowf = (g.G / PCM) * Q;

  for (int e = tid; e < 32 * 64; e += NT) {
    const int k = e >> 6, gg = (e & 63) * 2;
    const float v0 = (k < g.Kdim && gg < g.G) ? K[(int64_t)k * ks + gg] : 0.0f;
    const float v1 = (k < g.Kdim && gg + 1 < g.G) ? K[(int64_t)k * ks + gg + 1] : 0.0f;
    uint32_t h, m, lo;
    split2(v0, v1, h, m, lo);
    const int o = woff(k, gg);
    *reinterpret_cast<uint32_t *>(Wimg + o) = h;
    *reinterpret_cast<uint32_t *>(Wimg + WPL + o) = m;
    *reinterpret_cast<uint32_t *>(Wimg + 2 * WPL + o) = lo;
  }
  // byte offsets into Xs (8 B per element)
  uint32_t abase = (uint32_t)CHWp * 8, qmul = 0;
  if (l < g.Kdim) {
    uint32_t c, r, qx, qy;
    g.div_khkw.divmod((uint32_t)l, c, r);
    g.div_kh.divmod(r, qx, qy);
    abase = ((uint32_t)c * Hp * Wp + qx * Hp + qy) * 8;
    qmul = 1;
  }
  for (int e = tid; e < CHWp; e += NT) Xs[e] = make_uint2(0u, 0u);
  if (tid == 0) Xs[CHWp] = make_uint2(0x3f80u, 0u);  // 1.0f = h alone
  for (int p = tid; p < PP; p += NT) {
    uint32_t px, py;
    g.div_oh.divmod((uint32_t)p, px, py);
    // past P: past every lane's range (the clamp below reads the 1.0 entry)
    qtab[p] = p < P ? ((int)px * Hp + (int)py) * 8 : 0x00ffffff;
  }
  const int khkw0 = g.kh * g.kw;
  const bool c2fast = g.kw == 1 && g.kh <= 8;
  if (c2fast) {
    for (int e = tid; e < g.C * g.HW; e += NT) {
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)e, c, q);
      g.div_H.divmod(q, wi, hi);
      const int ty = (int)hi + g.pad_h, tx = (int)wi + g.pad_w;
      const int ylo = max(0, ty - g.oh + 1), ny = min(g.kh - 1, ty) - ylo;
      ctab[e] = ((int)c * khkw0 * PZ + tx * g.oh + ty) | (ylo << 16) | (ny << 20);
    }
  }
  const uint32_t amax = (uint32_t)CHWp * 8;
  const char *Xb = reinterpret_cast<const char *>(Xs);

  // ---- split units: (pooled row j, position quad p0), the same in every slab
  struct Unit {
    int j, p0, base, x0, x1;
    bool on;
  };
  auto make_unit = [&](int u, int npq, int pfirst) {
    Unit U;
    U.on = u < NJ * npq;
    const int uu = U.on ? u : 0;
    U.j = npq > 0 ? uu / npq : 0;
    U.p0 = pfirst + (uu - U.j * npq) * 4;
    const int r0 = PCM * U.j;
    U.base = r0 * ROWB + ((U.p0 >> 7) << 8) + ((U.p0 & 7) << 1);
    U.x0 = ((U.p0 >> 3) & 15) ^ ((r0 >> 2) & 3);
    U.x1 = ((U.p0 >> 3) & 15) ^ (((r0 >> 2) + 1) & 3);
    return U;
  };
  constexpr int NX = PH > 1 ? 2 : 4;
  auto load_raw = [&](const Unit &U, float (&rx)[NX], uint32_t (&rm)[2], int &rsh, int nn,
                      int cc) {
    // no branch: a unit that is off reads past the buffer (0s, unused), so
    // every path issues the same loads and the compiler's vmcnt waits stay
    // exact (a conditional load makes them vmcnt(0), which then also waits
    // for the dX stores)
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(dP + (int64_t)nn * dps), (short)0, rowf * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(pmask + (int64_t)nn * pms), (short)0, rowf * MB, 0x00020000);
    const int s = (cc * NJ + U.j) * Q + (PH > 1 ? U.p0 / PH : U.p0);
    const unsigned oob = 0x40000000u;
    if constexpr (NX == 4) {
      const auto v =
          __builtin_amdgcn_raw_buffer_load_b128(rd, U.on ? (unsigned)s * 4u : oob, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) rx[q] = __uint_as_float(v[q]);
    } else {
      const auto v =
          __builtin_amdgcn_raw_buffer_load_b64(rd, U.on ? (unsigned)s * 4u : oob, 0, 0);
      rx[0] = __uint_as_float(v[0]);
      rx[1] = __uint_as_float(v[1]);
    }
    const unsigned mo = (unsigned)s * MB;
    const auto w = __builtin_amdgcn_raw_buffer_load_b64(rk, U.on ? mo & ~3u : oob, 0, 0);
    rm[0] = w[0];
    rm[1] = w[1];
    rsh = (int)(mo & 3u);
  };
  auto split_raw = [&](const Unit &U, const float (&rx)[NX], const uint32_t (&rm)[2],
                       int rsh, uint32_t (&sres)[PCM][6]) {
    if (!U.on || KCNN_SKIP(128)) return;
    const int p0 = U.p0;
    const uint32_t mw = __builtin_amdgcn_alignbyte(rm[1], rm[0], (uint32_t)rsh);
    float x[4];
    unsigned mk[4];
    short rq[4];
    if constexpr (PH > 1) {
      const int pq0 = p0 / PH, r0 = p0 - pq0 * PH;
      const unsigned m0 = mw & 0xffffu, m1 = mw >> 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool sel = r0 + q >= PH;
        rq[q] = (short)(r0 + q - (sel ? PH : 0));
        x[q] = sel ? rx[1] : rx[0];
        mk[q] = p0 + q < P ? (sel ? m1 : m0) : 0u;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        rq[q] = 0;
        x[q] = rx[q];
        mk[q] = p0 + q < P ? (mw >> (8 * q)) & 0xffu : 0u;
      }
    }
    uint32_t h01, m01, l01, h23, m23, l23;
    split2(x[0], x[1], h01, m01, l01);
    split2(x[2], x[3], h23, m23, l23);
    const s16x2 w01 = __builtin_bit_cast(s16x2, mk[0] | (mk[1] << 16));
    const s16x2 w23 = __builtin_bit_cast(s16x2, mk[2] | (mk[3] << 16));
    const s16x2 b01 = {(short)(15 - rq[0]), (short)(15 - rq[1])};
    const s16x2 b23 = {(short)(15 - rq[2]), (short)(15 - rq[3])};
#pragma unroll
    for (int c = 0; c < PCM; ++c) {
      const s16x2 cc = {(short)(c * PH), (short)(c * PH)}, k15 = {15, 15};
      const s16x2 sh01 = b01 - cc, sh23 = b23 - cc;
      const uint32_t s01 = __builtin_bit_cast(uint32_t, (s16x2)((w01 << sh01) >> k15));
      const uint32_t s23 = __builtin_bit_cast(uint32_t, (s16x2)((w23 << sh23) >> k15));
      sres[c][0] = h01 & s01;
      sres[c][1] = h23 & s23;
      sres[c][2] = m01 & s01;
      sres[c][3] = m23 & s23;
      sres[c][4] = l01 & s01;
      sres[c][5] = l23 & s23;
    }
  };
  auto write_sres = [&](const Unit &U, const uint32_t (&sres)[PCM][6]) {
    if (!U.on || KCNN_SKIP(32)) return;
#pragma unroll
    for (int c = 0; c < PCM; ++c) {
      const int ux = (c >> 2) ? U.x1 : U.x0;
      const int o = U.base + c * ROWB + ((ux ^ ((c & 3) << 2)) << 4);
      *reinterpret_cast<uint2 *>(Yp + o) = make_uint2(sres[c][0], sres[c][1]);
      *reinterpret_cast<uint2 *>(Yp + YPL + o) = make_uint2(sres[c][2], sres[c][3]);
      *reinterpret_cast<uint2 *>(Yp + 2 * YPL + o) = make_uint2(sres[c][4], sres[c][5]);
    }
  };

  float xv[MAXX];
  auto load_x = [&](int n) {  // branch-free, as load_raw
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(X + (int64_t)n * xs), (short)0, CHW * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < MAXX; i++)
      xv[i] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rx, (unsigned)(tid + NT * i) * 4u, 0, 0));
  };
  auto commit_x = [&]() {
#pragma unroll
    for (int i = 0; i < MAXX; i++) {
      const int e = tid + NT * i;
      if (e < CHW) {
        int slot = e;
        if (!unpadded) {
          uint32_t c, q, wi, hi;
          g.div_HW.divmod((uint32_t)e, c, q);
          g.div_H.divmod(q, wi, hi);
          slot = (int)c * Hp * Wp + ((int)wi + g.pad_w) * Hp + (int)hi + g.pad_h;
        }
        uint32_t h, m, lo;  // bf16-split.h's parts of the one value (its split2 bits)
        split2(xv[i], xv[i], h, m, lo);
        Xs[slot] = make_uint2((m << 16) | (h & 0xffffu), lo & 0xffffu);
      }
    }
  };
  const int khkw = g.kh * g.kw;
  const int zax = g.kh * PZ - g.oh, zby = PZ - 1;
  const int ZMAX = g.Kdim * PZ - 1;  // (a tap past kh reads in-bounds Z, masked off)
  // elements tid + 256 i, i in [I0, I1), of the dgrad waves' share; a fixed
  // trip count and buffer stores (an element past the map is stored past
  // the row and dropped) keep the compiler's vmcnt counts exact
  auto col2im_v = [&](int nn, int I0, int I1, auto ACCc) {
    constexpr bool ACC = decltype(ACCc)::value;
    const __amdgpu_buffer_rsrc_t rdx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(dX + (int64_t)nn * dxs), (short)0, CHW * 4, 0x00020000);
    if (c2fast) {  // two elements at a time from the tap table (same sums, same order)
#pragma unroll 1
      for (int i = I0; i < I1; i += 2) {
        int e[2], t[2];
        float v[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          e[h] = tid + (NT / 2) * (i + h);
          t[h] = ctab[min(e[h], CHW - 1)];
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int u = 0; u < 8; u++) v[h][u] = Zt[min((t[h] & 0xffff) + u * zby, ZMAX)];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ylo = (t[h] >> 16) & 15, ny = t[h] >> 20;
          float sum = 0.0f;
#pragma unroll
          for (int u = 0; u < 8; u++) sum += (unsigned)(u - ylo) <= (unsigned)ny ? v[h][u] : 0.0f;
          const unsigned off = e[h] < CHW && i + h < I1 ? (unsigned)e[h] * 4u : 0x40000000u;
          if constexpr (ACC)
            sum += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rdx, off, 0, 0));
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sum), rdx, off, 0, 0);
        }
      }
      return;
    }
#pragma unroll 1
    for (int i = I0; i < I1; i++) {
      const int e = tid + (NT / 2) * i;
      const int ec = min(e, CHW - 1);
      uint32_t c, q, wi, hi;
      g.div_HW.divmod((uint32_t)ec, c, q);
      g.div_H.divmod(q, wi, hi);
      const int ty = (int)hi + g.pad_h, tx = (int)wi + g.pad_w;
      const int zb = (int)c * khkw * PZ + tx * g.oh + ty;
      const int ylo = max(0, ty - g.oh + 1), ny = min(g.kh - 1, ty) - ylo;
      const int xlo = max(0, tx - g.ow + 1), xhi = min(g.kw - 1, tx);
      float sum = 0.0f;
      for (int kx = xlo; kx <= xhi; kx++) {
        const int zk = zb + kx * zax;
        for (int k0 = 0; k0 < g.kh; k0 += 8) {
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; u++) v[u] = Zt[zk + (k0 + u) * zby];
#pragma unroll
          for (int u = 0; u < 8; u++)
            sum += (unsigned)(k0 + u - ylo) <= (unsigned)ny ? v[u] : 0.0f;
        }
      }
      const unsigned off = e < CHW ? (unsigned)e * 4u : 0x40000000u;
      if constexpr (ACC)  // (a runtime test here became an unconditional load + wait)
        sum += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rdx, off, 0, 0));
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, sum), rdx, off, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // one element's temporaries at a time
    }
  };
  auto col2im = [&](int nn, int I0, int I1) {
    if (dx_acc) col2im_v(nn, I0, I1, std::true_type{});
    else col2im_v(nn, I0, I1, std::false_type{});
  };

  const bool dgrad_wave = wave < 4;
  int my_steps = 0;
  int stp[MAXS];
#pragma unroll
  for (int s = 0; s < MAXS; ++s) {
    stp[s] = steps.s[wave][s];
    if (!dgrad_wave && stp[s] != 0xff) my_steps = s + 1;
  }
  // the frame's im2col values of this wave's steps [S0, S1), split once per
  // frame: every step's offsets (two 16-B qtab reads), then every value, then
  // the splits, so the LDS round trips overlap (a step past my_steps reads
  // clamped, in-bounds addresses; its planes are never used)
  auto gather = [&](auto &a, auto S0c, auto S1c) {
    constexpr int S0 = decltype(S0c)::value, S1 = decltype(S1c)::value;
    constexpr int NS = S1 - S0;
    int4 qv[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int pbase = min(16 * stp[S0 + s] + 8 * hf, PP - 8);
      qv[s][0] = *reinterpret_cast<const int4 *>(qtab + pbase);
      qv[s][1] = *reinterpret_cast<const int4 *>(qtab + pbase + 4);
    }
    uint2 v[NS][8];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int q[8] = {qv[s][0].x, qv[s][0].y, qv[s][0].z, qv[s][0].w,
                        qv[s][1].x, qv[s][1].y, qv[s][1].z, qv[s][1].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        // (24-bit multiply: one full-rate mad; qmul is 0 or 1)
        const uint32_t off = min(__umul24(qmul, (uint32_t)q[e]) + abase, amax);
        v[s][e] = *reinterpret_cast<const uint2 *>(Xb + off);
      }
    }
    // the three planes' fragments from the pre-split parts: the same bits
    // split8 gives for the values
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      uint32_t hh[4], mm[4], ll[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint2 w0 = v[s][2 * i], w1 = v[s][2 * i + 1];
        hh[i] = __builtin_amdgcn_perm(w1.x, w0.x, 0x05040100u);
        mm[i] = __builtin_amdgcn_perm(w1.x, w0.x, 0x07060302u);
        ll[i] = __builtin_amdgcn_perm(w1.y, w0.y, 0x05040100u);
      }
      a[S0 + s][0] = __builtin_bit_cast(bf16x8, make_uint4(hh[0], hh[1], hh[2], hh[3]));
      a[S0 + s][1] = __builtin_bit_cast(bf16x8, make_uint4(mm[0], mm[1], mm[2], mm[3]));
      a[S0 + s][2] = __builtin_bit_cast(bf16x8, make_uint4(ll[0], ll[1], ll[2], ll[3]));
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using CA = std::integral_constant<int, SA>;
  using CS = std::integral_constant<int, MAXS>;
  // A steps of the next frame gathered in P_A of the last slab, the rest in
  // its P_B (c2 pooled backward, 3 runs each: 0 178.5 us, 1 179.1, 2 176.7,
  // 4 174.6; moving the dgrad waves' col2im shares to P_B measured 184.5)
#ifndef KCNN_X6Q_GA
#define KCNN_X6Q_GA 4
#endif
  constexpr int GA = KCNN_X6Q_GA;
  static_assert(GA >= 0 && GA <= SA, "A-step gather split");
  using CGA = std::integral_constant<int, GA>;

  const int n0 = blockIdx.x;
  auto frames = [&](auto role) {
    constexpr bool RD = decltype(role)::value == 1;  // dgrad waves
    const Unit ua = make_unit(tid, NPQA, 0);
    const Unit ub = make_unit(RD ? tid : NT, NPQB, HALF);
    float rxA[NX], rxB[NX];
    uint32_t rmA[2], rmB[2];
    int rshA = 0, rshB = 0;
    uint32_t sresA[PCM][6], sresB[PCM][6];
    bf16x8 ain[RD ? 1 : MAXS][3];
#pragma unroll
    for (int s = 0; s < (RD ? 1 : MAXS); ++s)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) ain[s][pl] = bf16x8{};
    // ---- prologue: frame n0's map and A-step im2col values, the A half of
    // its first slab in the image, the B half split, slab 1's raw values
    load_x(n0);
    load_raw(ua, rxA, rmA, rshA, n0, 0);
    if constexpr (RD) load_raw(ub, rxB, rmB, rshB, n0, 0);
    __syncthreads();  // Xs zeroed, qtab and the W image written
    commit_x();
    if (n0 + G < g.R) load_x(n0 + G);
    split_raw(ua, rxA, rmA, rshA, sresA);
    if constexpr (RD) split_raw(ub, rxB, rmB, rshB, sresB);
    load_raw(ua, rxA, rmA, rshA, n0, 1);
    if constexpr (RD) load_raw(ub, rxB, rmB, rshB, n0, 1);
    write_sres(ua, sresA);
    __syncthreads();  // A(n0, 0) in the image, frame n0's map in Xs
    if constexpr (!RD) gather(ain, C0{}, CA{});

    floatx16 wacc[RD ? 1 : NCH];
#pragma unroll
    for (int c = 0; c < (RD ? 1 : NCH); c++) wacc[c] = zero16();
    int nprev = -1;

    for (int n = n0; n < g.R; n += G) {
      constexpr int TT = RD ? MAXT : 1;
      floatx16 zacc[TT];
#pragma unroll
      for (int t = 0; t < TT; ++t) zacc[t] = zero16();
      auto tile_of = [&](int t) { return wave + 4 * t; };
      // Z[p][k] += dY^T W on this wave's tiles [T0, T1): MFMA group gi = (tile
      // gi / 2, k16 slice gi % 2), the next group's transposed reads issued
      // before the current group's MFMAs
      auto dgrad = [&](int ch, auto T0c, auto T1c) {
        constexpr int T0 = decltype(T0c)::value, T1 = decltype(T1c)::value;
        if (tile_of(T0) >= ntile) return;
        bf16x8 wf[2][3];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            wf[s][pl] = *reinterpret_cast<const bf16x8 *>(
                Wimg + pl * WPL + woff(l, ch * 32 + 16 * s + 8 * hf));
        const int G4 = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
        auto load_af = [&](int gi, bf16x8 (&af)[3]) {
          const int col = tile_of(gi >> 1) * 32 + 16 * (G4 & 1) + 4 * pp;
          const int row = 16 * (gi & 1) + 8 * (G4 >> 1) + q;
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4 *)(Yp + pl * YPL + yoff(row, col)));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_s16x4 *)(Yp + pl * YPL + yoff(row + 4, col)));
            af[pl] = __builtin_bit_cast(
                bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
          }
        };
        bf16x8 afb[2][3];
        load_af(2 * T0, afb[0]);
#pragma unroll
        for (int gi = 2 * T0; gi < 2 * T1; ++gi) {
          if (tile_of(gi >> 1) >= ntile) break;  // uniform
          if (gi + 1 < 2 * T1) load_af(gi + 1, afb[(gi + 1 - 2 * T0) & 1]);  // unconditional
          __builtin_amdgcn_sched_barrier(0);
          if (!KCNN_SKIP(64))
            zacc[gi >> 1] = mfma6(afb[(gi - 2 * T0) & 1], wf[gi & 1], zacc[gi >> 1]);
        }
      };
      // gW[k][g] += im2col(X) dY^T over this wave's k16 steps [S0, S1) (the
      // next step's row reads issued before the current step's MFMAs; the
      // lane part of the address passes through an opaque move, so the
      // compiler does not hoist per-step addresses out of the frame loop)
      auto wgrad = [&](int ch, auto S0c, auto S1c) {
        constexpr int S0 = decltype(S0c)::value, S1 = decltype(S1c)::value;
        if (S0 >= my_steps) return;
        int lx, lrow;
        asm volatile("v_mov_b32 %0, %1" : "=v"(lx) : "v"((hf ^ swz4(l)) << 4));
        asm volatile("v_mov_b32 %0, %1" : "=v"(lrow) : "v"(l * ROWB));
        auto load_bf = [&](int s, bf16x8 (&bf)[3]) {
          const int off = lrow + ((stp[s] >> 3) << 8) + (((stp[s] & 7) << 5) ^ lx);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            bf[pl] = *reinterpret_cast<const bf16x8 *>(Yp + pl * YPL + off);
        };
        bf16x8 bfb[2][3];
        load_bf(S0, bfb[0]);
#pragma unroll
        for (int s = S0; s < S1; ++s) {
          if (s >= my_steps) break;
          // the prefetch is unconditional (a step past my_steps reads unused
          // in-bounds LDS): a branch here would make the compiler's LDS wait
          // counts at the MFMAs conservative and serialise the reads
          if (s + 1 < S1) load_bf(s + 1, bfb[(s + 1 - S0) & 1]);
          __builtin_amdgcn_sched_barrier(0);  // the next step's reads stay ahead of these MFMAs
          if (!KCNN_SKIP(64)) wacc[ch] = mfma6(ain[s], bfb[(s - S0) & 1], wacc[ch]);
        }
      };
      auto store_z = [&]() {
#pragma unroll
        for (int t = 0; t < TT; ++t) {
          const int pt = tile_of(t);
          if (pt >= ntile) break;
          if (l < g.Kdim) {
            float *zr = Zt + l * PZ + pt * 32 + 4 * hf;
#pragma unroll
            for (int i = 0; i < 4; i++)
              *reinterpret_cast<float4 *>(zr + 8 * i) =
                  make_float4(zacc[t][4 * i], zacc[t][4 * i + 1], zacc[t][4 * i + 2],
                              zacc[t][4 * i + 3]);
          }
        }
      };
#pragma unroll
      for (int ch = 0; ch < NCH; ch++) {
        const int n1 = ch + 1 < NCH ? n : n + G;
        const int n2 = ch + 2 < NCH ? n : n + G, c2 = ch + 2 < NCH ? ch + 2 : ch + 2 - NCH;
        const bool next = n1 < g.R;
        KCNN_TMARK(5 * ch + 4)
        // ---- P_A(t): half A's MFMAs; slab t's B planes -> image; A(t+1) split
        if constexpr (RD) {
          write_sres(ub, sresB);
          // the previous frame's dX (its Z went to LDS before the last Bb;
          // this frame's store of Z is in P_B of its last slab), here where
          // the fewest registers are live, beside the wgrad waves' MFMAs
          if (nprev >= 0 && !KCNN_SKIP(256 | 1024)) {  // spread over the frame's P_A phases
            constexpr int PER = (MAXC + NCH - 1) / NCH;
            col2im(nprev, ch * PER, min((ch + 1) * PER, MAXC));
          }
          if (next) {
            split_raw(ua, rxA, rmA, rshA, sresA);
            load_raw(ua, rxA, rmA, rshA, min(n2, g.R - 1), c2);
          }
          dgrad(ch, std::integral_constant<int, 0>{}, std::integral_constant<int, 2>{});
        } else {
          wgrad(ch, C0{}, CA{});
          if (next) {
            split_raw(ua, rxA, rmA, rshA, sresA);
            load_raw(ua, rxA, rmA, rshA, min(n2, g.R - 1), c2);
          }
          // frame n's B-step values (their last reader: P_B of frame n - G's
          // last slab; Xs holds frame n's map until P_B of this slab)
          if (ch == 0 && !KCNN_SKIP(256 | 512)) gather(ain, CA{}, CS{});
          // the next frame's first GA A-step values, behind this phase's MFMAs
          // on them (Xs has held the next frame's map since P_B of the first
          // slab): the wgrad waves' P_A is the shorter of the two roles'
          if constexpr (GA > 0)
            if (ch == NCH - 1 && n + G < g.R && !KCNN_SKIP(256 | 512)) gather(ain, C0{}, CGA{});
        }
        KCNN_TMARK(5 * ch + 0)
        __syncthreads();  // Ba: half A of slab t read, its B half published
        KCNN_TMARK(5 * ch + 1)
        // ---- P_B(t): half B's MFMAs; A(t+1) -> image; B(t+1) split
        if (next) write_sres(ua, sresA);
        if constexpr (RD) {
          if (next) {
            split_raw(ub, rxB, rmB, rshB, sresB);
            load_raw(ub, rxB, rmB, rshB, min(n2, g.R - 1), c2);
          }
          dgrad(ch, std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{});
          if (ch == NCH - 1 && !KCNN_SKIP(256)) store_z();
        } else {
          wgrad(ch, CA{}, CS{});
          // the next frame's other A-step values (their last reader was P_A
          // of this slab; its map went to Xs in P_B of the first slab)
          if constexpr (GA < SA)
            if (ch == NCH - 1 && n + G < g.R && !KCNN_SKIP(256 | 512)) gather(ain, CGA{}, CA{});
        }
        if (ch == 0) {
          if (n + G < g.R) commit_x();
          load_x(min(n + 2 * G, g.R - 1));  // unconditional (a clamped frame: unused)
        }
        KCNN_TMARK(5 * ch + 2)
        __syncthreads();  // Bb: slab t read, A(t+1) published
        KCNN_TMARK(5 * ch + 3)
      }
      nprev = n;
    }
    if (RD && nprev >= 0) col2im(nprev, 0, MAXC);  // the last frame's Z (stored before the last Bb)
#ifdef KCNN_PHASE_TIMING
    if ((dbg & 16) && blockIdx.x == 0 && lane == 0)
      for (int c = 0; c < NCH; ++c)
        printf("bwdx6q wave %d ch %d: PA %lld Ba %lld PB %lld Bb %lld top %lld\n", wave, c,
               tm[5 * c], tm[5 * c + 1], tm[5 * c + 2], tm[5 * c + 3], tm[5 * c + 4]);
#endif
    const int E = (g.Kdim + 1) * g.G;
    float *dst = ws_part + (int64_t)blockIdx.x * E;
    float *red = reinterpret_cast<float *>(Yp);
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
      __syncthreads();
      if constexpr (!RD) {
#pragma unroll
        for (int r = 0; r < 16; r++)
          red[(wave - 4) * 1024 + mfma32_row(r, lane) * 32 + l] = wacc[ch][r];
      }
      __syncthreads();
      for (int e = tid; e < 1024; e += NT) {
        const int i = e >> 5, j = e & 31;
        if (i > g.Kdim) continue;
        float sum = 0.0f;
#pragma unroll
        for (int w = 0; w < 4; w++) sum += red[w * 1024 + e];
        // (dbg bit 30: add to the partial an earlier frame range left there)
        dst[i * g.G + ch * 32 + j] = (dbg & (1 << 30)) ? dst[i * g.G + ch * 32 + j] + sum : sum;
      }
    }
  };
  if (dgrad_wave) frames(std::integral_constant<int, 1>{});
  else frames(std::integral_constant<int, 2>{});
#undef KCNN_TMARK
#undef KCNN_SKIP
}

size_t x6q_lds(const ConvGeom &g);
size_t x6p_lds(const ConvGeom &g) {
  const int CHWp = g.C * (g.H + 2 * g.pad_h) * (g.W + 2 * g.pad_w);
  return (size_t)3 * YPL + 3 * WPL + (size_t)g.Kdim * PZ * 4 +
         (size_t)round4(CHWp + 1) * 4 + (size_t)PP * 4;
}

// conv_bwd_x6q_kernel: x6p's plan and the col2im tap table
// (and the map's split parts, 8 B per element instead of x6p's 4)
size_t x6q_lds(const ConvGeom &g) {
  const int CHWp = g.C * (g.H + 2 * g.pad_h) * (g.W + 2 * g.pad_w);
  return x6p_lds(g) + (size_t)round4(g.C * g.HW) * 4 + (size_t)round4(CHWp + 1) * 4;
}

size_t x6_lds(const ConvGeom &g, bool dx, int pc, int ph) {
  const int CHWp = g.C * (g.H + 2 * g.pad_h) * (g.W + 2 * g.pad_w);
  const int ZZ = g.Kdim | 1;
  return (size_t)3 * YPL + (dx ? 3 * WPL : 0) +
         (dx && pc > 0 ? (size_t)round4(g.P * ZZ) * 4 : 0) +
         (size_t)round4(CHWp + 1) * 4 + (size_t)PP * 4 +
         (size_t)x6_stage_floats(g.P, pc, ph) * 4 + (size_t)x6_stage_mask_bytes(g.P, pc, ph);
}

}  // namespace

// Eligible shapes: Kdim <= 31, 1 <= P <= 384, G a multiple of 32 up to 128,
// C*H*W <= 2048, pc in {0, 4, 8}, a pool window ph x 1 x pc with ph in
// {1, 2, 3} dividing oh and ph * pc <= 16, and the LDS plan within 160 KB.
bool kcnn_conv_bwd_x6_eligible(const ConvGeom &g, bool dx, int pc, int ph) {
  if (g.Kdim > 31 || g.Kdim < 1 || g.P < 1 || g.P > PP) return false;
  if (g.G % 32 != 0 || g.G > 128 || g.G == 0) return false;
  if (g.C * g.HW > NT * MAXX) return false;
  if (!(pc == 0 || pc == 4 || pc == 8)) return false;
  if (ph < 1 || ph > 3 || (ph > 1 && (pc == 0 || ph * pc > 16 || g.oh % ph != 0)))
    return false;
  return x6_lds(g, dx, pc, ph) <= (size_t)160 * 1024;
}

// One filter chunk (G <= 128): the workgroup partials ws_part[S][(Kdim+1) G]
// (gW rows, then the bias row) for kcnn_conv_bwd_frame's reduction, S =
// gridDim = min(R, 256); dX written (or added, dx_acc) when dX != NULL.
int kcnn_conv_bwd_x6(const ConvGeom &g, const float *X, int xs, const float *dY, int dys,
                     const float *K, int ks, float *dX, int dxs, float *ws_part, int S,
                     int dx_acc, hipStream_t st, const unsigned char *pmask, int pms,
                     int pc, int ph, int dbg) {
  const bool dx = dX != nullptr, wg = ws_part != nullptr;
  if (!dx && !wg) return 0;
  if (!kcnn_conv_bwd_x6_eligible(g, dx, pc, ph)) return -1;
  // LDS-DMA of dP (16 B per lane) and of the mask (4 B per lane)
  if ((uintptr_t)dY % 16 || dys % 4) return -1;
  if (pc > 0 && ((uintptr_t)pmask % 4 || pms % 4)) return -1;
  // wgrad k16 steps dealt round-robin to waves 4-7 (the same table with or
  // without dX: it fixes how the gradient splits over the waves' partials)
  X6Steps tab;
  for (int w = 0; w < NW; ++w)
    for (int s = 0; s < MAXS; ++s) tab.s[w][s] = 0xff;
  {
    const int nstep = (g.P + 15) / 16;
    if (nstep > 4 * MAXS) return -1;
    for (int s = 0; s < nstep; ++s) tab.s[4 + s % 4][s / 4] = (uint8_t)s;
  }
  const int ZZ = g.Kdim | 1;
  // the software-pipelined kernel for the pooled backward with both outputs
  // (bitwise the same results); KCNN_BWD_X6P=0 (experiment build) keeps
  // conv_bwd_x6_kernel for it too
  static const int pipelined = KCNN_KNOB("KCNN_BWD_X6P", 2);
  const size_t plds = pipelined == 1 ? x6p_lds(g) : x6q_lds(g);
  if (pipelined && dx && wg && pc > 0 && g.G >= 64 && plds <= (size_t)160 * 1024) {
    const size_t lds = plds;
#define KCNN_X6PK(KER, NCH, PCM, PH)                                                       \
  do {                                                                                     \
    static bool attr = hipFuncSetAttribute(reinterpret_cast<const void *>(&KER<NCH, PCM, PH>), \
                                           hipFuncAttributeMaxDynamicSharedMemorySize,      \
                                           160 * 1024) == hipSuccess;                       \
    (void)attr;                                                                            \
    hipLaunchKernelGGL((KER<NCH, PCM, PH>), dim3(S), dim3(NT), lds, st, g, X, xs, dY, dys, K, \
                       ks, dX, dxs, ws_part, ZZ, tab, dx_acc, pmask, pms, dbg);            \
  } while (0)
#ifdef KCNN_EXPERIMENTS
#define KCNN_X6PP(NCH, PCM, PH)                                \
  do {                                                         \
    if (pipelined == 1) KCNN_X6PK(conv_bwd_x6p_kernel, NCH, PCM, PH); \
    else KCNN_X6PK(conv_bwd_x6q_kernel, NCH, PCM, PH);         \
  } while (0)
#else
#define KCNN_X6PP(NCH, PCM, PH) KCNN_X6PK(conv_bwd_x6q_kernel, NCH, PCM, PH)
#endif
#define KCNN_X6PM(NCH)                                      \
  do {                                                      \
    if (pc == 4 && ph == 3) KCNN_X6PP(NCH, 4, 3);           \
    else if (pc == 4 && ph == 2) KCNN_X6PP(NCH, 4, 2);      \
    else if (pc == 4) KCNN_X6PP(NCH, 4, 1);                 \
    else if (pc == 8 && ph == 2) KCNN_X6PP(NCH, 8, 2);      \
    else KCNN_X6PP(NCH, 8, 1);                              \
  } while (0)
    switch (g.G / 32) {
      case 2: KCNN_X6PM(2); break;
      case 3: KCNN_X6PM(3); break;
      default: KCNN_X6PM(4); break;
    }
#undef KCNN_X6PM
#undef KCNN_X6PP
#undef KCNN_X6PK
    return (int)hipGetLastError();
  }
  const size_t lds = x6_lds(g, dx, pc, ph);
#define KCNN_X6P(NCH, DXB, WGB, PCM, PH)                                                   \
  do {                                                                                     \
    static bool attr = hipFuncSetAttribute(                                               \
        reinterpret_cast<const void *>(&conv_bwd_x6_kernel<NCH, DXB, WGB, PCM, PH>),        \
        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;             \
    (void)attr;                                                                            \
    hipLaunchKernelGGL((conv_bwd_x6_kernel<NCH, DXB, WGB, PCM, PH>), dim3(S), dim3(NT), lds, \
                       st, g, X, xs, dY, dys, K, ks, dX, dxs, ws_part, ZZ, tab, dx_acc,     \
                       pmask, pms, dbg);                                                   \
  } while (0)
#define KCNN_X6M(NCH, DXB, WGB)                                  \
  do {                                                           \
    if (pc == 4 && ph == 3) KCNN_X6P(NCH, DXB, WGB, 4, 3);       \
    else if (pc == 4 && ph == 2) KCNN_X6P(NCH, DXB, WGB, 4, 2);  \
    else if (pc == 4) KCNN_X6P(NCH, DXB, WGB, 4, 1);             \
    else if (pc == 8 && ph == 2) KCNN_X6P(NCH, DXB, WGB, 8, 2);  \
    else if (pc == 8) KCNN_X6P(NCH, DXB, WGB, 8, 1);             \
    else KCNN_X6P(NCH, DXB, WGB, 0, 1);                          \
  } while (0)
#define KCNN_X6N(NCH)                          \
  do {                                         \
    if (dx && wg) KCNN_X6M(NCH, true, true);   \
    else if (wg) KCNN_X6M(NCH, false, true);   \
    else KCNN_X6M(NCH, true, false);           \
  } while (0)
  switch (g.G / 32) {
    case 1: KCNN_X6N(1); break;
    case 2: KCNN_X6N(2); break;
    case 3: KCNN_X6N(3); break;
    default: KCNN_X6N(4); break;
  }
#undef KCNN_X6N
#undef KCNN_X6M
#undef KCNN_X6P
  return (int)hipGetLastError();
}
