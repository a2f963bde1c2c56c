// kaldi-lite/cu-gemm-f16x3.hip -- fp32 GEMM on the f16 matrix cores from a
// two-part f16 split of each operand under a power-of-two scale per output
// row and column (the "f16x3" scheme, AddMatMat's default engine).
//
// Upstream Kaldi's CuMatrixBase::AddMatMat is cuBLAS sgemm; the reference
// calls it for the FullyConnectedComponent forward, data gradient and update
// (nnet-component.cc:1225-1227, :1247; nnet-component-nnet0.cc:1137-1142).
// The bf16x6 kernel (cu-gemm-x6.hip) reaches fp32 accuracy with six bf16
// products per fp32 product.  f16 carries 11 significant bits to bf16's 8,
// so two parts suffice once the operands are scaled into f16's range:
//
//   x' = x * 2^s   (s per row of op(A) / column of op(B): the row's largest
//                   |x'| lies in [2^14, 2^15))
//   hi = f16(x'),  lo = f16(x' - hi)        (x' - hi is exact in fp32)
//
// x' = hi + lo to within 2^-22 |x'| while |x'| >= 2^-3; below that lo is an
// f16 subnormal and the error is under 2^-25 absolute, 2^-39 of the row's
// largest element.  With every f16 product exact in fp32,
//
//   a'b' = hi.hi + (hi.lo + lo.hi) + lo.lo
//
// and the kernel keeps the first three (one v_mfma_f32_32x32x16_f16 each,
// smallest first, accumulated in fp32), then C = acc * 2^-(s_a + s_b) by an
// exact ldexp.  The error per product is under 3 * 2^-22 of |a b|, 14x inside
// the 1e-5 * S parity bound, and the f16 MFMA runs at the bf16
// rate: half the matrix-core work of bf16x6 for the same split VALU.  The
// scale also takes the operand range out of the question: a row of values
// near FLT_MAX or below 2^-110 is scaled like any other (the bf16x6 split
// loses bits there).
//
// The scales come from per-row / per-column max |x| (kl_absmax: the bit
// patterns of |x|, whose unsigned order is the magnitude order).  A row of
// op(A) or a column of op(B) holding Inf or NaN has no scale; every C
// element in it is Inf or NaN in IEEE arithmetic.  The kernels leave those
// elements alone and gemm_f16x3_fixup_kernel computes them as plain fp32 dot
// products, which gives sgemm's IEEE pattern (+Inf, -Inf or NaN); with no
// Inf / NaN among the operands it returns at once.
//
// Structure: gemm_x6d_kernel's (cu-gemm-x6.hip): 512 threads, a 256 x 128
// tile of C per workgroup (8 waves of 2 x 2 accumulators of 32 x 32), K steps
// of 32, operands loaded as fp32 by branch-free buffer loads two steps ahead,
// split in registers into two f16 planes of swizzled [row][k] LDS images
// (double-buffered, 2 x 48 KB), one barrier per step.  Thin outputs split K
// over workgroups; the partial tiles are summed in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "cnslmat/hip-util.h"
#include "kaldi-lite/cu-kernels-lite.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 256, BN = 128, BK = 32, NT = 512;
constexpr int ROWB = BK * 2;                  // bytes per LDS row of one plane
constexpr int A_PLANE = BM * ROWB;            // 16 KB
constexpr int B_PLANE = BN * ROWB;            // 8 KB
constexpr int BUF = 2 * (A_PLANE + B_PLANE);  // 48 KB
constexpr int LDS_BYTES = 2 * BUF + (BM + BN) * 4;
constexpr uint32_t NONFINITE = 0x7f800000u;   // |x| bits >= this: Inf or NaN
constexpr int SKIP = 0x40000000;              // scale of an Inf / NaN row or column

struct GemmF16Args {
  const float *A, *B;
  float *C;                      // direct output, or the partial slabs [ksplit][M][N]
  const uint32_t *amax, *bmax;   // max |x| bits per row of op(A), per column of op(B)
  int M, N, K, lda, ldb, ldc;
  int kps, ksplit, tiles_m, tiles_n;
  float alpha, beta;
  int partial;
};

__device__ __forceinline__ int swz(int r, int c) {
  return r * ROWB + ((c ^ ((r >> 2) & 3)) << 4);
}

// the scale exponent s for a row whose largest |x| has the bit pattern mb:
// max |x| * 2^s in [2^14, 2^15)
__device__ __forceinline__ int scale_exp(uint32_t mb) {
  if (mb >= NONFINITE) return SKIP;
  if (mb == 0) return 0;
  const int e = mb >= 0x00800000u ? (int)(mb >> 23) - 127
                                  : (31 - (int)__builtin_clz(mb)) - 149;  // subnormal
  return 14 - e;
}

// (x0, x1) * 2^e -> packed f16 pairs hi, lo
__device__ __forceinline__ void split2h(float x0, float x1, int e, uint32_t &h, uint32_t &l) {
  const float a = __builtin_amdgcn_ldexpf(x0, e), b = __builtin_amdgcn_ldexpf(x1, e);
  const f16x2 hp = __builtin_convertvector((f32x2){a, b}, f16x2);
  const f16x2 lp = __builtin_convertvector((f32x2){a - (float)hp[0], b - (float)hp[1]}, f16x2);
  h = __builtin_bit_cast(uint32_t, hp);
  l = __builtin_bit_cast(uint32_t, lp);
}

// One operand tile (R rows of C's side x BK) per K step, gemm_x6d_kernel's
// TileLoaderD with a two-plane f16 split.
//   KC (K-contiguous source, element (row, k) at src[row * ld + k]):
//     unit = (row, 8-k chunk), two 16-B loads;
//   !KC (source stored [k][row]): unit = (row, KPT consecutive k), lanes
//     along the row so each load instruction reads a contiguous run.
// A thread's units keep their rows for the whole kernel, so each has one
// scale exponent.
template <int R, bool KC>
struct Loader {
  static constexpr int KPT = KC ? 8 : R * BK / NT;
  static constexpr int UNITS = KC ? R * 4 : R * BK / KPT;
  static constexpr int UPT = (UNITS + NT - 1) / NT;
  static_assert(UNITS % NT == 0 && KPT % 8 == 0, "tile shape");
  float v[UPT][KPT];

  __device__ static __forceinline__ int row_of(int u, int tid) {
    const int unit = tid + u * NT;
    return KC ? unit >> 2 : unit % R;
  }
  __device__ static __forceinline__ int k_of(int u, int tid) {
    const int unit = tid + u * NT;
    return KC ? (unit & 3) * 8 : (unit / R) * KPT;
  }

  // base: KC, the tile's first row (src + row0 * ld); !KC, the split's first
  // k and the tile's first column (src + kbeg * ld + row0).  Rows past the
  // matrix read past the buffer's range (0).
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, int ld, int vrows, int kk,
                                       int tid) {
    constexpr unsigned OOB = 0x80000000u;
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int unit = tid + u * NT;
      if constexpr (KC) {
        const int r = unit >> 2, k = kk + (unit & 3) * 8;
        const unsigned off = r < vrows ? (unsigned)(r * ld + k) * 4u : OOB;
        const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        const auto b = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[u][j] = __uint_as_float(a[j]);
          v[u][4 + j] = __uint_as_float(b[j]);
        }
      } else {
        const int r = unit % R, k = kk + (unit / R) * KPT;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
          const unsigned off = r < vrows ? (unsigned)((k + j) * ld + r) * 4u : OOB;
          v[u][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
        }
      }
    }
  }

  // split and write the two planes (plane stride PL bytes); kv < BK: the
  // tile is the last, partial one and its k >= kv are zeroed (they are the
  // next row's values or a pitch's padding)
  template <int PL>
  __device__ __forceinline__ void store(char *lds, int tid, const int (&e)[UPT],
                                        int kv) const {
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int unit = tid + u * NT;
      int r, c0;
      if constexpr (KC) {
        r = unit >> 2;
        c0 = unit & 3;
      } else {
        r = unit % R;
        c0 = (unit / R) * (KPT / 8);
      }
      float x[KPT];
#pragma unroll
      for (int j = 0; j < KPT; ++j) x[j] = v[u][j];
      if (kv < BK) {
        const int kb = k_of(u, tid);
#pragma unroll
        for (int j = 0; j < KPT; ++j)
          if (kb + j >= kv) x[j] = 0.0f;
      }
#pragma unroll
      for (int cc = 0; cc < KPT / 8; ++cc) {
        uint32_t h[4], l[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          split2h(x[cc * 8 + 2 * i], x[cc * 8 + 2 * i + 1], e[u], h[i], l[i]);
        const int off = swz(r, c0 + cc);
        *reinterpret_cast<uint4 *>(lds + off) = make_uint4(h[0], h[1], h[2], h[3]);
        *reinterpret_cast<uint4 *>(lds + PL + off) = make_uint4(l[0], l[1], l[2], l[3]);
      }
    }
  }
};

__device__ __forceinline__ f32x16 mfma(const f16x8 &a, const f16x8 &b, const f32x16 &c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(NT, 1) void gemm_f16x3_kernel(GemmF16Args p) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int *sexp = reinterpret_cast<int *>(lds + 2 * BUF);  // [BM] rows, then [BN] columns
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware order (gemm_x6_kernel): consecutive logical ids on one XCD
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, q = nb >> 3, rr = nb & 7;
  const int lid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (b >> 3);
  const int split = lid % p.ksplit;
  const int rest = lid / p.ksplit;
  const int tn = rest % p.tiles_n, tm = rest / p.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kbeg = split * p.kps;
  const int kend = min(p.K, kbeg + p.kps);
  const int T = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int klast = kend - kbeg - (T - 1) * BK;  // valid k of the last tile

  for (int i = tid; i < BM + BN; i += NT) {
    int s = 0;
    if (i < BM) {
      if (row0 + i < p.M) s = scale_exp(p.amax[row0 + i]);
    } else if (col0 + i - BM < p.N) {
      s = scale_exp(p.bmax[col0 + i - BM]);
    }
    sexp[i] = s;
  }

  // descriptors whose range ends at the operand's last element: a partial
  // last tile reads 0 past it (and the split zeroes the pitch's padding)
  const float *baseA = A_KC ? p.A + (int64_t)row0 * p.lda : p.A + (int64_t)kbeg * p.lda + row0;
  const float *baseB = B_KC ? p.B + (int64_t)col0 * p.ldb : p.B + (int64_t)kbeg * p.ldb + col0;
  const int vra = p.M - row0, vrb = p.N - col0;
  const int64_t endA = A_KC ? ((int64_t)(vra - 1) * p.lda + p.K) * 4
                            : ((int64_t)(p.K - 1 - kbeg) * p.lda + vra) * 4;
  const int64_t endB = B_KC ? ((int64_t)(vrb - 1) * p.ldb + p.K) * 4
                            : ((int64_t)(p.K - 1 - kbeg) * p.ldb + vrb) * 4;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void *)baseA, (short)0, (int)(endA < 0x7fffffff ? endA : 0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void *)baseB, (short)0, (int)(endB < 0x7fffffff ? endB : 0x7fffffff), 0x00020000);
  // k of tile t relative to the base (clamped to the last tile: a re-read)
  auto kk = [&](int t, bool kc) { return (kc ? kbeg : 0) + min(t, T - 1) * BK; };

  using LA = Loader<BM, A_KC>;
  using LB = Loader<BN, B_KC>;
  LA la[2];
  LB lb[2];
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.0f;
  __syncthreads();  // sexp
  int ea[LA::UPT], eb[LB::UPT];
#pragma unroll
  for (int u = 0; u < LA::UPT; ++u) {
    const int s = sexp[LA::row_of(u, tid)];
    ea[u] = s == SKIP ? 0 : s;
  }
#pragma unroll
  for (int u = 0; u < LB::UPT; ++u) {
    const int s = sexp[BM + LB::row_of(u, tid)];
    eb[u] = s == SKIP ? 0 : s;
  }

  if (T > 0) {
    la[0].load(rsA, p.lda, vra, kk(0, A_KC), tid);
    lb[0].load(rsB, p.ldb, vrb, kk(0, B_KC), tid);
    la[0].template store<A_PLANE>(lds, tid, ea, T == 1 ? klast : BK);
    lb[0].template store<B_PLANE>(lds + 2 * A_PLANE, tid, eb, T == 1 ? klast : BK);
    // tiles 1, 2 into sets 1, 0 (as at every later loop entry)
    __builtin_amdgcn_sched_barrier(0);
    la[1].load(rsA, p.lda, vra, kk(1, A_KC), tid);
    lb[1].load(rsB, p.ldb, vrb, kk(1, B_KC), tid);
    __builtin_amdgcn_sched_barrier(0);
    la[0].load(rsA, p.lda, vra, kk(2, A_KC), tid);
    lb[0].load(rsB, p.ldb, vrb, kk(2, B_KC), tid);
    __syncthreads();

    const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);
    const int half = lane >> 5;
    // one k16 half of a step: 8 fragment reads, 12 MFMAs
    auto half_step = [&](const char *bufA, int s) {
      const char *bufB = bufA + 2 * A_PLANE;
      f16x8 a[2][2], bb[2][2];
      const int c = 2 * s + half;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          a[i][pl] = *reinterpret_cast<const f16x8 *>(bufA + pl * A_PLANE + swz(ar + 32 * i, c));
          bb[i][pl] = *reinterpret_cast<const f16x8 *>(bufB + pl * B_PLANE + swz(br + 32 * i, c));
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 x = acc[i][j];
          x = mfma(a[i][1], bb[j][0], x);  // lo hi
          x = mfma(a[i][0], bb[j][1], x);  // hi lo
          x = mfma(a[i][0], bb[j][0], x);  // hi hi
          acc[i][j] = x;
        }
    };
    // waves 4-7 split the next tile between their two MFMA halves, waves
    // 0-3 after both (gemm_x6_kernel's stagger)
    const bool late = wave < 4;
    // step t: tile t+1 is in set (t+1) & 1, which then takes tile t+3 (a
    // step past T issues its clamped loads too, so every path issues the
    // same loads and each split waits only for its own tile)
    auto step = [&](int t, LA &lan, LB &lbn) {
      if (t < T) {
        const char *buf = lds + (t & 1) * BUF;
        char *nA = lds + ((t + 1) & 1) * BUF;
        const int kv = t + 2 == T ? klast : BK;
        half_step(buf, 0);
        if (!late && t + 1 < T) {
          lan.template store<A_PLANE>(nA, tid, ea, kv);
          lbn.template store<B_PLANE>(nA + 2 * A_PLANE, tid, eb, kv);
        }
        half_step(buf, 1);
        if (late && t + 1 < T) {
          lan.template store<A_PLANE>(nA, tid, ea, kv);
          lbn.template store<B_PLANE>(nA + 2 * A_PLANE, tid, eb, kv);
        }
      }
      lan.load(rsA, p.lda, vra, kk(t + 3, A_KC), tid);
      lbn.load(rsB, p.ldb, vrb, kk(t + 3, B_KC), tid);
      __syncthreads();
    };
    for (int t = 0; t < T; t += 2) {
      step(t, la[1], lb[1]);
      step(t + 1, la[0], lb[0]);
    }
  }

  // C/D map of 32x32x16: register g of lane l holds
  // row (g & 3) + 8 (g >> 2) + 4 (l >> 5), column l & 31.
  float *out = p.partial ? p.C + (int64_t)split * p.M * p.N : p.C;
  const int ldo = p.partial ? p.N : p.ldc;
  const int half2 = lane >> 5;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl = wn * 64 + j * 32 + (lane & 31);
      const int col = col0 + cl;
      const int ec = sexp[BM + cl];
      if (col >= p.N || ec == SKIP) continue;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int rl = wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * half2;
        const int row = row0 + rl;
        const int er = sexp[rl];
        if (row >= p.M || er == SKIP) continue;
        const float v = __builtin_amdgcn_ldexpf(acc[i][j][g], -(er + ec));
        float *o = out + (int64_t)row * ldo + col;
        if (p.partial) *o = v;
        else *o = p.beta == 0.0f ? p.alpha * v : p.alpha * v + p.beta * *o;
      }
    }
}

// C = alpha * sum_s part[s] + beta * C, the splits added in increasing s;
// elements of an Inf / NaN row or column are the fixup kernel's
template <bool VEC>
__global__ void gemm_f16x3_reduce_kernel(const float *__restrict__ part, int S, int M, int N,
                                         float alpha, float beta, float *C, int ldc,
                                         const uint32_t *__restrict__ amax,
                                         const uint32_t *__restrict__ bmax) {
  constexpr int W = VEC ? 4 : 1;
  const int64_t nw = N / W;
  const int64_t total = (int64_t)M * nw;
  const int64_t plane = (int64_t)M * N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / nw, c = (e - r * nw) * W;
    float s[W];
    if constexpr (VEC) {
      const float4 v = *reinterpret_cast<const float4 *>(part + r * N + c);
      s[0] = v.x; s[1] = v.y; s[2] = v.z; s[3] = v.w;
    } else {
      s[0] = part[r * N + c];
    }
    for (int k = 1; k < S; ++k) {
      if constexpr (VEC) {
        const float4 v = *reinterpret_cast<const float4 *>(part + k * plane + r * N + c);
        s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
      } else {
        s[0] += part[k * plane + r * N + c];
      }
    }
    if (amax[r] >= NONFINITE) continue;
    float *o = C + r * ldc + c;
#pragma unroll
    for (int i = 0; i < W; ++i) {
      if (bmax[c + i] >= NONFINITE) continue;
      o[i] = beta == 0.0f ? alpha * s[i] : alpha * s[i] + beta * o[i];
    }
  }
}

struct FixupArgs {
  const float *A, *B;
  float *C;
  const uint32_t *amax, *bmax, *aflag, *bflag;
  int M, N, K, lda, ldb, ldc, transA, transB;
  float alpha, beta;
};

// The C elements of every row of op(A) / column of op(B) holding Inf or
// NaN, as fp32 dot products in increasing k (IEEE: the reference sgemm's
// Inf / NaN pattern).  Returns at once when no operand holds one.
__global__ void gemm_f16x3_fixup_kernel(FixupArgs f) {
  if ((*f.aflag | *f.bflag) == 0) return;
  const int64_t total = (int64_t)f.M * f.N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / f.N, c = e - r * f.N;
    if (f.amax[r] < NONFINITE && f.bmax[c] < NONFINITE) continue;
    float s = 0.0f;
    for (int k = 0; k < f.K; ++k) {
      const float a = f.transA ? f.A[(int64_t)k * f.lda + r] : f.A[r * f.lda + k];
      const float b = f.transB ? f.B[c * f.ldb + k] : f.B[(int64_t)k * f.ldb + c];
      s = fmaf(a, b, s);
    }
    float *o = f.C + r * f.ldc + c;
    *o = f.beta == 0.0f ? f.alpha * s : f.alpha * s + f.beta * *o;
  }
}

// Per-row and per-column max |x| of a pitched fp32 matrix as float bit
// patterns (atomicMax on the unsigned bits: order-independent, so the result
// is deterministic), and *flag = 1 when an element is Inf or NaN.  A block
// covers rb rows x AM_CW columns: thread t reads float4 t + 256 j (j <
// AM_NV) of each row (16-B loads when aligned, 1 KiB per wave instruction),
// keeps its 16 column maxima in registers over the rows, and the row maximum
// takes one wave reduction per row; the column maxima go out once per block.
constexpr int AM_NV = 4, AM_CW = 1024 * AM_NV;
template <bool VEC>
__global__ __launch_bounds__(256) void absmax_kernel(const float *__restrict__ X, int rows,
                                                    int cols, int ld, int rb, uint32_t *rmax,
                                                    uint32_t *cmax, uint32_t *flag) {
  const int c0 = blockIdx.x * AM_CW + threadIdx.x * 4;
  const int r0 = blockIdx.y * rb;
  const int rend = min(rows, r0 + rb);
  uint32_t cm[AM_NV][4];
#pragma unroll
  for (int j = 0; j < AM_NV; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) cm[j][i] = 0u;
  for (int r = r0; r < rend; ++r) {
    const float *x = X + (int64_t)r * ld;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < AM_NV; ++j) {
      const int c = c0 + j * 1024;
      uint32_t v[4];
      if (VEC && c + 4 <= cols) {
        const float4 q = *reinterpret_cast<const float4 *>(x + c);
        v[0] = __float_as_uint(q.x); v[1] = __float_as_uint(q.y);
        v[2] = __float_as_uint(q.z); v[3] = __float_as_uint(q.w);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = c + i < cols ? __float_as_uint(x[c + i]) : 0u;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] &= 0x7fffffffu;
        cm[j][i] = max(cm[j][i], v[i]);
        m = max(m, v[i]);
      }
    }
    if (rmax) {
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
      if ((threadIdx.x & 63) == 0 && m) atomicMax(rmax + r, m);
    }
  }
  uint32_t all = 0;
#pragma unroll
  for (int j = 0; j < AM_NV; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + j * 1024 + i;
      all = max(all, cm[j][i]);
      if (cmax && c < cols && cm[j][i]) atomicMax(cmax + c, cm[j][i]);
    }
  if (all >= NONFINITE) atomicOr(flag, 1u);
}

int choose_ksplit(int64_t tiles, int K) {
  int best = 1;
  double best_score = -1.0;
  for (int s = 1; s <= 4; ++s) {
    if (s > 1 && K / s < 1024) break;
    const int64_t nb = tiles * s;
    const int64_t waves = (nb + 255) / 256;
    const double score = (double)nb / (double)(waves * 256) - 0.02 * (s - 1);
    if (score > best_score + 1e-9) { best_score = score; best = s; }
  }
  return best;
}

template <bool A_KC, bool B_KC>
void launch(const GemmF16Args &a, unsigned blocks, hipStream_t st) {
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(&gemm_f16x3_kernel<A_KC, B_KC>),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS_BYTES) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_f16x3_kernel<A_KC, B_KC>), dim3(blocks), dim3(NT), LDS_BYTES, st, a);
}

size_t align16(size_t b) { return (b + 15) & ~(size_t)15; }
size_t partial_bytes(int M, int N, int K) {
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int s = choose_ksplit(tiles, K);
  return s > 1 ? align16(sizeof(float) * (size_t)s * M * N) : 0;
}
size_t stats_words(int rows, int cols) { return 4 + (size_t)rows + cols; }

}  // namespace

extern "C" int kl_absmax(const float *X, int rows, int cols, int ld, uint32_t *st,
                         int want_rows, int want_cols, kcnn_stream_t stream) {
  if (rows < 0 || cols < 0 || ld < cols || !st) return (int)hipErrorInvalidValue;
  hipStream_t s = kcnn::as_stream(stream);
  hipError_t e = hipMemsetAsync(st, 0, sizeof(uint32_t) * stats_words(rows, cols), s);
  if (e != hipSuccess) return (int)e;
  if (rows == 0 || cols == 0) return 0;
  // about 512 blocks of at least 8 rows (each block sends its AM_CW column
  // maxima out by atomics, so taller blocks for tall matrices)
  const int cb = (cols + AM_CW - 1) / AM_CW;
  const int rb = (int)std::max<int64_t>(8, ((int64_t)rows * cb + 511) / 512);
  const dim3 grid(cb, (rows + rb - 1) / rb);
  uint32_t *rm = want_rows ? st + 4 : nullptr;
  uint32_t *cm = want_cols ? st + 4 + rows : nullptr;
  if (ld % 4 == 0 && (uintptr_t)X % 16 == 0)
    hipLaunchKernelGGL(absmax_kernel<true>, grid, dim3(256), 0, s, X, rows, cols, ld, rb, rm, cm,
                       st);
  else
    hipLaunchKernelGGL(absmax_kernel<false>, grid, dim3(256), 0, s, X, rows, cols, ld, rb, rm,
                       cm, st);
  return kcnn::launch_status();
}

// C[M x N] = alpha * op(A) op(B) + beta * C with the operands' max |x| given:
// amax[i] for row i of op(A), bmax[j] for column j of op(B) (kl_absmax bit
// patterns), aflag / bflag their Inf / NaN flags.  Needs 16-B aligned
// K-contiguous operands (A untransposed, B transposed) with pitches % 4 == 0
// and every workgroup's buffer offsets below 2^31; returns
// hipErrorNotSupported otherwise (the caller uses kl_gemm_x6).
extern "C" size_t kl_gemm_f16x3_workspace_bytes(int M, int N, int K) {
  return partial_bytes(M, N, K);
}
extern "C" int kl_gemm_f16x3_st(int transA, int transB, int M, int N, int K, float alpha,
                                const float *A, int lda, const float *B, int ldb, float beta,
                                float *C, int ldc, const uint32_t *amax, const uint32_t *aflag,
                                const uint32_t *bmax, const uint32_t *bflag, void *ws,
                                size_t ws_bytes, kcnn_stream_t stream) {
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0 || K == 0) return (int)hipErrorNotSupported;
  const bool a_kc = !transA, b_kc = transB != 0;
  if ((a_kc && (lda % 4 || (uintptr_t)A % 16)) || (b_kc && (ldb % 4 || (uintptr_t)B % 16)))
    return (int)hipErrorNotSupported;
  GemmF16Args a;
  a.A = A; a.B = B; a.amax = amax; a.bmax = bmax;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.alpha = alpha; a.beta = beta;
  a.tiles_m = (M + BM - 1) / BM;
  a.tiles_n = (N + BN - 1) / BN;
  const int64_t tiles = (int64_t)a.tiles_m * a.tiles_n;
  int s = choose_ksplit(tiles, K);
  const size_t need = s > 1 ? sizeof(float) * (size_t)s * M * N : 0;
  if (need > ws_bytes || !ws) s = 1;
  a.ksplit = s;
  a.kps = ((K + s - 1) / s + BK - 1) / BK * BK;
  a.partial = s > 1;
  a.C = s > 1 ? static_cast<float *>(ws) : C;
  const int64_t nb = tiles * s;
  if (nb >= ((int64_t)1 << 31)) return (int)hipErrorNotSupported;
  // every offset a workgroup forms (rows of its tile, k up to K + 2 BK) < 2^31
  auto fits = [&](bool kc, int ld, int R) {
    if (kc) return (int64_t)R * ld * 4 + (int64_t)(K + 2 * BK) * 4 < ((int64_t)1 << 31);
    return (int64_t)(a.kps + 2 * BK) * ld * 4 + (int64_t)R * 4 < ((int64_t)1 << 31);
  };
  if (!fits(a_kc, lda, BM) || !fits(b_kc, ldb, BN)) return (int)hipErrorNotSupported;
  hipStream_t st = kcnn::as_stream(stream);
  if (a_kc && b_kc) launch<true, true>(a, (unsigned)nb, st);
  else if (a_kc) launch<true, false>(a, (unsigned)nb, st);
  else if (b_kc) launch<false, true>(a, (unsigned)nb, st);
  else launch<false, false>(a, (unsigned)nb, st);
  int rc = kcnn::launch_status();
  if (rc) return rc;
  if (s > 1) {
    if (N % 4 == 0 && ldc % 4 == 0 && (uintptr_t)C % 16 == 0)
      hipLaunchKernelGGL(gemm_f16x3_reduce_kernel<true>,
                         dim3(kcnn::grid_for((int64_t)M * (N / 4))), dim3(256), 0, st,
                         (const float *)ws, s, M, N, alpha, beta, C, ldc, amax, bmax);
    else
      hipLaunchKernelGGL(gemm_f16x3_reduce_kernel<false>, dim3(kcnn::grid_for((int64_t)M * N)),
                         dim3(256), 0, st, (const float *)ws, s, M, N, alpha, beta, C, ldc,
                         amax, bmax);
    rc = kcnn::launch_status();
    if (rc) return rc;
  }
  FixupArgs f;
  f.A = A; f.B = B; f.C = C; f.amax = amax; f.bmax = bmax; f.aflag = aflag; f.bflag = bflag;
  f.M = M; f.N = N; f.K = K; f.lda = lda; f.ldb = ldb; f.ldc = ldc;
  f.transA = transA != 0; f.transB = transB != 0; f.alpha = alpha; f.beta = beta;
  hipLaunchKernelGGL(gemm_f16x3_fixup_kernel, dim3(64), dim3(256), 0, st, f);
  return kcnn::launch_status();
}

// The same with the operand statistics computed here (two kl_absmax passes
// into the workspace after the partial slabs).
extern "C" size_t kl_gemm_f16x3_full_workspace_bytes(int M, int N, int K) {
  // A's statistics cover its stored shape (M x K or K x M), B's (K x N or N x K)
  return partial_bytes(M, N, K) + align16(sizeof(uint32_t) * stats_words(M, K)) +
         align16(sizeof(uint32_t) * stats_words(K, N));
}
extern "C" int kl_gemm_f16x3(int transA, int transB, int M, int N, int K, float alpha,
                             const float *A, int lda, const float *B, int ldb, float beta,
                             float *C, int ldc, void *ws, size_t ws_bytes,
                             kcnn_stream_t stream) {
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0 || K == 0) return (int)hipErrorNotSupported;
  const size_t pb = partial_bytes(M, N, K);
  const size_t sa = align16(sizeof(uint32_t) * stats_words(M, K));
  if (!ws || ws_bytes < kl_gemm_f16x3_full_workspace_bytes(M, N, K))
    return (int)hipErrorInvalidValue;
  uint32_t *stA = reinterpret_cast<uint32_t *>(static_cast<char *>(ws) + pb);
  uint32_t *stB = reinterpret_cast<uint32_t *>(static_cast<char *>(ws) + pb + sa);
  // op(A) rows: rows of A (M x K), or its columns when A is stored K x M
  const int ar = transA ? K : M, ac = transA ? M : K;
  const int br = transB ? N : K, bc = transB ? K : N;
  int rc = kl_absmax(A, ar, ac, lda, stA, !transA, transA, stream);
  if (rc) return rc;
  rc = kl_absmax(B, br, bc, ldb, stB, transB, !transB, stream);
  if (rc) return rc;
  const uint32_t *amax = transA ? stA + 4 + ar : stA + 4;
  const uint32_t *bmax = transB ? stB + 4 : stB + 4 + br;
  return kl_gemm_f16x3_st(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, amax,
                          stA, bmax, stB, pb ? ws : nullptr, pb, stream);
}
