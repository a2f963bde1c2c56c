// kaldi-lite/cu-gemm-x6.hip -- fp32 GEMM on the bf16 matrix cores by an exact
// three-way split of each operand (the "bf16x6" scheme).
//
// Upstream Kaldi's CuMatrixBase::AddMatMat is cuBLAS sgemm; the reference
// calls it for the FullyConnectedComponent forward, data gradient and update
// (nnet-component.cc:1225-1227, :1247; nnet-component-nnet0.cc:1137-1142).
// On gfx950 the fp32-input MFMA runs at 1/16 of the bf16 rate (157 TF), and
// rocBLAS sgemm already reaches ~86 % of that on these shapes.  This kernel
// computes the same fp32 product on the bf16 MFMAs instead:
//
//   x = h + m + l exactly, h = bf16(x), m = bf16(x - h), l = bf16(x - h - m)
//
// (each residual subtraction is exact in fp32 and leaves at most 16, then 8,
// significant bits).  Every product of two bf16 values is exact in fp32, so
//
//   a*b = hh + (hm + mh) + (mm + hl + lh) + (ml + lm + ll)
//
// with the terms of relative size 1, 2^-8, 2^-16 and < 2^-24.  The kernel
// keeps the first six, one v_mfma_f32_32x32x16_bf16 each, all accumulated in
// fp32.  The three it drops are below fp32's own rounding of the product
// (measured: max |c - c64| / (|A||B|) = 1.7e-7 against rocBLAS sgemm's 2.9e-7
// at K = 11616, scripts/fc_split_probe.py), so the result meets the same
// dot-product error bound as sgemm (tests/test_gpu_gemm.py).  Six bf16 MFMAs
// cost 6/16 of one fp32 MFMA.
//
// Structure: 512 threads, a 256 x 128 tile of C per workgroup (8 waves, each
// 64 x 64 = 2 x 2 accumulators of 32 x 32), K steps of 32.  Operands are read
// from HBM as fp32 once per K step into registers (one step ahead), split in
// registers, and written to LDS as three bf16 planes in the MFMA fragment
// layout ([row][k], 64-B rows, 16-B chunks XOR-swizzled by row), double
// buffered (2 x 72 KB).  The VALU split runs beside the bf16 MFMAs, which,
// unlike the fp32-input MFMA, do not hold the SIMD's vector pipe.  Either
// operand may be stored K-contiguous or M/N-contiguous (row-major Kaldi
// matrices, both transpose flags); the transpose happens in the split pass.
// Thin outputs split K over workgroups; partial tiles are summed in a fixed
// order (deterministic, no atomics).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cnslmat/hip-util.h"
#include "kaldi-lite/cu-kernels-lite.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 256, BN = 128, BK = 32, NT = 512;
constexpr int ROWB = BK * 2;                 // bytes per LDS row of one plane
constexpr int A_PLANE = BM * ROWB;           // 16 KB
constexpr int B_PLANE = BN * ROWB;           // 8 KB
constexpr int BUF = 3 * (A_PLANE + B_PLANE); // 72 KB
constexpr int LDS_BYTES = 2 * BUF;

struct GemmX6Args {
  const float *A, *B;
  float *C;          // direct output, or the partial slabs [ksplit][M][N]
  int M, N, K, lda, ldb, ldc;
  int kps;           // K per split (multiple of BK)
  int ksplit, tiles_m, tiles_n;
  float alpha, beta;
  int partial;       // 1: write raw sums to C + split * M * N (ld N)
};

// byte offset of (row r, 16-B chunk c) inside a plane
__device__ __forceinline__ int swz(int r, int c) {
  return r * ROWB + ((c ^ ((r >> 2) & 3)) << 4);
}

// 8 fp32 -> three bf16x8 planes, x = h + m + l exactly for finite x
__device__ __forceinline__ void split8(const float *x, uint4 &h, uint4 &m, uint4 &l) {
  uint32_t hv[4], mv[4], lv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x2 v = {x[2 * i], x[2 * i + 1]};
    bf16x2 a = __builtin_convertvector(v, bf16x2);
    f32x2 r = v - __builtin_convertvector(a, f32x2);
    bf16x2 b = __builtin_convertvector(r, bf16x2);
    f32x2 r2 = r - __builtin_convertvector(b, f32x2);
    bf16x2 c = __builtin_convertvector(r2, bf16x2);
    hv[i] = __builtin_bit_cast(uint32_t, a);
    mv[i] = __builtin_bit_cast(uint32_t, b);
    lv[i] = __builtin_bit_cast(uint32_t, c);
  }
  h = make_uint4(hv[0], hv[1], hv[2], hv[3]);
  m = make_uint4(mv[0], mv[1], mv[2], mv[3]);
  l = make_uint4(lv[0], lv[1], lv[2], lv[3]);
}

// One operand tile (R rows of C's side x BK) per K step.
//   KC (K-contiguous source, element (row, k) at src[row * ld + k]):
//     unit = (row, 8-k chunk), R * 4 units, two float4 loads each.
//   !KC (source stored [k][row], element at src[k * ld + row]):
//     unit = (row, KPT consecutive k), lanes along the row so each load
//     instruction reads a contiguous run; KPT = R * BK / NT.
template <int R, bool KC>
struct TileLoader {
  static constexpr int KPT = KC ? 8 : R * BK / NT;
  static constexpr int UNITS = KC ? R * 4 : R * BK / KPT;
  static constexpr int UPT = (UNITS + NT - 1) / NT;  // units per thread
  static_assert(KC ? (UNITS % NT == 0) : (KPT % 8 == 0), "tile shape");
  float v[UPT][KPT];

  __device__ __forceinline__ void load(const float *__restrict__ src, int ld,
                                       int row0, int rows, int k0, int kend,
                                       int tid) {
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int unit = tid + u * NT;
      if (unit >= UNITS) break;
      if constexpr (KC) {
        const int r = unit >> 2, k = k0 + (unit & 3) * 8;
        const int gr = row0 + r;
        const float *p = src + (int64_t)gr * ld + k;
        if (gr < rows && k + 8 <= kend) {
          const float4 a = *reinterpret_cast<const float4 *>(p);
          const float4 b = *reinterpret_cast<const float4 *>(p + 4);
          v[u][0] = a.x; v[u][1] = a.y; v[u][2] = a.z; v[u][3] = a.w;
          v[u][4] = b.x; v[u][5] = b.y; v[u][6] = b.z; v[u][7] = b.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[u][j] = (gr < rows && k + j < kend) ? p[j] : 0.0f;
        }
      } else {
        const int r = unit % R, kq = unit / R;
        const int gr = row0 + r, k = k0 + kq * KPT;
        const float *p = src + (int64_t)k * ld + gr;
        if (gr < rows && k + KPT <= kend) {
#pragma unroll
          for (int j = 0; j < KPT; ++j) v[u][j] = p[(int64_t)j * ld];
        } else {
#pragma unroll
          for (int j = 0; j < KPT; ++j)
            v[u][j] = (gr < rows && k + j < kend) ? p[(int64_t)j * ld] : 0.0f;
        }
      }
    }
  }

  // split and write the three planes (plane stride PL bytes)
  template <int PL>
  __device__ __forceinline__ void store(char *lds, int tid) const {
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int unit = tid + u * NT;
      if (unit >= UNITS) break;
      int r, c0;
      if constexpr (KC) {
        r = unit >> 2;
        c0 = unit & 3;
      } else {
        r = unit % R;
        c0 = (unit / R) * (KPT / 8);
      }
#pragma unroll
      for (int cc = 0; cc < KPT / 8; ++cc) {
        uint4 h, m, l;
        split8(&v[u][cc * 8], h, m, l);
        const int off = swz(r, c0 + cc);
        *reinterpret_cast<uint4 *>(lds + off) = h;
        *reinterpret_cast<uint4 *>(lds + PL + off) = m;
        *reinterpret_cast<uint4 *>(lds + 2 * PL + off) = l;
      }
    }
  }
};

__device__ __forceinline__ f32x16 mfma(const bf16x8 &a, const bf16x8 &b, const f32x16 &c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <bool A_KC, bool B_KC>
__global__ __launch_bounds__(NT, 1) void gemm_x6_kernel(GemmX6Args p) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware order: consecutive logical ids run on one XCD (blocks are
  // dealt round-robin over the 8 XCDs) and share the A rows of one tile_m.
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

  TileLoader<BM, A_KC> la;
  TileLoader<BN, B_KC> lb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[i][j][g] = 0.0f;

  if (T > 0) {
    la.load(p.A, p.lda, row0, p.M, kbeg, kend, tid);
    lb.load(p.B, p.ldb, col0, p.N, kbeg, kend, tid);
    la.template store<A_PLANE>(lds, tid);
    lb.template store<B_PLANE>(lds + 3 * A_PLANE, tid);
    __syncthreads();
    if (T > 1) {
      la.load(p.A, p.lda, row0, p.M, kbeg + BK, kend, tid);
      lb.load(p.B, p.ldb, col0, p.N, kbeg + BK, kend, tid);
    }
  }

  const int ar = wm * 64 + (lane & 31), br = wn * 64 + (lane & 31);
  const int half = lane >> 5;
  for (int t = 0; t < T; ++t) {
    const char *bufA = lds + (t & 1) * BUF;
    const char *bufB = bufA + 3 * A_PLANE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[2][3], bb[2][3];
      const int c = 2 * s + half;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          a[i][pl] = *reinterpret_cast<const bf16x8 *>(bufA + pl * A_PLANE + swz(ar + 32 * i, c));
          bb[i][pl] = *reinterpret_cast<const bf16x8 *>(bufB + pl * B_PLANE + swz(br + 32 * i, c));
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 x = acc[i][j];
          x = mfma(a[i][2], bb[j][0], x);  // lh
          x = mfma(a[i][0], bb[j][2], x);  // hl
          x = mfma(a[i][1], bb[j][1], x);  // mm
          x = mfma(a[i][1], bb[j][0], x);  // mh
          x = mfma(a[i][0], bb[j][1], x);  // hm
          x = mfma(a[i][0], bb[j][0], x);  // hh
          acc[i][j] = x;
        }
    }
    if (t + 1 < T) {
      char *nA = lds + ((t + 1) & 1) * BUF;
      la.template store<A_PLANE>(nA, tid);
      lb.template store<B_PLANE>(nA + 3 * A_PLANE, tid);
      if (t + 2 < T) {
        la.load(p.A, p.lda, row0, p.M, kbeg + (t + 2) * BK, kend, tid);
        lb.load(p.B, p.ldb, col0, p.N, kbeg + (t + 2) * BK, kend, tid);
      }
    }
    __syncthreads();
  }

  // C/D map of 32x32x16: register g of lane l holds
  // row (g & 3) + 8 (g >> 2) + 4 (l >> 5), column l & 31.
  float *out = p.partial ? p.C + (int64_t)split * p.M * p.N : p.C;
  const int ldo = p.partial ? p.N : p.ldc;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = col0 + wn * 64 + j * 32 + (lane & 31);
      if (col >= p.N) continue;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int row = row0 + wm * 64 + i * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        if (row >= p.M) continue;
        float *o = out + (int64_t)row * ldo + col;
        if (p.partial) *o = acc[i][j][g];
        else *o = p.beta == 0.0f ? p.alpha * acc[i][j][g]
                                 : p.alpha * acc[i][j][g] + p.beta * *o;
      }
    }
}

// C = alpha * sum_s part[s] + beta * C, the splits added in increasing s
__global__ void gemm_x6_reduce_kernel(const float *__restrict__ part, int S, int M,
                                      int N, float alpha, float beta, float *C,
                                      int ldc) {
  const int64_t n4 = N / 4;
  const int64_t total = (int64_t)M * n4;
  const int64_t plane = (int64_t)M * N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / n4, c = (e - r * n4) * 4;
    float4 s = *reinterpret_cast<const float4 *>(part + r * N + c);
    for (int k = 1; k < S; ++k) {
      const float4 v = *reinterpret_cast<const float4 *>(part + k * plane + r * N + c);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    float *o = C + r * ldc + c;
    if (beta == 0.0f) {
      o[0] = alpha * s.x; o[1] = alpha * s.y; o[2] = alpha * s.z; o[3] = alpha * s.w;
    } else {
      o[0] = alpha * s.x + beta * o[0]; o[1] = alpha * s.y + beta * o[1];
      o[2] = alpha * s.z + beta * o[2]; o[3] = alpha * s.w + beta * o[3];
    }
  }
}

__global__ void gemm_x6_reduce_scalar_kernel(const float *__restrict__ part, int S,
                                             int M, int N, float alpha, float beta,
                                             float *C, int ldc) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    float s = part[e];
    for (int k = 1; k < S; ++k) s += part[k * total + e];
    const int64_t r = e / N, c = e - r * N;
    float *o = C + r * ldc + c;
    *o = beta == 0.0f ? alpha * s : alpha * s + beta * *o;
  }
}

template <bool A_KC, bool B_KC>
void launch_x6(const GemmX6Args &a, unsigned blocks, hipStream_t st) {
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(&gemm_x6_kernel<A_KC, B_KC>),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               LDS_BYTES) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((gemm_x6_kernel<A_KC, B_KC>), dim3(blocks), dim3(NT), LDS_BYTES,
                     st, a);
}

// K splits for a tile count: the fraction of the last wave of workgroups
// that is busy, less a small charge per extra split (partials + reduction)
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

}  // namespace

extern "C" size_t kl_gemm_x6_workspace_bytes(int M, int N, int K) {
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int s = choose_ksplit(tiles, K);
  return s > 1 ? sizeof(float) * (size_t)s * M * N : 0;
}

// C[M x N] = alpha * op(A) op(B) + beta * C, row-major; op(A) is A^T when
// transA (A stored K x M), op(B) is B^T when transB (B stored N x K).
extern "C" int kl_gemm_x6(int transA, int transB, int M, int N, int K, float alpha,
                          const float *A, int lda, const float *B, int ldb, float beta,
                          float *C, int ldc, void *ws, size_t ws_bytes,
                          kcnn_stream_t stream) {
  if (M < 0 || N < 0 || K < 0) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  // 16-B operand loads on the K-contiguous side
  const bool a_kc = !transA, b_kc = transB != 0;
  if ((a_kc && (lda % 4 || (uintptr_t)A % 16)) || (b_kc && (ldb % 4 || (uintptr_t)B % 16)))
    return (int)hipErrorInvalidValue;
  hipStream_t st = kcnn::as_stream(stream);
  GemmX6Args a;
  a.A = A; a.B = B; a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb;
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
  a.ldc = ldc;
  const int64_t nb = tiles * s;
  if (nb >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  if (a_kc && b_kc) launch_x6<true, true>(a, (unsigned)nb, st);
  else if (a_kc) launch_x6<true, false>(a, (unsigned)nb, st);
  else if (b_kc) launch_x6<false, true>(a, (unsigned)nb, st);
  else launch_x6<false, false>(a, (unsigned)nb, st);
  int rc = kcnn::launch_status();
  if (rc || s == 1) return rc;
  if (N % 4 == 0 && ldc % 4 == 0 && (uintptr_t)C % 16 == 0)
    hipLaunchKernelGGL(gemm_x6_reduce_kernel, dim3(kcnn::grid_for((int64_t)M * (N / 4))),
                       dim3(256), 0, st, (const float *)ws, s, M, N, alpha, beta, C, ldc);
  else
    hipLaunchKernelGGL(gemm_x6_reduce_scalar_kernel, dim3(kcnn::grid_for((int64_t)M * N)),
                       dim3(256), 0, st, (const float *)ws, s, M, N, alpha, beta, C, ldc);
  return kcnn::launch_status();
}
