// kaldi-lite/kcnn-knobs.h -- run-time switches of libkcnn.so.
//
// Kernel-family selectors are product settings: each picks between
// implementations of the same math (f16x3 / bf16x6 on the f16 / bf16 matrix
// cores, or the fp32-input MFMA kernels), is documented in DESIGN.md §3 and is covered by
// tests/test_gpu_families.py.  They are set through the C-ABI
// (kcnn_set_kernel_family) or, once when the library loads, by the
// environment variable named in the table below.
//
//   family     env              values
//   fwd_x6     KCNN_FWD_X6      2 f16x3 frame-resident forward, 1 bf16x6, 0 fp32 MFMA
//   bwd_x6     KCNN_BWD_X6      1 bf16x6 fused backward, 0 fp32 MFMA
//   igemm_x6   KCNN_IGEMM_X6    2 f16x3 implicit GEMM for convolutions of >= 2^34 flop (bf16x6
//                               below), 3 f16x3 for all, 1 bf16x6, 0 fp32 MFMA
//   wgrad_x6   KCNN_WGRAD_X6    2 wide bf16x6, 3 wide f16x3 (slower on c5), 1 128-wide bf16x6,
//                               0 fp32 MFMA
//   gemm       KCNN_GEMM        2 f16x3 GEMM (AddMatMat), 1 bf16x6 GEMM, 0 rocBLAS sgemm
//
// (KCNN_FUSE, KCNN_LITERAL and KCNN_PROFILE are kcnn_set_fusion,
// kcnn_set_literal_path and kcnn_set_profiling.)
//
// Experiment knobs (KCNN_KNOB) are the A/B switches used while tuning a
// kernel.  Only the `make timing` build (-DKCNN_EXPERIMENTS) reads them from
// the environment; the product library compiles each one to its default.
#ifndef KCNN_KALDI_LITE_KCNN_KNOBS_H_
#define KCNN_KALDI_LITE_KCNN_KNOBS_H_

namespace kcnn {

enum Family { kFamFwdX6 = 0, kFamBwdX6, kFamIgemmX6, kFamWgradX6, kFamGemm, kNumFamilies };

int family(Family f);                 // current value of a selector
int set_family(Family f, int value);  // 0 on success, -1 for an invalid value
int family_by_name(const char *name);  // Family index, -1 when unknown
int experiment_env(const char *name, int dflt);

}  // namespace kcnn

#ifdef KCNN_EXPERIMENTS
#define KCNN_KNOB(name, dflt) (::kcnn::experiment_env(name, dflt))
#else
#define KCNN_KNOB(name, dflt) (dflt)
#endif

#endif  // KCNN_KALDI_LITE_KCNN_KNOBS_H_
