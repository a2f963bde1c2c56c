// cnslmat/momentum-step.h -- one element of the nnet0 momentum update, shared
// by the elementwise update kernel (hipF_momentum_update) and the f16x3
// weight-gradient GEMM's fused store (kl_gemm_f16x3_momentum), so that both
// give the same bits.
//
// Reference: FullyConnectedComponent::Update / ConvolutionComponent::Update
// (nnet-component-nnet0.cc:1133-1150, :738-777):
//   prev.Scale(momentum); prev.AddMat(-lr * wd, W); prev.AddMatMat(lr, dY^T X);
//   W.AddMat(1.0, prev)
// with the gradient g = (dY^T X)[i][j] given: p = momentum prev; p += a_wd W;
// p += a_g g; prev = p; W += p (each add one rounding, as the elementwise
// kernel has always compiled them).
#ifndef KCNN_CNSLMAT_MOMENTUM_STEP_H_
#define KCNN_CNSLMAT_MOMENTUM_STEP_H_

// The update's operands for a fused store (W nullptr: no update)
struct MomentumEpi {
  float *W = nullptr, *prev = nullptr;
  int ldw = 0, ldp = 0;
  float momentum = 0.0f, a_wd = 0.0f, a_g = 0.0f;
};

#ifdef __HIPCC__
namespace kcnn {
__device__ __forceinline__ void momentum_step(float g, float &prev, float &w, float momentum,
                                              float a_wd, float a_g) {
  float p = prev * momentum;        // Scale(momentum_)
  p = __builtin_fmaf(a_wd, w, p);   // AddMat(-lr * wd, W)
  p = __builtin_fmaf(a_g, g, p);    // AddMat(lr, grad)
  prev = p;
  w = p + w;                        // AddMat(1.0, prev)
}
}  // namespace kcnn
#endif

#endif  // KCNN_CNSLMAT_MOMENTUM_STEP_H_
