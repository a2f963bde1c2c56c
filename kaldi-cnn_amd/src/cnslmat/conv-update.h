// cnslmat/conv-update.h -- a ConvolutionComponent's update applied in its
// fused backward's gradient reduction.
//
// The reference's Update (nnet-component-nnet0.cc:738-777) writes the
// gradient, then steps prev_grad_ / W / b with it (:767-775); here the frame
// kernels' backward (kcnn_conv_bwd_frame) sums its workgroup partials in
// reduce_splits_kernel, which can take the step itself: momentum_step on each
// (k, filter) element of W and prev, b += a_g * sum on the bias row, with the
// same operations and operands as ApplyGradient's MomentumBiasUpdate (the
// same bits), one kernel fewer and no gradient buffer.
//
// The caller (ConvolutionComponent::Backprop / BackpropPooled) sets a request
// for the current thread (ConvUpdateScope) around its backward call; a
// launcher that applies it sets `applied`, otherwise the caller runs
// ApplyGradient on the gradient as before.
#ifndef KCNN_CNSLMAT_CONV_UPDATE_H_
#define KCNN_CNSLMAT_CONV_UPDATE_H_

struct ConvUpdateEpi {
  float *W, *prev, *b;  // W, prev: Kdim x G (pitches ldw, ldp); b: G
  int ldw, ldp, Kdim, G;
  float momentum, a_wd, a_g;
  int applied;          // host: set by the launcher that applied the step
};

// the current thread's request (nullable); set returns the previous one
ConvUpdateEpi *kcnn_conv_update_request(ConvUpdateEpi *u);
ConvUpdateEpi *kcnn_conv_update_current();

struct ConvUpdateScope {
  ConvUpdateEpi *prev_;
  explicit ConvUpdateScope(ConvUpdateEpi *u) : prev_(kcnn_conv_update_request(u)) {}
  ~ConvUpdateScope() { kcnn_conv_update_request(prev_); }
  ConvUpdateScope(const ConvUpdateScope &) = delete;
  ConvUpdateScope &operator=(const ConvUpdateScope &) = delete;
};

#endif  // KCNN_CNSLMAT_CONV_UPDATE_H_
