// Test custom operator: ReLU with a CPU kernel here and a gfx950 kernel in custom_relu.hip,
// registered with its gradient op (the reference's custom_relu_op.cc pattern).
#include <algorithm>
#include <vector>

#include "paddle/extension.h"

std::vector<paddle::Tensor> relu_hip_forward(const paddle::Tensor& x);
std::vector<paddle::Tensor> relu_hip_backward(const paddle::Tensor& out, const paddle::Tensor& grad_out);

template <typename data_t>
static void relu_fwd(const data_t* x, data_t* y, int64_t n) {
  for (int64_t i = 0; i < n; ++i) y[i] = std::max(static_cast<data_t>(0), x[i]);
}

std::vector<paddle::Tensor> ReluForward(const paddle::Tensor& x) {
  if (x.is_gpu()) return relu_hip_forward(x);
  auto out = paddle::empty_like(x);
  PD_DISPATCH_FLOATING_TYPES(x.type(), "relu_fwd", ([&] { relu_fwd<data_t>(x.data<data_t>(), out.data<data_t>(), x.numel()); }));
  return {out};
}

std::vector<paddle::Tensor> ReluBackward(const paddle::Tensor& x, const paddle::Tensor& out,
                                         const paddle::Tensor& grad_out) {
  if (x.is_gpu()) return relu_hip_backward(out, grad_out);
  auto gx = paddle::empty(x.shape(), x.dtype(), x.place());
  PD_DISPATCH_FLOATING_TYPES(x.type(), "relu_bwd", ([&] {
    const data_t* o = out.data<data_t>();
    const data_t* g = grad_out.data<data_t>();
    data_t* d = gx.mutable_data<data_t>(x.place());
    for (int64_t i = 0; i < x.numel(); ++i) d[i] = o[i] > static_cast<data_t>(0) ? g[i] : static_cast<data_t>(0);
  }));
  return {gx};
}

PD_BUILD_OP(custom_relu).Inputs({"X"}).Outputs({"Out"}).SetKernelFn(PD_KERNEL(ReluForward));

PD_BUILD_GRAD_OP(custom_relu)
    .Inputs({"X", "Out", paddle::Grad("Out")})
    .Outputs({paddle::Grad("X")})
    .SetKernelFn(PD_KERNEL(ReluBackward));

// attributes + two outputs: out1 = x * scale + shift, out2 = number of elements above `thr`
std::vector<paddle::Tensor> ScaleShift(const paddle::Tensor& x, const float& scale, const int& shift,
                                       const bool& negate, const std::vector<int64_t>& dims) {
  PD_CHECK(x.is_cpu(), "scale_shift runs on host tensors");
  PD_CHECK((int64_t)dims.size() == (int64_t)x.shape().size(), "dims attr must match the rank");
  auto y = paddle::empty_like(x);
  auto cnt = paddle::empty({1}, paddle::DataType::INT64, paddle::CPUPlace());
  int64_t c = 0;
  PD_DISPATCH_FLOATING_TYPES(x.type(), "scale_shift", ([&] {
    for (int64_t i = 0; i < x.numel(); ++i) {
      data_t v = x.data<data_t>()[i] * static_cast<data_t>(scale) + static_cast<data_t>(shift);
      y.data<data_t>()[i] = negate ? -v : v;
      c += v > 0;
    }
  }));
  cnt.data<int64_t>()[0] = c;
  return {y, cnt};
}

PD_BUILD_OP(scale_shift)
    .Inputs({"X"})
    .Outputs({"Y", "Count"})
    .Attrs({"scale: float", "shift: int", "negate: bool", "dims: std::vector<int64_t>"})
    .SetKernelFn(PD_KERNEL(ScaleShift));
