// gfx950 kernels of the test custom ReLU op (launched on the framework's stream)
#include "paddle/extension.h"

template <typename data_t>
__global__ void relu_fwd_kernel(const data_t* x, data_t* y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)blockDim.x * gridDim.x)
    y[i] = x[i] > static_cast<data_t>(0) ? x[i] : static_cast<data_t>(0);
}

template <typename data_t>
__global__ void relu_bwd_kernel(const data_t* out, const data_t* g, data_t* dx, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)blockDim.x * gridDim.x)
    dx[i] = out[i] > static_cast<data_t>(0) ? g[i] : static_cast<data_t>(0);
}

std::vector<paddle::Tensor> relu_hip_forward(const paddle::Tensor& x) {
  auto out = paddle::empty_like(x);
  const int64_t n = x.numel();
  const int block = 256, grid = (int)std::min<int64_t>((n + block - 1) / block, 4096);
  PD_DISPATCH_FLOATING_AND_HALF_TYPES(x.type(), "relu_hip_forward", ([&] {
    relu_fwd_kernel<data_t><<<grid, block, 0, x.stream()>>>(x.data<data_t>(), out.data<data_t>(), n);
  }));
  return {out};
}

std::vector<paddle::Tensor> relu_hip_backward(const paddle::Tensor& out, const paddle::Tensor& grad_out) {
  auto gx = paddle::empty_like(out);
  const int64_t n = out.numel();
  const int block = 256, grid = (int)std::min<int64_t>((n + block - 1) / block, 4096);
  PD_DISPATCH_FLOATING_AND_HALF_TYPES(out.type(), "relu_hip_backward", ([&] {
    relu_bwd_kernel<data_t><<<grid, block, 0, out.stream()>>>(out.data<data_t>(), grad_out.data<data_t>(),
                                                                gx.data<data_t>(), n);
  }));
  return {gx};
}
