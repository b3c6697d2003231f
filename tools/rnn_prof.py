"""LSTM B=64 T=64 H=512 forward + backward on the HIP recurrent kernels (for rocprofv3 --stats)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import paddle_hackathon_amd as paddle  # noqa: E402

paddle.set_device("gpu")
paddle.seed(0)
m = paddle.nn.LSTM(512, 512)
x = paddle.randn([64, 64, 512])
x.stop_gradient = False
for _ in range(3):
    y, _ = m(x)
    y.sum().backward()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    y, _ = m(x)
    y.sum().backward()
torch.cuda.synchronize()
print(f"LSTM B64 T64 H512 fwd+bwd {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms", flush=True)
