"""Bisect the wrapped-Layer autograd capture crash over the framework's own layers (child
processes; a native crash ends only that child)."""
import subprocess
import sys

CODE = r'''
import sys, os, torch
sys.path.insert(0, ".")
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.device.cuda import graphs as G
v = sys.argv[1]
paddle.set_device("gpu:0")
paddle.seed(0)
class M(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.linear = paddle.nn.Linear(10, 20)
    def forward(self, x):
        y = self.linear(x)
        if "relu" in v: y = paddle.nn.functional.relu(y)
        if "gelu" in v: y = paddle.nn.functional.gelu(y)
        return y
m = M()
if "debug0" in v: G._NO_DEBUG = True
f = G.wrap_cuda_graph(m)
for i in range(4):
    x = paddle.randn([3, 10], dtype="float32"); x.stop_gradient = False
    loss = f(x * x + 100).mean(); loss.backward()
    print("step", i, float(x.grad.abs().sum()), flush=True)
    m.clear_gradients()
torch.cuda.synchronize()
print("OK", v)
'''

for v in ["linear", "linear_relu", "linear_gelu", "linear_relu_gelu", "linear_relu_gelu_debug0"]:
    r = subprocess.run([sys.executable, "-c", CODE, v], capture_output=True, text=True, timeout=120)
    out = [l for l in (r.stdout + r.stderr).splitlines() if "Warning" not in l and "return Variable" not in l]
    print(v, "rc", r.returncode, out[-4:], flush=True)
