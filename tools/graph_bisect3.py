"""Third bisect of the wrapped-Layer capture crash: prior eager backward or not, torch vs
framework Linear (child processes)."""
import subprocess
import sys

CODE = r'''
import sys, torch
sys.path.insert(0, ".")
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.device.cuda import graphs as G
v = sys.argv[1]
paddle.set_device("gpu:0")
torch.manual_seed(0)
if v.startswith("torch"):
    lin = torch.nn.Linear(10, 20).cuda()
    params = list(lin.parameters())
    fn = lambda t: lin(t)
    mk = lambda: (torch.randn(3, 10, device="cuda") ** 2 + 100).requires_grad_()
else:
    lin = paddle.nn.Linear(10, 20)
    params = [p._t for p in lin.parameters()]
    fn = lambda t: lin(t)
    def mk():
        x = paddle.randn([3, 10], dtype="float32"); x.stop_gradient = False
        return x * x + 100
if "eager" in v:
    y = fn(mk()); (y._t if hasattr(y, "_t") else y).sum().backward()
    print("eager done", flush=True)
x = mk()
ent = G._AutogradGraphs(fn, (x,), {}, params, "global" if "global" in v else "thread_local", None)
print("captured", flush=True)
out = ent((x,), {})
o = out._t if hasattr(out, "_t") else out
o.sum().backward(); torch.cuda.synchronize()
print("OK", v)
'''

for v in ["torch_noeager", "torch_eager", "pha_noeager", "pha_eager", "pha_eager_global"]:
    r = subprocess.run([sys.executable, "-c", CODE, v], capture_output=True, text=True, timeout=120)
    out = [l for l in (r.stdout + r.stderr).splitlines() if "Warning" not in l and "return Variable" not in l
           and "amdgpu.ids" not in l]
    print(v, "rc", r.returncode, out[-5:], flush=True)
