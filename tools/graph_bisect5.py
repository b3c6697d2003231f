"""Fifth bisect: the bisect-3 setup (framework imported and device set first) against the
bisect-4 one, each run twice."""
import subprocess
import sys

CODE = r'''
import sys, torch
sys.path.insert(0, ".")
v = sys.argv[1]
if "seedfirst" in v:
    torch.manual_seed(0)
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.device.cuda import graphs as G
if "nosetdev" not in v:
    paddle.set_device("gpu:0")
torch.manual_seed(0)
lin = torch.nn.Linear(10, 20).cuda()
params = list(lin.parameters())
fn = lambda t: lin(t)
mk = lambda: (torch.randn(3, 10, device="cuda") ** 2 + 100).requires_grad_()
fn(mk()).sum().backward()
x = mk()
if "torchgraphed" in v:
    g = torch.cuda.make_graphed_callables(lin, (x,))
    g(x).sum().backward()
else:
    ent = G._AutogradGraphs(fn, (x,), {}, params, "thread_local", None)
    print("captured", flush=True)
    out = ent((x,), {})
    out.sum().backward()
torch.cuda.synchronize()
print("OK", v)
'''

for v in ["b3", "b3", "b3_seedfirst", "b3_nosetdev", "b3_torchgraphed", "b3_torchgraphed"]:
    r = subprocess.run([sys.executable, "-c", CODE, v], capture_output=True, text=True, timeout=120)
    out = [l for l in (r.stdout + r.stderr).splitlines() if "Warning" not in l and "return Variable" not in l
           and "amdgpu.ids" not in l]
    print(v, "rc", r.returncode, out[-3:], flush=True)
