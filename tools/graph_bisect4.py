"""Fourth bisect of the autograd-capture crash: what before the capture triggers it."""
import subprocess
import sys

CODE = r'''
import sys, torch
sys.path.insert(0, ".")
v = sys.argv[1]
torch.manual_seed(0)
if "setdev" in v:
    import paddle_hackathon_amd as paddle
    paddle.set_device("gpu:0")
from paddle_hackathon_amd.device.cuda import graphs as G
lin = torch.nn.Linear(10, 20).cuda()
params = list(lin.parameters())
fn = lambda t: lin(t)
mk = lambda: (torch.randn(3, 10, device="cuda") ** 2 + 100).requires_grad_()
if "fwdonly" in v:
    with torch.no_grad():
        fn(mk())
if "eagerbwd" in v:
    fn(mk()).sum().backward()
if "sync" in v:
    torch.cuda.synchronize(); torch.cuda.empty_cache()
if "nograd" in v:
    for p in params: p.grad = None
x = mk()
if "torchgraphed" in v:
    g = torch.cuda.make_graphed_callables(lin, (x,))
    g(x).sum().backward()
else:
    ent = G._AutogradGraphs(fn, (x,), {}, params, "thread_local", None)
    out = ent((x,), {})
    out.sum().backward()
torch.cuda.synchronize()
print("OK", v)
'''

for v in ["plain", "setdev", "fwdonly", "eagerbwd", "eagerbwd_sync", "eagerbwd_nograd", "eagerbwd_torchgraphed"]:
    r = subprocess.run([sys.executable, "-c", CODE, v], capture_output=True, text=True, timeout=120)
    out = [l for l in (r.stdout + r.stderr).splitlines() if "Warning" not in l and "return Variable" not in l
           and "amdgpu.ids" not in l]
    print(v, "rc", r.returncode, out[-3:], flush=True)
