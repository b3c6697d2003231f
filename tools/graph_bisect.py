"""Which autograd-graph capture variant instantiates on this HIP runtime? Each variant runs in a
child process (a native crash ends only that child)."""
import subprocess
import sys

VARIANTS = ["torch_make_graphed", "ours_nodebug_global", "ours_nodebug_thread", "ours_debug_thread"]

CODE = r'''
import sys, torch
sys.path.insert(0, ".")
v = sys.argv[1]
torch.manual_seed(0)
lin = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.GELU(), torch.nn.Linear(64, 8)).cuda()
x = torch.randn(16, 64, device="cuda", requires_grad=True)
if v == "torch_make_graphed":
    g = torch.cuda.make_graphed_callables(lin, (x,))
    y = g(x); y.sum().backward(); torch.cuda.synchronize()
else:
    from paddle_hackathon_amd.device.cuda import graphs as G
    if v.startswith("ours_nodebug"):
        G._NO_DEBUG = True
    mode = "global" if v.endswith("global") else "thread_local"
    ent = G._AutogradGraphs(lambda t: lin(t), (x,), {}, list(lin.parameters()), mode, None)
    y = ent((x,), {})[0] if isinstance(ent((x,), {}), (list, tuple)) else ent((x,), {})
    y.sum().backward(); torch.cuda.synchronize()
print("OK", v, float(x.grad.abs().sum()))
'''

for v in VARIANTS:
    r = subprocess.run([sys.executable, "-c", CODE, v], capture_output=True, text=True, timeout=120)
    tail = (r.stdout + r.stderr).strip().splitlines()[-3:]
    print(v, "rc", r.returncode, tail, flush=True)
