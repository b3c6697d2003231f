import numpy as np, traceback, tempfile, os
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd import fluid
paddle.enable_static()
main, start = paddle.static.Program(), paddle.static.Program()
with paddle.static.program_guard(main, start):
    x = paddle.static.data("x", [-1, 3], "float32")
    l = paddle.static.data("l", [-1, 1], "int64")
    h = paddle.static.nn.fc(x, 3)
    nz = paddle.nonzero(h > 0)
    ms = paddle.masked_select(h, h > 0)
    un = paddle.unique(paddle.cast(x > 0, "int64"))
    wh = fluid.layers.where(h > 0)
    pr = paddle.static.Print(h, message="h:", first_n=1)
    oh = fluid.layers.one_hot(l, 5)
    p = paddle.nn.functional.softmax(h)
    acc = fluid.layers.accuracy(p, l)
    g_auc, b_auc, _ = fluid.layers.auc(paddle.nn.functional.softmax(paddle.static.nn.fc(x, 2)), l, num_thresholds=99)
print([v.shape for v in (nz, ms, un, wh)])
exe = paddle.static.Executor(); exe.run(start)
X = np.random.RandomState(0).randn(4, 3).astype("float32"); L = np.array([[1],[0],[2],[1]], "int64")
outs = exe.run(main, feed={"x": X, "l": L}, fetch_list=[nz, ms, un, wh, pr, oh, acc, g_auc])
print([o.shape for o in outs])
d = tempfile.mkdtemp()
try:
    paddle.static.save_inference_model(os.path.join(d, "m"), [x, l], [nz, ms, un, wh, oh, acc], exe, program=main)
    from paddle_hackathon_amd.static import proto as pb
    prog, feeds, fetches = paddle.static.load_inference_model(os.path.join(d, "m"), exe)
    outs2 = exe.run(prog, feed={"x": X, "l": L}, fetch_list=fetches)
    for a, b in zip(outs[:4] + outs[5:7], outs2): np.testing.assert_allclose(a, b)
    print("saved+loaded OK")
    raw = open(os.path.join(d, "m.pdmodel"), "rb").read()
    desc = pb.ProgramDesc(); desc.ParseFromString(raw)
    print(sorted({o.type for o in desc.blocks[0].ops}))
except Exception:
    traceback.print_exc()
