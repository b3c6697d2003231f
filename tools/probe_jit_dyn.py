import numpy as np, traceback, tempfile, os
import paddle_hackathon_amd as paddle
class Net(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc = paddle.nn.Linear(4, 4)
    def forward(self, x):
        y = self.fc(x)
        nz = paddle.nonzero(y > 0)
        ms = paddle.masked_select(y, y > 0)
        u = paddle.unique(paddle.cast(x > 0, "int64"))
        return y, nz, ms, u
net = Net()
x = paddle.to_tensor(np.random.RandomState(0).randn(3, 4).astype("float32"))
ref = [o.numpy() for o in net(x)]
try:
    st = paddle.jit.to_static(net, input_spec=[paddle.static.InputSpec([None, 4], "float32")])
    got = [o.numpy() for o in st(x)]
    for a, b in zip(ref, got):
        np.testing.assert_allclose(a, b, rtol=1e-6)
    d = tempfile.mkdtemp()
    paddle.jit.save(st, os.path.join(d, "m"))
    ld = paddle.jit.load(os.path.join(d, "m"))
    got2 = [o.numpy() for o in ld(x)]
    for a, b in zip(ref, got2):
        np.testing.assert_allclose(a, b, rtol=1e-6)
    print("OK jit", [g.shape for g in got2])
except Exception:
    traceback.print_exc()
