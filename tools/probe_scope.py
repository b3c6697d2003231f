import numpy as np
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd import fluid
paddle.enable_static()
main, start = paddle.static.Program(), paddle.static.Program()
with paddle.static.program_guard(main, start):
    x = paddle.static.data("x", [-1, 3], "float32")
    y = paddle.static.data("y", [-1, 1], "float32")
    pred = paddle.static.nn.fc(x, 1, weight_attr=paddle.ParamAttr(name="w"), bias_attr=paddle.ParamAttr(name="b"))
    loss = paddle.mean((pred - y) ** 2)
    paddle.optimizer.Adam(0.1).minimize(loss)
exe = paddle.static.Executor()
exe.run(start)
X = np.ones((2, 3), "float32"); Y = np.zeros((2, 1), "float32")
v = fluid.global_scope().find_var("w")
print("find_var w:", v is not None, np.array(v.get_tensor()).shape)
v.get_tensor().set(np.full((3, 1), 2.0, "float32"), fluid.CPUPlace())
fluid.global_scope().find_var("b").get_tensor().set(np.zeros((1,), "float32"), fluid.CPUPlace())
p, = exe.run(main.clone(for_test=True), feed={"x": X, "y": Y}, fetch_list=[pred])
print("after set, pred =", p.ravel(), "(expect 6)")
s1, s2 = fluid.Scope(), fluid.Scope()
exe.run(start, scope=s1); exe.run(start, scope=s2)
w1 = np.array(s1.find_var("w").get_tensor()); w2 = np.array(s2.find_var("w").get_tensor())
print("fresh params differ:", not np.allclose(w1, w2))
for _ in range(3):
    exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss], scope=s1)
print("s1 trained, s2 untouched:", not np.allclose(np.array(s1.find_var("w").get_tensor()), w1),
      np.allclose(np.array(s2.find_var("w").get_tensor()), w2))
print("global w still 2:", np.array(fluid.global_scope().find_var("w").get_tensor()).ravel())
with fluid.scope_guard(s2):
    l2, = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])
print("scope_guard run uses s2:", not np.allclose(np.array(s2.find_var("w").get_tensor()), w2))
