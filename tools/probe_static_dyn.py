import numpy as np, traceback
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd import fluid
paddle.enable_static()
def run(name, build, feed):
    main, start = paddle.static.Program(), paddle.static.Program()
    try:
        with paddle.static.program_guard(main, start):
            outs = build()
        exe = paddle.static.Executor()
        exe.run(start)
        res = exe.run(main, feed=feed, fetch_list=list(outs))
        print("OK  ", name, [np.asarray(r).shape for r in res])
    except Exception as e:
        print("FAIL", name, type(e).__name__, str(e).split("\n")[0][:150])
X = np.array([[1., 0., 2.], [0., 3., 0.]], "float32")
def b1():
    x = paddle.static.data("x", [2, 3], "float32"); return [paddle.nonzero(x)]
run("nonzero", b1, {"x": X})
def b2():
    x = paddle.static.data("x", [2, 3], "float32"); return [paddle.unique(x)]
run("unique", b2, {"x": X})
def b3():
    x = paddle.static.data("x", [2, 3], "float32"); return [paddle.masked_select(x, x > 0)]
run("masked_select", b3, {"x": X})
def b3b():
    x = paddle.static.data("x", [2, 3], "float32"); return [fluid.layers.where(x > 0)]
run("fluid.where", b3b, {"x": X})
def b4():
    x = paddle.static.data("x", [2, 3], "float32"); y = paddle.static.Print(x); return [y]
run("Print", b4, {"x": X})
def b5():
    l = paddle.static.data("l", [4, 1], "int64"); return [fluid.layers.one_hot(l, 5)]
run("one_hot", b5, {"l": np.array([[1],[0],[4],[2]], "int64")})
def b6():
    p = paddle.static.data("p", [4, 3], "float32"); l = paddle.static.data("l", [4, 1], "int64")
    return [fluid.layers.accuracy(p, l)]
run("accuracy", b6, {"p": np.random.rand(4,3).astype("float32"), "l": np.array([[1],[0],[2],[2]], "int64")})
def b7():
    p = paddle.static.data("p", [4, 2], "float32"); l = paddle.static.data("l", [4, 1], "int64")
    r = fluid.layers.auc(p, l); return [r[0]]
run("fluid.auc", b7, {"p": np.random.rand(4,2).astype("float32"), "l": np.array([[1],[0],[1],[0]], "int64")})
def b7b():
    p = paddle.static.data("p", [4, 2], "float32"); l = paddle.static.data("l", [4, 1], "int64")
    r = paddle.static.auc(p, l); return [r[0]]
run("static.auc", b7b, {"p": np.random.rand(4,2).astype("float32"), "l": np.array([[1],[0],[1],[0]], "int64")})
def b8():
    x = paddle.static.data("x", [-1, 4], "float32", lod_level=1)
    h, c = fluid.layers.dynamic_lstm(fluid.layers.fc(x, 16), size=16); return [h]
t = fluid.create_lod_tensor(np.random.rand(5, 4).astype("float32"), [[2, 3]], fluid.CPUPlace())
run("dynamic_lstm", b8, {"x": t})
def b9():
    x = paddle.static.data("x", [-1, 4], "float32", lod_level=1)
    h = fluid.layers.dynamic_gru(fluid.layers.fc(x, 12), size=4); return [h]
run("dynamic_gru", b9, {"x": t})
def b10():
    x = paddle.static.data("x", [-1, 4], "float32", lod_level=1)
    return [paddle.static.nn.sequence_pool(x, "sum")]
run("static.nn.sequence_pool", b10, {"x": t})
def b11():
    h = paddle.static.data("h", [-1, 1], "int64", lod_level=1); r = paddle.static.data("r", [-1, 1], "int64", lod_level=1)
    d, n = fluid.layers.edit_distance(h, r); return [d]
th = fluid.create_lod_tensor(np.array([[1],[2],[3],[1],[2]], "int64"), [[3, 2]], fluid.CPUPlace())
tr = fluid.create_lod_tensor(np.array([[1],[3],[1],[2],[2]], "int64"), [[2, 3]], fluid.CPUPlace())
run("edit_distance", b11, {"h": th, "r": tr})
def b12():
    bb = paddle.static.data("bb", [1, 4, 4], "float32"); sc = paddle.static.data("sc", [1, 2, 4], "float32")
    return [fluid.layers.multiclass_nms(bb, sc, 0.1, 10, 5)]
boxes = np.array([[[0,0,1,1],[0,0,1,1.1],[2,2,3,3],[5,5,6,6]]], "float32")
scores = np.random.rand(1, 2, 4).astype("float32")
run("multiclass_nms", b12, {"bb": boxes, "sc": scores})
