"""Which aten ops (and shapes) launch the ResNet-50 step's torch-native kernels: two profiled
training steps (NHWC bf16 O2, batch 256), CPU ops grouped by input shape, sorted by the device time
of the kernels they launched. python tools/resnet_aten_ops.py [batch]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.vision.models import resnet50
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    paddle.set_device("gpu")
    paddle.seed(0)
    model = paddle.amp.decorate(resnet50(data_format="NHWC"), level="O2", dtype="bfloat16")
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    multi_precision=True)
    x = paddle.to_tensor(torch.randn(B, 224, 224, 3, device="cuda").bfloat16())
    y = paddle.to_tensor(torch.randint(0, 1000, (B,), device="cuda"))

    def step():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    steps = 2
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages(group_by_input_shape=True):
        if not e.key.startswith("aten::"):
            continue
        dev = getattr(e, "self_device_time_total", None)
        if dev is None:
            dev = e.self_cuda_time_total
        if dev <= 0:
            continue
        rows.append((dev / steps, e.count / steps, e.key, str(e.input_shapes)[:150]))
    rows.sort(reverse=True)
    print(f"aten self device time {sum(r[0] for r in rows) / 1e3:.3f} ms/step")
    for us, n, k, shp in rows[:30]:
        print(f"{us / 1e3:8.3f} ms/step {n:6.1f}/step  {k:28s} {shp}")


if __name__ == "__main__":
    main()
