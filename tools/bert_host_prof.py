"""Host-side profile of the BERT-base bench step (cProfile over timed steps after warmup): where the
Python time between kernel launches goes."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.models import bert_config, BertForPretraining, BertPretrainingCriterion

paddle.set_device("gpu:0")
paddle.seed(0)
S, B = 512, 32
cfg = bert_config("bert-base", max_position_embeddings=512)
model = BertForPretraining(cfg)
crit = BertPretrainingCriterion(cfg.vocab_size)
model = paddle.amp.decorate(model, level="O2", dtype="bfloat16")
opt = paddle.optimizer.AdamW(learning_rate=1e-4, weight_decay=0.01, parameters=model.parameters(), multi_precision=True)
g = torch.Generator(device="cuda").manual_seed(0)
ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (B, S), device="cuda", generator=g))
tt = paddle.to_tensor((torch.arange(S, device="cuda") >= S // 2).long().expand(B, S).contiguous())
n_mask = int(0.15 * S)
mpos = paddle.to_tensor((torch.randperm(S, device="cuda", generator=g)[:n_mask].unsqueeze(0)
                         + S * torch.arange(B, device="cuda").unsqueeze(1)).reshape(-1))
mlab = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (B * n_mask,), device="cuda", generator=g))
nlab = paddle.to_tensor(torch.randint(0, 2, (B,), device="cuda", generator=g))


def step():
    with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
        mlm, nsp = model(ids, tt, masked_positions=mpos)
    loss = crit(mlm, nsp, mlab, nlab)
    loss.backward()
    opt.step()
    opt.clear_grad(set_to_zero=False)
    return loss


for _ in range(5):
    step()
torch.cuda.synchronize()
# host time alone: launch everything, measure the Python time per step (the GPU queue absorbs it
# until it fills)
t0 = time.perf_counter()
for _ in range(10):
    step()
t_host = (time.perf_counter() - t0) / 10
torch.cuda.synchronize()
t_all = (time.perf_counter() - t0) / 10
print(f"host issue {t_host * 1e3:.2f} ms/step, wall {t_all * 1e3:.2f} ms/step", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(40)
