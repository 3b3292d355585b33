"""Weight-gradient GEMMs of the Solver update (dW = dY^T X over the 16,384-row minibatch:
fc_spatial 1024 -> 256, LSTM W_ih 256 -> 512, W_hh 128 -> 512, the two heads 128 -> 128):
one torch GEMM against a split-K form (K in S chunks as one batched GEMM, the S partials
summed in a fixed order).  HIP events, 50 reps after warm-up."""
import json
import torch

dev = torch.device("cuda:0")
M = 16384
shapes = [(1024, 256), (256, 512), (128, 512), (128, 128), (128, 128)]
torch.manual_seed(0)
xs = [torch.randn(M, i, device=dev) for i, o in shapes]
ds = [torch.randn(M, o, device=dev) for i, o in shapes]


def one():
    return [d.t() @ x for x, d in zip(xs, ds)]


def split(S):
    def f():
        out = []
        for x, d in zip(xs, ds):
            xb = x.view(S, M // S, x.shape[1])
            db = d.view(S, M // S, d.shape[1])
            out.append(torch.bmm(db.transpose(1, 2), xb).sum(0))
        return out
    return f


def t(f, reps=50):
    for _ in range(5):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


res = {"one_gemm_us": t(one)}
ref = one()
for S in (4, 8, 16, 32):
    res["split%d_us" % S] = t(split(S))
    res["split%d_maxrel" % S] = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(split(S)(), ref))
print(json.dumps(res))
