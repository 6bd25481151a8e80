import torch, time
x = torch.empty(1 << 26, dtype=torch.uint8, device="cuda")
y = torch.empty(1 << 26, dtype=torch.uint8, device="cuda")
def t(f, reps=200):
    for _ in range(10): f()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1000
print("fill_ 64MiB us", t(lambda: x.fill_(3)))
print("zero_ 64MiB us", t(lambda: x.zero_()))
print("copy 64MiB us", t(lambda: y.copy_(x)))
print("sum(read) 64MiB us", t(lambda: x.view(torch.int32).sum()))
