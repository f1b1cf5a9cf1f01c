"""Latency from an event recorded on stream 1 to a kernel waiting on it in stream 2
(run under rocprofv3 --kernel-trace)."""
import torch
torch.cuda.init()
a = torch.randn(4096, 4096, device='cuda')
b = torch.randn(4096, 4096, device='cuda')
x = torch.zeros(16, device='cuda')
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for it in range(5):
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        c = a @ b                     # long kernel A
        ev = torch.cuda.Event()
        ev.record(s1)
        d = b @ a                     # queued follow-up work C on s1
        e2 = a @ a
    with torch.cuda.stream(s2):
        s2.wait_event(ev)
        x.add_(1.0)                   # small kernel B
    torch.cuda.synchronize()
print('done')
