"""fp32 library GEMM times for the fc backward shapes (torch.matmul -> hipBLASLt/rocBLAS)."""
import torch
torch.backends.cuda.matmul.allow_tf32 = False
dev = 'cuda'
def t(f, it=50):
    for _ in range(5): f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it): f()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3
dl3 = torch.randn(1280, 256, device=dev); W = torch.randn(2592, 256, device=dev); l2 = torch.randn(1280, 2592, device=dev)
out = torch.empty(1280, 2592, device=dev)
print('dl2 = dl3 W^T      %.1f us' % t(lambda: torch.matmul(dl3, W.t(), out=out)))
o2 = torch.empty(2592, 256, device=dev)
print('dW = l2^T dl3      %.1f us' % t(lambda: torch.matmul(l2.t(), dl3, out=o2)))
o3 = torch.empty(256, 256, device=dev); a2 = torch.randn(256, 2592, device=dev)
print('fc fwd 256x2592x256 %.1f us' % t(lambda: torch.matmul(a2, W.t().contiguous()[:2592], out=o3) if False else torch.matmul(a2, torch.randn(2592,256,device=dev), out=o3)))
Wf = torch.randn(2592, 256, device=dev)
print('fc fwd (W only)     %.1f us' % t(lambda: torch.matmul(a2, Wf, out=o3)))
