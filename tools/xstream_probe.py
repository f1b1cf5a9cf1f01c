"""Cross-stream event latency without a profiler.
1. N ping-pongs of a fixed-length kernel between two streams (each waits on the other's event)
   against the same 2N kernels on one stream: the cost of a hop whose event completes just before.
2. A stream whose every kernel waits on an event of another stream recorded two kernels earlier
   (already complete when reached): the cost of waiting on a satisfied event.
python3 tools/xstream_probe.py"""
import time
import torch

torch.cuda.init()
A, B = torch.cuda.Stream(), torch.cuda.Stream()
N = 200
for cyc in (20000, 200000):
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2 * N):
        torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    one = (time.perf_counter() - t0) / (2 * N)
    evs = [torch.cuda.Event() for _ in range(2 * N)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        with torch.cuda.stream(A):
            if i:
                A.wait_event(evs[2 * i - 1])
            torch.cuda._sleep(cyc)
            evs[2 * i].record(A)
        with torch.cuda.stream(B):
            B.wait_event(evs[2 * i])
            torch.cuda._sleep(cyc)
            evs[2 * i + 1].record(B)
    torch.cuda.synchronize()
    two = (time.perf_counter() - t0) / (2 * N)
    print('sleep %d cycles: one stream %.2f us/kernel, ping-pong %.2f us/kernel -> cross-stream hop %.2f us'
          % (cyc, one * 1e6, two * 1e6, (two - one) * 1e6), flush=True)
    # satisfied waits: A runs 2-kernel-long sleeps, B waits on A's event from 2 A-kernels back
    evA = [torch.cuda.Event() for _ in range(N + 2)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(B):
        for i in range(N):
            torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    alone = (time.perf_counter() - t0) / N
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        with torch.cuda.stream(A):
            torch.cuda._sleep(cyc // 2)
            evA[i].record(A)
        with torch.cuda.stream(B):
            if i >= 2:
                B.wait_event(evA[i - 2])
            torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    waited = (time.perf_counter() - t0) / N
    print('sleep %d cycles: B alone %.2f us/kernel, B waiting on satisfied events %.2f us/kernel -> %.2f us per wait'
          % (cyc, alone * 1e6, waited * 1e6, (waited - alone) * 1e6), flush=True)
