"""Do the parallel branches of one captured hipGraph run concurrently, and what does a graph-internal
fork/join cost?  python3 tools/graph_branch_probe.py"""
import time
import torch

torch.cuda.init()
cyc = 200000
main, side = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, n=50):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def cap(body):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main):
            body()
    return g


def serial():
    torch.cuda._sleep(cyc)
    torch.cuda._sleep(cyc)


def forked():
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    side.wait_event(ev)
    torch.cuda._sleep(cyc)
    with torch.cuda.stream(side):
        torch.cuda._sleep(cyc)
    ev2 = torch.cuda.Event()
    ev2.record(side)
    cur.wait_event(ev2)


def single():
    torch.cuda._sleep(cyc)


g1, g2, g0 = cap(serial), cap(forked), cap(single)
with torch.cuda.stream(main):
    print('one sleep graph %.1f us' % timed(g0.replay))
    print('two sleeps, one stream %.1f us' % timed(g1.replay))
    print('two sleeps, forked branches %.1f us' % timed(g2.replay))
