"""Cross-stream hop via HIP stream memory operations (hipStreamWriteValue32 on the producer stream,
hipStreamWaitValue32 on the consumer stream) against hipEventRecord / hipStreamWaitEvent, in the
ping-pong pattern of tools/xstream_probe.py.  python3 tools/waitvalue_probe.py"""
import ctypes
import time
import torch

torch.cuda.init()
hip = ctypes.CDLL('libamdhip64.so')
hip.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint]
hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
GEQ = 0        # hipStreamWaitValueGte
A, B = torch.cuda.Stream(), torch.cuda.Stream()
N = 200


def run(kind, cyc, flag):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(N):
        with torch.cuda.stream(A):
            if i:
                if kind == 'event':
                    A.wait_event(evs[2 * i - 1])
                else:
                    assert hip.hipStreamWaitValue32(A.cuda_stream, flag.value + 4, i, GEQ, 0xffffffff) == 0
            torch.cuda._sleep(cyc)
            if kind == 'event':
                evs[2 * i].record(A)
            else:
                assert hip.hipStreamWriteValue32(A.cuda_stream, flag.value, i + 1, 0) == 0
        with torch.cuda.stream(B):
            if kind == 'event':
                B.wait_event(evs[2 * i])
            else:
                assert hip.hipStreamWaitValue32(B.cuda_stream, flag.value, i + 1, GEQ, 0xffffffff) == 0
            torch.cuda._sleep(cyc)
            if kind == 'event':
                evs[2 * i + 1].record(B)
            else:
                assert hip.hipStreamWriteValue32(B.cuda_stream, flag.value + 4, i + 1, 0) == 0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (2 * N)


for cyc in (200000,):
    torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2 * N):
        torch.cuda._sleep(cyc)
    torch.cuda.synchronize()
    one = (time.perf_counter() - t0) / (2 * N)
    evs = [torch.cuda.Event() for _ in range(2 * N)]
    ev = run('event', cyc, None)
    print('event hop %.2f us' % ((ev - one) * 1e6), flush=True)
    for name, alloc in (('hipMalloc', lambda p: hip.hipMalloc(ctypes.byref(p), 64)),
                        ('signal memory', lambda p: hip.hipExtMallocWithFlags(ctypes.byref(p), 64, 2))):
        flag = ctypes.c_void_p()
        rc = alloc(flag)
        if rc != 0:
            print(name, 'alloc failed', rc)
            continue
        hip.hipMemset(flag, 0, 64)
        torch.cuda.synchronize()
        wv = run('value', cyc, flag)
        print('%s wait-value hop %.2f us' % (name, (wv - one) * 1e6), flush=True)
