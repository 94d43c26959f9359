import ctypes, time, numpy as np, torch, sys
sys.path.insert(0, "/root/repo")
from ratis_amd import engine
hip = ctypes.CDLL("libamdhip64.so.7")
ctx = engine.Context(0)
buf = np.zeros(1 << 20, np.uint8)
reg = engine.HostRegistration(ctx, buf)
p = ctypes.c_void_p()
def t(f, n=2000):
    t0 = time.perf_counter()
    for _ in range(n): f()
    return (time.perf_counter() - t0) / n * 1e6
print("hipHostGetDevicePointer registered us", t(lambda: hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(buf.ctypes.data + 100), 0)))
pg = np.zeros(1 << 20, np.uint8)
print("hipHostGetDevicePointer pageable us", t(lambda: (hip.hipHostGetDevicePointer(ctypes.byref(p), ctypes.c_void_p(pg.ctypes.data + 100), 0), hip.hipGetLastError())))
ev = ctypes.c_void_p(); hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
s = ctypes.c_void_p(engine._lib.load().rh_ctx_stream(ctx.handle))
print("hipEventRecord us", t(lambda: hip.hipEventRecord(ev, s)))
print("hipEventQuery us", t(lambda: hip.hipEventQuery(ev)))
print("noop ctypes us", t(lambda: hip.hipGetLastError()))
reg.close(); ctx.close()
