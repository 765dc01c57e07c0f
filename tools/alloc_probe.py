"""hipMalloc / first-touch / hipFree cost per size on this box (host wall time).
Usage: python tools/alloc_probe.py"""
import ctypes, time
hip = ctypes.CDLL("libamdhip64.so")
p = ctypes.c_void_p()
hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
for rep in range(2):
    for gb in (1, 4, 16, 32):
        n = ctypes.c_size_t(gb << 30)
        t = time.perf_counter(); rc = hip.hipMalloc(ctypes.byref(p), n); t1 = time.perf_counter()
        hip.hipMemset(p, 0, n); hip.hipDeviceSynchronize(); t2 = time.perf_counter()
        hip.hipMemset(p, 1, n); hip.hipDeviceSynchronize(); t3 = time.perf_counter()
        hip.hipFree(p); t4 = time.perf_counter()
        print(f"rep {rep} {gb:3d} GB rc {rc}: malloc {1e3*(t1-t):8.2f} ms  first memset {1e3*(t2-t1):8.2f} ms  "
              f"second memset {1e3*(t3-t2):8.2f} ms  free {1e3*(t4-t3):8.2f} ms", flush=True)
