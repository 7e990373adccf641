"""Host-side costs behind the host-to-host pipeline: hipHostRegister of a
caller's numpy buffer (pinning in place, no staging copy) against pageable->pinned memcpy, and the
PCIe copy rates from each.  Prints one line per measurement."""
import ctypes as ct
import time

import numpy as np

hip = ct.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ct.c_void_p, ct.c_size_t, ct.c_uint]
hip.hipHostUnregister.argtypes = [ct.c_void_p]
hip.hipMalloc.argtypes = [ct.POINTER(ct.c_void_p), ct.c_size_t]
hip.hipHostMalloc.argtypes = [ct.POINTER(ct.c_void_p), ct.c_size_t, ct.c_uint]
hip.hipMemcpy.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_size_t, ct.c_int]
hip.hipDeviceSynchronize.argtypes = []
H2D, D2H = 1, 2


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


GB = 1 << 30
for size in (256 << 20, 1 << 30):
    a = np.ones(size // 4, np.float32)   # touched: resident pageable memory
    d = ct.c_void_p()
    ok(hip.hipMalloc(ct.byref(d), size), "hipMalloc")
    t = time.perf_counter()
    ok(hip.hipHostRegister(a.ctypes.data, size, 0), "hipHostRegister")
    tr = time.perf_counter() - t
    t = time.perf_counter()
    ok(hip.hipMemcpy(d, a.ctypes.data, size, H2D), "H2D")
    th = time.perf_counter() - t
    t = time.perf_counter()
    ok(hip.hipMemcpy(a.ctypes.data, d, size, D2H), "D2H")
    td = time.perf_counter() - t
    t = time.perf_counter()
    ok(hip.hipHostUnregister(a.ctypes.data), "hipHostUnregister")
    tu = time.perf_counter() - t
    print(f"register {size / GB:.2f} GB: {size / GB / tr:.1f} GB/s register, {size / GB / tu:.1f} GB/s "
          f"unregister, H2D {size / GB / th:.1f} GB/s, D2H {size / GB / td:.1f} GB/s (registered)")
    t = time.perf_counter()
    ok(hip.hipMemcpy(d, a.ctypes.data, size, H2D), "H2D pageable")
    th = time.perf_counter() - t
    t = time.perf_counter()
    ok(hip.hipMemcpy(a.ctypes.data, d, size, D2H), "D2H pageable")
    td = time.perf_counter() - t
    print(f"pageable {size / GB:.2f} GB: H2D {size / GB / th:.1f} GB/s, D2H {size / GB / td:.1f} GB/s")
    p = ct.c_void_p()
    ok(hip.hipHostMalloc(ct.byref(p), size, 0), "hipHostMalloc")
    pa = np.ctypeslib.as_array(ct.cast(p, ct.POINTER(ct.c_float)), (size // 4,))
    t = time.perf_counter()
    np.copyto(pa, a)
    tc = time.perf_counter() - t
    t = time.perf_counter()
    ok(hip.hipMemcpy(d, p, size, H2D), "H2D pinned")
    th = time.perf_counter() - t
    t = time.perf_counter()
    ok(hip.hipMemcpy(p, d, size, D2H), "D2H pinned")
    td = time.perf_counter() - t
    print(f"pinned {size / GB:.2f} GB: one-thread memcpy {size / GB / tc:.1f} GB/s, H2D {size / GB / th:.1f} GB/s, "
          f"D2H {size / GB / td:.1f} GB/s")


# both directions at once (two streams), registered (4 KiB pages) vs hipHostMalloc memory
hip.hipStreamCreate.argtypes = [ct.POINTER(ct.c_void_p)]
hip.hipMemcpyAsync.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_size_t, ct.c_int, ct.c_void_p]
hip.hipStreamSynchronize.argtypes = [ct.c_void_p]
s1, s2 = ct.c_void_p(), ct.c_void_p()
ok(hip.hipStreamCreate(ct.byref(s1)), "stream")
ok(hip.hipStreamCreate(ct.byref(s2)), "stream")
size = 1 << 30
d1, d2 = ct.c_void_p(), ct.c_void_p()
ok(hip.hipMalloc(ct.byref(d1), size), "hipMalloc")
ok(hip.hipMalloc(ct.byref(d2), size), "hipMalloc")
a = np.ones(size // 4, np.float32)
b = np.ones(size // 4, np.float32)
ok(hip.hipHostRegister(a.ctypes.data, size, 0), "reg")
ok(hip.hipHostRegister(b.ctypes.data, size, 0), "reg")
for label, src, dst in (("registered", a.ctypes.data, b.ctypes.data),):
    for _ in range(2):
        t = time.perf_counter()
        ok(hip.hipMemcpyAsync(d1, src, size, H2D, s1), "h2d")
        ok(hip.hipMemcpyAsync(dst, d2, size, D2H, s2), "d2h")
        ok(hip.hipStreamSynchronize(s1), "sync")
        ok(hip.hipStreamSynchronize(s2), "sync")
        dt = time.perf_counter() - t
    print(f"bidirectional {label} 1 GB each way: {2 * size / GB / dt:.1f} GB/s combined")
ok(hip.hipHostUnregister(a.ctypes.data), "unreg")
ok(hip.hipHostUnregister(b.ctypes.data), "unreg")
p1, p2 = ct.c_void_p(), ct.c_void_p()
ok(hip.hipHostMalloc(ct.byref(p1), size, 0), "hm")
ok(hip.hipHostMalloc(ct.byref(p2), size, 0), "hm")
for _ in range(2):
    t = time.perf_counter()
    ok(hip.hipMemcpyAsync(d1, p1, size, H2D, s1), "h2d")
    ok(hip.hipMemcpyAsync(p2, d2, size, D2H, s2), "d2h")
    ok(hip.hipStreamSynchronize(s1), "sync")
    ok(hip.hipStreamSynchronize(s2), "sync")
    dt = time.perf_counter() - t
print(f"bidirectional hipHostMalloc 1 GB each way: {2 * size / GB / dt:.1f} GB/s combined")
