"""Host-memory costs behind the serialize path on the GPU box: allocating,
first-touching and freeing ~545 MB bytes objects (fresh mmap vs a heap block
reused through glibc's free list), and the kernel's page settings.
    python tools/hostmem_probe.py"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

M_TRIM_THRESHOLD, M_MMAP_MAX = -1, -4


def main():
    import numpy as np
    from xfl_amd import _native as nat
    rec = {}
    for f in ("/proc/cmdline", "/sys/kernel/mm/transparent_hugepage/enabled",
              "/sys/kernel/mm/transparent_hugepage/defrag"):
        try:
            rec[f] = open(f).read().strip()[:300]
        except OSError as e:
            rec[f] = str(e)
    L = nat.lib()
    m = 534 << 20  # pickle bytes; n = the zstd raw frame holding them
    n = L.xhe_zstd_raw_frame_size(m)
    src = np.ones(m, np.uint8)
    libc = ctypes.CDLL(None)
    libc.mallopt.argtypes = [ctypes.c_int, ctypes.c_int]
    mk = ctypes.pythonapi.PyBytes_FromStringAndSize
    mk.restype = ctypes.py_object
    mk.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]

    def cycle(alloc, tag, reps=4):
        rows = []
        for _ in range(reps):
            t0 = time.time()
            b = alloc()
            t1 = time.time()
            out = ctypes.c_int64()
            nat.check(L.xhe_zstd_raw_frame(ctypes.c_void_p(src.ctypes.data), m, ctypes.cast(b, ctypes.c_void_p), n,
                                           ctypes.byref(out)))
            t2 = time.time()
            del b
            t3 = time.time()
            rows.append([round((t1 - t0) * 1e3, 2), round((t2 - t1) * 1e3, 2), round((t3 - t2) * 1e3, 2)])
        rec[tag + " [alloc, 16-thread fill, free] ms"] = rows

    def fresh():
        b = bytes(n)
        nat.advise_huge(ctypes.cast(b, ctypes.c_void_p).value, n)
        return b
    cycle(fresh, "bytes(n) + MADV_HUGEPAGE (mmap, calloc)")
    cycle(lambda: mk(None, n), "PyBytes_FromStringAndSize (mmap)")
    libc.mallopt(M_TRIM_THRESHOLD, 1 << 30)
    libc.mallopt(M_TRIM_THRESHOLD, 2147483647)

    def heap():
        libc.mallopt(M_MMAP_MAX, 0)
        try:
            return mk(None, n)
        finally:
            libc.mallopt(M_MMAP_MAX, 65536)
    cycle(heap, "PyBytes_FromStringAndSize (heap, no trim)")
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
