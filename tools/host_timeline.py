"""Workload for a rocprofv3 timeline of the host-buffer encrypt pipeline
(xhe_encrypt_f64_host, 1 M float64 -> reused host buffers), e.g.

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- \
        python tools/host_timeline.py

then tools/host_timeline.py --analyze DIR prints per-call busy/idle time of
the kernels and copies.
"""
import ctypes
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n=1_000_000, win=20, reps=3):
    from bench import make_key
    from xfl_amd import _native as nat
    p, q, nn, h = make_key(2048, seed=2024)
    dk = nat.DeviceKey(2048, nn, p, q, h, device=0, win_bits=win)
    L = nat.lib()
    x = np.random.default_rng(0).standard_normal(n)
    ct = np.empty((n, dk.n2w), np.uint32)
    ex = np.empty(n, np.int32)
    st = np.empty(n, np.int32)
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)
    for i in range(reps + 1):
        t0 = time.time()
        nat.check(L.xhe_encrypt_f64_host(dk.handle, vp(x), n, 7, 0, 0, 1, bytes(32), 1 + i, vp(ct), vp(ex), vp(st)))
        print(f"call {i}: {(time.time() - t0) * 1e3:.1f} ms", flush=True)


def analyze(d):
    import csv
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("K:" + r["Kernel_Name"].split("(")[0][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append(("C:" + r.get("Direction", r.get("Operation", "copy")), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"])))
    rows.sort(key=lambda r: r[1])
    t0 = rows[0][1]
    busy = {}
    for name, s, e in rows:
        b = busy.setdefault(name, [0, 0])
        b[0] += e - s
        b[1] += 1
    span = (rows[-1][2] - t0) / 1e6
    print(f"span {span:.1f} ms, {len(rows)} records")
    for k, (t, c) in sorted(busy.items(), key=lambda kv: -kv[1][0]):
        print(f"{k:50s} {c:5d} x  {t / 1e6 / max(c, 1):8.3f} ms avg  {t / 1e6:9.1f} ms total")
    # gaps with no kernel running, over the last call
    ks = [(s, e) for n, s, e in rows if n.startswith("K:")]
    last = ks[-len(ks) // 4:] if len(ks) > 8 else ks
    cur_end, idle = last[0][1], 0
    for s, e in last[1:]:
        if s > cur_end:
            idle += s - cur_end
        cur_end = max(cur_end, e)
    print(f"kernel-idle time in the last quarter of launches: {idle / 1e6:.2f} ms over "
          f"{(cur_end - last[0][0]) / 1e6:.2f} ms")
    for name, s, e in rows[-40:]:
        print(f"{(s - t0) / 1e6:10.3f} {(e - s) / 1e6:8.3f} {name}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
