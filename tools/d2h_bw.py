"""Device <-> host copy bandwidth on this box (the ceiling of the host-buffer
entry points: 512 B out per 2048-bit ciphertext):

    python tools/d2h_bw.py

Times 512 MB device->pinned-host and ->pageable copies, as one copy and split
over 2/4/8 streams, plus host->device."""
import json
import time

import torch


def main():
    nbytes = 512 << 20
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda").fill_(1)
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pageable = torch.empty(nbytes, dtype=torch.uint8)
    out = {"bytes": nbytes}

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.time() - t0) / reps

    for k in (1, 2, 4, 8):
        streams = [torch.cuda.Stream() for _ in range(k)]
        per = nbytes // k

        def split(dst, src):
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    dst[i * per:(i + 1) * per].copy_(src[i * per:(i + 1) * per], non_blocking=True)
            for s in streams:
                s.synchronize()
        out[f"d2h_pinned_{k}streams_GBps"] = nbytes / timed(lambda: split(pinned, dev)) / 1e9
        out[f"h2d_pinned_{k}streams_GBps"] = nbytes / timed(lambda: split(dev, pinned)) / 1e9
    out["d2h_pageable_GBps"] = nbytes / timed(lambda: pageable.copy_(dev)) / 1e9
    out["h2d_pageable_GBps"] = nbytes / timed(lambda: dev.copy_(pageable)) / 1e9
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
