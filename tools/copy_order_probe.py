#!/usr/bin/env python3
"""tools/copy_order_probe.py -- why do the host pipeline's 1 GiB copies run at
~53.2 GiB/s (18.81 ms each, profiles/r06/raw/timeline_*.jsonl) when the same
copy alone runs at 53.65 (18.64 ms, tools/copy2d_probe.py)?

Eight 1 GiB H2D copies out of a registered 8 GiB image into two 1 GiB device
buffers, timed per copy with HIP events, issued
  * one stream: all eight back to back on one stream;
  * two streams: alternating between two streams, each copy waiting for the
    previous one's event (the pipeline's serial copy order);
  * two streams + hash: the same with the pipeline's hash of each batch
    (bt_sha1_chunks_dev over the 2048 chunks just copied) queued behind its
    copy on the same stream.
Best of 3 of each; per-copy ms and the 8 GiB rate.
usage: copy_order_probe.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "bittorrent-with-congestion-control_amd"))
import btsha1 as bt  # noqa: E402  (after torch: one HIP runtime)

GIB = 1 << 30
CHUNK = 512 * 1024


def main():
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    img = np.empty(8 * GIB, dtype=np.uint8)
    img.view(np.uint64)[:] = np.arange(img.size // 8, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    bt.host_register(img.ctypes.data, img.nbytes)
    try:
        dev = [torch.empty(GIB, dtype=torch.uint8, device="cuda") for _ in range(2)]
        dig = [torch.empty(20 * (GIB // CHUNK), dtype=torch.uint8, device="cuda") for _ in range(2)]
        st = [torch.cuda.Stream(), torch.cuda.Stream()]
        for mode in ("one_stream", "two_streams", "two_streams_hash"):
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(8)]
                for k in range(8):
                    s = st[0] if mode == "one_stream" else st[k & 1]
                    if k and mode != "one_stream":
                        s.wait_event(ev[k - 1][1])
                    ev[k][0].record(s)
                    rc = hip.hipMemcpyAsync(ctypes.c_void_p(dev[k & 1].data_ptr()),
                                            ctypes.c_void_p(img.ctypes.data + k * GIB), GIB, 1,
                                            ctypes.c_void_p(s.cuda_stream))
                    assert rc == 0, rc
                    ev[k][1].record(s)
                    if mode == "two_streams_hash":
                        bt.chunks_dev(dev[k & 1].data_ptr(), GIB // CHUNK, CHUNK, CHUNK, dig[k & 1].data_ptr(),
                                      stream=s.cuda_stream)
                torch.cuda.synchronize()
                per = [ev[k][0].elapsed_time(ev[k][1]) for k in range(8)]
                span = ev[0][0].elapsed_time(ev[7][1])
                if best is None or span < best[0]:
                    best = (span, per)
            print(json.dumps({"mode": mode, "span_ms": round(best[0], 3), "GiB_per_s": round(8 / best[0] * 1e3, 2),
                              "copy_ms": [round(x, 3) for x in best[1]]}), flush=True)
    finally:
        bt.host_unregister(img.ctypes.data)


if __name__ == "__main__":
    main()
