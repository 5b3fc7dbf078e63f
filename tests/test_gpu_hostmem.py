"""GPU: HBM a host call holds beyond the device context's kept staging lanes
(2 x <= 1 GiB, include/bt_sha1.h) is freed before it returns, for the
default 1 GiB direct-DMA batches (kept, never freed) and for bigger ones
(BT_SHA1_DMA_BATCH_MB=4096: grown for the call, then shrunk back to the kept
lane), registered and pageable input (page-locked batch by batch), single worker and repeated device ids
(devs=[0,0,0]).  Both ways: no call holds more than the kept lanes after it
returns, and no call frees the kept lanes either (the next staged call would
pay for pinning them again).

The batch size is read once per process, so each setting runs in a child
process; hipMemGetInfo after each call is compared with the level after a
first pageable call (staged feed) that sized the kept lanes, and every call's digests with
the oracle on sampled chunks and with each other."""
import json
import os
import subprocess
import sys

import pytest

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu
CHUNK = 512 * 1024


def _child():
    import numpy as np
    import torch
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, PKG)
    import btsha1 as bt
    import py_oracle as orc

    n = 8192  # 4 GiB: 1 GiB batches by default, 2 GiB ones (the half-image cap) with 4096 MiB
    img = np.empty(n * CHUNK, dtype=np.uint8)
    words = img.view(np.uint64)
    words[:] = np.arange(words.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    addr = img.ctypes.data
    prev = bt.set_pageable_feed("stage")
    want = bt.chunks_host_addr(addr, img.nbytes)  # pageable, staged: sizes the kept lanes
    bt.set_pageable_feed(prev)
    ok = all(want[20 * i:20 * i + 20] == orc.sha1(img[i * CHUNK:(i + 1) * CHUNK].tobytes()) for i in (0, 4097, n - 1))

    def free_now():
        torch.cuda.synchronize()
        return torch.cuda.mem_get_info()[0]
    kept = free_now()
    levels = {}
    levels["pageable"] = (bt.chunks_host_addr(addr, img.nbytes) == want, free_now())  # page-locked batch by batch
    levels["pageable_devs3"] = (bt.chunks_host_addr(addr, img.nbytes, devs=[0, 0, 0]) == want, free_now())
    bt.host_register(addr, img.nbytes)
    try:
        levels["registered"] = (bt.chunks_host_addr(addr, img.nbytes) == want, free_now())
        levels["registered_devs3"] = (bt.chunks_host_addr(addr, img.nbytes, devs=[0, 0, 0]) == want, free_now())
    finally:
        bt.host_unregister(addr)
    print("HOSTMEM " + json.dumps({"sample_ok": ok, "kept_free": kept,
                                   "calls": {k: {"digests_ok": d, "free": f} for k, (d, f) in levels.items()}}),
          flush=True)


@pytest.mark.parametrize("batch_mb", [None, 4096])
def test_host_calls_give_their_hbm_back(batch_mb):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("BT_SHA1_DMA_BATCH_MB", None)
    if batch_mb:
        env["BT_SHA1_DMA_BATCH_MB"] = str(batch_mb)
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "child"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("HOSTMEM ")]
    assert len(line) == 1, r.stdout[-2000:]
    res = json.loads(line[0].split(" ", 1)[1])
    assert res["sample_ok"]
    slack = 64 << 20
    for name, c in res["calls"].items():
        assert c["digests_ok"], name
        assert c["free"] >= res["kept_free"] - slack, (name, c["free"], res["kept_free"])  # nothing extra held
        assert c["free"] <= res["kept_free"] + slack, (name, c["free"], res["kept_free"])  # kept lanes kept


if __name__ == "__main__" and sys.argv[1:] == ["child"]:
    _child()
