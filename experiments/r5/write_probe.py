"""Host write throughput of the output path's data writes (the example's 1 MiB blocks):
sequential write() vs concurrent pwrite() to disjoint ranges of one file, on the output's
filesystem.  Informs csrc/io/bp4.cpp's data path.

  python experiments/r5/write_probe.py [dir]
"""
import json
import os
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
import time

import numpy as np


POOL = ThreadPoolExecutor(8)


def run(d, nthreads, blocks=200, size=1 << 20, chunk=None):
    buf = np.random.default_rng(0).random(size // 8).astype(np.float64).tobytes()
    path = os.path.join(d, f"probe_{os.getpid()}_{nthreads}.bin")
    fd = os.open(path, os.O_CREAT | os.O_TRUNC | os.O_WRONLY, 0o644)
    try:
        t0 = time.perf_counter()
        if nthreads == 0:
            for _ in range(blocks):
                os.write(fd, buf)
        else:
            chunk = chunk or size // nthreads
            mv = memoryview(buf)
            for b in range(blocks):
                base = b * size
                fs = [POOL.submit(os.pwrite, fd, mv[i:i + chunk], base + i) for i in range(0, size, chunk)]
                for f in fs:
                    f.result()
        dt = time.perf_counter() - t0
    finally:
        os.close(fd)
        os.unlink(path)
    return {"dir": d, "threads": nthreads, "us_per_MiB": round(1e6 * dt / blocks * (1 << 20) / size, 1),
            "GBps": round(blocks * size / dt / 1e9, 2)}


def main():
    dirs = sys.argv[1:] or [tempfile.gettempdir(), os.getcwd()]
    for d in dirs:
        for n in (0, 0, 1, 2, 4):
            print(json.dumps(run(d, n)), flush=True)


if __name__ == "__main__":
    main()
