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


def run_mmap(d, nthreads, blocks=200, size=1 << 20, populate=True, cold=True):
    """Extend the file, map the new range (MAP_POPULATE: the kernel allocates the page-cache
    pages in one go), copy into it from ``nthreads`` threads.  cold: a fresh source buffer per
    block (as a D2H snapshot: not in the CPU caches)."""
    import mmap
    src = [np.random.default_rng(b).random(size // 8) for b in range(8 if cold else 1)]
    path = os.path.join(d, f"probe_mm_{os.getpid()}_{nthreads}.bin")
    fd = os.open(path, os.O_CREAT | os.O_TRUNC | os.O_RDWR, 0o644)
    flags = mmap.MAP_SHARED | (getattr(mmap, "MAP_POPULATE", 0x8000) if populate else 0)
    try:
        t0 = time.perf_counter()
        for b in range(blocks):
            off = b * size
            os.ftruncate(fd, off + size)
            m = mmap.mmap(fd, size, flags=flags, prot=mmap.PROT_WRITE | mmap.PROT_READ, offset=off)
            dst = np.frombuffer(m, dtype=np.float64)
            s = src[b % len(src)]
            if nthreads <= 1:
                np.copyto(dst, s)
            else:
                k = len(s) // nthreads
                fs = [POOL.submit(np.copyto, dst[i * k:(i + 1) * k], s[i * k:(i + 1) * k]) for i in range(nthreads)]
                for f in fs:
                    f.result()
            del dst
            m.close()
        dt = time.perf_counter() - t0
    finally:
        os.close(fd)
        os.unlink(path)
    return {"dir": d, "mmap_threads": nthreads, "populate": populate, "cold": cold,
            "us_per_MiB": round(1e6 * dt / blocks * (1 << 20) / size, 1)}


def run_cold(d, blocks=200, size=1 << 20):
    """write() from a source that is not in the CPU caches (8 rotating 1 MiB buffers)."""
    src = [np.random.default_rng(b).random(size // 8).tobytes() for b in range(8)]
    path = os.path.join(d, f"probe_cold_{os.getpid()}.bin")
    fd = os.open(path, os.O_CREAT | os.O_TRUNC | os.O_WRONLY, 0o644)
    try:
        t0 = time.perf_counter()
        for b in range(blocks):
            os.write(fd, src[b % 8])
        dt = time.perf_counter() - t0
    finally:
        os.close(fd)
        os.unlink(path)
    return {"dir": d, "write_cold": True, "us_per_MiB": round(1e6 * dt / blocks, 1)}


def main():
    dirs = sys.argv[1:] or [tempfile.gettempdir(), os.getcwd()]
    for d in dirs:
        for n in (0, 0, 2):
            print(json.dumps(run(d, n)), flush=True)
        print(json.dumps(run_cold(d)), flush=True)
        for n in (1, 2, 4, 8):
            print(json.dumps(run_mmap(d, n)), flush=True)
        print(json.dumps(run_mmap(d, 4, populate=False)), flush=True)


if __name__ == "__main__":
    main()
