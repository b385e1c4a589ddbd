"""Host cost of the output snapshot's pieces on one MI355X (the example's L=64 rank): the native
snapshot call vs its parts (compaction launch, D2H copies into pinned memory, events).

  python experiments/r5/snap_probe.py [L]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def c_void(x):
    import ctypes
    return ctypes.c_void_p(x)


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    s = Settings(L=L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU")
    sim = GrayScott(s, init_domain(L, 1, 0), fuse=3)
    sim.init_fields()
    n = 200

    def timeit(name, fn, sync=True):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        if sync:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"what": name, "host_us_per_call": round(1e6 * (t1 - t0) / n, 1),
                          "with_sync_us_per_call": round(1e6 * (t2 - t0) / n, 1)}), flush=True)

    for native_snap in (True, False):
        for mm in (True, False):
            GrayScott.native_snapshot = native_snap
            slot = f"probe{int(native_snap)}{int(mm)}"
            timeit(f"snapshot_fields native={native_snap} minmax={mm}",
                   lambda: sim.snapshot_fields(slot, depth=2, minmax=mm))
    GrayScott.native_snapshot = True
    dev = torch.empty(sim.local_shape, device=sim.device)
    dev2 = torch.empty(sim.local_shape, device=sim.device)
    timeit("engine.extract (launch)", lambda: sim.engine.extract(dev.data_ptr(), dev2.data_ptr()))
    pin = torch.empty(sim.local_shape, pin_memory=True)
    io = torch.cuda.Stream(sim.device)

    def d2h():
        with torch.cuda.stream(io):
            pin.copy_(dev, non_blocking=True)
    timeit("torch D2H 1 MiB pinned (io stream)", d2h)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                   ctypes.c_void_p]
    nb = pin.numel() * 4
    timeit("hipMemcpyAsync D2H 1 MiB torch-pinned",
           lambda: hip.hipMemcpyAsync(pin.data_ptr(), dev.data_ptr(), nb, 2, c_void(io.cuda_stream)))
    hp = ctypes.c_void_p()
    hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(nb), ctypes.c_uint(0))
    timeit("hipMemcpyAsync D2H 1 MiB hipHostMalloc",
           lambda: hip.hipMemcpyAsync(hp.value, dev.data_ptr(), nb, 2, c_void(io.cuda_stream)))
    timeit("hipMemcpyAsync D2D 1 MiB",
           lambda: hip.hipMemcpyAsync(dev2.data_ptr(), dev.data_ptr(), nb, 3, c_void(io.cuda_stream)))
    # the native call's sequence, one HIP call at a time (host us per call, back to back)
    comp = torch.cuda.current_stream(sim.device).cuda_stream
    evs = [native.NativeEvent() for _ in range(6)]
    hip.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    acc = {}
    pk = [0]
    for it in range(n + 1):
        prev, ready, done = evs[pk[0] % 6], evs[(pk[0] + 1) % 6], evs[(pk[0] + 2) % 6]
        pk[0] += 2
        steps = [("wait prev", lambda: hip.hipStreamWaitEvent(c_void(comp), c_void(prev.ptr), 0)),
                 ("extract", lambda: sim.engine.extract(dev.data_ptr(), dev2.data_ptr())),
                 ("record ready", lambda: hip.hipEventRecord(c_void(ready.ptr), c_void(comp))),
                 ("io waits ready", lambda: hip.hipStreamWaitEvent(c_void(io.cuda_stream), c_void(ready.ptr), 0)),
                 ("D2H u", lambda: hip.hipMemcpyAsync(pin.data_ptr(), dev.data_ptr(), nb, 2, c_void(io.cuda_stream))),
                 ("D2H v", lambda: hip.hipMemcpyAsync(hp.value, dev2.data_ptr(), nb, 2, c_void(io.cuda_stream))),
                 ("record done", lambda: hip.hipEventRecord(c_void(done.ptr), c_void(io.cuda_stream)))]
        for name, fn in steps:
            t0 = time.perf_counter()
            fn()
            if it:
                acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
    torch.cuda.synchronize()
    print(json.dumps({"what": "native sequence, host us per HIP call",
                      **{k: round(1e6 * v / n, 1) for k, v in acc.items()}}), flush=True)
    # the native call itself, without the Python ring around it
    hu = torch.empty(sim.local_shape, pin_memory=True)
    hv = torch.empty(sim.local_shape, pin_memory=True)
    dpart = torch.empty(4 * 2048, device=sim.device)
    hpart = torch.empty(4 * 2048, pin_memory=True)
    for label, use_prev, mm in (("native call", True, False), ("native call, no prev", False, False),
                                ("native call, minmax", True, True)):
        state = {"k": 0, "prev": None}

        def call():
            k = state["k"]
            state["k"] = (k + 2) % 6
            ready, done = evs[k], evs[k + 1]
            sim.engine.snapshot(dev.data_ptr(), dev2.data_ptr(), dpart.data_ptr() if mm else 0, 2048,
                                hu.data_ptr(), hv.data_ptr(), hpart.data_ptr() if mm else 0,
                                io.cuda_stream, state["prev"] if use_prev else None, ready, done)
            state["prev"] = done
        timeit(label, call)
    ev = native.NativeEvent()
    timeit("native event sync", ev.synchronize)
    a = torch.empty(1, device=sim.device)
    timeit("torch tiny kernel", lambda: a.add_(1))
    sim.close()


if __name__ == "__main__":
    main()
