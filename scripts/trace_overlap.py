#!/usr/bin/env python3
"""Kernel timeline of overlapped passes on ONE MI355X through the RCCL loopback transport.

A single rank with periodic wraps sends its halos to itself through RCCL (GrayScott(...,
loopback=True)), so the real multi-rank device schedule runs: the RCCL kernel on the comm
stream next to the inner-tile / inner-plane fused kernel, then the post-exchange launches.
Run under `rocprofv3 --kernel-trace --output-format csv` and summarise with --summarise:

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl -o run -- \
      python3 scripts/trace_overlap.py --mode zplanes --L 512 --nz 64
  python3 scripts/trace_overlap.py --summarise gpurun_out/ovl
"""
import argparse
import csv
import dataclasses
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(a):
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    from grayscott_amd.ops import native

    torch.cuda.set_device(0)
    # modelling switches (csrc/include/gs/debug.h; the round-2/3 scripts passed them as
    # GS_IPC_EMULATE_US / GS_OVERLAP_CHAIN, which the libraries no longer read)
    emu = a.emulate_us if a.emulate_us is not None else float(os.environ.get("GS_IPC_EMULATE_US", 0))
    chain = a.chain if a.chain is not None else int(os.environ.get("GS_OVERLAP_CHAIN", 1))
    native.debug_set("ipc_emulate_us", emu)
    native.debug_set("overlap_chain", chain)
    L = (a.L, a.L, a.nz)
    s = Settings(L=a.L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU", overlap=a.overlap)
    dom = init_domain(L, 1, 0, periodic=True)
    if a.mode == "zplanes":  # only the z wraps: whole-plane in-place messages
        nbr = [r if (i // 9 == 1 and (i // 3) % 3 == 1) or i == 13 else -1
               for i, r in enumerate(dom.nbr27)]
        dom = dataclasses.replace(dom, periodic=False, nbr27=nbr)
    sim = GrayScott(s, dom, fuse=a.fuse, loopback=True, transport=a.transport)
    sim.init_fields()
    sim.randomize_fields(seed=1)
    sim.iterate(a.fuse * 4)
    sim.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sim.iterate(a.fuse * a.passes)
    sim.synchronize()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / a.passes * 1e6
    print(f"mode={a.mode} overlap={a.overlap} overlapped={sim.overlapped} "
          f"transport={sim.transport} chain={chain} emulate_us={emu:g} "
          f"fuse={a.fuse} us_per_pass={us:.1f}", flush=True)
    sim.close()


def summarise(root):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = [r for r in rows if "k_fused" in r["Kernel_Name"] or "ccl" in r["Kernel_Name"].lower()
            or "k_pack" in r["Kernel_Name"] or "k_ipc" in r["Kernel_Name"]
            or "k_slab" in r["Kernel_Name"]][-24:]
    t0 = int(last[0]["Start_Timestamp"])
    print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>7} queue  kernel")
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"]
        if "k_fused" in name:
            name = "k_fused<" + ",".join(name.split("FCfg<")[1].split(",")[:5]) + ">"
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {r.get('Queue_Id', '?'):>5}  "
              f"{name[:70]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["zplanes", "packed"], default="zplanes")
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--nz", type=int, default=64)
    ap.add_argument("--fuse", type=int, default=3)
    ap.add_argument("--passes", type=int, default=6)
    ap.add_argument("--overlap", choices=["on", "off"], default="on")
    ap.add_argument("--summarise", default="")
    ap.add_argument("--transport", choices=["rccl", "ipc"], default="rccl")
    ap.add_argument("--emulate-us", type=float, default=None,
                    help="hold every IPC exchange at least this long (debug switch ipc_emulate_us)")
    ap.add_argument("--chain", type=int, default=None, help="0: overlapped passes one at a time")
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a)


if __name__ == "__main__":
    main()
