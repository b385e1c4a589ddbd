"""The RCCL halo transport on ONE MI355X: loopback mode.

RCCL refuses two ranks on one GPU, so the multi-rank runs in test_gpu_multirank.py use the
host-staged transport.  Here a single rank with periodic wraps sends its halos to ITSELF
through RCCL (``GrayScott(..., loopback=True)``, engine.h ``set_loopback``): the grouped
ncclSend/ncclRecv calls, the packed and the in-place (z-plane) message paths, the comm stream,
the overlapped inner-plane update and the watchdog wait all run on the device exactly as they
do between ranks on the 8-GPU node.  The result must be bit-identical to the same rank
exchanging through plain device self copies.
"""
import dataclasses

import numpy as np
import pytest
import torch

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _settings(prec="Float32", overlap="auto"):
    return Settings(L=32, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                    backend="AMDGPU", seed=4321, overlap=overlap)


def _z_only(dom):
    """1-rank domain whose only neighbours are the z wraps (x, y keep the reference's
    non-periodic boundary): the halo plan becomes whole contiguous planes (zplanes)."""
    nbr = [r if (i // 9 == 1 and (i // 3) % 3 == 1) or i == 13 else -1
           for i, r in enumerate(dom.nbr27)]
    return dataclasses.replace(dom, periodic=False, nbr27=nbr)


def _run(dom, s, fuse, steps, loopback, randomize=True):
    sim = GrayScott(s, dom, fuse=fuse, loopback=loopback)
    try:
        sim.init_fields()
        if randomize:
            sim.randomize_fields(seed=7)
        sim.iterate(steps)
        sim.synchronize()
        u, v = sim.get_fields()
        info = {"transport": sim.transport, "overlapped": sim.overlapped,
                "zplanes": sim.engine.plan()["zplanes"]}
    finally:
        sim.close()
    return u, v, info


@pytest.mark.parametrize("L,fuse,prec", [(32, 2, "Float32"), (40, 3, "Float32"),
                                         (32, 1, "Float64"), (36, 2, "Float64")])
def test_rccl_loopback_periodic_packed(L, fuse, prec):
    """Fully periodic rank: 26 packed messages to itself through one RCCL group."""
    dom = init_domain(L, 1, 0, periodic=True)
    s = _settings(prec)
    s.L = L
    u0, v0, i0 = _run(dom, s, fuse, 11, loopback=False)
    u1, v1, i1 = _run(dom, s, fuse, 11, loopback=True)
    assert i0["transport"] == "none" and i1["transport"] == "rccl"
    assert not i1["zplanes"]
    # fused passes overlap the packed exchange with the inner tiles (engine.h overlapped)
    assert i1["overlapped"] == (fuse > 1 and L >= 2 * fuse + 1)
    assert np.isfinite(u1).all() and np.isfinite(v1).all()
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)


@pytest.mark.parametrize("L,fuse,prec", [(48, 2, "Float32"), (48, 3, "Float32"),
                                         (40, 2, "Float64")])
def test_rccl_loopback_zplanes_overlapped(L, fuse, prec):
    """z wraps only: in-place RCCL plane halos on the comm stream, overlapped with the
    inner-plane kernel (the 8-GPU z-slab data path), vs device self copies."""
    dom = _z_only(init_domain(L, 1, 0, periodic=True))
    s = _settings(prec, overlap="on")
    s.L = L
    u0, v0, i0 = _run(dom, s, fuse, 13, loopback=False)
    u1, v1, i1 = _run(dom, s, fuse, 13, loopback=True)
    assert i1["transport"] == "rccl" and i1["zplanes"] and i1["overlapped"]
    assert not i0["overlapped"]
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)


def test_rccl_loopback_zplanes_not_inplace(monkeypatch):
    """GS_INPLACE_HALO=0 (bench.py's first fallback): packed z-plane messages via RCCL."""
    monkeypatch.setenv("GS_INPLACE_HALO", "0")
    dom = _z_only(init_domain(48, 1, 0, periodic=True))
    s = _settings(overlap="on")
    s.L = 48
    u0, v0, _ = _run(dom, s, 3, 10, loopback=False)
    u1, v1, i1 = _run(dom, s, 3, 10, loopback=True)
    assert i1["transport"] == "rccl"
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)


@pytest.mark.parametrize("mode", ["zplanes", "packed"])
@pytest.mark.parametrize("chain", ["1", "0"])
def test_rccl_loopback_chained_long_run(mode, chain, debug_knob):
    """Many chained passes (advance_chained: exchange -> end slabs -> next exchange on the comm
    stream, inner part on the compute stream) stay bit-identical to self copies, also with a
    trailing partial pass that leaves the chain; and the same run one overlapped pass at a time
    (debug switch overlap_chain = 0: inner launch ordered after the RCCL launch by an event
    mark)."""
    debug_knob("overlap_chain", int(chain))
    L = 48
    dom = init_domain(L, 1, 0, periodic=True)
    if mode == "zplanes":
        dom = _z_only(dom)
    s = _settings(overlap="on")
    s.L = L
    u0, v0, _ = _run(dom, s, 3, 3 * 20 + 2, loopback=False)
    u1, v1, i1 = _run(dom, s, 3, 3 * 20 + 2, loopback=True)
    assert i1["overlapped"] and i1["transport"] == "rccl"
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)

