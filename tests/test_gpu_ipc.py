"""The IPC peer-write halo transport (transport = "ipc", HipBackend::ipc_*) on ONE MI355X.

Each rank exports a landing buffer and a flag array (uncached device memory) through
hipIpcGetMemHandle; the pack kernel stores every message straight into the receiving peer's
landing slot and device-side sequence flags order the exchange (no host handshake, no RCCL).
On one GPU this runs two ways:
  * loopback: one rank with periodic wraps sends its halos to ITSELF through the landing buffer
    and the flag protocol (packed and z-plane plans, overlapped and chained passes);
  * several processes sharing the device, each mapping its neighbours' buffers through IPC --
    the same code path as between GPUs, minus the xGMI hop.
Every result must be bit-identical to the single-rank run with device self copies.
"""
import dataclasses

import numpy as np
import pytest
import torch

from grayscott_amd.models.grayscott import GrayScott
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings

from .mp_utils import run_ranks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _settings(L, prec="Float32", overlap="auto"):
    return Settings(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                    backend="AMDGPU", seed=4321, overlap=overlap)


def _z_only(dom):
    nbr = [r if (i // 9 == 1 and (i // 3) % 3 == 1) or i == 13 else -1
           for i, r in enumerate(dom.nbr27)]
    return dataclasses.replace(dom, periodic=False, nbr27=nbr)


def _run(dom, s, fuse, steps, transport=None, loopback=False):
    sim = GrayScott(s, dom, fuse=fuse, transport=transport, loopback=loopback)
    try:
        sim.init_fields()
        sim.randomize_fields(seed=7)
        sim.iterate(steps)
        sim.synchronize()
        u, v = sim.get_fields()
        info = {"transport": sim.transport, "overlapped": sim.overlapped,
                "zplanes": sim.engine.plan()["zplanes"]}
    finally:
        sim.close()
    return u, v, info


@pytest.mark.parametrize("L,fuse,prec,overlap", [(32, 2, "Float32", "auto"),
                                                 (40, 3, "Float32", "on"),
                                                 (36, 3, "Float32", "off"),
                                                 (32, 2, "Float64", "auto")])
def test_ipc_loopback_periodic_packed(L, fuse, prec, overlap):
    """26 packed messages to itself through the landing buffer, 2 x 11+ exchanges (both slots
    reused)."""
    dom = init_domain(L, 1, 0, periodic=True)
    s = _settings(L, prec, overlap)
    u0, v0, _ = _run(dom, s, fuse, 23, loopback=False)
    u1, v1, i1 = _run(dom, s, fuse, 23, transport="ipc", loopback=True)
    assert i1["transport"] == "ipc" and not i1["zplanes"]
    assert np.isfinite(u1).all()
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)


@pytest.mark.parametrize("prec", ["Float32", "Float64"])
def test_ipc_system_coherent_stores(prec, debug_knob):
    """The pack's store path for peers on another GPU (relaxed system-scope stores, sc0 sc1;
    kernels.hpp store_system), forced for the loopback peer on this GPU: bit-identical to self
    copies, fp32 (one 8-byte word per cell) and fp64 (two)."""
    debug_knob("ipc_system_stores", 1)
    L = 32
    dom = init_domain(L, 1, 0, periodic=True)
    s = _settings(L, prec, "auto")
    u0, v0, _ = _run(dom, s, 2, 13, loopback=False)
    u1, v1, i1 = _run(dom, s, 2, 13, transport="ipc", loopback=True)
    assert i1["transport"] == "ipc"
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)


def test_ipc_c_api_rejects_wrong_engine():
    """The IPC / RCCL entry points check the engine's backend type: a dtype that does not match
    the engine is an error, not an unchecked cast."""
    from grayscott_amd.ops import native
    L = 16
    dom = init_domain(L, 1, 0, periodic=True)
    sim = GrayScott(_settings(L), dom, fuse=2)
    try:
        lib = sim.engine.lib
        buf = __import__("ctypes").create_string_buffer(int(lib.gs_ipc_handle_bytes()))
        assert lib.gs_ipc_export(sim.engine.h, native.DTYPE_CODES["float64"], 1, 0, buf) == -1
        assert b"fp64" in lib.gs_last_error()
        out = (__import__("ctypes").c_int32 * 3)()
        assert lib.gs_rccl_info(sim.engine.h, native.DTYPE_CODES["float64"], out) == -1
    finally:
        sim.close()


@pytest.mark.parametrize("chain", ["1", "0"])
def test_ipc_loopback_zplanes_chained(chain, debug_knob):
    """z wraps only: whole-plane messages through the landing buffer, overlapped passes chained
    on two streams (or one at a time), with a trailing partial pass."""
    debug_knob("overlap_chain", int(chain))
    L = 48
    dom = _z_only(init_domain(L, 1, 0, periodic=True))
    s = _settings(L, overlap="on")
    u0, v0, _ = _run(dom, s, 3, 3 * 15 + 2, loopback=False)
    u1, v1, i1 = _run(dom, s, 3, 3 * 15 + 2, transport="ipc", loopback=True)
    assert i1["transport"] == "ipc" and i1["zplanes"] and i1["overlapped"]
    np.testing.assert_array_equal(u1, u0)
    np.testing.assert_array_equal(v1, v0)


def _cfg(L, steps, fuse, prec="Float32", **extra):
    s = dict(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
             backend="AMDGPU", seed=1234)
    s.update(extra)
    return {"settings": s, "steps": steps, "fuse": fuse, "transport": "ipc"}


@pytest.mark.parametrize("world,L,fuse,prec,extra", [
    (2, 48, 3, "Float32", dict(decomposition="z", overlap="on")),
    (4, 40, 2, "Float64", dict(decomposition="z", overlap="off")),
    (8, 36, 2, "Float32", dict(decomposition="balanced", overlap="on")),
    (4, 32, 3, "Float32", dict(decomposition="balanced", periodic=True, overlap="auto")),
    # fuse_steps = 4 with neighbours: H = 4 halos, then the T = 4 LDS-ring pass over the whole
    # interior (no overlapped / gated T = 4 pass exists: the sequential path)
    (2, 64, 4, "Float32", dict(decomposition="z", overlap="auto")),
    (4, 64, 4, "Float32", dict(decomposition="balanced", overlap="off")),
])
def test_ipc_multiprocess_matches_single_rank(world, L, fuse, prec, extra):
    """Several processes on the GPU, neighbours' buffers mapped through IPC handles."""
    steps = 13
    u1, v1, _ = run_ranks(1, _cfg(L, steps, fuse, prec, **{k: v for k, v in extra.items()
                                                           if k == "periodic"}))
    un, vn, meta = run_ranks(world, _cfg(L, steps, fuse, prec, **extra))
    assert all(m["transport"] == "ipc" for m in meta)
    # every rank reports the peers it mapped; all on this one device here
    for m in meta:
        peers = m["info"]["ipc_peers"]
        assert peers and all(p["device"] == m["info"]["device"] for p in peers)
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


def test_ipc_halo_poisoning():
    """Every non-interior cell (ghosts, padding, halos) NaN-poisoned before the run: the IPC
    exchange must refill every ghost a stencil reads."""
    steps = 10
    u1, v1, _ = run_ranks(1, _cfg(36, steps, 3))
    cfg = _cfg(36, steps, 3, decomposition="balanced", overlap="on")
    cfg["poison"] = True
    un, vn, meta = run_ranks(4, cfg)
    assert all(m["transport"] == "ipc" for m in meta)
    assert np.isfinite(un).all() and np.isfinite(vn).all()
    np.testing.assert_array_equal(un, u1)
    np.testing.assert_array_equal(vn, v1)


def test_ipc_random_init_decomposition_invariant_L256():
    """The benchmarks' random init is keyed on the global cell: 4 ranks (2x2x1, IPC, overlapped)
    and 1 rank start from the same global state and end bit-identical at L=256 (VERDICT r2
    next #2)."""
    cfg1 = _cfg(256, 9, 3)
    cfg4 = _cfg(256, 9, 3, decomposition="balanced", overlap="on")
    cfg1.pop("transport")
    cfg1["random_init"] = cfg4["random_init"] = 2024
    u1, v1, _ = run_ranks(1, cfg1)
    u4, v4, meta = run_ranks(4, cfg4)
    assert all(m["transport"] == "ipc" for m in meta)
    assert np.isfinite(u4).all()
    np.testing.assert_array_equal(u4, u1)
    np.testing.assert_array_equal(v4, v1)


def test_ipc_long_run_matches_single_rank():
    """A long soak of the IPC flag protocol (both landing slots reused hundreds of times, the
    overlapped chain free-running ahead of the host): 4 processes, 2x2x1 grid, overlap on, 600
    steps from the random init -- bit-identical to one rank (VERDICT r2 / ADVICE r2: ordering
    of the pack's peer stores before the ready flag)."""
    cfg1 = _cfg(40, 600, 3)
    cfg4 = _cfg(40, 600, 3, decomposition="balanced", overlap="on")
    cfg1.pop("transport")
    cfg1["random_init"] = cfg4["random_init"] = 31
    u1, v1, _ = run_ranks(1, cfg1)
    u4, v4, meta = run_ranks(4, cfg4)
    assert all(m["transport"] == "ipc" and m["step"] == 600 for m in meta)
    assert np.isfinite(u4).all()
    np.testing.assert_array_equal(u4, u1)
    np.testing.assert_array_equal(v4, v1)
