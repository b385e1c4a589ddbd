"""Noise stream: bit-identical to rocRAND's Philox4x32-10 engine, decomposition-invariant,
and statistically U(-1, 1) (the reference draws rand(Uniform(-1,1)), Simulation_CPU.jl:103)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from grayscott_amd.ops import native
from grayscott_amd.ops import reference as ref

from .mp_utils import ROOT


@pytest.fixture(scope="module")
def rocrand_tool(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc) or not os.path.exists("/opt/rocm/include/rocrand"):
        pytest.skip("hipcc / rocRAND headers not available")
    exe = str(tmp_path_factory.mktemp("rr") / "rocrand_parity")
    subprocess.run([hipcc, "-O1", "-std=c++17", "-I/opt/rocm/include",
                    os.path.join(ROOT, "csrc", "tools", "rocrand_parity.cpp"), "-o", exe],
                   check=True, capture_output=True)
    return exe


def test_matches_rocrand_engine(rocrand_tool):
    rng = np.random.default_rng(3)
    triples = [(int(rng.integers(0, 2**63)), int(rng.integers(0, 2**40)), int(rng.integers(0, 2**44)))
               for _ in range(200)] + [(0, 0, 0), (2**64 - 1, 2**33 + 5, 2**34 + 3)]
    inp = "\n".join(f"{s} {u} {o}" for s, u, o in triples) + "\n"
    out = subprocess.run([rocrand_tool], input=inp, capture_output=True, text=True, check=True)
    expect = [int(x) for x in out.stdout.split()]
    got_np, got_native = [], []
    for (seed, sub, off) in triples:
        q = off // 4
        w = ref.philox4x32_10(np.array([q & 0xFFFFFFFF]), np.array([q >> 32]),
                              np.array([sub & 0xFFFFFFFF]), np.array([sub >> 32]), seed)
        got_np.append(int(w[off % 4][0]))
    assert got_np == expect
    # the native helper evaluates block q of column layout: gx + Lx*(gy4 + Ly4*gz) with Lx=1
    for (seed, sub, off) in triples[:50]:
        q = off // 4
        blk = native.noise_block(q, 0, 0, 1, 4, sub, seed)
        got_native.append(blk[off % 4])
    assert got_native == expect[:50]


def test_cell_mapping_and_statistics():
    L, step, seed = (20, 12, 9), 5, 77
    full = ref.noise(L, (0, 0, 0), L, step, seed)
    part = ref.noise(L, (3, 4, 2), (10, 5, 6), step, seed)
    np.testing.assert_array_equal(part, full[2:8, 4:9, 3:13])  # decomposition invariant
    assert full.min() >= -1.0 and full.max() < 1.0
    big = ref.noise((64, 64, 64), (0, 0, 0), (64, 64, 64), 1, 1)
    assert abs(big.mean()) < 0.01
    assert abs(big.var() - 1.0 / 3.0) < 0.01
    other = ref.noise((64, 64, 64), (0, 0, 0), (64, 64, 64), 2, 1)
    assert abs(np.corrcoef(big.ravel(), other.ravel())[0, 1]) < 0.01


def test_native_block_equals_reference_layout():
    Lx, Ly = 10, 7
    for (gx, gy, gz, step) in [(0, 0, 0, 0), (9, 6, 3, 11), (4, 3, 100, 2**33)]:
        blk = native.noise_block(gx, gy >> 2, gz, Lx, Ly, step, 1234)
        w = ref.noise((Lx, Ly, 200), (gx, gy, gz), (1, 1, 1), step, 1234, dtype=np.float64)
        assert np.int32(np.uint32(blk[gy & 3])) * 2.0 ** -31 == w[0, 0, 0]


@pytest.mark.parametrize("impl", [0, 1])
def test_cpu_row_blocks_equal_reference_philox(impl):
    """The CPU step's row routine (backend_cpu.cpp noise_blocks: scalar, and the AVX2 form that
    runs eight counters per vector) equals the independent Python Philox4x32-10 for counters
    below and above 2^32, steps above 2^32 and row lengths that leave a scalar tail."""
    rng = np.random.default_rng(11)
    q = np.concatenate([rng.integers(0, 2**32, 21, dtype=np.uint64),
                        rng.integers(2**32, 2**40, 16, dtype=np.uint64)])
    for step, seed in ((3, 0x5EED6A5C), (2**33 + 5, 2**63 + 12345)):
        got = native.noise_blocks(q, step, seed, impl)
        if got is None:
            pytest.skip("no AVX2 on this CPU")
        for i, qi in enumerate(q.tolist()):
            want = ref.philox4x32_10(qi & 0xFFFFFFFF, qi >> 32, step & 0xFFFFFFFF, step >> 32, seed)
            assert tuple(int(w) for w in got[i]) == tuple(int(w) for w in want), (i, impl)


def test_cpu_step_flushes_denormals_but_restores_the_callers_fp_mode():
    """The CPU solver flushes denormals inside its parallel step region (backend_cpu.cpp: MXCSR
    FTZ + DAZ, a ~100x slowdown avoided on the reference example) and restores the calling
    thread's mode afterwards: numpy on the main thread keeps IEEE denormals."""
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    s = Settings(L=12, precision="Float32", noise=0.0, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 backend="CPU")
    sim = GrayScott(s, init_domain(12, 1, 0))
    sim.init_fields()
    u = np.full(sim.local_shape, 0.5, np.float32)
    v = np.full(sim.local_shape, 1e-39, np.float32)  # denormal v everywhere
    sim.set_fields(u, v)
    sim.iterate(1)
    _, v1 = sim.get_fields()
    sim.close()
    tiny = np.finfo(np.float32).tiny
    assert not ((v1 != 0) & (np.abs(v1) < tiny)).any()  # no denormal survives the step
    d = np.float32(1e-39)
    assert d != 0 and d * np.float32(1.0) == d  # the main thread still computes denormals


def test_cpu_ftz_knob_keeps_ieee_denormals(debug_knob):
    """Debug knob cpu_ftz = 0: the CPU solver keeps IEEE denormals (the reference's and the
    GPU's fp32 behaviour) for exact-parity runs; fp64 never flushes."""
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    tiny = {"Float32": np.finfo(np.float32).tiny, "Float64": np.finfo(np.float64).tiny}
    for prec, knob in (("Float32", 0), ("Float64", 1)):
        debug_knob("cpu_ftz", knob, "core")
        dt = np.float32 if prec == "Float32" else np.float64
        s = Settings(L=12, precision=prec, noise=0.0, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                     backend="CPU")
        sim = GrayScott(s, init_domain(12, 1, 0))
        sim.init_fields()
        sim.set_fields(np.full(sim.local_shape, 0.5, dt),
                       np.full(sim.local_shape, 4 * tiny[prec] / 2 ** 10, dt))  # denormal v
        sim.iterate(1)
        _, v1 = sim.get_fields()
        sim.close()
        assert ((v1 != 0) & (np.abs(v1) < tiny[prec])).any(), prec  # denormals survive
