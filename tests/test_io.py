"""BP4 writer/reader and the SimulationOutput schema (reference src/simulation/IO.jl; the
reference's own unit-IO.jl is disabled/stale, D11).  There is no libadios2 in this environment:
the C++ writer is checked against the independent Python reader, golden header bytes and a
byte-level walk of the data subfiles."""
import os
import struct

import numpy as np
import pytest

from grayscott_amd.io.bp4 import BP4Error, BP4Reader, BP4Writer
from grayscott_amd.io.output import SimulationOutput, vtk_schema
from grayscott_amd.parallel.decomp import init_domain
from grayscott_amd.utils.config import Settings

from .mp_utils import ROOT


def _write(path, steps=3, shape=(4, 5, 6), dtype=np.float32):
    w = BP4Writer(path, "TestIO", 0, 1)
    w.define_attribute("F", 0.02)
    w.define_attribute("arr", [1.0, 2.0, 3.0])
    w.define_attribute("name", "uniform")
    w.define_attribute("list", ["U", "V"])
    w.define_variable("step", np.int32)
    w.define_variable("A", dtype, shape, (0, 0, 0), shape)
    data = []
    for s in range(steps):
        w.begin_step()
        w.put("step", np.int32(s * 10))
        a = (np.arange(np.prod(shape)).reshape(shape) + 100 * s).astype(dtype)
        data.append(a)
        w.put("A", a)
        w.write_metadata([w.end_step()])
    w.close()
    return data


def test_header_bytes(tmp_path):
    p = str(tmp_path / "h.bp")
    _write(p, 1)
    for fname, kind in (("data.0", b"D"), ("md.0", b"M"), ("md.idx", b"I")):
        with open(os.path.join(p, fname), "rb") as fh:
            h = fh.read(64)
        assert h[:16] == b"ADIOS-BP v2.10.2"
        assert h[31:32] == kind
        assert h[32:35] == b"212"
        assert h[36] == 0 and h[37] == 4 and h[39] == 2
    with open(os.path.join(p, "md.idx"), "rb") as fh:
        idx = fh.read()
    assert idx[38] == 0  # closed writer -> index table inactive
    assert (len(idx) - 64) % 64 == 0


def test_roundtrip_steps_attributes_selection(tmp_path):
    p = str(tmp_path / "r.bp")
    data = _write(p, 3)
    with BP4Reader(p) as r:
        assert r.steps == 3
        assert r.attributes["F"] == 0.02
        np.testing.assert_array_equal(r.attributes["arr"], [1.0, 2.0, 3.0])
        assert r.attributes["name"] == "uniform"
        assert r.attributes["list"] == ["U", "V"]
        for s in range(3):
            assert r.read("step", s) == 10 * s
            np.testing.assert_array_equal(r.read("A", s), data[s])
        np.testing.assert_array_equal(r.read("A", 1, (1, 2, 3), (2, 2, 2)), data[1][1:3, 2:4, 3:5])
        vi = r.variables(2)["A"]
        assert vi.blocks[0].vmin == data[2].min() and vi.blocks[0].vmax == data[2].max()
        assert r.process_groups(1)[0]["step"] == 2
        with pytest.raises(BP4Error):
            r.read("nope")


def test_fp64_and_multiple_blocks(tmp_path):
    p = str(tmp_path / "m.bp")
    shape = (6, 4, 4)
    full = np.random.default_rng(0).random(shape)
    w = BP4Writer(p, "Blocks", 0, 1)
    w.define_variable("X", np.float64, shape, (0, 0, 0), (3, 4, 4))
    w.begin_step()
    w.put("X", full[:3])
    w.set_selection("X", (3, 0, 0), (3, 4, 4))
    w.put("X", full[3:])
    w.write_metadata([w.end_step()])
    w.close()
    with BP4Reader(p) as r:
        assert len(r.variables(0)["X"].blocks) == 2
        np.testing.assert_array_equal(r.read("X"), full)
        np.testing.assert_array_equal(r.read("X", 0, (2, 1, 0), (2, 3, 4)), full[2:4, 1:4, :])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_block_minmax_vectorised(tmp_path, dtype):
    """The writer's block min / max characteristics (SSE2 folds, OpenMP chunks above 2M
    elements) equal numpy's for lengths that do not fill the vector lanes, with NaNs that must
    not win (the scalar rule `v < a ? v : a`) and a leading NaN that does."""
    rng = np.random.default_rng(3)
    cases = []
    for n in (1, 2, 7, 17, 33, 1000, 65537, (1 << 21) + 5):
        a = (rng.random(n) * 200 - 100).astype(dtype)
        if n > 2:
            a[n // 2] = np.nan
            a[-1] = -250.0  # the extreme in the scalar tail
        cases.append(a)
    lead = (rng.random(40) - 0.5).astype(dtype)
    lead[0] = np.nan
    cases.append(lead)
    p = str(tmp_path / "mm.bp")
    w = BP4Writer(p, "MinMax", 0, 1)
    for i, a in enumerate(cases):
        w.define_variable(f"X{i}", dtype, (a.size,), (0,), (a.size,))
    w.begin_step()
    for i, a in enumerate(cases):
        w.put(f"X{i}", a)
    w.write_metadata([w.end_step()])
    w.close()
    with BP4Reader(p) as r:
        vs = r.variables(0)
        for i, a in enumerate(cases[:-1]):
            b = vs[f"X{i}"].blocks[0]
            assert b.vmin == np.nanmin(a) and b.vmax == np.nanmax(a), (a.size, b.vmin, b.vmax)
        b = vs[f"X{len(cases) - 1}"].blocks[0]
        assert np.isnan(b.vmin) and np.isnan(b.vmax)


def _walk_data_file(path):
    """Parse every process group of a data subfile; returns [(step, nvars, [var names])]."""
    with open(path, "rb") as fh:
        buf = fh.read()
    pos, out = 64, []
    while pos < len(buf):
        pglen = struct.unpack_from("<Q", buf, pos)[0]
        end = pos + 8 + pglen
        p = pos + 8 + 1
        n = struct.unpack_from("<H", buf, p)[0]
        p += 2 + n + 4
        n = struct.unpack_from("<H", buf, p)[0]
        p += 2 + n
        step = struct.unpack_from("<I", buf, p)[0]
        p += 4
        nmeth = buf[p]
        mlen = struct.unpack_from("<H", buf, p + 1)[0]
        p += 3 + mlen
        assert mlen == 3 * nmeth
        nvars, vlen = struct.unpack_from("<IQ", buf, p)
        p += 12
        vend = p + vlen
        names = []
        for _ in range(nvars):
            vl = struct.unpack_from("<Q", buf, p)[0]
            q = p + 8 + 4
            n = struct.unpack_from("<H", buf, q)[0]
            names.append(buf[q + 2:q + 2 + n].decode())
            p += 8 + vl
        assert p == vend
        natt, alen = struct.unpack_from("<IQ", buf, p)
        p += 12
        for _ in range(natt):
            al = struct.unpack_from("<I", buf, p)[0]
            assert buf[p:p + al].find(b"[AMD") > 0 and buf[p + al - 4:p + al] == b"AMD]"
            p += al
        assert p == end, (p, end)
        out.append((step, nvars, names, natt))
        pos = end
    return out


def test_data_subfile_structure(tmp_path):
    p = str(tmp_path / "d.bp")
    _write(p, 2)
    pgs = _walk_data_file(os.path.join(p, "data.0"))
    assert [(s, n, names) for s, n, names, _ in pgs] == [(1, 2, ["step", "A"]), (2, 2, ["step", "A"])]
    assert pgs[0][3] == 4 and pgs[1][3] == 0  # attributes only with the first step


def test_simulation_output_schema(tmp_path):
    s = Settings(L=12, precision="Float32", output=str(tmp_path / "gs.bp"), noise=0.1)
    dom = init_domain(12, 1, 0)
    out = SimulationOutput(s, dom)
    u = np.random.default_rng(1).random((12, 12, 12)).astype(np.float32)
    out.write_fields(10, u, 1 - u)
    out.write_fields(20, u * 2, u)
    out.close()
    with BP4Reader(s.output) as r:
        a = r.attributes
        for key, val in (("F", 0.04), ("k", 0.0), ("dt", 0.2), ("Du", 0.05), ("Dv", 0.1),
                         ("noise", 0.1)):
            assert a[key] == pytest.approx(val)
        assert a["Fides_Data_Model"] == "uniform"
        np.testing.assert_array_equal(a["Fides_Origin"], [0, 0, 0])
        np.testing.assert_array_equal(a["Fides_Spacing"], [0.1, 0.1, 0.1])
        assert a["Fides_Dimension_Variable"] == "U"
        assert a["Fides_Variable_List"] == ["U", "V"]
        assert a["Fides_Variable_Associations"] == ["points", "points"]
        assert 'WholeExtent="0 12 0 12 0 12"' in a["vtk.xml"] and "TIME" in a["vtk.xml"]
        assert [r.read("step", i) for i in range(2)] == [10, 20]
        assert r.variables(0)["U"].dtype == np.float32
        assert r.variables(0)["U"].shape == (12, 12, 12)
        np.testing.assert_array_equal(r.read("V", 0), 1 - u)
        assert r.process_groups(0)[0]["io"] == "SimulationOutput"


def test_vtk_schema_extent():
    assert 'Extent="0 64 0 64 0 64"' in vtk_schema(64)


def _async_output_vs_sync(tmp_path, backend, L, queues):
    from grayscott_amd import driver

    out = {}
    for mode in [False] + list(queues):
        s = Settings(L=L, steps=12, plotgap=3, noise=0.1, F=0.02, k=0.048, dt=1.0, Du=0.2,
                     Dv=0.1, precision="Float32", backend=backend, async_output=bool(mode),
                     output_queue=int(mode) or 1, output=str(tmp_path / f"gs_{mode}.bp"))
        driver.run(s, out=open(os.devnull, "w"))
        with BP4Reader(s.output) as r:
            out[mode] = [(int(r.read("step", i)), r.read("U", i), r.read("V", i))
                         for i in range(r.steps)]
    for q in queues:
        assert len(out[q]) == len(out[False]) == 4
        for (sa, ua, va), (sb, ub, vb) in zip(out[False], out[q]):
            assert sa == sb
            np.testing.assert_array_equal(ua, ub)
            np.testing.assert_array_equal(va, vb)


def test_async_output_matches_sync(tmp_path):
    """async_output (snapshot + background data write, metadata committed when the step
    `output_queue` steps later is written) writes the same steps and bytes as the synchronous
    path, for one to three steps in flight."""
    _async_output_vs_sync(tmp_path, "CPU", 20, (1, 2, 3))


@pytest.mark.gpu
def test_async_output_queue_gpu(tmp_path):
    """The output queue on the HIP path: a ring of pinned host snapshot buffers behind one
    device staging pair; every queued step's bytes equal the synchronous writer's."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _async_output_vs_sync(tmp_path, "AMDGPU", 64, (1, 2, 3))


def test_output_queue_is_a_setting():
    from grayscott_amd.utils.config import EXTENSION_KEYS
    assert Settings().output_queue == 2 and "output_queue" in EXTENSION_KEYS


def _async_vs_sync(tmp_path, backend, L, steps, plotgap, freqs):
    """Run the driver with asynchronous output + checkpoints and fully synchronously; every
    output step and the final checkpoint must be bitwise equal."""
    from grayscott_amd import driver

    for freq in freqs:
        res, outs = {}, {}
        for mode in (False, True):
            s = Settings(L=L, steps=steps, plotgap=plotgap, noise=0.1, F=0.02, k=0.048, dt=1.0,
                         Du=0.2, Dv=0.1, precision="Float32", backend=backend,
                         async_checkpoint=mode, async_output=mode, checkpoint=True,
                         checkpoint_freq=freq,
                         checkpoint_output=str(tmp_path / f"ck_{freq}_{mode}.bp"),
                         output=str(tmp_path / f"gs_{freq}_{mode}.bp"))
            driver.run(s, out=open(os.devnull, "w"))
            assert not os.path.exists(s.checkpoint_output + ".tmp")
            with BP4Reader(s.checkpoint_output) as r:
                res[mode] = (int(r.read("step")), r.read("U", -1), r.read("V", -1))
            with BP4Reader(s.output) as r:
                outs[mode] = [(int(r.read("step", i)), r.read("U", i), r.read("V", i))
                              for i in range(r.steps)]
        assert res[True][0] == res[False][0] == (steps // freq) * freq
        np.testing.assert_array_equal(res[True][1], res[False][1])
        np.testing.assert_array_equal(res[True][2], res[False][2])
        assert [o[0] for o in outs[True]] == [o[0] for o in outs[False]] == \
            list(range(plotgap, steps + 1, plotgap))
        for a, b in zip(outs[True], outs[False]):
            np.testing.assert_array_equal(a[1], b[1])
            np.testing.assert_array_equal(a[2], b[2])


def test_async_checkpoint_matches_sync(tmp_path):
    """async_checkpoint / async_output (data written on host threads, committed at the next
    event / end) leave the same checkpoint and output as the synchronous writers, including
    when the checkpoint shares the output step's snapshot (plotgap 3, checkpoint_freq 6) and
    when it does not (freq 4)."""
    _async_vs_sync(tmp_path, "CPU", 20, 14, 3, (6, 4))


@pytest.mark.gpu
def test_async_checkpoint_matches_sync_gpu(tmp_path):
    """The same on the HIP path, where the snapshots live in reused pinned host buffers and
    device staging buffers ordered by events: checkpoints that do not share an output step's
    snapshot (freq 4 vs plotgap 3) must not disturb the output step still being written."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _async_vs_sync(tmp_path, "AMDGPU", 96, 40, 3, (4, 6))


def test_put_with_given_minmax(tmp_path):
    """BP4Writer.put(minmax=...) stores the caller's block min / max (the GPU snapshot's) as the
    block characteristics; the data round-trips unchanged."""
    import numpy as np

    from grayscott_amd.io.bp4 import BP4Reader, BP4Writer
    w = BP4Writer(str(tmp_path / "mm.bp"), "T")
    w.define_variable("U", np.float32, (2, 3, 4), (0, 0, 0), (2, 3, 4))
    a = np.arange(24, dtype=np.float32).reshape(2, 3, 4) - 5
    w.begin_step()
    w.put("U", a, minmax=(a.min(), a.max()))
    w.write_metadata([w.end_step()])
    w.close()
    r = BP4Reader(str(tmp_path / "mm.bp"))
    np.testing.assert_array_equal(r.read("U", 0), a)
    blk = r.variables(0)["U"].blocks[0]
    assert (blk.vmin, blk.vmax) == (-5.0, 18.0)
    r.close()


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_write_step_uv_matches_put_sequence(tmp_path, dtype):
    """BP4Writer.write_step_uv (one native call per output step: begin, step, U, V with the
    snapshot kernel's min / max partials reduced in C++, end) writes the same bytes as the
    begin / put / put / put / end sequence -- data subfile, md.0 and md.idx."""
    import numpy as np

    from grayscott_amd.io.bp4 import BP4Writer
    rng = np.random.default_rng(3)
    shape = (5, 6, 7)
    steps = [(rng.random(shape).astype(dtype), rng.random(shape).astype(dtype)) for _ in range(3)]
    outs = []
    for mode in ("puts", "one_call", "one_call_scan"):
        p = str(tmp_path / f"{mode}.bp")
        w = BP4Writer(p, "SimulationOutput", 0, 1)
        w.define_variable("step", np.int32)
        w.define_variable("U", np.dtype(dtype).type, shape, (0, 0, 0), shape)
        w.define_variable("V", np.dtype(dtype).type, shape, (0, 0, 0), shape)
        for i, (u, v) in enumerate(steps):
            if mode == "puts":
                w.begin_step()
                w.put("step", np.int32(10 * i))
                w.put("U", u)
                w.put("V", v)
                blob = w.end_step()
            else:
                part = None
                if mode == "one_call":  # two chunks' (u min, u max, v min, v max)
                    h = shape[0] // 2
                    part = np.array([[u[:h].min(), u[:h].max(), v[:h].min(), v[:h].max()],
                                     [u[h:].min(), u[h:].max(), v[h:].min(), v[h:].max()]],
                                    dtype=dtype)
                blob = w.write_step_uv(10 * i, u, v, part)
            w.write_metadata([blob])
        w.close()
        outs.append({f: open(os.path.join(p, f), "rb").read() for f in ("data.0", "md.0", "md.idx")})
        # md.idx records (64 B after a 64 B header) carry a wall-clock ms stamp at +48
        idx = bytearray(outs[-1]["md.idx"])
        for r in range(64, len(idx), 64):
            idx[r + 48:r + 56] = bytes(8)
        outs[-1]["md.idx"] = bytes(idx)
    for f in ("data.0", "md.0", "md.idx"):
        assert outs[1][f] == outs[0][f], f
        assert outs[2][f] == outs[0][f], f
