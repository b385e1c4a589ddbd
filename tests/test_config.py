"""Settings / TOML loader parity (reference test/unit/simulation/unit-Inputs.jl, Inputs.jl,
Structs.jl)."""
import os

import pytest

from grayscott_amd.utils.config import (EXTENSION_KEYS, SETTINGS_KEYS, ArgumentError, Settings,
                                        get_settings, load_backend_and_lang, parse_precision,
                                        parse_settings_toml, write_settings_toml)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(ROOT, "examples", "settings-files.toml")


def test_get_settings_example_file():
    s = get_settings([EXAMPLE])
    assert (s.L, s.steps, s.plotgap) == (64, 1000, 10)
    assert (s.F, s.k, s.dt, s.Du, s.Dv, s.noise) == (0.02, 0.048, 1.0, 0.2, 0.1, 0.1)
    assert s.output == "gs-1MPI-1GPU-64L-F32.bp"
    assert s.checkpoint is False and s.checkpoint_freq == 700
    assert s.precision == "Float32" and s.mesh_type == "image"


def test_non_toml_raises_argument_error():
    # unit-Inputs.jl:11
    with pytest.raises(ArgumentError):
        get_settings(["hello.nojson"])


def test_defaults_match_reference_struct():
    s = Settings()
    assert s.L == 128 and s.steps == 20000 and s.plotgap == 200
    assert s.F == 0.04 and s.k == 0.0 and s.dt == 0.2 and s.Du == 0.05 and s.Dv == 0.1
    assert s.noise == 0.0 and s.output == "foo.bp"
    assert s.checkpoint is False and s.checkpoint_freq == 2000
    assert s.checkpoint_output == "ckpt.bp" and s.restart is False and s.restart_input == "ckpt.bp"
    assert s.mesh_type == "image" and s.precision == "Float64"
    assert s.backend == "CPU" and s.kernel_language == "Plain" and s.verbose is False


def test_whitelist_is_the_reference_key_set():
    assert set(SETTINGS_KEYS) == {
        "L", "steps", "plotgap", "F", "k", "dt", "Du", "Dv", "noise", "output", "checkpoint",
        "checkpoint_freq", "checkpoint_output", "restart", "restart_input", "mesh_type",
        "precision", "backend", "kernel_language", "verbose"}
    assert not set(SETTINGS_KEYS) & set(EXTENSION_KEYS)


def test_unknown_keys_ignored_and_values_converted():
    s = parse_settings_toml('L = 64.0\ndt = 1\nfoo = "bar"\nadios_span = false\n'
                            'verbose = true\nsteps = 7\n')
    assert s.L == 64 and isinstance(s.L, int)
    assert s.dt == 1.0 and isinstance(s.dt, float)
    assert s.verbose is True and s.steps == 7
    assert not hasattr(s, "foo")


def test_inexact_conversion_raises():
    with pytest.raises(ArgumentError):
        parse_settings_toml("L = 64.5\n")
    with pytest.raises(ArgumentError):
        parse_settings_toml("steps = 3000000000\n")  # Int32 overflow
    with pytest.raises(ArgumentError):
        parse_settings_toml("verbose = 2\n")


def test_backend_and_language_case_insensitive():
    assert load_backend_and_lang(Settings(backend="cpu", kernel_language="PLAIN")) == ("cpu", "plain")
    assert load_backend_and_lang(Settings(backend="AMDGPU"))[0] == "hip"
    assert load_backend_and_lang(Settings(backend="Hip", kernel_language="KernelAbstractions")) == \
        ("hip", "kernelabstractions")
    with pytest.warns(UserWarning):
        assert load_backend_and_lang(Settings(backend="CUDA"))[0] == "hip"
    with pytest.raises(ArgumentError):
        load_backend_and_lang(Settings(backend="tpu"))


def test_precision_whitelist_no_eval():
    assert parse_precision("Float32") == "float32"
    assert parse_precision("Float64") == "float64"
    for bad in ("Int64", "__import__('os')", "Float16"):
        with pytest.raises(ArgumentError):
            parse_precision(bad)


def test_write_roundtrip(tmp_path):
    s = Settings(L=33, noise=0.25, backend="AMDGPU", periodic=True, fuse_steps=2)
    p = str(tmp_path / "s.toml")
    write_settings_toml(s, p)
    assert get_settings([p]) == s


def test_every_example_config_loads():
    """examples/*.toml (the reference example and the BASELINE configs' settings) load through the
    same loader as the CLI, with the reference's keys and the extensions they use."""
    import glob
    import os

    from grayscott_amd.utils.config import load_settings
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(root, "examples", "*.toml")))
    assert len(files) >= 4
    for f in files:
        s = load_settings(f)
        assert s.L > 0 and s.precision in ("Float32", "Float64"), f
        assert s.backend in ("CPU", "AMDGPU", "HIP", "CUDA"), f
