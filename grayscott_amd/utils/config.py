"""Settings schema and TOML config loader.

Parity with the reference:
  * ``Settings`` fields/defaults       -- src/simulation/Structs.jl:4-28
  * accepted-key whitelist             -- src/simulation/Structs.jl:31-52
  * ``get_settings`` / ``parse_args``  -- src/simulation/Inputs.jl:20-68
  * ``parse_settings_toml``            -- src/simulation/Inputs.jl:80-97 (unknown keys ignored,
                                          values converted to the field's type)
  * ``load_backend_and_lang``          -- src/simulation/Inputs.jl:110-120 (case-insensitive)

Deliberate fixes: ``precision`` is whitelisted instead of ``eval``-ed (D7).

Extension keys (not in the reference, all optional, documented in README):
  ``periodic`` (bool), ``seed`` (int, noise stream key), ``fuse_steps`` (int, steps fused per
  halo exchange / temporal blocking depth, 0 = auto), ``transport`` ("auto"|"rccl"|"ipc"|"torch"|"host";
  "ipc": direct peer writes over xGMI, opt-in),
  ``output_engine`` ("bp4"), ``perf_log`` (path of a JSON-lines perf log), ``diagnostics`` (bool),
  ``decomposition`` ("auto"|"balanced"|"z": process grid, see parallel/decomp.choose_dims;
  "tune": self-check and time the candidate grids / fuse depths, parallel/autotune.py),
  ``overlap`` ("auto"|"on"|"off": overlap the halo exchange with the inner-plane update),
  ``async_output`` (bool, default true: output steps are written behind the simulation),
  ``output_queue`` (int 1-4, default 2: output steps in flight behind the simulation --
  snapshot buffers per rank; 1 when one step's snapshot exceeds 1 GiB),
  ``async_checkpoint`` (bool, default true: checkpoint data is written behind the simulation and
  committed -- metadata, atomic rename -- at the next output/checkpoint event or at the end).
"""
from __future__ import annotations

import argparse
import dataclasses
import math
import os
import sys
import warnings
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence

try:  # Python >= 3.11
    import tomllib as _toml  # type: ignore
except ModuleNotFoundError:  # pragma: no cover - 3.10 image
    import tomli as _toml  # type: ignore


class ArgumentError(ValueError):
    """Mirror of Julia's ``ArgumentError`` (Inputs.jl:25-28)."""


# Julia field types of Structs.jl:4-28, mapped to converters below.
_INT64, _INT32, _FLOAT64, _STRING, _BOOL = "Int64", "Int32", "Float64", "String", "Bool"


@dataclass
class Settings:
    """All configuration keys with the reference's defaults (Structs.jl:4-28)."""

    L: int = 128
    steps: int = 20000
    plotgap: int = 200
    F: float = 0.04
    k: float = 0.0
    dt: float = 0.2
    Du: float = 0.05
    Dv: float = 0.1
    noise: float = 0.0
    output: str = "foo.bp"
    checkpoint: bool = False
    checkpoint_freq: int = 2000
    checkpoint_output: str = "ckpt.bp"
    restart: bool = False
    restart_input: str = "ckpt.bp"
    mesh_type: str = "image"
    precision: str = "Float64"
    backend: str = "CPU"
    kernel_language: str = "Plain"
    verbose: bool = False
    # ---- extensions (not in the reference) -------------------------------------------
    periodic: bool = False
    seed: int = 0x5EED_6A5C
    fuse_steps: int = 0
    transport: str = "auto"
    output_engine: str = "bp4"
    perf_log: str = ""
    diagnostics: bool = False
    decomposition: str = "auto"
    overlap: str = "auto"
    async_output: bool = True
    output_queue: int = 2
    async_checkpoint: bool = True

    # -------------------------------------------------------------------------------------
    @property
    def dtype_name(self) -> str:
        return parse_precision(self.precision)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


# Whitelist (Structs.jl:31-52) and the Julia type of each key.
SETTINGS_KEYS: Dict[str, str] = {
    "L": _INT64,
    "steps": _INT32,
    "plotgap": _INT32,
    "F": _FLOAT64,
    "k": _FLOAT64,
    "dt": _FLOAT64,
    "Du": _FLOAT64,
    "Dv": _FLOAT64,
    "noise": _FLOAT64,
    "output": _STRING,
    "checkpoint": _BOOL,
    "checkpoint_freq": _INT32,
    "checkpoint_output": _STRING,
    "restart": _BOOL,
    "restart_input": _STRING,
    "mesh_type": _STRING,
    "precision": _STRING,
    "backend": _STRING,
    "kernel_language": _STRING,
    "verbose": _BOOL,
}

EXTENSION_KEYS: Dict[str, str] = {
    "periodic": _BOOL,
    "seed": _INT64,
    "fuse_steps": _INT32,
    "transport": _STRING,
    "output_engine": _STRING,
    "perf_log": _STRING,
    "diagnostics": _BOOL,
    "decomposition": _STRING,
    "overlap": _STRING,
    "async_output": _BOOL,
    "output_queue": _INT32,
    "async_checkpoint": _BOOL,
}

# Keys present in reference configs but commented out of the struct (Structs.jl:20-22):
# accepted and ignored, like the reference does silently.
IGNORED_KEYS = ("adios_config", "adios_span", "adios_memory_selection")

_INT_RANGES = {_INT32: (-(2**31), 2**31 - 1), _INT64: (-(2**63), 2**63 - 1)}


def _convert(key: str, jtype: str, value: Any) -> Any:
    """Julia ``convert(T, value)`` semantics: exact conversions only (InexactError otherwise)."""
    if jtype in (_INT32, _INT64):
        if isinstance(value, bool):
            ivalue = int(value)
        elif isinstance(value, int):
            ivalue = value
        elif isinstance(value, float):
            if not math.isfinite(value) or value != int(value):
                raise ArgumentError(f"InexactError: cannot convert {key}={value!r} to {jtype}")
            ivalue = int(value)
        else:
            raise ArgumentError(f"cannot convert {key}={value!r} to {jtype}")
        lo, hi = _INT_RANGES[jtype]
        if not lo <= ivalue <= hi:
            raise ArgumentError(f"InexactError: {key}={value!r} out of range for {jtype}")
        return ivalue
    if jtype == _FLOAT64:
        if isinstance(value, (int, float)) and not isinstance(value, bool):
            return float(value)
        if isinstance(value, bool):
            return float(value)
        raise ArgumentError(f"cannot convert {key}={value!r} to Float64")
    if jtype == _BOOL:
        if isinstance(value, bool):
            return value
        if isinstance(value, (int, float)) and value in (0, 1):
            return bool(value)
        raise ArgumentError(f"InexactError: cannot convert {key}={value!r} to Bool")
    if jtype == _STRING:
        if isinstance(value, str):
            return value
        raise ArgumentError(f"cannot convert {key}={value!r} to String")
    raise AssertionError(jtype)


def parse_settings_toml(contents: str) -> Settings:
    """Parse TOML text into ``Settings`` (Inputs.jl:80-97).

    Unknown keys are ignored; known values are converted to the field type.
    """
    table = _toml.loads(contents)
    settings = Settings()
    for key, value in table.items():
        jtype = SETTINGS_KEYS.get(key) or EXTENSION_KEYS.get(key)
        if jtype is None:
            continue  # silently ignored, like the reference
        setattr(settings, key, _convert(key, jtype, value))
    return settings


def parse_args(args: Sequence[str]) -> str:
    """Positional ``config_file`` argument (Inputs.jl:47-68)."""
    parser = argparse.ArgumentParser(
        prog="gray-scott",
        description="gray-scott workflow simulation example configuration file, "
        "MI355X-native version (grayscott_amd)",
    )
    parser.add_argument("config_file", help="configuration file")
    ns = parser.parse_args(list(args))
    return ns.config_file


def get_settings(args: Sequence[str]) -> Settings:
    """Read the TOML config named in ``args`` (Inputs.jl:20-35)."""
    config_file = parse_args(args)
    return load_settings(config_file)


def load_settings(config_file: str) -> Settings:
    if not str(config_file).endswith(".toml"):
        ext = str(config_file).split(".")[-1]
        raise ArgumentError(
            f"Config file must be in TOML format. Extension not recognized: {ext}\n")
    with open(config_file, "r", encoding="utf-8") as fh:
        return parse_settings_toml(fh.read())


# ------------------------------------------------------------------------------------------
_PRECISIONS = {
    "float32": "float32", "fp32": "float32", "single": "float32",
    "float64": "float64", "fp64": "float64", "double": "float64",
}


def parse_precision(precision: str) -> str:
    """Whitelisted replacement for ``eval(Meta.parse(precision))`` (communication.jl:27, D7)."""
    key = str(precision).strip().lower()
    if key not in _PRECISIONS:
        raise ArgumentError(
            f"precision must be Float32 or Float64, got {precision!r}")
    return _PRECISIONS[key]


_BACKENDS = {
    "cpu": "cpu",
    "amdgpu": "hip", "hip": "hip", "rocm": "hip", "gpu": "hip", "mi355x": "hip",
    "cuda": "hip",  # accepted for config compatibility; runs on the HIP backend
}

_LANGS = ("plain", "kernelabstractions")


def load_backend_and_lang(settings: Settings):
    """Lowercased (backend, kernel_language) pair (Inputs.jl:110-120).

    Returns the canonical backend ("cpu" | "hip") and the lowercased language, which is
    accepted for compatibility and otherwise ignored (there is one kernel per backend).
    """
    b = str(settings.backend).strip().lower()
    lang = str(settings.kernel_language).strip().lower()
    if b not in _BACKENDS:
        raise ArgumentError(f"unknown backend {settings.backend!r}")
    if b == "cuda":
        warnings.warn("backend = \"CUDA\" runs on the MI355X HIP backend", stacklevel=2)
    if lang not in _LANGS:
        raise ArgumentError(f"unknown kernel_language {settings.kernel_language!r}")
    return _BACKENDS[b], lang


def settings_from_dict(d: Dict[str, Any]) -> Settings:
    s = Settings()
    for key, value in d.items():
        jtype = SETTINGS_KEYS.get(key) or EXTENSION_KEYS.get(key)
        if jtype is None:
            continue
        setattr(s, key, _convert(key, jtype, value))
    return s


def write_settings_toml(settings: Settings, path: str) -> None:
    """Write settings back as TOML (used by scripts/tests)."""
    lines: List[str] = []
    for key in list(SETTINGS_KEYS) + list(EXTENSION_KEYS):
        v = getattr(settings, key)
        if isinstance(v, bool):
            lines.append(f"{key} = {'true' if v else 'false'}")
        elif isinstance(v, (int, float)):
            lines.append(f"{key} = {v!r}")
        else:
            lines.append(f'{key} = "{v}"')
    with open(path, "w", encoding="utf-8") as fh:
        fh.write("\n".join(lines) + "\n")
