"""The device-resident PyTorch oracle (ops/reference.py run_torch) agrees with the numpy
oracle: the int64-tensor Philox stream bit for bit, the random init bit for bit, and the
trajectory within fp32 rounding.  The GPU tests (test_gpu_oracle.py) run it on the MI355X
against the production kernels."""
import numpy as np
import pytest
import torch

from grayscott_amd.ops import reference as ref


def test_torch_philox_matches_numpy():
    rng = np.random.default_rng(1)
    c = [rng.integers(0, 2 ** 32, 500, dtype=np.uint64) for _ in range(4)]
    for seed in (0, 2024, 0xDEADBEEF12345678):
        a = ref.philox4x32_10(*c, seed)
        b = ref.philox4x32_10_torch(*(torch.as_tensor(x.astype(np.int64)) for x in c), seed)
        for x, y in zip(a, b):
            assert np.array_equal(x.astype(np.int64), y.numpy())


@pytest.mark.parametrize("L", [(12, 10, 9), (16, 16, 16), (7, 13, 5)])
def test_torch_noise_and_init_match_numpy(L):
    r0 = ref.noise(L, (0, 0, 0), L, 5, 77, dtype=np.float32)
    r1 = ref.noise_torch(L, 5, 77, dtype=torch.float32).numpy()
    assert np.array_equal(r0, r1)
    u0, v0 = ref.random_fields(L, seed=9, lo=-0.2, hi=0.9, dtype=np.float32)
    u1, v1 = ref.random_fields_torch(L, 9, -0.2, 0.9, torch.float32)
    assert np.array_equal(u0, u1.numpy()) and np.array_equal(v0, v1.numpy())


def test_torch_run_matches_numpy_run():
    L = (14, 12, 10)
    a = ref.run(L, 7, noise_amp=0.1, seed=3, dtype=np.float64, init_seed=4)
    b = ref.run_torch(L, 7, noise_amp=0.1, seed=3, dtype=torch.float64, init_seed=4)
    assert np.abs(a[0] - b[0].numpy()).max() < 1e-13
    assert np.abs(a[1] - b[1].numpy()).max() < 1e-13
    c = ref.run_torch(L, 7, noise_amp=0.1, seed=3, dtype=torch.float32, init_seed=4)
    assert np.abs(a[0] - c[0].numpy()).max() < 2e-6
    # from the reference's seed cube as well
    d = ref.run(L, 5, noise_amp=0.0, dtype=np.float64)
    e = ref.run_torch(L, 5, noise_amp=0.0, dtype=torch.float64)
    assert np.abs(d[0] - e[0].numpy()).max() < 1e-13


def test_julia_semantics_oracle_sits_between_fp32_and_fp64():
    """The reference's mixed Float32 arithmetic (run_torch arith="julia") is closer to a
    Float64 run than the all-Float32 oracle is, and differs from it by rounding only."""
    a = ref.run_torch(24, 40, noise_amp=0.1, seed=9, arith="julia")
    b = ref.run_torch(24, 40, noise_amp=0.1, seed=9)
    c = ref.run(24, 40, noise_amp=0.1, seed=9, dtype=np.float64)
    dj = max(float(np.abs(x.numpy() - y).max()) for x, y in zip(a, c))
    df = max(float(np.abs(x.numpy() - y).max()) for x, y in zip(b, c))
    assert a[0].dtype == torch.float32
    assert dj < df < 1e-5
    assert 0 < max(float((x - y).abs().max()) for x, y in zip(a, b)) < 1e-5
