"""Synthetic data generation (csrc/include/mireduce/rng.hpp) — host side; the GPU tests check
device == host bit for bit."""
import pytest
import torch

from cuda_mpi_reductions_amd.ops import PATTERNS, fill_, synthetic

DTS = [torch.int32, torch.int64, torch.float32, torch.float64]


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("pattern", sorted(PATTERNS))
def test_offset_consistency(dt, pattern):
    # element i is f(seed, offset + i): a shard filled at offset k equals the slice of the whole.
    whole = synthetic(10_000, dt, pattern=pattern, seed=3, value=2.5)
    part = synthetic(3_000, dt, pattern=pattern, seed=3, offset=4_321, value=2.5)
    assert torch.equal(whole[4_321:7_321], part)


@pytest.mark.parametrize("dt", DTS)
def test_seed_changes_stream(dt):
    a = synthetic(1000, dt, seed=1)
    b = synthetic(1000, dt, seed=2)
    assert not torch.equal(a, b)


def test_value_ranges():
    u = synthetic(100_000, torch.float64)
    assert 0.0 <= float(u.min()) and float(u.max()) < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.01
    s = synthetic(100_000, torch.int32, pattern="smallint")
    assert int(s.min()) >= 0 and int(s.max()) <= 255
    f = synthetic(100_000, torch.float32, pattern="smallint")
    assert float(f.max()) <= 255 / 2147483647.0 + 1e-12    # (rand() & 0xFF) / RAND_MAX
    i = synthetic(4096, torch.int64, pattern="iotamod")
    assert i.tolist() == [k % 1024 for k in range(4096)]
    c = synthetic(10, torch.float64, pattern="constant", value=7.0)
    assert c.tolist() == [7.0] * 10
    fr = synthetic(100_000, torch.int32, pattern="fullrange")
    assert int(fr.min()) < -2**30 and int(fr.max()) > 2**30


def test_unknown_pattern_rejected():
    with pytest.raises(ValueError):
        fill_(torch.empty(4), "gaussian")
