"""Replay-safe host seeds (kernels/rng.py) and the CPU channel dropout (ops.nn._dropout2d):
host seeds repeat per step on the GPU path (the device counter varies them), vary per step
on the CPU path, restart with the executor seed, and are distinct per op and per call."""
import numpy as np
import torch

from hetu_61a7_amd.kernels import rng


def test_gpu_host_seeds_repeat_per_step_cpu_seeds_vary():
    rng.set_base_seed(7)
    rng._ADVANCED[0] = None
    seen = []
    for _ in range(3):
        rng.new_step()
        rng._ADVANCED[rng._base.cur_device()] = rng.epoch()     # no device here: skip the advance
        seen.append((rng.next_seed(11), rng.next_seed(11), rng.next_seed(12)))
    assert seen[0] == seen[1] == seen[2]
    a, b, c = seen[0]
    assert len({a, b, c}) == 3 and all(0 < v < (1 << 63) for v in (a, b, c))
    cpu = []
    for _ in range(3):
        rng.new_step()
        cpu.append(rng.next_seed(11, on_gpu=False))
    assert len(set(cpu)) == 3
    rng.set_base_seed(8)
    rng.new_step()
    rng._ADVANCED[rng._base.cur_device()] = rng.epoch()
    assert rng.next_seed(11) != a


def test_cpu_dropout2d_drops_whole_planes():
    from hetu_61a7_amd.ops.nn import _dropout2d
    x = torch.ones(8, 32, 5, 5)
    y = _dropout2d(x, 0.6, 12345)
    planes = y.reshape(8, 32, -1)
    assert torch.all((planes == 0).all(-1) | (planes == 1 / 0.6).all(-1))
    kept = (planes != 0).any(-1).float().mean().item()
    assert 0.45 < kept < 0.75
    y2 = _dropout2d(x, 0.6, 12345)
    assert torch.equal(y, y2)
    assert not torch.equal(y, _dropout2d(x, 0.6, 54321))
    np.testing.assert_allclose(y.mean().item(), 1.0, atol=0.2)
