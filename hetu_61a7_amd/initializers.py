"""Parameter initializers (reference ``python/hetu/initializers.py:9-373``).

Each initializer fills a tensor on the parameter's device.  The random stream
is seeded with ``config.seed + node.id`` like the reference, using
a counter-based generator on the device (Philox on ROCm) so initialisation is
reproducible per parameter and independent of execution order.  PS-managed
parameters are initialised on the server through ``init_on_ps`` with the
reference's param-type codes (Dense=0, Sparse=1, CacheSparse=2).
"""
from __future__ import annotations

import math

import numpy as np
import torch


class BaseInit(object):
    def __init__(self, shape):
        self.shape = tuple(shape)

    def __call__(self, node, seed, np_rand=None, stream=None, device='cpu'):
        return self.generate(seed + node.id, device)

    def generate(self, seed, device='cpu') -> torch.Tensor:
        # Values are drawn on the host (same numbers on every device type and every
        # data-parallel rank) unless the tensor is huge (embedding tables), where
        # the device's own counter-based generator fills HBM directly.
        numel = 1
        for s in self.shape:
            numel *= int(s)
        gen_dev = torch.device('cpu') if numel < (1 << 26) else torch.device(device)
        t = torch.empty(self.shape, dtype=torch.float32, device=gen_dev)
        from .kernels import cpu_native
        spec = self.native_spec()
        if gen_dev.type == 'cpu' and spec is not None and cpu_native.enabled():
            # the native CPU backend's counter-based Philox (csrc/cpu/cpu_tensor_ops.cc)
            kind, a, b = spec
            if kind == 'constant':
                cpu_native.fill(t, a)
            else:
                cpu_native.random_init(t, kind, a, b, int(seed))
            return t.to(device)
        g = torch.Generator(device=gen_dev)
        g.manual_seed(int(seed) & 0x7FFFFFFF)
        self.init_on_device(t, g)
        return t.to(device)

    def init_on_device(self, t, gen):
        raise NotImplementedError

    def native_spec(self):
        """(kind, a, b) of the native CPU generator ('constant', 'uniform', 'normal',
        'truncated_normal'), or None for the torch generator"""
        return None

    def init_numpy(self, seed):
        return self.generate(seed, 'cpu').numpy()

    # PS path: (param_type, opt args) consumed by ps.Worker.init_tensor
    def init_on_ps(self, agent, node_id, param_type, seed, opt=None):
        agent.init_tensor(node_id, param_type, self.shape, self, seed, opt)


class ConstantInit(BaseInit):
    def __init__(self, constant, shape):
        super().__init__(shape)
        self.constant = constant

    def init_on_device(self, t, gen):
        t.fill_(self.constant)

    def native_spec(self):
        return ('constant', float(self.constant), 0.0)


class ZerosInit(ConstantInit):
    def __init__(self, shape):
        super().__init__(0.0, shape)


class OnesInit(ConstantInit):
    def __init__(self, shape):
        super().__init__(1.0, shape)


class UniformInit(BaseInit):
    def __init__(self, low, high, shape):
        super().__init__(shape)
        self.low, self.high = low, high

    def init_on_device(self, t, gen):
        t.uniform_(self.low, self.high, generator=gen)

    def native_spec(self):
        return ('uniform', float(self.low), float(self.high))


def _fans(shape, mode):
    hw = 1.0
    for s in shape[2:]:
        hw *= s
    if len(shape) >= 2:
        fan_in, fan_out = shape[1] * hw, shape[0] * hw
        if len(shape) == 2:
            # (in, out) matrices in Hetu's matmul convention
            fan_in, fan_out = shape[0], shape[1]
    else:
        fan_in = fan_out = shape[0] if shape else 1
    return {'fan_in': fan_in, 'fan_out': fan_out, 'avg': (fan_in + fan_out) / 2.0}[mode]


class GeneralXavierUniformInit(UniformInit):
    def __init__(self, gain, mode, shape):
        assert mode in ('fan_in', 'fan_out', 'avg')
        limit = math.sqrt(gain / _fans(shape, mode)) * math.sqrt(3.0)
        super().__init__(-limit, limit, shape)


class XavierUniformInit(GeneralXavierUniformInit):
    def __init__(self, shape):
        super().__init__(1.0, 'avg', shape)


class HeUniformInit(GeneralXavierUniformInit):
    def __init__(self, shape):
        super().__init__(2.0, 'fan_in', shape)


class LecunUniformInit(GeneralXavierUniformInit):
    def __init__(self, shape):
        super().__init__(1.0, 'fan_in', shape)


class NormalInit(BaseInit):
    def __init__(self, mean, stddev, shape):
        super().__init__(shape)
        self.mean, self.stddev = mean, stddev

    def init_on_device(self, t, gen):
        t.normal_(self.mean, self.stddev, generator=gen)

    def native_spec(self):
        return ('normal', float(self.mean), float(self.stddev))


class GeneralXavierNormalInit(NormalInit):
    def __init__(self, gain, mode, shape):
        assert mode in ('fan_in', 'fan_out', 'avg')
        super().__init__(0.0, math.sqrt(gain / _fans(shape, mode)), shape)


class XavierNormalInit(GeneralXavierNormalInit):
    def __init__(self, shape):
        super().__init__(1.0, 'avg', shape)


class HeNormalInit(GeneralXavierNormalInit):
    def __init__(self, shape):
        super().__init__(2.0, 'fan_in', shape)


class LecunNormalInit(GeneralXavierNormalInit):
    def __init__(self, shape):
        super().__init__(1.0, 'fan_in', shape)


class TruncatedNormalInit(BaseInit):
    """Normal truncated at 2 stddev (resampling semantics)."""

    def __init__(self, mean, stddev, shape):
        super().__init__(shape)
        self.mean, self.stddev = mean, stddev

    def init_on_device(self, t, gen):
        t.normal_(0.0, 1.0, generator=gen)
        for _ in range(8):
            bad = t.abs() > 2.0
            if not bool(bad.any()):
                break
            t[bad] = torch.randn(int(bad.sum()), generator=gen, device=t.device)
        t.clamp_(-2.0, 2.0).mul_(self.stddev).add_(self.mean)

    def native_spec(self):
        return ('truncated_normal', float(self.mean), float(self.stddev))


# ---- factories returning Variables (reference initializers.py:214-311) -----

def _var(init, name, trainable, ctx):
    from .ops.variable import Variable
    return Variable(name=name, initializer=init, trainable=trainable, ctx=ctx)


def zeros(shape, name=None, trainable=True, ctx=None):
    return _var(ZerosInit(shape), name, trainable, ctx)


def ones(shape, name=None, trainable=True, ctx=None):
    return _var(OnesInit(shape), name, trainable, ctx)


def constant(shape, fill_value=0.0, name=None, trainable=True, ctx=None):
    return _var(ConstantInit(fill_value, shape), name, trainable, ctx)


def truncated_normal(shape, mean=0.0, stddev=1.0, name=None, trainable=True, ctx=None):
    return _var(TruncatedNormalInit(mean, stddev, shape), name, trainable, ctx)


def random_normal(shape, mean=0.0, stddev=1.0, name=None, trainable=True, ctx=None):
    return _var(NormalInit(mean, stddev, shape), name, trainable, ctx)


def random_uniform(shape, minval=-1.0, maxval=1.0, name=None, trainable=True, ctx=None):
    return _var(UniformInit(minval, maxval, shape), name, trainable, ctx)


def general_xavier_normal(shape, gain, mode, name=None, trainable=True, ctx=None):
    return _var(GeneralXavierNormalInit(gain, mode, shape), name, trainable, ctx)


def general_xavier_uniform(shape, gain, mode, name=None, trainable=True, ctx=None):
    return _var(GeneralXavierUniformInit(gain, mode, shape), name, trainable, ctx)


def xavier_normal(shape, name=None, trainable=True, ctx=None):
    return _var(XavierNormalInit(shape), name, trainable, ctx)


def xavier_uniform(shape, name=None, trainable=True, ctx=None):
    return _var(XavierUniformInit(shape), name, trainable, ctx)


def he_normal(shape, name=None, trainable=True, ctx=None):
    return _var(HeNormalInit(shape), name, trainable, ctx)


def he_uniform(shape, name=None, trainable=True, ctx=None):
    return _var(HeUniformInit(shape), name, trainable, ctx)


def lecun_normal(shape, name=None, trainable=True, ctx=None):
    return _var(LecunNormalInit(shape), name, trainable, ctx)


def lecun_uniform(shape, name=None, trainable=True, ctx=None):
    return _var(LecunUniformInit(shape), name, trainable, ctx)


# ---- generator factories (used by layers) -----------------------------------

def _generate(init_cls, **kw):
    def gen(shape, name=None, trainable=True, ctx=None):
        return _var(init_cls(shape=shape, **kw), name, trainable, ctx)
    return gen


def GenZeros():
    return _generate(ZerosInit)


def GenOnes():
    return _generate(OnesInit)


def GenConstant(fill_value=0.0):
    return _generate(ConstantInit, constant=fill_value)


def GenTruncatedNormal(mean=0.0, stddev=1.0):
    return _generate(TruncatedNormalInit, mean=mean, stddev=stddev)


def GenNormal(mean=0.0, stddev=1.0):
    return _generate(NormalInit, mean=mean, stddev=stddev)


def GenUniform(minval=-1.0, maxval=1.0):
    return _generate(UniformInit, low=minval, high=maxval)


def GenGeneralXavierNormal(gain, mode):
    return _generate(GeneralXavierNormalInit, gain=gain, mode=mode)


def GenGeneralXavierUniform(gain, mode):
    return _generate(GeneralXavierUniformInit, gain=gain, mode=mode)


def GenXavierNormal():
    return _generate(XavierNormalInit)


def GenXavierUniform():
    return _generate(XavierUniformInit)


def GenHeNormal():
    return _generate(HeNormalInit)


def GenHeUniform():
    return _generate(HeUniformInit)


def GenLecunNormal():
    return _generate(LecunNormalInit)


def GenLecunUniform():
    return _generate(LecunUniformInit)
