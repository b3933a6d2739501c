"""Keras-like layers (reference ``python/hetu/layers/*.py``)."""
from __future__ import annotations

from ..ops.node import Op
from .. import ops as O
from .. import initializers as init


class BaseLayer(object):
    def __call__(self, *args, **kwargs):
        raise NotImplementedError


class Linear(BaseLayer):
    def __init__(self, in_features, out_features, initializer=None, bias=True, activation=None,
                 weight_transpose=False, name='linear'):
        initializer = initializer or init.GenXavierUniform()
        self.in_features, self.out_features = in_features, out_features
        self.bias = bias
        self.fused_act = None
        if isinstance(activation, str):
            assert activation in ('relu', 'gelu')
            self.fused_act = activation
            activation = None
        self.activation = activation
        self.weight_transpose = weight_transpose
        self.name = name
        if isinstance(initializer, Op):
            self.weight_var = initializer
        else:
            shape = (out_features, in_features) if weight_transpose else (in_features, out_features)
            self.weight_var = initializer(shape=shape, name=name + '_weight')
        if bias:
            self.bias_var = init.zeros(shape=(out_features,), name=name + '_bias')

    def __call__(self, x):
        if self.bias:
            x = O.linear_op(x, self.weight_var, self.bias_var, trans_B=self.weight_transpose,
                            activation=self.fused_act)
        else:
            x = O.matmul_op(x, self.weight_var, trans_B=self.weight_transpose)
            if self.fused_act == 'relu':
                x = O.relu_op(x)
            elif self.fused_act == 'gelu':
                x = O.gelu_op(x)
        if self.activation is not None:
            x = self.activation(x)
        return x


class Conv2d(BaseLayer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 initializer=None, bias=True, activation=None, name='conv2d'):
        initializer = initializer or init.GenXavierUniform()
        self.height, self.width = (kernel_size if isinstance(kernel_size, tuple) else (kernel_size, kernel_size))
        self.in_channels, self.out_channels = in_channels, out_channels
        self.stride, self.padding = stride, padding
        self.bias, self.activation, self.name = bias, activation, name
        self.weight_var = initializer(shape=(out_channels, in_channels, self.height, self.width),
                                      name=name + '_weight')
        if bias:
            self.bias_var = init.zeros(shape=(out_channels,), name=name + '_bias')

    def __call__(self, x):
        if self.bias:
            x = O.conv2d_add_bias_op(x, self.weight_var, self.bias_var, stride=self.stride, padding=self.padding)
        else:
            x = O.conv2d_op(x, self.weight_var, stride=self.stride, padding=self.padding)
        if self.activation is not None:
            x = self.activation(x)
        return x


class BatchNorm(BaseLayer):
    def __init__(self, num_channels, name='batchnorm', momentum=0.1, eps=1e-5):
        self.num_channels, self.name = num_channels, name
        self.momentum, self.eps = momentum, eps
        self.scale_var = init.ones(shape=(num_channels,), name=name + '_weight')
        self.bias_var = init.zeros(shape=(num_channels,), name=name + '_bias')

    def __call__(self, x):
        return O.batch_normalization_op(x, self.scale_var, self.bias_var, self.momentum, self.eps)


class LayerNorm(BaseLayer):
    def __init__(self, num_channels, name='layernorm', eps=1e-05):
        self.num_channels, self.name, self.eps = num_channels, name, eps
        self.scale_var = init.ones(shape=(num_channels,), name=name + '_weight')
        self.bias_var = init.zeros(shape=(num_channels,), name=name + '_bias')

    def __call__(self, x):
        return O.layer_normalization_op(x, self.scale_var, self.bias_var, eps=self.eps)


class MaxPool2d(BaseLayer):
    def __init__(self, kernel_size, stride, padding=0):
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding

    def __call__(self, x):
        return O.max_pool2d_op(x, self.kernel_size, self.kernel_size, self.padding, self.stride)


class AvgPool2d(BaseLayer):
    def __init__(self, kernel_size, stride, padding=0):
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding

    def __call__(self, x):
        return O.avg_pool2d_op(x, self.kernel_size, self.kernel_size, self.padding, self.stride)


class DropOut(BaseLayer):
    def __init__(self, p=0.5):
        self.p = p

    def __call__(self, x):
        return O.dropout_op(x, 1 - self.p)


class Embedding(BaseLayer):
    def __init__(self, num_embeddings, embedding_dim, initializer=None, name='embedding', ctx=None):
        initializer = initializer or init.GenXavierNormal()
        self.num_embeddings, self.embedding_dim, self.name = num_embeddings, embedding_dim, name
        self.embedding_table = initializer(shape=(num_embeddings, embedding_dim), name=name, ctx=ctx)

    def __call__(self, x):
        return O.embedding_lookup_op(self.embedding_table, x)


class Identity(BaseLayer):
    def __call__(self, x):
        return x


class Relu(BaseLayer):
    def __call__(self, x):
        return O.relu_op(x)


class Gelu(BaseLayer):
    def __call__(self, x):
        return O.gelu_op(x)


class Reshape(BaseLayer):
    def __init__(self, shape):
        self.shape = shape

    def __call__(self, x):
        return O.array_reshape_op(x, self.shape)


class Sequence(BaseLayer):
    def __init__(self, *args):
        self.layers = args

    def __call__(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class Slice(BaseLayer):
    def __init__(self, begin, size):
        self.begin, self.size = begin, size

    def __call__(self, x):
        return O.slice_op(x, self.begin, self.size)


class SumLayers(BaseLayer):
    def __init__(self, layers):
        self.layers = layers

    def __call__(self, xs):
        return O.sum_op([layer(x) for layer, x in zip(self.layers, xs)])


class Concatenate(BaseLayer):
    def __init__(self, axis):
        self.axis = axis

    def __call__(self, *args):
        if len(args) == 1 and isinstance(args[0], (list, tuple)):
            args = args[0]
        return O.concatenate_op(list(args), axis=self.axis)


class ConcatenateLayers(BaseLayer):
    def __init__(self, layers, axis=0):
        self.layers, self.axis = layers, axis

    def __call__(self, x):
        return O.concatenate_op([layer(x) for layer in self.layers], axis=self.axis)
