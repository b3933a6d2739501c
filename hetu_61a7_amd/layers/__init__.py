"""Layers (reference ``python/hetu/layers/__init__.py:1-22``)."""
from .basic import (BaseLayer, Linear, Conv2d, BatchNorm, LayerNorm, MaxPool2d, AvgPool2d, DropOut,
                    Embedding, Identity, Relu, Gelu, Reshape, Sequence, Slice, SumLayers, Concatenate,
                    ConcatenateLayers)
from .moe import (TopKGate, KTop1Gate, HashGate, SAMGate, BalanceAssignmentGate, DenseToSparseGate,
                  DTSTemperature, Expert, MoELayer, KTop1Layer, HashLayer, SAMLayer, topkgating,
                  balance_loss)
