"""Implicit-GEMM MFMA convolution dispatch (``conv.hip``).

Placeholder selection table: returns None (vendor path) until the HIP kernel
for a shape class is built and measured faster.
"""
from __future__ import annotations


def try_forward(x, w, stride, padding):
    return None


def try_backward_data(g, w, x_shape, stride, padding):
    return None


def try_backward_filter(g, x, w_shape, stride, padding):
    return None
