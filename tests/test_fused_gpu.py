"""Fused transformer kernels on the GPU vs torch fp32 references."""
import pytest
import torch

from test_fused_ln_cpu import fused_ln_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('N', [768, 1024, 64, 2048])
@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_fused_dropout_add_ln_fp32(N, keep):
    fused_ln_check('cuda', torch.float32, R=300, N=N, keep=keep, tol=2e-5)


@pytest.mark.parametrize('keep', [1.0, 0.9])
def test_fused_dropout_add_ln_bf16(keep):
    fused_ln_check('cuda', torch.bfloat16, R=257, N=768, keep=keep)
