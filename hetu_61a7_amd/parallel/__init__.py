"""Parallelism: RCCL communicators, data/pipeline/tensor/expert parallel
strategies, the dispatch lowering pass and the Galvatron-style planner."""
from . import comm
from .strategies import DataParallel, ModelParallel4CNN, ModelParallel4LM, OneWeirdTrick4CNN, Strategy
from .sequence import ulysses_attention_op, UlyssesAttentionOp  # noqa: F401
from .ring_attention import ring_attention_op, RingAttentionOp  # noqa: F401
