"""Distributed strategies (reference ``distributed_strategies/base.py:11-21``,
``simple.py:6-39``).

``DataParallel(aggregate='allreduce'|'ps'|'hybrid')`` assigns raw contexts to
parameters (dense params replicated over the workers, embeddings additionally
on the PS for ps/hybrid).  The cluster description comes from
``/tmp/hetu_config.yml`` when ``heturun`` wrote one, otherwise from the
process environment (``WORLD_SIZE`` workers on this node).
"""
from __future__ import annotations

import os

from ..context import DeviceGroup, DistConfig, dist_env


class Strategy(object):
    def __init__(self, save_path=None):
        path = os.environ.get('HETU_CONFIG', '/tmp/hetu_config.yml')
        _, world, _ = dist_env()
        if os.path.exists(path) and os.environ.get('HETU_USE_CONFIG', '1') == '1':
            self.settings = DistConfig(path)
            if self.settings.num_workers != world and world > 1:
                self.settings = DistConfig(None, num_local_workers=world)
        else:
            self.settings = DistConfig(None, num_local_workers=max(world, 1))
        self.save_path = save_path
        self.overlap = True
        self.use_nccl_collectives = True

    def set_raw_ctxs_n_states(self, node_list, memory_pool):
        raise NotImplementedError

    def set_overlap(self, overlap):
        self.overlap = overlap


class DataParallel(Strategy):
    def __init__(self, aggregate=None):
        super().__init__()
        if aggregate is None:
            aggregate = 'ps' if self.settings.enable_PS else 'allreduce'
        aggregate = aggregate.lower()
        assert aggregate in ('allreduce', 'ps', 'hybrid')
        self.aggregate = aggregate
        embedding_ctxs = ['cpu:0'] if aggregate != 'allreduce' else []
        ctxs = ['cpu:0'] if aggregate == 'ps' else []
        for host, num_worker in self.settings.workers.items():
            devices = ['gpu:%d' % i for i in range(num_worker)]
            embedding_ctxs.extend(devices)
            ctxs.extend(devices)
        self.embedding_raw_ctx = DeviceGroup(embedding_ctxs)
        self.raw_ctx = DeviceGroup(ctxs)

    def set_raw_ctxs_n_states(self, node_list, memory_pool):
        from ..ops.variable import PlaceholderOp
        from ..ops.executor import find_topo_sort
        for node in find_topo_sort(node_list):
            if isinstance(node, PlaceholderOp) and node.trainable and not node.is_embed:
                node.raw_ctx = self.raw_ctx
            else:
                node.raw_ctx = self.embedding_raw_ctx
        return self.raw_ctx


class ModelParallel4CNN(Strategy):
    """Split the last dense layers' weights across workers (tensor parallel)."""

    def __init__(self):
        super().__init__()

    def set_raw_ctxs_n_states(self, node_list, memory_pool):
        from .dispatch import apply_model_parallel_cnn
        return apply_model_parallel_cnn(node_list, self.settings)


class ModelParallel4LM(Strategy):
    def __init__(self):
        super().__init__()

    def set_raw_ctxs_n_states(self, node_list, memory_pool):
        from .dispatch import apply_model_parallel_lm
        return apply_model_parallel_lm(node_list, self.settings)


class OneWeirdTrick4CNN(Strategy):
    """Krizhevsky's one-weird-trick: data parallel convs, model parallel FCs."""

    def __init__(self):
        super().__init__()

    def set_raw_ctxs_n_states(self, node_list, memory_pool):
        from .dispatch import apply_one_weird_trick
        return apply_one_weird_trick(node_list, self.settings)
