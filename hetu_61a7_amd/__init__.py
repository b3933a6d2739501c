"""hetu_61a7_amd: an MI355X-native (gfx950 / CDNA4) static-dataflow deep-learning
framework with the capabilities and Python API of Hetu.

    import hetu_61a7_amd as ht
    x = ht.Variable(name='x'); y_ = ht.Variable(name='y_')
    W = ht.init.zeros((784, 10), name='W')
    loss = ht.reduce_mean_op(ht.softmaxcrossentropy_op(ht.matmul_op(x, W), y_), [0])
    train_op = ht.optim.SGDOptimizer(0.1).minimize(loss)
    ex = ht.Executor({'train': [loss, train_op]}, ctx=ht.gpu(0))

Compute path: torch-ROCm tensors + hand-written HIP kernels for gfx950
(``csrc/kernels``, loaded from ``hetu_61a7_amd/lib/libhetu_kernels.so``),
RCCL over xGMI for collectives, a C++ host runtime for the parameter server,
HET embedding cache, and a BFC allocator for HBM and pinned DRAM
(``memory_pool``; the process-wide device allocator unless ``HETU_ALLOCATOR=torch``).
"""
from __future__ import annotations

import os as _os

# The native BFC pool is the process-wide device allocator (HETU_ALLOCATOR=torch keeps
# torch's caching allocator).  It must be installed before the first device allocation;
# counting devices does not initialise the GPU.
if _os.environ.get('HETU_ALLOCATOR', 'bfc') == 'bfc':
    try:
        import torch as _torch
        if _torch.cuda.device_count() > 0:
            from .memory_pool import enable_torch_bfc as _enable_bfc
            _enable_bfc()
    except Exception as _e:   # a device allocation happened before this import
        import warnings as _warnings
        _warnings.warn('hetu_61a7_amd: BFC device allocator not installed (%s); torch caching allocator in use' % (_e,))

from .ops import *  # noqa: F401,F403
from .ops import Executor, HetuConfig, gradients, Variable, placeholder_op
from .context import context, get_current_context, DistConfig, DeviceGroup
from .dataloader import dataloader_op, Dataloader, GNNDataLoaderOp
from .ndarray import cpu, gpu, rcpu, rgpu, array, sparse_array, empty, is_gpu_ctx, IndexedSlices, NDArray
from . import optimizer as optim
from . import lr_scheduler as lr
from . import initializers as init
from . import parallel as dist
from .parallel.dispatch import dispatch
from .parallel.comm import new_group_comm
from . import kernels
from . import layers
from . import data
from . import metrics
from . import onnx
from . import graphboard
from .utils.profiler import HetuProfiler, NCCLProfiler
from .launcher_api import (wrapped_mpi_nccl_init, worker_init, worker_finish, server_init,
                           server_finish, scheduler_init, scheduler_finish, get_worker_communicate)

__version__ = '0.1.0'
