"""Device groups, the ``with ht.context(...)`` stack and cluster configuration.

Parity: reference ``python/hetu/context.py`` (DeviceGroup ``:19-150``, context
stack ``:153-181``, launch-mode inference ``:184-234``, DistConfig ``:237-319``).

Strings follow the reference grammar: ``"gpu:0"``, ``"host:gpu:3"``, ``"cpu:0"``;
a *tuple* of contexts inside a group denotes one model-parallel group; ``cpu``
entries denote parameter servers, ``gpu`` entries workers.

MI355X mapping: every GPU worker is its own OS process (one process per GPU,
``torch.distributed`` over RCCL/xGMI).  ``local_rank`` == HIP device ordinal.
"""
from __future__ import annotations

import contextlib
import os
import re
import socket
from typing import Iterator, List, Optional, Tuple, Union

import yaml

from .ndarray import DLContext, cpu, gpu, rcpu, rgpu, is_gpu_ctx


class DeviceGroup(object):
    def __init__(self, ctxs):
        self._contexts = self.parse_contexts(ctxs)
        self.get_servers_n_workers()

    @classmethod
    def parse_contexts(cls, ctxs):
        if isinstance(ctxs, DeviceGroup):
            return list(ctxs._contexts)
        if isinstance(ctxs, str):
            ctxs = [c for c in re.split(';|,| +', ctxs.lower()) if c]
        if not isinstance(ctxs, (list,)):
            ctxs = [ctxs]
        out = []
        for c in ctxs:
            if isinstance(c, tuple):
                out.append(tuple(cls.str2ctx(x) for x in c))
            else:
                c = cls.str2ctx(c)
                if c is not None:
                    out.append(c)
        return out

    @classmethod
    def str2ctx(cls, c):
        if isinstance(c, str):
            parts = c.lower().split(':')
            assert parts[-2] in ('cpu', 'gpu'), 'Context invalid: %s' % c
            hostname = 'localhost' if len(parts) == 2 else parts[0]
            idx = int(parts[-1])
            c = rcpu(hostname, idx) if parts[-2] == 'cpu' else rgpu(hostname, idx)
        assert isinstance(c, DLContext), 'Context invalid: %s' % (c,)
        return c

    def index(self, ctx):
        return self._contexts.index(ctx)

    def __getitem__(self, key):
        return self._workers[key]

    def __iter__(self):
        return iter(self._contexts)

    def __len__(self):
        return len(self._contexts)

    @property
    def is_mp(self) -> bool:
        return self._is_mp

    @property
    def mp_dev_num(self) -> int:
        return self._mp_dev_num

    def check_mp_num(self, n):
        assert n == self._mp_dev_num

    @property
    def worker_num(self) -> int:
        return len(self._workers)

    @property
    def server_num(self) -> int:
        return len(self._servers)

    @property
    def workers(self):
        return self._workers

    @property
    def servers(self):
        return self._servers

    def get_servers_n_workers(self):
        workers, servers = [], []
        mp = None
        for ctx in self._contexts:
            if isinstance(ctx, tuple):
                workers.append(ctx)
                mp = len(ctx) if mp is None else mp
                assert mp == len(ctx), 'all model-parallel groups must have the same size'
            elif is_gpu_ctx(ctx):
                workers.append(ctx)
            else:
                servers.append(ctx)
        self._workers = tuple(workers)
        self._servers = tuple(servers)
        self._is_mp = mp is not None
        self._mp_dev_num = mp if mp is not None else 1

    def all_devices(self):
        out = []
        for c in self._contexts:
            if isinstance(c, tuple):
                out.extend(c)
            else:
                out.append(c)
        return out

    def __repr__(self):
        return 'DeviceGroup(%s)' % ', '.join(str(c) for c in self._contexts)

    def full_repr(self):
        return str([c.full_repr() if isinstance(c, DLContext) else tuple(x.full_repr() for x in c)
                    for c in self._contexts])

    def __hash__(self):
        return hash(tuple(self._contexts))

    def __eq__(self, other):
        return isinstance(other, DeviceGroup) and hash(self) == hash(other)

    def get_sorted(self):
        return DeviceGroup(sorted(self._contexts, key=lambda x: '{}:{}:{}'.format(
            x.hostname, x.device_type, x.device_id)))

    def get_only(self) -> DLContext:
        assert self.server_num + self.worker_num == 1, 'DeviceGroup %s is not a single device' % self
        if self.server_num == 1:
            return self._servers[0]
        res = self._workers[0]
        if isinstance(res, tuple):
            assert len(res) == 1
            res = res[0]
        return res


class ContextStack(object):
    def __init__(self):
        self._stack: List[DeviceGroup] = []

    def peek(self):
        return self._stack[-1] if self._stack else None

    def push(self, ctx):
        self._stack.append(ctx)

    def pop(self):
        self._stack.pop()


_default_ctx_stack = ContextStack()


def get_current_context() -> Optional[DeviceGroup]:
    return _default_ctx_stack.peek()


@contextlib.contextmanager
def context(ctx):
    try:
        ctx = DeviceGroup(ctx)
        _default_ctx_stack.push(ctx)
        yield ctx
    finally:
        _default_ctx_stack.pop()


# ---------------------------------------------------------------------------
# process topology (one process per GPU)
# ---------------------------------------------------------------------------

def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v is not None and v != '':
            return int(v)
    return default


def dist_env():
    """(rank, world_size, local_rank) from torchrun/heturun or mpirun env vars."""
    rank = _env_int('RANK', 'OMPI_COMM_WORLD_RANK', 'PMI_RANK', default=0)
    world = _env_int('WORLD_SIZE', 'OMPI_COMM_WORLD_SIZE', 'PMI_SIZE', default=1)
    local = _env_int('LOCAL_RANK', 'OMPI_COMM_WORLD_LOCAL_RANK', default=rank)
    return rank, world, local


def get_launch_config_by_traverse_nodes(node_list, default_ctx):
    """Infer (launchMPI, launchPS, node_strategy, devices, min_worker_num).

    Same decision rule as reference ``context.py:184-234``: a node whose
    raw context contains servers and workers is PS-managed; a node replicated
    over >1 workers is AllReduce-managed.
    """
    from .optimizer import OptimizerOp
    node_strategy = {}
    devices = set()
    default_ctx = DeviceGroup(default_ctx) if not isinstance(default_ctx, DeviceGroup) else default_ctx
    for c in default_ctx:
        if isinstance(c, tuple):
            devices.update(c)
        else:
            devices.add(c)
    min_worker_num = default_ctx.worker_num
    launch_ps = default_ctx.server_num > 0
    launch_mpi = (not launch_ps) and min_worker_num > 1

    visited = set()
    stack = list(node_list)
    while stack:
        node = stack.pop()
        if node in visited:
            continue
        visited.add(node)
        strategy = None
        rc = node.raw_ctx
        wn = 1 if rc is None else rc.worker_num
        if rc is not None and rc.server_num > 0 and wn > 0:
            strategy = 'PS'
        elif rc is not None and wn > 1:
            strategy = 'AllReduce'
        node_strategy[node] = strategy
        if rc is not None and not isinstance(node, OptimizerOp):
            for c in rc:
                if isinstance(c, tuple):
                    devices.update(c)
                else:
                    devices.add(c)
        stack.extend(node.inputs)
    launch_ps = launch_ps or any(v == 'PS' for v in node_strategy.values())
    launch_mpi = launch_mpi or any(v == 'AllReduce' for v in node_strategy.values())
    return launch_mpi, launch_ps, node_strategy, devices, min_worker_num


class DistConfig(object):
    """Cluster YAML: ``nodes: [{host, servers, workers, chief}]``.

    Reference ``context.py:237-319``.  Loaded with ``yaml.safe_load``.
    """

    def __init__(self, file: Optional[str] = None, num_local_servers: int = 0, num_local_workers: int = 1):
        if file is None or not os.path.exists(file):
            assert num_local_workers > 0
            if file is None or True:
                # env-derived single-node default: one worker per local rank
                _, world, _ = dist_env()
                nw = max(num_local_workers, world if file is not None else num_local_workers)
            self.settings = {'nodes': [{
                'host': socket.gethostname(), 'servers': num_local_servers,
                'workers': nw, 'chief': True}]}
        else:
            with open(file) as f:
                self.settings = yaml.safe_load(f.read())
        attributes = {'host', 'servers', 'workers', 'chief'}
        hosts, servers, workers, chief = [], {}, {}, None
        for node in self.settings['nodes']:
            assert set(node.keys()) <= attributes, 'Attributes of nodes invalid: %s' % set(node.keys())
            hosts.append(node['host'])
            if node.get('servers', 0):
                servers[node['host']] = node['servers']
            if node.get('workers', 0):
                workers[node['host']] = node['workers']
            if node.get('chief', False):
                assert chief is None, 'There should be only one chief.'
                chief = node['host']
        assert chief, 'There should be one chief.'
        self.num_servers = sum(servers.values())
        self.num_workers = sum(workers.values())
        self.enable_PS = self.num_servers > 0
        self.servers = servers
        self.workers = workers
        self.chief = chief
        self.hosts = hosts
        self.chief_address = '127.0.0.1'

    def __str__(self):
        return '\n'.join(['Cluster: {', '  Chief: %s,' % self.chief,
                          '  Servers(%d): %s,' % (self.num_servers, self.servers),
                          '  Workers(%d): %s,' % (self.num_workers, self.workers), '}'])

    def __iter__(self):
        return iter(self.settings['nodes'])

    def save(self, path: str):
        with open(path, 'w') as fw:
            yaml.safe_dump(self.settings, fw)

    def make_ps_config(self):
        return {
            'DMLC_PS_ROOT_URI': self.chief_address,
            'DMLC_PS_ROOT_PORT': self.get_available_port(self.chief_address),
            'DMLC_NUM_WORKER': self.num_workers,
            'DMLC_NUM_SERVER': self.num_servers,
            'DMLC_PS_VAN_TYPE': 'shm',
        }

    @staticmethod
    def get_available_port(localhost='127.0.0.1'):
        for p in range(13100, 13400):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            try:
                s.bind((localhost, p))
                return p
            except OSError:
                continue
            finally:
                s.close()
        raise RuntimeError('no free port')
